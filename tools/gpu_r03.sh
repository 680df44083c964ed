#!/bin/bash
# Round-3 validation on the GPU box: the new tests first, then the whole GPU
# suite, smoke and the driver's bench command.  Usage: tools/gpu_r03.sh OUTDIR [pytest -k expr]
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r03}; mkdir -p $OUT
if [ -n "${2:-}" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "$2" --timeout 300 --timeout-method thread > $OUT/pytest_new.log 2>&1 || { tail -40 $OUT/pytest_new.log; exit 1; }
  tail -1 $OUT/pytest_new.log
fi
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['roofline']['plan']); print(json.dumps(d['encode_decode']))"
