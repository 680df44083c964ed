#!/bin/bash
# Round 3 validation: full GPU suite, smoke, rocprof evidence of the headline
# (kernel trace + separate FETCH/WRITE PMC passes), the driver's bench command.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r03n}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
tools/profile_headline.sh || exit 1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python -c "import json; d=json.loads(open('$OUT/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['roofline']['plan']); print(json.dumps(d['encode_decode'])[:400]); print(d['extras']['c2_decode']); print(d['extras']['c2_recode']); print(d['extras']['encode_batch_sweep'])"
