#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r02d; mkdir -p $OUT
timeout -k 10 120 python3 tools/c4_probe.py > $OUT/c4.json 2>&1 || { cat $OUT/c4.json; exit 1; }
cat $OUT/c4.json
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python - <<'PY'
import json; d=json.load(open("gpurun_out/r02d/bench.json")); x=d["extras"]
print(d["value"], "c4", json.dumps({k: x["c4_systematic_decode"][k] for k in ("systematic","full_coded_only","speedup_vs_full")}))
print("c2", json.dumps(x["c2_decode"]))
PY
