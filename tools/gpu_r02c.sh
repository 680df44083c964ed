#!/bin/bash
# Host elimination A/B on the box's CPU (old vs new DecoderCore harness,
# build_tune/dc_*), then the GPU suite and the bench.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r02c; mkdir -p $OUT
for rep in 1 2; do for b in old new; do for a in "128 12 0" "128 12 1" "256 25 0" "256 25 1"; do
  echo -n "$b: "; taskset -c 3 build_tune/dc_$b $a; done; done; done | tee $OUT/dc_ab.txt
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -2 $OUT/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python - <<'PY'
import json; d=json.load(open("gpurun_out/r02c/bench.json"))
print(d["value"], json.dumps(d["extras"]["c4_systematic_decode"]), json.dumps(d["extras"]["c2_decode"]))
PY
