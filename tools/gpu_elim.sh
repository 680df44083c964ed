#!/bin/bash
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/elim; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_elim.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 200 python tools/elim_time.py 64,128,256 1,8,32 256 > $OUT/time.log 2>&1 || { tail -20 $OUT/time.log; exit 1; }
cat $OUT/time.log
