#!/bin/bash
# blocked GPU elimination: parity tests, then host vs GPU (per-step vs blocked) timing
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_elim.py tests/test_gpu_progressive.py -x -q --timeout 120 --timeout-method thread > gpurun_out/elim_blk_tests.log 2>&1 || { tail -30 gpurun_out/elim_blk_tests.log; exit 1; }
tail -2 gpurun_out/elim_blk_tests.log
timeout -k 10 200 python -u tools/elim_time.py 64,128,256 1,8,32,128 > gpurun_out/elim_blk_time.log 2>&1 || { cat gpurun_out/elim_blk_time.log; exit 1; }
KODR_ELIM_BLOCKED=0 timeout -k 10 200 python -u tools/elim_time.py 256 1,32 > gpurun_out/elim_step_time.log 2>&1 || { cat gpurun_out/elim_step_time.log; exit 1; }
cat gpurun_out/elim_blk_time.log gpurun_out/elim_step_time.log
