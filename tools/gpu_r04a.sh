#!/bin/bash
# Round-4 first look: GPU suite, the driver's bench command, and the phases
# of one decoder's batched AddPiece (host solve vs the one-CU GPU kernel).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r04a}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
echo "tests: $(tail -1 $OUT/pytest_gpu.log)"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 1; }
KODR_ADD_TIMING=1 timeout -k 10 120 python -u tools/elim_time.py 256 1 256 > $OUT/elim1.log 2>&1 || { tail -20 $OUT/elim1.log; exit 1; }
tail -3 $OUT/elim1.log
