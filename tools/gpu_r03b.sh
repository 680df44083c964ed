#!/bin/bash
# Round 3: lazy AddPiece tests, then the direct-variant A/B.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r03b}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu -k "lazy or progressive or decode or elim" --timeout 300 --timeout-method thread > $OUT/pytest_lazy.log 2>&1 || { tail -40 $OUT/pytest_lazy.log; exit 1; }
tail -1 $OUT/pytest_lazy.log
tools/gpu_direct_ab.sh ${1:-r03b}/direct_ab
