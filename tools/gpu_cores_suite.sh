#!/bin/bash
# the co-residency test after the other elimination tests in one pytest
# session (as the GPU suite runs it), with the batched AddPiece's phase times
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-cores_suite}; mkdir -p $OUT
KODR_ADD_TIMING=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_compact_rows.py tests/test_gpu_group_decode.py tests/test_gpu_headline.py tests/test_gpu_coresidency.py -x -q -s -m gpu --timeout 150 --timeout-method thread > $OUT/suite.log 2>&1
echo "rc $?"
grep -n "call .* ms" $OUT/suite.log | cut -c1-200
L=$(grep -n "call .* ms" $OUT/suite.log | head -1 | cut -d: -f1)
[ -n "$L" ] && sed -n "$((L-12)),$((L))p" $OUT/suite.log | cut -c1-250
tail -3 $OUT/suite.log
