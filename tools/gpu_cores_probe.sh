#!/bin/bash
# the co-residency test with the batched AddPiece's phase times
# (KODR_ADD_TIMING=1), this tree's library and r5lib_pre's
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-cores}; mkdir -p $OUT
for v in new; do
  libp=kodr_amd/libkodr_rlnc.so; [ $v = pre ] && libp=kodr_amd/r5lib_pre/libkodr_rlnc.so
  KODR_ADD_TIMING=1 KODR_RLNC_LIB=$libp timeout -k 10 120 python -u -m pytest tests/test_gpu_coresidency.py -x -q -s -m gpu --timeout 100 --timeout-method thread > $OUT/$v.log 2>&1
  echo "== $v rc $?"; grep -E "add_pieces_gpu|call .* ms|passed|failed" $OUT/$v.log | cut -c1-300
done
