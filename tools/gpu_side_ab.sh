#!/bin/bash
# A/B: batched GPU AddPiece with the row copies on a side stream (current
# build) against the same stream (kodr_amd/base/), interleaved.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/side_ab; mkdir -p $OUT
for rep in 1 2 3; do
  for V in base new; do
    LIB=kodr_amd/libkodr_rlnc.so; [ $V = base ] && LIB=kodr_amd/base/libkodr_rlnc.so
    KODR_RLNC_LIB=$LIB timeout -k 10 120 python -u tools/group_add_time.py 16 > $OUT/t_${V}_r$rep.log 2>&1 \
      || { tail -20 $OUT/t_${V}_r$rep.log; exit 1; }
    echo "$V rep $rep $(tail -1 $OUT/t_${V}_r$rep.log)"
  done
done
