#!/bin/bash
# occupancy sensitivity of the grouped direct bit-sliced launch: workgroups
# (one wave each) per CU capped by LDS padding (tuning build kodr_amd/tune_m/,
# KODR_BS_WG_PER_CU): 16 = 4 waves per SIMD (the register limit), 12 = 3,
# 8 = 2, 4 = 1; tools/group_bs_time.py at B = 32 and 256
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-occ}; mkdir -p $OUT
for rep in 1 2; do
  for n in 16 12 8 4; do
    KODR_BS_WG_PER_CU=$n KODR_RLNC_LIB=kodr_amd/tune_m/libkodr_rlnc.so timeout -k 10 120 python -u tools/group_bs_time.py 32 256 > $OUT/o_${n}_$rep.log 2>&1 || { tail -5 $OUT/o_${n}_$rep.log; exit 1; }
    echo "wg/cu $n rep $rep: $(grep -E '^(32|256) ' $OUT/o_${n}_$rep.log | sed 's/"single[^,]*, //; s/, "speedup[^}]*//' | tr '\n' ' ')"
  done
done
