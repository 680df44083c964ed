#!/bin/bash
# Phase totals per wave of the GPU elimination kernel at k = 256 (tuning build
# -DKODR_ELIM_TIMING in kodr_amd/tune_e/: s_memtime stamps, no result).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-elim_phases}; mkdir -p $OUT
for C in 1 0; do
  KODR_ELIM_CIRC=$C KODR_RLNC_LIB=kodr_amd/tune_e/libkodr_rlnc.so KODR_ELIM_DUMP=/tmp/elim_dump_$C.bin timeout -k 10 60 python -u tools/elim_blk_timing.py 256 > $OUT/phases_c$C.log 2>&1 || { tail -20 $OUT/phases_c$C.log; exit 1; }
  echo "circ=$C"; cat $OUT/phases_c$C.log
done
