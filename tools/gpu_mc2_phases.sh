#!/bin/bash
# Timeline of gf_elim_mc2_kernel (tuning build in kodr_amd/tune_e: -DKODR_ELIM_TIMING).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-mc2_phases}; mkdir -p $OUT
for G in ${GS:-1 16}; do
  KODR_RLNC_LIB=kodr_amd/tune_e/libkodr_rlnc.so KODR_ELIM_DUMP=/tmp/mc2_dump_$G.bin timeout -k 10 60 python -u tools/elim_mc2_timing.py ${K:-256} $G > $OUT/phases_G$G.log 2>&1 || { tail -20 $OUT/phases_G$G.log; exit 1; }
  tail -4 $OUT/phases_G$G.log
done
