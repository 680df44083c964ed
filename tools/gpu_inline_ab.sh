#!/bin/bash
# Dispatch-free bound of the grouped bit-sliced launch: tuning build
# (kodr_amd/tune_i/, -DKODR_TUNE_MODES) MODE 0 (threaded bodies) against MODE 30
# (every body inlined for one coefficient: no jumps, no stubs, wrong products),
# interleaved, tools/group_bs_time.py (16 prepared 32 MiB/256 generations).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-inline}; mkdir -p $OUT
for rep in 1 2 3; do
  for M in 0 30; do
    KODR_BS_MODE=$M KODR_RLNC_LIB=kodr_amd/tune_i/libkodr_rlnc.so timeout -k 10 120 python -u tools/group_bs_time.py 32 64 256 \
      > $OUT/t_m${M}_r$rep.log 2>&1 || { tail -20 $OUT/t_m${M}_r$rep.log; exit 1; }
    echo "mode $M rep $rep"; head -3 $OUT/t_m${M}_r$rep.log
  done
done
