#!/bin/bash
# Wave-priority rotation in grouped launches: tuning build (kodr_amd/tune_g/,
# -DKODR_TUNE_MODES) MODE 0 (rotation per row), 10 (no s_setprio), 11 (second
# half of each row at another priority), interleaved, tools/group_bs_time.py.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/prio; mkdir -p $OUT
for rep in 1 2; do
  for M in 0 10 11; do
    KODR_BS_MODE=$M KODR_RLNC_LIB=kodr_amd/tune_g/libkodr_rlnc.so timeout -k 10 120 python -u tools/group_bs_time.py 32 64 \
      > $OUT/t_m${M}_r$rep.log 2>&1 || { tail -20 $OUT/t_m${M}_r$rep.log; exit 1; }
    echo "mode $M rep $rep"; head -2 $OUT/t_m${M}_r$rep.log
  done
done
