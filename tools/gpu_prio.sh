#!/bin/bash
# the grouped direct launch's wave-priority rotation: product (row j: j % 4),
# none (MODE 35), over row pairs (MODE 36); tuning build, back-to-back
# launches with clocks and power (tools/clock_probe.py), B = 32 and 256
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-prio}; mkdir -p $OUT
T=kodr_amd/tune_m/libkodr_rlnc.so
for rep in 1 2; do
  for m in ${MODES:-0 35 36}; do
    KODR_BS_MODE=$m KODR_RLNC_LIB=$T timeout -k 10 120 python -u tools/clock_probe.py $OUT/m${m}_$rep.jsonl 32 256 > $OUT/m${m}_$rep.log 2>&1 || { tail -5 $OUT/m${m}_$rep.log; exit 1; }
    echo "mode $m rep $rep: $(grep '^B=' $OUT/m${m}_$rep.log | awk '{print $1, $3, $4, $10, $14}' | tr '\n' ' ')"
  done
done
