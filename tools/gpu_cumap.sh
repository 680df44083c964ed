#!/bin/bash
# round 5: the row groups of a (generation, column chunk) co-located on one CU
# (tuning MODE 34, kodr_amd/tune_m/) against the product mapping (MODE 0 of
# the same build): parity of the headline and round-trip steps under MODE 34,
# then back-to-back launches with clocks and power (tools/clock_probe.py)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-cumap}; mkdir -p $OUT
T=kodr_amd/tune_m/libkodr_rlnc.so
KODR_BS_MODE=34 KODR_RLNC_LIB=$T timeout -k 10 300 python -u -m pytest tests/test_gpu_headline.py -x -q -m gpu --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1; echo "mode 34 headline tests rc $? $(tail -1 $OUT/tests.log)"
for rep in 1 2; do
  for m in 0 34; do
    KODR_BS_MODE=$m KODR_RLNC_LIB=$T timeout -k 10 120 python -u tools/clock_probe.py $OUT/m${m}_$rep.jsonl 32 256 > $OUT/m${m}_$rep.log 2>&1 || { tail -5 $OUT/m${m}_$rep.log; exit 1; }
    echo "mode $m rep $rep:"; grep "^B=" $OUT/m${m}_$rep.log
  done
done
