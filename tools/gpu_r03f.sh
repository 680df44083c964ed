#!/bin/bash
# Recode side product staged in LDS (KODR_SIDE_STAGE=1, KW = 16 plans) against
# the register path (0) and the separate vector launch (KODR_REC_SIDE=0):
# parity of the recode paths under each, then interleaved timings.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r03f}; mkdir -p $OUT
for S in 1 0; do
  KODR_SIDE_STAGE=$S timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_gpu_recode_side.py \
    tests/test_gpu_headline.py -k "recode or recoder" > $OUT/pytest_stage$S.log 2>&1 || { tail -40 $OUT/pytest_stage$S.log; exit 1; }
  echo "stage=$S $(tail -1 $OUT/pytest_stage$S.log)"
done
for rep in 1 2 3; do
  for V in "1 1" "1 0" "0 1"; do
    set -- $V
    KODR_REC_SIDE=$1 KODR_SIDE_STAGE=$2 timeout -k 10 120 python -u tools/recode_time.py 16 32 64 > $OUT/rec_s$1_t$2_r$rep.json 2>&1 || { tail -20 $OUT/rec_s$1_t$2_r$rep.json; exit 1; }
    echo "side=$1 stage=$2 rep $rep $(tail -1 $OUT/rec_s$1_t$2_r$rep.json)"
  done
done
