#!/bin/bash
# A/B of the bit-sliced row ring depth in grouped launches (KODR_BS_P=2 build
# in kodr_amd/p2/, made on the CPU side): parity of the headline tests under
# the variant, then tools/group_bs_time.py interleaved over the two builds.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/ring; mkdir -p $OUT
KODR_RLNC_LIB=kodr_amd/p2/libkodr_rlnc.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 \
  --timeout-method thread tests/test_gpu_headline.py tests/test_gpu_parity.py > $OUT/tests_p2.log 2>&1 \
  || { tail -30 $OUT/tests_p2.log; exit 1; }
tail -1 $OUT/tests_p2.log
for rep in 1 2; do
  for V in p1 p2; do
    LIB=kodr_amd/libkodr_rlnc.so; [ $V = p2 ] && LIB=kodr_amd/p2/libkodr_rlnc.so
    KODR_RLNC_LIB=$LIB timeout -k 10 120 python -u tools/group_bs_time.py 16 32 64 256 > $OUT/t_${V}_r$rep.log 2>&1 \
      || { tail -20 $OUT/t_${V}_r$rep.log; exit 1; }
    echo "$V rep $rep"; head -4 $OUT/t_${V}_r$rep.log
  done
done
