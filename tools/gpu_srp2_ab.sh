#!/bin/bash
# A/B: the two-row ring also for single launches with >= 32 rows per wave
# (kodr_amd/srp2/) against grouped-only (current build), interleaved:
# single-generation encode B = 64 / 256 and a C2 GetPieces.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/srp2; mkdir -p $OUT
KODR_RLNC_LIB=kodr_amd/srp2/libkodr_rlnc.so timeout -k 10 300 python -u -m pytest -x -q --timeout 120 \
  --timeout-method thread tests/test_gpu_headline.py tests/test_gpu_parity.py > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for rep in 1 2 3; do
  for V in cur srp2; do
    LIB=kodr_amd/libkodr_rlnc.so; [ $V = srp2 ] && LIB=kodr_amd/srp2/libkodr_rlnc.so
    KODR_RLNC_LIB=$LIB timeout -k 10 120 python -u tools/group_bs_time.py 64 256 > $OUT/e_${V}_r$rep.log 2>&1 || { tail $OUT/e_${V}_r$rep.log; exit 1; }
    KODR_RLNC_LIB=$LIB timeout -k 10 120 python -u tools/group_get_time.py 16 > $OUT/g_${V}_r$rep.log 2>&1 || { tail $OUT/g_${V}_r$rep.log; exit 1; }
    echo "$V rep $rep enc $(python3 -c "import json; d=json.loads(open('$OUT/e_${V}_r$rep.log').read().strip().splitlines()[-1]); print([d[k]['single_us_per_generation'] for k in ('B64','B256')])") get $(python3 -c "import json; d=json.loads(open('$OUT/g_${V}_r$rep.log').read().strip().splitlines()[-1]); print(d['per_decoder_us_per_generation'])")"
  done
done
