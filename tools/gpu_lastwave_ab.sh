#!/bin/bash
# A/B: grouped launches with the last-arriving wave storing (current build)
# against the barrier fold (kodr_amd/base/, the previous commit), interleaved.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/lastw; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_headline.py \
  tests/test_gpu_group_decode.py > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for rep in 1 2 3; do
  for V in base new; do
    LIB=kodr_amd/libkodr_rlnc.so; [ $V = base ] && LIB=kodr_amd/base/libkodr_rlnc.so
    KODR_RLNC_LIB=$LIB timeout -k 10 120 python -u tools/group_bs_time.py 16 32 64 256 > $OUT/t_${V}_r$rep.log 2>&1 \
      || { tail -20 $OUT/t_${V}_r$rep.log; exit 1; }
    echo "$V rep $rep $(python3 -c "import json,sys; d=json.loads(open('$OUT/t_${V}_r$rep.log').read().strip().splitlines()[-1]); print([d[k]['grouped_us_per_generation'] for k in ('B16','B32','B64','B256')])")"
  done
done
