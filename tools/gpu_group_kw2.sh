#!/bin/bash
# Waves per workgroup for grouped launches with the two-row ring: tuning build
# (kodr_amd/tune_g/, KODR_BS_KW forces KW), interleaved reps.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/kw2; mkdir -p $OUT
for rep in 1 2; do
  for KW in 4 8 2; do
    KODR_BS_KW=$KW KODR_RLNC_LIB=kodr_amd/tune_g/libkodr_rlnc.so timeout -k 10 120 python -u tools/group_bs_time.py 16 32 64 256 \
      > $OUT/kw${KW}_r$rep.log 2>&1 || { tail -20 $OUT/kw${KW}_r$rep.log; exit 1; }
    echo "KW $KW rep $rep $(python3 -c "import json; d=json.loads(open('$OUT/kw${KW}_r$rep.log').read().strip().splitlines()[-1]); print([d[k]['grouped_us_per_generation'] for k in ('B16','B32','B64','B256')])")"
  done
done
