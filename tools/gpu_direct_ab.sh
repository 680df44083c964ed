#!/bin/bash
# A/B of the direct grouped variant (KW = 1 waves per workgroup, no LDS fold)
# against the default plan, interleaved reps on one box; parity first.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-direct_ab}; mkdir -p $OUT
KODR_BS_DIRECT=1 timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -k "every_kw or grouped or group_wire or bench_headline" --timeout 300 --timeout-method thread > $OUT/tests_direct.log 2>&1 || { tail -30 $OUT/tests_direct.log; exit 1; }
tail -1 $OUT/tests_direct.log
for rep in 1 2 3; do
  for D in 0 1; do
    KODR_BS_DIRECT=$D timeout -k 10 180 python -u tools/group_bs_time.py 16 32 64 256 > $OUT/d${D}_r$rep.log 2>&1 || { tail -20 $OUT/d${D}_r$rep.log; exit 1; }
    echo "direct=$D rep $rep $(python3 -c "import json; d=json.loads(open('$OUT/d${D}_r$rep.log').read().strip().splitlines()[-1]); print([d[k]['grouped_us_per_generation'] for k in ('B16','B32','B64','B256')])")"
  done
done
