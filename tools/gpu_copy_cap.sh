#!/bin/bash
# The round trip's row copy + twin beside the elimination at several
# residency caps (KODR_COPY_WG_PER_CU workgroups per CU): bench.py
# --no-extras encode_decode per cap, two interleaved reps.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-copycap}; mkdir -p $OUT
for rep in 1 2; do
  for c in ${CAPS:-2 4 8}; do
    KODR_COPY_WG_PER_CU=$c timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > $OUT/c${c}_$rep.json 2> $OUT/c${c}_$rep.err || { tail -5 $OUT/c${c}_$rep.err; exit 1; }
    echo "cap $c rep $rep: $(python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); e=d['encode_decode']; print(e['ms_per_step'], e['us_per_generation'])" $OUT/c${c}_$rep.json)"
  done
done
