#!/bin/bash
# The round trip with the batched AddPiece's row copies beside the
# elimination (KODR_ADD_SIDE=1, default) or after it on the context stream
# (0): bench.py --no-extras encode_decode, interleaved reps.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-side_ab}; mkdir -p $OUT
for rep in 1 2 3; do
  for s in 1 0; do
    KODR_ADD_SIDE=$s timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > $OUT/s${s}_$rep.json 2> $OUT/s${s}_$rep.err || { tail -5 $OUT/s${s}_$rep.err; exit 1; }
    echo "side $s rep $rep: $(python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); e=d['encode_decode']; print(e['ms_per_step'], e['us_per_generation'])" $OUT/s${s}_$rep.json)"
  done
done
