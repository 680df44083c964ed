#!/bin/bash
# (Measurement recipe, round 4; the KODR_ELIM_CHUNK knob it set is removed.)
# Decoders per elimination launch in the round trip (KODR_ELIM_CHUNK: 0 =
# the policy's, one mc2 launch for 16; 7 = mc4 launches of 7, 7, 2; 4 = mc4
# launches of 4): bench.py --no-extras encode_decode, interleaved reps, and a
# kernel trace of each setting.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-chunk_ab}; mkdir -p $OUT
R=$(pwd)
for rep in 1 2 3; do
  for c in ${CHUNKS:-0 7 4}; do
    KODR_ELIM_CHUNK=$c timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > $OUT/c${c}_$rep.json 2> $OUT/c${c}_$rep.err || { tail -5 $OUT/c${c}_$rep.err; exit 1; }
    echo "chunk $c rep $rep: $(python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1]); e=d['encode_decode']; print(e['ms_per_step'], e['us_per_generation'], e['roundtrip_ok'])" $OUT/c${c}_$rep.json)"
  done
done
for c in ${CHUNKS:-0 7 4}; do
  cd /tmp
  KODR_ELIM_CHUNK=$c timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/$OUT/prof_c$c -o run --output-format csv -- python3 $R/bench.py --steps 10 --warmup 3 --no-extras --no-cpu-baseline > $R/$OUT/prof_c$c.json 2> $R/$OUT/prof_c$c.err || { tail -5 $R/$OUT/prof_c$c.err; exit 1; }
  cd $R
  python3 tools/kernel_durations.py $OUT/prof_c$c | cut -c1-600
done
