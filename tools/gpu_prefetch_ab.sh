#!/bin/bash
# round 5: the host route's vector download beside every launch, merged over
# decoders whose rows share an allocation (this tree), against r5lib_pre
# (no download): the co-residency and elimination route tests, then the round
# trip interleaved
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-pfab}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_coresidency.py tests/test_gpu_elim_route.py tests/test_gpu_elim.py tests/test_gpu_headline.py -x -q -s -m gpu --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
grep "call .* ms" $OUT/tests.log | cut -c1-120; echo "tests $(tail -1 $OUT/tests.log)"
for rep in 1 2 3; do
  for v in new pre; do
    libp=kodr_amd/libkodr_rlnc.so; [ $v = pre ] && libp=kodr_amd/r5lib_pre/libkodr_rlnc.so
    KODR_RLNC_LIB=$libp timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > $OUT/b_${v}_$rep.json 2> $OUT/b_${v}_$rep.err || { tail -20 $OUT/b_${v}_$rep.err; exit 1; }
    python3 - $OUT/b_${v}_$rep.json $v <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(sys.argv[2], "rt us/gen", d["roundtrip"]["us_per_generation"], "add", d["roofline"]["legs"]["add_pieces_call"]["avg_us"], d["roundtrip"]["elimination_routes"])
PY
  done
done
