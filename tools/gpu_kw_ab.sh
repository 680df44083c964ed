#!/bin/bash
# round 5: the round trip's B = k + 2 = 258 encode launch planned folded
# (KW = 4, the cost model's pick) or direct (KW = 1, KODR_BS_KW in the tuning
# build kodr_amd/tune_m/): tools/group_bs_time.py at B = 258, then the bench's
# round trip (--no-extras), interleaved
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-kwab}; mkdir -p $OUT
T=kodr_amd/tune_m/libkodr_rlnc.so
for rep in 1 2; do
  for kw in dflt 1; do
    if [ $kw = dflt ]; then E=""; else E="KODR_BS_KW=$kw"; fi
    env $E KODR_RLNC_LIB=$T timeout -k 10 120 python -u tools/group_bs_time.py 258 > $OUT/g_${kw}_$rep.log 2>&1 || { tail -5 $OUT/g_${kw}_$rep.log; exit 1; }
    echo "group kw=$kw rep $rep: $(grep -E '^258 ' $OUT/g_${kw}_$rep.log | sed 's/"single[^,]*, //; s/, "speedup[^}]*//')"
    env $E KODR_RLNC_LIB=$T timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > $OUT/b_${kw}_$rep.json 2> $OUT/b_${kw}_$rep.err || { tail -20 $OUT/b_${kw}_$rep.err; exit 1; }
    python3 - $OUT/b_${kw}_$rep.json $kw <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
lg = d["roofline"]["legs"]
print("bench kw=" + sys.argv[2], "rt us/gen", d["roundtrip"]["us_per_generation"], "enc", lg["encode_launch"]["avg_us"], lg["encode_launch"]["plan"]["waves"], "get", lg["get_pieces_call"]["avg_us"], "ok", d["roundtrip"]["roundtrip_ok"])
PY
  done
done
