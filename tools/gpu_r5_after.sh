#!/bin/bash
# round 5: the default copy order (after the elimination) -- the elimination
# and decode tests, the C2 AddPiece phases, the round trip against r5lib_pre
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r5after}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_elim.py tests/test_gpu_elim_route.py tests/test_gpu_compact_rows.py tests/test_gpu_group_decode.py tests/test_gpu_lazy_decode.py tests/test_gpu_headline.py tests/test_gpu_coresidency.py -x -q -m gpu --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
echo "tests $(tail -1 $OUT/tests.log)"
bash tools/gpu_c2_phases.sh ${1:-r5after}/c2 || exit 1
for rep in 1 2; do
  for v in pre new; do
    libp=kodr_amd/libkodr_rlnc.so; [ $v = pre ] && libp=kodr_amd/r5lib_pre/libkodr_rlnc.so
    KODR_RLNC_LIB=$libp timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b_${v}_$rep.json 2> $OUT/b_${v}_$rep.err || { tail -20 $OUT/b_${v}_$rep.err; exit 1; }
    python3 - $OUT/b_${v}_$rep.json $v <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
c2 = d["extras"]["c2_decode"]
print(sys.argv[2], "rt us/gen", d["roundtrip"]["us_per_generation"], "enc B32", d["encode"]["ms_per_step"], "c2", c2["s"], "add", c2["add_s"], c2.get("add_s_median"), c2.get("add_s_max"), "get", c2["get_s"], c2.get("elimination_routes"))
PY
  done
done
