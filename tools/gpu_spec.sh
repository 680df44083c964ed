#!/bin/bash
# round 5: a lone decoder's elimination attempts side by side (mc4 x 4):
# elimination tests, C2 AddPiece phases for a vector set that needs a
# rotated attempt (seed 7) and one that does not (11), then the bench's
# c2_decode over fresh sets (this tree against r5lib_pre)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-spec}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_elim.py tests/test_gpu_elim_route.py tests/test_gpu_lazy_decode.py tests/test_gpu_coresidency.py tests/test_gpu_compact_rows.py -x -q -m gpu --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
echo "tests $(tail -1 $OUT/tests.log)"
for seed in 7 11; do
  KODR_ADD_TIMING=1 timeout -k 10 120 python -u tools/c2_add_phases.py 12 $seed > $OUT/ph_$seed.log 2>&1 || { tail -5 $OUT/ph_$seed.log; exit 1; }
  echo "seed $seed: $(grep '^rep' $OUT/ph_$seed.log | tail -8 | awk '{print $4}' | tr '\n' ' ')"
done
for v in new pre new pre; do
  libp=kodr_amd/libkodr_rlnc.so; [ $v = pre ] && libp=kodr_amd/r5lib_pre/libkodr_rlnc.so
  KODR_RLNC_LIB=$libp timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/b_$v.json 2> $OUT/b_$v.err || { tail -10 $OUT/b_$v.err; exit 1; }
  python3 - $OUT/b_$v.json $v <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
c = d["extras"]["c2_decode"]
print(sys.argv[2], "c2 s", c["s"], "add", c["add_s"], c.get("add_s_median"), c.get("add_s_max"), c.get("elimination_routes"), "rt", d["roundtrip"]["us_per_generation"])
PY
done
