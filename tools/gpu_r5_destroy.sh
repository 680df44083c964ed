#!/bin/bash
# round 5: decoder destroy without a host wait -- the decode tests, then the
# round trip against r5lib_pre and a trace timeline
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-r5destroy}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 200 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
echo "tests $(tail -1 $OUT/pytest_gpu.log)"
for rep in 1 2 3; do
  for v in new pre; do
    libp=kodr_amd/libkodr_rlnc.so; [ $v = pre ] && libp=kodr_amd/r5lib_pre/libkodr_rlnc.so
    KODR_RLNC_LIB=$libp timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > $OUT/b_${v}_$rep.json 2> $OUT/b_${v}_$rep.err || { tail -20 $OUT/b_${v}_$rep.err; exit 1; }
    python3 - $OUT/b_${v}_$rep.json $v <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
lg = d["roofline"]["legs"]
print(sys.argv[2], "rt us/gen", d["roundtrip"]["us_per_generation"], "enc", lg["encode_launch"]["avg_us"], "add", lg["add_pieces_call"]["avg_us"], lg["add_pieces_call"].get("call_wall_us"), "get", lg["get_pieces_call"]["avg_us"], "ok", d["roundtrip"]["roundtrip_ok"], "B32", d["encode"]["ms_per_step"])
PY
  done
done
