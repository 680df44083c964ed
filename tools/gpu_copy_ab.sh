#!/bin/bash
# round 5: the rows' twin copy beside the elimination handed out in chunks
# from a counter (this tree) against the capped grid-stride copy
# (kodr_amd/r5lib_pre/): the tests that run it, then the round trip of
# bench.py (--no-extras) interleaved, then a kernel trace of this tree's.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-copyab}; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_compact_rows.py tests/test_gpu_group_decode.py tests/test_gpu_headline.py tests/test_gpu_coresidency.py tests/test_gpu_elim_route.py -x -q -m gpu --timeout 150 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
echo "tests $(tail -1 $OUT/tests.log)"
for rep in 1 2 3; do
  for v in pre new; do
    libp=kodr_amd/libkodr_rlnc.so; [ $v = pre ] && libp=kodr_amd/r5lib_pre/libkodr_rlnc.so
    KODR_RLNC_LIB=$libp timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > $OUT/b_${v}_$rep.json 2> $OUT/b_${v}_$rep.err || { tail -20 $OUT/b_${v}_$rep.err; exit 1; }
    python3 - $OUT/b_${v}_$rep.json $v $rep <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
lg = d["roofline"]["legs"]
print(sys.argv[2], sys.argv[3], "rt us/gen", d["roundtrip"]["us_per_generation"], "enc", lg["encode_launch"]["avg_us"],
      "add", lg["add_pieces_call"]["avg_us"], "get", lg["get_pieces_call"]["avg_us"], "ok", d["roundtrip"]["roundtrip_ok"],
      d["roundtrip"]["elimination_routes"])
PY
  done
done
R=$(pwd)
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$OUT/rt -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > $R/$OUT/bench_rt.json 2> $R/$OUT/rt.err || { tail -20 $R/$OUT/rt.err; exit 1; }
cd $R
python3 tools/prof_roundtrip.py $OUT/rt/run_kernel_trace.csv $OUT/bench_rt.json | python3 -c "
import json,sys; d=json.load(sys.stdin)
for k,v in d['legs'].items(): print(k, v.get('rocprof_avg_us'), v.get('error',''))"
