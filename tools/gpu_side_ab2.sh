#!/bin/bash
# round 5: the round trip with the row copies beside the elimination (side
# stream, this tree) or ahead of it on the context stream (KODR_ADD_SIDE=0,
# tuning build kodr_amd/tune_c/), and r5lib_pre (before the vector download
# and the shared rows_ready event), interleaved; then timelines
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-sideab2}; mkdir -p $OUT
run() {  # tag lib side
  KODR_ADD_SIDE=$3 KODR_RLNC_LIB=$2 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > $OUT/b_$1.json 2> $OUT/b_$1.err || { tail -20 $OUT/b_$1.err; return 1; }
  python3 - $OUT/b_$1.json $1 <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
lg = d["roofline"]["legs"]
print(sys.argv[2], "rt us/gen", d["roundtrip"]["us_per_generation"], "add", lg["add_pieces_call"]["avg_us"], "ok", d["roundtrip"]["roundtrip_ok"])
PY
}
for rep in 1 2 3; do
  run pre_$rep kodr_amd/r5lib_pre/libkodr_rlnc.so 1 || exit 1
  run new_$rep kodr_amd/libkodr_rlnc.so 1 || exit 1
  run after_$rep kodr_amd/tune_c/libkodr_rlnc.so 2 || exit 1
done
R=$(pwd)
cd /tmp
for v in new:1 after:2; do
  t=${v%%:*}; sd=${v##*:}
  libp=$R/kodr_amd/libkodr_rlnc.so; [ $t = after ] && libp=$R/kodr_amd/tune_c/libkodr_rlnc.so
  KODR_ADD_SIDE=$sd KODR_RLNC_LIB=$libp timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/tr_$t -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > $R/$OUT/tr_$t.json 2> $R/$OUT/tr_$t.err || { tail -20 $R/$OUT/tr_$t.err; exit 1; }
  echo "== $t"; python3 $R/tools/rt_timeline.py $R/$OUT/tr_$t/run_kernel_trace.csv 3
done
