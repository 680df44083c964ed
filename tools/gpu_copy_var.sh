#!/bin/bash
# round 5: the twin copy beside the elimination, workgroups per CU of the
# chunked copy (tuning build kodr_amd/tune_c/, KODR_COPY_WG_PER_CU) against
# the round-4 grid-stride copy (kodr_amd/r5lib_pre/), bench.py round trip
# (--no-extras) interleaved, then kernel-trace timelines of two of them
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-copyvar}; mkdir -p $OUT
run() {  # tag lib wg
  KODR_COPY_WG_PER_CU=$3 KODR_RLNC_LIB=$2 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > $OUT/b_$1.json 2> $OUT/b_$1.err || { tail -20 $OUT/b_$1.err; return 1; }
  python3 - $OUT/b_$1.json $1 <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
lg = d["roofline"]["legs"]
print(sys.argv[2], "rt us/gen", d["roundtrip"]["us_per_generation"], "add", lg["add_pieces_call"]["avg_us"], "ok", d["roundtrip"]["roundtrip_ok"])
PY
}
for rep in 1 2; do
  run pre_$rep kodr_amd/r5lib_pre/libkodr_rlnc.so 4 || exit 1
  for wg in 2 4 8; do run c${wg}_$rep kodr_amd/tune_c/libkodr_rlnc.so $wg || exit 1; done
done
R=$(pwd)
cd /tmp
for v in pre:4 c:8 c:4; do
  t=${v%%:*}; wg=${v##*:}
  libp=$R/kodr_amd/tune_c/libkodr_rlnc.so; [ $t = pre ] && libp=$R/kodr_amd/r5lib_pre/libkodr_rlnc.so
  KODR_COPY_WG_PER_CU=$wg KODR_RLNC_LIB=$libp timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/tr_${t}$wg -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > $R/$OUT/tr_${t}$wg.json 2> $R/$OUT/tr_${t}$wg.err || { tail -20 $R/$OUT/tr_${t}$wg.err; exit 1; }
  echo "== $t wg $wg"; python3 $R/tools/rt_timeline.py $R/$OUT/tr_${t}$wg/run_kernel_trace.csv 4
done
