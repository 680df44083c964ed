#!/bin/bash
# kernel traces of the round trip (bench.py --no-extras) for this tree and
# r5lib_pre: the AddPiece timeline per step and the runtime's own copy kernels
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-rttr}; mkdir -p $OUT
R=$(pwd)
cd /tmp
for v in new pre; do
  libp=$R/kodr_amd/libkodr_rlnc.so; [ $v = pre ] && libp=$R/kodr_amd/r5lib_pre/libkodr_rlnc.so
  KODR_RLNC_LIB=$libp timeout -k 10 300 rocprofv3 --kernel-trace -d $R/$OUT/tr_$v -o run --output-format csv -- python3 $R/bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline > $R/$OUT/tr_$v.json 2> $R/$OUT/tr_$v.err || { tail -20 $R/$OUT/tr_$v.err; exit 1; }
  echo "== $v"; python3 $R/tools/rt_timeline.py $R/$OUT/tr_$v/run_kernel_trace.csv 3
  python3 - $R/$OUT/tr_$v/run_kernel_trace.csv <<'PY'
import csv, sys, collections, statistics
rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(sys.argv[1]))))
c = collections.Counter(r[2][:40] for r in rows if "rocclr" in r[2])
print("runtime kernels:", dict(c))
# step period: starts of the grouped encode launches (grid y 16, B = 258 plan) over the last 10
enc = [r for r in rows if "gf_bs_kernel<4, 0, true" in r[2]]
st = [b[0] - a[0] for a, b in zip(enc[-11:], enc[-10:])]
print("step period us (last 10):", [round(x / 1e3, 1) for x in st])
PY
done
