#!/bin/bash
# gf_gemv_kernel with non-temporal row loads (KODR_GEMV=3) against the default
# (2): parity, interleaved events, rocprof kernel durations.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-b1c}; mkdir -p $OUT
KODR_GEMV=3 timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "matmul or encode_vs or headline_launch or c2_roundtrip" --timeout 300 --timeout-method thread > $OUT/tests_gemv3.log 2>&1 || { tail -30 $OUT/tests_gemv3.log; exit 1; }
tail -1 $OUT/tests_gemv3.log
for rep in 1 2 3; do
  for G in 2 3; do
    KODR_GEMV=$G timeout -k 10 180 python -u tools/b1_ab.py > $OUT/gemv${G}_r$rep.log 2>&1 || { tail -20 $OUT/gemv${G}_r$rep.log; exit 1; }
    echo "gemv=$G rep $rep $(tail -1 $OUT/gemv${G}_r$rep.log)"
  done
done
for G in 2 3; do
  KODR_GEMV=$G timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/prof_gemv$G -o run --output-format csv -- python3 tools/b1_ab.py > $OUT/prof_gemv$G.log 2>&1 || { tail -20 $OUT/prof_gemv$G.log; exit 1; }
done
python3 - $OUT <<'PY'
import csv, glob, statistics, sys
o = sys.argv[1]
for G in (2, 3):
    f = glob.glob(f"{o}/prof_gemv{G}/**/*kernel_trace.csv", recursive=True)
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(f[0])) if "gemv" in r["Kernel_Name"]]
    print(f"gemv={G} rocprof gf_gemv_kernel n={len(d)} median {statistics.median(d) / 1e3:.2f} us")
PY
