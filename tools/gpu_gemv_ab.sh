#!/bin/bash
# gf_gemv_kernel variants (KODR_GEMV): parity under each, interleaved events
# (tools/b1_ab.py), rocprof kernel durations.  Usage: gpu_gemv_ab.sh OUT "2 5 6 7"
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-gemv_ab}; mkdir -p $OUT
VARIANTS=${2:-"2 5"}
for G in $VARIANTS; do
  KODR_GEMV=$G timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "gemv or c2_roundtrip or encode_batch_full" --timeout 200 --timeout-method thread > $OUT/tests_gemv$G.log 2>&1 || { tail -30 $OUT/tests_gemv$G.log; exit 1; }
  echo "gemv=$G $(tail -1 $OUT/tests_gemv$G.log)"
done
for rep in 1 2; do
  for G in $VARIANTS; do
    KODR_GEMV=$G timeout -k 10 180 python -u tools/b1_ab.py > $OUT/gemv${G}_r$rep.log 2>&1 || { tail -20 $OUT/gemv${G}_r$rep.log; exit 1; }
    echo "gemv=$G rep $rep $(tail -1 $OUT/gemv${G}_r$rep.log)"
  done
done
for G in $VARIANTS; do
  KODR_GEMV=$G timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/prof_gemv$G -o run --output-format csv -- python3 tools/b1_ab.py > $OUT/prof_gemv$G.log 2>&1 || { tail -20 $OUT/prof_gemv$G.log; exit 1; }
done
python3 - $OUT "$VARIANTS" <<'PY'
import csv, glob, statistics, sys
o = sys.argv[1]
for G in sys.argv[2].split():
    f = glob.glob(f"{o}/prof_gemv{G}/**/*kernel_trace.csv", recursive=True)
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(f[0])) if "gemv" in r["Kernel_Name"]]
    print(f"gemv={G} rocprof gf_gemv_kernel n={len(d)} median {statistics.median(d) / 1e3:.2f} us")
PY
