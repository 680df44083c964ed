#!/bin/bash
# GPU elimination: the circular one-dword-per-lane kernel (KODR_ELIM_CIRC=1)
# against the [C | T] blocked kernel (0): parity under the new default, then
# interleaved timings (tools/elim_time.py: G = 1 and 16 at k = 256; the
# batched AddPiece at 32 MiB/256 over 16 decoders) and a kernel trace.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-elim_ab}; mkdir -p $OUT
VARIANTS=${2:-"0 1"}
TESTV=${3:-1}
KODR_ELIM_CIRC=$TESTV timeout -k 10 400 python -u -m pytest tests/test_gpu_elim.py tests/test_gpu_group_decode.py tests/test_gpu_lazy_decode.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
echo "tests $(tail -1 $OUT/tests.log)"
for rep in 1 2; do
  for C in $VARIANTS; do
    KODR_ELIM_CIRC=$C timeout -k 10 200 python -u tools/elim_time.py 128,256 1,16 > $OUT/e_c${C}_r$rep.log 2>&1 || { tail -20 $OUT/e_c${C}_r$rep.log; exit 1; }
    KODR_ELIM_CIRC=$C timeout -k 10 120 python -u tools/group_add_time.py 16 > $OUT/a_c${C}_r$rep.log 2>&1 || { tail -20 $OUT/a_c${C}_r$rep.log; exit 1; }
    echo "circ=$C rep $rep: $(cat $OUT/e_c${C}_r$rep.log | tr '\n' ' ') | $(tail -1 $OUT/a_c${C}_r$rep.log)"
  done
done
for C in $VARIANTS; do
  KODR_ELIM_CIRC=$C timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof_c$C -o run --output-format csv -- python3 tools/group_add_time.py 16 > $OUT/prof_c$C.log 2>&1 || { tail -20 $OUT/prof_c$C.log; exit 1; }
done
python3 - $OUT "$VARIANTS" <<'PY'
import csv, glob, statistics, sys
o = sys.argv[1]
for C in sys.argv[2].split():
    f = glob.glob(f"{o}/prof_c{C}/**/*kernel_trace.csv", recursive=True)
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(f[0])) if "elim" in r["Kernel_Name"]]
    print(f"circ={C} rocprof elimination kernel n={len(d)} median {statistics.median(d) / 1e3:.1f} us")
PY
