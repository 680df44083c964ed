#!/bin/bash
# Multi-workgroup elimination (gf_elim_mc_kernel): parity of the elimination
# and decode tests under it, then one decoder's batched AddPiece and the
# 16-decoder batched AddPiece, mc (KODR_ELIM_MC=1) against the one-workgroup
# circular kernel (0), and a kernel trace of each.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-mc}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_elim.py tests/test_gpu_lazy_decode.py tests/test_gpu_group_decode.py tests/test_gpu_headline.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
echo "tests $(tail -1 $OUT/tests.log)"
for rep in 1 2; do
  for M in ${MC_MODES:-1 2}; do
    KODR_ELIM_MC=$M timeout -k 10 120 python -u tools/elim_time.py 64,128,256 1,16 > $OUT/e_m${M}_r$rep.log 2>&1 || { tail -20 $OUT/e_m${M}_r$rep.log; exit 1; }
    echo "mc=$M rep $rep:"; cat $OUT/e_m${M}_r$rep.log
  done
done
KODR_ADD_TIMING=1 timeout -k 10 120 python -u tools/elim_time.py 256 1 > $OUT/phases.log 2>&1 || { tail -20 $OUT/phases.log; exit 1; }
tail -3 $OUT/phases.log
for M in ${MC_MODES:-1 2}; do
  KODR_ELIM_MC=$M timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof_m$M -o run --output-format csv -- python3 tools/elim_time.py 256 1,16 > $OUT/prof_m$M.log 2>&1 || { tail -20 $OUT/prof_m$M.log; exit 1; }
done
python3 - $OUT <<'PY'
import csv, glob, statistics, sys
o = sys.argv[1]
for M in [int(x) for x in __import__("os").environ.get("MC_MODES", "1 2").split()]:
    f = glob.glob(f"{o}/prof_m{M}/**/*kernel_trace.csv", recursive=True)
    d = {}
    for r in csv.DictReader(open(f[0])):
        if "elim" in r["Kernel_Name"]:
            d.setdefault(r["Kernel_Name"].split("(")[0][-40:], []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for n, v in d.items():
        print(f"mc={M} {n}: n={len(v)} min {min(v):.1f} median {statistics.median(v):.1f} max {max(v):.1f} us")
PY
