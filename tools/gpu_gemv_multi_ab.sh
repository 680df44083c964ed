#!/bin/bash
# gf_gemv_multi_kernel (2..4 coded pieces per call, KODR_GEMV_MULTI=1) against
# gf_gemm_kernel (0): parity, interleaved events (tools/b1_ab.py B = 1, 2, 4),
# rocprof kernel durations.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-gemv_multi_ab}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_api.py tests/test_gpu_elim.py -x -q -m gpu --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
echo "tests $(tail -1 $OUT/tests.log)"
for rep in 1 2 3; do
  for V in 0 1; do
    KODR_GEMV_MULTI=$V timeout -k 10 180 python -u tools/b1_ab.py > $OUT/m${V}_r$rep.log 2>&1 || { tail -20 $OUT/m${V}_r$rep.log; exit 1; }
    echo "multi=$V rep $rep $(tail -1 $OUT/m${V}_r$rep.log)"
  done
done
for V in 0 1; do
  KODR_GEMV_MULTI=$V timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $OUT/prof_m$V -o run --output-format csv -- python3 tools/b1_ab.py > $OUT/prof_m$V.log 2>&1 || { tail -20 $OUT/prof_m$V.log; exit 1; }
done
python3 - $OUT <<'PY'
import csv, glob, statistics, sys, collections
o = sys.argv[1]
for V in (0, 1):
    f = glob.glob(f"{o}/prof_m{V}/**/*kernel_trace.csv", recursive=True)
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        if "gemv" in r["Kernel_Name"] or "gf_gemm_kernel" in r["Kernel_Name"]:
            d[r["Kernel_Name"].split("(")[0][-60:]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    for k, v in d.items():
        print(f"multi={V} {k}: n={len(v)} median {statistics.median(v) / 1e3:.2f} us")
PY
