#!/bin/bash
# gf_elim_mc4_kernel (KODR_ELIM_MC=4): elimination and lazy-decode parity
# under it (the single-decoder route forced on), then one and 16 decoders'
# batched AddPiece against mc2, two interleaved reps,
# and a kernel trace of both.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-mc4}; mkdir -p $OUT
KODR_ELIM_MC=4 KODR_ROUTE_MIN_K=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_elim.py tests/test_gpu_lazy_decode.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
echo "tests (mc4) $(tail -1 $OUT/tests.log)"
for rep in 1 2; do
  for M in 2 4; do
    KODR_ELIM_MC=$M timeout -k 10 120 python -u tools/elim_time.py 64,128,256 1,4 > $OUT/e_${M}_r$rep.log 2>&1 || { tail -20 $OUT/e_${M}_r$rep.log; exit 1; }
    echo "mc=$M rep $rep: $(python3 -c "import json,sys; print(' '.join(f\"k{d['k']}G{d['G']} {d['gpu_us']}/{d['host_us']}\" for d in map(json.loads, open(sys.argv[1]))))" $OUT/e_${M}_r$rep.log)"
  done
done
for M in 2 4; do
  KODR_ELIM_MC=$M timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof_m$M -o run --output-format csv -- python3 tools/elim_time.py 256 1 > $OUT/prof_m$M.log 2>&1 || { tail -20 $OUT/prof_m$M.log; exit 1; }
done
python3 - $OUT <<'PY'
import csv, glob, statistics, sys
o = sys.argv[1]
for M in (2, 4):
    f = glob.glob(f"{o}/prof_m{M}/**/*kernel_trace.csv", recursive=True)
    d = {}
    for r in csv.DictReader(open(f[0])):
        if "elim" in r["Kernel_Name"]:
            d.setdefault(r["Kernel_Name"].split("(")[0][-30:], []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for n, v in d.items():
        print(f"mc={M} {n}: n={len(v)} min {min(v):.1f} median {statistics.median(v):.1f} max {max(v):.1f} us")
PY
