#!/bin/bash
# Quick loop for gf_elim_mc_kernel: elimination parity, its timeline (tuning
# build), one and 16 decoders' batched AddPiece, rocprof kernel durations.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-mcq}; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_elim.py -x -q -m gpu --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
echo "tests $(tail -1 $OUT/tests.log)"
[ -n "${MC_PHASES:-}" ] && { bash tools/gpu_mc_phases.sh ${1:-mcq} || exit 1; }
timeout -k 10 120 python -u tools/elim_time.py 256 1,16 > $OUT/e.log 2>&1 || { tail -20 $OUT/e.log; exit 1; }
cat $OUT/e.log
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 tools/elim_time.py 256 1,16 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python3 - $OUT <<'PY'
import csv, glob, statistics, sys
o = sys.argv[1]
f = glob.glob(f"{o}/prof/**/*kernel_trace.csv", recursive=True)
d = {}
for r in csv.DictReader(open(f[0])):
    if "elim" in r["Kernel_Name"]:
        d.setdefault(r["Kernel_Name"].split("(")[0][-40:], []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for n, v in d.items():
    print(f"{n}: n={len(v)} min {min(v):.1f} median {statistics.median(v):.1f} max {max(v):.1f} us")
PY
