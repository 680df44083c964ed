#!/bin/bash
# C2 single-decoder AddPiece phases (KODR_ADD_TIMING=1) and the kernel trace
# of the same run (the elimination's duration per call)
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-c2ph}; mkdir -p $OUT
KODR_ADD_TIMING=1 timeout -k 10 120 python -u tools/c2_add_phases.py 12 11 > $OUT/phases.log 2>&1 || { tail -20 $OUT/phases.log; exit 1; }
grep -E "add_pieces_gpu G=1|rep" $OUT/phases.log | tail -12
R=$(pwd)
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/$OUT/tr -o run --output-format csv -- python3 $R/tools/c2_add_phases.py 12 11 > $R/$OUT/tr.log 2>&1 || { tail -20 $R/$OUT/tr.log; exit 1; }
cd $R
python3 - $OUT/tr/run_kernel_trace.csv <<'PY'
import csv, sys, statistics, collections
g = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    g[r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-60:]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(g.items(), key=lambda kv: -sum(kv[1]))[:8]:
    print(f"{k:60s} n={len(v):3d} median {statistics.median(v):8.2f} us")
PY
