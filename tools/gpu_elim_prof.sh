#!/bin/bash
# kernel durations of the GPU elimination (blocked and per-step), k = 32-256, G = 1 and 32
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/elim_prof"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for B in 1 0; do
  KODR_ELIM_BLOCKED=$B timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/b$B" -o run --output-format csv -- \
    python3 "$R/tools/elim_time.py" 32,64,128,256 1,32 > "$OUT/b$B.log" 2>&1 || { tail -5 "$OUT/b$B.log"; exit 1; }
  cat "$OUT/b$B.log"
  python3 - "$OUT/b$B" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if "elim" in r["Kernel_Name"]:
        d[(r["Kernel_Name"][:60], r.get("Grid_Size_X", r.get("Grid_Size", "")), r.get("LDS_Block_Size", ""))].append(
            (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for key, v in d.items():
    v.sort()
    print(key, "n", len(v), "median us", v[len(v) // 2])
PY
done
