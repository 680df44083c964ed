#!/bin/bash
# Kernel trace of the C4 decode probe (tools/c4_probe.py): which kernels make
# up one decode, with start offsets and durations of the last 40 launches.
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/c4trace"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
  python3 "$R/tools/c4_probe.py" > "$OUT/c4.json" 2> "$OUT/c4.err" || { tail -20 "$OUT/c4.err"; exit 1; }
cat "$OUT/c4.json"
python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/trace/**/*kernel_trace.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
for r in rows[-40:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f'{(s - t0) / 1e3:10.1f} us  {(e - s) / 1e3:7.2f} us  {r["Kernel_Name"][:90]}')
PY
