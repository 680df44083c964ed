#!/bin/bash
# A/B of the blocked elimination's panel step (KODR_ELIM_GJ 0/1) on one box:
# kernel durations (rocprofv3) and wall time per call
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/elim_gj"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for V in 0 1 0 1; do
  KODR_ELIM_GJ=$V timeout -k 10 120 rocprofv3 --kernel-trace -d "$OUT/v$V" -o run --output-format csv -- \
    python3 "$R/tools/elim_time.py" 256 1,32 > "$OUT/v$V.log" 2>&1 || { tail -5 "$OUT/v$V.log"; exit 1; }
  python3 - "$OUT/v$V" "$V" <<'PY'
import csv, glob, sys
f = sorted(glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True))[-1]
v = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in csv.DictReader(open(f))
           if "elim_blocked" in r["Kernel_Name"])
print("GJ", sys.argv[2], "blocked kernel n", len(v), "median us", v[len(v) // 2] if v else None)
PY
  grep '"k"' "$OUT/v$V.log"
done
