#!/bin/bash
# Per-launch durations of the grouped headline launch in order (rocprofv3
# kernel trace of bench.py --no-extras), to see whether the first timed
# launches run slower than steady state (clock ramp after an idle GPU).
set -uo pipefail
R="${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}"
OUT="$R/gpurun_out/warm"; mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
for W in 5 200; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/w$W" -o run --output-format csv -- \
    python3 "$R/bench.py" --no-extras --cpu-seconds 2 --steps 20 --warmup $W > "$OUT/bench_w$W.json" 2> "$OUT/w$W.err" \
    || { tail -20 "$OUT/w$W.err"; exit 1; }
  python3 - "$OUT/w$W" <<'PY'
import csv, glob, sys
rows = []
for f in glob.glob(sys.argv[1] + "/**/*kernel_trace.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows
     if "gf_bs_kernel" in r["Kernel_Name"] and int(r["Grid_Size_Y"]) > 1]
print(len(d), "launches; first 10:", [round(x, 1) for x in d[:10]], "last 20 avg:", round(sum(d[-20:]) / 20, 1))
PY
  python3 -c "import json,sys; l=json.loads(open('$OUT/bench_w$W.json').read().strip().splitlines()[-1]); print('W', $W, l['value'], l['roofline']['avg_launch_us'])"
done
