#!/bin/bash
# Kernel trace of the bench's encode_decode round trip (headline steps kept short).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ed_prof}; mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-extras --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 - $OUT <<'PY'
import csv, glob, sys, json
o = sys.argv[1]
f = glob.glob(f"{o}/prof/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
# the encode_decode section: from the first gf_elim launch back to the wire encode before it, to the end
names = [r["Kernel_Name"] for r in rows]
ie = max(i for i, n in enumerate(names) if "elim" in n)
i0 = ie
while i0 > 0 and not ("gf_bs_kernel" in names[i0] and int(rows[i0]["Grid_Size_Y"] if "Grid_Size_Y" in rows[i0] else 1) >= 1 and i0 < ie - 2):
    i0 -= 1
t0 = int(rows[max(0, ie - 12)]["Start_Timestamp"])
for r in rows[max(0, ie - 12):]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(s - t0) / 1e3:10.1f} us  dur {(e - s) / 1e3:9.1f} us  {r['Kernel_Name'][:110]}")
print(json.load(open(f"{o}/bench.json"))["encode_decode"])
PY
