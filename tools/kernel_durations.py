"""Median rocprofv3 kernel durations (us) by kernel name and grid from one or
more --kernel-trace --output-format csv directories.  usage:
kernel_durations.py DIR [DIR ...]"""
import collections
import csv
import glob
import json
import statistics
import sys

for d in sys.argv[1:]:
    f = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
    if not f:
        print(d, "no trace")
        continue
    c = collections.defaultdict(list)
    for r in csv.DictReader(open(f[0])):
        name = r["Kernel_Name"].replace("void ", "").replace("kodr_amd::(anonymous namespace)::", "").split("(")[0]
        c[(name, r["Grid_Size_X"], r["Grid_Size_Y"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = {f"{k[0]} grid {k[1]}x{k[2]}": {"n": len(v), "median_us": round(statistics.median(v), 2)}
           for k, v in sorted(c.items(), key=lambda kv: -sum(kv[1]))[:8]}
    print(d, json.dumps(out))
