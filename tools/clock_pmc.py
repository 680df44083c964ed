#!/usr/bin/env python3
"""Effective GPU clock during each kernel of a rocprofv3 --pmc GRBM_GUI_ACTIVE
GRBM_COUNT run: GUI_ACTIVE cycles / the dispatch's duration, per (kernel,
grid), launches with >= MIN_US duration.  usage: clock_pmc.py DIR [MIN_US]"""
import collections
import csv
import glob
import os
import statistics
import sys

d = sys.argv[1]
min_us = float(sys.argv[2]) if len(sys.argv) > 2 else 20.0
per = collections.defaultdict(dict)
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        key = (r["Dispatch_Id"], r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-60:],
               int(r["Grid_Size"]))
        per[key][r["Counter_Name"]] = float(r["Counter_Value"])
        per[key]["us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
groups = collections.defaultdict(list)
for (disp, name, grid), v in per.items():
    if v["us"] >= min_us and "GRBM_GUI_ACTIVE" in v:
        groups[(name, grid)].append(v)
for (name, grid), vs in sorted(groups.items(), key=lambda kv: -len(kv[1])):
    us = statistics.median(v["us"] for v in vs)
    ga = statistics.median(v["GRBM_GUI_ACTIVE"] for v in vs)
    gc = statistics.median(v.get("GRBM_COUNT", 0) for v in vs)
    print(f"{name:60s} grid {grid:9d} n {len(vs):4d} median {us:8.2f} us  GUI_ACTIVE {ga:12.0f} "
          f"COUNT {gc:12.0f}  GUI_ACTIVE/us {ga / us / 1e3:7.3f} G/s  COUNT/us {gc / us / 1e3:7.3f} G/s")
