#!/usr/bin/env python3
"""Average rocprofv3 --pmc counters per (kernel, grid) for gf_bs_kernel
launches (median per launch) and the derived fractions of SQ_WAVE_CYCLES:
waiting on dependencies (SQ_WAIT_ANY), on instruction fetch
(SQ_WAIT_INST_ANY), issuing (SQ_ACTIVE_INST_ANY).  usage: pmc_sq_grid.py DIR"""
import collections
import csv
import glob
import os
import statistics
import sys

root = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "gf_bs_kernel" not in r["Kernel_Name"]:
            continue
        key = (r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0][-40:], r["Grid_Size"])
        acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for key, cs in sorted(acc.items(), key=lambda kv: -len(next(iter(kv[1].values())))):
    m = {c: statistics.median(v) for c, v in cs.items()}
    n = max(len(v) for v in cs.values())
    line = f"{key[0]} grid {key[1]} launches {n}: " + ", ".join(f"{c} {m[c]:.4g}" for c in sorted(m))
    wc = m.get("SQ_WAVE_CYCLES")
    if wc:
        fr = {c: m[c] / wc for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY") if c in m}
        line += " | of wave-cycles: " + ", ".join(f"{c} {v:.3f}" for c, v in fr.items())
    print(line)
