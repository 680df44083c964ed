#!/usr/bin/env python3
"""HBM bytes per launch of the round trip's grouped encode (bench.py's value
leg: G generations x k + 2 coded pieces in one gf_bs_kernel launch) from two
rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE; MI355X_MICROARCH.md HBM
section: KB units, FETCH_SIZE x2 on gfx950 for wide streaming reads) of
`bench.py --no-extras --no-cpu-baseline` (tools/gpu_r5_val.sh).  The launches
are those whose grid is the kernel instance the bench line's
roofline.legs.encode_launch.plan records.

  python tools/pmc_roundtrip.py <OUT dir with fetch/ write/> <bench.json>"""
import csv
import glob
import json
import os
import statistics
import sys

out, bj = sys.argv[1], sys.argv[2]
line = json.loads([x for x in open(bj) if x.startswith("{")][-1])
plan = line["roofline"]["legs"]["encode_launch"]["plan"]
grid = plan["workgroups"] * 64 * plan["waves"] * plan["generations"]
G, k, L = line["config"]["generations_per_step"], line["config"]["piece_count"], line["config"]["piece_size"]
n = k + 2


sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from rt_roles import get_ids  # noqa: E402


def vals(sub, counter):
    """the counter per encode launch (GetPieces may share the grid: tools/rt_roles.py)"""
    rows = {}
    for f in glob.glob(os.path.join(out, sub, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            key = (int(r["Dispatch_Id"]), int(r["Grid_Size"]))
            kind = "bs" if "gf_bs_kernel" in r["Kernel_Name"] else "copy" if "copy_bitslice" in r["Kernel_Name"] else ""
            rows.setdefault(key, [kind, None])
            if r["Counter_Name"] == counter:
                rows[key][1] = float(r["Counter_Value"])
    keys = sorted(rows)
    gets = get_ids(keys, lambda x: x[1] if rows[x][0] == "bs" else None, lambda x: rows[x][0] == "copy", lambda x: x)
    return [rows[x][1] for x in keys if rows[x][0] == "bs" and x[1] == grid and x not in gets and rows[x][1] is not None]


fetch, write = vals("fetch", "FETCH_SIZE"), vals("write", "WRITE_SIZE")
rd = int(statistics.mean(fetch) * 1024 * 2)
wr = int(statistics.mean(write) * 1024)
compulsory = G * (k * L + n * k + n * L)
print(json.dumps({
    "launch": f"round-trip grouped encode, G = {G}, B = k + 2 = {n}, k = {k}, L = {L}",
    "plan": plan, "counter_grid_threads": grid, "counter_launches": [len(fetch), len(write)],
    "fetch_size_kb_per_launch_raw": round(statistics.mean(fetch), 1),
    "write_size_kb_per_launch": round(statistics.mean(write), 1),
    "hbm_read_bytes_per_launch": rd, "hbm_write_bytes_per_launch": wr, "hbm_bytes_per_launch": rd + wr,
    "compulsory_bytes_per_launch": compulsory, "traffic_over_compulsory": round((rd + wr) / compulsory, 4),
    "source": "tools/gpu_r6_val.sh: rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE of bench.py --steps 20 "
              "--warmup 5 --no-extras --no-cpu-baseline"}, indent=1))
