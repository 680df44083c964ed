#!/usr/bin/env python3
"""Timeline of the round trip's AddPiece kernels in a rocprofv3 kernel trace:
for the last N steps, the elimination (gf_elim_mc*, grid y = 16) and the
rows' twin copy (copy_bitslice_grouped) starts and ends relative to the end
of the grouped encode launch before them.  usage: rt_timeline.py TRACE [N]"""
import csv
import sys

rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r["Grid_Size_Y"]))
               for r in csv.DictReader(open(sys.argv[1]))), key=lambda x: x[0])
n = int(sys.argv[2]) if len(sys.argv) > 2 else 5
elim = [r for r in rows if "gf_elim_mc" in r[2] and r[3] == 16]
out = []
for e in elim:
    prev = [r for r in rows if "gf_bs_kernel" in r[2] and r[1] <= e[0] + 1000]
    cp = [r for r in rows if "copy_bitslice_grouped" in r[2] and abs(r[0] - e[0]) < 2_000_000]
    if not prev or not cp:
        continue
    t0 = prev[-1][1]
    c = min(cp, key=lambda r: abs(r[0] - e[0]))
    nxt = [r for r in rows if "gf_bs_kernel" in r[2] and r[0] >= max(e[1], c[1]) - 1000]
    out.append((e[0] - t0, e[1] - t0, c[0] - t0, c[1] - t0, (nxt[0][0] - t0) if nxt else -1))
for o in out[-n:]:
    print("elim %7.1f .. %7.1f us | copy %7.1f .. %7.1f us | next launch %7.1f" % tuple(x / 1e3 for x in o))
