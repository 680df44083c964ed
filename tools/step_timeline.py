#!/usr/bin/env python3
"""Per-step kernel timeline of the round trip in a rocprofv3 kernel trace
(tools/gpu_r6_val.sh): for each of the first N eliminations of 16 decoders
(gf_elim_mc*, grid y = 16) from the index FIRST on, every kernel that starts
between it and the next one, as (start, end) in us relative to the
elimination's start, and the step length.  Shows what runs beside what in
the pipelined step (the next encode beside the elimination and the twin
copy, GetPieces after it) and the gaps.

  python tools/step_timeline.py run_kernel_trace.csv [FIRST] [N]"""
import csv
import sys

rows = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], int(r["Grid_Size_X"]),
                int(r["Grid_Size_Y"])) for r in csv.DictReader(open(sys.argv[1]))), key=lambda x: x[0])
first = int(sys.argv[2]) if len(sys.argv) > 2 else 0
n = int(sys.argv[3]) if len(sys.argv) > 3 else 5


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("kodr_amd::", "").replace("void ", "")
    return name.split("(")[0][:34]


elim = [r for r in rows if "gf_elim_mc" in r[2] and r[4] == 16]
for i in range(first, min(first + n, len(elim) - 1)):
    t0, t1 = elim[i][0], elim[i + 1][0]
    print(f"step {i}: {(t1 - t0) / 1e3:8.1f} us to the next elimination")
    for r in rows:
        if t0 <= r[0] < t1 or (r[0] < t0 < r[1]):
            print(f"   {short(r[2]):34s} grid {r[3]:7d} x {r[4]:2d}  {(r[0] - t0) / 1e3:8.1f} .. {(r[1] - t0) / 1e3:8.1f}")
