#!/usr/bin/env python3
"""VALU instructions, wave count and clock per launch of the round trip's two
gf_bs_kernel legs (the encode launch and the grouped GetPieces) from one
rocprofv3 --pmc pass of the driver's bench command (SQ_INSTS_VALU
SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT; no tracing domains), and
the hardware VALU-busy fraction each implies (over every launch, and over
the serial phase's launches -- the ones the line's legs are timed on):

  SIMD-cycles of a launch  = 1,024 SIMDs x GRBM_GUI_ACTIVE / 8
                             (GRBM_GUI_ACTIVE sums the 8 XCDs' busy cycles,
                             MI355X_MICROARCH.md "DVFS give-back")
  VALU-busy                = SQ_INSTS_VALU x 2 / SIMD-cycles
                             (a wave64 VALU instruction holds a SIMD-32 for 2
                             cycles, MI355X_MICROARCH.md wave scheduling)
  VALU-busy at 2.4 GHz     = SQ_INSTS_VALU x 2 / (1,024 x 2.4e9 x duration)

The launches are those whose grid is the kernel instance the bench line
(same run) records in roofline.legs.*.plan.  Writes the JSON that bench.py
reads (profiles/pmc_valu_G{G}_k{k}_L{L}.json) to stdout.

  python tools/pmc_valu.py <pmc dir> <bench.json>"""
import collections
import csv
import glob
import json
import os
import statistics
import sys

SIMDS, NOMINAL_HZ = 1024, 2.4e9

d, bj = sys.argv[1], sys.argv[2]
line = json.loads([x for x in open(bj) if x.startswith("{")][-1])
legs = line["roofline"]["legs"]
G, k, L = line["config"]["generations_per_step"], line["config"]["piece_count"], line["config"]["piece_size"]
rt = line.get("roundtrip", {})

per = collections.defaultdict(dict)
kind = {}
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        key = (int(r["Dispatch_Id"]), int(r["Grid_Size"]))
        kind[key] = ("bs" if "gf_bs_kernel" in r["Kernel_Name"] else
                     "copy" if "copy_bitslice" in r["Kernel_Name"] else "other")
        if kind[key] != "bs":
            continue
        per[key][r["Counter_Name"]] = float(r["Counter_Value"])
        if r.get("Start_Timestamp") and r.get("End_Timestamp"):
            per[key]["us"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
# GetPieces and the encode's bit-sliced launch may share a grid (tools/rt_roles.py)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from rt_roles import get_ids  # noqa: E402
getset = get_ids(sorted(kind), lambda x: x[1] if kind[x] == "bs" else None, lambda x: kind[x] == "copy",
                 lambda x: x)

out = {"source": "rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT of "
                 "bench.py --steps 20 --warmup 5 --no-extras --no-cpu-baseline (tools/gpu_r6_val.sh)",
       "simds": SIMDS, "cycles_per_wave64_valu": 2, "nominal_clock_hz": NOMINAL_HZ}
for leg, macs in (("encode_launch", G * (k + 2) * k * L), ("get_pieces_call", G * k * k * L)):
    plan = legs[leg]["plan"]
    grid = plan["workgroups"] * 64 * plan["waves"] * plan["generations"]
    want_get = leg == "get_pieces_call"
    ordered = [(key, v) for key, v in sorted(per.items()) if key[1] == grid and "SQ_INSTS_VALU" in v and
               (key in getset) == want_get]
    vs = [v for _, v in ordered]
    if not vs:
        continue
    med = {c: statistics.median(v[c] for v in vs if c in v)
           for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_WAVES", "GRBM_GUI_ACTIVE", "GRBM_COUNT", "us")
           if any(c in v for v in vs)}
    # the serial phase the line's legs are timed in: every launch after the
    # pipelined phase (its warmup encodes / steps and its timed steps)
    n_pipe = (rt.get("warmup_encodes_run", 0) if not want_get else rt.get("warmup_steps_run", 0)) + line["steps"]
    ser = [v for v in vs[n_pipe:] if "us" in v]
    e = {"plan": plan, "counter_grid_threads": grid, "launches": len(vs),
         "valu_insts_per_launch": int(med["SQ_INSTS_VALU"]), "salu_insts_per_launch": int(med.get("SQ_INSTS_SALU", 0)),
         "waves_per_launch": int(med.get("SQ_WAVES", 0)), "gf_macs_per_launch": macs,
         "gf_macs_per_valu_inst": round(macs / med["SQ_INSTS_VALU"], 2)}
    if "GRBM_GUI_ACTIVE" in med:
        simd_cycles = SIMDS * med["GRBM_GUI_ACTIVE"] / 8
        e["grbm_gui_active_per_launch"] = int(med["GRBM_GUI_ACTIVE"])
        e["valu_busy_at_measured_clock"] = round(med["SQ_INSTS_VALU"] * 2 / simd_cycles, 4)
        if "us" in med:
            e["pmc_launch_us"] = round(med["us"], 2)
            e["clock_ghz"] = round(med["GRBM_GUI_ACTIVE"] / 8 / (med["us"] * 1e3), 3)
            e["valu_busy_at_nominal_clock"] = round(med["SQ_INSTS_VALU"] * 2 / (SIMDS * NOMINAL_HZ * med["us"] * 1e-6), 4)
    if ser:
        us = statistics.median(v["us"] for v in ser)
        e["serial_phase"] = {
            "launches": len(ser), "pmc_launch_us": round(us, 2),
            "valu_busy_at_nominal_clock": round(med["SQ_INSTS_VALU"] * 2 / (SIMDS * NOMINAL_HZ * us * 1e-6), 4),
            "valu_busy_at_measured_clock": round(statistics.median(
                v["SQ_INSTS_VALU"] * 2 / (SIMDS * v["GRBM_GUI_ACTIVE"] / 8) for v in ser if "GRBM_GUI_ACTIVE" in v), 4)}
    out[leg] = e
print(json.dumps(out, indent=1))
