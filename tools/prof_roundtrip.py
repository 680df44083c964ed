#!/usr/bin/env python3
"""rocprofv3 kernel trace of the driver's exact bench command
(`rocprofv3 --kernel-trace --stats -- python3 bench.py --gpus 1 --steps 20
--warmup 5`) against the bench line that same run printed.

  python tools/prof_roundtrip.py <run_kernel_trace.csv> <bench.json> [--out FILE]

The launches are told apart by the kernel instance each leg recorded
(bench.py: legs[*].plan, encode.roofline.plan -- workgroups x 64 x waves
threads in grid x, generations in grid y) and by their order: bench.py runs
the round trip's warmup + timed steps first, then the encode leg's warmup +
timed launches, then the extras.  For each leg: the timed launches' rocprof
average against the HIP-event average in the bench line, and the fraction of
its bound recomputed from the rocprof duration."""
import argparse
import csv
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import bench  # noqa: E402


def launches(trace):
    rows = []
    for r in csv.DictReader(open(trace)):
        rows.append((int(r["Start_Timestamp"]), r["Kernel_Name"], int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]),
                     (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    rows.sort()
    return rows


def of_plan(rows, plan, after=0):
    """The gf_bs_kernel launches of a recorded plan, in start order, that start after `after`."""
    gx = plan["workgroups"] * 64 * plan["waves"]
    return [r for r in rows if "gf_bs_kernel" in r[1] and r[2] == gx and r[3] == plan["generations"] and r[0] > after]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("bench")
    ap.add_argument("--out")
    a = ap.parse_args()
    with open(a.bench) as f:
        line = json.loads([x for x in f if x.startswith("{")][-1])
    rows = launches(a.trace)
    rt = line["roundtrip"]
    legs = line["roofline"]["legs"]
    steps, n_warm = line["steps"], rt["warmup_steps_run"]
    G = line["config"]["generations_per_step"]
    k, L = line["config"]["piece_count"], line["config"]["piece_size"]
    n = k + 2
    peak = bench.VALU_FLOOR_MACS_PER_S
    out = {"command": "rocprofv3 --kernel-trace --stats -- python3 bench.py --gpus 1 --steps %d --warmup %d"
                      % (steps, line["warmup"]),
           "bench_value": line["value"], "bench_ms_per_step": line["ms_per_step"], "legs": {}}

    def leg(name, sel, events_us, macs=None, hbm=None, first=None, count=None):
        first = n_warm if first is None else first
        count = steps if count is None else count
        if len(sel) < first + count:
            out["legs"][name] = {"error": f"{len(sel)} launches, expected {first + count}"}
            return None
        timed = [r[4] for r in sel[first:first + count]]
        avg = statistics.mean(timed)
        e = {"kernel": sel[0][1].replace("(anonymous namespace)::", "").split("(")[0][-100:],
             "grid": [sel[0][2], sel[0][3]], "timed_launches": len(timed), "rocprof_avg_us": round(avg, 2),
             "rocprof_min_us": round(min(timed), 2), "rocprof_max_us": round(max(timed), 2)}
        if events_us is not None:
            e["bench_events_avg_us"] = events_us
            e["events_over_rocprof"] = round(events_us / avg, 4)
        if macs is not None:
            e["issue_frac_from_rocprof"] = round(macs / avg * 1e6 / peak, 4)
        if hbm is not None:
            e["hbm_frac_from_rocprof"] = round(hbm / avg / 1e3 / bench.HBM_PEAK_GBS, 4)
        out["legs"][name] = e
        return sel[first + count - 1][0]

    # the round trip's launches in order: the pipelined warmup (which queues
    # one encode more than its steps) and timed steps, then -- when the line
    # is pipelined -- the same round trip in series (legs.serial_warmup_steps
    # untimed, then the timed steps whose events make `legs`)
    wenc = rt.get("warmup_encodes_run", n_warm)
    nws = legs.get("serial_warmup_steps", 0)
    pip = line["config"].get("pipelined", False)
    pis = legs.get("pipelined_in_step", {})
    # (with the split tail the encode's bit-sliced launch and GetPieces are one
    # kernel instance on one grid: tools/rt_roles.py tells them apart by order)
    from rt_roles import get_ids
    gget = of_plan(rows, legs["get_pieces_call"]["plan"])
    gset = {id(r) for r in gget}
    gets = get_ids(rows, lambda r: r[2] if id(r) in gset else None, lambda r: "copy_bitslice" in r[1], id)
    enc_sel = [r for r in of_plan(rows, legs["encode_launch"]["plan"]) if id(r) not in gets]
    get_sel = [r for r in gget if id(r) in gets]
    elim = [r for r in rows if "gf_elim_mc" in r[1] and r[3] == G]
    twin = [r for r in rows if "copy_bitslice" in r[1]]
    ser_enc = wenc + steps + nws if pip else wenc
    ser = n_warm + steps + nws if pip else n_warm
    leg("roundtrip_encode", enc_sel, legs["encode_launch"]["avg_us"], macs=G * n * k * L, first=ser_enc)
    leg("roundtrip_get_pieces", get_sel, legs["get_pieces_call"]["avg_us"], macs=G * k * k * L, first=ser)
    leg("roundtrip_elimination", elim, None, macs=G * k ** 3, first=ser)
    leg("roundtrip_rows_twin", twin, None, hbm=G * 2 * n * L, first=ser)
    if pip:
        leg("pipelined_encode", enc_sel, pis.get("encode_launch", {}).get("avg_us"), macs=G * n * k * L, first=wenc)
        leg("pipelined_get_pieces", get_sel, pis.get("get_pieces_call", {}).get("avg_us"), macs=G * k * k * L)
        leg("pipelined_elimination", elim, None, macs=G * k ** 3)
        leg("pipelined_rows_twin", twin, None, hbm=G * 2 * n * L)
    # the encode leg (bench.py's second timed phase): its own warmup count
    enc = line["encode"]["roofline"]
    last_rt = max((r[0] for r in enc_sel[:ser_enc + steps]), default=0)
    sel = of_plan(rows, enc["plan"], after=last_rt)
    w = enc["warmup_launches"]
    if len(sel) >= w + steps:
        timed = [r[4] for r in sel[w:w + steps]]
        avg = statistics.mean(timed)
        out["legs"]["encode_B32"] = {
            "grid": [sel[0][2], sel[0][3]], "timed_launches": steps, "rocprof_avg_us": round(avg, 2),
            "bench_events_avg_us": enc["avg_launch_us"], "events_over_rocprof": round(enc["avg_launch_us"] / avg, 4),
            "hbm_frac_from_rocprof": round(enc["hbm_bytes_per_launch"] / avg / 1e3 / bench.HBM_PEAK_GBS, 4),
            "issue_frac_from_rocprof": round(enc["issue"]["gf_macs_per_launch"] / avg * 1e6 / peak, 4)}
    else:
        out["legs"]["encode_B32"] = {"error": f"{len(sel)} launches, expected {w + steps}"}
    out["roofline_frac_bench"] = line["roofline"]["frac"]
    rte = out["legs"].get("roundtrip_encode", {})
    if "rocprof_avg_us" in rte:
        out["roofline_frac_from_rocprof"] = rte["issue_frac_from_rocprof"]
    with open(a.out, "w") if a.out else sys.stdout as f:
        json.dump(out, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
