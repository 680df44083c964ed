#!/usr/bin/env python3
"""Per-launch summary of a rocprofv3 kernel trace of `bench.py`.

  python tools/prof_headline.py <run_kernel_trace.csv> <bench.json> [--warm W] [--steps K] [--gens G]

bench.py launches the headline kernel max(W, G) times untimed, then K times
in the timed region, before any extra measurement.  This picks those K
launches out of the trace (first launches of the headline kernel name with
the headline grid), averages their durations and compares them with the
bench line's `roofline.avg_launch_us` (HIP events on the same stream).  It
also prints every (kernel, grid) group of the trace, so the extras' launches
of the same kernel template (decode apply, recode, sweeps) are not mixed into
the headline figure.
"""
import argparse
import csv
import json
import statistics
from collections import OrderedDict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("bench")
    ap.add_argument("--warm", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--gens", type=int, default=16)
    ap.add_argument("--out")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    with open(a.bench) as f:
        line = json.loads([l for l in f if l.startswith("{")][-1])
    kname = line["roofline"]["kernel"]
    groups = OrderedDict()
    for r in rows:
        key = (r["Kernel_Name"], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"], r["Workgroup_Size_X"])
        groups.setdefault(key, []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    # the headline group: the first (kernel, grid) group of the headline
    # kernel with at least the warmup + timed launches (the library's one-off
    # probe launch of the same template comes earlier, on a one-wave grid)
    nwarm = line["roofline"].get("warmup_launches", max(a.warm, a.gens))
    head_key = next(k for k, v in groups.items()
                    if (kname + "<" in k[0] or k[0].endswith(kname)) and len(v) >= nwarm + a.steps)
    first = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows
             if (r["Kernel_Name"], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"],
                 r["Workgroup_Size_X"]) == head_key]
    timed = first[nwarm:nwarm + a.steps]
    avg_ns = statistics.mean(timed)
    ev_us = line["roofline"]["avg_launch_us"]
    res = {
        "kernel": head_key[0],
        "grid": [int(x) for x in head_key[1:4]], "workgroup": int(head_key[4]),
        "timed_launches": len(timed),
        "rocprof_avg_us": round(avg_ns / 1e3, 3),
        "rocprof_median_us": round(statistics.median(timed) / 1e3, 3),
        "rocprof_min_us": round(min(timed) / 1e3, 3), "rocprof_max_us": round(max(timed) / 1e3, 3),
        "bench_events_avg_launch_us": ev_us,
        "events_over_rocprof": round(ev_us / (avg_ns / 1e3), 4),
        "bench_value": line["value"], "bench_ms_per_step": line["ms_per_step"],
        "hbm_bytes_per_launch": line["roofline"]["hbm_bytes_per_launch"],
        "hbm_frac_from_rocprof": round(line["roofline"]["hbm_bytes_per_launch"] / (avg_ns / 1e9) / 8e12, 4),
        "groups": [{"kernel": k[0][:90], "grid": [int(x) for x in k[1:4]], "calls": len(v),
                    "avg_us": round(statistics.mean(v) / 1e3, 3)} for k, v in groups.items()],
    }
    s = json.dumps(res, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s + "\n")


if __name__ == "__main__":
    main()
