#!/usr/bin/env python3
"""Per-kernel roofline of bench.py's encode_decode round trip from a
rocprofv3 kernel trace of `bench.py --no-extras` (headline + round trip only).

  python tools/prof_roundtrip.py <run_kernel_trace.csv> <bench.json> [--out FILE]

Groups the trace by (kernel, grid); the round trip's launches are
  * the grouped encode: gf_bs_kernel<..., true, ...> with G x (k + 2) rows of
    output per launch (told from the headline's B = 32 launch by its grid);
  * the elimination: gf_elim_mc_kernel (one launch per AddPiece call);
  * the rows' copy and bit-sliced twin: copy_bitslice_rows_grouped's kernel;
  * GetPieces: the grouped gf_bs_kernel launch over the decoders' twins;
and prints each group's count and median duration with its bound: GF MACs
against the bit-sliced VALU floor (bench.VALU_FLOOR_MACS_PER_S) or bytes
against the 8 TB/s HBM peak."""
import argparse
import csv
import json
import os
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("bench")
    ap.add_argument("--out")
    a = ap.parse_args()
    with open(a.bench) as f:
        line = json.loads([l for l in f if l.startswith("{")][-1])
    ed = line["encode_decode"]
    G = ed["generations_per_step"]
    k, L = bench.K_PIECES, bench.L_BYTES
    n = k + 2
    groups = {}
    for r in csv.DictReader(open(a.trace)):
        key = (r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0], int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]), int(r["Workgroup_Size_X"]))
        groups.setdefault(key, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = {"generations_per_step": G, "steps": ed["steps"], "warmup_steps_run": ed["warmup_steps_run"],
           "kernels": []}
    peak_mac = bench.VALU_FLOOR_MACS_PER_S
    for (name, gx, gy, wg), d in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        med = statistics.median(d)
        e = {"kernel": name[-90:], "grid": [gx, gy], "workgroup": wg, "launches": len(d),
             "median_us": round(med, 2), "total_ms": round(sum(d) / 1e3, 3)}
        if "gf_elim_mc" in name:
            macs = gy * k ** 3
            e.update(leg="elimination (AddPiece)", gf_macs=macs,
                     gf_macs_per_s=float(f"{macs / med * 1e6:.4g}"), issue_frac=round(macs / med * 1e6 / peak_mac, 4))
        elif "copy_bitslice" in name:
            b = G * 3 * n * L
            e.update(leg="rows' copy + twin (AddPiece)", hbm_bytes=b, hbm_frac=round(b / med / 1e3 / bench.HBM_PEAK_GBS, 4))
        elif "gf_bs_kernel" in name and "true" in name:
            # grouped launches: grid y = generations; the encode writes n rows per
            # generation, GetPieces k (gf_bs plans 8-row tiles: rows = 8 x tiles)
            e["leg"] = "grouped gf_bs_kernel"
        out["kernels"].append(e)
    # attribute the grouped bit-sliced groups by launch count: per timed+warm step
    # one encode launch and one GetPieces launch per 16 decoders
    steps = ed["steps"] + ed["warmup_steps_run"]
    bs = [e for e in out["kernels"] if e.get("leg") == "grouped gf_bs_kernel"]
    for e in bs:
        if e["launches"] == steps and e["grid"][1] == G:
            pass
    with open(a.out, "w") if a.out else sys.stdout as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
