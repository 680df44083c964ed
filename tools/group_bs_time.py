"""Grouped bit-sliced encode at 32 MiB/256: B coded pieces of each of G
prepared generations in ONE launch (rlnc_encoder_group_coded_pieces_device)
against G single-generation launches of the same work
(rlnc_encoder_coded_pieces_device per generation), HIP events on the context
stream, median of REPS repetitions.  Generations rotate as in bench.py (16 x
32 MiB: HBM-cold)."""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kodr_amd import device as kdev, errors  # noqa: E402
from kodr_amd._lib import lib, _u8p  # noqa: E402

L_ = lib()
ctx = kdev.Context(0)
k, L, REPS = 256, 131072, 15
G = int(os.environ.get("KODR_GROUP_G", "16"))
rng = np.random.default_rng(3)
encs = []
for g in range(G):
    P = rng.integers(0, 256, k * L, dtype=np.uint8)
    h = ctypes.c_void_p()
    errors.check(L_.rlnc_encoder_create(ctx.handle, 0, P.ctypes.data_as(_u8p), k, L, ctypes.byref(h)))
    errors.check(L_.rlnc_encoder_prepare(h))
    encs.append(h)
arr = (ctypes.c_void_p * G)(*[e.value for e in encs])
a, b = ctx.event(), ctx.event()
res = {"k": k, "L": L, "G": G}
Bs = [int(x) for x in (sys.argv[1:] or ["9", "16", "32", "64", "256"])]
for B in Bs:
    dV, dY = ctx.alloc(G * B * k), ctx.alloc(G * B * L)
    ctx.h2d(dV, rng.integers(0, 256, G * B * k, dtype=np.uint8))
    row = {}
    for mode in ("single", "grouped"):
        ts = []
        for i in range(REPS + 3):
            ctx.record(a)
            if mode == "grouped":
                errors.check(L_.rlnc_encoder_group_coded_pieces_device(arr, G, dV, B, dY, L))
            else:
                for g in range(G):
                    errors.check(L_.rlnc_encoder_coded_pieces_device(encs[g], dV + g * B * k, B, dY + g * B * L, L))
            ctx.record(b)
            ctx.synchronize()
            if i >= 3:
                ts.append(kdev.Context.elapsed_ms(a, b) * 1e3)
        t = float(np.median(ts))
        row[mode + "_us_per_generation"] = round(t / G, 3)
    row["speedup"] = round(row["single_us_per_generation"] / row["grouped_us_per_generation"], 3)
    res[f"B{B}"] = row
    print(B, json.dumps(row), flush=True)
    ctx.free(dV)
    ctx.free(dY)
for h in encs:
    L_.rlnc_encoder_destroy(h)
print(json.dumps(res), flush=True)
