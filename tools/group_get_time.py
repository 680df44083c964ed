"""Grouped GetPieces at 32 MiB/256 (BASELINE configs[2] over many
generations): G decoders fed k engine-coded wire rows each (one
rlnc_decoders_add_pieces_gpu call), then the data side timed per decoder
(rlnc_decoder_get_pieces_device x G) against one grouped call
(rlnc_decoders_get_pieces_device), HIP events on the context stream,
median of REPS; outputs checked against the generations."""
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
k, L, REPS = 256, 131072, 10
G = int(sys.argv[1]) if len(sys.argv) > 1 else 16
W = k + L
rng = np.random.default_rng(9)
datas, encs, wires, decs = [], [], [], []
for g in range(G):
    P = rng.integers(0, 256, k * L, dtype=np.uint8)
    datas.append(P)
    h = ctypes.c_void_p()
    errors.check(L_.rlnc_encoder_create(ctx.handle, 0, P.ctypes.data_as(_u8p), k, L, ctypes.byref(h)))
    errors.check(L_.rlnc_encoder_seed(h, 100 + g))
    dw = ctx.alloc(k * W)
    errors.check(L_.rlnc_encoder_coded_wire_device(h, k, dw, W))
    encs.append(h)
    wires.append(dw)
    d = ctypes.c_void_p()
    errors.check(L_.rlnc_decoder_create(ctx.handle, k, ctypes.byref(d)))
    decs.append(d)
ctx.synchronize()
darr = (ctypes.c_void_p * G)(*[d.value for d in decs])
rarr = (ctypes.c_void_p * G)(*wires)
counts = (ctypes.c_size_t * G)(*([k] * G))
consumed = (ctypes.c_size_t * G)()
status = (ctypes.c_int * G)()
errors.check(L_.rlnc_decoders_add_pieces_gpu(darr, G, rarr, counts, W, L, consumed, status))
ctx.synchronize()
assert all(s in (0, 3) for s in status) and all(L_.rlnc_decoder_is_decoded(d) for d in decs)
dO = ctx.alloc(G * k * L)
a, b = ctx.event(), ctx.event()
res = {"G": G, "k": k, "L": L}
for mode in ("per_decoder", "grouped", "per_decoder", "grouped"):
    ts = []
    for i in range(REPS + 2):
        ctx.record(a)
        if mode == "grouped":
            errors.check(L_.rlnc_decoders_get_pieces_device(darr, G, dO, L))
        else:
            for g in range(G):
                errors.check(L_.rlnc_decoder_get_pieces_device(decs[g], dO + g * k * L, L))
        ctx.record(b)
        ctx.synchronize()
        if i >= 2:
            ts.append(kdev.Context.elapsed_ms(a, b) * 1e3)
    res[mode + "_us_per_generation"] = round(float(np.median(ts)) / G, 2)
    out = ctx.d2h(dO, G * k * L).reshape(G, k * L)
    res[mode + "_ok"] = all(np.array_equal(out[g], datas[g]) for g in range(G))
res["gf_macs_per_s_grouped"] = float(f"{k * k * L / (res['grouped_us_per_generation'] * 1e-6):.4g}")
print(json.dumps(res), flush=True)
for d in decs:
    L_.rlnc_decoder_destroy(d)
for h in encs:
    L_.rlnc_encoder_destroy(h)
