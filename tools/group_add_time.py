"""Batched GPU AddPiece at 32 MiB/256 over G fresh decoders (one
rlnc_decoders_add_pieces_gpu call: row copies + twins and the elimination),
host wall time per call, best of REPS, decoder construction outside."""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kodr_amd import device as kdev, errors  # noqa: E402
from kodr_amd._lib import lib, _u8p  # noqa: E402

L_ = lib()
ctx = kdev.Context(0)
k, L, REPS = 256, 131072, 7
G = int(sys.argv[1]) if len(sys.argv) > 1 else 16
W = k + L
rng = np.random.default_rng(5)
wires = []
P = rng.integers(0, 256, k * L, dtype=np.uint8)
h = ctypes.c_void_p()
errors.check(L_.rlnc_encoder_create(ctx.handle, 0, P.ctypes.data_as(_u8p), k, L, ctypes.byref(h)))
for g in range(G):
    errors.check(L_.rlnc_encoder_seed(h, 100 + g))
    dw = ctx.alloc((k + 2) * W)
    errors.check(L_.rlnc_encoder_coded_wire_device(h, k + 2, dw, W))
    wires.append(dw)
ctx.synchronize()
best = None
for rep in range(REPS):
    decs = []
    for g in range(G):
        d = ctypes.c_void_p()
        errors.check(L_.rlnc_decoder_create(ctx.handle, k, ctypes.byref(d)))
        decs.append(d)
    darr = (ctypes.c_void_p * G)(*[d.value for d in decs])
    cons, sts = (ctypes.c_size_t * G)(), (ctypes.c_int * G)()
    ctx.synchronize()
    t0 = time.perf_counter()
    errors.check(L_.rlnc_decoders_add_pieces_gpu(darr, G, (ctypes.c_void_p * G)(*wires), (ctypes.c_size_t * G)(*([k + 2] * G)),
                                                 W, L, cons, sts))
    ctx.synchronize()
    t = time.perf_counter() - t0
    assert all(s in (0, 3) for s in sts) and all(L_.rlnc_decoder_is_decoded(d) for d in decs)
    for d in decs:
        L_.rlnc_decoder_destroy(d)
    best = t if best is None else min(best, t)
print(json.dumps({"G": G, "add_ms": round(best * 1e3, 3), "add_us_per_generation": round(best / G * 1e6, 1)}), flush=True)
