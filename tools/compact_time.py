"""Device encode time per call at 32 MiB/256 for a plain-resident encoder
(plain rows + bit-sliced twin after rlnc_encoder_prepare) and a compact one
(twin only, rlnc_encoder_compact), B pieces per call, median of REPS calls
timed with HIP events on the context stream (encoder state warm)."""
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
k, L, REPS = 256, 131072, 50
rng = np.random.default_rng(1)
P = rng.integers(0, 256, k * L, dtype=np.uint8)
res = {"k": k, "L": L}
a, b = ctx.event(), ctx.event()
for mode in ("plain", "compact"):
    h = ctypes.c_void_p()
    errors.check(L_.rlnc_encoder_create(ctx.handle, 0, P.ctypes.data_as(_u8p), k, L, ctypes.byref(h)))
    errors.check(L_.rlnc_encoder_prepare(h) if mode == "plain" else L_.rlnc_encoder_compact(h))
    row = {"resident_MiB": (2 if mode == "plain" else 1) * k * L / 2**20}
    for B in (1, 2, 4, 8, 16, 32):
        dV, dY = ctx.alloc(B * k), ctx.alloc(B * L)
        ctx.h2d(dV, rng.integers(0, 256, B * k, dtype=np.uint8))
        ts = []
        for i in range(REPS + 5):
            ctx.record(a)
            errors.check(L_.rlnc_encoder_coded_pieces_device(h, dV, B, dY, L))
            ctx.record(b)
            ctx.synchronize()
            if i >= 5:
                ts.append(kdev.Context.elapsed_ms(a, b) * 1e3)
        row[f"B{B}_us"] = round(float(np.median(ts)), 2)
        ctx.free(dV)
        ctx.free(dY)
    res[mode] = row
    L_.rlnc_encoder_destroy(h)
print(json.dumps(res), flush=True)
