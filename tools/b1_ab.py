"""One coded piece per launch at 32 MiB/256 (B = 1, rlnc_encoder_coded_pieces_device),
16 rotating prepared generations (HBM-cold), HIP events over back-to-back
launches, median of reps; the piece is checked against the oracle.  Run with
KODR_GEMV=0 (gf_gemm_kernel) / 1 (per-lane tables) / 2 (default, shared tables) for A/B."""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import oracle  # noqa: E402  (checker only)
from kodr_amd import device as kdev, errors  # noqa: E402
from kodr_amd._lib import lib, _u8p, last_launch_plan  # noqa: E402

L_ = lib()
ctx = kdev.Context(0)
k, L, G = 256, 131072, 16
rng = np.random.default_rng(9)
datas, encs = [], []
for g in range(G):
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    h = ctypes.c_void_p()
    errors.check(L_.rlnc_encoder_create(ctx.handle, 0, P.ctypes.data_as(_u8p), k, L, ctypes.byref(h)))
    encs.append(h)
    if g < 2:
        datas.append(P)
V = rng.integers(0, 256, (64, k), dtype=np.uint8)
dV, dY = ctx.alloc(V.nbytes), ctx.alloc(64 * L)
ctx.h2d(dV, V)
# correctness: piece of generation 1 with vector 5
errors.check(L_.rlnc_encoder_coded_pieces_device(encs[1], dV + 5 * k, 1, dY, L))
plan = last_launch_plan()
ctx.synchronize()
ok = bool(np.array_equal(ctx.d2h(dY, L), oracle.encode(datas[1], V[5:6])[0]))
a, b = ctx.event(), ctx.event()
res = {"plan": plan, "ok": ok}
for B in (1, 2, 4):
    ts = []
    for rep in range(7):
        for i in range(20):
            errors.check(L_.rlnc_encoder_coded_pieces_device(encs[i % G], dV + (i % 64) * k, B, dY, L))
        ctx.record(a)
        for i in range(200):
            errors.check(L_.rlnc_encoder_coded_pieces_device(encs[i % G], dV + (i % 60) * k, B, dY, L))
        ctx.record(b)
        ts.append(kdev.Context.elapsed_ms(a, b) * 1e3 / 200)
    res[f"B{B}_us"] = round(float(np.median(ts)), 3)
print(json.dumps(res), flush=True)
