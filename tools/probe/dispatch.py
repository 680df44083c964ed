"""Run the dispatch probe (gen_dispatch.py): check every variant against a
Python model, then time it at 1-4 waves per SIMD.  Measurement only."""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
sys.path.insert(0, HERE)
from gen_dispatch import VARIANTS, X, coef, planes  # noqa: E402

from kodr_amd import device  # noqa: E402

p = ctypes.CDLL(os.path.join(HERE, "libdispatch.so"))
ctx = device.Context(0)
rng = np.random.default_rng(1)
inp = rng.integers(0, 2**32, 4096, dtype=np.uint32)
din = ctx.alloc(inp.nbytes)
ctx.h2d(din, inp.view(np.uint8))
out = ctx.alloc(64 << 20)
st = ctypes.c_void_p(ctx.stream)


def model(t, mode, nb, dyn, ncopy=8):
    x = [int(inp[(t * 8 + i) & 4095]) for i in range(8)]
    acc = [0] * 64
    if mode == "W":  # 4 rows, two blocks per lane (the second = words rotated by one)
        x2 = [x[(i + 1) % 8] for i in range(8)]
        for m in range(4):
            c = (5 * m + 3 + 232) % nb
            for j in range(8):
                a, b = planes(c, j)
                acc[16 * m + j] ^= x[a - X] ^ x[b - X]
                acc[16 * m + 8 + j] ^= x2[a - X] ^ x2[b - X]
        return [acc[r] ^ acc[r + 16] ^ acc[r + 32] ^ acc[r + 48] for r in range(16)]
    for m0 in range(8):
        m = m0 % ncopy
        c = (5 * m0 + 3 + 232) % nb if mode == "T" else coef(m0, nb, 1 if dyn else None)
        for j in range(8):
            a, b = planes(c, j)
            acc[8 * m + j] ^= x[a - X] ^ x[b - X]
    return [acc[r] ^ acc[r + 16] ^ acc[r + 32] ^ acc[r + 48] for r in range(16)]


e0, e1 = ctx.event(), ctx.event()
iters = 200
blocks = 8192
only = sys.argv[1].split(",") if len(sys.argv) > 1 else None
for vi, (name, mode, nb, dyn, *rest) in enumerate(VARIANTS):
    if only and name not in only:
        continue
    p.probe_dispatch(vi, ctypes.c_void_p(out), ctypes.c_void_p(din), 1, 1, st, 0)
    ctx.synchronize()
    got = ctx.d2h(out, 256 * 16 * 4).view(np.uint32).reshape(256, 16)
    ok = mode == "BANK" or all(list(got[t]) == model(t, mode, nb, dyn, *rest) for t in (0, 1, 63, 200))
    for wps in (1, 2, 3, 4):
        lds = (160 * 1024) // wps // 4 * 4 if wps < 4 else 0
        p.probe_dispatch(vi, ctypes.c_void_p(out), ctypes.c_void_p(din), blocks, 5, st, lds)
        ctx.record(e0)
        p.probe_dispatch(vi, ctypes.c_void_p(out), ctypes.c_void_p(din), blocks, iters, st, lds)
        ctx.record(e1)
        ms = device.Context.elapsed_ms(e0, e1)
        bodies = blocks * 4 * iters * 8
        print(f"{name} ok={ok} waves/SIMD {wps}: {ms:8.3f} ms  SIMD-cycles per body @2.4GHz "
              f"= {ms * 1e-3 * 2.4e9 * 1024 / bodies:6.2f}", flush=True)
