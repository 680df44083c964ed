#!/usr/bin/env python3
"""B = 1 gap hunt: read_tiles<2> with the gemm kernel's phases added one at a
time (probe.hip read_tiles_v), over 16 rotating 32 MiB buffers."""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from kodr_amd import device

HERE = os.path.dirname(os.path.abspath(__file__))
p = ctypes.CDLL(os.path.join(HERE, "libprobe.so"))
ctx = device.Context(0)
G, K, L = 16, 256, 131072
S = K * L
buf = ctx.alloc(G * S)
ctx.h2d(buf, np.random.default_rng(0).integers(0, 256, G * S, dtype=np.uint8))
out = ctx.alloc(64 << 20)
coef = ctx.alloc(256)
ctx.h2d(coef, np.random.default_rng(1).integers(0, 256, 256, dtype=np.uint8))
st = ctypes.c_void_p(ctx.stream)
e0, e1 = ctx.event(), ctx.event()


def timeit(fn, iters=200):
    for i in range(10):
        fn(i)
    ctx.record(e0)
    for i in range(iters):
        fn(i)
    ctx.record(e1)
    return device.Context.elapsed_ms(e0, e1) * 1e3 / iters


for rep in range(2):
    us = timeit(lambda i: p.probe_tiles(ctypes.c_void_p(buf + (i % G) * S), K, L, L, 2, ctypes.c_void_p(out), st))
    print(f"read_tiles S=2 {us:7.2f} us", flush=True)
    for v in range(8):
        us = timeit(lambda i: p.probe_tiles_v(ctypes.c_void_p(buf + (i % G) * S), K, L, L, v, ctypes.c_void_p(out),
                                              ctypes.c_void_p(coef), st))
        print(f"read_tiles_v V={v} (lds_pro={v & 1} fold={v >> 1 & 1} buffer={v >> 2 & 1}) {us:7.2f} us", flush=True)
