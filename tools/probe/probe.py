#!/usr/bin/env python3
"""Time the calibration kernels of probe.hip over 16 rotating 32 MiB buffers."""
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

for blocks in (256, 512, 1024, 2048, 4096, 8192):
    for threads in (256, 512, 1024):
        us = timeit(lambda i: p.probe_read(ctypes.c_void_p(buf + (i % G) * S), ctypes.c_size_t(S), ctypes.c_void_p(out), blocks, threads, st))
        print(f"read_stream blocks={blocks:5d} threads={threads:4d} {us:7.2f} us {S/us/1e3:7.1f} GB/s", flush=True)
for s_ in (1, 2, 4):
    us = timeit(lambda i: p.probe_tiles(ctypes.c_void_p(buf + (i % G) * S), K, L, L, s_, ctypes.c_void_p(out), st))
    print(f"read_tiles S={s_} {us:7.2f} us {S/us/1e3:7.1f} GB/s", flush=True)
# hot (one buffer, MALL-resident)
us = timeit(lambda i: p.probe_read(ctypes.c_void_p(buf), ctypes.c_size_t(S), ctypes.c_void_p(out), 2048, 256, st))
print(f"read_stream HOT {us:7.2f} us {S/us/1e3:7.1f} GB/s")
# large stream: all 512 MiB at once
us = timeit(lambda i: p.probe_read(ctypes.c_void_p(buf), ctypes.c_size_t(G * S), ctypes.c_void_p(out), 8192, 256, st), 20)
print(f"read_stream 512MiB {us:7.2f} us {G*S/us/1e3:7.1f} GB/s")
# launch floor: the same kernel with nothing to read
for blocks in (256, 2048):
    us = timeit(lambda i: p.probe_read(ctypes.c_void_p(buf), ctypes.c_size_t(0), ctypes.c_void_p(out), blocks, 256, st))
    print(f"empty launch blocks={blocks} {us:7.2f} us")
