"""Run the jump-body probe variants: correctness vs a Python model and
throughput (see gen_jump.py)."""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kodr_amd import device
from gen_jump import VARIANTS, NB
p = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libjump.so"))
ctx = device.Context(0)
rng = np.random.default_rng(1)
inp = rng.integers(0, 2**32, 4096, dtype=np.uint32)
din = ctx.alloc(inp.nbytes)
ctx.h2d(din, inp.view(np.uint8))
out = ctx.alloc(64 << 20)
st = ctypes.c_void_p(ctx.stream)


def model(t, MT, PER):
    x = [int(inp[(t * 8 + i) & 4095]) for i in range(8)]
    acc = [0] * (8 * MT)
    for m in range(MT):
        c = (m * 5 + 3) % NB
        for pp in range(PER):
            for j in range(8):
                acc[8 * m + j] ^= x[(j + c + pp) % 8] ^ x[(j + 3 * c + 2 * pp + 1) % 8]
    return acc


e0, e1 = ctx.event(), ctx.event()
iters = 400
for vi, (name, vb, MT, PER, mode) in enumerate(VARIANTS):
    p.probe_jump(vi, ctypes.c_void_p(out), ctypes.c_void_p(din), 1, 1, st, 0)
    ctx.synchronize()
    got = ctx.d2h(out, 256 * 64 * 4).view(np.uint32).reshape(256, 64)
    ok = mode == 3 or all(list(got[t][:8 * MT]) == model(t, MT, PER) for t in (0, 1, 63, 200))
    blocks = 8192
    for wps, lds in ((1, 160 * 1024), (2, 80 * 1024), (3, 0)):
        p.probe_jump(vi, ctypes.c_void_p(out), ctypes.c_void_p(din), blocks, 5, st, lds)
        ctx.record(e0)
        p.probe_jump(vi, ctypes.c_void_p(out), ctypes.c_void_p(din), blocks, iters, st, lds)
        ctx.record(e1)
        ms = device.Context.elapsed_ms(e0, e1)
        insts = blocks * 4 * iters * MT * PER * 8
        print(f"{name:16s} ok={ok} waves/SIMD {wps}: {ms:.3f} ms  {insts*64/ms/1e9:.2f} T lane-op/s  "
              f"cyc/inst/SIMD@2.4 = {ms*1e-3*2.4e9*1024/insts:.2f}", flush=True)
