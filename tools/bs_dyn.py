"""A/B of the bit-sliced kernel's row split (tuning build, KODR_RLNC_LIB):
mode 0 = static K split per wave, mode 20 = dynamic rows from an LDS counter.
Times both over rotating 32 MiB/256 generations and checks that both give
the same bytes.  usage: python tools/bs_dyn.py [B,...] [modes]"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kodr_amd import device, errors
from kodr_amd._lib import lib

L_ = lib()
ctx = device.Context(0)
k, L = 256, 131072
G = 16
rng = np.random.default_rng(1)
gens = []
for g in range(G):
    d = ctx.alloc(k * L)
    ctx.h2d(d, rng.integers(0, 256, k * L, dtype=np.uint8))
    errors.check(L_.rlnc_bitslice_device(ctx.handle, d, L, k, L))
    gens.append(d)
e0, e1 = ctx.event(), ctx.event()
Bs = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "16,32,64,256").split(",")]
modes = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "0,20,0,20").split(",")]
for B in Bs:
    V = rng.integers(0, 256, (B, k), dtype=np.uint8)
    dV, dO = ctx.alloc(V.nbytes), ctx.alloc(B * L)
    ctx.h2d(dV, V)
    line, ref = [], None
    for mode in modes:
        os.environ["KODR_BS_MODE"] = str(mode)
        errors.check(L_.rlnc_gf_matmul_bs_device(ctx.handle, dV, k, B, k, gens[0], L, dO, L, L))
        out = ctx.d2h(dO, B * L)
        ok = True if ref is None else bool(np.array_equal(out, ref))
        ref = out if ref is None else ref
        for i in range(3):
            errors.check(L_.rlnc_gf_matmul_bs_device(ctx.handle, dV, k, B, k, gens[i % G], L, dO, L, L))
        iters = 40 if B <= 64 else 10
        ctx.record(e0)
        for i in range(iters):
            errors.check(L_.rlnc_gf_matmul_bs_device(ctx.handle, dV, k, B, k, gens[i % G], L, dO, L, L))
        ctx.record(e1)
        line.append(f"m{mode}={device.Context.elapsed_ms(e0, e1) * 1e3 / iters:7.2f}us{'' if ok else ' MISMATCH'}")
    print(f"B={B:4d} " + " ".join(line), flush=True)
    ctx.free(dV)
    ctx.free(dO)
