"""Time gf_gemm_bs per tuning mode (needs the KODR_TUNE_MODES build, loaded via
KODR_RLNC_LIB): 0 normal, 1 empty bodies, 2 empty bodies without reading A,
3 no dispatch, 4 = 3 without the row stream, 5 no main loop,
6 = 4 without v_readfirstlane, 7 = 6 without the LDS program read.  32 MiB/256 generation, B rows per launch."""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kodr_amd import device, errors
from kodr_amd._lib import lib

L_ = lib()
ctx = device.Context(0)
k, L = 256, 131072
G = 8
rng = np.random.default_rng(1)
gens = []
for g in range(G):
    d = ctx.alloc(k * L)
    ctx.h2d(d, rng.integers(0, 256, k * L, dtype=np.uint8))
    errors.check(L_.rlnc_bitslice_device(ctx.handle, d, L, k, L))
    gens.append(d)
e0, e1 = ctx.event(), ctx.event()
Bs = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "8,16,32,64,256").split(",")]
for B in Bs:
    V = rng.integers(1, 256, (B, k), dtype=np.uint8)
    dV, dO = ctx.alloc(V.nbytes), ctx.alloc(B * L)
    ctx.h2d(dV, V)
    line = []
    for mode in [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "0,3,5").split(",")]:
        os.environ["KODR_BS_MODE"] = str(mode)
        for i in range(3):
            errors.check(L_.rlnc_gf_matmul_bs_device(ctx.handle, dV, k, B, k, gens[i % G], L, dO, L, L))
        iters = 40
        ctx.record(e0)
        for i in range(iters):
            errors.check(L_.rlnc_gf_matmul_bs_device(ctx.handle, dV, k, B, k, gens[i % G], L, dO, L, L))
        ctx.record(e1)
        line.append(f"m{mode}={device.Context.elapsed_ms(e0, e1) * 1e3 / iters:7.2f}us")
    print(f"B={B:4d} " + " ".join(line), flush=True)
    ctx.free(dV)
    ctx.free(dO)
