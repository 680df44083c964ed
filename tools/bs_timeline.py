"""Per-wave phase timeline of gf_bs_kernel (MODE 8, tune build): prologue
(coefficients, program build), main loop, reduction + store.  B rows of a
32 MiB/256 generation, one launch after warm-up.  Debug/measurement only."""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kodr_amd import device, errors
from kodr_amd._lib import lib

L_ = lib()
ctx = device.Context(0)
k, L = 256, 131072
rng = np.random.default_rng(1)
gens = []
for g in range(4):
    d = ctx.alloc(k * L)
    ctx.h2d(d, rng.integers(0, 256, k * L, dtype=np.uint8))
    errors.check(L_.rlnc_bitslice_device(ctx.handle, d, L, k, L))
    gens.append(d)
for B in [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "8,32,256").split(",")]:
    V = rng.integers(1, 256, (B, k), dtype=np.uint8)
    dV, dO = ctx.alloc(V.nbytes), ctx.alloc(B * L + (1 << 22))
    ctx.h2d(dV, V)
    os.environ["KODR_BS_MODE"] = "0"
    for i in range(5):
        errors.check(L_.rlnc_gf_matmul_bs_device(ctx.handle, dV, k, B, k, gens[i % 4], L, dO, L, L))
    os.environ["KODR_BS_MODE"] = "8"
    ctx.h2d(dO + B * L, np.zeros(1 << 22, np.uint8))
    ctx.synchronize()
    errors.check(L_.rlnc_gf_matmul_bs_device(ctx.handle, dV, k, B, k, gens[3], L, dO, L, L))
    ctx.synchronize()
    raw = ctx.d2h(dO + B * L, (1 << 22) // 40 * 40).view(np.uint64).reshape(-1, 5)
    raw = raw[raw[:, 4] > 0]
    t0 = raw[:, 0].min()
    st = (raw[:, :4] - t0).astype(np.float64)
    # shader clock from s_memtime vs s_memrealtime (100 MHz) is not derivable from
    # one stamp; report cycles and assume 2.4e9 for us
    q = lambda a: f"p10={np.percentile(a, 10):8.0f} p50={np.percentile(a, 50):8.0f} p90={np.percentile(a, 90):8.0f} max={a.max():8.0f}"
    print(f"B={B} waves={len(raw)}")
    print("  start        ", q(st[:, 0]))
    print("  prologue     ", q(st[:, 1] - st[:, 0]))
    print("  main loop    ", q(st[:, 2] - st[:, 1]))
    print("  reduce+store ", q(st[:, 3] - st[:, 2]))
    print("  end          ", q(st[:, 3]))
    ctx.free(dV)
    ctx.free(dO)
