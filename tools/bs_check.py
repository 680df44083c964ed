"""Bit-sliced kernel bring-up on the GPU: body offsets vs the generator,
bitslice transform vs a numpy model, gf_gemm_bs vs the oracle, then timing
against gf_gemm.  Stops at the first mismatch (before any timed launch)."""
import ctypes, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "kodr_amd", "csrc"))
import oracle
from gen_bs_bodies import body_bytes
from kodr_amd import device, errors
from kodr_amd._lib import lib

L_ = lib()
ctx = device.Context(0)
offs = np.zeros(256, np.uint32)
errors.check(L_.rlnc_bs_body_offsets(ctx.handle, offs.ctypes.data_as(ctypes.c_void_p)))
exp = np.zeros(256, np.uint32)
for c in range(1, 256):
    exp[c] = exp[c - 1] + body_bytes(c - 1)
assert np.array_equal(offs, exp), (offs[:8], exp[:8])
print("body offsets ok", offs[-1], flush=True)


def bitslice_np(x):  # x: (..., 32) uint8 -> same shape, planes
    d = x.reshape(-1, 8, 4).copy().view(np.uint32).reshape(-1, 8)
    for sh, m, di in ((4, 0x0F0F0F0F, 4), (2, 0x33333333, 2), (1, 0x55555555, 1)):
        for q in range(8):
            if q & di:
                continue
            t = ((d[:, q] >> sh) ^ d[:, q + di]) & m
            d[:, q + di] ^= t
            d[:, q] ^= (t << sh).astype(np.uint32)
    return d.view(np.uint8).reshape(x.shape)


rng = np.random.default_rng(3)
X = rng.integers(0, 256, (5, 320), dtype=np.uint8)
dX = ctx.alloc(X.nbytes)
ctx.h2d(dX, X)
errors.check(L_.rlnc_bitslice_device(ctx.handle, dX, 320, 5, 320))
ctx.synchronize()
got = ctx.d2h(dX, X.nbytes).reshape(5, 320)
assert np.array_equal(got, bitslice_np(X.reshape(5, 10, 32)).reshape(5, 320))
ctx.free(dX)
print("bitslice ok", flush=True)


def bs_gemm(A, X, ldx_pad=0):
    M, K = A.shape
    n = X.shape[1]
    ldx = (n + 31) // 32 * 32 + ldx_pad
    Xp = np.zeros((K, ldx), np.uint8)
    Xp[:, :n] = X
    dA, dXb, dY = ctx.alloc(max(A.nbytes, 1)), ctx.alloc(Xp.nbytes), ctx.alloc(M * ldx + 64)
    ctx.h2d(dA, A)
    ctx.h2d(dXb, Xp)
    errors.check(L_.rlnc_bitslice_device(ctx.handle, dXb, ldx, K, n))
    errors.check(L_.rlnc_gf_matmul_bs_device(ctx.handle, dA, K, M, K, dXb, ldx, dY, ldx, n))
    ctx.synchronize()
    Y = ctx.d2h(dY, M * ldx).reshape(M, ldx)[:, :n]
    for p in (dA, dXb, dY):
        ctx.free(p)
    return Y


for (M, K, n) in [(1, 1, 32), (8, 8, 2048), (8, 16, 2048), (3, 5, 77), (16, 40, 5000), (9, 300, 4096),
                  (32, 256, 8192), (64, 256, 2048 * 3 + 5), (256, 258, 4096)]:
    A = rng.integers(0, 256, (M, K), dtype=np.uint8)
    A[rng.random((M, K)) < 0.1] = 0
    X = rng.integers(0, 256, (K, n), dtype=np.uint8)
    Y = bs_gemm(A, X)
    ref = oracle.encode(X, A)
    assert np.array_equal(Y, ref), (M, K, n, np.argwhere(Y != ref)[:5])
    print(f"gemm_bs ok M={M} K={K} n={n}", flush=True)

# timing: B coded pieces of a 32 MiB / 256 generation, 16 rotating generations
k, L = 256, 131072
G = 8
gens = []
for g in range(G):
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    d = ctx.alloc(P.nbytes)
    ctx.h2d(d, P)
    db = ctx.alloc(P.nbytes)
    ctx.h2d(db, P)
    errors.check(L_.rlnc_bitslice_device(ctx.handle, db, L, k, L))
    gens.append((d, db))
e0, e1 = ctx.event(), ctx.event()
for B in [int(b) for b in os.environ.get("KODR_BS_CHECK_B", "1,8,16,32,64,256").split(",")]:
    V = rng.integers(0, 256, (B, k), dtype=np.uint8)
    dV, dO = ctx.alloc(V.nbytes), ctx.alloc(B * L)
    ctx.h2d(dV, V)
    res = {}
    for name, fn in (("perm", lambda i: L_.rlnc_gf_matmul_device(ctx.handle, dV, k, B, k, gens[i % G][0], L, dO, L, L)),
                     ("bs", lambda i: L_.rlnc_gf_matmul_bs_device(ctx.handle, dV, k, B, k, gens[i % G][1], L, dO, L, L))):
        for i in range(3):
            errors.check(fn(i))
        iters = 40 if B <= 64 else 10
        ctx.record(e0)
        for i in range(iters):
            errors.check(fn(i))
        ctx.record(e1)
        res[name] = device.Context.elapsed_ms(e0, e1) * 1e3 / iters
    ok = np.array_equal(ctx.d2h(dO, B * L).reshape(B, L)[:2], oracle.encode(ctx.d2h(gens[(iters - 1) % G][0], k * L).reshape(k, L), V[:2]))
    print(f"B={B:4d}  perm {res['perm']:8.2f} us   bs {res['bs']:8.2f} us   speedup {res['perm']/res['bs']:.2f}  ok={ok}", flush=True)
    ctx.free(dV)
    ctx.free(dO)
