"""Repeatability stress for gf_bs_kernel: the same product launched many
times must give identical bytes every time (a missing wait state or an LDS
race shows up as a rare mismatch).  Shapes: the B = 32 headline and the
recoder's M = 258 over wire rows (ncols = k + L, ldx = pitch)."""
import ctypes, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import oracle
from kodr_amd import device, errors
from kodr_amd._lib import lib

L_ = lib()
ctx = device.Context(0)
rng = np.random.default_rng(11)
iters = int(os.environ.get("ITERS", 500))
for (M, K, n, ldx) in [(32, 256, 131072, 131072), (258, 256, 131328, 131584), (16, 256, 131072, 131072)]:
    X = rng.integers(0, 256, (K, ldx), dtype=np.uint8)
    A = rng.integers(0, 256, (M, K), dtype=np.uint8)
    dA, dX, dY = ctx.alloc(A.nbytes), ctx.alloc(X.nbytes), ctx.alloc(M * ldx)
    ctx.h2d(dA, A)
    ctx.h2d(dX, X)
    errors.check(L_.rlnc_bitslice_device(ctx.handle, dX, ldx, K, n))
    errors.check(L_.rlnc_gf_matmul_bs_device(ctx.handle, dA, K, M, K, dX, ldx, dY, ldx, n))
    ctx.synchronize()
    first = ctx.d2h(dY, M * ldx).reshape(M, ldx)[:, :n].copy()
    ref = oracle.encode(np.ascontiguousarray(X[:, :4096]), A)
    assert np.array_equal(first[:, :4096], ref), "first launch differs from the oracle"
    bad = 0
    t0 = time.time()
    for it in range(iters):
        errors.check(L_.rlnc_gf_matmul_bs_device(ctx.handle, dA, K, M, K, dX, ldx, dY, ldx, n))
        ctx.synchronize()
        got = ctx.d2h(dY, M * ldx).reshape(M, ldx)[:, :n]
        if not np.array_equal(got, first):
            bad += 1
            w = np.argwhere(got != first)
            print(f"  M={M} iter {it}: {len(w)} bytes differ, rows {np.unique(w[:, 0])[:10].tolist()} "
                  f"blocks {np.unique(w[:, 1] // 32)[:10].tolist()}", flush=True)
            if bad >= 5:
                break
    print(f"M={M} K={K} n={n}: {iters} launches, {bad} differing, {time.time() - t0:.1f}s", flush=True)
    for p in (dA, dX, dY):
        ctx.free(p)

# the recoder flow: fresh recoder (pool buffers, out-of-place twin) per round
k, L = 256, 131072
clen, pitch = k + L, (k + L + 255) // 256 * 256
W = rng.integers(0, 256, (k, pitch), dtype=np.uint8)
R = rng.integers(0, 256, (k + 2, k), dtype=np.uint8)
dW, dR, dO = ctx.alloc(W.nbytes), ctx.alloc(R.nbytes), ctx.alloc((k + 2) * pitch)
ctx.h2d(dW, W)
ctx.h2d(dR, R)
first, bad = None, 0
t0 = time.time()
for it in range(iters // 2):
    rh = ctypes.c_void_p()
    errors.check(L_.rlnc_recoder_create_device(ctx.handle, dW, k, clen, pitch, k, ctypes.byref(rh)))
    errors.check(L_.rlnc_recoder_coded_pieces_device(rh, dR, k + 2, dO, pitch))
    ctx.synchronize()
    L_.rlnc_recoder_destroy(rh)
    got = ctx.d2h(dO, (k + 2) * pitch).reshape(k + 2, pitch)[:, :clen].copy()
    if first is None:
        first = got
        assert np.array_equal(first[:, :4096], oracle.recode(np.ascontiguousarray(W[:, :4096]), k, R))
    elif not np.array_equal(got, first):
        bad += 1
        w = np.argwhere(got != first)
        print(f"  recoder round {it}: {len(w)} bytes differ, rows {np.unique(w[:, 0])[:10].tolist()} "
              f"blocks {np.unique(w[:, 1] // 32)[:10].tolist()}", flush=True)
        if bad >= 5:
            break
print(f"recoder rounds: {iters // 2}, {bad} differing, {time.time() - t0:.1f}s", flush=True)
