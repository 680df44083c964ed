#!/usr/bin/env python3
"""Bit-sliced kernel vs gf_gemm for 9..32 output rows over few rows of X.

The encoder takes gf_bs_kernel from 9 coded pieces per call (capi.cpp
kBsMinRows, measured at k = 256); this times both kernels on the same product
at small K: the encoder path (bit-sliced, twin built once) against the raw
rlnc_gf_matmul_device (gf_gemm_kernel), device-resident, wall time per call.

usage: python tools/bs_vs_gemm_small_k.py
"""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kodr_amd import device, errors  # noqa: E402
from kodr_amd._codec import FULL  # noqa: E402
from kodr_amd._lib import lib  # noqa: E402


def timed(ctx, fn, iters=50):
    fn()
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    ctx.synchronize()
    return (time.perf_counter() - t0) / iters * 1e6


def main():
    L_ = lib()
    ctx = device.Context(0)
    rng = np.random.default_rng(9)
    for K in (16, 32, 64, 128):
        for L in (131072, 1 << 20):
            dP = ctx.alloc(K * L)
            ctx.h2d(dP, rng.integers(0, 256, K * L, dtype=np.uint8))
            eh = ctypes.c_void_p()
            errors.check(L_.rlnc_encoder_create_device(ctx.handle, FULL, dP, K, L, L, ctypes.byref(eh)))
            for M in (9, 16, 32):
                V = rng.integers(0, 256, (M, K), dtype=np.uint8)
                dV, dY, dY2 = ctx.alloc(V.nbytes), ctx.alloc(M * L), ctx.alloc(M * L)
                ctx.h2d(dV, V)
                t_bs = timed(ctx, lambda: errors.check(L_.rlnc_encoder_coded_pieces_device(eh, dV, M, dY, L)))
                t_gm = timed(ctx, lambda: errors.check(
                    L_.rlnc_gf_matmul_device(ctx.handle, dV, K, M, K, dP, L, dY2, L, L)))
                same = np.array_equal(ctx.d2h(dY, M * L), ctx.d2h(dY2, M * L))
                print(f"K={K:4d} L={L:8d} M={M:3d}  bs {t_bs:8.2f} us  gemm {t_gm:8.2f} us  "
                      f"bs/gemm {t_bs / t_gm:5.2f}  same={same}", flush=True)
                for p in (dV, dY, dY2):
                    ctx.free(p)
            L_.rlnc_encoder_destroy(eh)
            ctx.free(dP)


if __name__ == "__main__":
    main()
