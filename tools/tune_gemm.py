#!/usr/bin/env python3
"""Sweep gf_gemm tiles (KODR_GEMM_CFG) on the GPU at the encode/decode shapes.

usage: python tools/tune_gemm.py [--M 1,4,8,16,256] [--K 256] [--L 131072] [--gens 16]
Prints one line per (M, tile): us/launch, compulsory GB/s, GF-MAC/s; checks
every tile's output equals the default tile's output.
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kodr_amd import device, errors  # noqa: E402
from kodr_amd._lib import lib  # noqa: E402

TILES = ["1,16,4", "1,16,2", "1,16,1", "2,16,4", "2,16,2", "4,16,4", "4,16,2", "4,16,1", "8,16,4",
         "8,16,2", "8,8,2", "4,8,2", "8,8,4", "16,8,2", "8,4,1", "16,4,1", "8,4,2", "16,4,2"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--M", default="1,2,4,8,16,32,256")
    ap.add_argument("--K", type=int, default=256)
    ap.add_argument("--L", type=int, default=131072)
    ap.add_argument("--gens", type=int, default=16)
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--tiles", default="")
    args = ap.parse_args()
    tiles = args.tiles.split(";") if args.tiles else TILES
    ctx = device.Context(0)
    K, L, G = args.K, args.L, args.gens
    rng = np.random.default_rng(0)
    gen = ctx.alloc(G * K * L)
    for g in range(G):
        ctx.h2d(gen + g * K * L, rng.integers(0, 256, K * L, dtype=np.uint8))
    Mmax = max(int(m) for m in args.M.split(","))
    A = rng.integers(0, 256, (Mmax, K), dtype=np.uint8)
    dA = ctx.alloc(A.nbytes)
    ctx.h2d(dA, A)
    dY = ctx.alloc(Mmax * L)
    e0, e1 = ctx.event(), ctx.event()
    L_ = lib()
    for M in [int(m) for m in args.M.split(",")]:
        os.environ.pop("KODR_GEMM_CFG", None)
        errors.check(L_.rlnc_gf_matmul_device(ctx.handle, dA, K, M, K, gen, L, dY, L, L))
        ref = ctx.d2h(dY, M * L)
        for t in tiles:
            mt = int(t.split(",")[0])
            if mt > M * 2 and mt > 1:
                continue
            os.environ["KODR_GEMM_CFG"] = t
            st = L_.rlnc_gf_matmul_device(ctx.handle, dA, K, M, K, gen, L, dY, L, L)
            if st != 0:
                print(f"M={M} tile={t}: status {st}")
                continue
            ok = np.array_equal(ctx.d2h(dY, M * L), ref)
            for i in range(5):
                L_.rlnc_gf_matmul_device(ctx.handle, dA, K, M, K, gen + (i % G) * K * L, L, dY, L, L)
            ctx.record(e0)
            for i in range(args.iters):
                L_.rlnc_gf_matmul_device(ctx.handle, dA, K, M, K, gen + (i % G) * K * L, L, dY, L, L)
            ctx.record(e1)
            us = device.Context.elapsed_ms(e0, e1) * 1e3 / args.iters
            gbs = (K * L + M * L) / us / 1e3
            macs = M * K * L / us / 1e6
            print(f"M={M:4d} tile={t:8s} {us:9.2f} us  {gbs:8.1f} GB/s  {macs:8.1f} TMAC/s  ok={ok}", flush=True)
    os.environ.pop("KODR_GEMM_CFG", None)


if __name__ == "__main__":
    main()
