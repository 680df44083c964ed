#!/usr/bin/env python3
"""Encode and decode rates of generations past the kernels' 32-bit offsets
(4 and 8 GiB), where the products run as row chunks XOR-folded together
(capi.cpp gemm_k_chunked).  Device-resident, wall time over back-to-back calls.
Content does not change the timing, so every 64 MiB of the generation is the
same random block; bit-exactness at these sizes is test_generation_past_4_gib.

usage: python tools/big_gen.py [--shapes 256x16,64x128] (k x L in MiB)
"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kodr_amd import device, errors  # noqa: E402
from kodr_amd._codec import FULL  # noqa: E402
from kodr_amd._lib import lib  # noqa: E402


def timed(ctx, fn, iters):
    fn()
    ctx.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    ctx.synchronize()
    return (time.perf_counter() - t0) / iters


def run(ctx, k, L, rng):
    L_ = lib()
    S = k * L
    blk = np.frombuffer(rng.bytes(64 << 20), np.uint8)
    dP = ctx.alloc(S)
    for off in range(0, S, blk.size):
        ctx.h2d(dP + off, blk[:min(blk.size, S - off)])
    eh = ctypes.c_void_p()
    errors.check(L_.rlnc_encoder_create_device(ctx.handle, FULL, dP, k, L, L, ctypes.byref(eh)))
    ctx.free(dP)
    B = 32
    V = rng.integers(0, 256, (k, k), dtype=np.uint8)
    dV, dOut = ctx.alloc(V.nbytes), ctx.alloc(k * L)
    ctx.h2d(dV, V)
    res = {"k": k, "L_MiB": L >> 20, "generation_GiB": S / 2**30}
    for b in (1, B):
        t = timed(ctx, lambda: errors.check(L_.rlnc_encoder_coded_pieces_device(eh, dV, b, dOut, L)), 10)
        res[f"encode_B{b}_ms"] = round(t * 1e3, 3)
        res[f"encode_B{b}_generation_read_GBps"] = round(S / t / 1e9, 1)
    # decode: k coded pieces in, GetPieces out (T x R over the received rows)
    errors.check(L_.rlnc_encoder_coded_pieces_device(eh, dV, k, dOut, L))
    ctx.synchronize()
    dh = ctypes.c_void_p()
    errors.check(L_.rlnc_decoder_create(ctx.handle, k, ctypes.byref(dh)))
    t0 = time.perf_counter()
    for i in range(k):
        v = np.ascontiguousarray(V[i])
        st = L_.rlnc_decoder_add_piece_device(dh, v.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), k,
                                              dOut + i * L, L)
        if st:
            break
    ctx.synchronize()
    t1 = time.perf_counter()
    decoded = bool(L_.rlnc_decoder_is_decoded(dh))
    dDec = ctx.alloc(k * L) if decoded else None
    if decoded:
        errors.check(L_.rlnc_decoder_get_pieces_device(dh, dDec, L))
        ctx.synchronize()
        t2 = time.perf_counter()
        res.update(decode_add_ms=round((t1 - t0) * 1e3, 2), decode_get_ms=round((t2 - t1) * 1e3, 2),
                   decode_gf_macs_per_s=round(k * S / (t2 - t1) / 1e12, 1) * 1e12)
        ok = np.array_equal(ctx.d2h(dDec + (k // 2) * L, 1 << 20), blk[:1 << 20]) if L >= 64 << 20 else None
        res["decoded_row_matches"] = ok
    res["decoded"] = decoded
    L_.rlnc_decoder_destroy(dh)
    L_.rlnc_encoder_destroy(eh)
    for p in (dV, dOut, dDec):
        if p:
            ctx.free(p)
    L_.rlnc_device_pool_trim(ctx.device, 0)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="256x16,64x128")
    args = ap.parse_args()
    ctx = device.Context(0)
    rng = np.random.default_rng(5)
    for sh in args.shapes.split(","):
        k, mib = (int(x) for x in sh.split("x"))
        print(run(ctx, k, mib << 20, rng), flush=True)


if __name__ == "__main__":
    main()
