"""C2 single-decoder decode as bench.time_decode runs it (one batched
rlnc_decoder_add_pieces call over k + 2 device wire rows, then
rlnc_decoder_get_pieces_device), per repetition, with the AddPiece call's own
phases when KODR_ADD_TIMING=1.  usage: python tools/c2_add_phases.py [reps]
[seed] (seed: rlnc_encoder_seed before the wire rows, as bench.py's c2_decode
uses 7)"""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kodr_amd import device as kdev, errors  # noqa: E402
from kodr_amd._lib import lib  # noqa: E402

L_ = lib()
ctx = kdev.Context(0)
k, L = 256, 131072
n, W = k + 2, k + L
rng = np.random.default_rng(7)
P = rng.integers(0, 256, (k, L), dtype=np.uint8)
e = ctypes.c_void_p()
dP = ctx.alloc(k * L)
ctx.h2d(dP, P)
errors.check(L_.rlnc_encoder_create_device(ctx.handle, 0, dP, k, L, L, ctypes.byref(e)))
dWire, dDec = ctx.alloc(n * W), ctx.alloc(k * L)
if len(sys.argv) > 2:
    L_.rlnc_encoder_seed(e, int(sys.argv[2]))
errors.check(L_.rlnc_encoder_coded_wire_device(e, n, dWire, W))
ctx.synchronize()
for rep in range(int(sys.argv[1]) if len(sys.argv) > 1 else 8):
    dh = ctypes.c_void_p()
    errors.check(L_.rlnc_decoder_create(ctx.handle, k, ctypes.byref(dh)))
    consumed = ctypes.c_size_t()
    t0 = time.perf_counter()
    st = L_.rlnc_decoder_add_pieces(dh, dWire, n, W, L, 1, ctypes.byref(consumed))
    assert st in (0, 3), st
    t1 = time.perf_counter()
    errors.check(L_.rlnc_decoder_get_pieces_device(dh, dDec, L))
    t2 = time.perf_counter()
    ctx.synchronize()
    t3 = time.perf_counter()
    ok = bool(np.array_equal(ctx.d2h(dDec, k * L).reshape(k, L), P)) if rep == 0 else None
    L_.rlnc_decoder_destroy(dh)
    print(f"rep {rep}: add {1e6 * (t1 - t0):7.1f} us, get call {1e6 * (t2 - t1):7.1f}, get to idle "
          f"{1e6 * (t3 - t2):7.1f}, total {1e6 * (t3 - t0):7.1f}" + ("" if ok is None else f", decoded ok {ok}"),
          flush=True)
L_.rlnc_encoder_destroy(e)
for p_ in (dP, dWire, dDec):
    ctx.free(p_)
