"""The relay hop's recode step on one GPU (bench.py HipRelayEngine.recode:
rlnc_recoder_create_device on k received wire rows, k recoded pieces,
destroy), timed per repetition with the phases split, to see where its
milliseconds go.  usage: python tools/relay_recode_time.py"""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kodr_amd import device as kdev, errors, dist as kdist  # noqa: E402
from kodr_amd._lib import lib, _u8p  # noqa: E402

L_ = lib()
ctx = kdev.Context(0)
k, L = 256, 131072
clen = k + L
pitch = kdist.wire_pitch(k, L)
rng = np.random.default_rng(2)
data = rng.integers(0, 256, k * L, dtype=np.uint8)
eh = ctypes.c_void_p()
errors.check(L_.rlnc_encoder_create(ctx.handle, 0, data.ctypes.data_as(_u8p), k, L, ctypes.byref(eh)))
errors.check(L_.rlnc_encoder_prepare(eh))
dW, dO = ctx.alloc(k * pitch), ctx.alloc(k * pitch)
dR = ctx.alloc(k * k)
ctx.h2d(dR, rng.integers(0, 256, k * k, dtype=np.uint8))
for rep in range(6):
    ctx.synchronize()
    t0 = time.perf_counter()
    errors.check(L_.rlnc_encoder_coded_wire_device(eh, k, dW, pitch))
    ctx.synchronize()
    t1 = time.perf_counter()
    rh = ctypes.c_void_p()
    errors.check(L_.rlnc_recoder_create_device(ctx.handle, dW, k, clen, pitch, k, ctypes.byref(rh)))
    ctx.synchronize()
    t2 = time.perf_counter()
    errors.check(L_.rlnc_recoder_coded_pieces_device(rh, dR, k, dO, pitch))
    ctx.synchronize()
    t3 = time.perf_counter()
    L_.rlnc_recoder_destroy(rh)
    t4 = time.perf_counter()
    print(f"rep {rep}: encode {1e3 * (t1 - t0):.3f} ms, create {1e3 * (t2 - t1):.3f}, recode {1e3 * (t3 - t2):.3f},"
          f" destroy {1e3 * (t4 - t3):.3f}", flush=True)
