"""Host phases of bench.RoundTripStep (the encode_decode step): wall time of
the add and get calls and of decoder construction, per step, with the
AddPiece call's own phases (KODR_ADD_TIMING=1 prints them to stderr).
usage: KODR_ADD_TIMING=1 python tools/rt_phases.py [steps]"""
import ctypes
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from kodr_amd import device as kdev, errors  # noqa: E402
from kodr_amd._lib import lib  # noqa: E402

L_ = lib()
ctx = kdev.Context(0)
hs = bench.HeadlineStep(ctx, L_, errors, 256, 131072, 32, 16, grouped=True, rng=np.random.default_rng(1), nvec=2)
rt = bench.RoundTripStep(ctx, L_, errors, hs.encs, 256, 131072, np.random.default_rng(2))
G, k, L = rt.G, rt.k, rt.L
for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 6):
    tc0 = time.perf_counter()
    decs = rt._decoders()
    tc1 = time.perf_counter()
    darr = (ctypes.c_void_p * G)(*[x.value for x in decs])
    errors.check(L_.rlnc_encoder_group_coded_pieces_device(rt.earr, G, rt.dV[0], rt.n, rt.dW[0] + k, rt.W))
    ctx.synchronize()
    t0 = time.perf_counter()
    cons, sts = (ctypes.c_size_t * G)(), (ctypes.c_int * G)()
    errors.check(L_.rlnc_decoders_add_pieces_gpu(darr, G, rt.rows[0], rt.counts, rt.W, L, cons, sts))
    t1 = time.perf_counter()
    errors.check(L_.rlnc_decoders_get_pieces_device(darr, G, rt.dO, L))
    t2 = time.perf_counter()
    ctx.synchronize()
    t3 = time.perf_counter()
    for x in decs:
        L_.rlnc_decoder_destroy(x)
    t4 = time.perf_counter()
    print(f"step {i}: create {1e6 * (tc1 - tc0):7.1f} us, add call {1e6 * (t1 - t0):7.1f}, get call (host) "
          f"{1e6 * (t2 - t1):7.1f}, get to idle {1e6 * (t3 - t2):7.1f}, destroy {1e6 * (t4 - t3):7.1f}", flush=True)
rt.close()
hs.close()
