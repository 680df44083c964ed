"""Host time of each call in bench.RoundTripStep (encode launch, AddPiece,
GetPieces, the next decoders' construction, the destroys) over steps run
back to back, medians over the last 10 of 30 steps.  usage: python
tools/rt_host_phases.py (KODR_RLNC_LIB picks the library)"""
import ctypes
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from kodr_amd import device as kdev, errors  # noqa: E402
from kodr_amd._lib import lib  # noqa: E402

L_ = lib()
ctx = kdev.Context(0)
k, L, G = 256, 131072, 16
hs = bench.HeadlineStep(ctx, L_, errors, k, L, 32, G, grouped=True, rng=np.random.default_rng(1))
rt = bench.RoundTripStep(ctx, L_, errors, hs.encs, k, L, np.random.default_rng(2))
ph = {x: [] for x in ("encode", "add", "get", "create", "destroy", "step")}
decs = rt._decoders()
for i in range(30):
    t0 = time.perf_counter()
    s_ = i % len(rt.dW)
    darr = (ctypes.c_void_p * G)(*[x.value for x in decs])
    errors.check(L_.rlnc_encoder_group_coded_pieces_device(rt.earr, G, rt.dV[s_], rt.n, rt.dW[s_] + k, rt.W))
    t1 = time.perf_counter()
    cons, sts = (ctypes.c_size_t * G)(), (ctypes.c_int * G)()
    errors.check(L_.rlnc_decoders_add_pieces_gpu(darr, G, rt.rows[s_], rt.counts, rt.W, L, cons, sts))
    t2 = time.perf_counter()
    errors.check(L_.rlnc_decoders_get_pieces_device(darr, G, rt.dO, L))
    t3 = time.perf_counter()
    nxt = rt._decoders()
    t4 = time.perf_counter()
    for x in decs:
        L_.rlnc_decoder_destroy(x)
    t5 = time.perf_counter()
    decs = nxt
    for key, a, b in (("encode", t0, t1), ("add", t1, t2), ("get", t2, t3), ("create", t3, t4), ("destroy", t4, t5),
                      ("step", t0, t5)):
        ph[key].append((b - a) * 1e6)
ctx.synchronize()
print({key: round(statistics.median(v[-10:]), 1) for key, v in ph.items()}, flush=True)
