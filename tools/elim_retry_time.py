"""The 16-decoder elimination's time against its retries: for many fresh
vector sets, one batched AddPiece of G = 16 fresh k = 256 decoders
(rlnc_decoders_add_pieces_gpu, device rows of L = 256 bytes: the
elimination dominates the call), the call's wall time and how many of the
decoders needed a rotated attempt (rlnc_decoder_elim_stats gpu_retried).
Prints one JSON line per set and a summary by retry count.
usage: python tools/elim_retry_time.py [sets] [G]"""
import ctypes
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kodr_amd import device as kdev, errors  # noqa: E402
from kodr_amd._codec import elim_stats  # noqa: E402
from kodr_amd._lib import lib  # noqa: E402

L_ = lib()
ctx = kdev.Context(0)
sets = int(sys.argv[1]) if len(sys.argv) > 1 else 40
G = int(sys.argv[2]) if len(sys.argv) > 2 else 16
k, L = 256, 256
n, pitch = k + 2, ((k + L + 15) // 16) * 16
rng = np.random.default_rng(11)
bufs = [ctx.alloc(n * pitch) for _ in range(G)]
by = {}
for s in range(sets + 2):
    for d in bufs:
        ctx.h2d(d, rng.integers(0, 256, (n, pitch), dtype=np.uint8))
    decs = []
    for _ in range(G):
        h = ctypes.c_void_p()
        errors.check(L_.rlnc_decoder_create(ctx.handle, k, ctypes.byref(h)))
        decs.append(h)
    ctx.synchronize()
    arr = (ctypes.c_void_p * G)(*[x.value for x in decs])
    rp = (ctypes.c_void_p * G)(*bufs)
    cn = (ctypes.c_size_t * G)(*([n] * G))
    cons, sts = (ctypes.c_size_t * G)(), (ctypes.c_int * G)()
    t0 = time.perf_counter()
    errors.check(L_.rlnc_decoders_add_pieces_gpu(arr, G, rp, cn, pitch, L, cons, sts))
    ctx.synchronize()
    t = (time.perf_counter() - t0) * 1e6
    st = [elim_stats(h) for h in decs]
    retried = sum(x["gpu_retried"] for x in st)
    host = sum(x["host_after_gpu"] + x["host"] for x in st)
    for h in decs:
        L_.rlnc_decoder_destroy(h)
    if s < 2:
        continue  # warm-up sets
    print(json.dumps({"set": s, "call_us": round(t, 1), "retried": retried, "host": host}), flush=True)
    by.setdefault(retried, []).append(t)
print(json.dumps({"G": G, "by_retried": {r: {"sets": len(v), "median_call_us": round(statistics.median(v), 1)}
                                         for r, v in sorted(by.items())}}), flush=True)
