"""Batched AddPiece on G fresh decoders: the elimination on the host
(rlnc_decoder_add_pieces per decoder) vs on the GPU (one
rlnc_decoders_add_pieces_gpu call, a workgroup per decoder), device wire
rows, wall time per call, best of REPS.  usage: python tools/elim_time.py
[k,...] [G,...] [L]"""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kodr_amd import device as kdev, errors  # noqa: E402
from kodr_amd._lib import lib  # noqa: E402

L_ = lib()
ctx = kdev.Context(0)
ks = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "64,128,256").split(",")]
Gs = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,8,32").split(",")]
L = int(sys.argv[3]) if len(sys.argv) > 3 else 256
REPS = 5
rng = np.random.default_rng(3)
for k in ks:
    n = k + 2
    pitch = ((k + L + 15) // 16) * 16
    for G in Gs:
        bufs = []
        for g in range(G):
            rows = rng.integers(0, 256, (n, pitch), dtype=np.uint8)
            d = ctx.alloc(rows.nbytes)
            ctx.h2d(d, rows)
            bufs.append(d)
        res = {"k": k, "G": G, "L": L}
        for mode in ("host", "gpu"):
            best = None
            for rep in range(REPS):
                decs = []
                for g in range(G):
                    h = ctypes.c_void_p()
                    errors.check(L_.rlnc_decoder_create(ctx.handle, k, ctypes.byref(h)))
                    decs.append(h)
                ctx.synchronize()
                t0 = time.perf_counter()
                if mode == "host":
                    ctx.set_route_min_k(100000)  # kodr's elimination on the host (no GPU route)
                    for g in range(G):
                        c = ctypes.c_size_t()
                        st = L_.rlnc_decoder_add_pieces(decs[g], bufs[g], n, pitch, L, 1, ctypes.byref(c))
                        assert st in (0, 3), st
                    ctx.set_route_min_k(224)
                else:
                    arr = (ctypes.c_void_p * G)(*[x.value for x in decs])
                    rp = (ctypes.c_void_p * G)(*bufs)
                    cn = (ctypes.c_size_t * G)(*([n] * G))
                    cons = (ctypes.c_size_t * G)()
                    sts = (ctypes.c_int * G)()
                    errors.check(L_.rlnc_decoders_add_pieces_gpu(arr, G, rp, cn, pitch, L, cons, sts))
                    assert all(s in (0, 3) for s in sts), list(sts)
                ctx.synchronize()
                t = time.perf_counter() - t0
                ok = all(L_.rlnc_decoder_is_decoded(x) for x in decs)
                for x in decs:
                    L_.rlnc_decoder_destroy(x)
                best = t if best is None else min(best, t)
            res[mode + "_us"] = round(best * 1e6, 1)
            res[mode + "_decoded"] = ok
        res["gpu_speedup"] = round(res["host_us"] / res["gpu_us"], 2)
        print(json.dumps(res), flush=True)
        for d in bufs:
            ctx.free(d)
