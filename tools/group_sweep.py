"""Grouped-encode tile sweep (tuning only): one coded piece of each of G
resident 32 MiB/256 generations per launch, for each KODR_GEMM_CFG tile and
load policy (KODR_GROUP_AUX, tuning build), HIP events over `iters` launches.
Usage: KODR_RLNC_LIB=kodr_amd/tune/libkodr_rlnc.so python tools/group_sweep.py"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kodr_amd import device as kdev, errors  # noqa: E402
from kodr_amd._lib import lib  # noqa: E402

k, L = 256, 131072
G = int(os.environ.get("G", "16"))
CFGS = os.environ.get("CFGS", "1,16,2,8;1,16,1,8;1,4,1,8;1,4,1,16;1,2,1,16;1,1,1,16;1,8,1,8;1,8,2,16").split(";")
L_ = lib()
ctx = kdev.Context(0)
rng = np.random.default_rng(1)
encs = []
for g in range(G):
    d = rng.integers(0, 256, k * L, dtype=np.uint8)
    h = ctypes.c_void_p()
    errors.check(L_.rlnc_encoder_create(ctx.handle, 0, d.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), k, L,
                                        ctypes.byref(h)))
    encs.append(h)
arr = (ctypes.c_void_p * G)(*[e.value for e in encs])
e0, e1 = ctx.event(), ctx.event()
for count in [int(c) for c in os.environ.get("COUNTS", "1").split(",")]:
    V = rng.integers(0, 256, (G, count, k), dtype=np.uint8)
    dV, dO = ctx.alloc(V.nbytes), ctx.alloc(G * count * L)
    ctx.h2d(dV, V)
    ref = None
    for aux in os.environ.get("AUXS", "0,2").split(","):
        os.environ["KODR_GROUP_AUX"] = aux
        for cfg in CFGS:
            os.environ["KODR_GEMM_CFG"] = cfg
            for i in range(5):
                errors.check(L_.rlnc_encoder_group_coded_pieces_device(arr, G, dV, count, dO, L))
            ctx.record(e0)
            it = 40
            for i in range(it):
                errors.check(L_.rlnc_encoder_group_coded_pieces_device(arr, G, dV, count, dO, L))
            ctx.record(e1)
            t = kdev.Context.elapsed_ms(e0, e1) / 1e3 / it
            out = ctx.d2h(dO, G * count * L)
            ok = True if ref is None else bool(np.array_equal(out, ref))
            ref = out if ref is None else ref
            print(f"count={count} aux={aux} cfg={cfg:10s} {t * 1e6:8.2f} us/launch {t / G * 1e6:6.3f} us/gen "
                  f"{G * k * L / t / 1e12:5.2f} TB/s ok={ok}", flush=True)
    ctx.free(dV)
    ctx.free(dO)
