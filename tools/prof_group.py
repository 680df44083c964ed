"""Grouped encode for the profiler: one coded piece (COUNT) of each of G
resident 32 MiB/256 generations per launch (rlnc_encoder_group_coded_pieces_device,
the north-star shape), ITERS launches after 5 warm-ups, production tile
choice.  Prints the HIP-event average per launch; tools/pmc_group.sh runs it
under rocprofv3 kernel-trace and FETCH_SIZE / WRITE_SIZE passes."""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kodr_amd import device as kdev, errors  # noqa: E402
from kodr_amd._lib import lib  # noqa: E402

k, L = 256, 131072
G = int(os.environ.get("G", "16"))
COUNT = int(os.environ.get("COUNT", "1"))
ITERS = int(os.environ.get("ITERS", "40"))
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
V = rng.integers(0, 256, (G, COUNT, k), dtype=np.uint8)
dV, dO = ctx.alloc(V.nbytes), ctx.alloc(G * COUNT * L)
ctx.h2d(dV, V)
for i in range(5):
    errors.check(L_.rlnc_encoder_group_coded_pieces_device(arr, G, dV, COUNT, dO, L))
e0, e1 = ctx.event(), ctx.event()
ctx.record(e0)
for i in range(ITERS):
    errors.check(L_.rlnc_encoder_group_coded_pieces_device(arr, G, dV, COUNT, dO, L))
ctx.record(e1)
t = kdev.Context.elapsed_ms(e0, e1) / 1e3 / ITERS
hbm = G * (k * L + COUNT * (k + L))
print(json.dumps({"G": G, "count": COUNT, "iters": ITERS, "events_us_per_launch": round(t * 1e6, 3),
                  "compulsory_hbm_bytes_per_launch": hbm, "hbm_GBps": round(hbm / t / 1e9, 1)}))
for h in encs:
    L_.rlnc_encoder_destroy(h)
