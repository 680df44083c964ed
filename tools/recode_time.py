"""Recode at 32 MiB/256 (bench.py recode_c2's shape): a prepared recoder of
n = k coded wire rows, B recoded pieces per rlnc_recoder_coded_pieces_device
call, median over REPS batches of ITERS back-to-back calls timed with HIP
events on the context stream; the launch plan of the last call.  Prints one
JSON line.  KODR_REC_SIDE=0 runs the vector columns as a launch of their own."""
import ctypes
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kodr_amd import device as kdev, errors  # noqa: E402
from kodr_amd._lib import lib, _u8p, last_launch_plan  # noqa: E402

L_ = lib()
ctx = kdev.Context(0)
k, L, REPS, ITERS = 256, 131072, 7, 20
n, clen = k, k + L
pitch = (clen + 255) // 256 * 256
rng = np.random.default_rng(5)
P = rng.integers(0, 256, k * L, dtype=np.uint8)
enc = ctypes.c_void_p()
errors.check(L_.rlnc_encoder_create(ctx.handle, 0, P.ctypes.data_as(_u8p), k, L, ctypes.byref(enc)))
dW = ctx.alloc(n * pitch)
errors.check(L_.rlnc_encoder_coded_wire_device(enc, n, dW, pitch))
rh = ctypes.c_void_p()
errors.check(L_.rlnc_recoder_create_device(ctx.handle, dW, n, clen, pitch, k, ctypes.byref(rh)))
errors.check(L_.rlnc_recoder_prepare(rh))
R = rng.integers(0, 256, (256, n), dtype=np.uint8)
dR, dO = ctx.alloc(R.nbytes), ctx.alloc(256 * pitch)
ctx.h2d(dR, R)
a, b = ctx.event(), ctx.event()
res = {"side": os.environ.get("KODR_REC_SIDE", "1")}
for B in [int(x) for x in (sys.argv[1:] or ["1", "8", "16", "32", "64", "256"])]:
    ts = []
    for rep in range(REPS + 1):
        ctx.record(a)
        for i in range(ITERS):
            errors.check(L_.rlnc_recoder_coded_pieces_device(rh, dR, B, dO, pitch))
        ctx.record(b)
        ctx.synchronize()
        if rep:
            ts.append(kdev.Context.elapsed_ms(a, b) * 1e3 / ITERS)
    plan = last_launch_plan()
    res[f"B{B}"] = {"us": round(float(np.median(ts)), 2), "plan": [plan[x] for x in ("kernel", "waves", "workgroups")]}
print(json.dumps(res))
L_.rlnc_recoder_destroy(rh)
L_.rlnc_encoder_destroy(enc)
