"""Config-4 decode timeline probe: the bench's c4_systematic_decode leg
(16 MiB/128, 10 % of the systematic pieces lost, device rows, one batched
AddPiece + GetPieces into device memory), repeated REPS times for each of
the systematic and the all-coded stream, with host timestamps per phase.
Run it under `rocprofv3 --hip-trace --kernel-trace` to see where add_s and
get_s go."""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kodr_amd import device as kdev, errors  # noqa: E402
from kodr_amd._lib import lib  # noqa: E402

REPS = int(os.environ.get("REPS", "6"))
L_ = lib()
ctx = kdev.Context(0)
rng = np.random.default_rng(3)
k, L = 128, 131072
W = k + L
data = rng.integers(0, 256, k * L, dtype=np.uint8)
eh = ctypes.c_void_p()
errors.check(L_.rlnc_encoder_create(ctx.handle, 1, data.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), k, L,
                                    ctypes.byref(eh)))
errors.check(L_.rlnc_encoder_seed(eh, 4))
n = 2 * k + 4
dAll = ctx.alloc(n * W)
errors.check(L_.rlnc_encoder_coded_wire_device(eh, n, dAll, W))
rows = ctx.d2h(dAll, n * W).reshape(n, W)
lost = set(rng.choice(k, k // 10, replace=False).tolist())
keep = [i for i in range(k) if i not in lost] + list(range(k, n))
streams = {"systematic": np.ascontiguousarray(rows[keep]), "coded": np.ascontiguousarray(rows[k:])}
dDec = ctx.alloc(k * L)
res = {}
for name, R in streams.items():
    dR = ctx.alloc(R.nbytes)
    ctx.h2d(dR, R)
    ts = []
    for rep in range(REPS):
        dh = ctypes.c_void_p()
        errors.check(L_.rlnc_decoder_create(ctx.handle, k, ctypes.byref(dh)))
        ctx.synchronize()
        c = ctypes.c_size_t()
        t0 = time.perf_counter()
        st = L_.rlnc_decoder_add_pieces(dh, dR, R.shape[0], W, L, 1, ctypes.byref(c))
        t1 = time.perf_counter()
        errors.check(L_.rlnc_decoder_get_pieces_device(dh, dDec, L))
        ctx.synchronize()
        t2 = time.perf_counter()
        assert st == 3, st
        L_.rlnc_decoder_destroy(dh)
        ts.append((round((t1 - t0) * 1e6, 1), round((t2 - t1) * 1e6, 1)))
    ok = bool(np.array_equal(ctx.d2h(dDec, k * L), data))
    res[name] = {"add_get_us": ts, "ok": ok}
    ctx.free(dR)
print(json.dumps(res))
