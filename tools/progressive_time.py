"""Progressive decode at config 4 (16 MiB / 128, systematic, 10 % of the
systematic pieces lost): wire rows arrive in batches of BATCH on the device;
after each batch the consumer reads every newly decoded piece to device
memory.  Policies: EAGER with the generation buffer bound
(rlnc_decoder_bind_output: pieces land in place, the consumer only reads the
mask), EAGER (the AddPiece call materializes what it decoded),
LAZY (each read materializes its piece), and kodr's own API (nothing until
full rank, then GetPieces).  Reports the wall time of the whole stream and
the mean time at which a piece became readable, best of REPS.
With PACE (GB/s of wire bytes) > 0, batch b is not added before
b * batch_bytes / PACE after the start (rows arriving over a link).
usage: python tools/progressive_time.py [BATCH] [PACE]"""
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
BATCH = int(sys.argv[1]) if len(sys.argv) > 1 else 16
PACE = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
REPS = 5
k, L = 128, 131072
rng = np.random.default_rng(4)
lost = set(rng.choice(k, k // 10, replace=False).tolist())
data = rng.integers(0, 256, k * L, dtype=np.uint8)
eh = ctypes.c_void_p()
errors.check(L_.rlnc_encoder_create(ctx.handle, 1, data.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), k, L,
                                    ctypes.byref(eh)))
W = k + L
n_all = k + len(lost) + 2
dAll = ctx.alloc(n_all * W)
errors.check(L_.rlnc_encoder_coded_wire_device(eh, n_all, dAll, W))  # k systematic, then coded
keep = [i for i in range(n_all) if i not in lost]
wire = ctx.d2h(dAll, n_all * W).reshape(n_all, W)[keep]  # drop the lost systematic rows
rows = ctx.alloc(wire.nbytes)
ctx.h2d(rows, np.ascontiguousarray(wire))
ctx.synchronize()
n = len(keep)
dOut = ctx.alloc(k * L)
mask = np.zeros(k, np.uint8)
res = {"k": k, "L": L, "lost": len(lost), "batch": BATCH, "pace_GBps": PACE}
for mode in ("bound", "eager", "lazy", "kodr"):
    best = None
    for rep in range(REPS):
        h = ctypes.c_void_p()
        errors.check(L_.rlnc_decoder_create(ctx.handle, k, ctypes.byref(h)))
        if mode in ("eager", "bound"):
            errors.check(L_.rlnc_decoder_set_policy(h, 1))
        ready = np.zeros(k, bool)
        t_ready = []
        ctx.synchronize()
        t0 = time.perf_counter()
        pos = 0
        while pos < n:
            cnt = min(BATCH, n - pos)
            if PACE > 0:
                due = pos * W / (PACE * 1e9)
                while time.perf_counter() - t0 < due:
                    pass
            c = ctypes.c_size_t()
            st = L_.rlnc_decoder_add_pieces(h, ctypes.c_void_p(rows + pos * W), cnt, W, L, 1, ctypes.byref(c))
            pos += cnt
            if mode == "bound" and pos == cnt:  # the length is known after the first call
                errors.check(L_.rlnc_decoder_bind_output(h, dOut, L))
            if mode == "kodr":
                if L_.rlnc_decoder_is_decoded(h):
                    errors.check(L_.rlnc_decoder_get_pieces_device(h, dOut, L))
                    ctx.synchronize()
                    t_ready += [time.perf_counter() - t0] * k
                    break
                continue
            L_.rlnc_decoder_decoded_mask(h, mask.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
            new = [j for j in range(k) if mask[j] and not ready[j]]
            for j in (new if mode != "bound" else []):
                errors.check(L_.rlnc_decoder_get_decoded(h, j, ctypes.c_void_p(dOut + j * L), 1))
            ctx.synchronize()
            t = time.perf_counter() - t0
            t_ready += [t] * len(new)
            ready[new] = True
            if st == 3 or ready.all():
                break
        total = time.perf_counter() - t0
        assert len(t_ready) == k, (mode, len(t_ready))
        ok = np.array_equal(ctx.d2h(dOut, k * L), data)
        L_.rlnc_decoder_destroy(h)
        cur = (total, float(np.mean(t_ready)), ok)
        best = cur if best is None or cur[0] < best[0] else best
    res[mode] = {"total_us": round(best[0] * 1e6, 1), "mean_ready_us": round(best[1] * 1e6, 1), "ok": best[2]}
if PACE > 0:
    res["last_arrival_us"] = round(((n - 1) // BATCH * BATCH) * W / (PACE * 1e9) * 1e6, 1)
print(json.dumps(res), flush=True)
