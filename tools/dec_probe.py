"""Decoder apply-path probe: one-shot systematic decodes of a 32 MiB/256
generation with `lost` systematic pieces replaced by coded ones, timed per
phase (bench.time_decode).  KODR_BS_MIN_ROWS_DEC (tuning build) moves the
plain/bit-sliced switch of the decoder's apply product."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import ctypes
import bench
from kodr_amd import device, errors
from kodr_amd._lib import lib

L_ = lib()
ctx = device.Context(0)
rng = np.random.default_rng(5)
k, L = int(os.environ.get("K", 256)), int(os.environ.get("L", 131072))
W = k + L
data = rng.integers(0, 256, k * L, dtype=np.uint8)
eh = ctypes.c_void_p()
errors.check(L_.rlnc_encoder_create(ctx.handle, 1, data.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), k, L,
                                    ctypes.byref(eh)))
errors.check(L_.rlnc_encoder_seed(eh, 4))
n = k + 64
dAll = ctx.alloc(n * W)
errors.check(L_.rlnc_encoder_coded_wire_device(eh, n, dAll, W))
rows = ctx.d2h(dAll, n * W).reshape(n, W)
dDec = ctx.alloc(k * L)
for lost_n in [int(x) for x in os.environ.get("LOST", "4,8,12,16,24,32,48,64").split(",")]:
    lost = set(rng.choice(k, lost_n, replace=False).tolist())
    keep = [i for i in range(k) if i not in lost] + list(range(k, k + lost_n))
    kept = np.ascontiguousarray(rows[keep])
    dK = ctx.alloc(kept.nbytes)
    ctx.h2d(dK, kept)
    r = bench.time_decode(ctx, L_, errors, dK, kept.shape[0], W, k, L, dDec, reps=5)
    ok = np.array_equal(ctx.d2h(dDec, k * L), data)
    print(f"lost={lost_n:3d} gf_rows={r['gf_rows']:3d} copy={r['copy_rows']:3d} add {r['add_s']*1e6:7.1f} us"
          f"  get {r['get_s']*1e6:7.1f} us  total {r['s']*1e6:7.1f} us  ok={ok}", flush=True)
    ctx.free(dK)
