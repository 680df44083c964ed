"""GetPieces-to-device cost of a decoded decoder, repeated: config 4
(16 MiB/128, 10 % of the systematic pieces replaced by coded ones) and the
all-coded decode of the same generation.  Prints us per call; run under
rocprofv3 --kernel-trace for the per-kernel split."""
import ctypes, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np
from kodr_amd import device, errors
from kodr_amd._lib import lib

L_ = lib()
ctx = device.Context(0)
rng = np.random.default_rng(4)
k, L = int(os.environ.get("K", 128)), 131072
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
cases = {"systematic": [i for i in range(k) if i not in lost] + list(range(k, n)), "coded": list(range(k, n))}
dDec = ctx.alloc(k * L)
for name, keep in cases.items():
    kept = np.ascontiguousarray(rows[keep])
    dK = ctx.alloc(kept.nbytes)
    ctx.h2d(dK, kept)
    dh = ctypes.c_void_p()
    errors.check(L_.rlnc_decoder_create(ctx.handle, k, ctypes.byref(dh)))
    c = ctypes.c_size_t()
    t0 = time.perf_counter()
    st = L_.rlnc_decoder_add_pieces(dh, dK, kept.shape[0], W, L, 1, ctypes.byref(c))
    t1 = time.perf_counter()
    ts = []
    for i in range(30):
        a = time.perf_counter()
        errors.check(L_.rlnc_decoder_get_pieces_device(dh, dDec, L))
        b = time.perf_counter()
        ctx.synchronize()
        ts.append((b - a, time.perf_counter() - a))
    ok = np.array_equal(ctx.d2h(dDec, k * L), data)
    ts.sort(key=lambda x: x[1])
    print(f"{name}: add {1e6 * (t1 - t0):.1f} us; get (call returns, +sync) best {1e6 * ts[0][0]:.1f} / "
          f"{1e6 * ts[0][1]:.1f} us, median {1e6 * ts[15][0]:.1f} / {1e6 * ts[15][1]:.1f} us, ok={ok}", flush=True)
    L_.rlnc_decoder_destroy(dh)
    ctx.free(dK)
