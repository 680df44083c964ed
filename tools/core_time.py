"""Host elimination cost alone (decoder without a device context): k + 4
random coded rows through one batched AddPiece, best of 3, 40 seeds."""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from kodr_amd._lib import lib
from kodr_amd import errors
L_ = lib()
U8 = ctypes.POINTER(ctypes.c_uint8)
k = int(os.environ.get("K", 256))
ts = []
for s in range(40):
    rng = np.random.default_rng(s)
    R = rng.integers(0, 256, (k + 4, k + 32), dtype=np.uint8)
    best = 1e9
    for rep in range(3):
        dh = ctypes.c_void_p()
        errors.check(L_.rlnc_decoder_create(None, k, ctypes.byref(dh)))
        c = ctypes.c_size_t()
        t0 = time.perf_counter()
        L_.rlnc_decoder_add_pieces(dh, R.ctypes.data_as(U8), R.shape[0], k + 32, 32, 0, ctypes.byref(c))
        best = min(best, time.perf_counter() - t0)
        L_.rlnc_decoder_destroy(dh)
    ts.append(best * 1e6)
ts.sort()
print(f"k={k}: host elimination us p10 {ts[4]:.0f} p50 {ts[20]:.0f} p90 {ts[36]:.0f}")
