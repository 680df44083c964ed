"""Host elimination cost of a systematic stream (BASELINE config 4 shape:
k systematic rows with `LOST` random ones missing, then coded rows) against
an all-coded stream of the same k, one batched AddPiece each, best of 3 over
20 seeds.  Decoder without a device context (coefficient side only)."""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
from kodr_amd._lib import lib
from kodr_amd import errors
L_ = lib()
U8 = ctypes.POINTER(ctypes.c_uint8)
k = int(os.environ.get("K", 128))
lost = int(os.environ.get("LOST", k // 10))
W = k + 32


def run(R):
    best = 1e9
    for rep in range(3):
        dh = ctypes.c_void_p()
        errors.check(L_.rlnc_decoder_create(None, k, ctypes.byref(dh)))
        c = ctypes.c_size_t()
        t0 = time.perf_counter()
        st = L_.rlnc_decoder_add_pieces(dh, R.ctypes.data_as(U8), R.shape[0], W, 32, 0, ctypes.byref(c))
        best = min(best, time.perf_counter() - t0)
        assert st in (0, 3) and L_.rlnc_decoder_is_decoded(dh), st
        L_.rlnc_decoder_destroy(dh)
    return best * 1e6


ts, tc = [], []
for s in range(20):
    rng = np.random.default_rng(s)
    gone = set(rng.choice(k, lost, replace=False).tolist())
    sysr = [i for i in range(k) if i not in gone]
    R = np.zeros((len(sysr) + lost + 4, W), np.uint8)
    for n, i in enumerate(sysr):
        R[n, i] = 1
    R[len(sysr):] = rng.integers(0, 256, (lost + 4, W), dtype=np.uint8)
    ts.append(run(R))
    tc.append(run(rng.integers(0, 256, (k + 4, W), dtype=np.uint8)))
ts.sort()
tc.sort()
print(f"k={k} lost={lost}: systematic us p50 {ts[10]:.1f} (p10 {ts[2]:.1f}); all-coded p50 {tc[10]:.1f}")
