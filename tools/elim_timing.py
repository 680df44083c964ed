"""Phase timeline of gf_elim (tuning build with -DKODR_ELIM_TIMING, via
KODR_RLNC_LIB): s_memtime stamps of step 10 per wave, read back from the
kernel's output buffer through a throwaway decoder call."""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kodr_amd import device as kdev, errors
from kodr_amd._lib import lib
L_ = lib()
ctx = kdev.Context(0)
rng = np.random.default_rng(1)
k = int(sys.argv[1]) if len(sys.argv) > 1 else 256
n = k + 2
pitch = k + 256
rows = rng.integers(0, 256, (n, pitch), dtype=np.uint8)
d = ctx.alloc(rows.nbytes)
ctx.h2d(d, rows)
h = ctypes.c_void_p()
errors.check(L_.rlnc_decoder_create(ctx.handle, k, ctypes.byref(h)))
c = ctypes.c_size_t()
L_.rlnc_decoder_add_pieces_gpu(h, d, n, pitch, 256, ctypes.byref(c))
ctx.synchronize()
# the stamps sit where the state would: read the context's elim_out via a decoder transform is not
# possible; the library's d2h copy of it is in the decoder's state -> print through load failure path
print("consumed", c.value)
buf = np.fromfile(os.environ["KODR_ELIM_DUMP"], dtype=np.uint8)
st = buf[256:256 + 16 * 64].view(np.uint64).reshape(16, 8).astype(np.int64)
names = ["A-cand", "barrierA", "owner", "barrierB", "elim", "->step11 end", "->loop end"]
for w in range(16):
    t = st[w]
    print(f"wave {w:2d}: " + " ".join(f"{names[i]} {t[i + 1] - t[i]:6d}" for i in range(5)),
          f"step {t[5] - t[0]:6d}", f"step11 {t[6] - t[5]:6d}")
