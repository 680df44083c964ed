"""Phase totals of the blocked gf_elim kernel (tuning build with
-DKODR_ELIM_TIMING, via KODR_RLNC_LIB and KODR_ELIM_DUMP): s_memtime cycles
per wave summed over the panels."""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kodr_amd import device as kdev, errors  # noqa: E402
from kodr_amd._lib import lib  # noqa: E402
L_ = lib()
ctx = kdev.Context(0)
rng = np.random.default_rng(1)
k = int(sys.argv[1]) if len(sys.argv) > 1 else 256
n = k + 2
pitch = k + 256
rows = rng.integers(0, 256, (n, pitch), dtype=np.uint8)
d = ctx.alloc(rows.nbytes)
ctx.h2d(d, rows)
for rep in range(2):
    h = ctypes.c_void_p()
    errors.check(L_.rlnc_decoder_create(ctx.handle, k, ctypes.byref(h)))
    c = ctypes.c_size_t()
    L_.rlnc_decoder_add_pieces_gpu(h, d, n, pitch, 256, ctypes.byref(c))
    ctx.synchronize()
    L_.rlnc_decoder_destroy(h)
buf = np.fromfile(os.environ["KODR_ELIM_DUMP"], dtype=np.uint8)
st = buf[256:256 + 16 * 64].view(np.uint64).reshape(16, 8).astype(np.int64)
names = ["owner", "bar1", "pivots", "bar2", "update", "total"]
for w in range(16):
    print(f"wave {w:2d}: " + " ".join(f"{names[i]} {st[w][i]:8d}" for i in range(6)))
