"""Kernel-time probe of gf_elim (run under rocprofv3 --kernel-trace): one
fresh decoder per call, k = 256 (and 64), n rows in the batch."""
import ctypes, os, sys
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kodr_amd import device as kdev, errors
from kodr_amd._lib import lib
L_ = lib()
ctx = kdev.Context(0)
rng = np.random.default_rng(1)
for k in (256, 64):
    for n in (4, 64, k + 2):
        pitch = k + 256
        rows = rng.integers(0, 256, (n, pitch), dtype=np.uint8)
        d = ctx.alloc(rows.nbytes)
        ctx.h2d(d, rows)
        for rep in range(3):
            h = ctypes.c_void_p()
            errors.check(L_.rlnc_decoder_create(ctx.handle, k, ctypes.byref(h)))
            c = ctypes.c_size_t()
            L_.rlnc_decoder_add_pieces_gpu(h, d, n, pitch, 256, ctypes.byref(c))
            L_.rlnc_decoder_destroy(h)
        ctx.synchronize()
        print(k, n, c.value, flush=True)
        ctx.free(d)
