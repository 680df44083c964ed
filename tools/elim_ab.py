"""A/B of the batched GPU AddPiece (rlnc_decoders_add_pieces_gpu) between two
builds of the library: fresh decoders, k + 2 random device wire rows each,
wall time per call (median of REPS) -- run under rocprofv3 --kernel-trace
--stats for the elimination kernels' durations.  Binds only the entry points
both builds export.  usage: python tools/elim_ab.py LIB k G L [reps] [seed]"""
import ctypes
import statistics
import sys
import time

import numpy as np

lib = ctypes.CDLL(sys.argv[1])
k, G, L = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
REPS = int(sys.argv[5]) if len(sys.argv) > 5 else 30
seed = int(sys.argv[6]) if len(sys.argv) > 6 else 3
vp, sz = ctypes.c_void_p, ctypes.c_size_t
lib.rlnc_ctx_create.argtypes = [ctypes.c_int, vp, ctypes.POINTER(vp)]
lib.rlnc_dev_alloc.argtypes = [vp, sz, ctypes.POINTER(vp)]
lib.rlnc_memcpy_h2d.argtypes = [vp, vp, vp, sz]
lib.rlnc_decoder_create.argtypes = [vp, sz, ctypes.POINTER(vp)]
lib.rlnc_decoder_destroy.argtypes = [vp]
lib.rlnc_ctx_synchronize.argtypes = [vp]
lib.rlnc_decoders_add_pieces_gpu.argtypes = [ctypes.POINTER(vp), sz, ctypes.POINTER(vp), ctypes.POINTER(sz), sz, sz,
                                             ctypes.POINTER(sz), ctypes.POINTER(ctypes.c_int)]
ctx = vp()
assert lib.rlnc_ctx_create(0, None, ctypes.byref(ctx)) == 0
n = k + 2
pitch = (k + L + 15) // 16 * 16
rng = np.random.default_rng(seed)
bufs = []
for g in range(G):
    rows = rng.integers(0, 256, (n, pitch), dtype=np.uint8)
    d = vp()
    assert lib.rlnc_dev_alloc(ctx, rows.nbytes, ctypes.byref(d)) == 0
    assert lib.rlnc_memcpy_h2d(ctx, d, rows.ctypes.data, rows.nbytes) == 0
    bufs.append(d.value)
ts = []
for rep in range(REPS + 3):
    decs = [vp() for _ in range(G)]
    for h in decs:
        assert lib.rlnc_decoder_create(ctx, k, ctypes.byref(h)) == 0
    lib.rlnc_ctx_synchronize(ctx)
    arr = (vp * G)(*[h.value for h in decs])
    rws = (vp * G)(*bufs)
    cnt = (sz * G)(*([n] * G))
    cons, sts = (sz * G)(), (ctypes.c_int * G)()
    t0 = time.perf_counter()
    assert lib.rlnc_decoders_add_pieces_gpu(arr, G, rws, cnt, pitch, L, cons, sts) == 0
    t1 = time.perf_counter()
    if rep >= 3:
        ts.append(t1 - t0)
    for h in decs:
        lib.rlnc_decoder_destroy(h)
print(f"{sys.argv[1]} k={k} G={G} L={L}: call median {statistics.median(ts) * 1e6:.1f} us, "
      f"min {min(ts) * 1e6:.1f}, max {max(ts) * 1e6:.1f}", flush=True)
