"""D2H of coded wire rows (258 x 131,328 B out of a 131,584-B device pitch)
into pinned host memory: one 2-D copy vs the same rows split over 2 or 4
streams (separate copy engines).  Measurement only."""
import ctypes, time
hip = ctypes.CDLL("libamdhip64.so")
vp, sz = ctypes.c_void_p, ctypes.c_size_t
hip.hipMemcpy2DAsync.argtypes = [vp, sz, vp, sz, sz, sz, ctypes.c_int, vp]
hip.hipMemcpyAsync.argtypes = [vp, vp, sz, ctypes.c_int, vp]
rows, w, pitch = 258, 131328, 131584
d, h = vp(), vp()
assert hip.hipMalloc(ctypes.byref(d), sz(rows * pitch)) == 0
assert hip.hipHostMalloc(ctypes.byref(h), sz(rows * w), 0) == 0
streams = [vp() for _ in range(4)]
for s in streams:
    assert hip.hipStreamCreate(ctypes.byref(s)) == 0
D2H = 2


def run(nsplit, contiguous=False):
    best = 1e9
    for rep in range(8):
        hip.hipDeviceSynchronize()
        t0 = time.perf_counter()
        per = (rows + nsplit - 1) // nsplit
        for i in range(nsplit):
            r0, n = i * per, min(per, rows - i * per)
            if contiguous:
                hip.hipMemcpyAsync(vp(h.value + r0 * w), vp(d.value + r0 * w), sz(n * w), D2H, streams[i])
            else:
                hip.hipMemcpy2DAsync(vp(h.value + r0 * w), sz(w), vp(d.value + r0 * pitch), sz(pitch), sz(w), sz(n),
                                     D2H, streams[i])
        for i in range(nsplit):
            hip.hipStreamSynchronize(streams[i])
        best = min(best, time.perf_counter() - t0)
    return best


for ns in (1, 2, 4):
    for c in (False, True):
        t = run(ns, c)
        print(f"streams={ns} {'contiguous' if c else '2-D pitched'}: {t * 1e3:.3f} ms  {rows * w / t / 1e9:.1f} GB/s",
              flush=True)
