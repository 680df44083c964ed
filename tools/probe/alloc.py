"""Cost of hipMalloc/hipMemset/hipFree at decoder-buffer sizes (32-35 MiB) on the
box.  Measurement only."""
import ctypes, time
hip = ctypes.CDLL("libamdhip64.so")
hip.hipSetDevice(0)
p = ctypes.c_void_p()
for size in (1 << 20, 34 << 20, 256 << 20):
    ts = []
    for i in range(6):
        t0 = time.perf_counter()
        hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(size))
        t1 = time.perf_counter()
        hip.hipMemset(p, 0, ctypes.c_size_t(size))
        hip.hipDeviceSynchronize()
        t2 = time.perf_counter()
        hip.hipFree(p)
        t3 = time.perf_counter()
        ts.append((t1 - t0, t2 - t1, t3 - t2))
    ts = ts[1:]
    f = lambda j: sum(t[j] for t in ts) / len(ts) * 1e6
    print(f"{size >> 20:4d} MiB: hipMalloc {f(0):8.1f} us  memset+sync {f(1):8.1f} us  hipFree {f(2):8.1f} us", flush=True)
