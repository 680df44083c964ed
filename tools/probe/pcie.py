"""PCIe copy rates on the box: contiguous and 2-D (wire-layout) D2H/H2D
between HBM and pinned host memory, 32 MiB-class transfers.  Measurement only."""
import ctypes
import time

import torch

hip = ctypes.CDLL("libamdhip64.so")
k, L = 256, 131072
clen = k + L
n = 256
dev = torch.empty(n * clen, dtype=torch.uint8, device="cuda")
host = torch.empty(n * clen, dtype=torch.uint8).pin_memory()
s = torch.cuda.current_stream()
st = ctypes.c_void_p(s.cuda_stream)
D2H, H2D = 2, 1


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def cont(kind, nbytes):
    def f():
        if kind == D2H:
            hip.hipMemcpyAsync(ctypes.c_void_p(host.data_ptr()), ctypes.c_void_p(dev.data_ptr()),
                               ctypes.c_size_t(nbytes), D2H, st)
        else:
            hip.hipMemcpyAsync(ctypes.c_void_p(dev.data_ptr()), ctypes.c_void_p(host.data_ptr()),
                               ctypes.c_size_t(nbytes), H2D, st)
    return f


def two_d(kind, rows, width, dpitch, spitch):
    def f():
        if kind == D2H:
            hip.hipMemcpy2DAsync(ctypes.c_void_p(host.data_ptr()), ctypes.c_size_t(dpitch),
                                 ctypes.c_void_p(dev.data_ptr()), ctypes.c_size_t(spitch),
                                 ctypes.c_size_t(width), ctypes.c_size_t(rows), D2H, st)
        else:
            hip.hipMemcpy2DAsync(ctypes.c_void_p(dev.data_ptr()), ctypes.c_size_t(dpitch),
                                 ctypes.c_void_p(host.data_ptr()), ctypes.c_size_t(spitch),
                                 ctypes.c_size_t(width), ctypes.c_size_t(rows), H2D, st)
    return f


for name, f, nb in [
        ("D2H contiguous 32.1 MiB", cont(D2H, n * clen), n * clen),
        ("H2D contiguous 32.1 MiB", cont(H2D, n * clen), n * clen),
        ("D2H 2D 256 x 128 KiB, dst pitch k+L", two_d(D2H, n, L, clen, L), n * L),
        ("D2H 2D 256 x 128 KiB, both pitch k+L", two_d(D2H, n, L, clen, clen), n * L),
        ("H2D 2D 256 x 128 KiB, src pitch k+L", two_d(H2D, n, L, L, clen), n * L),
        ("D2H contiguous 4 MiB", cont(D2H, 4 << 20), 4 << 20),
        ("D2H contiguous 1 MiB", cont(D2H, 1 << 20), 1 << 20)]:
    t = timeit(f)
    print(f"{name:40s} {t * 1e3:7.3f} ms  {nb / t / 1e9:6.1f} GB/s", flush=True)
