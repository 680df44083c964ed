"""Host-path timing: k+2 coded pieces of a 32 MiB/256 generation into (registered,
REG=1) host memory in calls of 16/64/258 pieces, then a batched AddPiece from
those rows and GetPieces back to host.  Measurement only."""
import ctypes, os, sys, time
import numpy as np
sys.path.insert(0, "/root/repo")
from kodr_amd import device, errors
from kodr_amd._lib import lib
L_ = lib(); ctx = device.Context(0)
k, L = 256, 131072; n = k + 2
u8p = ctypes.POINTER(ctypes.c_uint8)
def pa(nb):
    raw = np.empty(nb + 4096, np.uint8); off = (-raw.ctypes.data) % 4096; return raw[off:off + nb]
rng = np.random.default_rng(0)
data = rng.integers(0, 256, k * L, dtype=np.uint8)
V = pa(n * k).reshape(n, k); V[:] = rng.integers(0, 256, (n, k), dtype=np.uint8)
wire = pa(n * (k + L)).reshape(n, k + L)
reg = os.environ.get("REG", "1") == "1"
if reg:
    ctx.register(V); ctx.register(wire)
eh = ctypes.c_void_p()
errors.check(L_.rlnc_encoder_create_with_piece_count(ctx.handle, 0, data.ctypes.data_as(u8p), data.size, k, ctypes.byref(eh)))
for cnt in (16, 64, 258):
    for rep in range(3):
        t0 = time.perf_counter()
        for i in range(0, n, cnt):
            b = min(cnt, n - i)
            errors.check(L_.rlnc_encoder_coded_pieces(eh, V[i:i+b].ctypes.data_as(u8p), b, wire[i:i+b].ctypes.data_as(u8p)))
        t1 = time.perf_counter()
    print(f"REG={int(reg)} encode in calls of {cnt:3d}: {(t1-t0)*1e3:7.3f} ms", flush=True)
outp = pa(k * L)
if reg:
    ctx.register(outp)
for rep in range(3):
    dh = ctypes.c_void_p()
    errors.check(L_.rlnc_decoder_create(ctx.handle, k, ctypes.byref(dh)))
    consumed = ctypes.c_size_t()
    t0 = time.perf_counter()
    st = L_.rlnc_decoder_add_pieces(dh, wire.ctypes.data_as(u8p), n, k + L, L, 0, ctypes.byref(consumed))
    t1 = time.perf_counter()
    errors.check(L_.rlnc_decoder_get_pieces(dh, outp.ctypes.data_as(u8p)))
    t2 = time.perf_counter()
    L_.rlnc_decoder_destroy(dh)
print(f"REG={int(reg)} decode add {(t1-t0)*1e3:.3f} ms get {(t2-t1)*1e3:.3f} ms ok={np.array_equal(outp, data)}", flush=True)
