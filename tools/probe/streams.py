"""Concurrent encode steps on S streams (one rlnc_ctx per stream, each with its
own resident generations): per-step time vs S.  Measurement only."""
import ctypes, os, sys, time
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from kodr_amd import device, errors
from kodr_amd._lib import lib

L_ = lib()
k, L, G, STEPS = 256, 131072, 16, 200
rng = np.random.default_rng(0)
u8p = ctypes.POINTER(ctypes.c_uint8)
for B in (1, 8, 32, 64, 256):
    for S in (1, 2, 3, 4):
        ctxs = [device.Context(0) for _ in range(S)]
        encs, bufs = [], []
        for s in range(S):
            es = []
            for g in range(G // S if S > 1 else G):
                data = rng.integers(0, 256, k * L, dtype=np.uint8)
                h = ctypes.c_void_p()
                errors.check(L_.rlnc_encoder_create(ctxs[s].handle, 0, data.ctypes.data_as(u8p), k, L, ctypes.byref(h)))
                es.append(h)
            V = rng.integers(0, 256, (64, B, k), dtype=np.uint8)
            dV = ctxs[s].alloc(V.nbytes)
            ctxs[s].h2d(dV, V)
            dO = ctxs[s].alloc(B * L)
            encs.append(es)
            bufs.append((dV, dO))

        def step(i):
            s = i % S
            es, (dV, dO) = encs[s], bufs[s]
            errors.check(L_.rlnc_encoder_coded_pieces_device(es[(i // S) % len(es)], dV + ((i // S) % 64) * B * k, B, dO, L))
        for i in range(20):
            step(i)
        for c in ctxs:
            c.synchronize()
        t0 = time.perf_counter()
        for i in range(STEPS):
            step(i)
        for c in ctxs:
            c.synchronize()
        dt = (time.perf_counter() - t0) / STEPS
        print(f"B={B:4d} streams={S}: {dt * 1e6:8.2f} us/step  coded {B * (k * L + k + L) / dt / 1e6 / 1e6:7.2f} e6 MB/s", flush=True)
        for s in range(S):
            for h in encs[s]:
                L_.rlnc_encoder_destroy(h)
            ctxs[s].free(bufs[s][0])
            ctxs[s].free(bufs[s][1])
            ctxs[s].close()
