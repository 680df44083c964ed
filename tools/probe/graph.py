"""Launch overhead: the same encode steps (B coded pieces of a resident 32
MiB/256 generation per launch) issued one by one on a stream vs replayed from
a captured hipGraph (torch.cuda.CUDAGraph over the library's stream), and an
empty-kernel floor.  Measurement only."""
import ctypes, os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from kodr_amd import device, errors
from kodr_amd._lib import lib

L_ = lib()
k, L, G, STEPS = 256, 131072, 16, 200
rng = np.random.default_rng(0)
torch.cuda.init()
cap = torch.cuda.Stream()
ctx = device.Context(0, stream=cap.cuda_stream)
u8p = ctypes.POINTER(ctypes.c_uint8)
encs = []
for g in range(G):
    data = rng.integers(0, 256, k * L, dtype=np.uint8)
    h = ctypes.c_void_p()
    errors.check(L_.rlnc_encoder_create(ctx.handle, 0, data.ctypes.data_as(u8p), k, L, ctypes.byref(h)))
    encs.append(h)
for B in (1, 8, 32, 256):
    V = rng.integers(0, 256, (64, B, k), dtype=np.uint8)
    dV = ctx.alloc(V.nbytes)
    ctx.h2d(dV, V)
    dO = ctx.alloc(B * L)
    step = lambda i: errors.check(L_.rlnc_encoder_coded_pieces_device(encs[i % G], dV + (i % 64) * B * k, B, dO, L))
    for i in range(20):
        step(i)
    ctx.synchronize()
    e0, e1 = ctx.event(), ctx.event()
    ctx.record(e0)
    for i in range(STEPS):
        step(i)
    ctx.record(e1)
    ctx.synchronize()
    t_stream = device.Context.elapsed_ms(e0, e1) * 1e3 / STEPS
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=cap):
        for i in range(STEPS):
            step(i)
    g.replay()
    torch.cuda.synchronize()
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(cap):
        s0.record()
        g.replay()
        s1.record()
    torch.cuda.synchronize()
    t_graph = s0.elapsed_time(s1) * 1e3 / STEPS
    print(f"B={B:4d} stream {t_stream:8.2f} us/launch   graph {t_graph:8.2f} us/launch", flush=True)
    ctx.free(dV)
    ctx.free(dO)
