"""Timeline of the multi-workgroup elimination (gf_elim_mc_kernel), tuning
build with -DKODR_ELIM_TIMING (KODR_RLNC_LIB, KODR_ELIM_DUMP): per workgroup
of decoder 0, s_memrealtime stamps (10 ns) relative to the earliest entry.
usage: python tools/elim_mc_timing.py [k] [G]"""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from kodr_amd import device as kdev, errors  # noqa: E402
from kodr_amd._lib import lib  # noqa: E402

L_ = lib()
ctx = kdev.Context(0)
rng = np.random.default_rng(1)
k = int(sys.argv[1]) if len(sys.argv) > 1 else 256
G = int(sys.argv[2]) if len(sys.argv) > 2 else 1
n, L = k + 2, 256
pitch = k + L
P = (k + 31) // 32
bufs = []
for g in range(G):
    rows = rng.integers(0, 256, (n, pitch), dtype=np.uint8)
    d = ctx.alloc(rows.nbytes)
    ctx.h2d(d, rows)
    bufs.append(d)
for rep in range(3):
    decs = []
    for g in range(G):
        h = ctypes.c_void_p()
        errors.check(L_.rlnc_decoder_create(ctx.handle, k, ctypes.byref(h)))
        decs.append(h)
    arr = (ctypes.c_void_p * G)(*[x.value for x in decs])
    rp = (ctypes.c_void_p * G)(*bufs)
    cn = (ctypes.c_size_t * G)(*([n] * G))
    cons, sts = (ctypes.c_size_t * G)(), (ctypes.c_int * G)()
    errors.check(L_.rlnc_decoders_add_pieces_gpu(arr, G, rp, cn, pitch, L, cons, sts))
    ctx.synchronize()
    for x in decs:
        L_.rlnc_decoder_destroy(x)
buf = np.fromfile(os.environ["KODR_ELIM_DUMP"], dtype=np.uint8)
hdr, opitch = 1024, (256 if k <= 128 else 512)
ostride = k * opitch
for g in sorted({0, G - 1}):
    st = np.stack([buf[hdr + g * ostride + 32 * q * opitch:][:17 * 8].view(np.uint64).astype(np.int64)
                   for q in range(P)])
    t0 = st[:, 0].min()
    rel = lambda x: (x - t0) / 100.0  # us
    print(f"decoder {g} (k = {k}, G = {G}, {P} workgroups), us from the first entry:")
    for q in range(P):
        grp = " ".join(f"{rel(st[q, 2 + gp]):7.2f}" for gp in range(P))
        own = " ".join(f"{(st[q, 3 + P + j] - st[q, 2 + q - 1 if q else 1]) / 100.0:6.2f}" for j in range(6))
        print(f"  wg {q}: entry {rel(st[q, 0]):6.2f} loaded {rel(st[q, 1]):6.2f} | after groups {grp} | "
              f"end {rel(st[q, 2 + P]):7.2f} | own sub-steps (from the previous group) {own}")
