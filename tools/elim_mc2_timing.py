"""Timeline of gf_elim_mc2_kernel, tuning build with -DKODR_ELIM_TIMING
(KODR_RLNC_LIB, KODR_ELIM_DUMP): per workgroup of decoder 0, s_memrealtime
stamps (10 ns) relative to the earliest entry; the stamps overwrite the T
rows, so the results come from kodr's route on the host.
usage: python tools/elim_mc2_timing.py [k] [G]"""
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
n, L = k, 256
pitch = k + L
P = (k + 31) // 32
NP = 2 * P
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
hdr = 1024
for g in sorted({0, G - 1}):
    st = np.stack([buf[hdr + g * k * k + q * 1024:][:128 * 8].view(np.uint64).astype(np.int64) for q in range(P)])
    t0 = st[:, 80].min()
    rel = lambda x: (x - t0) / 100.0  # us
    print(f"decoder {g} (k = {k}, G = {G}, {P} workgroups), us from the first entry:")
    for q in range(P):
        print(f"  wg {q}: entry {rel(st[q, 80]):6.2f} loaded {rel(st[q, 81]):6.2f} last apply {rel(st[q, 82]):7.2f} "
              f"out {rel(st[q, 83]):7.2f}")
        for p in range(NP):
            own = "own" if p >> 1 == q else "   "
            c = st[q, 4 * p:4 * p + 4]
            print(f"    panel {p:2d} {own}: start {rel(c[0]):7.2f} ready {rel(c[1]):7.2f} mid {rel(c[2]):7.2f} "
                  f"end {rel(c[3]):7.2f} | rows wake {rel(st[q, 96 + p]):7.2f} F {rel(st[q, 112 + p - 1]) if p else 0.0:7.2f} "
                  f"iter done {rel(st[q, 64 + p]):7.2f}")
    # the critical path: each panel's S out (owner's end) after the previous
    ends = [rel(st[p >> 1, 4 * p + 3]) for p in range(NP)]
    print("  S_p out:", " ".join(f"{e:6.2f}" for e in ends))
    print("  per panel:", " ".join(f"{b - a:5.2f}" for a, b in zip([0.0] + ends[:-1], ends)))
