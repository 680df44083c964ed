"""Timeline of gf_elim_mc4_kernel, tuning build with -DKODR_ELIM_TIMING
(KODR_RLNC_LIB, KODR_ELIM_DUMP, KODR_ELIM_MC=4): s_memrealtime stamps (10 ns)
of decoder 0 relative to the earliest entry; the stamps overwrite T, so the
results come from kodr's route on the host.
usage: python tools/elim_mc4_timing.py [k]"""
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
n, L = k, 256
pitch = k + L
NP = (k + 15) // 16
RPW = int(os.environ.get("KODR_MC4_RPW", "2"))
NRW = NP * 16 // (4 * RPW)
rows = rng.integers(0, 256, (n, pitch), dtype=np.uint8)
dbuf = ctx.alloc(rows.nbytes)
ctx.h2d(dbuf, rows)
for rep in range(3):
    h = ctypes.c_void_p()
    errors.check(L_.rlnc_decoder_create(ctx.handle, k, ctypes.byref(h)))
    c = ctypes.c_size_t()
    L_.rlnc_decoder_add_pieces_gpu(h, ctypes.c_void_p(dbuf), n, pitch, L, ctypes.byref(c))
    ctx.synchronize()
    L_.rlnc_decoder_destroy(h)
buf = np.fromfile(os.environ["KODR_ELIM_DUMP"], dtype=np.uint8)
hdr = 1024
st = np.stack([buf[hdr + x * 1024:][:128 * 8].view(np.uint64).astype(np.int64) for x in range(NRW + 1)])
t0 = st[:, 96].min()
rel = lambda v: (v - t0) / 100.0  # us
ch = st[NRW]
print(f"k = {k}, {NRW} row workgroups + the chain; us from the first entry")
print(f"chain: entry {rel(ch[96]):6.2f} tables {rel(ch[97]):6.2f}")
for p in range(NP):
    print(f"  panel {p:2d}: staged {rel(ch[48 + p]):7.2f} chain has it {rel(ch[p]):7.2f} updated {rel(ch[16 + p]):7.2f} "
          f"S out {rel(ch[32 + p]):7.2f} | update {rel(ch[16 + p]) - rel(ch[p]):5.2f} gj {rel(ch[32 + p]) - rel(ch[16 + p]):5.2f}")
for r in range(NRW):
    x = st[r]
    line = " ".join(f"{rel(x[j]):6.2f}/{rel(x[16 + j]):6.2f}" for j in range(NP))
    print(f"row wg {r:2d}: entry {rel(x[96]):5.2f} tables {rel(x[97]):5.2f} | staged/applied: {line}")
ends = [rel(ch[32 + p]) for p in range(NP)]
print("S_p out:", " ".join(f"{e:6.2f}" for e in ends))
print("per panel:", " ".join(f"{b - a:5.2f}" for a, b in zip([0.0] + ends[:-1], ends)))
