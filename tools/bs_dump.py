"""Bring-up: run gf_bs_kernel in MODE 9 (tune build) -- prologue and the
first row's target loads, then s[60:89] and M0 dumped, no jump -- and check
the targets against the generator's body layout.  Measurement/debug only."""
import ctypes, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "kodr_amd", "csrc"))
import gen_bs_bodies as gen
from kodr_amd import device, errors
from kodr_amd._lib import lib

L_ = lib()
ctx = device.Context(0)
os.environ["KODR_BS_MODE"] = "9"
M, K, n = 8, 2, 2048
rng = np.random.default_rng(5)
A = rng.integers(0, 256, (M, K), dtype=np.uint8)
dA, dX, dY = ctx.alloc(A.nbytes), ctx.alloc(K * n), ctx.alloc(M * n)
ctx.h2d(dA, A)
ctx.h2d(dX, np.zeros(K * n, np.uint8))
ctx.h2d(dY, np.zeros(M * n, np.uint8))
errors.check(L_.rlnc_gf_matmul_bs_device(ctx.handle, dA, K, M, K, dX, n, dY, n, n))
ctx.synchronize()
d = ctx.d2h(dY, 4 * 128).view(np.uint32)
print("pl", hex(d[64]), "prog", [hex(x) for x in d[65:81]])
print("tgt_l", [hex(x) for x in d[81:89]], "tgt", [hex(x) for x in d[89:93]], "ne", d[93], "c0", d[94])
names = [f"s{i}" for i in range(gen.T0, gen.CNT + 1)] + ["m0"]
for nm, v in zip(names, d):
    print(f"{nm:4s} {v:#010x}")
offs, _ = gen.body_offsets()
t = [int(d[2 * m]) for m in range(4)] + [int(d[10 + 2 * m]) for m in range(4)]
print("A[:,0] =", list(A[:, 0]))
base = [t[m] - offs[(m & 3) * 256 + int(A[m, 0])] for m in range(8)]
print("implied body base lo per m:", [hex(b & 0xFFFFFFFF) for b in base])
print("thi:", hex(int(d[1])))
