"""The GPU elimination's pivot rule on the CPU: Gauss-Jordan with pivots
searched only inside each 16-row panel (gf_elim_mc2/mc4), which fails exactly
when a leading 16j x 16j block of C is singular.  Reports the first failing
panel for device-drawn vectors (fill_vectors_kernel's splitmix64 stream,
rlnc_encoder_seed = seed, rows 0 .. k - 1) or the failure count over random
matrices.  usage: python tools/panel_sim.py seed S [S ...] | random N"""
import numpy as np, sys
# GF(256) poly 0x11D
exp = np.zeros(512, np.int32); log = np.zeros(256, np.int32)
x = 1
for i in range(255):
    exp[i] = x; log[x] = i
    x <<= 1
    if x & 0x100: x ^= 0x11D
exp[255:510] = exp[:255]
def mul(a, b):
    a = np.asarray(a, np.int32); b = np.asarray(b, np.int32)
    r = exp[(log[a] + log[b]) % 255]
    return np.where((a == 0) | (b == 0), 0, r)
def inv(a): return exp[(255 - log[a]) % 255]
def first_fail(M, w=16):
    """leading principal minors of size w, 2w, ...: the first singular one (panel index) or -1"""
    M = M.copy().astype(np.int32); k = M.shape[0]
    for c in range(k):
        if c % w == 0: panel = c // w
        # pivot within the panel's rows [panel*w, panel*w + w) at or below row c
        rows = [r for r in range(c, (panel + 1) * w) if M[r, c]]
        if not rows: return panel
        r = rows[0]
        M[[c, r]] = M[[r, c]]
        M[c] = mul(M[c], inv(M[c, c]))
        f = M[:, c].copy(); f[c] = 0
        nz = np.nonzero(f)[0]
        if len(nz): M[nz] ^= mul(f[nz, None], M[c][None, :])
    return -1
def splitmix(z):
    z = (z + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return z ^ (z >> 31)
k = 256
if sys.argv[1] == "seed":
    for seed in map(int, sys.argv[2:]):
        M = np.array([[splitmix(seed + (r << 32) + j) & 0xff for j in range(k)] for r in range(k)])
        print("seed", seed, "first singular panel", first_fail(M), flush=True)
else:
    rng = np.random.default_rng(1); n = int(sys.argv[2]); f = 0
    for t in range(n):
        f += first_fail(rng.integers(0, 256, (k, k))) >= 0
    print("random", n, "fail", f)
