"""CPU model of the GPU elimination's attempts (gf_elim.hip, mc2 / mc4), for
the tests: block Gauss-Jordan over 16-column panels with pivots searched only
inside each panel's 16 rows, so an attempt fails exactly when a leading
16j x 16j block of its row order is singular; the attempts take the rows
rotated by mc_rot (0, k/2, k/4, 3k/4) and stop early on an abort (a singular
last panel -- C itself singular -- or a panel block with a zero column).
Also the device vector stream (fill_vectors_kernel's splitmix64) and GF(2^8)
helpers (poly 0x11D, gf256.go:15-44).  Test infrastructure only."""
import numpy as np

EXP = np.zeros(512, np.int32)
LOG = np.zeros(256, np.int32)
_x = 1
for _i in range(255):
    EXP[_i] = _x
    LOG[_x] = _i
    _x <<= 1
    if _x & 0x100:
        _x ^= 0x11D
EXP[255:510] = EXP[:255]

ATTEMPTS = 4


def mul(a, b):
    a = np.asarray(a, np.int32)
    b = np.asarray(b, np.int32)
    r = EXP[(LOG[a] + LOG[b]) % 255]
    return np.where((a == 0) | (b == 0), 0, r)


def inv(a):
    return EXP[(255 - LOG[a]) % 255]


def rot(att, k):
    """gf_elim.hip mc_rot."""
    return (0, k // 2, k // 4, (3 * k) // 4)[att]


def rotate_rows(C, s):
    """row i of the attempt's matrix is row (i + s) mod k of C."""
    k = C.shape[0]
    return C[[(i + s) % k for i in range(k)]]


def attempt(M, w=16):
    """One attempt on M (k x k): 'ok', 'retry' (a singular panel block) or
    'abort' (the last panel's block singular, or a block column all zero)."""
    M = M.astype(np.int32).copy()
    k = M.shape[0]
    last = (k - 1) // w
    for c in range(k):
        panel = c // w
        if c % w == 0:
            hi = min(k, (panel + 1) * w)
            blk = M[panel * w:hi, panel * w:hi]
            zero_col = bool((blk == 0).all(axis=0).any())
        rows = [r for r in range(c, min(k, (panel + 1) * w)) if M[r, c]]
        if not rows:
            return "abort" if panel == last or zero_col else "retry"
        r = rows[0]
        M[[c, r]] = M[[r, c]]
        M[c] = mul(M[c], inv(M[c, c]))
        f = M[:, c].copy()
        f[c] = 0
        nz = np.nonzero(f)[0]
        if len(nz):
            M[nz] ^= mul(f[nz, None], M[c][None, :])
    return "ok"


def expected_attempt(C):
    """The attempt (0 .. 3) whose rotation the GPU elimination succeeds with,
    or None when the launch fails (the host then runs kodr's route)."""
    k = C.shape[0]
    for a in range(ATTEMPTS):
        r = attempt(rotate_rows(C, rot(a, k)))
        if r == "ok":
            return a
        if r == "abort":
            return None
    return None


def splitmix(z):
    z = (z + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return z ^ (z >> 31)


def device_vectors(seed, rows, k, row0=0):
    """rlnc_encoder_coded_wire_device's vectors for an encoder seeded with
    `seed` (fill_vectors_kernel: low byte of splitmix64(seed + (row0 + r) << 32 + j))."""
    return np.array([[splitmix(seed + ((row0 + r) << 32) + j) & 0xFF for j in range(k)] for r in range(rows)],
                    np.uint8)


def gf_inverse(C):
    """C^-1 over GF(2^8) by Gauss-Jordan with full pivot search (None if singular)."""
    k = C.shape[0]
    A = np.concatenate([C.astype(np.int32), np.eye(k, dtype=np.int32)], axis=1)
    for c in range(k):
        rows = np.nonzero(A[c:, c])[0]
        if not len(rows):
            return None
        r = c + rows[0]
        A[[c, r]] = A[[r, c]]
        A[c] = mul(A[c], inv(A[c, c]))
        f = A[:, c].copy()
        f[c] = 0
        nz = np.nonzero(f)[0]
        if len(nz):
            A[nz] ^= mul(f[nz, None], A[c][None, :])
    return A[:, k:].astype(np.uint8)


def unrotate_columns(Tp, s):
    """T = T' Pi for (Pi C)_i = C_{(i + s) mod k}: T[:, j] = T'[:, (j - s) mod k]
    (gf_elim.hip mc_unrotate)."""
    k = Tp.shape[1]
    return Tp[:, [(j - s) % k for j in range(k)]]
