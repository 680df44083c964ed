"""Recode with the coding-vector columns as the bit-sliced launch's side
product (gf_bs.hip BsSideK, capi.cpp rec_product): one launch writes whole
recoded wire rows r x [C | P] (full/recoder.go:32-40).  Every row against
the oracle's recode (oracle/kodr_oracle.c, a restatement of
full/recoder.go:27-46) with canaries past each row, over the prologue path
(the block's first row, K <= 8 x waves x lane groups) and the remainder
path (larger K, several column blocks, blocks past the column chunks), for
plain and compact recoders and for an output that cannot take the side
product (unaligned pitch: separate vector launch)."""
import ctypes

import numpy as np
import pytest

import oracle
from kodr_amd import _lib, errors

pytestmark = pytest.mark.gpu


def ptr(a):
    return a.ctypes.data_as(_lib._u8p)


@pytest.mark.parametrize("k,L,n,B,mode", [
    (32, 4096 + 48, 40, 12, "plain"),
    (256, 16384, 256, 64, "plain"),
    (256, 16384, 256, 64, "compact"),
    (512, 8192, 512, 32, "plain"),
    (1024, 4096, 64, 16, "plain"),
    (2048, 2048, 24, 9, "compact"),
    (64, 2048, 64, 256, "plain"),
    (48, 6144, 48, 40, "unaligned"),
])
def test_recode_side_product_vs_oracle(gpu_ctx, k, L, n, B, mode):
    rng = np.random.default_rng(k * 7 + L + n + B)
    lib = _lib.lib()
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    V = rng.integers(0, 256, (n, k), dtype=np.uint8)
    flat = np.ascontiguousarray(np.concatenate([V, oracle.encode(P, V)], axis=1))
    clen = k + L
    rh = ctypes.c_void_p()
    errors.check(lib.rlnc_recoder_create(gpu_ctx.handle, ptr(flat), flat.size, n, k, ctypes.byref(rh)))
    errors.check(lib.rlnc_recoder_compact(rh) if mode == "compact" else lib.rlnc_recoder_prepare(rh))
    R = rng.integers(0, 256, (B, n), dtype=np.uint8)
    R[0] = 0
    R[B - 1] = 0
    R[B - 1, n - 1] = 1                # the last held piece itself
    pitch = (clen + 15) // 16 * 16 + (8 if mode == "unaligned" else 16)
    size = B * pitch + 64
    dR, dO = gpu_ctx.alloc(R.nbytes), gpu_ctx.alloc(size)
    try:
        gpu_ctx.h2d(dR, R)
        gpu_ctx.h2d(dO, np.full(size, 0xA5, np.uint8))
        errors.check(lib.rlnc_recoder_coded_pieces_device(rh, dR, B, dO, pitch))
        gpu_ctx.synchronize()
        raw = gpu_ctx.d2h(dO, size)
    finally:
        gpu_ctx.free(dR)
        gpu_ctx.free(dO)
        lib.rlnc_recoder_destroy(rh)
    assert (raw[B * pitch:] == 0xA5).all()
    rows = raw[:B * pitch].reshape(B, pitch)
    assert (rows[:, clen:] == 0xA5).all(), "wrote past the recoded piece"
    exp = oracle.recode(flat, k, R)
    bad = np.nonzero((rows[:, :clen] != exp).any(axis=1))[0]
    assert bad.size == 0, (bad[:8], "vector columns" if (rows[bad[0], :k] != exp[bad[0], :k]).any() else "piece")
    assert not rows[0, :clen].any() and np.array_equal(rows[B - 1, :clen], flat[n - 1])
