"""rlnc_decoder_destroy without a host wait (capi_decoder.cpp; pool.hpp defer_free):
a decoder destroyed right after its GetPieces, with the product still
queued, gives its buffers back ordered behind it by one event.  The next
decoder on the same stream reuses them in stream order, and a decoder on
another context's stream waits for the event, so the first product is never
overwritten early.  Decoded bytes against the original pieces (the oracle's
encode makes the coded rows: full/encoder.go:61-71)."""
import ctypes

import numpy as np
import pytest

import oracle
from kodr_amd import _lib, device, errors

pytestmark = pytest.mark.gpu


def _rows(ctx, rng, k, L):
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    V = rng.integers(0, 256, (k + 2, k), dtype=np.uint8)
    C = oracle.encode(P, V)
    pitch = (k + L + 15) // 16 * 16
    rows = np.zeros((k + 2, pitch), np.uint8)
    rows[:, :k] = V
    rows[:, k:k + L] = C
    d = ctx.alloc(rows.nbytes)
    ctx.h2d(d, rows)
    return P, d, pitch


def _decode_to(ctx, k, L, d, pitch, dout):
    lib = _lib.lib()
    h = ctypes.c_void_p()
    errors.check(lib.rlnc_decoder_create(ctx.handle, k, ctypes.byref(h)))
    c = ctypes.c_size_t()
    st = lib.rlnc_decoder_add_pieces(h, ctypes.c_void_p(d), k + 2, pitch, L, 1, ctypes.byref(c))
    assert st in (0, 3) and c.value == k
    errors.check(lib.rlnc_decoder_get_pieces_device(h, ctypes.c_void_p(dout), L))
    return h


@pytest.mark.parametrize("k,L", [(64, 1 << 16), (256, 1 << 15)])
def test_destroy_behind_pending_work(gpu_ctx, k, L):
    lib = _lib.lib()
    rng = np.random.default_rng(k)
    other = device.Context(0)  # its own stream
    sets = [_rows(gpu_ctx, rng, k, L) for _ in range(3)]
    outs = [gpu_ctx.alloc(k * L) for _ in range(3)]
    gpu_ctx.synchronize()
    for rep in range(3):
        h0 = _decode_to(gpu_ctx, k, L, sets[0][1], sets[0][2], outs[0])
        lib.rlnc_decoder_destroy(h0)               # GetPieces still queued
        h1 = _decode_to(gpu_ctx, k, L, sets[1][1], sets[1][2], outs[1])   # same stream: reuses in order
        lib.rlnc_decoder_destroy(h1)
        h2 = _decode_to(other, k, L, sets[2][1], sets[2][2], outs[2])     # another stream: waits on the event
        lib.rlnc_decoder_destroy(h2)
        other.synchronize()
        gpu_ctx.synchronize()
        for i in range(3):
            got = gpu_ctx.d2h(outs[i], k * L).reshape(k, L)
            assert np.array_equal(got, sets[i][0]), (rep, i)
    for _, d, _ in sets:
        gpu_ctx.free(d)
    for o in outs:
        gpu_ctx.free(o)
