"""Compact residency (rlnc_encoder_compact / rlnc_recoder_compact): only the
bit-sliced copy of a generation stays in HBM.  Every product then runs on the
bit-sliced kernel, for any batch size; systematic pieces are converted back
from the bit-sliced rows.  Checked against the oracle: full and systematic
encoders (host and device outputs, wire rows), grouped calls mixing compact
and plain encoders, the recoder, and the 32 MiB/256 headline shape."""
import ctypes

import numpy as np
import pytest

import oracle
from kodr_amd import _lib, errors

pytestmark = pytest.mark.gpu
U8P = _lib._u8p
FULL, SYSTEMATIC = 0, 1


def _encoder(ctx, kind, P):
    k, L = P.shape
    h = ctypes.c_void_p()
    flat = np.ascontiguousarray(P)
    errors.check(_lib.lib().rlnc_encoder_create(ctx.handle, kind, flat.ctypes.data_as(U8P), k, L, ctypes.byref(h)))
    return h


def _device_encode(ctx, h, V, L):
    B, k = V.shape
    pitch = (L + 15) // 16 * 16
    dV, dY = ctx.alloc(V.size), ctx.alloc(B * pitch)
    ctx.h2d(dV, np.ascontiguousarray(V))
    errors.check(_lib.lib().rlnc_encoder_coded_pieces_device(h, dV, B, dY, pitch))
    ctx.synchronize()
    Y = ctx.d2h(dY, B * pitch).reshape(B, pitch)[:, :L]
    ctx.free(dV)
    ctx.free(dY)
    return Y


@pytest.mark.parametrize("k,L", [(64, 5000), (9, 4096), (200, 1 << 16)])
def test_compact_full_encoder_matches_oracle(gpu_ctx, k, L):
    rng = np.random.default_rng(k + L)
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    h = _encoder(gpu_ctx, FULL, P)
    lib = _lib.lib()
    assert lib.rlnc_encoder_device_pieces(h, None) is not None
    errors.check(lib.rlnc_encoder_compact(h))
    errors.check(lib.rlnc_encoder_compact(h))  # idempotent
    assert lib.rlnc_encoder_device_pieces(h, None) is None
    for B in (1, 3, 8, 9, 32):
        V = rng.integers(0, 256, (B, k), dtype=np.uint8)
        assert np.array_equal(_device_encode(gpu_ctx, h, V, L), oracle.encode(P, V)), B
    # host vectors and output (wire rows)
    B = 5
    V = rng.integers(0, 256, (B, k), dtype=np.uint8)
    out = np.zeros((B, k + L), np.uint8)
    errors.check(lib.rlnc_encoder_coded_pieces(h, np.ascontiguousarray(V).ctypes.data_as(U8P), B,
                                               out.ctypes.data_as(U8P)))
    assert np.array_equal(out[:, :k], V) and np.array_equal(out[:, k:], oracle.encode(P, V))
    lib.rlnc_encoder_destroy(h)


def test_compact_systematic_encoder(gpu_ctx):
    """The first k pieces are e_i ++ P_i (systematic/encoder.go:83-96), read
    back from the bit-sliced rows; host calls crossing the k boundary, and
    device wire rows."""
    rng = np.random.default_rng(3)
    k, L = 40, 3000
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    lib = _lib.lib()
    h = _encoder(gpu_ctx, SYSTEMATIC, P)
    errors.check(lib.rlnc_encoder_compact(h))
    got = []
    for count in (7, 30, 13):  # 7 + 30 + 3 systematic, then 10 coded
        vecs = np.zeros((count, k), np.uint8)
        out = np.zeros((count, k + L), np.uint8)
        vecs[:] = rng.integers(0, 256, (count, k), dtype=np.uint8)
        V = vecs.copy()
        errors.check(lib.rlnc_encoder_coded_pieces(h, vecs.ctypes.data_as(U8P), count, out.ctypes.data_as(U8P)))
        got.append((V, vecs.copy(), out))
    n = 0
    for V, vecs, out in got:
        for r in range(out.shape[0]):
            if n < k:
                e = np.zeros(k, np.uint8)
                e[n] = 1
                assert np.array_equal(out[r, :k], e) and np.array_equal(out[r, k:], P[n]), n
            else:
                assert np.array_equal(out[r, :k], V[r])
                assert np.array_equal(out[r, k:], oracle.encode(P, V[r:r + 1])[0]), n
            n += 1
    lib.rlnc_encoder_destroy(h)
    # device wire rows: k systematic + 6 coded, vectors drawn on the device
    h = _encoder(gpu_ctx, SYSTEMATIC, P)
    errors.check(lib.rlnc_encoder_compact(h))
    n, W = k + 6, (k + L + 15) // 16 * 16
    dW = gpu_ctx.alloc(n * W)
    errors.check(lib.rlnc_encoder_coded_wire_device(h, n, dW, W))
    gpu_ctx.synchronize()
    wire = gpu_ctx.d2h(dW, n * W).reshape(n, W)
    assert np.array_equal(wire[:k, :k], np.eye(k, dtype=np.uint8))
    assert np.array_equal(wire[:k, k:k + L], P)
    assert np.array_equal(wire[k:, k:k + L], oracle.encode(P, wire[k:, :k]))
    gpu_ctx.free(dW)
    lib.rlnc_encoder_destroy(h)


def test_compact_group_call_mixes_layouts(gpu_ctx):
    rng = np.random.default_rng(8)
    k, L, G, B = 32, 8192, 5, 2
    Ps = [rng.integers(0, 256, (k, L), dtype=np.uint8) for _ in range(G)]
    lib = _lib.lib()
    hs = [_encoder(gpu_ctx, FULL, P) for P in Ps]
    for g in (1, 3):
        errors.check(lib.rlnc_encoder_compact(hs[g]))
    V = rng.integers(0, 256, (G, B, k), dtype=np.uint8)
    dV, dY = gpu_ctx.alloc(V.size), gpu_ctx.alloc(G * B * L)
    gpu_ctx.h2d(dV, np.ascontiguousarray(V))
    arr = (ctypes.c_void_p * G)(*[h.value for h in hs])
    errors.check(lib.rlnc_encoder_group_coded_pieces_device(arr, G, dV, B, dY, L))
    gpu_ctx.synchronize()
    Y = gpu_ctx.d2h(dY, G * B * L).reshape(G, B, L)
    for g in range(G):
        assert np.array_equal(Y[g], oracle.encode(Ps[g], V[g])), g
    gpu_ctx.free(dV)
    gpu_ctx.free(dY)
    for h in hs:
        lib.rlnc_encoder_destroy(h)


def test_compact_recoder(gpu_ctx):
    rng = np.random.default_rng(12)
    k, L, n = 24, 6000, 30
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    C = rng.integers(0, 256, (n, k), dtype=np.uint8)
    flat = np.ascontiguousarray(np.concatenate([C, oracle.encode(P, C)], axis=1))
    lib = _lib.lib()
    h = ctypes.c_void_p()
    errors.check(lib.rlnc_recoder_create(gpu_ctx.handle, flat.ctypes.data_as(U8P), flat.size, n, k,
                                         ctypes.byref(h)))
    errors.check(lib.rlnc_recoder_compact(h))
    for B in (1, 20):
        r = rng.integers(0, 256, (B, n), dtype=np.uint8)
        out = np.zeros((B, k + L), np.uint8)
        errors.check(lib.rlnc_recoder_coded_pieces(h, np.ascontiguousarray(r).ctypes.data_as(U8P), B,
                                                   out.ctypes.data_as(U8P)))
        assert np.array_equal(out, oracle.matmul(r, flat)[1]), B
    lib.rlnc_recoder_destroy(h)


def test_compact_headline_shape(gpu_ctx):
    """32 MiB / 256 (BASELINE config 2): B = 1 and the B = 32 headline batch
    from a compact encoder, byte for byte."""
    rng = np.random.default_rng(32)
    k, L = 256, 131072
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    h = _encoder(gpu_ctx, FULL, P)
    errors.check(_lib.lib().rlnc_encoder_compact(h))
    for B in (1, 32):
        V = rng.integers(0, 256, (B, k), dtype=np.uint8)
        assert np.array_equal(_device_encode(gpu_ctx, h, V, L), oracle.encode(P, V)), B
    _lib.lib().rlnc_encoder_destroy(h)
