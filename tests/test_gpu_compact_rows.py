"""Compact received rows (capi_decoder.cpp dec_batch_pre, dec_uncompact): a batched
AddPiece of device rows writes only their bit-sliced twin; the plain bytes
are rebuilt from it when a plain-row path needs them (the v_perm kernel of a
few-row product, a growing receive buffer) and systematic rows are gathered
from the twin un-sliced on the fly.  Every path against the oracle's literal
decoder (decoder_state.go:15-261) and the original pieces: the counters, the
coefficients, pieces decoded before full rank and GetPieces."""
import ctypes

import numpy as np
import pytest

import oracle
from kodr_amd import _lib, errors

pytestmark = pytest.mark.gpu
U8P = _lib._u8p


def _dev_rows(ctx, V, C):
    n, k = V.shape
    L = C.shape[1]
    pitch = (k + L + 15) // 16 * 16
    rows = np.zeros((n, pitch), np.uint8)
    rows[:, :k] = V
    rows[:, k:k + L] = C
    d = ctx.alloc(rows.nbytes)
    ctx.h2d(d, rows)
    return d, pitch


def _state_eq(h, ref, k):
    lib = _lib.lib()
    assert (lib.rlnc_decoder_useful(h), lib.rlnc_decoder_received(h), lib.rlnc_decoder_required(h),
            bool(lib.rlnc_decoder_is_decoded(h))) == (ref.useful(), ref.received(), ref.required(),
                                                       ref.is_decoded())
    r = lib.rlnc_decoder_useful(h)
    co = np.empty((r, k), np.uint8)
    errors.check(lib.rlnc_decoder_coefficients(h, co.ctypes.data_as(U8P)))
    assert np.array_equal(co, ref.coeffs())


def _decoded_piece(h, j, L):
    out = np.empty(L, np.uint8)
    st = _lib.lib().rlnc_decoder_get_decoded(h, j, ctypes.c_void_p(out.ctypes.data), 0)
    return st, out


@pytest.mark.parametrize("k,L", [(64, 4096), (128, 8192 + 32)])
def test_compact_rows_every_plain_path(gpu_ctx, k, L):
    lib = _lib.lib()
    rng = np.random.default_rng(k + L)
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    # a systematic-order stream with losses, then a low-rank stretch (kept
    # dependent: received grows past the first receive buffer), then coded rows
    sys_rows = [i for i in range(k) if i % 7 != 3]
    V1 = np.eye(k, dtype=np.uint8)[sys_rows[: k // 2]]
    B = rng.integers(0, 256, (3, k), dtype=np.uint8)
    low = oracle.matmul(rng.integers(0, 256, (24, 3), dtype=np.uint8), B)[1]
    V2 = np.eye(k, dtype=np.uint8)[sys_rows[k // 2:]]
    V3 = rng.integers(0, 256, (k, k), dtype=np.uint8)
    batches = [V1[:16], V1[16:], low, V2, V3]
    ref = oracle.Decoder(k)
    h = ctypes.c_void_p()
    errors.check(lib.rlnc_decoder_create(gpu_ctx.handle, k, ctypes.byref(h)))
    bufs = []
    for bi, V in enumerate(batches):
        C = oracle.encode(P, V)
        d, pitch = _dev_rows(gpu_ctx, V, C)
        bufs.append(d)
        c = ctypes.c_size_t()
        st = lib.rlnc_decoder_add_pieces(h, ctypes.c_void_p(d), V.shape[0], pitch, L, 1, ctypes.byref(c))
        n_ok = 0
        for i in range(V.shape[0]):
            if ref.add(V[i], C[i]) != 0:
                break
            n_ok += 1
        assert c.value == n_ok and st in (0, 3)
        _state_eq(h, ref, k)
        if bi == 1:
            # systematic pieces decoded before full rank: gathered from the twin
            for j in sys_rows[:20:3]:
                s, out = _decoded_piece(h, j, L)
                assert s == 0 and np.array_equal(out, P[j]), j
        if bi == 2:
            # a single plain AddPiece between compact batches: 5 e_0 + 9 e_1 +
            # 7 e_3 with pieces 0 and 1 held and 3 lost, so piece 3 decodes
            # through a non-unit row of T: the few-row (plain-row) product
            v = np.zeros(k, np.uint8)
            v[0], v[1], v[3] = 5, 9, 7
            cp = np.ascontiguousarray(oracle.encode(P, v[None, :])[0])
            assert lib.rlnc_decoder_add_piece(h, v.ctypes.data_as(U8P), k, cp.ctypes.data_as(U8P), L) == \
                ref.add(v, cp)
            _state_eq(h, ref, k)
            for j in (3, sys_rows[5]):
                s, out = _decoded_piece(h, j, L)
                assert s == 0 and np.array_equal(out, P[j]), j
        if ref.is_decoded():
            break
    assert ref.is_decoded()
    out = np.empty((k, L), np.uint8)
    errors.check(lib.rlnc_decoder_get_pieces(h, out.ctypes.data_as(U8P)))
    assert np.array_equal(out, P)
    lib.rlnc_decoder_destroy(h)
    gpu_ctx.synchronize()
    for d in bufs:
        gpu_ctx.free(d)


def test_compact_rows_partial_get_piece_and_grouped(gpu_ctx):
    """GetPiece before full rank (decoder_state.go:233-256's availability rule
    through the few-row product, un-slicing the compact rows) and the grouped
    GetPieces (twins only) on decoders fed by one batched GPU AddPiece."""
    lib = _lib.lib()
    k, L, G = 32, 4096, 3
    rng = np.random.default_rng(77)
    hs, Ps, ds = [], [], []
    for g in range(G):
        P = rng.integers(0, 256, (k, L), dtype=np.uint8)
        V = rng.integers(0, 256, (k + 2, k), dtype=np.uint8)
        C = oracle.encode(P, V)
        d, pitch = _dev_rows(gpu_ctx, V, C)
        h = ctypes.c_void_p()
        errors.check(lib.rlnc_decoder_create(gpu_ctx.handle, k, ctypes.byref(h)))
        hs.append(h)
        Ps.append(P)
        ds.append(d)
    arr = (ctypes.c_void_p * G)(*[h.value for h in hs])
    rows = (ctypes.c_void_p * G)(*ds)
    counts = (ctypes.c_size_t * G)(*([k + 2] * G))
    cons, sts = (ctypes.c_size_t * G)(), (ctypes.c_int * G)()
    errors.check(lib.rlnc_decoders_add_pieces_gpu(arr, G, rows, counts, pitch, L, cons, sts))
    dO = gpu_ctx.alloc(G * k * L)
    errors.check(lib.rlnc_decoders_get_pieces_device(arr, G, dO, L))
    got = gpu_ctx.d2h(dO, G * k * L).reshape(G, k, L)
    for g in range(G):
        assert np.array_equal(got[g], Ps[g])
        # and one piece through GetPiece (a fresh materialisation of the state)
        one = np.empty(L, np.uint8)
        errors.check(lib.rlnc_decoder_get_piece(hs[g], 5, one.ctypes.data_as(U8P)))
        assert np.array_equal(one, Ps[g][5])
    # partial GetPiece on a decoder holding a compact batch short of full rank
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    V = np.zeros((k // 2, k), np.uint8)
    V[np.arange(k // 2), np.arange(k // 2)] = 1
    V[3, :] = 0
    V[3, 3] = 1
    V[3, k - 1] = 0
    C = oracle.encode(P, V)
    d, pitch2 = _dev_rows(gpu_ctx, V, C)
    h = ctypes.c_void_p()
    errors.check(lib.rlnc_decoder_create(gpu_ctx.handle, k, ctypes.byref(h)))
    c = ctypes.c_size_t()
    lib.rlnc_decoder_add_pieces(h, ctypes.c_void_p(d), V.shape[0], pitch2, L, 1, ctypes.byref(c))
    ref = oracle.Decoder(k)
    for i in range(V.shape[0]):
        ref.add(V[i], C[i])
    for idx in (0, 3, k // 2 - 1, k // 2):
        one = np.empty(L, np.uint8)
        st = lib.rlnc_decoder_get_piece(h, idx, one.ctypes.data_as(U8P))
        exp_st, exp = ref.get_piece(idx)
        assert st == exp_st, idx
        if st == 0:
            assert np.array_equal(one, exp)
    for x in hs + [h]:
        lib.rlnc_decoder_destroy(x)
    gpu_ctx.synchronize()
    for x in ds + [d, dO]:
        gpu_ctx.free(x)
