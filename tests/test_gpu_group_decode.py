"""Grouped GetPieces (rlnc_decoders_get_pieces_device): G decoded generations
applied in one bit-sliced launch per 16 decoders, or per decoder when a T has
unit (systematic) rows or the received counts differ.  Every byte is checked
against the original pieces (what kodr's GetPieces returns once decoded,
full/decoder.go:83-99) and against the per-decoder call."""
import ctypes

import numpy as np
import pytest

import oracle
from kodr_amd import _lib, errors

pytestmark = pytest.mark.gpu
U8P = _lib._u8p


def _decoder(ctx, P, rng, extra=0, systematic=0, gpu_elim=False, dup=False):
    """A decoder fed k + extra wire rows of P (the first `systematic` of them
    unit vectors; dup: row 1 repeats row 0, so k + 1 rows are received),
    through one batched AddPiece."""
    k, L = P.shape
    n = k + extra
    V = rng.integers(0, 256, (n, k), dtype=np.uint8)
    if dup:
        V[1] = V[0]
    for i in range(systematic):
        V[i] = 0
        V[i, i] = 1
    rows = np.ascontiguousarray(np.concatenate([V, oracle.encode(P, V)], axis=1))
    h = ctypes.c_void_p()
    lib = _lib.lib()
    errors.check(lib.rlnc_decoder_create(ctx.handle, k, ctypes.byref(h)))
    used = ctypes.c_size_t()
    if gpu_elim:
        d = ctx.alloc(rows.nbytes)
        ctx.h2d(d, rows)
        st = lib.rlnc_decoder_add_pieces_gpu(h, d, n, k + L, L, ctypes.byref(used))
        ctx.synchronize()
        ctx.free(d)
    else:
        st = lib.rlnc_decoder_add_pieces(h, rows.ctypes.data_as(U8P), n, k + L, L, 0, ctypes.byref(used))
    assert st in (0, 3), st   # 3: ALL_USEFUL_PIECES_RECEIVED past full rank
    return h


def _grouped_get(ctx, hs, k, L, pitch):
    G = len(hs)
    arr = (ctypes.c_void_p * G)(*[h.value for h in hs])
    dO = ctx.alloc(G * k * pitch + 64)
    try:
        ctx.h2d(dO, np.full(G * k * pitch + 64, 0x5A, np.uint8))
        st = _lib.lib().rlnc_decoders_get_pieces_device(arr, G, dO, pitch)
        ctx.synchronize()
        raw = ctx.d2h(dO, G * k * pitch + 64)
    finally:
        ctx.free(dO)
    assert (raw[G * k * pitch:] == 0x5A).all()
    return st, raw[:G * k * pitch].reshape(G, k, pitch)


def _stats(h):
    g, c = ctypes.c_size_t(), ctypes.c_size_t()
    errors.check(_lib.lib().rlnc_decoder_apply_stats(h, ctypes.byref(g), ctypes.byref(c)))
    return g.value, c.value, bool(_lib.lib().rlnc_decoder_last_apply_bitsliced(h))


@pytest.mark.parametrize("G,k,L,extra", [(4, 64, 8192, 0), (3, 100, 4096 + 64, 2), (33, 16, 2048, 0),
                                         (2, 256, 16384, 1)])
def test_grouped_get_coded(gpu_ctx, G, k, L, extra):
    rng = np.random.default_rng(G * 7 + k + L)
    gens = [rng.integers(0, 256, (k, L), dtype=np.uint8) for _ in range(G)]
    hs = [_decoder(gpu_ctx, P, rng, extra=extra) for P in gens]
    try:
        pitch = (L + 15) // 16 * 16 + 16
        st, got = _grouped_get(gpu_ctx, hs, k, L, pitch)
        assert st == 0
        for g in range(G):
            assert np.array_equal(got[g, :, :L], gens[g]), g
            assert (got[g, :, L:] == 0x5A).all(), "wrote past L"
        # the grouped bit-sliced launch ran (k = 16: few narrow rows, the
        # per-decoder v_perm route)
        assert _stats(hs[0]) == (k, 0, k > 32)
    finally:
        for h in hs:
            _lib.lib().rlnc_decoder_destroy(h)


def test_grouped_get_mixed_falls_back(gpu_ctx):
    # one systematic decoder (unit rows of T are copies) and one with a
    # different received count: per-decoder route, same bytes
    rng = np.random.default_rng(91)
    k, L = 32, 4096
    gens = [rng.integers(0, 256, (k, L), dtype=np.uint8) for _ in range(3)]
    hs = [_decoder(gpu_ctx, gens[0], rng), _decoder(gpu_ctx, gens[1], rng, systematic=20),
          _decoder(gpu_ctx, gens[2], rng, extra=3, dup=True)]
    try:
        st, got = _grouped_get(gpu_ctx, hs, k, L, L)
        assert st == 0
        for g in range(3):
            assert np.array_equal(got[g], gens[g]), g
        assert _stats(hs[1])[1] == 20      # the systematic decoder copied its 20 unit rows
        assert _lib.lib().rlnc_decoder_received(hs[2]) == k + 1
    finally:
        for h in hs:
            _lib.lib().rlnc_decoder_destroy(h)


def test_grouped_get_mixed_received(gpu_ctx):
    # a decoder that received a dependent piece (k + 1 received, rank k)
    # shares the grouped launch: its T is padded with a zero column
    rng = np.random.default_rng(93)
    k, L = 64, 8192
    gens = [rng.integers(0, 256, (k, L), dtype=np.uint8) for _ in range(4)]
    hs = [_decoder(gpu_ctx, P, rng, extra=3, dup=(g == 2)) for g, P in enumerate(gens)]
    try:
        assert _lib.lib().rlnc_decoder_received(hs[2]) == k + 1
        assert _lib.lib().rlnc_decoder_received(hs[0]) == k
        st, got = _grouped_get(gpu_ctx, hs, k, L, L)
        assert st == 0
        for g in range(4):
            assert np.array_equal(got[g], gens[g]), g
            assert _stats(hs[g]) == (k, 0, True), g   # every decoder in the one bit-sliced launch
    finally:
        for h in hs:
            _lib.lib().rlnc_decoder_destroy(h)


def test_grouped_get_not_decoded(gpu_ctx):
    rng = np.random.default_rng(5)
    k, L = 16, 1024
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    a = _decoder(gpu_ctx, P, rng)
    b = ctypes.c_void_p()
    errors.check(_lib.lib().rlnc_decoder_create(gpu_ctx.handle, k, ctypes.byref(b)))
    try:
        arr = (ctypes.c_void_p * 2)(a.value, b.value)
        dO = gpu_ctx.alloc(2 * k * L)
        try:
            assert _lib.lib().rlnc_decoders_get_pieces_device(arr, 2, dO, L) == 4  # MORE_USEFUL_PIECES_REQUIRED
        finally:
            gpu_ctx.free(dO)
    finally:
        _lib.lib().rlnc_decoder_destroy(a)
        _lib.lib().rlnc_decoder_destroy(b)


def test_grouped_get_c2(gpu_ctx):
    # three 32 MiB/256 generations decoded through the GPU elimination, then
    # one grouped apply (8.6 G GF MACs per generation)
    rng = np.random.default_rng(0xC2)
    k, L = 256, 131072
    gens = [rng.integers(0, 256, (k, L), dtype=np.uint8) for _ in range(3)]
    hs = [_decoder(gpu_ctx, P, rng, extra=2, gpu_elim=True) for P in gens]
    try:
        st, got = _grouped_get(gpu_ctx, hs, k, L, L)
        assert st == 0
        for g in range(3):
            assert np.array_equal(got[g], gens[g]), g
        assert _stats(hs[2]) == (k, 0, True)
    finally:
        for h in hs:
            _lib.lib().rlnc_decoder_destroy(h)


def test_grouped_get_chunk_fallback(gpu_ctx):
    # decoders 0-15 form a grouped launch; the chunk holding the systematic
    # decoder 17 goes decoder by decoder
    rng = np.random.default_rng(17)
    k, L = 64, 4096
    gens = [rng.integers(0, 256, (k, L), dtype=np.uint8) for _ in range(18)]
    hs = [_decoder(gpu_ctx, P, rng, systematic=(10 if g == 17 else 0)) for g, P in enumerate(gens)]
    try:
        st, got = _grouped_get(gpu_ctx, hs, k, L, L)
        assert st == 0
        for g in range(18):
            assert np.array_equal(got[g], gens[g]), g
        assert _stats(hs[0]) == (k, 0, True)
        assert _stats(hs[17])[:2] == (k - 10, 10)
    finally:
        for h in hs:
            _lib.lib().rlnc_decoder_destroy(h)
