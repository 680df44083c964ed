"""Which route eliminated a decoder's batch, and that the GPU route is total
for invertible C (gf_elim.hip attempts: a singular panel block re-runs the
launch with the rows rotated; capi_decoder.cpp rlnc_decoder_elim_stats reports it).

kodr eliminates on every AddPiece (full/decoder.go:50-66) with a pivot search
down the whole column (kodr_internals/matrix/decoder_state.go:23-35); the GPU
pivots inside 16-row panels, so about 6 % of uniform k = 256 batches have a
singular leading panel block (tests/panel_rule.py models it).  Every test
here checks the decoder against the oracle's literal decoder and the route
against the model: states the GPU produced (gpu), after a rotated attempt
(gpu_retried), launches that fell back to the host (host_after_gpu)."""
import ctypes

import numpy as np
import pytest

import oracle
import panel_rule as pr
from kodr_amd import _lib, errors
from kodr_amd._codec import elim_stats

pytestmark = pytest.mark.gpu
U8P = _lib._u8p


@pytest.fixture(autouse=True)
def default_route(gpu_ctx):
    prev = gpu_ctx.route_min_k
    gpu_ctx.set_route_min_k(224)
    yield
    gpu_ctx.set_route_min_k(prev)


def _new(ctx, k):
    h = ctypes.c_void_p()
    errors.check(_lib.lib().rlnc_decoder_create(ctx.handle, k, ctypes.byref(h)))
    return h


def _rows(ctx, V, C):
    n, k = V.shape
    L = C.shape[1]
    pitch = (k + L + 15) // 16 * 16
    rows = np.zeros((n, pitch), np.uint8)
    rows[:, :k] = V
    rows[:, k:k + L] = C
    d = ctx.alloc(rows.nbytes)
    ctx.h2d(d, rows)
    return d, pitch


def _check_vs_oracle(h, P, V, C, consumed=None):
    lib = _lib.lib()
    k, L = P.shape
    ref = oracle.Decoder(k)
    n_ok = 0
    for i in range(V.shape[0]):
        if ref.add(V[i], C[i]) != 0:
            break
        n_ok += 1
    if consumed is not None:
        assert consumed == n_ok
    assert (lib.rlnc_decoder_useful(h), lib.rlnc_decoder_required(h), bool(lib.rlnc_decoder_is_decoded(h))) == \
        (ref.useful(), ref.required(), ref.is_decoded())
    r = lib.rlnc_decoder_useful(h)
    co = np.empty((r, k), np.uint8)
    errors.check(lib.rlnc_decoder_coefficients(h, co.ctypes.data_as(U8P)))
    assert np.array_equal(co, ref.coeffs())
    if ref.is_decoded():
        out = np.empty((k, L), np.uint8)
        errors.check(lib.rlnc_decoder_get_pieces(h, out.ctypes.data_as(U8P)))
        assert np.array_equal(out, P)


def _stats(h):
    return elim_stats(h)


@pytest.mark.parametrize("seed", [7, 8, 11, 12])
def test_single_decoder_route_and_retry(gpu_ctx, seed):
    """rlnc_decoder_add_pieces (device rows, k = 256) routes the batch to
    gf_elim_mc4; the device vectors of seeds 7 and 8 need a rotated attempt
    (profiles/r04/c2_seeds/), 11 and 12 do not.  No host fallback either way."""
    k, L = 256, 64
    V = pr.device_vectors(seed, k + 2, k)
    att = pr.expected_attempt(V[:k])
    assert att is not None
    rng = np.random.default_rng(seed)
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    C = oracle.encode(P, V)
    d, pitch = _rows(gpu_ctx, V, C)
    h = _new(gpu_ctx, k)
    c = ctypes.c_size_t()
    st = _lib.lib().rlnc_decoder_add_pieces(h, ctypes.c_void_p(d), k + 2, pitch, L, 1, ctypes.byref(c))
    assert st == 3  # ErrAllUsefulPiecesReceived after the k-th row (full/decoder.go:52-54)
    _check_vs_oracle(h, P, V, C, consumed=c.value)
    s = _stats(h)
    assert s["gpu"] == 1 and s["host_after_gpu"] == 0, s
    assert s["gpu_retried"] == (1 if att > 0 else 0), (s, att)
    _lib.lib().rlnc_decoder_destroy(h)
    gpu_ctx.synchronize()
    gpu_ctx.free(d)


def test_fresh_c2_vector_sets_never_leave_the_gpu(gpu_ctx):
    """64 fresh uniform k = 256 vector sets: every invertible C is eliminated
    on the GPU (host_after_gpu == 0); a singular one (1 in 255) falls back."""
    k, L = 256, 32
    rng = np.random.default_rng(20251018)
    retried = 0
    for t in range(64):
        V = rng.integers(0, 256, (k + 2, k), dtype=np.uint8)
        P = rng.integers(0, 256, (k, L), dtype=np.uint8)
        C = oracle.encode(P, V)
        d, pitch = _rows(gpu_ctx, V, C)
        h = _new(gpu_ctx, k)
        c = ctypes.c_size_t()
        _lib.lib().rlnc_decoder_add_pieces(h, ctypes.c_void_p(d), k + 2, pitch, L, 1, ctypes.byref(c))
        _check_vs_oracle(h, P, V, C, consumed=c.value)
        s = _stats(h)
        invertible = pr.gf_inverse(V[:k]) is not None
        assert s["host_after_gpu"] == (0 if invertible else 1), (t, s)
        retried += s["gpu_retried"]
        _lib.lib().rlnc_decoder_destroy(h)
        gpu_ctx.synchronize()
        gpu_ctx.free(d)
    print("retried", retried, "of 64")


def test_grouped_launch_retries_per_decoder(gpu_ctx):
    """rlnc_decoders_add_pieces_gpu with 16 decoders (gf_elim_mc2), seeds 7
    and 8 among them: each decoder's attempts are its own; none leaves the GPU."""
    k, L, G = 256, 48, 16
    seeds = [7, 8] + list(range(100, 100 + G - 2))
    hs, ds, Ps, Vs, Cs = [], [], [], [], []
    for seed in seeds:
        V = pr.device_vectors(seed, k + 2, k)
        P = np.random.default_rng(seed).integers(0, 256, (k, L), dtype=np.uint8)
        C = oracle.encode(P, V)
        d, pitch = _rows(gpu_ctx, V, C)
        hs.append(_new(gpu_ctx, k))
        ds.append(d)
        Ps.append(P)
        Vs.append(V)
        Cs.append(C)
    G = len(hs)
    arr = (ctypes.c_void_p * G)(*[h.value for h in hs])
    rows = (ctypes.c_void_p * G)(*ds)
    counts = (ctypes.c_size_t * G)(*([k + 2] * G))
    cons, sts = (ctypes.c_size_t * G)(), (ctypes.c_int * G)()
    errors.check(_lib.lib().rlnc_decoders_add_pieces_gpu(arr, G, rows, counts, pitch, L, cons, sts))
    for g in range(G):
        assert sts[g] in (0, 3)
        _check_vs_oracle(hs[g], Ps[g], Vs[g], Cs[g], consumed=cons[g])
        s = _stats(hs[g])
        att = pr.expected_attempt(Vs[g][:k])
        assert s["gpu"] == 1 and s["host_after_gpu"] == 0, (g, s)
        assert s["gpu_retried"] == (1 if att > 0 else 0), (g, s, att)
    for h in hs:
        _lib.lib().rlnc_decoder_destroy(h)
    gpu_ctx.synchronize()
    for d in ds:
        gpu_ctx.free(d)


def test_lazy_flush_retries_and_structured_batches_abort(gpu_ctx):
    """The lazy AddPiece queue (one call per borrowed device piece) of a seed-7
    decoder is eliminated on the GPU after a rotated attempt when a state read
    flushes it; a systematic-order queue at k = 256 stays on the host
    (queue_looks_systematic), and a systematic batch through
    rlnc_decoder_add_pieces aborts on the GPU at once (a zero block column)
    and takes kodr's route."""
    lib = _lib.lib()
    k, L = 256, 64
    V = pr.device_vectors(7, k + 1, k)
    P = np.random.default_rng(3).integers(0, 256, (k, L), dtype=np.uint8)
    C = oracle.encode(P, V)
    d, pitch = _rows(gpu_ctx, V, C)
    h = _new(gpu_ctx, k)
    for i in range(k + 1):
        v = np.ascontiguousarray(V[i])
        st = lib.rlnc_decoder_add_piece_device_borrowed(h, v.ctypes.data_as(U8P), k, d + i * pitch + k, L)
        assert st == (0 if i < k else 3)
    _check_vs_oracle(h, P, V, C)
    s = _stats(h)
    assert s["gpu"] == 1 and s["gpu_retried"] == 1 and s["host_after_gpu"] == 0, s
    lib.rlnc_decoder_destroy(h)
    # systematic batch through the batched entry point
    eye = np.eye(k, dtype=np.uint8)[[i for i in range(k) if i not in (5, 77)]]
    S = np.concatenate([eye, np.random.default_rng(4).integers(0, 256, (4, k), dtype=np.uint8)])
    CS = oracle.encode(P, S)
    d2, pitch2 = _rows(gpu_ctx, S, CS)
    h2 = _new(gpu_ctx, k)
    c = ctypes.c_size_t()
    lib.rlnc_decoder_add_pieces(h2, ctypes.c_void_p(d2), S.shape[0], pitch2, L, 1, ctypes.byref(c))
    _check_vs_oracle(h2, P, S, CS, consumed=c.value)
    s = _stats(h2)
    assert s["gpu"] == 0 and s["host_after_gpu"] == 1, s
    lib.rlnc_decoder_destroy(h2)
    gpu_ctx.synchronize()
    gpu_ctx.free(d)
    gpu_ctx.free(d2)


def test_singular_queue_is_launched_once(gpu_ctx):
    """A queue whose C is singular fails the GPU elimination of the grouped
    flush; the decoder's next state read goes straight to the host (one
    failed launch, not two: the ADVICE r04 medium finding)."""
    lib = _lib.lib()
    k, L = 256, 32
    rng = np.random.default_rng(17)
    V = rng.integers(0, 256, (k + 2, k), dtype=np.uint8)
    V[k - 1] = V[4] ^ pr.mul(9, V[200]).astype(np.uint8)  # row k - 1 dependent: C singular
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    C = oracle.encode(P, V)
    d, pitch = _rows(gpu_ctx, V, C)
    h = _new(gpu_ctx, k)
    for i in range(k):
        v = np.ascontiguousarray(V[i])
        assert lib.rlnc_decoder_add_piece_device_borrowed(h, v.ctypes.data_as(U8P), k, d + i * pitch + k, L) == 0
    arr = (ctypes.c_void_p * 1)(h.value)
    errors.check(lib.rlnc_decoders_flush_gpu(arr, 1))
    assert not lib.rlnc_decoder_is_decoded(h)
    for i in range(k, k + 2):
        v = np.ascontiguousarray(V[i])
        lib.rlnc_decoder_add_piece_device_borrowed(h, v.ctypes.data_as(U8P), k, d + i * pitch + k, L)
    _check_vs_oracle(h, P, V, C)
    s = _stats(h)
    assert s["host_after_gpu"] == 1, s
    lib.rlnc_decoder_destroy(h)
    gpu_ctx.synchronize()
    gpu_ctx.free(d)


def test_tags_stay_fresh_across_buffer_growth(gpu_ctx):
    """a k = 256 single-decoder launch, then a grouped
    k = 128 launch of 4 decoders on the same context (its hand-off buffer
    grows, the pinned status buffer does not).  The second launch's tags are
    new, so no status word of the first can pass for one of its own; every
    decoder equals the oracle."""
    lib = _lib.lib()
    for k, G, seed in ((256, 1, 31), (128, 4, 32), (256, 1, 33), (64, 8, 34)):
        rng = np.random.default_rng(seed)
        L = 40
        hs, ds, Ps, Vs, Cs = [], [], [], [], []
        for g in range(G):
            V = rng.integers(0, 256, (k + 2, k), dtype=np.uint8)
            P = rng.integers(0, 256, (k, L), dtype=np.uint8)
            C = oracle.encode(P, V)
            d, pitch = _rows(gpu_ctx, V, C)
            hs.append(_new(gpu_ctx, k))
            ds.append(d)
            Ps.append(P)
            Vs.append(V)
            Cs.append(C)
        arr = (ctypes.c_void_p * G)(*[h.value for h in hs])
        rows = (ctypes.c_void_p * G)(*ds)
        counts = (ctypes.c_size_t * G)(*([k + 2] * G))
        cons, sts = (ctypes.c_size_t * G)(), (ctypes.c_int * G)()
        errors.check(lib.rlnc_decoders_add_pieces_gpu(arr, G, rows, counts, pitch, L, cons, sts))
        for g in range(G):
            _check_vs_oracle(hs[g], Ps[g], Vs[g], Cs[g], consumed=cons[g])
            lib.rlnc_decoder_destroy(hs[g])
        gpu_ctx.synchronize()
        for d in ds:
            gpu_ctx.free(d)


@pytest.mark.parametrize("G", [2, 7])
def test_largest_mc4_launch(gpu_ctx, G):
    """rlnc_decoders_add_pieces_gpu at k = 256 with up to 7 decoders: one
    gf_elim_mc4 launch of G x 33 workgroups (7: 231, the most the
    kElimMcMaxBlocks = 256 cap admits), seed 7 (a rotated attempt) among
    them; every decoder equals the oracle and stays on the GPU."""
    k, L = 256, 48
    seeds = [7] + list(range(200, 200 + G - 1))
    hs, ds, Ps, Vs, Cs = [], [], [], [], []
    for seed in seeds:
        V = pr.device_vectors(seed, k + 2, k)
        P = np.random.default_rng(seed).integers(0, 256, (k, L), dtype=np.uint8)
        C = oracle.encode(P, V)
        d, pitch = _rows(gpu_ctx, V, C)
        hs.append(_new(gpu_ctx, k))
        ds.append(d)
        Ps.append(P)
        Vs.append(V)
        Cs.append(C)
    arr = (ctypes.c_void_p * G)(*[h.value for h in hs])
    rows = (ctypes.c_void_p * G)(*ds)
    counts = (ctypes.c_size_t * G)(*([k + 2] * G))
    cons, sts = (ctypes.c_size_t * G)(), (ctypes.c_int * G)()
    errors.check(_lib.lib().rlnc_decoders_add_pieces_gpu(arr, G, rows, counts, pitch, L, cons, sts))
    for g in range(G):
        assert sts[g] in (0, 3)
        _check_vs_oracle(hs[g], Ps[g], Vs[g], Cs[g], consumed=cons[g])
        s = _stats(hs[g])
        att = pr.expected_attempt(Vs[g][:k])
        assert s["gpu"] == 1 and s["host_after_gpu"] == 0, (g, s)
        assert s["gpu_retried"] == (1 if att > 0 else 0), (g, s, att)
    for h in hs:
        _lib.lib().rlnc_decoder_destroy(h)
    gpu_ctx.synchronize()
    for d in ds:
        gpu_ctx.free(d)
