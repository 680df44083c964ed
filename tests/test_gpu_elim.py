"""GPU elimination (gf_elim.hip through rlnc_decoder_add_pieces_gpu /
rlnc_decoders_add_pieces_gpu) against the host elimination (DecoderCore,
itself tied to the oracle's literal restatement of decoder_state.go in
tests/test_capi_host.py) and the oracle: return codes, rows consumed,
counters, the coefficient matrix and the transform T byte for byte, and the
decoded pieces."""
import ctypes

import numpy as np
import pytest

import oracle
import panel_rule as pr
from kodr_amd import _lib, errors
from kodr_amd._codec import elim_stats

pytestmark = pytest.mark.gpu
U8P = _lib._u8p


class Dec:
    def __init__(self, ctx, k):
        self.k = k
        self.h = ctypes.c_void_p()
        errors.check(_lib.lib().rlnc_decoder_create(ctx.handle, k, ctypes.byref(self.h)))

    def state(self):
        L = _lib.lib()
        return (L.rlnc_decoder_useful(self.h), L.rlnc_decoder_received(self.h),
                L.rlnc_decoder_required(self.h), bool(L.rlnc_decoder_is_decoded(self.h)))

    def coefficients(self):
        r = _lib.lib().rlnc_decoder_useful(self.h)
        out = np.empty((r, self.k), np.uint8)
        if r:
            errors.check(_lib.lib().rlnc_decoder_coefficients(self.h, out.ctypes.data_as(U8P)))
        return out

    def transform(self):
        L = _lib.lib()
        r, n = L.rlnc_decoder_useful(self.h), L.rlnc_decoder_received(self.h)
        out = np.empty((r, n), np.uint8)
        if r:
            errors.check(L.rlnc_decoder_transform(self.h, out.ctypes.data_as(U8P)))
        return out

    def get_all(self):
        L = _lib.lib()
        n, pl = L.rlnc_decoder_useful(self.h), L.rlnc_decoder_piece_length(self.h)
        out = np.empty((n, pl), np.uint8)
        st = L.rlnc_decoder_get_pieces(self.h, out.ctypes.data_as(U8P))
        return st, out

    def __del__(self):
        _lib.lib().rlnc_decoder_destroy(self.h)


def _vectors(rng, kind, n, k):
    if kind == "dense":
        return rng.integers(0, 256, (n, k), dtype=np.uint8)
    if kind == "tiny":  # zero diagonals, dependent rows, duplicates
        return rng.integers(0, 3, (n, k), dtype=np.uint8)
    if kind == "lowrank":
        B = rng.integers(0, 256, (max(1, k // 2), k), dtype=np.uint8)
        return oracle.matmul(rng.integers(0, 256, (n, B.shape[0]), dtype=np.uint8), B)[1]
    if kind == "zero_mid":  # a zero row in the middle of a clean run
        V = rng.integers(0, 256, (n, k), dtype=np.uint8)
        V[min(n - 1, k // 2)] = 0
        return V
    if kind == "systematic":  # units in order with a loss, then coded rows
        eye = np.eye(k, dtype=np.uint8)[[i for i in range(k) if i != k // 3]]
        return np.concatenate([eye, rng.integers(0, 256, (n, k), dtype=np.uint8)])[:n]
    if kind == "first_zero":  # the first piece is all zero (counted useful, full/decoder.go:58-61)
        V = rng.integers(0, 256, (n, k), dtype=np.uint8)
        V[0] = 0
        return V
    raise ValueError(kind)


def _rows(ctx, V, P, L):
    n, k = V.shape
    pitch = ((k + L + 15) // 16) * 16 + 16
    rows = np.zeros((n, pitch), np.uint8)
    rows[:, :k] = V
    rows[:, k:k + L] = oracle.encode(P, V)
    d = ctx.alloc(rows.nbytes)
    ctx.h2d(d, rows)
    return d, pitch


@pytest.fixture(autouse=True)
def host_references(gpu_ctx):
    # the reference decoders here run kodr's elimination on the host:
    # rlnc_decoder_add_pieces and the lazy flush would otherwise route large
    # full batches to the GPU elimination themselves (capi_decoder.cpp dec_route_gpu)
    prev = gpu_ctx.route_min_k
    gpu_ctx.set_route_min_k(100000)
    yield
    gpu_ctx.set_route_min_k(prev)


def _same(a, b):
    assert a.state() == b.state()
    assert np.array_equal(a.coefficients(), b.coefficients())
    assert np.array_equal(a.transform(), b.transform())


@pytest.mark.parametrize("kind", ["dense", "tiny", "lowrank", "zero_mid", "systematic", "first_zero"])
@pytest.mark.parametrize("k", [2, 3, 16, 65, 128, 200, 256])
def test_gpu_elimination_matches_host(gpu_ctx, kind, k):
    rng = np.random.default_rng(k * 31 + len(kind))
    L = 40
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    n = k + 3
    V = _vectors(rng, kind, n, k)
    drows, pitch = _rows(gpu_ctx, V, P, L)
    host, gpu = Dec(gpu_ctx, k), Dec(gpu_ctx, k)
    ch, cg = ctypes.c_size_t(), ctypes.c_size_t()
    sh = _lib.lib().rlnc_decoder_add_pieces(host.h, ctypes.c_void_p(drows), n, pitch, L, 1, ctypes.byref(ch))
    sg = _lib.lib().rlnc_decoder_add_pieces_gpu(gpu.h, ctypes.c_void_p(drows), n, pitch, L, ctypes.byref(cg))
    assert (sg, cg.value) == (sh, ch.value)
    _same(host, gpu)
    if kind == "dense" and pr.gf_inverse(V[:k]) is not None:
        # the state came from the GPU elimination, not a host fallback
        s = elim_stats(gpu.h)
        assert s["gpu"] == 1 and s["host_after_gpu"] == 0, s
        assert elim_stats(host.h)["gpu"] == 0
    # and the oracle's literal decoder, step by step
    ref = oracle.Decoder(k)
    C = oracle.encode(P, V)
    exp_n = 0
    for i in range(n):
        if ref.add(V[i], C[i]) != 0:
            break
        exp_n += 1
    assert cg.value == exp_n
    assert gpu.state() == (ref.useful(), ref.received(), ref.required(), ref.is_decoded())
    assert np.array_equal(gpu.coefficients(), ref.coeffs())
    if ref.is_decoded():
        st, out = gpu.get_all()
        assert st == 0 and np.array_equal(out, P)
    gpu_ctx.synchronize()
    gpu_ctx.free(drows)


def test_gpu_elimination_batched_generations(gpu_ctx):
    """Several decoders in one launch: fresh ones with clean and quirky
    batches, one that already holds a piece (a continued decoder: its batch
    completes the rank), one with a single row (host path); each ends exactly
    as rlnc_decoder_add_pieces leaves it."""
    rng = np.random.default_rng(77)
    k, L = 64, 100
    kinds = ["dense", "tiny", "dense", "lowrank", "dense", "systematic", "dense"]
    gens = []
    for gi, kind in enumerate(kinds):
        P = rng.integers(0, 256, (k, L), dtype=np.uint8)
        n = 1 if gi == 4 else k + int(rng.integers(0, 5))
        V = _vectors(rng, kind, n, k)
        gens.append((P, V))
    pitch = ((k + L + 15) // 16) * 16
    bufs, hosts, gpus = [], [], []
    for gi, (P, V) in enumerate(gens):
        rows = np.zeros((V.shape[0], pitch), np.uint8)
        rows[:, :k], rows[:, k:k + L] = V, oracle.encode(P, V)
        d = gpu_ctx.alloc(rows.nbytes)
        gpu_ctx.h2d(d, rows)
        bufs.append(d)
        hosts.append(Dec(gpu_ctx, k))
        gpus.append(Dec(gpu_ctx, k))
    # decoder 2 already holds one piece: not fresh, eliminated from [its row ; the batch]
    c0 = ctypes.c_size_t()
    for dec in (hosts[2], gpus[2]):
        assert _lib.lib().rlnc_decoder_add_pieces(dec.h, ctypes.c_void_p(bufs[2]), 1, pitch, L, 1,
                                                  ctypes.byref(c0)) == 0
    G = len(gens)
    off = [1 if gi == 2 else 0 for gi in range(G)]
    counts = (ctypes.c_size_t * G)(*[gens[gi][1].shape[0] - off[gi] for gi in range(G)])
    rows_p = (ctypes.c_void_p * G)(*[bufs[gi] + off[gi] * pitch for gi in range(G)])
    decs = (ctypes.c_void_p * G)(*[g.h.value for g in gpus])
    consumed = (ctypes.c_size_t * G)()
    status = (ctypes.c_int * G)()
    errors.check(_lib.lib().rlnc_decoders_add_pieces_gpu(decs, G, rows_p, counts, pitch, L, consumed, status))
    for gi in range(G):
        c = ctypes.c_size_t()
        st = _lib.lib().rlnc_decoder_add_pieces(hosts[gi].h, ctypes.c_void_p(rows_p[gi]), counts[gi], pitch, L, 1,
                                                ctypes.byref(c))
        assert (status[gi], consumed[gi]) == (st, c.value), gi
        _same(hosts[gi], gpus[gi])
        if hosts[gi].state()[3]:
            s1, a = gpus[gi].get_all()
            assert s1 == 0 and np.array_equal(a, gens[gi][0])
    gpu_ctx.synchronize()
    for d in bufs:
        gpu_ctx.free(d)


def test_gpu_elimination_c2_round_trip(gpu_ctx):
    """32 MiB / 256 (BASELINE config 2): k + 2 device wire rows drawn by the
    engine, eliminated on the GPU, GetPieces equals the generation."""
    k, L = 256, 131072
    rng = np.random.default_rng(5)
    data = rng.integers(0, 256, k * L, dtype=np.uint8)
    eh = ctypes.c_void_p()
    errors.check(_lib.lib().rlnc_encoder_create(gpu_ctx.handle, 0, data.ctypes.data_as(U8P), k, L,
                                                ctypes.byref(eh)))
    W = k + L
    n = k + 2
    dW = gpu_ctx.alloc(n * W)
    errors.check(_lib.lib().rlnc_encoder_coded_wire_device(eh, n, dW, W))
    dec, host = Dec(gpu_ctx, k), Dec(gpu_ctx, k)
    c = ctypes.c_size_t()
    st = _lib.lib().rlnc_decoder_add_pieces_gpu(dec.h, ctypes.c_void_p(dW), n, W, L, ctypes.byref(c))
    ch = ctypes.c_size_t()
    sh = _lib.lib().rlnc_decoder_add_pieces(host.h, ctypes.c_void_p(dW), n, W, L, 1, ctypes.byref(ch))
    assert (st, c.value) == (sh, ch.value)
    assert dec.state()[3]
    assert np.array_equal(dec.transform(), host.transform())
    V = gpu_ctx.d2h(dW, n * W).reshape(n, W)[:k, :k]
    s = elim_stats(dec.h)
    assert s["gpu"] == 1 and s["host_after_gpu"] == 0, s
    assert s["gpu_retried"] == (1 if pr.expected_attempt(V) else 0), s
    dDec = gpu_ctx.alloc(k * L)
    errors.check(_lib.lib().rlnc_decoder_get_pieces_device(dec.h, dDec, L))
    assert np.array_equal(gpu_ctx.d2h(dDec, k * L), data)
    _lib.lib().rlnc_encoder_destroy(eh)
    gpu_ctx.synchronize()
    gpu_ctx.free(dW)
    gpu_ctx.free(dDec)


@pytest.mark.parametrize("k", [32, 48, 256])
def test_gpu_elimination_many_decoders(gpu_ctx, k):
    """More decoders than one launch takes (kElimMaxGens = 64, and as many
    grouped row copies; at k = 256 the multi-workgroup kernel's 32 decoders
    of 8 workgroups each): full dense batches (blocked kernel), {0,1,2}-valued
    ones (zero diagonals, panel blocks that are singular while C is not: the
    host route), a panel-local dependence, and a few short batches; every
    decoder ends as rlnc_decoder_add_pieces leaves it, pieces included."""
    rng = np.random.default_rng(4242 + k)
    L = 96
    G = 70
    pitch = ((k + L + 15) // 16) * 16
    gens, bufs, hosts, gpus = [], [], [], []
    for gi in range(G):
        P = rng.integers(0, 256, (k, L), dtype=np.uint8)
        n = k + int(rng.integers(0, 3)) if gi % 9 else int(rng.integers(2, k))
        if gi % 5 == 1:
            V = rng.integers(0, 3, (n, k), dtype=np.uint8)
        else:
            V = rng.integers(0, 256, (n, k), dtype=np.uint8)
        if gi % 7 == 3 and n > 17:  # rows 1..16 equal row 0 on the first 16 columns, up to scale
            V[1:17, :16] = oracle.matmul(rng.integers(0, 256, (16, 1), dtype=np.uint8), V[:1, :16])[1]
        rows = np.zeros((n, pitch), np.uint8)
        rows[:, :k], rows[:, k:k + L] = V, oracle.encode(P, V)
        d = gpu_ctx.alloc(rows.nbytes)
        gpu_ctx.h2d(d, rows)
        gens.append((P, V))
        bufs.append(d)
        hosts.append(Dec(gpu_ctx, k))
        gpus.append(Dec(gpu_ctx, k))
    counts = (ctypes.c_size_t * G)(*[V.shape[0] for _, V in gens])
    rows_p = (ctypes.c_void_p * G)(*bufs)
    decs = (ctypes.c_void_p * G)(*[g.h.value for g in gpus])
    consumed = (ctypes.c_size_t * G)()
    status = (ctypes.c_int * G)()
    errors.check(_lib.lib().rlnc_decoders_add_pieces_gpu(decs, G, rows_p, counts, pitch, L, consumed, status))
    for gi in range(G):
        c = ctypes.c_size_t()
        st = _lib.lib().rlnc_decoder_add_pieces(hosts[gi].h, ctypes.c_void_p(bufs[gi]), counts[gi], pitch, L, 1,
                                                ctypes.byref(c))
        assert (status[gi], consumed[gi]) == (st, c.value), gi
        _same(hosts[gi], gpus[gi])
        if hosts[gi].state()[3]:
            s1, a = gpus[gi].get_all()
            assert s1 == 0 and np.array_equal(a, gens[gi][0]), gi
    gpu_ctx.synchronize()
    for d in bufs:
        gpu_ctx.free(d)


def test_gpu_elimination_rejects_a_decoder_listed_twice(gpu_ctx):
    """The batched call loads the decoders' host mirrors concurrently, so a
    handle listed twice is a bad argument, and nothing is consumed."""
    k, L = 32, 64
    rng = np.random.default_rng(11)
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    V = rng.integers(0, 256, (k, k), dtype=np.uint8)
    d, pitch = _rows(gpu_ctx, V, P, L)
    a, b = Dec(gpu_ctx, k), Dec(gpu_ctx, k)
    decs = (ctypes.c_void_p * 3)(a.h.value, b.h.value, a.h.value)
    rows_p = (ctypes.c_void_p * 3)(d, d, d)
    counts = (ctypes.c_size_t * 3)(k, k, k)
    consumed, status = (ctypes.c_size_t * 3)(), (ctypes.c_int * 3)()
    rc = _lib.lib().rlnc_decoders_add_pieces_gpu(decs, 3, rows_p, counts, pitch, L, consumed, status)
    assert rc == -1  # RLNC_ERR_INVALID_ARGUMENT
    assert a.state()[1] == 0 and b.state()[1] == 0
    gpu_ctx.synchronize()
    gpu_ctx.free(d)


def _split(rng, n, k, scheme):
    if scheme == "one_then_rest":
        cuts = [1]
    elif scheme == "halves":
        cuts = [k // 2]
    elif scheme == "quarters":
        cuts = [k // 4, k // 2, 3 * k // 4]
    elif scheme == "random":
        cuts = sorted(set(int(x) for x in rng.integers(1, n, 4)))
    elif scheme == "tail_pair":  # the last batch is 2 rows
        cuts = [n - 2]
    else:
        raise ValueError(scheme)
    b = [0] + [c for c in cuts if 0 < c < n] + [n]
    return [(b[i], b[i + 1]) for i in range(len(b) - 1)]


CONT_KINDS = ["dense", "tiny", "lowrank", "zero_mid", "systematic", "first_zero", "dense", "dense"]
CONT_SCHEMES = ["one_then_rest", "halves", "quarters", "random", "tail_pair", "quarters", "random", "halves"]


@pytest.mark.parametrize("k", [4, 16, 64, 129, 256])
def test_gpu_elimination_continued_batches(gpu_ctx, k):
    """Decoders fed in several batched GPU AddPiece calls (rounds): after the
    first batch a decoder is no longer fresh; a later batch that can complete
    the rank of a decoder whose rows were all kept is eliminated on the GPU
    from M = [its coefficient rows ; the batch's vectors] (DecoderCore::
    load_continued: C^-1 = M^-1 x diag(T_r, I)), other batches on the host.  Each round's status,
    rows consumed, counters, coefficients and transform equal host decoders
    fed the same batches (rlnc_decoder_add_pieces), the final coefficients
    equal the oracle's literal decoder (decoder_state.go:15-182) fed the rows
    one by one, and decoded generations come back byte for byte."""
    rng = np.random.default_rng(1000 + k)
    L = 72
    G = len(CONT_KINDS)
    gens = []
    for gi, kind in enumerate(CONT_KINDS):
        P = rng.integers(0, 256, (k, L), dtype=np.uint8)
        n = k + int(rng.integers(0, 4))
        V = _vectors(rng, kind, n, k)
        gens.append((P, V, _split(rng, n, k, CONT_SCHEMES[gi])))
    pitch = ((k + L + 15) // 16) * 16
    bufs, hosts, gpus = [], [], []
    for P, V, _ in gens:
        rows = np.zeros((V.shape[0], pitch), np.uint8)
        rows[:, :k], rows[:, k:k + L] = V, oracle.encode(P, V)
        d = gpu_ctx.alloc(rows.nbytes)
        gpu_ctx.h2d(d, rows)
        bufs.append(d)
        hosts.append(Dec(gpu_ctx, k))
        gpus.append(Dec(gpu_ctx, k))
    rounds = max(len(sp) for _, _, sp in gens)
    for rd in range(rounds):
        part = [gi for gi in range(G) if rd < len(gens[gi][2])]
        n_ = len(part)
        counts = (ctypes.c_size_t * n_)(*[gens[gi][2][rd][1] - gens[gi][2][rd][0] for gi in part])
        rows_p = (ctypes.c_void_p * n_)(*[bufs[gi] + gens[gi][2][rd][0] * pitch for gi in part])
        decs = (ctypes.c_void_p * n_)(*[gpus[gi].h.value for gi in part])
        consumed = (ctypes.c_size_t * n_)()
        status = (ctypes.c_int * n_)()
        errors.check(_lib.lib().rlnc_decoders_add_pieces_gpu(decs, n_, rows_p, counts, pitch, L, consumed, status))
        for j, gi in enumerate(part):
            c = ctypes.c_size_t()
            st = _lib.lib().rlnc_decoder_add_pieces(hosts[gi].h, ctypes.c_void_p(rows_p[j]), counts[j], pitch, L, 1,
                                                    ctypes.byref(c))
            assert (status[j], consumed[j]) == (st, c.value), (gi, rd)
            _same(hosts[gi], gpus[gi])
    for gi, (P, V, _) in enumerate(gens):
        ref = oracle.Decoder(k)
        C = oracle.encode(P, V)
        for i in range(V.shape[0]):
            if ref.add(V[i], C[i]) != 0:
                break
        assert gpus[gi].state() == (ref.useful(), ref.received(), ref.required(), ref.is_decoded()), gi
        assert np.array_equal(gpus[gi].coefficients(), ref.coeffs()), gi
        if ref.is_decoded():
            st, out = gpus[gi].get_all()
            assert st == 0 and np.array_equal(out, P), gi
    gpu_ctx.synchronize()
    for d in bufs:
        gpu_ctx.free(d)


@pytest.mark.parametrize("kind", ["dense", "systematic", "first_zero", "tiny"])
@pytest.mark.parametrize("k", [128, 200, 256])
def test_routed_single_decoder_vs_oracle(gpu_ctx, monkeypatch, kind, k):
    """rlnc_decoder_add_pieces (device rows) and lazy AddPiece flushes route a
    large decoder's full batch to the multi-workgroup GPU elimination
    (capi_decoder.cpp dec_route_gpu); singular blocks fall back to the host.  Both
    entry points against the oracle's literal decoder: return code, rows
    consumed, counters, coefficients and decoded pieces."""
    gpu_ctx.set_route_min_k(128)
    rng = np.random.default_rng(k * 7 + len(kind))
    L = 64
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    n = k + 3
    V = _vectors(rng, kind, n, k)
    drows, pitch = _rows(gpu_ctx, V, P, L)
    ref = oracle.Decoder(k)
    C = oracle.encode(P, V)
    sts = [ref.add(V[i], C[i]) for i in range(n)]
    exp_n = next((i for i, s_ in enumerate(sts) if s_ != 0), n)
    lib = _lib.lib()
    # batched
    bat = Dec(gpu_ctx, k)
    c = ctypes.c_size_t()
    st = lib.rlnc_decoder_add_pieces(bat.h, ctypes.c_void_p(drows), n, pitch, L, 1, ctypes.byref(c))
    assert (st, c.value) == (sts[exp_n] if exp_n < n else 0, exp_n)
    # one AddPiece call per piece (lazy queue, flushed when it completes the rank)
    pw = Dec(gpu_ctx, k)
    got = []
    for i in range(n):
        v = np.ascontiguousarray(V[i])
        got.append(lib.rlnc_decoder_add_piece_device(pw.h, v.ctypes.data_as(U8P), k, drows + i * pitch + k, L))
    assert got == sts
    for d in (bat, pw):
        assert d.state() == (ref.useful(), ref.received(), ref.required(), ref.is_decoded())
        assert np.array_equal(d.coefficients(), ref.coeffs())
        if ref.is_decoded():
            s1, out = d.get_all()
            assert s1 == 0 and np.array_equal(out, P)
        if kind == "dense" and pr.gf_inverse(V[:k]) is not None:
            s = elim_stats(d.h)  # both entry points took the GPU elimination
            assert s["gpu"] == 1 and s["host_after_gpu"] == 0, s
    gpu_ctx.synchronize()
    gpu_ctx.free(drows)
