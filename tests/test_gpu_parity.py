"""GPU parity: the HIP engine (through the C ABI) vs the golden fixtures and
the CPU oracle, bit-exact.  Sizes the oracle finishes in seconds are compared
byte for byte; the BASELINE.json shapes (32 MiB/256, 16 MiB/128) are compared
in full for a batch of coded pieces and through round trips."""
import ctypes

import numpy as np
import pytest

import oracle
from kodr_amd import _lib, errors
from kodr_amd._codec import FULL, SYSTEMATIC

pytestmark = pytest.mark.gpu
ERR = {None: 0, **{name: cls.code for name, cls in errors.BY_NAME.items()}}
U8P = _lib._u8p


def h(s):
    return np.frombuffer(bytes.fromhex(s), dtype=np.uint8)


def ptr(a):
    return a.ctypes.data_as(U8P)


class Enc:
    def __init__(self, ctx, pieces, kind=FULL):
        P = np.ascontiguousarray(pieces, np.uint8)
        self.k, self.L = P.shape
        self.h = ctypes.c_void_p()
        errors.check(_lib.lib().rlnc_encoder_create(ctx.handle, kind, ptr(P), self.k, self.L,
                                                    ctypes.byref(self.h)))

    def code(self, V):
        V = np.array(V, np.uint8).reshape(-1, self.k)
        out = np.empty((V.shape[0], self.k + self.L), np.uint8)
        errors.check(_lib.lib().rlnc_encoder_coded_pieces(self.h, ptr(V), V.shape[0], ptr(out)))
        return V, out

    def __del__(self):
        _lib.lib().rlnc_encoder_destroy(self.h)


class Dec:
    def __init__(self, ctx, k):
        self.h = ctypes.c_void_p()
        errors.check(_lib.lib().rlnc_decoder_create(ctx.handle, k, ctypes.byref(self.h)))

    def add(self, v, p):
        v = np.ascontiguousarray(v, np.uint8)
        p = np.ascontiguousarray(p, np.uint8)
        return _lib.lib().rlnc_decoder_add_piece(self.h, ptr(v), v.size, ptr(p), p.size)

    def state(self):
        L = _lib.lib()
        return (L.rlnc_decoder_useful(self.h), L.rlnc_decoder_received(self.h),
                L.rlnc_decoder_required(self.h), bool(L.rlnc_decoder_is_decoded(self.h)))

    def get(self, i):
        L = _lib.lib().rlnc_decoder_piece_length(self.h)
        out = np.empty(max(L, 1), np.uint8)
        st = _lib.lib().rlnc_decoder_get_piece(self.h, i, ptr(out))
        return st, out[:L]

    def get_all(self):
        n, L = _lib.lib().rlnc_decoder_useful(self.h), _lib.lib().rlnc_decoder_piece_length(self.h)
        out = np.empty((n, L), np.uint8)
        st = _lib.lib().rlnc_decoder_get_pieces(self.h, ptr(out))
        return st, out

    def __del__(self):
        _lib.lib().rlnc_decoder_destroy(self.h)


def test_encode_golden(gpu_ctx, golden):
    for c in golden["vectors"]["encode"]:
        e = Enc(gpu_ctx, np.stack([h(p) for p in c["pieces"]]))
        V, out = e.code(np.stack([h(v) for v in c["vectors"]]))
        for i, exp in enumerate(c["coded"]):
            assert out[i, :c["k"]].tobytes() == V[i].tobytes()
            assert out[i, c["k"]:].tobytes().hex() == exp, (c["k"], c["L"], i)


def test_recode_golden(gpu_ctx, golden):
    for c in golden["vectors"]["recode"]:
        flat = h(c["flat"])
        rh = ctypes.c_void_p()
        errors.check(_lib.lib().rlnc_recoder_create(gpu_ctx.handle, ptr(flat), flat.size, c["n"], c["k"],
                                                    ctypes.byref(rh)))
        R = np.stack([h(r) for r in c["r"]])
        out = np.empty((R.shape[0], c["k"] + c["L"]), np.uint8)
        errors.check(_lib.lib().rlnc_recoder_coded_pieces(rh, ptr(R), R.shape[0], ptr(out)))
        _lib.lib().rlnc_recoder_destroy(rh)
        assert [o.tobytes().hex() for o in out] == c["out"]


def test_systematic_golden(gpu_ctx, golden):
    for c in golden["vectors"]["systematic"]:
        e = Enc(gpu_ctx, np.stack([h(p) for p in c["pieces"]]), SYSTEMATIC)
        V = np.stack([h(v) for v in c["random_vectors"]])
        # split into two calls to cross the systematic -> coded boundary mid-batch
        _, o1 = e.code(V[:c["k"] - 1])
        _, o2 = e.code(V[c["k"] - 1:])
        got = [r.tobytes().hex() for r in np.concatenate([o1, o2])]
        assert got == c["out"]


def test_decode_golden_traces(gpu_ctx, golden):
    for c in golden["vectors"]["decode"]:
        d = Dec(gpu_ctx, c["k"])
        for (vh, ph), step in zip(c["stream"], c["steps"]):
            assert d.add(h(vh), h(ph)) == ERR[step["err"]], c["name"]
            assert d.state() == (step["useful"], step["received"], step["required"], step["decoded"])
            for idx, (e, p) in enumerate(step.get("get", [])):
                st, got = d.get(idx)
                assert st == ERR[e], (c["name"], idx)
                if p is not None:
                    assert got.tobytes().hex() == p
        if c["decoded"] is not None:
            st, allp = d.get_all()
            assert st == 0
            assert [r.tobytes().hex() for r in allp] == c["decoded"], c["name"]


@pytest.mark.parametrize("M", [1, 2, 3, 4, 5, 8, 9, 16, 17, 40, 256])
@pytest.mark.parametrize("K", [1, 2, 15, 256, 257, 300])
def test_gf_matmul_vs_oracle(gpu_ctx, M, K):
    rng = np.random.default_rng(M * 1000 + K)
    for ncols in (16, 1000, 1024 * 3 + 48, 4096 + 7):
        ld = (ncols + 255) // 256 * 256
        A = rng.integers(0, 256, (M, K), dtype=np.uint8)
        X = np.zeros((K, ld), np.uint8)
        X[:, :ncols] = rng.integers(0, 256, (K, ncols), dtype=np.uint8)
        dA, dX, dY = gpu_ctx.alloc(A.nbytes), gpu_ctx.alloc(X.nbytes), gpu_ctx.alloc(M * ld)
        try:
            gpu_ctx.h2d(dA, A)
            gpu_ctx.h2d(dX, X)
            gpu_ctx.h2d(dY, np.full(M * ld, 0xA5, np.uint8))  # canary beyond ncols
            errors.check(_lib.lib().rlnc_gf_matmul_device(gpu_ctx.handle, dA, K, M, K, dX, ld, dY, ld, ncols))
            Y = gpu_ctx.d2h(dY, M * ld).reshape(M, ld)
        finally:
            for p in (dA, dX, dY):
                gpu_ctx.free(p)
        st, ref = oracle.matmul(A, X[:, :ncols])
        assert np.array_equal(Y[:, :ncols], ref), (M, K, ncols)
        assert (Y[:, ncols:] == 0xA5).all(), "wrote past ncols"


@pytest.mark.parametrize("M,K,ncols", [(1, 32, 262144 + 48), (3, 64, 262144), (8, 100, (1 << 20) + 16),
                                       (5, 17, 300000 + 3), (2, 255, 262144), (8, 16, 65536 + 5),
                                       (20, 24, 262144 + 32), (33, 64, 131072)])
def test_gf_matmul_few_rows_wide_vs_oracle(gpu_ctx, M, K, ncols):
    # the one-wave gf_gemm tiles (choose_gemm_config: K <= 32 always, K <= 64
    # from 128 KiB rows or M >= 4, K <= 128 from 256 KiB rows), split over row
    # tiles, including more than 8 output rows: bit-exact, nothing written
    # past ncols
    rng = np.random.default_rng(M * 7919 + K)
    ld = (ncols + 255) // 256 * 256
    A = rng.integers(0, 256, (M, K), dtype=np.uint8)
    X = np.zeros((K, ld), np.uint8)
    X[:, :ncols] = rng.integers(0, 256, (K, ncols), dtype=np.uint8)
    dA, dX, dY = gpu_ctx.alloc(A.nbytes), gpu_ctx.alloc(X.nbytes), gpu_ctx.alloc(M * ld)
    try:
        gpu_ctx.h2d(dA, A)
        gpu_ctx.h2d(dX, X)
        gpu_ctx.h2d(dY, np.full(M * ld, 0xA5, np.uint8))
        errors.check(_lib.lib().rlnc_gf_matmul_device(gpu_ctx.handle, dA, K, M, K, dX, ld, dY, ld, ncols))
        Y = gpu_ctx.d2h(dY, M * ld).reshape(M, ld)
    finally:
        for p in (dA, dX, dY):
            gpu_ctx.free(p)
    st, ref = oracle.matmul(A, X[:, :ncols])
    assert np.array_equal(Y[:, :ncols], ref), (M, K, ncols)
    assert (Y[:, ncols:] == 0xA5).all(), "wrote past ncols"


@pytest.mark.parametrize("M,K,ncols", [(1, 129, 16384), (1, 200, 65536 + 16), (1, 256, 131072), (1, 256, 131072 + 48),
                                       (1, 255, 40000 + 7), (2, 256, 131072), (2, 130, 16384 + 5), (3, 256, 65536 + 48),
                                       (4, 256, 131072), (4, 177, 40000 + 7)])
def test_gf_gemv_vs_oracle(gpu_ctx, M, K, ncols):
    # a few coded pieces of a wide generation (M = 1..4, 129..256 rows,
    # >= 16 KiB rows): the streaming gf_gemv_kernel / gf_gemv_multi_kernel
    # (plan kernel 3, M <= 2), gf_gemm_kernel for 3-4 rows, bit-exact with zero coefficients, lda > K, ragged
    # columns, nothing written past ncols or past row M
    rng = np.random.default_rng(M * 7 + K * 131 + ncols)
    ld = (ncols + 255) // 256 * 256
    lda = K + 5
    A = np.zeros((M, lda), np.uint8)
    A[:, :K] = rng.integers(0, 256, (M, K), dtype=np.uint8)
    A[:, :K][rng.random((M, K)) < 0.2] = 0
    X = np.zeros((K, ld), np.uint8)
    X[:, :ncols] = rng.integers(0, 256, (K, ncols), dtype=np.uint8)
    dA, dX, dY = gpu_ctx.alloc(A.nbytes), gpu_ctx.alloc(X.nbytes), gpu_ctx.alloc((M + 1) * ld)
    try:
        gpu_ctx.h2d(dA, A)
        gpu_ctx.h2d(dX, X)
        gpu_ctx.h2d(dY, np.full((M + 1) * ld, 0xA5, np.uint8))
        errors.check(_lib.lib().rlnc_gf_matmul_device(gpu_ctx.handle, dA, lda, M, K, dX, ld, dY, ld, ncols))
        plan = _lib.last_launch_plan()
        Y = gpu_ctx.d2h(dY, (M + 1) * ld).reshape(M + 1, ld)
    finally:
        for p in (dA, dX, dY):
            gpu_ctx.free(p)
    assert plan["kernel"] == (3 if M <= 2 else 1), plan   # 3-4 rows: gf_gemm_kernel
    _, ref = oracle.matmul(A[:, :K], X[:, :ncols])
    assert np.array_equal(Y[:M, :ncols], ref), (M, K, ncols)
    assert (Y[:M, ncols:] == 0xA5).all() and (Y[M] == 0xA5).all(), "wrote past ncols or row M"


def test_c2_encode_batch_full_compare(gpu_ctx):
    # BASELINE config 2: 32 MiB / 256 pieces, 8 coded pieces compared in full
    rng = np.random.default_rng(0x6B6F6472)
    k, L = 256, 131072
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    e = Enc(gpu_ctx, P)
    V = rng.integers(0, 256, (8, k), dtype=np.uint8)
    V[1] = 0
    V[2] = 1
    _, out = e.code(V)
    ref = oracle.encode(P, V)
    assert np.array_equal(out[:, k:], ref)
    assert np.array_equal(out[:, :k], V)


def test_c2_device_encode_decode_round_trip(gpu_ctx):
    # BASELINE configs 2+3 device-resident: encode k+2 pieces on the device,
    # feed them to the decoder from device memory, decode, compare originals
    rng = np.random.default_rng(3)
    k, L = 256, 131072
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    e = Enc(gpu_ctx, P)
    n = k + 2
    V = rng.integers(0, 256, (n, k), dtype=np.uint8)
    dV, dOut = gpu_ctx.alloc(V.nbytes), gpu_ctx.alloc(n * L)
    try:
        gpu_ctx.h2d(dV, V)
        errors.check(_lib.lib().rlnc_encoder_coded_pieces_device(e.h, dV, n, dOut, L))
        gpu_ctx.synchronize()
        # spot-check two coded pieces against the oracle
        got = gpu_ctx.d2h(dOut, 2 * L).reshape(2, L)
        assert np.array_equal(got, oracle.encode(P, V[:2]))
        d = Dec(gpu_ctx, k)
        for i in range(n):
            v = np.ascontiguousarray(V[i])
            st = _lib.lib().rlnc_decoder_add_piece_device(d.h, ptr(v), k, dOut + i * L, L)
            if st == ERR["ErrAllUsefulPiecesReceived"]:
                break
            assert st == 0
        assert d.state()[3]
        st, dec = d.get_all()
        assert st == 0 and np.array_equal(dec, P)
    finally:
        gpu_ctx.free(dV)
        gpu_ctx.free(dOut)


def test_c4_systematic_round_trip_with_drops(gpu_ctx):
    # BASELINE config 4: systematic 16 MiB / 128, random 50% piece loss
    rng = np.random.default_rng(4)
    k, L = 128, 131072
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    e = Enc(gpu_ctx, P, SYSTEMATIC)
    d = Dec(gpu_ctx, k)
    sent = n_sys = 0
    while not d.state()[3]:
        V, out = e.code(rng.integers(0, 256, (16, k), dtype=np.uint8))
        for i in range(16):
            sent += 1
            if rng.random() < 0.5:
                continue
            assert bool(_lib.lib().rlnc_is_systematic(ptr(V[i]), k)) == (sent <= k)
            st = d.add(out[i, :k], out[i, k:])
            if st == ERR["ErrAllUsefulPiecesReceived"]:
                break
            n_sys += sent <= k
    st, dec = d.get_all()
    assert st == 0 and np.array_equal(dec, P)
    # systematic fast path: with exactly k pieces received T = C^-1 is unique,
    # so every received systematic piece is a unit row and is copied
    gf_rows, copy_rows = ctypes.c_size_t(), ctypes.c_size_t()
    errors.check(_lib.lib().rlnc_decoder_apply_stats(d.h, ctypes.byref(gf_rows), ctypes.byref(copy_rows)))
    assert gf_rows.value + copy_rows.value == k
    if d.state()[1] == k:
        assert copy_rows.value == n_sys and 0 < n_sys < k


def test_c2_recode_matches_oracle_and_decodes(gpu_ctx):
    # config 5's per-GPU step: recode n = k held pieces of a 32 MiB/256 generation
    rng = np.random.default_rng(5)
    k, L = 256, 131072
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    V = rng.integers(0, 256, (k, k), dtype=np.uint8)
    e = Enc(gpu_ctx, P)
    _, flat = e.code(V)                    # k wire rows
    rh = ctypes.c_void_p()
    errors.check(_lib.lib().rlnc_recoder_create(gpu_ctx.handle, ptr(flat), flat.size, k, k, ctypes.byref(rh)))
    R = rng.integers(0, 256, (k + 2, k), dtype=np.uint8)
    out = np.empty((k + 2, k + L), np.uint8)
    errors.check(_lib.lib().rlnc_recoder_coded_pieces(rh, ptr(R), k + 2, ptr(out)))
    _lib.lib().rlnc_recoder_destroy(rh)
    assert np.array_equal(out[:2], oracle.recode(flat, k, R[:2]))
    d = Dec(gpu_ctx, k)
    for row in out:
        if d.add(row[:k], row[k:]) == ERR["ErrAllUsefulPiecesReceived"]:
            break
    st, dec = d.get_all()
    assert st == 0 and np.array_equal(dec, P)


def test_decode_matches_oracle_with_dependent_and_quirky_pieces(gpu_ctx):
    rng = np.random.default_rng(6)
    for k, L in [(5, 33), (16, 1000), (40, 4096)]:
        P = rng.integers(0, 256, (k, L), dtype=np.uint8)
        d, ref = Dec(gpu_ctx, k), oracle.Decoder(k)
        n = 0
        while not ref.is_decoded() and n < 10 * k:
            n += 1
            v = rng.integers(0, 3, k, dtype=np.uint8)   # many zero / dependent rows
            p = oracle.encode(P, v[None, :])[0] if rng.random() < 0.8 else rng.integers(0, 256, L, dtype=np.uint8)
            assert d.add(v, p) == ref.add(v, p)
            assert d.state() == (ref.useful(), ref.received(), ref.required(), ref.is_decoded())
            for idx in range(k):
                st_r, got_r = ref.get_piece(idx)
                st, got = d.get(idx)
                assert st == st_r
                if st == 0:
                    assert np.array_equal(got, got_r)


def _add_rows(d, rows_ptr, count, pitch, dev, plen=None):
    consumed = ctypes.c_size_t()
    k = _lib.lib().rlnc_decoder_piece_count(d.h)
    plen = pitch - k if plen is None else plen
    st = _lib.lib().rlnc_decoder_add_pieces(d.h, rows_ptr, count, pitch, plen, int(dev), ctypes.byref(consumed))
    return st, consumed.value


def test_batch_add_golden_traces(gpu_ctx, golden):
    """rlnc_decoder_add_pieces over a whole golden stream == AddPiece row by row."""
    for c in golden["vectors"]["decode"]:
        rows = [np.concatenate([h(v), h(p)]) for v, p in c["stream"]]
        if len({r.size for r in rows}) != 1:
            continue
        W = np.stack(rows)
        errs = [s["err"] for s in c["steps"]]
        first_bad = next((i for i, e in enumerate(errs) if e is not None), len(errs))
        for dev in (False, True):
            d = Dec(gpu_ctx, c["k"])
            if dev:
                dW = gpu_ctx.alloc(W.nbytes)
                gpu_ctx.h2d(dW, W)
                st, n = _add_rows(d, ctypes.c_void_p(dW), W.shape[0], W.shape[1], True)
            else:
                st, n = _add_rows(d, ptr(W), W.shape[0], W.shape[1], False)
            assert n == first_bad, c["name"]
            assert st == (ERR[errs[first_bad]] if first_bad < len(errs) else 0), c["name"]
            last = c["steps"][first_bad - 1] if first_bad else None
            if last is not None:
                assert d.state() == (last["useful"], last["received"], last["required"], last["decoded"])
            if c["decoded"] is not None:
                st, allp = d.get_all()
                assert st == 0
                assert [r.tobytes().hex() for r in allp] == c["decoded"], c["name"]
            if dev:
                gpu_ctx.synchronize()
                gpu_ctx.free(dW)


@pytest.mark.parametrize("k,L", [(7, 45), (32, 4096), (64, 1024)])
def test_batch_add_random_batches_vs_oracle(gpu_ctx, k, L):
    """Random batch sizes, host and device rows at a padded pitch, mixed with
    single AddPiece calls; state and pieces bit-exact vs the oracle decoder."""
    rng = np.random.default_rng(k * 1000 + L)
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    d, ref = Dec(gpu_ctx, k), oracle.Decoder(k)
    pitch = ((k + L + 255) // 256) * 256 + 32
    dbuf = gpu_ctx.alloc(pitch * 4 * k)
    it = 0
    while not ref.is_decoded() and it < 50:
        it += 1
        n = int(rng.integers(1, k + 3))
        V = rng.integers(0, 256 if rng.random() < 0.5 else 3, (n, k), dtype=np.uint8)
        C = oracle.encode(P, V)
        rows = np.zeros((n, pitch), np.uint8)
        rows[:, :k], rows[:, k:k + L] = V, C
        mode = it % 3
        if mode == 2:  # piecewise
            for i in range(n):
                assert d.add(V[i], C[i]) == ref.add(V[i], C[i])
            continue
        exp_n, exp_st = 0, 0
        for i in range(n):
            s = ref.add(V[i], C[i])
            if s != 0:
                exp_st = s
                break
            exp_n += 1
        if mode == 1:
            gpu_ctx.h2d(dbuf, rows)
            st, got_n = _add_rows(d, ctypes.c_void_p(dbuf), n, pitch, True, L)
        elif it % 2:  # page-locked rows: the DMA starts before the elimination
            pinned = _page_aligned(rows.shape)
            pinned[:] = rows
            gpu_ctx.register(pinned)
            try:
                st, got_n = _add_rows(d, ptr(pinned), n, pitch, False, L)
            finally:
                gpu_ctx.unregister(pinned)
        else:
            st, got_n = _add_rows(d, ptr(rows), n, pitch, False, L)
        assert (st, got_n) == (exp_st, exp_n)
        assert d.state() == (ref.useful(), ref.received(), ref.required(), ref.is_decoded())
    assert ref.is_decoded()
    st, allp = d.get_all()
    assert st == 0 and np.array_equal(allp, P)
    gpu_ctx.synchronize()
    gpu_ctx.free(dbuf)


def test_batch_add_argument_errors(gpu_ctx):
    k, L = 4, 16
    d = Dec(gpu_ctx, k)
    rows = np.zeros((2, k + L), np.uint8)
    assert _add_rows(d, ptr(rows), 0, k + L, False) == (0, 0)
    assert _add_rows(d, ptr(rows), 2, k + L, False, L + 1)[0] == -1   # pitch < k + piece_len
    assert d.add(np.eye(k, dtype=np.uint8)[0], np.zeros(L, np.uint8)) == 0   # fixes L = 16
    assert _add_rows(d, ptr(rows), 1, k + L, False, L - 1)[0] == -1  # piece length differs
    assert _add_rows(d, ptr(rows), 2, k + L, False) == (0, 2)


def test_rows_wider_than_staging_chunk(gpu_ctx):
    """Pieces longer than the 8 MiB pinned staging chunk take the direct-copy
    path: encode + batched decode round trip through host buffers."""
    rng = np.random.default_rng(11)
    k, L = 3, (9 << 20) + 5
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    e = Enc(gpu_ctx, P)
    V, out = e.code(rng.integers(0, 256, (k + 1, k), dtype=np.uint8))
    assert np.array_equal(out[:, k:], oracle.encode(P, V))
    d = Dec(gpu_ctx, k)
    st, n = _add_rows(d, ptr(out), out.shape[0], out.shape[1], False)
    assert st in (0, 3) and n >= k
    st, allp = d.get_all()
    assert st == 0 and np.array_equal(allp, P)


@pytest.mark.parametrize("k,L,drop", [(8, 77, 0.0), (16, 1000, 0.3), (32, 4099, 0.6), (24, 333, 1.0)])
def test_systematic_fast_path_vs_oracle(gpu_ctx, k, L, drop):
    """Systematic pieces (some dropped) + coded repairs, fed through the
    decoder: per-step state, partial GetPiece and the decoded bytes match the
    oracle; the copy/GF split of the materialization is reported."""
    rng = np.random.default_rng(k + L)
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    e = Enc(gpu_ctx, P, SYSTEMATIC)
    d, ref = Dec(gpu_ctx, k), oracle.Decoder(k)
    V, out = e.code(rng.integers(0, 256, (3 * k, k), dtype=np.uint8))
    keep = [i for i in range(3 * k) if i >= k or rng.random() >= drop]
    n_sys = 0
    for i in keep:
        v, p = out[i, :k], out[i, k:]
        assert d.add(v, p) == ref.add(v, p)
        assert d.state() == (ref.useful(), ref.received(), ref.required(), ref.is_decoded())
        n_sys += i < k
        if ref.is_decoded():
            break
        idx = int(rng.integers(0, k))
        st_r, got_r = ref.get_piece(idx)
        st, got = d.get(idx)
        assert st == st_r and (st != 0 or np.array_equal(got, got_r))
    st, dec = d.get_all()
    assert st == 0 and np.array_equal(dec, P)
    gf_rows, copy_rows = ctypes.c_size_t(), ctypes.c_size_t()
    errors.check(_lib.lib().rlnc_decoder_apply_stats(d.h, ctypes.byref(gf_rows), ctypes.byref(copy_rows)))
    assert gf_rows.value + copy_rows.value == k
    if d.state()[1] == k:
        assert copy_rows.value == n_sys


def _wire_device(ctx, e, count, pitch):
    d = ctx.alloc(count * pitch)
    try:
        errors.check(_lib.lib().rlnc_encoder_coded_wire_device(e.h, count, ctypes.c_void_p(d), pitch))
        return ctx.d2h(d, count * pitch).reshape(count, pitch)
    finally:
        ctx.synchronize()
        ctx.free(d)


@pytest.mark.parametrize("kind", [FULL, SYSTEMATIC])
@pytest.mark.parametrize("k,L,pad", [(16, 1000, 24), (7, 45, 0), (32, 4096, 256)])
def test_coded_wire_device_rng(gpu_ctx, kind, k, L, pad):
    """Device-drawn vectors travel with their pieces: every wire row is
    (v, v x P) bit-exact vs the oracle; systematic encoders emit e_i ++ P_i
    first; reseeding reproduces the stream; the rows decode to P."""
    rng = np.random.default_rng(k * L)
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    pitch = k + L + pad
    e = Enc(gpu_ctx, P, kind)
    errors.check(_lib.lib().rlnc_encoder_seed(e.h, 1234))
    n1, n2 = k // 2 + 1, k + 5
    W = np.concatenate([_wire_device(gpu_ctx, e, n1, pitch), _wire_device(gpu_ctx, e, n2, pitch)])[:, :k + L]
    V, C = W[:, :k], W[:, k:]
    n_sys = k if kind == SYSTEMATIC else 0
    if n_sys:
        assert np.array_equal(V[:n_sys], np.eye(k, dtype=np.uint8))
        assert np.array_equal(C[:n_sys], P)
    assert np.array_equal(C, oracle.encode(P, V))
    coded = V[n_sys:]
    assert len({r.tobytes() for r in coded}) == coded.shape[0]          # fresh vectors per piece
    assert 100 < coded.mean() < 155                                      # uniform bytes
    e2 = Enc(gpu_ctx, P, kind)
    errors.check(_lib.lib().rlnc_encoder_seed(e2.h, 1234))
    W2 = _wire_device(gpu_ctx, e2, n1 + n2, pitch)[:, :k + L]
    assert np.array_equal(W2, W)                                         # reproducible stream
    d = Dec(gpu_ctx, k)
    st, n = _add_rows(d, ptr(np.ascontiguousarray(W)), W.shape[0], k + L, False)
    assert st in (0, 3)
    st, dec = d.get_all()
    assert st == 0 and np.array_equal(dec, P)


def _page_aligned(shape):
    n = int(np.prod(shape))
    npg = (n + 4095) // 4096 * 4096
    buf = np.zeros(npg + 4096, np.uint8)
    off = (-buf.ctypes.data) % 4096
    return buf[off:off + npg][:n].reshape(shape)


def test_registered_host_buffers(gpu_ctx):
    """Page-locked caller buffers take the direct DMA path: same bytes."""
    rng = np.random.default_rng(21)
    k, L = 16, 70001
    P, V = _page_aligned((k, L)), _page_aligned((k + 3, k))
    P[:] = rng.integers(0, 256, (k, L), dtype=np.uint8)
    V[:] = rng.integers(0, 256, (k + 3, k), dtype=np.uint8)
    out = _page_aligned((k + 3, k + L))
    dec = _page_aligned((k, L))
    for a in (P, V, out, dec):
        gpu_ctx.register(a)
    try:
        e = Enc(gpu_ctx, P)
        errors.check(_lib.lib().rlnc_encoder_coded_pieces(e.h, ptr(V), V.shape[0], ptr(out)))
        assert np.array_equal(out[:, k:], oracle.encode(P, V))
        d = Dec(gpu_ctx, k)
        st, n = _add_rows(d, ptr(out), out.shape[0], k + L, False)
        assert st in (0, 3)
        assert _lib.lib().rlnc_decoder_get_pieces(d.h, ptr(dec)) == 0
        assert np.array_equal(dec, P)
    finally:
        for a in (P, V, out, dec):
            gpu_ctx.unregister(a)


def bitslice_np(x):
    """numpy model of the bit-sliced layout (32-byte blocks -> 8 planes)."""
    d = x.reshape(-1, 8, 4).copy().view(np.uint32).reshape(-1, 8)
    for sh, m, di in ((4, 0x0F0F0F0F, 4), (2, 0x33333333, 2), (1, 0x55555555, 1)):
        for q in range(8):
            if q & di:
                continue
            t = ((d[:, q] >> sh) ^ d[:, q + di]) & m
            d[:, q + di] ^= t
            d[:, q] ^= (t << sh).astype(np.uint32)
    return d.view(np.uint8).reshape(x.shape)


def test_bitslice_layout(gpu_ctx):
    rng = np.random.default_rng(31)
    X = rng.integers(0, 256, (7, 640), dtype=np.uint8)
    # plane i of a block holds bit i of its 32 bytes
    blk = np.zeros(32, np.uint8)
    blk[5] = 0x81
    planes = bitslice_np(blk).view(np.uint32)
    assert planes[0] == planes[7] and planes[0] != 0 and not planes[1:7].any()
    dX = gpu_ctx.alloc(X.nbytes)
    try:
        gpu_ctx.h2d(dX, X)
        errors.check(_lib.lib().rlnc_bitslice_device(gpu_ctx.handle, ctypes.c_void_p(dX), 640, 7, 600))
        gpu_ctx.synchronize()
        got = gpu_ctx.d2h(dX, X.nbytes).reshape(7, 640)
        # ncols = 600 covers 19 blocks (608 bytes); the 20th block is untouched
        assert np.array_equal(got[:, :608], bitslice_np(X[:, :608].reshape(7, 19, 32)).reshape(7, 608))
        assert np.array_equal(got[:, 608:], X[:, 608:])
        errors.check(_lib.lib().rlnc_bitslice_device(gpu_ctx.handle, ctypes.c_void_p(dX), 640, 7, 600))
        gpu_ctx.synchronize()
        assert np.array_equal(gpu_ctx.d2h(dX, X.nbytes).reshape(7, 640), X)   # self-inverse
    finally:
        gpu_ctx.free(dX)


@pytest.mark.parametrize("M,K,n", [(1, 1, 32), (8, 8, 2048), (3, 5, 77), (16, 40, 5000), (17, 300, 4096),
                                   (32, 256, 8192), (40, 7, 3000), (64, 256, 6149), (256, 258, 4096),
                                   # shapes whose plan splits K across workgroups
                                   (1, 256, 65536), (8, 256, 131072), (12, 128, 131072 - 96),
                                   (16, 256, 131072)])
def test_gf_matmul_bs_vs_oracle(gpu_ctx, M, K, n):
    """Bit-sliced kernel: bit-exact vs the oracle, with zero coefficients,
    lda > K, ragged columns and a canary row beyond the output."""
    rng = np.random.default_rng(M * 1000 + K + n)
    lda = K + 3
    A = np.zeros((M, lda), np.uint8)
    A[:, :K] = rng.integers(0, 256, (M, K), dtype=np.uint8)
    A[:, :K][rng.random((M, K)) < 0.15] = 0
    X = rng.integers(0, 256, (K, n), dtype=np.uint8)
    ldx = (n + 31) // 32 * 32 + 32
    Xp = np.zeros((K, ldx), np.uint8)
    Xp[:, :n] = X
    ldy = (n + 15) // 16 * 16 + 16
    dA, dX, dY = gpu_ctx.alloc(A.nbytes), gpu_ctx.alloc(Xp.nbytes), gpu_ctx.alloc((M + 1) * ldy)
    try:
        gpu_ctx.h2d(dA, A)
        gpu_ctx.h2d(dX, Xp)
        gpu_ctx.h2d(dY, np.full((M + 1) * ldy, 0xA5, np.uint8))
        L = _lib.lib()
        errors.check(L.rlnc_bitslice_device(gpu_ctx.handle, ctypes.c_void_p(dX), ldx, K, n))
        errors.check(L.rlnc_gf_matmul_bs_device(gpu_ctx.handle, ctypes.c_void_p(dA), lda, M, K, ctypes.c_void_p(dX),
                                                ldx, ctypes.c_void_p(dY), ldy, n))
        gpu_ctx.synchronize()
        Y = gpu_ctx.d2h(dY, (M + 1) * ldy).reshape(M + 1, ldy)
        assert np.array_equal(Y[:M, :n], oracle.encode(X, A[:, :K]))
        assert (Y[:M, n:] == 0xA5).all() and (Y[M] == 0xA5).all()
    finally:
        for p in (dA, dX, dY):
            gpu_ctx.free(p)


def test_device_pool_reuse_across_generations_and_streams(gpu_ctx):
    """Encoders/decoders created one after another (and on two streams) reuse
    pooled device buffers: every generation still decodes bit-exactly, and the
    pool holds the freed buffers until trimmed."""
    import kodr_amd.device as dev
    L_ = _lib.lib()
    other = dev.Context(0)   # a second stream: reuse across streams is event-ordered
    rng = np.random.default_rng(33)
    for it in range(6):
        ctx = gpu_ctx if it % 2 == 0 else other
        k, L = (32, 4096) if it < 3 else (16, 8192 + 32 * it)
        P = rng.integers(0, 256, (k, L), dtype=np.uint8)
        e = Enc(ctx, P)
        V, out = e.code(rng.integers(0, 256, (k + 2, k), dtype=np.uint8))
        assert np.array_equal(out[:, k:], oracle.encode(P, V))
        d = Dec(ctx, k)
        st, n = _add_rows(d, ptr(out), out.shape[0], k + L, False)
        assert st in (0, 3) and n >= k
        st, allp = d.get_all()
        assert st == 0 and np.array_equal(allp, P)
        del e, d
    assert L_.rlnc_device_pool_cached(0) > 0
    errors.check(L_.rlnc_device_pool_trim(0, 0))
    assert L_.rlnc_device_pool_cached(0) == 0
    other.close()


def test_c1_round_trip_vs_oracle(gpu_ctx):
    """BASELINE config 1's shape (1 MiB / 16 pieces) on the engine: every coded
    piece vs the oracle, and the decoder's counters after every AddPiece."""
    rng = np.random.default_rng(0xC1)
    k, L = 16, 65536
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    e = Enc(gpu_ctx, P)
    V, out = e.code(rng.integers(0, 256, (k + 4, k), dtype=np.uint8))
    assert np.array_equal(out[:, k:], oracle.encode(P, V))
    d, ref = Dec(gpu_ctx, k), oracle.Decoder(k)
    for row in out:
        st = d.add(row[:k], row[k:])
        assert st == ref.add(row[:k], row[k:])
        assert d.state() == (ref.useful(), ref.received(), ref.required(), ref.is_decoded())
        if st == ERR["ErrAllUsefulPiecesReceived"]:
            break
    st, dec = d.get_all()
    assert st == 0 and np.array_equal(dec, P)


def test_c5_generations_encode_relay_recode_one_gpu(gpu_ctx):
    """BASELINE config 5 on one GPU: 8 generations of 32 MiB / 256, each encoded
    into device wire rows with device-drawn vectors, handed to the next
    "rank" (a device copy standing in for the RCCL ring shift), recoded there
    from device memory, checked against the oracle and decoded.  Each rank
    sends n = k + 4 pieces: k random vectors over GF(256) are singular with
    probability ~1/255, and the device vector stream is seeded at random."""
    L_ = _lib.lib()
    k, L, G = 256, 131072, 8
    n = k + 4
    clen = k + L
    pitch = (clen + 255) // 256 * 256
    rng = np.random.default_rng(0xC5)
    gens = [rng.integers(0, 256, (k, L), dtype=np.uint8) for _ in range(G)]
    encs = [Enc(gpu_ctx, P) for P in gens]
    wire = [gpu_ctx.alloc(n * pitch) for _ in range(G)]
    recv, out = gpu_ctx.alloc(n * pitch), gpu_ctx.alloc((k + 2) * pitch)
    R = rng.integers(0, 256, (k + 2, n), dtype=np.uint8)
    dR = gpu_ctx.alloc(R.nbytes)
    gpu_ctx.h2d(dR, R)
    try:
        for g in range(G):
            errors.check(L_.rlnc_encoder_coded_wire_device(encs[g].h, n, wire[g], pitch))
        for g in range(G):
            src = (g - 1) % G                     # rank g receives rank g-1's pieces
            errors.check(L_.rlnc_memcpy_d2d_async(gpu_ctx.handle, recv, wire[src], n * pitch))
            rh = ctypes.c_void_p()
            errors.check(L_.rlnc_recoder_create_device(gpu_ctx.handle, recv, n, clen, pitch, k, ctypes.byref(rh)))
            errors.check(L_.rlnc_recoder_coded_pieces_device(rh, dR, k + 2, out, pitch))
            gpu_ctx.synchronize()
            L_.rlnc_recoder_destroy(rh)
            rows = np.ascontiguousarray(gpu_ctx.d2h(out, (k + 2) * pitch).reshape(k + 2, pitch)[:, :clen])
            held = np.ascontiguousarray(gpu_ctx.d2h(recv, n * pitch).reshape(n, pitch)[:, :clen])
            assert np.array_equal(held[:, k:], oracle.encode(gens[src], held[:, :k]))
            assert np.array_equal(rows[:2], oracle.recode(held, k, R[:2]))
            # every row's vector and first data block (column separability)
            assert np.array_equal(rows[:, :k + 64], oracle.recode(np.ascontiguousarray(held[:, :k + 64]), k, R)), g
            d = Dec(gpu_ctx, k)
            st, used = _add_rows(d, ptr(rows), k + 2, clen, False)
            assert st in (0, 3) and used >= k
            st, dec = d.get_all()
            assert st == 0 and np.array_equal(dec, gens[src]), g
    finally:
        gpu_ctx.synchronize()
        for p in wire + [recv, out, dR]:
            gpu_ctx.free(p)


def test_contexts_on_threads_run_concurrently(gpu_ctx):
    """Three host threads, each with its own context (stream), encode and
    decode different generations at the same time through the C ABI (ctypes
    releases the GIL): every result bit-exact vs the oracle."""
    import threading

    import kodr_amd.device as dev
    errs = []

    def worker(seed):
        try:
            ctx = dev.Context(0)
            rng = np.random.default_rng(seed)
            for it in range(4):
                k, L = 64, 32768 + 32 * seed
                P = rng.integers(0, 256, (k, L), dtype=np.uint8)
                e = Enc(ctx, P)
                V, out = e.code(rng.integers(0, 256, (k + 1, k), dtype=np.uint8))
                if not np.array_equal(out[:3, k:], oracle.encode(P, V[:3])):
                    errs.append(("encode", seed, it))
                d = Dec(ctx, k)
                st, n = _add_rows(d, ptr(out), out.shape[0], k + L, False)
                st, dec = d.get_all()
                if st != 0 or not np.array_equal(dec, P):
                    errs.append(("decode", seed, it))
                del e, d
            ctx.close()
        except Exception as ex:  # reported below, in the main thread
            errs.append(repr(ex))

    ts = [threading.Thread(target=worker, args=(s,)) for s in (1, 2, 3)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(120)
    assert not any(t.is_alive() for t in ts)
    assert not errs, errs


@pytest.mark.parametrize("k,lost,bs", [(128, 12, True), (256, 12, False), (256, 20, True), (64, 5, False)])
def test_decoder_kernel_choice_and_result(gpu_ctx, k, lost, bs):
    """Systematic decode with `lost` pieces replaced by coded ones: the GF
    rows run on the bit-sliced kernel from 16 rows, or from 9 rows when the
    twin to build is at most 16 MiB (capi_decoder.cpp dec_gemm); bytes equal P
    either way."""
    L = 131072
    rng = np.random.default_rng(k + lost)
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    e = Enc(gpu_ctx, P, SYSTEMATIC)
    errors.check(_lib.lib().rlnc_encoder_seed(e.h, 9))
    W = _wire_device(gpu_ctx, e, k + lost + 4, k + L)
    drop = set(rng.choice(k, lost, replace=False).tolist())
    rows = np.ascontiguousarray(W[[i for i in range(k) if i not in drop] + list(range(k, W.shape[0]))])
    d = Dec(gpu_ctx, k)
    st, used = _add_rows(d, ptr(rows), rows.shape[0], k + L, False)
    assert st in (0, 3) and used >= k
    st, dec = d.get_all()
    assert st == 0 and np.array_equal(dec, P)
    gf_rows, copy_rows = ctypes.c_size_t(), ctypes.c_size_t()
    errors.check(_lib.lib().rlnc_decoder_apply_stats(d.h, ctypes.byref(gf_rows), ctypes.byref(copy_rows)))
    assert (gf_rows.value, copy_rows.value) == (lost, k - lost)
    assert bool(_lib.lib().rlnc_decoder_last_apply_bitsliced(d.h)) == bs


@pytest.mark.parametrize("count", [255, 256, 257])
def test_host_vectors_across_small_upload_limit(gpu_ctx, count):
    """count x k coefficient bytes around the 64 KiB limit where staging
    switches from the upload kernel to a DMA copy (staging.hpp): the coded
    pieces match the oracle on both sides, and a device batch decode whose
    vectors come back through the small-download kernel decodes."""
    k, L = 256, 96
    rng = np.random.default_rng(count)
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    e = Enc(gpu_ctx, P)
    V, out = e.code(rng.integers(0, 256, (count, k), dtype=np.uint8))
    assert np.array_equal(out[:, :k], V)
    assert np.array_equal(out[:, k:], oracle.encode(P, V))
    rows = np.ascontiguousarray(out)
    d_rows = gpu_ctx.alloc(rows.nbytes)
    try:
        gpu_ctx.h2d(d_rows, rows)
        d = Dec(gpu_ctx, k)
        st, used = _add_rows(d, ctypes.c_void_p(d_rows), count, k + L, True)
        ref = oracle.Decoder(k)
        for r in rows[:used]:
            ref.add(r[:k], r[k:])
        assert d.state() == (ref.useful(), ref.received(), ref.required(), ref.is_decoded())
    finally:
        gpu_ctx.synchronize()
        gpu_ctx.free(d_rows)


@pytest.mark.parametrize("dev", [True, False])
def test_batch_add_many_dependent_rows_past_the_precopy(gpu_ctx, dev):
    """A batch whose accepted rows exceed what AddPieces copies ahead of the
    elimination (required + 16): 40 rows spanning only 8 dimensions come
    first, then independent ones; the late rows are copied after the
    elimination and the decode still equals P (capi_decoder.cpp rlnc_decoder_add_pieces)."""
    k, L = 16, 4096
    rng = np.random.default_rng(77 + dev)
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    base = rng.integers(0, 256, (8, k), dtype=np.uint8)
    V = np.concatenate([oracle.matmul(rng.integers(0, 256, (40, 8), dtype=np.uint8), base)[1],
                        rng.integers(0, 256, (k + 4, k), dtype=np.uint8)])
    rows = np.ascontiguousarray(np.concatenate([V, oracle.encode(P, V)], axis=1))
    d, ref = Dec(gpu_ctx, k), oracle.Decoder(k)
    if dev:
        d_rows = gpu_ctx.alloc(rows.nbytes)
        gpu_ctx.h2d(d_rows, rows)
        st, used = _add_rows(d, ctypes.c_void_p(d_rows), rows.shape[0], k + L, True)
    else:
        hb = _page_aligned(rows.shape)
        hb[:] = rows
        gpu_ctx.register(hb)
        st, used = _add_rows(d, ptr(hb), rows.shape[0], k + L, False)
    try:
        for r in rows[:used]:
            ref.add(r[:k], r[k:])
        assert used > 40 and st in (0, 3)
        assert d.state() == (ref.useful(), ref.received(), ref.required(), ref.is_decoded())
        st, dec = d.get_all()
        assert st == 0 and np.array_equal(dec, P)
    finally:
        gpu_ctx.synchronize()
        if dev:
            gpu_ctx.free(d_rows)
        else:
            gpu_ctx.unregister(hb)


def test_generation_past_4_gib(gpu_ctx):
    # A 5 GiB generation (40 pieces of 128 MiB): past the kernels' 32-bit
    # buffer offsets, so gf_gemm (B = 1) runs it in 3 row chunks and gf_bs
    # (B >= 9, decode) in 2, with the partial products XORed together
    # (capi_internal.hpp gemm_k_chunked).  Column windows at the start, the middle
    # (unaligned) and the ragged end are checked against the oracle; the
    # round trip through the decoder is checked on the same windows.
    L_ = _lib.lib()
    k, L = 40, 128 << 20
    rng = np.random.default_rng(11)
    wins = [(0, 4096), (L // 2 + 96, 4096), (L - 4000, 4000)]
    keep = {o: np.empty((k, w), np.uint8) for o, w in wins}
    dP = gpu_ctx.alloc(k * L)
    eh = ctypes.c_void_p()
    try:
        for r in range(k):
            row = np.frombuffer(rng.bytes(L), np.uint8)
            gpu_ctx.h2d(dP + r * L, row)
            for o, w in wins:
                keep[o][r] = row[o:o + w]
        del row
        errors.check(L_.rlnc_encoder_create_device(gpu_ctx.handle, FULL, dP, k, L, L, ctypes.byref(eh)))
    finally:
        gpu_ctx.free(dP)
    n = k + 8
    V = rng.integers(0, 256, (n, k), dtype=np.uint8)
    dV, dOut, dDec = gpu_ctx.alloc(V.nbytes), gpu_ctx.alloc(n * L), gpu_ctx.alloc(k * L)
    dh = ctypes.c_void_p()
    try:
        gpu_ctx.h2d(dV, V)
        # B = 1 (gf_gemm, row-chunked), then the rest in one call (gf_bs, row-chunked)
        errors.check(L_.rlnc_encoder_coded_pieces_device(eh, dV, 1, dOut, L))
        errors.check(L_.rlnc_encoder_coded_pieces_device(eh, dV + k, n - 1, dOut + L, L))
        gpu_ctx.synchronize()
        for o, w in wins:
            ref = oracle.encode(keep[o], V)
            for i in list(range(0, n, 5)) + [n - 1]:
                got = gpu_ctx.d2h(dOut + i * L + o, w)
                assert np.array_equal(got, ref[i]), f"coded piece {i}, columns [{o}, {o + w})"
        errors.check(L_.rlnc_decoder_create(gpu_ctx.handle, k, ctypes.byref(dh)))
        for i in range(n):
            v = np.ascontiguousarray(V[i])
            st = L_.rlnc_decoder_add_piece_device(dh, ptr(v), k, dOut + i * L, L)
            if st == ERR["ErrAllUsefulPiecesReceived"]:
                break
            assert st == 0
        assert L_.rlnc_decoder_is_decoded(dh)
        errors.check(L_.rlnc_decoder_get_pieces_device(dh, dDec, L))
        gpu_ctx.synchronize()
        for o, w in wins:
            for r in range(k):
                assert np.array_equal(gpu_ctx.d2h(dDec + r * L + o, w), keep[o][r]), f"decoded piece {r}"
    finally:
        if dh.value:
            L_.rlnc_decoder_destroy(dh)
        L_.rlnc_encoder_destroy(eh)
        for p in (dV, dOut, dDec):
            gpu_ctx.free(p)
        L_.rlnc_device_pool_trim(0, 0)
