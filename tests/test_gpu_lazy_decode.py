"""GPU parity of lazy AddPiece (capi_decoder.cpp dec_add): coding vectors that cannot
complete the rank are queued and eliminated as one batch when the state is
next observed, and device pieces are copied by one gather at the next data
flush (the opt-in borrowed entry point; the default one copies each piece in
the call, so the caller may reuse its buffer at once).  kodr's AddPiece (full/decoder.go:50-66, decoder_state.go:15-182) is
the reference: every call's return code, the counters whenever they are read,
the coefficient state and the decoded bytes equal the oracle's
(oracle/kodr_oracle.c, the literal restatement), for streams with dependent,
zero and systematic rows, misaligned and host pieces mixed in, reads in the
middle of the stream and a generation larger than the gather's queue.
"""
import ctypes

import numpy as np
import pytest

import oracle
from kodr_amd import _lib, errors

pytestmark = pytest.mark.gpu
U8P = _lib._u8p


def stream(rng, P, n, kind):
    k, L = P.shape
    V = rng.integers(0, 256, (n, k), dtype=np.uint8)
    if kind == "quirky":
        V[0] = 0                       # first piece all-zero: kodr still counts it
        V[3] = V[2]                    # duplicate: dependent
        V[5] = 0
        V[5, 1] = 7                    # scaled unit rows
        V[6] = 0
        V[6, 4] = 1
        V[9] = V[1] ^ V[1]             # zero row
    elif kind == "systematic":
        m = min(n, k)
        V[:m] = 0
        V[np.arange(m), np.arange(m)] = 1
        V[2] = 0                       # a lost systematic piece replaced by a coded one
        V[2] = rng.integers(0, 256, k, dtype=np.uint8)
    return V, oracle.encode(P, V)


def run(ctx, P, V, C, place, reads=(), check_every=False, oracle_cols=None):
    """Feed (V, C) piece by piece; place(i) -> 'dev' (borrowed), 'dev_copy'
    (rlnc_decoder_add_piece_device: copied in the call), 'dev_misaligned' or
    'host'.
    reads: indices after which useful()/required() and a GetPiece are read.
    oracle_cols: feed the oracle only that many bytes of each piece (its
    coefficient side, all that return codes and counters depend on; the
    decoded bytes are then checked against P alone)."""
    lib = _lib.lib()
    k, L = P.shape
    n = V.shape[0]
    pitch = (L + 15) // 16 * 16 + 16
    dbuf = ctx.alloc(n * pitch + 64)
    host = np.zeros((n, pitch + 1), np.uint8)
    for i in range(n):
        host[i, :L] = C[i]
    stage = np.zeros(n * pitch + 64, np.uint8)
    for i in range(n):
        off = i * pitch + (1 if place(i) == "dev_misaligned" else 0)
        stage[off:off + L] = C[i]
    ctx.h2d(dbuf, stage)
    dh = ctypes.c_void_p()
    errors.check(lib.rlnc_decoder_create(ctx.handle, k, ctypes.byref(dh)))
    od = oracle.Decoder(k)
    try:
        for i in range(n):
            v = np.ascontiguousarray(V[i])
            pl = place(i)
            if pl == "host":
                st = lib.rlnc_decoder_add_piece(dh, v.ctypes.data_as(U8P), k, host[i].ctypes.data_as(U8P), L)
            else:
                off = i * pitch + (1 if pl == "dev_misaligned" else 0)
                add = lib.rlnc_decoder_add_piece_device if pl == "dev_copy" else lib.rlnc_decoder_add_piece_device_borrowed
                st = add(dh, v.ctypes.data_as(U8P), k, dbuf + off, L)
            ost = od.add(V[i], C[i] if oracle_cols is None else C[i][:oracle_cols])
            assert st == ost, (i, st, ost)
            if check_every or i in reads:
                assert lib.rlnc_decoder_useful(dh) == od.useful(), i
                assert lib.rlnc_decoder_required(dh) == od.required(), i
                assert bool(lib.rlnc_decoder_is_decoded(dh)) == od.is_decoded(), i
            if i in reads:
                out = np.empty(L, np.uint8)
                for idx in (0, 1):
                    st_g = lib.rlnc_decoder_get_piece(dh, idx, out.ctypes.data_as(U8P))
                    ost_g, ref = od.get_piece(idx)
                    assert st_g == ost_g, (i, idx)
                    if st_g == 0:
                        assert np.array_equal(out, ref), (i, idx)
            assert lib.rlnc_decoder_received(dh) == od.received(), i
        assert lib.rlnc_decoder_useful(dh) == od.useful()
        coeffs = np.empty((od.useful(), k), np.uint8)
        errors.check(lib.rlnc_decoder_coefficients(dh, coeffs.ctypes.data_as(U8P)))
        assert np.array_equal(coeffs, od.coeffs())
        if od.is_decoded():
            out = np.empty((k, L), np.uint8)
            # the caller may reuse its device buffer once GetPieces has returned
            errors.check(lib.rlnc_decoder_get_pieces(dh, out.ctypes.data_as(U8P)))
            ctx.h2d(dbuf, np.full(n * pitch + 64, 0x5A, np.uint8))
            out2 = np.empty((k, L), np.uint8)
            errors.check(lib.rlnc_decoder_get_pieces(dh, out2.ctypes.data_as(U8P)))
            assert np.array_equal(out, P) and np.array_equal(out2, P)
    finally:
        lib.rlnc_decoder_destroy(dh)
        ctx.free(dbuf)


@pytest.mark.parametrize("kind", ["coded", "quirky", "systematic"])
@pytest.mark.parametrize("k,L", [(16, 1024), (64, 4096 + 48), (256, 2048)])
def test_lazy_device_pieces_vs_oracle(gpu_ctx, kind, k, L):
    rng = np.random.default_rng(k * 7 + L + len(kind))
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    V, C = stream(rng, P, k + 6, kind)
    run(gpu_ctx, P, V, C, lambda i: "dev")


def test_lazy_mixed_placement_and_reads(gpu_ctx):
    # device, misaligned device (copied at once) and host pieces interleaved;
    # counters and a partial GetPiece read in the middle (each read flushes)
    rng = np.random.default_rng(0x1A2)
    k, L = 48, 3000
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    V, C = stream(rng, P, k + 5, "quirky")
    kinds = ["dev", "dev", "dev_misaligned", "host", "dev", "dev_copy"]
    run(gpu_ctx, P, V, C, lambda i: kinds[i % len(kinds)], reads=(4, 20, 47, 50))


@pytest.mark.parametrize("k,L", [(16, 1024), (64, 4096)])
def test_default_device_add_copies_in_call(gpu_ctx, k, L):
    # rlnc_decoder_add_piece_device copies the piece in the call: ONE receive
    # slot (as an RCCL receive buffer) is overwritten by the next piece, and
    # finally by garbage, right after each call, on the context stream
    lib = _lib.lib()
    rng = np.random.default_rng(0xD0 + k)
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    V, C = stream(rng, P, k + 3, "quirky")
    slot = gpu_ctx.alloc(L)
    dh = ctypes.c_void_p()
    errors.check(lib.rlnc_decoder_create(gpu_ctx.handle, k, ctypes.byref(dh)))
    od = oracle.Decoder(k)
    try:
        for i in range(V.shape[0]):
            gpu_ctx.h2d(slot, C[i])
            v = np.ascontiguousarray(V[i])
            st = lib.rlnc_decoder_add_piece_device(dh, v.ctypes.data_as(U8P), k, slot, L)
            gpu_ctx.h2d(slot, np.full(L, 0xA5, np.uint8))
            assert st == od.add(V[i], C[i]), i
        assert lib.rlnc_decoder_is_decoded(dh)
        out = np.empty((k, L), np.uint8)
        errors.check(lib.rlnc_decoder_get_pieces(dh, out.ctypes.data_as(U8P)))
        assert np.array_equal(out, P)
    finally:
        lib.rlnc_decoder_destroy(dh)
        gpu_ctx.free(slot)


def test_lazy_counters_every_call(gpu_ctx):
    # reading the counters after every AddPiece observes kodr's state each time
    rng = np.random.default_rng(0x77)
    k, L = 32, 512
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    V, C = stream(rng, P, k + 3, "quirky")
    run(gpu_ctx, P, V, C, lambda i: "dev", check_every=True)


def test_lazy_queue_past_gather_limit(gpu_ctx):
    # k = 1100: more queued device pieces than one gather takes (capi_decoder.cpp
    # kPendMax = 1024), short pieces
    rng = np.random.default_rng(0x44C)
    k, L = 1100, 64
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    V, C = stream(rng, P, k + 2, "coded")
    run(gpu_ctx, P, V, C, lambda i: "dev", oracle_cols=1)


def test_lazy_c2_piecewise(gpu_ctx):
    # BASELINE configs[2] fed one AddPiece call per device piece (the bench's
    # piecewise leg): k + 2 rows, kodr's return codes, the decoded generation
    rng = np.random.default_rng(0xC2)
    k, L = 256, 131072
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    V, C = stream(rng, P, k + 2, "coded")
    run(gpu_ctx, P, V, C, lambda i: "dev", oracle_cols=1)


def _feed(lib, dh, V, dbuf, pitch, idx):
    st = []
    for i in idx:
        v = np.ascontiguousarray(V[i])
        st.append(lib.rlnc_decoder_add_piece_device_borrowed(dh, v.ctypes.data_as(U8P), V.shape[1],
                                                             dbuf + i * pitch, pitch))
    return st


@pytest.mark.parametrize("k,L", [(16, 1024), (64, 4096), (256, 2048)])
def test_grouped_flush_gpu_vs_host_flush(gpu_ctx, k, L):
    """rlnc_decoders_flush_gpu: decoders fed one AddPiece per device piece
    (lazy queues) are flushed together -- the queues that complete the rank
    from kept rows on the GPU (fresh, or continued after a mid-stream read),
    the others on the host -- and end exactly as twins whose own state reads
    flush them on the host: counters, coefficients, transform, every later
    AddPiece's return code and the decoded bytes; the coefficients also equal
    the oracle's (decoder_state.go:15-182) fed the same pieces."""
    lib = _lib.lib()
    rng = np.random.default_rng(k + L)
    # (stream kind, pieces fed, index of a mid-stream read or None)
    plans = [("coded", k, None), ("coded", k, k // 3), ("quirky", k + 2, None), ("systematic", k, None),
             ("coded", k - 3, None), ("dup", k + 1, k // 2), ("coded", k, 1), ("systematic", k, k // 2)]
    pitch = L
    gens, dec_g, dec_h, bufs = [], [], [], []
    for kind, n, rd in plans:
        P = rng.integers(0, 256, (k, L), dtype=np.uint8)
        V, C = stream(rng, P, n, "coded" if kind == "dup" else kind)
        if kind == "dup":  # a dependent piece before the read: not every row kept
            V[rd - 1] = V[rd - 2]
            C = oracle.encode(P, V)
        d = gpu_ctx.alloc(n * pitch)
        gpu_ctx.h2d(d, np.ascontiguousarray(C))
        hs = []
        for _ in range(2):
            h = ctypes.c_void_p()
            errors.check(lib.rlnc_decoder_create(gpu_ctx.handle, k, ctypes.byref(h)))
            hs.append(h)
        gens.append((P, V, C, n, rd))
        dec_g.append(hs[0])
        dec_h.append(hs[1])
        bufs.append(d)
    try:
        for gi, (P, V, C, n, rd) in enumerate(gens):
            for dh in (dec_g[gi], dec_h[gi]):
                if rd is None:
                    st = _feed(lib, dh, V, bufs[gi], pitch, range(n))
                else:
                    st = _feed(lib, dh, V, bufs[gi], pitch, range(rd))
                    lib.rlnc_decoder_useful(dh)  # a state read: the queue so far is eliminated (host)
                    st += _feed(lib, dh, V, bufs[gi], pitch, range(rd, n))
                od = oracle.Decoder(k)
                assert st == [od.add(V[i], C[i]) for i in range(n)], gi
        arr = (ctypes.c_void_p * len(gens))(*[h.value for h in dec_g])
        errors.check(lib.rlnc_decoders_flush_gpu(arr, len(gens)))
        for gi, (P, V, C, n, rd) in enumerate(gens):
            a, b = dec_g[gi], dec_h[gi]
            state = [(lib.rlnc_decoder_useful(h), lib.rlnc_decoder_received(h), lib.rlnc_decoder_required(h),
                      bool(lib.rlnc_decoder_is_decoded(h))) for h in (a, b)]
            assert state[0] == state[1], gi
            u, r = state[0][0], state[0][1]
            mats = []
            for h in (a, b):
                cf = np.empty((u, k), np.uint8)
                tf = np.empty((u, r), np.uint8)
                errors.check(lib.rlnc_decoder_coefficients(h, cf.ctypes.data_as(U8P)))
                errors.check(lib.rlnc_decoder_transform(h, tf.ctypes.data_as(U8P)))
                mats.append((cf, tf))
            assert np.array_equal(mats[0][0], mats[1][0]) and np.array_equal(mats[0][1], mats[1][1]), gi
            od = oracle.Decoder(k)
            for i in range(n):
                od.add(V[i], C[i])
            assert np.array_equal(mats[0][0], od.coeffs()), gi
            extra = rng.integers(0, 256, k, dtype=np.uint8)
            piece = oracle.encode(P, extra[None, :])[0]
            sts = [lib.rlnc_decoder_add_piece(h, extra.ctypes.data_as(U8P), k, piece.ctypes.data_as(U8P), L)
                   for h in (a, b)]
            assert sts[0] == sts[1] == od.add(extra, piece), gi
            if od.is_decoded():
                out = np.empty((k, L), np.uint8)
                errors.check(lib.rlnc_decoder_get_pieces(a, out.ctypes.data_as(U8P)))
                assert np.array_equal(out, P), gi
    finally:
        for h in dec_g + dec_h:
            lib.rlnc_decoder_destroy(h)
        for d in bufs:
            gpu_ctx.free(d)


def test_grouped_flush_more_decoders_than_one_launch(gpu_ctx):
    """70 decoders (more than the elimination's 64 generations per launch):
    two launches, every queue eliminated and every piece gathered."""
    lib = _lib.lib()
    rng = np.random.default_rng(70)
    k, L, G = 8, 64, 70
    Ps = [rng.integers(0, 256, (k, L), dtype=np.uint8) for _ in range(G)]
    Vs = []
    for _ in range(G):
        while True:  # an invertible coding matrix, so every queue completes the rank
            V = rng.integers(0, 256, (k, k), dtype=np.uint8)
            od = oracle.Decoder(k)
            if all(od.add(V[i], np.zeros(1, np.uint8)) == 0 for i in range(k)) and od.is_decoded():
                break
        Vs.append(V)
    rows = np.concatenate([oracle.encode(P, V) for P, V in zip(Ps, Vs)])
    d = gpu_ctx.alloc(rows.nbytes)
    gpu_ctx.h2d(d, np.ascontiguousarray(rows))
    hs = []
    try:
        for g in range(G):
            h = ctypes.c_void_p()
            errors.check(lib.rlnc_decoder_create(gpu_ctx.handle, k, ctypes.byref(h)))
            hs.append(h)
            assert _feed(lib, h, Vs[g], d + g * k * L, L, range(k)) == [0] * k
        errors.check(lib.rlnc_decoders_flush_gpu((ctypes.c_void_p * G)(*[h.value for h in hs]), G))
        for g, h in enumerate(hs):
            assert lib.rlnc_decoder_is_decoded(h)
            out = np.empty((k, L), np.uint8)
            errors.check(lib.rlnc_decoder_get_pieces(h, out.ctypes.data_as(U8P)))
            assert np.array_equal(out, Ps[g]), g
    finally:
        for h in hs:
            lib.rlnc_decoder_destroy(h)
        gpu_ctx.free(d)
