"""GPU parity of the exact launches bench.py times, byte for byte against the
CPU oracle (oracle/kodr_oracle.c, a restatement of full/encoder.go:61-71 and
full/recoder.go:27-46):

- the headline: B coded pieces of a prepared 32 MiB/256 generation through
  rlnc_encoder_coded_pieces_device (B = 32 is the bench's step; 64 and 256 are
  the sweep's), every byte of every piece;
- the grouped multi-generation launch (rlnc_encoder_group_coded_pieces_device,
  the north-star leg): every generation's pieces, small shapes, more than one
  launch's worth of generations, the grouped bit-sliced launch (count >= 9),
  C2-sized generations;
- a prepared recoder at C2 (the bench's recode leg).
"""
import ctypes
import os

import numpy as np
import pytest

import oracle
from kodr_amd import _lib, errors

pytestmark = pytest.mark.gpu
U8P = _lib._u8p


def ptr(a):
    return a.ctypes.data_as(U8P)


def make_encoder(ctx, P, prepare=True):
    h = ctypes.c_void_p()
    k, L = P.shape
    errors.check(_lib.lib().rlnc_encoder_create(ctx.handle, 0, ptr(np.ascontiguousarray(P)), k, L,
                                                ctypes.byref(h)))
    if prepare:
        errors.check(_lib.lib().rlnc_encoder_prepare(h))
    return h


@pytest.fixture(scope="module")
def c2_generation():
    rng = np.random.default_rng(0x5EED32)
    return rng.integers(0, 256, (256, 131072), dtype=np.uint8)


@pytest.mark.parametrize("B", [32, 64, 256])
def test_headline_launch_full_compare(gpu_ctx, c2_generation, B):
    # bench.py's step: device vectors -> B pieces at pitch L, bit-sliced kernel
    P = c2_generation
    k, L = P.shape
    rng = np.random.default_rng(B)
    V = rng.integers(0, 256, (B, k), dtype=np.uint8)
    V[0] = 0                     # the zero vector codes the zero piece
    V[1] = 0
    V[1, 7] = 1                  # a unit vector codes piece 7 itself
    e = make_encoder(gpu_ctx, P)
    dV, dO = gpu_ctx.alloc(V.nbytes), gpu_ctx.alloc(B * L + 64)
    try:
        gpu_ctx.h2d(dV, V)
        gpu_ctx.h2d(dO + B * L, np.full(64, 0xA5, np.uint8))   # canary past the last piece
        errors.check(_lib.lib().rlnc_encoder_coded_pieces_device(e, dV, B, dO, L))
        gpu_ctx.synchronize()
        got = gpu_ctx.d2h(dO, B * L + 64)
    finally:
        gpu_ctx.free(dV)
        gpu_ctx.free(dO)
        _lib.lib().rlnc_encoder_destroy(e)
    ref = oracle.encode(P, V)
    assert np.array_equal(got[:B * L].reshape(B, L), ref)
    assert (got[B * L:] == 0xA5).all()
    assert not ref[0].any() and np.array_equal(ref[1], P[7])


# the launch bench.py times: the direct variant, one wave per workgroup
# running all 256 rows (KODR_BS_DIRECT=0, A/B runs only: the folded KW = 4 plan)
HEADLINE_PLAN = ({"kernel": 2, "tile_rows": 8, "waves": 4, "lane_groups": 1, "ring": 2, "rows_per_wave": 64,
                  "generations": 16, "workgroups": 256}
                 if os.environ.get("KODR_BS_DIRECT") == "0" else
                 {"kernel": 2, "tile_rows": 8, "waves": 1, "lane_groups": 1, "ring": 2, "rows_per_wave": 256,
                  "generations": 16, "workgroups": 256})


def test_bench_headline_step_exact(gpu_ctx):
    # The bench's timed step itself (bench.HeadlineStep, the object bench.py
    # times): 16 prepared 32 MiB/256 generations x B = 32 coded pieces in one
    # grouped call.  The launch must be the instance the bench reports
    # (HEADLINE_PLAN: gf_bs_kernel, the direct variant with one wave per
    # workgroup, the two-row ring, 256 rows per wave, 16 generations), and
    # every one of the 512 pieces must equal the oracle's encode
    # (full/encoder.go:61-71).
    import bench
    hs = bench.HeadlineStep(gpu_ctx, _lib.lib(), errors, 256, 131072, 32, 16, grouped=True,
                            rng=np.random.default_rng(0xBE7C), nvec=2, keep_data=True)
    try:
        hs.step(1)
        plan = _lib.last_launch_plan()
        gpu_ctx.synchronize()
        got = gpu_ctx.d2h(hs.dOut, 16 * 32 * 131072).reshape(16, 32, 131072)
    finally:
        hs.close()
    assert plan == HEADLINE_PLAN, plan
    for g in range(16):
        P = hs.datas[g].reshape(256, 131072)
        assert np.array_equal(got[g], oracle.encode(P, hs.V[1, g])), g


def test_bench_roundtrip_step_exact(gpu_ctx):
    # The bench's encode_decode step itself (bench.RoundTripStep over 16
    # prepared 32 MiB/256 generations): k + 2 coded pieces of each in one
    # grouped encode launch, 16 fresh decoders in one batched GPU AddPiece
    # call (the multi-workgroup elimination), one grouped GetPieces.  Two
    # steps (both vector sets); after each, every decoded generation equals
    # the original bytes, and every decoder took exactly k pieces.
    import bench
    L_ = _lib.lib()
    hs = bench.HeadlineStep(gpu_ctx, L_, errors, 256, 131072, 32, 16, grouped=True,
                            rng=np.random.default_rng(0x5EED), nvec=2, keep_data=True)
    rt = bench.RoundTripStep(gpu_ctx, L_, errors, hs.encs, 256, 131072, np.random.default_rng(0x7E), nsets=2)
    r0 = gpu_ctx.elim_stats()
    try:
        for i in range(2):
            rt.step(i, timed=True)
            got = gpu_ctx.d2h(rt.dO, 16 * 256 * 131072).reshape(16, -1)
            for g in range(16):
                assert np.array_equal(got[g], hs.datas[g]), (i, g)
            assert rt.ok and rt.decoded_ok(list(range(16)))
        assert len(rt.t_enc) == len(rt.t_add) == len(rt.t_get) == 2
        # every decoder of both steps eliminated on the GPU (rlnc_ctx_elim_stats)
        r1 = gpu_ctx.elim_stats()
        d = {key: r1[key] - r0[key] for key in r0}
        assert d["gpu"] == 32 and d["host_after_gpu"] == 0 and d["host"] == 0, d
    finally:
        rt.close()
        hs.close()


@pytest.mark.parametrize("overlap", ["elim", "elim_sync", "elim_only", "copy", "get"])
def test_bench_roundtrip_pipelined_exact(gpu_ctx, overlap):
    # The bench's pipelined round trip (the decoders on a context of their
    # own; step i + 1's encode queued beside step i's elimination -- from the
    # AddPiece call's hook --, its twin copy or its GetPieces): a phase of
    # three steps over both vector sets, every decoded generation equal to the
    # original bytes after each step, no encode queued past the phase, every
    # decoder on the GPU route.
    import bench
    from kodr_amd import device
    L_ = _lib.lib()
    hs = bench.HeadlineStep(gpu_ctx, L_, errors, 256, 131072, 32, 16, grouped=True,
                            rng=np.random.default_rng(0x5EEE), nvec=2, keep_data=True)
    dctx = device.Context(0)
    rt = bench.RoundTripStep(gpu_ctx, L_, errors, hs.encs, 256, 131072, np.random.default_rng(0x7F), nsets=2,
                             dctx=dctx, overlap=overlap)
    r0 = dctx.elim_stats()
    try:
        assert rt.pipelined
        rt.begin_phase(3)
        for i in range(3):
            rt.step(i, timed=True)
            assert (rt.ahead is not None) == (i < 2)
            rt.synchronize()
            got = dctx.d2h(rt.dO, 16 * 256 * 131072).reshape(16, -1)
            for g in range(16):
                assert np.array_equal(got[g], hs.datas[g]), (i, g)
            assert rt.ok and rt.decoded_ok(list(range(16)))
        assert len(rt.t_enc) == len(rt.t_add) == len(rt.t_get) == 3
        r1 = dctx.elim_stats()
        d = {key: r1[key] - r0[key] for key in r0}
        assert d["gpu"] == 48 and d["host_after_gpu"] == 0 and d["host"] == 0, d
    finally:
        rt.close()
        hs.close()
        dctx.close()


# grouped bit-sliced launches that plan each KW instance of
# gf_bs_kernel<KW, 0, true, 2> (gf_bs.hip plan_gemm_bs): (G, k, L, count) -> KW
GROUPED_KW_SHAPES = [((2, 8, 4096, 40), 1), ((2, 16, 4096, 40), 2), ((2, 24, 4096, 17), 3),
                     ((2, 32, 4096, 17), 4), ((2, 40, 4096, 9), 6), ((2, 64, 4096, 9), 8),
                     ((2, 96, 4096, 9), 16)]


@pytest.mark.parametrize("shape,kw", GROUPED_KW_SHAPES)
def test_grouped_bitsliced_every_kw(gpu_ctx, shape, kw):
    G, k, L, count = shape
    rng = np.random.default_rng(kw * 101 + k)
    gens = [rng.integers(0, 256, (k, L), dtype=np.uint8) for _ in range(G)]
    V = rng.integers(0, 256, (G, count, k), dtype=np.uint8)
    V[0, 0] = 0
    got = group_run(gpu_ctx, gens, count, V, out_pitch=L + 16, prepare=True)
    plan = _lib.last_launch_plan()
    assert (plan["kernel"], plan["waves"], plan["ring"], plan["generations"]) == (2, kw, 2, G), plan
    for g in range(G):
        assert np.array_equal(got[g], oracle.encode(gens[g], V[g])), g


def test_prepare_matches_lazy_twin(gpu_ctx):
    # prepare (eager twin) and the lazy twin of the first large batch give
    # the same bytes; prepare is idempotent
    rng = np.random.default_rng(11)
    k, L = 64, 8192 + 32
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    V = rng.integers(0, 256, (20, k), dtype=np.uint8)
    outs = []
    for prep in (0, 1, 2):
        e = make_encoder(gpu_ctx, P, prepare=False)
        for _ in range(prep):
            errors.check(_lib.lib().rlnc_encoder_prepare(e))
        out = np.empty((20, k + L), np.uint8)
        errors.check(_lib.lib().rlnc_encoder_coded_pieces(e, ptr(V), 20, ptr(out)))
        _lib.lib().rlnc_encoder_destroy(e)
        outs.append(out)
    ref = oracle.encode(P, V)
    for out in outs:
        assert np.array_equal(out[:, k:], ref)


def group_run(ctx, gens, count, V, out_pitch=None, expect=0, prepare=False):
    """Encode `count` pieces of every generation in one grouped call; returns
    (G, count, L) from the device output."""
    G = len(gens)
    k, L = gens[0].shape
    out_pitch = out_pitch or L
    encs = [make_encoder(ctx, P, prepare=prepare) for P in gens]
    arr = (ctypes.c_void_p * G)(*[e.value for e in encs])
    dV, dO = ctx.alloc(max(V.nbytes, 1)), ctx.alloc(G * count * out_pitch + 64)
    try:
        ctx.h2d(dV, V)
        ctx.h2d(dO, np.full(G * count * out_pitch + 64, 0xA5, np.uint8))
        st = _lib.lib().rlnc_encoder_group_coded_pieces_device(arr, G, dV, count, dO, out_pitch)
        assert st == expect
        ctx.synchronize()
        raw = ctx.d2h(dO, G * count * out_pitch + 64)
    finally:
        ctx.free(dV)
        ctx.free(dO)
        for e in encs:
            _lib.lib().rlnc_encoder_destroy(e)
    assert (raw[G * count * out_pitch:] == 0xA5).all()
    rows = raw[:G * count * out_pitch].reshape(G, count, out_pitch)
    if out_pitch > L:
        assert (rows[:, :, L:] == 0xA5).all(), "wrote past L"
    return rows[:, :, :L]


@pytest.mark.parametrize("G,k,L,count,prepare", [(3, 64, 4096, 66, True), (2, 64, 4096, 65, True),
                                                  (2, 128, 8192, 130, False), (34, 32, 2048, 66, True),
                                                  (2, 64, 4096, 67, True), (2, 64, 4096 + 16, 72, True),
                                                  (2, 64, 4096, 258, True), (3, 32, 2048 + 16, 300, True),
                                                  (2, 32, 4096, 512, False), (2, 16, 2048, 520, True)])
def test_grouped_encode_ragged_row_groups(gpu_ctx, G, k, L, count, prepare):
    # grouped bit-sliced batches of 8m + 1 / 8m + 2 pieces (the round trip's
    # k + 2: a last 8-row group with one or two real rows, zero and unit
    # vectors among them), 8m + 3 and 8m (67, 72), prepared and lazily built
    # twins, 34 generations over two launches; past 32 row groups the blocks
    # go in bands of 32 (gf_bs.hip): 33, 38, 64 and 65 groups (258, 300, 512,
    # 520 pieces); every piece against the oracle
    rng = np.random.default_rng(G * 7 + k + count)
    gens = [rng.integers(0, 256, (k, L), dtype=np.uint8) for _ in range(G)]
    V = rng.integers(0, 256, (G, count, k), dtype=np.uint8)
    V[0, count - 1] = 0                       # a zero vector in the tail codes the zero piece
    V[-1, count - 2, :] = 0
    V[-1, count - 2, 3] = 1                   # a unit vector in the tail codes piece 3 itself
    got = group_run(gpu_ctx, gens, count, V, out_pitch=L + 32, prepare=prepare)
    plan = _lib.last_launch_plan()
    assert plan["kernel"] == 2, plan
    for g in range(G):
        assert np.array_equal(got[g], oracle.encode(gens[g], V[g])), g


@pytest.mark.parametrize("G,k,L,count", [(1, 16, 4096, 1), (3, 16, 4096 + 16, 2), (5, 100, 8192 + 48, 1),
                                         (8, 256, 65536, 4), (40, 32, 1024, 1), (33, 64, 2048, 8),
                                         (6, 64, 4096, 12), (4, 20, 1000, 3), (35, 64, 2048, 9),
                                         (5, 100, 8192 + 48, 40), (3, 300, 4096, 17), (5, 16, 4096, 20),
                                         (3, 24, 65536, 32)])
def test_grouped_encode_vs_oracle(gpu_ctx, G, k, L, count):
    # (40, ...) and (33, ...) span two launches of <= 32 generations; count >= 9
    # takes the grouped bit-sliced launch ((35, ...) over two launches, k = 100
    # and 300 with a ragged last program chunk); L = 1000 is not a multiple of
    # 16 (ragged last chunk, padded pitch); k = 16 / 24 with 20 / 32 pieces:
    # few narrow rows, the grouped v_perm launch with more than 8 output rows
    rng = np.random.default_rng(G * 1000 + k + count)
    gens = [rng.integers(0, 256, (k, L), dtype=np.uint8) for _ in range(G)]
    V = rng.integers(0, 256, (G, count, k), dtype=np.uint8)
    got = group_run(gpu_ctx, gens, count, V, out_pitch=(L + 15) // 16 * 16 + 32)
    for g in range(G):
        assert np.array_equal(got[g], oracle.encode(gens[g], V[g])), g


@pytest.mark.parametrize("G,k,L,count", [(4, 64, 8192, 5), (3, 256, 131072, 8), (34, 32, 4096, 6)])
def test_grouped_encode_prepared_small_batches(gpu_ctx, G, k, L, count):
    # prepared encoders (twins resident): 5-8 pieces per generation take the
    # grouped bit-sliced launch instead of gf_gemm; (34, ...) spans two launches
    rng = np.random.default_rng(G * 77 + k + count)
    gens = [rng.integers(0, 256, (k, L), dtype=np.uint8) for _ in range(G)]
    V = rng.integers(0, 256, (G, count, k), dtype=np.uint8)
    got = group_run(gpu_ctx, gens, count, V, out_pitch=L + 32, prepare=True)
    for g in range(G):
        assert np.array_equal(got[g], oracle.encode(gens[g], V[g])), g


def test_grouped_encode_c2_generations(gpu_ctx):
    # the north-star shape: one coded piece of each of 4 generations of
    # 32 MiB / 256 in one launch
    rng = np.random.default_rng(0x6E5)
    gens = [rng.integers(0, 256, (256, 131072), dtype=np.uint8) for _ in range(4)]
    V = rng.integers(0, 256, (4, 1, 256), dtype=np.uint8)
    got = group_run(gpu_ctx, gens, 1, V)
    for g in range(4):
        assert np.array_equal(got[g], oracle.encode(gens[g], V[g])), g


def test_grouped_bitsliced_c2_generations(gpu_ctx, c2_generation):
    # 32 coded pieces of each of 3 generations of 32 MiB / 256 in one
    # bit-sliced launch (the headline's batch, grouped); one generation is
    # compact (twin only) and one prepared, one builds its twin in the call
    rng = np.random.default_rng(0x6B32)
    gens = [c2_generation, rng.integers(0, 256, (256, 131072), dtype=np.uint8),
            rng.integers(0, 256, (256, 131072), dtype=np.uint8)]
    G, count, k, L = 3, 32, 256, 131072
    V = rng.integers(0, 256, (G, count, k), dtype=np.uint8)
    V[1, 0] = 0
    V[2, 3] = 0
    V[2, 3, 255] = 1
    encs = [make_encoder(gpu_ctx, P, prepare=(i == 1)) for i, P in enumerate(gens)]
    errors.check(_lib.lib().rlnc_encoder_compact(encs[0]))
    arr = (ctypes.c_void_p * G)(*[e.value for e in encs])
    dV, dO = gpu_ctx.alloc(V.nbytes), gpu_ctx.alloc(G * count * L + 64)
    try:
        gpu_ctx.h2d(dV, V)
        gpu_ctx.h2d(dO + G * count * L, np.full(64, 0xA5, np.uint8))
        errors.check(_lib.lib().rlnc_encoder_group_coded_pieces_device(arr, G, dV, count, dO, L))
        gpu_ctx.synchronize()
        got = gpu_ctx.d2h(dO, G * count * L + 64)
    finally:
        gpu_ctx.free(dV)
        gpu_ctx.free(dO)
        for e in encs:
            _lib.lib().rlnc_encoder_destroy(e)
    assert (got[G * count * L:] == 0xA5).all()
    got = got[:G * count * L].reshape(G, count, L)
    for g in range(G):
        assert np.array_equal(got[g], oracle.encode(gens[g], V[g])), g
    assert not got[1, 0].any() and np.array_equal(got[2, 3], gens[2][255])


def test_grouped_encode_rejects_mixed_shapes(gpu_ctx):
    rng = np.random.default_rng(5)
    a = make_encoder(gpu_ctx, rng.integers(0, 256, (16, 1024), dtype=np.uint8), prepare=False)
    b = make_encoder(gpu_ctx, rng.integers(0, 256, (17, 1024), dtype=np.uint8), prepare=False)
    arr = (ctypes.c_void_p * 2)(a.value, b.value)
    dV = gpu_ctx.alloc(64)
    try:
        st = _lib.lib().rlnc_encoder_group_coded_pieces_device(arr, 2, dV, 1, dV, 1024)
        assert st == -1  # RLNC_ERR_INVALID_ARGUMENT
    finally:
        gpu_ctx.free(dV)
        _lib.lib().rlnc_encoder_destroy(a)
        _lib.lib().rlnc_encoder_destroy(b)


def test_prepared_recoder_c2(gpu_ctx, c2_generation):
    # the bench's recode leg: n = k = 256 wire rows, B = 32 recoded pieces
    P = c2_generation
    k, L = P.shape
    rng = np.random.default_rng(77)
    n, clen = k, k + L
    V = rng.integers(0, 256, (n, k), dtype=np.uint8)
    flat = np.concatenate([V, oracle.encode(P, V)], axis=1)
    rh = ctypes.c_void_p()
    errors.check(_lib.lib().rlnc_recoder_create(gpu_ctx.handle, ptr(flat), flat.size, n, k, ctypes.byref(rh)))
    errors.check(_lib.lib().rlnc_recoder_prepare(rh))
    R = rng.integers(0, 256, (32, n), dtype=np.uint8)
    out = np.empty((32, clen), np.uint8)
    try:
        errors.check(_lib.lib().rlnc_recoder_coded_pieces(rh, ptr(R), 32, ptr(out)))
    finally:
        _lib.lib().rlnc_recoder_destroy(rh)
    assert np.array_equal(out, oracle.recode(flat, k, R))


@pytest.mark.parametrize("G,k,L,n,count,compact", [(3, 32, 4096, 40, 12, False), (5, 16, 2048 + 16, 16, 4, False),
                                                   (34, 8, 1024, 10, 9, False), (3, 64, 8192, 64, 20, True),
                                                   (2, 256, 131072, 256, 32, False), (4, 64, 8192, 64, 6, "prepare"),
                                                   (3, 64, 8192, 64, 7, True)])
def test_grouped_recode_vs_oracle(gpu_ctx, G, k, L, n, count, compact):
    # rlnc_recoder_group_coded_pieces_device: gf_gemm launch below 9 pieces,
    # bit-sliced from 9 ((34, ...): two launches; compact: recoder 0 holds
    # only its twin); every recoded wire row against the oracle's recode
    rng = np.random.default_rng(G * 31 + k + count)
    lib = _lib.lib()
    flats, recs = [], []
    for g in range(G):
        P = rng.integers(0, 256, (k, L), dtype=np.uint8)
        V = rng.integers(0, 256, (n, k), dtype=np.uint8)
        flat = np.ascontiguousarray(np.concatenate([V, oracle.encode(P, V)], axis=1))
        rh = ctypes.c_void_p()
        errors.check(lib.rlnc_recoder_create(gpu_ctx.handle, ptr(flat), flat.size, n, k, ctypes.byref(rh)))
        flats.append(flat)
        recs.append(rh)
    if compact == "prepare":     # twins resident: 5-8 pieces take the bit-sliced launch
        for r in recs:
            errors.check(lib.rlnc_recoder_prepare(r))
    elif compact:
        errors.check(lib.rlnc_recoder_compact(recs[0]))
    clen = k + L
    pitch = (clen + 15) // 16 * 16 + 16
    R = rng.integers(0, 256, (G, count, n), dtype=np.uint8)
    arr = (ctypes.c_void_p * G)(*[r.value for r in recs])
    dR, dO = gpu_ctx.alloc(R.nbytes), gpu_ctx.alloc(G * count * pitch + 64)
    try:
        gpu_ctx.h2d(dR, R)
        gpu_ctx.h2d(dO, np.full(G * count * pitch + 64, 0xA5, np.uint8))
        errors.check(lib.rlnc_recoder_group_coded_pieces_device(arr, G, dR, count, dO, pitch))
        gpu_ctx.synchronize()
        raw = gpu_ctx.d2h(dO, G * count * pitch + 64)
    finally:
        gpu_ctx.free(dR)
        gpu_ctx.free(dO)
        for r in recs:
            lib.rlnc_recoder_destroy(r)
    assert (raw[G * count * pitch:] == 0xA5).all()
    rows = raw[:G * count * pitch].reshape(G, count, pitch)
    assert (rows[:, :, clen:] == 0xA5).all(), "wrote past the coded piece"
    for g in range(G):
        assert np.array_equal(rows[g, :, :clen], oracle.recode(flats[g], k, R[g])), g


def test_recode_c2_device_split_plan(gpu_ctx, c2_generation):
    # the bench's c2_recode leg at B = 32 through the device API: the piece
    # columns take the encoder's launch shape (64 column chunks x 4 row
    # groups, one round of KW = 16 workgroups) and the vector columns are
    # that launch's side product; every recoded wire row against the oracle
    P = c2_generation
    k, L = P.shape
    rng = np.random.default_rng(0x2EC0)
    n, clen = k, k + L
    V = rng.integers(0, 256, (n, k), dtype=np.uint8)
    flat = np.ascontiguousarray(np.concatenate([V, oracle.encode(P, V)], axis=1))
    lib = _lib.lib()
    rh = ctypes.c_void_p()
    errors.check(lib.rlnc_recoder_create(gpu_ctx.handle, ptr(flat), flat.size, n, k, ctypes.byref(rh)))
    errors.check(lib.rlnc_recoder_prepare(rh))
    R = rng.integers(0, 256, (32, n), dtype=np.uint8)
    R[0] = 0
    R[1] = 0
    R[1, 5] = 1                  # a unit recoding vector returns held piece 5 itself
    pitch = (clen + 255) // 256 * 256
    dR, dO = gpu_ctx.alloc(R.nbytes), gpu_ctx.alloc(32 * pitch)
    try:
        gpu_ctx.h2d(dR, R)
        errors.check(lib.rlnc_recoder_coded_pieces_device(rh, dR, 32, dO, pitch))
        plan = _lib.last_launch_plan()
        gpu_ctx.synchronize()
        got = gpu_ctx.d2h(dO, 32 * pitch).reshape(32, pitch)[:, :clen]
    finally:
        gpu_ctx.free(dR)
        gpu_ctx.free(dO)
        lib.rlnc_recoder_destroy(rh)
    assert (plan["kernel"], plan["waves"], plan["workgroups"]) == (2, 16, 256), plan
    assert np.array_equal(got, oracle.recode(flat, k, R))
    assert np.array_equal(got[1], flat[5]) and not got[0].any()


@pytest.mark.parametrize("k,L,n,counts", [(32, 4096 + 48, 40, (1, 3, 12)), (16, 2048, 16, (2, 9)),
                                          (20, 1024, 24, (1, 10))])
def test_compact_recoder_vs_oracle(gpu_ctx, k, L, n, counts):
    # compact recoders: the split layout (k a multiple of 16: piece twin +
    # a copy of the coding vectors) for every batch size, and the wire-row
    # twin for k = 20; device and host entry points against the oracle
    rng = np.random.default_rng(k * 1000 + L + n)
    lib = _lib.lib()
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    V = rng.integers(0, 256, (n, k), dtype=np.uint8)
    flat = np.ascontiguousarray(np.concatenate([V, oracle.encode(P, V)], axis=1))
    clen = k + L
    rh = ctypes.c_void_p()
    errors.check(lib.rlnc_recoder_create(gpu_ctx.handle, ptr(flat), flat.size, n, k, ctypes.byref(rh)))
    errors.check(lib.rlnc_recoder_compact(rh))
    try:
        for c in counts:
            R = rng.integers(0, 256, (c, n), dtype=np.uint8)
            out = np.empty((c, clen), np.uint8)
            errors.check(lib.rlnc_recoder_coded_pieces(rh, ptr(R), c, ptr(out)))
            assert np.array_equal(out, oracle.recode(flat, k, R)), c
            pitch = (clen + 15) // 16 * 16 + 16
            dR, dO = gpu_ctx.alloc(R.nbytes), gpu_ctx.alloc(c * pitch)
            try:
                gpu_ctx.h2d(dR, R)
                errors.check(lib.rlnc_recoder_coded_pieces_device(rh, dR, c, dO, pitch))
                gpu_ctx.synchronize()
                got = gpu_ctx.d2h(dO, c * pitch).reshape(c, pitch)[:, :clen]
            finally:
                gpu_ctx.free(dR)
                gpu_ctx.free(dO)
            assert np.array_equal(got, out), c
    finally:
        lib.rlnc_recoder_destroy(rh)
