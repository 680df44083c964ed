"""GPU parity of rlnc_encoder_group_coded_wire_device: many generations'
coded wire rows (vector ++ piece, CodedPiece.Flatten, data.go:52-57) in one
call, vectors drawn from each encoder's own device stream, systematic
encoders emitting e_id ++ P_id first (systematic/encoder.go:82-109).

Each case runs the grouped call on one set of encoders and
rlnc_encoder_coded_wire_device encoder by encoder on a clone set (same data,
same seeds): the rows must be byte-identical, and every coded row must be a
codeword of its generation per the oracle (oracle.encode of its own vector,
full/encoder.go:61-71).  A second call continues each stream, as a second
per-encoder call would.
"""
import ctypes

import numpy as np
import pytest

import oracle
from kodr_amd import _lib, errors

pytestmark = pytest.mark.gpu
U8P = _lib._u8p


def make(ctx, P, kind, seed, prepare):
    lib = _lib.lib()
    h = ctypes.c_void_p()
    k, L = P.shape
    errors.check(lib.rlnc_encoder_create(ctx.handle, kind, np.ascontiguousarray(P).ctypes.data_as(U8P), k, L,
                                         ctypes.byref(h)))
    errors.check(lib.rlnc_encoder_seed(h, seed))
    if prepare:
        errors.check(lib.rlnc_encoder_prepare(h))
    return h


def run_case(ctx, gens, kinds, counts, wp, prepare=False, advance=None, plan_kernel=None, oracle_rows=None):
    lib = _lib.lib()
    G = len(gens)
    k, L = gens[0].shape
    A = [make(ctx, P, kinds[i], 1000 + i, prepare) for i, P in enumerate(gens)]
    B = [make(ctx, P, kinds[i], 1000 + i, prepare) for i, P in enumerate(gens)]
    arr = (ctypes.c_void_p * G)(*[e.value for e in A])
    try:
        if advance:  # move some encoders' streams forward first (mixed positions)
            for i, n in advance.items():
                d = ctx.alloc(n * wp)
                errors.check(lib.rlnc_encoder_coded_wire_device(A[i], n, d, wp))
                errors.check(lib.rlnc_encoder_coded_wire_device(B[i], n, d, wp))
                ctx.synchronize()
                ctx.free(d)
        for count in counts:
            size = G * count * wp
            dA, dB = ctx.alloc(size + 64), ctx.alloc(size + 64)
            try:
                ctx.h2d(dA, np.full(size + 64, 0xA5, np.uint8))
                ctx.h2d(dB, np.full(size + 64, 0xA5, np.uint8))
                errors.check(lib.rlnc_encoder_group_coded_wire_device(arr, G, count, dA, wp))
                plan = _lib.last_launch_plan()
                for i in range(G):
                    errors.check(lib.rlnc_encoder_coded_wire_device(B[i], count, dB + i * count * wp, wp))
                ctx.synchronize()
                got, ref = ctx.d2h(dA, size + 64), ctx.d2h(dB, size + 64)
            finally:
                ctx.free(dA)
                ctx.free(dB)
            assert (got[size:] == 0xA5).all(), "wrote past the last row"
            assert np.array_equal(got, ref), "grouped rows differ from per-encoder rows"
            rows = got[:size].reshape(G, count, wp)
            sel = list(range(count)) if oracle_rows is None else [r for r in oracle_rows if r < count]
            for g in range(G):
                V = np.ascontiguousarray(rows[g, sel, :k])
                assert np.array_equal(rows[g, sel, k:k + L], oracle.encode(gens[g], V)), g
            if plan_kernel is not None:
                assert plan["kernel"] == plan_kernel and plan["generations"] == G, plan
            for i in range(G):
                assert lib.rlnc_encoder_systematic_remaining(A[i]) == lib.rlnc_encoder_systematic_remaining(B[i])
    finally:
        for e in A + B:
            lib.rlnc_encoder_destroy(e)
    return rows


@pytest.mark.parametrize("G,k,L,count,prepare,kernel", [(5, 64, 8192, 12, False, 2), (3, 32, 4096, 3, False, 1),
                                                         (34, 16, 1024, 2, False, None),
                                                         (4, 64, 8192, 6, True, 2)])
def test_group_wire_full(gpu_ctx, G, k, L, count, prepare, kernel):
    # count >= 9: the grouped bit-sliced launch on the twins; 3: gf_gemm over
    # the plain rows; 34 generations: two vector launches and two products;
    # 6 pieces on prepared twins: the bit-sliced launch from 5 pieces
    rng = np.random.default_rng(G * 7 + k + count)
    gens = [rng.integers(0, 256, (k, L), dtype=np.uint8) for _ in range(G)]
    wp = (k + L + 15) // 16 * 16 + 16
    run_case(gpu_ctx, gens, [0] * G, [count, count + 1], wp, prepare=prepare, plan_kernel=kernel)


def test_group_wire_systematic_crosses_k(gpu_ctx):
    # systematic encoders created together: the first call is all e_id ++ P_id,
    # the second crosses k mid-batch (6 systematic + 6 coded rows), the third
    # is coded only
    rng = np.random.default_rng(0x5E5)
    G, k, L = 3, 16, 4096
    gens = [rng.integers(0, 256, (k, L), dtype=np.uint8) for _ in range(G)]
    rows = run_case(gpu_ctx, gens, [1] * G, [10, 12, 9], k + L)
    for g in range(G):
        assert (rows[g, :, :k] != 0).sum() > 0


def test_group_wire_mixed_positions_and_kinds(gpu_ctx):
    # one systematic encoder already 5 pieces in, one full encoder: encoder
    # by encoder, same bytes
    rng = np.random.default_rng(0x313)
    G, k, L = 3, 16, 2048
    gens = [rng.integers(0, 256, (k, L), dtype=np.uint8) for _ in range(G)]
    run_case(gpu_ctx, gens, [1, 1, 0], [8, 12], k + L, advance={1: 5})


def test_group_wire_unaligned_pitch(gpu_ctx):
    # k + L = 2053 bytes per row, no padding: piece columns not 16-byte
    # aligned, encoder by encoder
    rng = np.random.default_rng(0x0DD)
    G, k, L = 2, 5, 2048
    gens = [rng.integers(0, 256, (k, L), dtype=np.uint8) for _ in range(G)]
    run_case(gpu_ctx, gens, [0, 0], [9, 2], k + L)


def test_group_wire_c2(gpu_ctx):
    # two 32 MiB / 256 generations, k + 2 = 258 wire rows each at pitch k + L
    # (the bench's encode+decode leg): one vector launch, one bit-sliced launch
    rng = np.random.default_rng(0xC2C2)
    G, k, L = 2, 256, 131072
    gens = [rng.integers(0, 256, (k, L), dtype=np.uint8) for _ in range(G)]
    # (every row equals the per-encoder call's; rows 0, 1, 129 and 257 also
    # against the oracle, to keep the CPU check short)
    run_case(gpu_ctx, gens, [0, 0], [k + 2], k + L, prepare=True, plan_kernel=2, oracle_rows=[0, 1, 129, 257])
