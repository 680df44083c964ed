"""Progressive decode: rlnc_decoder_decoded_mask /
rlnc_decoder_get_decoded read every original piece that is decoded before
full rank (a systematic piece on arrival), under the LAZY and EAGER data-side
policies; checked against the oracle's literal decoder state (which rows are
a*e_j) and the original pieces, and the two policies leave identical kodr
state."""
import ctypes

import numpy as np
import pytest

import oracle
from kodr_amd import _lib, errors

pytestmark = pytest.mark.gpu
U8P = _lib._u8p
LAZY, EAGER = 0, 1


def _decoded_by_oracle(ref, k):
    out = set()
    for row in ref.coeffs():
        nz = np.nonzero(row)[0]
        if len(nz) == 1:
            out.add(int(nz[0]))
    return out


class Dec:
    def __init__(self, ctx, k, policy):
        self.k = k
        self.h = ctypes.c_void_p()
        errors.check(_lib.lib().rlnc_decoder_create(ctx.handle, k, ctypes.byref(self.h)))
        errors.check(_lib.lib().rlnc_decoder_set_policy(self.h, policy))

    def add(self, v, p):
        v, p = np.ascontiguousarray(v, np.uint8), np.ascontiguousarray(p, np.uint8)
        return _lib.lib().rlnc_decoder_add_piece(self.h, v.ctypes.data_as(U8P), v.size, p.ctypes.data_as(U8P), p.size)

    def mask(self):
        m = np.zeros(self.k, np.uint8)
        n = _lib.lib().rlnc_decoder_decoded_mask(self.h, m.ctypes.data_as(U8P))
        assert n == int(m.sum())
        return {int(j) for j in np.nonzero(m)[0]}

    def get(self, j, L):
        out = np.zeros(L, np.uint8)
        st = _lib.lib().rlnc_decoder_get_decoded(self.h, j, ctypes.c_void_p(out.ctypes.data), 0)
        return st, out

    def state(self):
        L_ = _lib.lib()
        return (L_.rlnc_decoder_useful(self.h), L_.rlnc_decoder_received(self.h),
                bool(L_.rlnc_decoder_is_decoded(self.h)))

    def __del__(self):
        _lib.lib().rlnc_decoder_destroy(self.h)


def _stream(rng, k, L, kind):
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    rows = []
    if kind in ("systematic", "scaled"):
        lost = set(rng.choice(k, max(1, k // 6), replace=False).tolist())
        for i in range(k):
            if i in lost:
                continue
            v = np.zeros(k, np.uint8)
            v[i] = 1 if kind == "systematic" else int(rng.integers(2, 256))
            rows.append(v)
        rows += [rng.integers(0, 256, k, dtype=np.uint8) for _ in range(len(lost) + 2)]
    else:
        rows = [rng.integers(0, 256, k, dtype=np.uint8) for _ in range(k + 2)]
    V = np.stack(rows)
    return P, V, oracle.encode(P, V)


@pytest.mark.parametrize("kind", ["systematic", "scaled", "coded"])
@pytest.mark.parametrize("k,L", [(12, 1000), (40, 4096)])
def test_progressive_piecewise_vs_oracle(gpu_ctx, kind, k, L):
    rng = np.random.default_rng(k + L + len(kind))
    P, V, C = _stream(rng, k, L, kind)
    lazy, eager, ref = Dec(gpu_ctx, k, LAZY), Dec(gpu_ctx, k, EAGER), oracle.Decoder(k)
    for i in range(V.shape[0]):
        s_ref = ref.add(V[i], C[i])
        assert lazy.add(V[i], C[i]) == s_ref
        assert eager.add(V[i], C[i]) == s_ref
        if s_ref != 0:
            break
        assert lazy.state() == eager.state() == (ref.useful(), ref.received(), ref.is_decoded())
        exp = _decoded_by_oracle(ref, k)
        assert lazy.mask() == eager.mask() == exp
        if kind == "coded" and not ref.is_decoded():
            assert not exp
        for j in range(k):
            for d in (lazy, eager):
                st, out = d.get(j, L)
                if j in exp:
                    assert st == 0 and np.array_equal(out, P[j]), (i, j)
                else:
                    assert st == errors.ErrPieceNotDecodedYet.code
    assert lazy.mask() == set(range(k))
    st, _ = lazy.get(k, L)
    assert st == errors.ErrPieceOutOfBound.code


def test_progressive_batches_device_out_and_gpu_elimination(gpu_ctx):
    """Batched AddPiece under EAGER (host and GPU elimination paths): after
    each batch the decoded pieces are ready; device-side reads."""
    rng = np.random.default_rng(9)
    k, L = 64, 2048
    P, V, C = _stream(rng, k, L, "systematic")
    pitch = ((k + L + 15) // 16) * 16
    rows = np.zeros((V.shape[0], pitch), np.uint8)
    rows[:, :k], rows[:, k:k + L] = V, C
    drows = gpu_ctx.alloc(rows.nbytes)
    gpu_ctx.h2d(drows, rows)
    dout = gpu_ctx.alloc(L)
    # host elimination, three batches
    d, ref = Dec(gpu_ctx, k, EAGER), oracle.Decoder(k)
    pos = 0
    for cut in (20, 50, V.shape[0]):
        c = ctypes.c_size_t()
        st = _lib.lib().rlnc_decoder_add_pieces(d.h, ctypes.c_void_p(drows + pos * pitch), cut - pos, pitch, L, 1,
                                                ctypes.byref(c))
        n_ref, st_ref = 0, 0
        for i in range(pos, cut):
            s = ref.add(V[i], C[i])
            if s:
                st_ref = s
                break
            n_ref += 1
        assert (st, c.value) == (st_ref, n_ref)
        exp = _decoded_by_oracle(ref, k)
        assert d.mask() == exp
        for j in sorted(exp)[:8]:
            errors.check(_lib.lib().rlnc_decoder_get_decoded(d.h, j, ctypes.c_void_p(dout), 1))
            assert np.array_equal(gpu_ctx.d2h(dout, L), P[j])
        pos += c.value
        if st:
            break
    # GPU elimination of the whole batch on a fresh EAGER decoder
    g = Dec(gpu_ctx, k, EAGER)
    c = ctypes.c_size_t()
    st = _lib.lib().rlnc_decoder_add_pieces_gpu(g.h, ctypes.c_void_p(drows), V.shape[0], pitch, L, ctypes.byref(c))
    assert st in (0, 3) and g.mask() == set(range(k))
    for j in range(0, k, 7):
        s2, out = g.get(j, L)
        assert s2 == 0 and np.array_equal(out, P[j])
    gpu_ctx.synchronize()
    gpu_ctx.free(drows)
    gpu_ctx.free(dout)


@pytest.mark.parametrize("policy", [EAGER, LAZY])
def test_bound_output_in_place(gpu_ctx, policy):
    """rlnc_decoder_bind_output: decoded pieces land at row j of the caller's
    buffer (EAGER: during AddPiece; LAZY: on get_decoded, whose in-place read
    is then a no-op); rows not yet decoded are left untouched."""
    rng = np.random.default_rng(21 + policy)
    k, L = 48, 3000
    opitch = 3008
    P, V, C = _stream(rng, k, L, "scaled")
    d, ref = Dec(gpu_ctx, k, policy), oracle.Decoder(k)
    dout = gpu_ctx.alloc(k * opitch)
    gpu_ctx.h2d(dout, np.full(k * opitch, 0xA5, np.uint8))
    lib = _lib.lib()
    assert lib.rlnc_decoder_bind_output(d.h, ctypes.c_void_p(dout), opitch) < 0  # length not known yet
    assert d.add(V[0], C[0]) == ref.add(V[0], C[0])
    assert lib.rlnc_decoder_bind_output(d.h, ctypes.c_void_p(dout), L) < 0  # pitch not a multiple of 16
    errors.check(lib.rlnc_decoder_bind_output(d.h, ctypes.c_void_p(dout), opitch))
    for i in range(1, V.shape[0]):
        s_ref = ref.add(V[i], C[i])
        assert d.add(V[i], C[i]) == s_ref
        if s_ref:
            break
        exp = _decoded_by_oracle(ref, k)
        assert d.mask() == exp
        if policy == LAZY:
            for j in exp:
                errors.check(lib.rlnc_decoder_get_decoded(d.h, j, ctypes.c_void_p(dout + j * opitch), 1))
        if i % 5 == 0 or ref.is_decoded():
            gpu_ctx.synchronize()
            got = gpu_ctx.d2h(dout, k * opitch).reshape(k, opitch)
            for j in range(k):
                if j in exp:
                    assert np.array_equal(got[j, :L], P[j]), (i, j)
                else:
                    assert (got[j, :L] == 0xA5).all(), (i, j)
                assert (got[j, L:] == 0xA5).all()
    assert ref.is_decoded() and d.mask() == set(range(k))
    st, out = d.get(5, L)  # host read from the bound row
    assert st == 0 and np.array_equal(out, P[5])
    errors.check(lib.rlnc_decoder_bind_output(d.h, None, 0))
    st, out = d.get(7, L)
    assert st == 0 and np.array_equal(out, P[7])
    gpu_ctx.synchronize()
    gpu_ctx.free(dout)


def test_python_mirror_extensions(gpu_ctx):
    """The Python mirror's extensions: compact encoder, EAGER decoder,
    decoded_mask / GetDecodedPiece while a systematic stream arrives."""
    from kodr_amd import systematic
    rng = np.random.default_rng(44)
    k, L = 32, 1500
    pieces = [rng.integers(0, 256, L, dtype=np.uint8).tobytes() for _ in range(k)]
    enc = systematic.NewSystematicRLNCEncoder(pieces, ctx=gpu_ctx)
    enc.compact()
    assert enc.device_pieces()[0] is None
    dec = systematic.NewSystematicRLNCDecoder(k, ctx=gpu_ctx)
    dec.set_policy(True)
    lost = {3, 17, 30}
    sent = 0
    while not dec.IsDecoded():
        p = enc.CodedPiece()
        i = sent
        sent += 1
        if i < k and i in lost:
            continue
        dec.AddPiece(p)
        if i < k:
            assert dec.decoded_mask()[i] and dec.GetDecodedPiece(i) == pieces[i]
            with pytest.raises(errors.ErrPieceNotDecodedYet):
                dec.GetDecodedPiece(30)
    assert dec.decoded_mask().all()
    assert [dec.GetDecodedPiece(j) for j in range(k)] == pieces == dec.GetPieces()
