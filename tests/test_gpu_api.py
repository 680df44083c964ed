"""kodr's own test suite, restated against the drop-in API (kodr_amd.full /
kodr_amd.systematic / kodr_amd.kodr_internals) running on the GPU.

Each test names the Go test it follows.  kodr's tests are unseeded
(crypto/rand, math/rand); these use seeded numpy generators so failures
reproduce, at the same shapes.
"""
import math

import numpy as np
import pytest

from kodr_amd import errors, full, kodr_internals, systematic

pytestmark = pytest.mark.gpu


def rng_bytes(rng):
    return lambda n: rng.integers(0, 256, n, dtype=np.uint8).tobytes()


def gen_pieces(rng, count, length):
    return [rng.integers(0, 256, length, dtype=np.uint8).tobytes() for _ in range(count)]


def encoder_flow(enc, piece_count, coded_count, pieces):
    """full/encoder_test.go:34-77."""
    coded = [enc.CodedPiece() for _ in range(coded_count)]
    dec = full.NewFullRLNCDecoder(piece_count)
    for i in range(coded_count):
        if i < piece_count:
            with pytest.raises(errors.ErrMoreUsefulPiecesRequired):
                dec.GetPieces()
        try:
            dec.AddPiece(coded[i])
        except errors.ErrAllUsefulPiecesReceived:
            break
    assert dec.IsDecoded()
    for i in range(coded_count - piece_count):
        with pytest.raises(errors.ErrAllUsefulPiecesReceived):
            dec.AddPiece(coded[piece_count + i])
    d = dec.GetPieces()
    assert len(d) == len(pieces)
    assert d == [bytes(p) for p in pieces]


def test_new_full_rlnc_encoder(gpu_ctx):
    # full/encoder_test.go:79-87
    rng = np.random.default_rng(1)
    pieces = gen_pieces(rng, 128, 8192)
    enc = full.NewFullRLNCEncoder(pieces, rng=rng_bytes(rng))
    encoder_flow(enc, 128, 130, pieces)


@pytest.mark.parametrize("seed", range(4))
def test_new_full_rlnc_encoder_with_piece_count(gpu_ctx, seed):
    # full/encoder_test.go:89-107
    rng = np.random.default_rng(10 + seed)
    size = int((2 << 10) + rng.integers(0, 2 << 10))
    count = int((2 << 1) + rng.integers(0, 2 << 8))
    data = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
    pieces, _ = kodr_internals.OriginalPiecesFromDataAndPieceCount(data, count)
    enc = full.NewFullRLNCEncoderWithPieceCount(data, count, rng=rng_bytes(rng))
    encoder_flow(enc, count, count + 2, pieces)


@pytest.mark.parametrize("seed", range(4))
def test_new_full_rlnc_encoder_with_piece_size(gpu_ctx, seed):
    # full/encoder_test.go:109-128
    rng = np.random.default_rng(20 + seed)
    size = int((2 << 10) + rng.integers(0, 2 << 10))
    psize = int((2 << 5) + rng.integers(0, 2 << 5))
    count = math.ceil(size / psize)
    data = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
    pieces, _ = kodr_internals.OriginalPiecesFromDataAndPieceSize(data, psize)
    enc = full.NewFullRLNCEncoderWithPieceSize(data, psize, rng=rng_bytes(rng))
    encoder_flow(enc, count, count + 2, pieces)


def test_encoder_padding_and_coded_piece_len(gpu_ctx):
    # full/encoder_test.go:130-210 and systematic/encoder_test.go:141-221
    rng = np.random.default_rng(30)
    for mod in (full, systematic):
        mk_count = getattr(mod, "NewFullRLNCEncoderWithPieceCount", None) or mod.NewSystematicRLNCEncoderWithPieceCount
        mk_size = getattr(mod, "NewFullRLNCEncoderWithPieceSize", None) or mod.NewSystematicRLNCEncoderWithPieceSize
        for _ in range(8):
            size = int((2 << 10) + rng.integers(0, 2 << 10))
            count = int((2 << 1) + rng.integers(0, 2 << 8))
            data = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
            enc = mk_count(data, count, rng=rng_bytes(rng))
            assert len(enc.CodedPiece().Piece) == (size + enc.Padding()) // count
            psize = int((2 << 5) + rng.integers(0, 2 << 5))
            enc = mk_size(data, psize, rng=rng_bytes(rng))
            pc = math.ceil(size / psize)
            assert (size + enc.Padding()) // pc == psize
            for _ in range(pc + 1):
                assert enc.CodedPiece().Len() == enc.CodedPieceLen()


def test_decodable_len_with_random_drops(gpu_ctx):
    # full/encoder_test.go:212-262
    rng = np.random.default_rng(40)
    size = int((2 << 10) + rng.integers(0, 2 << 10))
    count = int((2 << 1) + rng.integers(0, 2 << 8))
    data = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
    enc = full.NewFullRLNCEncoderWithPieceCount(data, count, rng=rng_bytes(rng))
    dec = full.NewFullRLNCDecoder(count)
    consumed = 0
    while not dec.IsDecoded():
        cp = enc.CodedPiece()
        if rng.integers(0, 2) == 0:
            continue
        try:
            dec.AddPiece(cp)
        except errors.ErrAllUsefulPiecesReceived:
            break
        consumed += cp.Len()
    assert consumed >= enc.DecodableLen()


def test_decoder_required_monotone(gpu_ctx):
    # full/decoder_test.go:13-74
    rng = np.random.default_rng(50)
    pieces = gen_pieces(rng, 128, 8192)
    enc = full.NewFullRLNCEncoder(pieces, rng=rng_bytes(rng))
    coded = [enc.CodedPiece() for _ in range(130)]
    dec = full.NewFullRLNCDecoder(128)
    needed = 128
    for i, cp in enumerate(coded):
        req = dec.Required()
        if i == 0:
            assert req == needed
        else:
            assert req <= needed
            needed = req
        try:
            dec.AddPiece(cp)
        except errors.ErrAllUsefulPiecesReceived:
            break
    assert dec.IsDecoded()
    assert dec.GetPieces() == pieces


def recoder_flow(rec, count, pieces):
    """full/recoder_test.go:13-39."""
    dec = full.NewFullRLNCDecoder(count)
    while True:
        try:
            dec.AddPiece(rec.CodedPiece())
        except errors.ErrAllUsefulPiecesReceived:
            break
    assert dec.GetPieces() == pieces


def test_new_full_rlnc_recoder(gpu_ctx):
    # full/recoder_test.go:41-55
    rng = np.random.default_rng(60)
    pieces = gen_pieces(rng, 128, 8192)
    enc = full.NewFullRLNCEncoder(pieces, rng=rng_bytes(rng))
    coded = [enc.CodedPiece() for _ in range(130)]
    recoder_flow(full.NewFullRLNCRecoder(coded, rng=rng_bytes(rng)), 128, pieces)


def test_new_full_rlnc_recoder_with_flatten_data(gpu_ctx):
    # full/recoder_test.go:57-80
    rng = np.random.default_rng(61)
    pieces = gen_pieces(rng, 128, 8192)
    enc = full.NewFullRLNCEncoder(pieces, rng=rng_bytes(rng))
    flat = b"".join(enc.CodedPiece().Flatten() for _ in range(130))
    rec = full.NewFullRLNCRecoderWithFlattenData(flat, 130, 128, rng=rng_bytes(rng))
    recoder_flow(rec, 128, pieces)


def test_coded_pieces_for_recoding(gpu_ctx):
    # kodr_internals/data_test.go:88-134
    rng = np.random.default_rng(62)
    data = rng.integers(0, 256, 6, dtype=np.uint8).tobytes()
    enc = full.NewFullRLNCEncoderWithPieceCount(data, 3, rng=rng_bytes(rng))
    coded = [enc.CodedPiece() for _ in range(5)]
    flat = b"".join(c.Flatten() for c in coded)
    with pytest.raises(errors.ErrCodedDataLengthMismatch):
        kodr_internals.CodedPiecesForRecoding(flat, 3, 3)
    with pytest.raises(errors.ErrCodingVectorLengthMismatch):
        kodr_internals.CodedPiecesForRecoding(flat, 5, 5)
    back = kodr_internals.CodedPiecesForRecoding(flat, 5, 3)
    assert [(c.Vector, c.Piece) for c in back] == [(c.Vector, c.Piece) for c in coded]


def test_split_errors():
    # kodr_internals/data_test.go:24-74 (error paths; no device needed but the
    # library is, so it runs with the GPU suite as well)
    data = bytes(3000)
    with pytest.raises(errors.ErrBadPieceCount):
        kodr_internals.OriginalPiecesFromDataAndPieceCount(data, 0)
    with pytest.raises(errors.ErrPieceCountMoreThanTotalBytes):
        kodr_internals.OriginalPiecesFromDataAndPieceCount(data, 3001)
    with pytest.raises(errors.ErrZeroPieceSize):
        kodr_internals.OriginalPiecesFromDataAndPieceSize(data, 0)
    with pytest.raises(errors.ErrBadPieceCount):
        kodr_internals.OriginalPiecesFromDataAndPieceSize(data, 3000)


def test_systematic_coding_flags(gpu_ctx):
    # systematic/encoder_test.go:35-56
    rng = np.random.default_rng(70)
    count = int((2 << 1) + rng.integers(0, 2 << 8))
    pieces = gen_pieces(rng, count, 8192)
    enc = systematic.NewSystematicRLNCEncoder(pieces, rng=rng_bytes(rng))
    for i in range(2 * count):
        assert enc.CodedPiece().IsSystematic() == (i < count)


@pytest.mark.parametrize("ctor", ["pieces", "count", "size"])
def test_systematic_round_trip_with_drops(gpu_ctx, ctor):
    # systematic/encoder_test.go:58-139
    rng = np.random.default_rng(80 + len(ctor))
    if ctor == "pieces":
        count, pieces = 256, gen_pieces(rng, 256, 8192)
        enc = systematic.NewSystematicRLNCEncoder(pieces, rng=rng_bytes(rng))
    else:
        size = int((2 << 10) + rng.integers(0, 2 << 10))
        data = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
        if ctor == "count":
            count = int((2 << 1) + rng.integers(0, 2 << 8))
            enc = systematic.NewSystematicRLNCEncoderWithPieceCount(data, count, rng=rng_bytes(rng))
            pieces, _ = kodr_internals.OriginalPiecesFromDataAndPieceCount(data, count)
        else:
            psize = int((2 << 5) + rng.integers(0, 2 << 5))
            enc = systematic.NewSystematicRLNCEncoderWithPieceSize(data, psize, rng=rng_bytes(rng))
            pieces, _ = kodr_internals.OriginalPiecesFromDataAndPieceSize(data, psize)
            count = len(pieces)
    dec = systematic.NewSystematicRLNCDecoder(count)
    while True:
        cp = enc.CodedPiece()
        if rng.integers(0, 2) == 0:
            continue
        try:
            dec.AddPiece(cp)
        except errors.ErrAllUsefulPiecesReceived:
            assert dec.Required() == 0
            break
    assert dec.GetPieces() == [bytes(p) for p in pieces]


def test_get_piece_errors(gpu_ctx):
    # decoder_state.go:221-227 error paths through the API
    dec = full.NewFullRLNCDecoder(4)
    assert dec.PieceLength() == 0
    with pytest.raises(errors.ErrMoreUsefulPiecesRequired):
        dec.GetPieces()
    dec.AddPiece(kodr_internals.CodedPiece(bytes([1, 2, 3, 4]), bytes(range(10))))
    assert dec.PieceLength() == 10
    with pytest.raises(errors.ErrPieceOutOfBound):
        dec.GetPiece(4)
    with pytest.raises(errors.ErrPieceNotDecodedYet):
        dec.GetPiece(1)
    # first piece is not RREF'd; [1, 2, 3, 4] passes the :237-251 check as is
    assert dec.GetPiece(0) == bytes(range(10))
    dec1 = full.NewFullRLNCDecoder(4)
    dec1.AddPiece(kodr_internals.CodedPiece(bytes([2, 2, 3, 4]), bytes(range(10))))
    with pytest.raises(errors.ErrPieceNotDecodedYet):
        dec1.GetPiece(0)  # coeffs[0][0] != 1
    dec2 = full.NewFullRLNCDecoder(3)
    dec2.AddPiece(kodr_internals.CodedPiece(bytes([1, 5, 7]), bytes([9, 8, 7])))
    assert dec2.GetPiece(0) == bytes([9, 8, 7])  # the :237-251 quirk: passes, not decoded


def test_minimal_shapes(gpu_ctx):
    # k = 2, L = 1 (smallest generation kodr accepts)
    rng = np.random.default_rng(90)
    data = bytes([7, 200])
    enc = full.NewFullRLNCEncoderWithPieceCount(data, 2, rng=rng_bytes(rng))
    assert (enc.PieceCount(), enc.PieceSize(), enc.Padding()) == (2, 1, 0)
    dec = full.NewFullRLNCDecoder(2)
    while not dec.IsDecoded():
        dec.AddPiece(enc.CodedPiece())
    assert b"".join(dec.GetPieces()) == data


def test_flush_decoders_groups_piecewise_feeds(gpu_ctx):
    # kodr's decoder loop (full/decoder_test.go:20-40: AddPiece per coded
    # piece) on several generations at once, their queued eliminations run
    # together by full.flush_decoders (rlnc_decoders_flush_gpu); the counters,
    # the refusal once decoded and GetPieces are kodr's
    rng = np.random.default_rng(5)
    k = 32
    gens = [gen_pieces(rng, k, 1024 + 16 * g) for g in range(4)]
    encs = [full.NewFullRLNCEncoder(p, rng=rng_bytes(rng)) for p in gens]
    decs = [full.NewFullRLNCDecoder(k) for _ in gens]
    for i in range(k):
        for e, d in zip(encs, decs):
            d.AddPiece(e.CodedPiece())
    full.flush_decoders(decs)
    for e, d, p in zip(encs, decs, gens):
        assert d.IsDecoded() and d.Required() == 0
        with pytest.raises(errors.ErrAllUsefulPiecesReceived):
            d.AddPiece(e.CodedPiece())
        assert d.GetPieces() == [bytes(x) for x in p]
