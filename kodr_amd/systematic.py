"""Mirror of kodr's ``systematic`` package (systematic/encoder.go,
systematic/decoder.go).  The first PieceCount() calls of CodedPiece() return
the original pieces under unit vectors (systematic/encoder.go:83-96); later
calls are full RLNC (:98-108).  The decoder is kodr's full decoder
(systematic/decoder.go:96-104 states it does not exploit systematic rows)."""
from . import errors
from ._codec import SYSTEMATIC, _Decoder, _Encoder
from ._lib import lib


class SystematicRLNCEncoder(_Encoder):
    """systematic/encoder.go:7-11."""


class SystematicRLNCDecoder(_Decoder):
    """systematic/decoder.go:9-12."""


def NewSystematicRLNCEncoder(pieces, ctx=None, rng=None, batch=16):
    """systematic/encoder.go:115-117."""
    pieces = [bytes(p) for p in pieces]
    if not pieces:
        raise errors.ErrBadPieceCount("minimum 2 pieces required for RLNC")
    return SystematicRLNCEncoder._create(lib().rlnc_encoder_create, ctx, SYSTEMATIC, b"".join(pieces),
                                         len(pieces), len(pieces[0]), rng=rng, batch=batch)


def NewSystematicRLNCEncoderWithPieceCount(data, pieceCount, ctx=None, rng=None, batch=16):
    """systematic/encoder.go:123-132."""
    return SystematicRLNCEncoder._create(lib().rlnc_encoder_create_with_piece_count, ctx, SYSTEMATIC,
                                         bytes(data), len(data), pieceCount, rng=rng, batch=batch)


def NewSystematicRLNCEncoderWithPieceSize(data, pieceSize, ctx=None, rng=None, batch=16):
    """systematic/encoder.go:137-146."""
    return SystematicRLNCEncoder._create(lib().rlnc_encoder_create_with_piece_size, ctx, SYSTEMATIC,
                                         bytes(data), len(data), pieceSize, rng=rng, batch=batch)


def NewSystematicRLNCDecoder(pieceCount, ctx=None):
    """systematic/decoder.go:105-108."""
    return SystematicRLNCDecoder(pieceCount, ctx)
