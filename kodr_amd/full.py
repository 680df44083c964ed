"""Mirror of kodr's ``full`` package (full/encoder.go, full/recoder.go,
full/decoder.go) on the MI355X engine.  Go's (value, error) returns become a
return value or a raised kodr_amd.errors.Err* exception."""
import ctypes

from . import errors
from ._codec import FULL, _Decoder, _Encoder, _Recoder, flush_decoders  # noqa: F401 (extension)
from ._lib import lib, u8
from .device import default_context


class FullRLNCEncoder(_Encoder):
    """full/encoder.go:7-10."""


class FullRLNCRecoder(_Recoder):
    """full/recoder.go:8-11."""


class FullRLNCDecoder(_Decoder):
    """full/decoder.go:9-12."""


def NewFullRLNCEncoder(pieces, ctx=None, rng=None, batch=16):
    """full/encoder.go:76-78 -- pieces: list of equal-length byte strings."""
    pieces = [bytes(p) for p in pieces]
    if not pieces:
        raise errors.ErrBadPieceCount("minimum 2 pieces required for RLNC")
    return FullRLNCEncoder._create(lib().rlnc_encoder_create, ctx, FULL, b"".join(pieces),
                                   len(pieces), len(pieces[0]), rng=rng, batch=batch)


def NewFullRLNCEncoderWithPieceCount(data, pieceCount, ctx=None, rng=None, batch=16):
    """full/encoder.go:84-93."""
    return FullRLNCEncoder._create(lib().rlnc_encoder_create_with_piece_count, ctx, FULL, bytes(data),
                                   len(data), pieceCount, rng=rng, batch=batch)


def NewFullRLNCEncoderWithPieceSize(data, pieceSize, ctx=None, rng=None, batch=16):
    """full/encoder.go:98-107."""
    return FullRLNCEncoder._create(lib().rlnc_encoder_create_with_piece_size, ctx, FULL, bytes(data),
                                   len(data), pieceSize, rng=rng, batch=batch)


def NewFullRLNCRecoder(pieces, ctx=None, rng=None, batch=16):
    """full/recoder.go:52-57 -- pieces: list of CodedPiece."""
    flat = b"".join(p.Flatten() for p in pieces)
    k = len(pieces[0].Vector) if pieces else 0
    return NewFullRLNCRecoderWithFlattenData(flat, len(pieces), k, ctx=ctx, rng=rng, batch=batch)


def NewFullRLNCRecoderWithFlattenData(data, pieceCount, piecesCodedTogether, ctx=None, rng=None, batch=16):
    """full/recoder.go:63-70."""
    ctx = ctx or default_context()
    h = ctypes.c_void_p()
    arr, p = u8(bytes(data))
    errors.check(lib().rlnc_recoder_create(ctx.handle, p, len(data), pieceCount, piecesCodedTogether,
                                           ctypes.byref(h)))
    return FullRLNCRecoder(h, ctx, piecesCodedTogether, rng=rng, batch=batch)


def NewFullRLNCDecoder(pieceCount, ctx=None):
    """full/decoder.go:109-112."""
    return FullRLNCDecoder(pieceCount, ctx)
