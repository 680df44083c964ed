"""Mirror of kodr_internals (kodr_internals/data.go) over the C ABI.

Pieces and vectors are ``bytes``.  Splitting and validation follow
data.go:103-193 exactly (the C ABI does the arithmetic, errors map to
kodr_amd.errors).  Unlike kodr, nothing aliases the caller's buffers.
"""
import ctypes
import os

from . import errors
from ._lib import lib, u8

Piece = bytes
CodingVector = bytes


class CodedPiece:
    """data.go:38-41 -- a coded piece and the vector that produced it."""

    __slots__ = ("Vector", "Piece")

    def __init__(self, Vector, Piece):
        self.Vector = bytes(Vector)
        self.Piece = bytes(Piece)

    def Len(self):  # data.go:44-46
        return len(self.Vector) + len(self.Piece)

    def Flatten(self):  # data.go:52-57
        return self.Vector + self.Piece

    def IsSystematic(self):  # data.go:64-84
        a, p = u8(self.Vector)
        return bool(lib().rlnc_is_systematic(p, len(self.Vector))) if self.Vector else False

    def __repr__(self):
        return f"CodedPiece(k={len(self.Vector)}, L={len(self.Piece)})"


def GenerateCodingVector(n, rng=None):
    """data.go:90-95 -- n uniform bytes from the OS CSPRNG (crypto/rand).
    ``rng(n) -> bytes`` may be injected for reproducible tests."""
    return bytes(rng(n)) if rng is not None else os.urandom(n)


def split_by_piece_size(length, piece_size):
    """(pieceCount, padding) per data.go:103-132."""
    c, pad = ctypes.c_size_t(), ctypes.c_size_t()
    errors.check(lib().rlnc_split_by_piece_size(length, piece_size, ctypes.byref(c), ctypes.byref(pad)))
    return c.value, pad.value


def split_by_piece_count(length, piece_count):
    """(pieceSize, padding) per data.go:137-166."""
    s, pad = ctypes.c_size_t(), ctypes.c_size_t()
    errors.check(lib().rlnc_split_by_piece_count(length, piece_count, ctypes.byref(s), ctypes.byref(pad)))
    return s.value, pad.value


def _split(data, size, count):
    data = bytes(data)
    padded = data + bytes(size * count - len(data))
    return [padded[i * size:(i + 1) * size] for i in range(count)]


def OriginalPiecesFromDataAndPieceSize(data, pieceSize):
    """data.go:103-132 -> (pieces, padding)."""
    count, pad = split_by_piece_size(len(data), pieceSize)
    return _split(data, pieceSize, count), pad


def OriginalPiecesFromDataAndPieceCount(data, pieceCount):
    """data.go:137-166 -> (pieces, padding)."""
    size, pad = split_by_piece_count(len(data), pieceCount)
    return _split(data, size, pieceCount), pad


def CodedPiecesForRecoding(data, pieceCount, piecesCodedTogether):
    """data.go:173-193 -> list of CodedPiece views of a flattened buffer."""
    cpl = ctypes.c_size_t()
    errors.check(lib().rlnc_coded_pieces_for_recoding(len(data), pieceCount, piecesCodedTogether,
                                                      ctypes.byref(cpl)))
    n = cpl.value
    data = bytes(data)
    return [CodedPiece(data[i * n:i * n + piecesCodedTogether], data[i * n + piecesCodedTogether:(i + 1) * n])
            for i in range(pieceCount)]
