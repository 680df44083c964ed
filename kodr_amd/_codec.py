"""Shared encoder / recoder / decoder machinery behind full.py and systematic.py.

Each object owns one C-ABI handle on a device Context.  Encoders and recoders
draw coding vectors on the host (crypto/rand analogue, injectable) and fetch
coded pieces from the device in batches of ``batch`` consecutive
CodedPiece() calls; the returned sequence is exactly what one-at-a-time calls
would return, since every piece carries its own vector.
"""
import ctypes
from collections import deque

import numpy as np

from . import errors
from ._lib import lib, u8
from .device import default_context
from .kodr_internals import CodedPiece, GenerateCodingVector

FULL, SYSTEMATIC = 0, 1


def _u8arr(b):
    return np.frombuffer(bytes(b), dtype=np.uint8)


class _Encoder:
    def __init__(self, handle, ctx, rng=None, batch=16):
        self._h = handle
        self._ctx = ctx
        self._rng = rng
        self._batch = max(1, int(batch))
        self._queue = deque()

    @classmethod
    def _create(cls, fn, ctx, kind, buf, a, b, **kw):
        ctx = ctx or default_context()
        h = ctypes.c_void_p()
        arr, p = u8(buf)
        errors.check(fn(ctx.handle, kind, p, a, b, ctypes.byref(h)))
        return cls(h, ctx, **kw)

    def __del__(self):
        try:
            if self._h:
                lib().rlnc_encoder_destroy(self._h)
                self._h = None
        except Exception:
            pass

    # accessors: full/encoder.go:15-55, systematic/encoder.go:16-56
    def PieceCount(self):
        return lib().rlnc_encoder_piece_count(self._h)

    def PieceSize(self):
        return lib().rlnc_encoder_piece_size(self._h)

    def DecodableLen(self):
        return lib().rlnc_encoder_decodable_len(self._h)

    def CodedPieceLen(self):
        return lib().rlnc_encoder_coded_piece_len(self._h)

    def Padding(self):
        return lib().rlnc_encoder_padding(self._h)

    def device_pieces(self):
        pitch = ctypes.c_size_t()
        ptr = lib().rlnc_encoder_device_pieces(self._h, ctypes.byref(pitch))
        return ptr, pitch.value

    def coded_pieces(self, vectors):
        """Run len(vectors)//k consecutive CodedPiece() calls with the given
        vectors (bytes, count*k).  Returns (vectors_used, wire_rows) as numpy
        arrays; systematic encoders overwrite the vectors they emit as e_i."""
        k, clen = self.PieceCount(), self.CodedPieceLen()
        vec = np.array(_u8arr(vectors), dtype=np.uint8)
        count = vec.size // k
        out = np.empty(count * clen, dtype=np.uint8)
        if count:
            errors.check(lib().rlnc_encoder_coded_pieces(
                self._h, vec.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), count,
                out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))))
        return vec.reshape(count, k), out.reshape(count, clen)

    def compact(self):
        """Extension (rlnc_encoder_compact): keep only the bit-sliced copy of
        the generation in HBM; device_pieces() is then (None, pitch)."""
        errors.check(lib().rlnc_encoder_compact(self._h))

    def seed(self, seed):
        """Reseed the device-side vector stream of coded_wire_device."""
        errors.check(lib().rlnc_encoder_seed(self._h, ctypes.c_uint64(seed)))

    def coded_wire_device(self, count, d_wire, pitch):
        """`count` coded pieces in wire layout (vector ++ piece) written to
        device rows d_wire at `pitch`, vectors drawn on the device."""
        errors.check(lib().rlnc_encoder_coded_wire_device(self._h, count, ctypes.c_void_p(d_wire), pitch))

    def CodedPiece(self):
        """full/encoder.go:61-71 / systematic/encoder.go:82-109."""
        if not self._queue:
            k = self.PieceCount()
            vec = b"".join(GenerateCodingVector(k, self._rng) for _ in range(self._batch))
            vecs, rows = self.coded_pieces(vec)
            for v, r in zip(vecs, rows):
                self._queue.append(CodedPiece(v.tobytes(), r[k:].tobytes()))
        return self._queue.popleft()


class _Recoder:
    """full/recoder.go."""

    def __init__(self, handle, ctx, k, rng=None, batch=16):
        self._h = handle
        self._ctx = ctx
        self._k = k          # pieces coded together: the vector part of a wire row
        self._rng = rng
        self._batch = max(1, int(batch))
        self._queue = deque()

    def __del__(self):
        try:
            if self._h:
                lib().rlnc_recoder_destroy(self._h)
                self._h = None
        except Exception:
            pass

    def PieceCount(self):
        return lib().rlnc_recoder_piece_count(self._h)

    def CodedPieceLen(self):
        return lib().rlnc_recoder_coded_piece_len(self._h)

    def recode(self, r):
        """count consecutive CodedPiece() calls with caller-supplied recoding
        vectors r (count*n bytes) -> wire rows (count, k+L)."""
        n, clen = self.PieceCount(), self.CodedPieceLen()
        rv = np.array(_u8arr(r), dtype=np.uint8)
        count = rv.size // n
        out = np.empty(count * clen, dtype=np.uint8)
        if count:
            errors.check(lib().rlnc_recoder_coded_pieces(
                self._h, rv.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), count,
                out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))))
        return out.reshape(count, clen)

    def compact(self):
        """Extension (rlnc_recoder_compact): keep only the bit-sliced copy."""
        errors.check(lib().rlnc_recoder_compact(self._h))

    def CodedPiece(self):
        """full/recoder.go:27-46 -> CodedPiece(Vector = r x C, Piece = sum r_i P_i)."""
        if not self._queue:
            n = self.PieceCount()
            r = b"".join(GenerateCodingVector(n, self._rng) for _ in range(self._batch))
            rows = self.recode(r)
            kk = self._k
            for row in rows:
                self._queue.append(CodedPiece(row[:kk].tobytes(), row[kk:].tobytes()))
        return self._queue.popleft()


class _Decoder:
    """full/decoder.go (== systematic/decoder.go)."""

    def __init__(self, pieceCount, ctx=None):
        self._ctx = ctx or default_context()
        h = ctypes.c_void_p()
        errors.check(lib().rlnc_decoder_create(self._ctx.handle, pieceCount, ctypes.byref(h)))
        self._h = h
        self._k = pieceCount

    def __del__(self):
        try:
            if self._h:
                lib().rlnc_decoder_destroy(self._h)
                self._h = None
        except Exception:
            pass

    def PieceLength(self):  # full/decoder.go:18-25
        return lib().rlnc_decoder_piece_length(self._h)

    def IsDecoded(self):  # :32-34
        return bool(lib().rlnc_decoder_is_decoded(self._h))

    def Required(self):  # :38-40
        return lib().rlnc_decoder_required(self._h)

    def useful(self):
        return lib().rlnc_decoder_useful(self._h)

    def received(self):
        return lib().rlnc_decoder_received(self._h)

    def AddPiece(self, piece):  # :50-66
        va, vp = u8(piece.Vector)
        pa, pp = u8(piece.Piece)
        errors.check(lib().rlnc_decoder_add_piece(self._h, vp, len(piece.Vector), pp, len(piece.Piece)))

    def add_wire_rows(self, rows):
        """AddPiece over each row of a (count, k + L) uint8 array of flattened
        coded pieces (kodr_internals/coded.go Flatten), in one C-ABI call.
        Returns the number of pieces accepted; stops quietly once decoded."""
        rows = np.ascontiguousarray(rows, dtype=np.uint8)
        if rows.ndim != 2:
            raise ValueError("rows must be a 2-D array of wire rows")
        return self._add_rows(rows.ctypes.data, rows.shape[0], rows.shape[1], rows.shape[1] - self._k, False)

    def add_wire_rows_device(self, d_rows, count, pitch, piece_len):
        """Same, with the wire rows resident on the device (pointer, row pitch)."""
        return self._add_rows(d_rows, count, pitch, piece_len, True)

    def _add_rows(self, ptr, count, pitch, piece_len, dev):
        consumed = ctypes.c_size_t()
        st = lib().rlnc_decoder_add_pieces(self._h, ctypes.c_void_p(ptr), count, pitch, piece_len, int(dev),
                                           ctypes.byref(consumed))
        if st != 3:
            errors.check(st)
        return consumed.value

    def GetPiece(self, i):  # :77-79
        L = self.PieceLength()
        out = np.empty(max(L, 1), dtype=np.uint8)
        errors.check(lib().rlnc_decoder_get_piece(self._h, i, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))))
        return out[:L].tobytes()

    def GetPieces(self):  # :83-99
        if not self.IsDecoded():
            raise errors.ErrMoreUsefulPiecesRequired("not enough pieces received yet to decode")
        L, n = self.PieceLength(), self.useful()
        out = np.empty(max(L * n, 1), dtype=np.uint8)
        errors.check(lib().rlnc_decoder_get_pieces(self._h, out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8))))
        return [out[i * L:(i + 1) * L].tobytes() for i in range(n)]

    # extensions (no kodr counterpart): pieces decoded before full rank
    def set_policy(self, eager):
        """EAGER (True): every AddPiece materializes the pieces it decoded."""
        errors.check(lib().rlnc_decoder_set_policy(self._h, 1 if eager else 0))

    def decoded_mask(self):
        m = np.zeros(max(self._k, 1), dtype=np.uint8)
        lib().rlnc_decoder_decoded_mask(self._h, m.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)))
        return m[:self._k].astype(bool)

    def GetDecodedPiece(self, i):
        """Original piece i if it is decoded now (a systematic piece on
        arrival, any piece at full rank), else ErrPieceNotDecodedYet."""
        L = self.PieceLength()
        out = np.empty(max(L, 1), dtype=np.uint8)
        errors.check(lib().rlnc_decoder_get_decoded(self._h, i, ctypes.c_void_p(out.ctypes.data), 0))
        return out[:L].tobytes()

    def bind_output(self, d_out, pitch):
        """Decoded pieces land at row j of the device buffer d_out (None unbinds)."""
        errors.check(lib().rlnc_decoder_bind_output(self._h, None if d_out is None else ctypes.c_void_p(d_out), pitch))

    def elim_stats(self):
        """Which route eliminated this decoder's batches (rlnc_decoder_elim_stats)."""
        return elim_stats(self._h)


def elim_stats(h):
    """rlnc_decoder_elim_stats of a decoder handle as a dict: gpu, gpu_retried,
    host_after_gpu, host."""
    v = [ctypes.c_size_t() for _ in range(4)]
    errors.check(lib().rlnc_decoder_elim_stats(h, *[ctypes.byref(x) for x in v]))
    return dict(zip(("gpu", "gpu_retried", "host_after_gpu", "host"), (x.value for x in v)))


def flush_decoders(decoders):
    """Extension (no kodr counterpart): the pending AddPiece calls of many
    decoders (one context, one piece count), eliminated together -- every
    queue that completes its decoder's rank in one GPU launch
    (rlnc_decoders_flush_gpu), the rest as each decoder's next read would.
    A receiver keeping kodr's one-AddPiece-per-piece loop calls it once per
    tick; the decoders' observable state is the same either way."""
    decoders = list(decoders)
    if not decoders:
        return
    arr = (ctypes.c_void_p * len(decoders))(*[d._h.value for d in decoders])
    errors.check(lib().rlnc_decoders_flush_gpu(arr, len(decoders)))
