"""ctypes loader for the CPU restatement of kodr (oracle/kodr_oracle.c).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, always as the checker / the timed kodr-equivalent
scalar path, never as a product code path.  kodr_amd never imports this.
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
SO = os.path.join(HERE, "liboracle.so")

_u8p = ctypes.POINTER(ctypes.c_uint8)
_sz = ctypes.c_size_t
_szp = ctypes.POINTER(ctypes.c_size_t)

_SIG = {
    "oracle_tables": (None, [_u8p, _u8p]),
    "oracle_gf_mul": (ctypes.c_uint8, [ctypes.c_uint8, ctypes.c_uint8]),
    "oracle_gf_inv": (ctypes.c_int, [ctypes.c_uint8, _u8p]),
    "oracle_gf_div": (ctypes.c_int, [ctypes.c_uint8, ctypes.c_uint8, _u8p]),
    "oracle_piece_multiply": (None, [_u8p, _u8p, _sz, ctypes.c_uint8]),
    "oracle_split_by_count": (ctypes.c_int, [_sz, _sz, _szp, _szp]),
    "oracle_split_by_size": (ctypes.c_int, [_sz, _sz, _szp, _szp]),
    "oracle_is_systematic": (ctypes.c_int, [_u8p, _sz]),
    "oracle_coded_pieces_for_recoding": (ctypes.c_int, [_sz, _sz, _sz, _szp]),
    "oracle_encode": (None, [_u8p, _sz, _sz, _u8p, _sz, _u8p]),
    "oracle_matmul": (ctypes.c_int, [_u8p, _sz, _sz, _u8p, _sz, _sz, _u8p]),
    "oracle_recode": (ctypes.c_int, [_u8p, _sz, _sz, _sz, _u8p, _sz, _u8p]),
    "oracle_systematic_encode": (None, [_u8p, _sz, _sz, _sz, _u8p, _sz, _u8p]),
    "oracle_decoder_new": (ctypes.c_void_p, [_sz]),
    "oracle_decoder_free": (None, [ctypes.c_void_p]),
    "oracle_ds_from_matrix": (ctypes.c_void_p, [_u8p, _sz, _sz, _u8p, _sz]),
    "oracle_ds_rref": (None, [ctypes.c_void_p]),
    "oracle_ds_rows": (_sz, [ctypes.c_void_p]),
    "oracle_ds_cols": (_sz, [ctypes.c_void_p]),
    "oracle_ds_coeffs": (None, [ctypes.c_void_p, _u8p]),
    "oracle_ds_coded": (None, [ctypes.c_void_p, _u8p]),
    "oracle_decoder_is_decoded": (ctypes.c_int, [ctypes.c_void_p]),
    "oracle_decoder_required": (_sz, [ctypes.c_void_p]),
    "oracle_decoder_useful": (_sz, [ctypes.c_void_p]),
    "oracle_decoder_received": (_sz, [ctypes.c_void_p]),
    "oracle_decoder_piece_length": (_sz, [ctypes.c_void_p]),
    "oracle_decoder_add_piece": (ctypes.c_int, [ctypes.c_void_p, _u8p, _sz, _u8p, _sz]),
    "oracle_decoder_get_piece": (ctypes.c_int, [ctypes.c_void_p, _sz, _u8p]),
    "oracle_decoder_get_pieces": (ctypes.c_int, [ctypes.c_void_p, _u8p]),
}

_lib = None


def build():
    r = subprocess.run(["make", "-s", "-C", HERE], capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("oracle build failed: " + r.stdout + r.stderr)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(SO) or os.path.getmtime(SO) < os.path.getmtime(os.path.join(HERE, "kodr_oracle.c")):
            build()
        h = ctypes.CDLL(SO)
        for name, (res, args) in _SIG.items():
            f = getattr(h, name)
            f.restype = res
            f.argtypes = args
        _lib = h
    return _lib


def _p(a):
    return a.ctypes.data_as(_u8p)


def _arr(b):
    a = b if isinstance(b, np.ndarray) else np.frombuffer(bytes(b), dtype=np.uint8)
    return np.ascontiguousarray(a, dtype=np.uint8)


def tables():
    log, exp = np.zeros(256, np.uint8), np.zeros(510, np.uint8)
    lib().oracle_tables(_p(log), _p(exp))
    return log, exp


def gf_mul(a, b):
    return int(lib().oracle_gf_mul(a, b))


def encode(pieces, vectors):
    """pieces (k, L) uint8, vectors (B, k) -> (B, L): full/encoder.go:61-71."""
    P = np.ascontiguousarray(pieces, dtype=np.uint8)
    V = np.ascontiguousarray(vectors, dtype=np.uint8)
    k, L = P.shape
    B = V.shape[0]
    out = np.empty((B, L), np.uint8)
    lib().oracle_encode(_p(P), k, L, _p(V), B, _p(out))
    return out


def matmul(a, b):
    A = np.ascontiguousarray(a, dtype=np.uint8)
    Bm = np.ascontiguousarray(b, dtype=np.uint8)
    out = np.empty((A.shape[0], Bm.shape[1]), np.uint8)
    st = lib().oracle_matmul(_p(A), A.shape[0], A.shape[1], _p(Bm), Bm.shape[0], Bm.shape[1], _p(out))
    return st, out


def recode(flat_rows, k, r):
    """flat_rows (n, k+L) wire rows, r (B, n) -> (B, k+L): full/recoder.go:27-46."""
    F = np.ascontiguousarray(flat_rows, dtype=np.uint8)
    R = np.ascontiguousarray(r, dtype=np.uint8)
    n, clen = F.shape
    out = np.empty((R.shape[0], clen), np.uint8)
    st = lib().oracle_recode(_p(F), n, k, clen, _p(R), R.shape[0], _p(out))
    assert st == 0
    return out


class Decoder:
    """full/decoder.go over the literal decoder_state.go restatement."""

    def __init__(self, k):
        self._h = lib().oracle_decoder_new(k)
        self.k = k

    def __del__(self):
        try:
            lib().oracle_decoder_free(self._h)
        except Exception:
            pass

    def add(self, vec, piece):
        v, p = _arr(vec), _arr(piece)
        return lib().oracle_decoder_add_piece(self._h, _p(v), v.size, _p(p), p.size)

    def useful(self):
        return lib().oracle_decoder_useful(self._h)

    def received(self):
        return lib().oracle_decoder_received(self._h)

    def required(self):
        return lib().oracle_decoder_required(self._h)

    def is_decoded(self):
        return bool(lib().oracle_decoder_is_decoded(self._h))

    def rows(self):
        return lib().oracle_ds_rows(self._h)

    def coeffs(self):
        r, c = lib().oracle_ds_rows(self._h), lib().oracle_ds_cols(self._h)
        out = np.empty((r, c), np.uint8)
        if r:
            lib().oracle_ds_coeffs(self._h, _p(out))
        return out

    def coded(self):
        r, L = lib().oracle_ds_rows(self._h), lib().oracle_decoder_piece_length(self._h)
        out = np.empty((r, L), np.uint8)
        if r:
            lib().oracle_ds_coded(self._h, _p(out))
        return out

    def get_piece(self, idx):
        L = lib().oracle_decoder_piece_length(self._h)
        out = np.empty(max(L, 1), np.uint8)
        st = lib().oracle_decoder_get_piece(self._h, idx, _p(out))
        return st, (out[:L].copy() if st == 0 else None)


def rref_matrix(m, coded_cols):
    """NewDecoderState(m, zeros) + Rref (matrix_test.go:18-20) -> (coeffs, rank)."""
    M = np.ascontiguousarray(m, dtype=np.uint8)
    Z = np.zeros((M.shape[0], coded_cols), np.uint8)
    h = lib().oracle_ds_from_matrix(_p(M), M.shape[0], M.shape[1], _p(Z), coded_cols)
    lib().oracle_ds_rref(h)
    r = lib().oracle_ds_rows(h)
    out = np.empty((r, M.shape[1]), np.uint8)
    if r:
        lib().oracle_ds_coeffs(h, _p(out))
    lib().oracle_decoder_free(h)
    return out, r
