"""kodr's RREF and rank known-answer tests (kodr_internals/matrix/
matrix_test.go:12-87) run through the PRODUCT's decoder core -- the C ABI's
AddPiece / batched AddPiece with ctx = NULL (coefficient side only, no GPU) --
not only through the oracle (tests/test_oracle.py).

kodr's test builds a DecoderState from all rows and calls Rref once; a
decoder receives the rows one AddPiece at a time, each followed by Rref
(full/decoder.go:50-66).  For these matrices both end in the same state: the
reduced row echelon form is unique, the dependent row of the first KAT is
removed as all-zero (decoder_state.go:136-165), and rank = rows kept.
"""
import ctypes

import numpy as np
import pytest

from kodr_amd import _lib, errors

U8P = _lib._u8p


def decoder(k):
    h = ctypes.c_void_p()
    errors.check(_lib.lib().rlnc_decoder_create(None, k, ctypes.byref(h)))
    return h


def coefficients(h, k):
    L = _lib.lib()
    n = L.rlnc_decoder_useful(h)
    out = np.zeros((max(n, 1), k), np.uint8)
    errors.check(L.rlnc_decoder_coefficients(h, out.ctypes.data_as(U8P)))
    return out[:n]


@pytest.mark.parametrize("batched", [False, True])
def test_rref_rank_kats_through_decoder(golden, batched):
    lib = _lib.lib()
    for case in golden["kats"]["rref"]:
        m = np.array(case["m"], np.uint8)
        rows, k = m.shape
        h = decoder(k)
        try:
            piece = np.zeros(1, np.uint8)   # coefficient side only: any piece length
            if batched:
                wire = np.concatenate([m, np.zeros((rows, 1), np.uint8)], axis=1)
                used = ctypes.c_size_t()
                st = lib.rlnc_decoder_add_pieces(h, wire.ctypes.data, rows, k + 1, 1, 0, ctypes.byref(used))
                assert st in (0, 3) and used.value <= rows
            else:
                for r in range(rows):
                    v = np.ascontiguousarray(m[r])
                    st = lib.rlnc_decoder_add_piece(h, v.ctypes.data_as(U8P), k, piece.ctypes.data_as(U8P), 1)
                    assert st in (0, 3)
            got = coefficients(h, k)
            assert got.tolist() == case["rref"], case["m"]
            assert lib.rlnc_decoder_useful(h) == case["rank"]
            assert bool(lib.rlnc_decoder_is_decoded(h)) == (case["rank"] == k)
        finally:
            lib.rlnc_decoder_destroy(h)
