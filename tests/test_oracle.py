"""Pin the CPU oracle (oracle/kodr_oracle.c) before trusting it.

1. The field tables equal the literal tables of kodr_internals/gf256/gf256.go:15-44
   (tests/golden/gf256_tables.json, text-parsed from the reference).
2. The reference's own known-answer tests: RREF / rank
   (kodr_internals/matrix/matrix_test.go:12-87), matrix multiply (:89-109),
   IsSystematic (kodr_internals/data_test.go:136-156), and the field
   property test (kodr_internals/gf256/gf256_test.go:11-40).
3. The seeded vectors of tests/golden/vectors.json, produced by an independent
   pure-Python transcription (tests/golden/gen_golden.py).
"""
import numpy as np
import pytest

import oracle

ERR = {None: 0, "ErrCannotInvertGf256AdditiveIndentity": 1, "ErrMatrixDimensionMismatch": 2,
       "ErrAllUsefulPiecesReceived": 3, "ErrMoreUsefulPiecesRequired": 4,
       "ErrPieceCountMoreThanTotalBytes": 6, "ErrZeroPieceSize": 7, "ErrBadPieceCount": 8,
       "ErrCodedDataLengthMismatch": 9, "ErrCodingVectorLengthMismatch": 10,
       "ErrPieceNotDecodedYet": 11, "ErrPieceOutOfBound": 12}


def h(s):
    return np.frombuffer(bytes.fromhex(s), dtype=np.uint8)


def test_tables_match_reference_literals(golden):
    log, exp = oracle.tables()
    t = golden["tables"]
    assert list(log) == t["LOG"]
    assert list(exp) == t["EXP"]


def test_field_properties():
    # gf256_test.go:11-40 over every pair instead of 100k random ones
    import ctypes
    lib = oracle.lib()
    for a in range(256):
        for b in range(256):
            m = lib.oracle_gf_mul(a, b)
            out = ctypes.c_uint8()
            st = lib.oracle_gf_div(m, b, ctypes.byref(out))
            if b == 0:
                assert st == 1
            else:
                assert st == 0 and out.value == a
            assert (a ^ b) ^ b == a


def test_rref_rank_kats(golden):
    for case in golden["kats"]["rref"]:
        coeffs, rank = oracle.rref_matrix(case["m"], case["coded_cols"])
        assert rank == case["rank"]
        assert coeffs.tolist() == case["rref"]


def test_matmul_kat(golden):
    kat = golden["kats"]["matmul"]
    st, out = oracle.matmul(kat["a"], kat["b"])
    assert st == 0 and out.tolist() == kat["expected"]
    st, _ = oracle.matmul(kat["bad_a"], kat["b"])
    assert st == ERR["ErrMatrixDimensionMismatch"]


def test_is_systematic_kat(golden):
    for case in golden["kats"]["is_systematic"]:
        v = np.array(case["vector"], np.uint8)
        assert bool(oracle.lib().oracle_is_systematic(oracle._p(v), v.size)) == case["expected"]


def test_encode_vectors(golden):
    for c in golden["vectors"]["encode"]:
        P = np.stack([h(p) for p in c["pieces"]])
        V = np.stack([h(v) for v in c["vectors"]])
        out = oracle.encode(P, V)
        assert [o.tobytes().hex() for o in out] == c["coded"]


def test_recode_vectors(golden):
    for c in golden["vectors"]["recode"]:
        flat = h(c["flat"]).reshape(c["n"], c["k"] + c["L"])
        R = np.stack([h(r) for r in c["r"]])
        out = oracle.recode(flat, c["k"], R)
        assert [o.tobytes().hex() for o in out] == c["out"]


def test_systematic_vectors(golden):
    lib = oracle.lib()
    for c in golden["vectors"]["systematic"]:
        k, L = c["k"], c["L"]
        P = np.stack([h(p) for p in c["pieces"]])
        V = np.stack([h(v) for v in c["random_vectors"]]).copy()
        out = np.empty((V.shape[0], L), np.uint8)
        lib.oracle_systematic_encode(oracle._p(P), k, L, 0, oracle._p(V), V.shape[0], oracle._p(out))
        got = [(V[i].tobytes() + out[i].tobytes()).hex() for i in range(V.shape[0])]
        assert got == c["out"]


def test_decode_traces(golden):
    for c in golden["vectors"]["decode"]:
        d = oracle.Decoder(c["k"])
        for (vh, ph), step in zip(c["stream"], c["steps"]):
            st = d.add(h(vh), h(ph))
            assert st == ERR[step["err"]], c["name"]
            assert (d.useful(), d.received(), d.required(), d.is_decoded()) == \
                (step["useful"], step["received"], step["required"], step["decoded"]), c["name"]
            for idx, (e, p) in enumerate(step.get("get", [])):
                gst, got = d.get_piece(idx)
                assert gst == ERR[e], (c["name"], idx)
                if p is not None:
                    assert got.tobytes().hex() == p
        if c["decoded"] is not None:
            for i, p in enumerate(c["decoded"]):
                st, got = d.get_piece(i)
                assert st == 0 and got.tobytes().hex() == p, c["name"]


def test_split_vectors(golden):
    import ctypes
    lib = oracle.lib()
    for c in golden["vectors"]["split_count"]:
        a, b = ctypes.c_size_t(), ctypes.c_size_t()
        st = lib.oracle_split_by_count(c["len"], c["count"], ctypes.byref(a), ctypes.byref(b))
        assert st == ERR[c["err"]]
        if st == 0:
            assert (a.value, b.value) == (c["piece_size"], c["padding"])
    for c in golden["vectors"]["split_size"]:
        a, b = ctypes.c_size_t(), ctypes.c_size_t()
        st = lib.oracle_split_by_size(c["len"], c["size"], ctypes.byref(a), ctypes.byref(b))
        assert st == ERR[c["err"]]
        if st == 0:
            assert (a.value, b.value) == (c["piece_count"], c["padding"])


@pytest.mark.parametrize("seed", range(3))
def test_decode_round_trip_random(seed):
    # full/encoder_test.go:34-77 shape of flow at a small size
    rng = np.random.default_rng(seed)
    k, L = 24, 96
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    d = oracle.Decoder(k)
    while not d.is_decoded():
        v = rng.integers(0, 256, (1, k), dtype=np.uint8)
        d.add(v[0], oracle.encode(P, v)[0])
    for i in range(k):
        st, got = d.get_piece(i)
        assert st == 0 and np.array_equal(got, P[i])
