"""CPU tests of libkodr_rlnc.so: it loads, exports every symbol of
include/kodr_rlnc.h, and its host logic matches kodr:

- splitting / validation rules (data.go:103-193) vs the golden vectors;
- the mirrored decoder state (decoder_state.go + full/decoder.go) run
  coefficient-side only (ctx = NULL, no GPU): per-AddPiece counters, errors and
  coefficient matrix equal the oracle's literal restatement, and the tracked
  transform T satisfies  T x received == the oracle's coded rows  exactly, on
  the golden streams and on randomized / adversarial streams.

No data-plane compute is called here (that needs the GPU: test_gpu_*.py).
"""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle
from kodr_amd import _lib, errors

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ERR = {None: 0, **{name: cls.code for name, cls in errors.BY_NAME.items()}}


def h(s):
    return np.frombuffer(bytes.fromhex(s), dtype=np.uint8)


def header_symbols():
    src = open(os.path.join(ROOT, "include", "kodr_rlnc.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rlnc_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    lib = _lib.lib()
    syms = header_symbols()
    assert len(syms) > 50
    for s in syms:
        assert hasattr(lib, s), s
    # the ctypes binding declares exactly the header's entry points
    assert sorted(_lib.SIGNATURES) == syms


def test_exported_symbols_via_nm():
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(re.findall(r"\bT (rlnc_\w+)", out))
    assert set(header_symbols()) <= exported


def test_library_does_not_link_oracle():
    import subprocess
    out = subprocess.run(["ldd", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle" not in out
    nm = subprocess.run(["nm", "-D", _lib.LIB_PATH], capture_output=True, text=True).stdout
    assert "oracle_" not in nm


def test_status_strings_match_errors_go():
    lib = _lib.lib()
    assert lib.rlnc_status_string(3).decode() == "no more pieces required for decoding"
    assert lib.rlnc_status_string(12).decode().startswith("requested piece index >= pieceCount")
    for name, code in ERR.items():
        if name:
            assert errors.BY_CODE[code].__name__ == name


def test_split_rules(golden):
    lib = _lib.lib()
    for c in golden["vectors"]["split_count"]:
        a, b = ctypes.c_size_t(), ctypes.c_size_t()
        st = lib.rlnc_split_by_piece_count(c["len"], c["count"], ctypes.byref(a), ctypes.byref(b))
        assert st == ERR[c["err"]], c
        if st == 0:
            assert (a.value, b.value) == (c["piece_size"], c["padding"])
    for c in golden["vectors"]["split_size"]:
        a, b = ctypes.c_size_t(), ctypes.c_size_t()
        st = lib.rlnc_split_by_piece_size(c["len"], c["size"], ctypes.byref(a), ctypes.byref(b))
        assert st == ERR[c["err"]], c
        if st == 0:
            assert (a.value, b.value) == (c["piece_count"], c["padding"])


def test_coded_pieces_for_recoding_rules():
    # data_test.go:88-134 shapes: 5 coded pieces of 3+2 bytes
    lib = _lib.lib()
    n = ctypes.c_size_t()
    assert lib.rlnc_coded_pieces_for_recoding(25, 3, 3, ctypes.byref(n)) == ERR["ErrCodedDataLengthMismatch"]
    assert lib.rlnc_coded_pieces_for_recoding(25, 5, 5, ctypes.byref(n)) == ERR["ErrCodingVectorLengthMismatch"]
    assert lib.rlnc_coded_pieces_for_recoding(25, 5, 3, ctypes.byref(n)) == 0 and n.value == 5


def test_is_systematic(golden):
    lib = _lib.lib()
    for c in golden["kats"]["is_systematic"]:
        a, p = _lib.u8(bytes(c["vector"]))
        assert bool(lib.rlnc_is_systematic(p, a.size)) == c["expected"]


class CoreDecoder:
    """rlnc_decoder with ctx = NULL: the coefficient side only."""

    def __init__(self, k):
        self.lib = _lib.lib()
        self.h = ctypes.c_void_p()
        assert self.lib.rlnc_decoder_create(None, k, ctypes.byref(self.h)) == 0
        self.k = k

    def __del__(self):
        self.lib.rlnc_decoder_destroy(self.h)

    def add(self, vec):
        a, p = _lib.u8(vec)
        return self.lib.rlnc_decoder_add_piece(self.h, p, a.size, None, 0)

    def state(self):
        L = self.lib
        return (L.rlnc_decoder_useful(self.h), L.rlnc_decoder_received(self.h),
                L.rlnc_decoder_required(self.h), bool(L.rlnc_decoder_is_decoded(self.h)))

    def coefficients(self):
        r = self.lib.rlnc_decoder_useful(self.h)
        out = np.empty((r, self.k), np.uint8)
        if r:
            self.lib.rlnc_decoder_coefficients(self.h, out.ctypes.data_as(_lib._u8p))
        return out

    def transform(self):
        r, n = self.lib.rlnc_decoder_useful(self.h), self.lib.rlnc_decoder_received(self.h)
        out = np.empty((r, n), np.uint8)
        if r:
            self.lib.rlnc_decoder_transform(self.h, out.ctypes.data_as(_lib._u8p))
        return out


def check_stream(k, stream, strict_steps=None):
    """Feed (vec, piece) pairs to the C-ABI core and to the oracle; compare."""
    core, ref = CoreDecoder(k), oracle.Decoder(k)
    accepted = []
    for n, (v, p) in enumerate(stream):
        st_ref = ref.add(v, p)
        st = core.add(v)
        assert st == st_ref, n
        if st == 0:
            accepted.append(np.asarray(p, np.uint8))
        assert core.state() == (ref.useful(), ref.received(), ref.required(), ref.is_decoded()), n
        if strict_steps is not None:
            s = strict_steps[n]
            assert core.state() == (s["useful"], s["received"], s["required"], s["decoded"])
        if core.state()[0] == 0 or st != 0:
            continue
        # coefficient halves identical; data half == T x R exactly
        assert np.array_equal(core.coefficients(), ref.coeffs()), n
        T = core.transform()
        R = np.stack(accepted)
        st_m, TR = oracle.matmul(T, R)
        assert st_m == 0
        assert np.array_equal(TR, ref.coded()), n
    return core, ref


def test_core_matches_oracle_on_golden_streams(golden):
    for c in golden["vectors"]["decode"]:
        stream = [(h(v), h(p)) for v, p in c["stream"]]
        check_stream(c["k"], stream, c["steps"])


def _random_stream(rng, k, L, n, kind):
    P = rng.integers(0, 256, (k, L), dtype=np.uint8)
    out = []
    for i in range(n):
        if kind == "dense":
            v = rng.integers(0, 256, k, dtype=np.uint8)
        elif kind == "sparse":
            v = (rng.integers(0, 256, k) * (rng.random(k) < 0.15)).astype(np.uint8)
        elif kind == "tiny_field":  # many zeros / duplicates / dependencies
            v = rng.integers(0, 3, k, dtype=np.uint8)
        elif kind == "systematic":
            v = np.zeros(k, np.uint8)
            if rng.random() < 0.6:
                v[rng.integers(0, k)] = 1
            else:
                v[:] = rng.integers(0, 256, k)
        elif kind == "lowrank":  # combinations of only k//2 base vectors
            base = np.random.default_rng(7).integers(0, 256, (max(1, k // 2), k), dtype=np.uint8)
            c = rng.integers(0, 256, (1, base.shape[0]), dtype=np.uint8)
            v = oracle.matmul(c, base)[1][0]
        out.append((v, oracle.encode(P, v[None, :])[0]))
    return out


@pytest.mark.parametrize("kind", ["dense", "sparse", "tiny_field", "systematic", "lowrank"])
@pytest.mark.parametrize("k", [2, 3, 7, 16, 33])
def test_core_matches_oracle_randomized(kind, k):
    rng = np.random.default_rng(1000 * k + sum(map(ord, kind)))
    stream = _random_stream(rng, k, 8, 3 * k + 4, kind)
    check_stream(k, stream)


def test_core_arbitrary_rows_not_codewords():
    # pieces inconsistent with their vectors: T-tracking must still equal
    # kodr's in-place data rows bit for bit
    rng = np.random.default_rng(5)
    k = 12
    stream = [(rng.integers(0, 4, k, dtype=np.uint8), rng.integers(0, 256, 10, dtype=np.uint8))
              for _ in range(40)]
    check_stream(k, stream)


def test_core_k256_counters_only():
    # C2 shape on the coefficient side: 256 random vectors reach full rank
    rng = np.random.default_rng(11)
    k = 256
    core, ref = CoreDecoder(k), oracle.Decoder(k)
    while not ref.is_decoded():
        v = rng.integers(0, 256, k, dtype=np.uint8)
        assert core.add(v) == ref.add(v, np.zeros(1, np.uint8))
        assert core.state() == (ref.useful(), ref.received(), ref.required(), ref.is_decoded())
    assert np.array_equal(core.coefficients(), np.eye(k, dtype=np.uint8))
    assert core.add(rng.integers(0, 256, k, dtype=np.uint8)) == ERR["ErrAllUsefulPiecesReceived"]


def test_core_vector_length_mismatch_is_rejected():
    core = CoreDecoder(4)
    a, p = _lib.u8(b"\x01\x02\x03")
    assert _lib.lib().rlnc_decoder_add_piece(core.h, p, 3, None, 0) == -1


def test_get_piece_without_device_reports_no_device():
    core = CoreDecoder(2)
    core.add(np.array([1, 0], np.uint8))
    core.add(np.array([0, 1], np.uint8))
    out = np.empty(4, np.uint8)
    assert _lib.lib().rlnc_decoder_get_piece(core.h, 0, out.ctypes.data_as(_lib._u8p)) == -4
    assert _lib.lib().rlnc_decoder_get_piece(core.h, 5, out.ctypes.data_as(_lib._u8p)) == 12


@pytest.mark.parametrize("seed", range(40))
def test_core_fuzz_mixed_streams(seed):
    # every step draws from a different generator: zero rows, unit vectors,
    # duplicates of earlier rows, tiny-field noise and dense rows, so the
    # fast-path invariants (dirty rows, clean columns, touched rows) are hit
    # in all orders
    rng = np.random.default_rng(7000 + seed)
    k = int(rng.integers(2, 40))
    L = 4
    seen = []
    stream = []
    for _ in range(4 * k + 8):
        kind = rng.integers(0, 6)
        if kind == 0:
            v = np.zeros(k, np.uint8)
        elif kind == 1:
            v = np.zeros(k, np.uint8)
            v[rng.integers(0, k)] = rng.integers(1, 256)
        elif kind == 2 and seen:
            v = seen[rng.integers(0, len(seen))].copy()
        elif kind == 3:
            v = rng.integers(0, 2, k, dtype=np.uint8)
        else:
            v = rng.integers(0, 256, k, dtype=np.uint8)
        seen.append(v)
        stream.append((v, rng.integers(0, 256, L, dtype=np.uint8)))
    check_stream(k, stream)


@pytest.mark.parametrize("seed", range(30))
def test_core_systematic_order_streams(seed):
    # systematic pieces in encoder order with losses (and sometimes scaled,
    # duplicated, or interrupted by coded or zero rows), then coded pieces:
    # the unit-row bookkeeping (append without a pass, two-byte row
    # operations from unit pivots, sparse column scans) against the oracle
    # after every AddPiece
    rng = np.random.default_rng(8800 + seed)
    k = int(rng.choice([3, 8, 17, 40, 64]))
    lost = set(rng.choice(k, int(rng.integers(0, k // 3 + 2)), replace=False).tolist())
    rows = []
    for i in range(k):
        if i in lost:
            continue
        v = np.zeros(k, np.uint8)
        v[i] = 1 if rng.random() < 0.8 else rng.integers(2, 256)
        rows.append(v)
        r = rng.random()
        if r < 0.05:
            rows.append(v.copy())                       # duplicate systematic piece
        elif r < 0.08:
            rows.append(rng.integers(0, 256, k, dtype=np.uint8))  # coded piece in between
        elif r < 0.10:
            rows.append(np.zeros(k, np.uint8))
    rows += [rng.integers(0, 256 if seed % 3 else 3, k, dtype=np.uint8) for _ in range(len(lost) + 4)]
    stream = [(v, rng.integers(0, 256, 6, dtype=np.uint8)) for v in rows]
    check_stream(k, stream)
    R = np.ascontiguousarray(np.stack(rows))
    _batch_vs_rows(k, R, sorted(set(rng.integers(1, len(rows) + 1, 2).tolist()) | {len(rows)}))


def _batch_vs_rows(k, R, cuts):
    """rlnc_decoder_add_pieces over R (one row per received piece) split at
    `cuts` == the same rows through rlnc_decoder_add_piece one by one (which
    the tests above tie to the oracle): return codes, rows consumed, and the
    coefficient and transform matrices byte for byte."""
    L = _lib.lib()
    seq, bat = CoreDecoder(k), CoreDecoder(k)
    seq_st = []
    for v in R:
        seq_st.append(seq.add(v))
        if seq_st[-1] != 0:
            break
    W = np.ascontiguousarray(np.concatenate([R, np.zeros((R.shape[0], 1), np.uint8)], axis=1))
    pos = 0
    for c1 in cuts:
        if c1 <= pos:
            continue
        used = ctypes.c_size_t()
        st = L.rlnc_decoder_add_pieces(bat.h, W[pos:].ctypes.data_as(_lib._u8p), c1 - pos, k + 1, 1, 0,
                                       ctypes.byref(used))
        exp_used = sum(1 for s in seq_st[pos:c1] if s == 0)
        exp_st = seq_st[pos + exp_used] if exp_used < c1 - pos and pos + exp_used < len(seq_st) else 0
        assert (st, used.value) == (exp_st, exp_used), (pos, c1)
        pos += used.value
        if st != 0:
            break
    assert seq.state() == bat.state()
    assert np.array_equal(seq.coefficients(), bat.coefficients())
    assert np.array_equal(seq.transform(), bat.transform())


@pytest.mark.parametrize("seed", range(60))
def test_batch_add_matches_row_by_row(seed):
    # the batched path eliminates runs of clean rows 4 at a time
    # (decoder_core.cpp add_panel); it must leave exactly the state of
    # one-by-one AddPiece, including when a row of a run is not a pivot
    rng = np.random.default_rng(9100 + seed)
    k = int(rng.choice([2, 3, 5, 8, 16, 33, 64, 256]))
    n = k + int(rng.integers(0, 6))
    kind = seed % 5
    if kind == 0:
        R = rng.integers(0, 256, (n, k), dtype=np.uint8)
    elif kind == 1:
        R = (rng.integers(0, 256, (n, k)) * (rng.random((n, k)) < 0.2)).astype(np.uint8)
    elif kind == 2:  # systematic stream with losses, coded rows after
        lost = set(rng.choice(k, max(1, k // 5), replace=False).tolist())
        R = np.concatenate([np.eye(k, dtype=np.uint8)[[i for i in range(k) if i not in lost]],
                            rng.integers(0, 256, (n, k), dtype=np.uint8)])[:n]
    elif kind == 3:  # rank-deficient combinations, some zero rows
        B = rng.integers(0, 256, (max(1, k // 2), k), dtype=np.uint8)
        R = oracle.matmul(rng.integers(0, 256, (n, B.shape[0]), dtype=np.uint8), B)[1]
        R[rng.random(n) < 0.1] = 0
    else:  # tiny field: frequent zero diagonals inside a run
        R = rng.integers(0, 3, (n, k), dtype=np.uint8)
    cuts = sorted(set(rng.integers(1, n + 1, 3).tolist()) | {n})
    _batch_vs_rows(k, np.ascontiguousarray(R), cuts)


@pytest.mark.parametrize("seed", range(40))
def test_systematic_full_batch_solve(seed):
    # one batched AddPiece of >= k rows on a fresh decoder, mostly systematic
    # pieces (any order, some scaled) plus a few coded ones anywhere among
    # them: DecoderCore solves the small block of coded rows instead of
    # eliminating row by row (decoder_core.cpp solve_systematic_batch); the
    # state, counters and T must equal row-by-row AddPiece -- also when the
    # coded rows are dependent (C singular: the row-by-row route is taken)
    rng = np.random.default_rng(5500 + seed)
    k = int(rng.choice([4, 9, 16, 40, 64, 128]))
    m = int(rng.integers(1, max(2, k // 8) + 1))
    lost = rng.choice(k, m, replace=False)
    units = [i for i in range(k) if i not in set(lost.tolist())]
    if seed % 2:
        rng.shuffle(units)
    rows = []
    for i in units:
        v = np.zeros(k, np.uint8)
        v[i] = 1 if rng.random() < 0.85 else rng.integers(2, 256)
        rows.append(v)
    coded = rng.integers(0, 256, (m, k), dtype=np.uint8)
    if seed % 5 == 3 and m >= 2:
        coded[1] = coded[0]                           # dependent: C singular
    if seed % 7 == 4:
        coded[0, lost] = 0                            # zero on every lost column: singular
    for v in coded:
        rows.insert(int(rng.integers(0, len(rows) + 1)), v)
    rows += [rng.integers(0, 256, k, dtype=np.uint8) for _ in range(int(rng.integers(0, 4)))]
    R = np.ascontiguousarray(np.stack(rows))
    _batch_vs_rows(k, R, [R.shape[0]])


@pytest.mark.parametrize("seed", range(36))
def test_full_batch_solve(seed):
    # one batched AddPiece of >= k coded rows on a fresh decoder (k >= 240):
    # DecoderCore inverts the first k vectors by blocked Gauss-Jordan
    # (decoder_core.cpp solve_full_batch) instead of taking kodr's route; the
    # state, counters and T must equal row-by-row AddPiece -- for dense rows,
    # {0,1,2}-valued rows (zero diagonals, panels whose first candidate rows are
    # dependent), and singular batches (duplicates, low rank: kodr's route)
    rng = np.random.default_rng(6100 + seed)
    k = int(rng.choice([240, 250, 256]))
    n = k + int(rng.integers(0, 4))
    kind = seed % 6
    if kind in (0, 1):
        R = rng.integers(0, 256, (n, k), dtype=np.uint8)
    elif kind == 2:
        R = rng.integers(0, 3, (n, k), dtype=np.uint8)
    elif kind == 3:  # panel-local dependence: rows 0..16 agree on the first 16 columns up to scale
        R = rng.integers(0, 256, (n, k), dtype=np.uint8)
        R[1:17, :16] = oracle.matmul(rng.integers(0, 256, (16, 1), dtype=np.uint8), R[:1, :16])[1]
    elif kind == 4:  # singular: a duplicate among the first k
        R = rng.integers(0, 256, (n, k), dtype=np.uint8)
        R[int(rng.integers(1, k))] = R[0]
    else:  # singular: rank k - 3
        B = rng.integers(0, 256, (k - 3, k), dtype=np.uint8)
        R = oracle.matmul(rng.integers(0, 256, (n, k - 3), dtype=np.uint8), B)[1]
    _batch_vs_rows(k, np.ascontiguousarray(R), [n])


def test_grouped_entry_points_argument_checks():
    # the many-generation entry points reject bad arguments before any device
    # work, and a decoder group reports kodr's GetPieces errors
    # (full/decoder.go:84-86) or the missing device
    L = _lib.lib()
    vp = ctypes.c_void_p
    assert L.rlnc_encoder_group_coded_pieces_device(None, 1, None, 1, None, 16) == -1
    assert L.rlnc_recoder_group_coded_pieces_device(None, 1, None, 1, None, 16) == -1
    assert L.rlnc_decoders_get_pieces_device(None, 1, None, 16) == -1
    empty = (vp * 1)(None)
    assert L.rlnc_encoder_group_coded_pieces_device(empty, 0, None, 1, None, 16) == 0
    assert L.rlnc_recoder_group_coded_pieces_device(empty, 0, None, 1, None, 16) == 0
    a, b = CoreDecoder(2), CoreDecoder(2)
    a.add(np.array([1, 0], np.uint8))
    a.add(np.array([0, 1], np.uint8))
    buf = ctypes.create_string_buffer(64)
    both = (vp * 2)(a.h.value, b.h.value)
    assert L.rlnc_decoders_get_pieces_device(both, 2, buf, 16) == 4   # b: MORE_USEFUL_PIECES_REQUIRED
    b.add(np.array([1, 1], np.uint8))
    b.add(np.array([0, 1], np.uint8))
    assert L.rlnc_decoders_get_pieces_device(both, 2, buf, 16) == -4  # coefficient-side decoders: no device


def test_grouped_flush_argument_checks():
    # rlnc_decoders_flush_gpu rejects bad arguments before any device work
    # (no decoders, a null handle); coefficient-side decoders (no context)
    # have no device to eliminate on, and keep their state
    L = _lib.lib()
    vp = ctypes.c_void_p
    assert L.rlnc_decoders_flush_gpu(None, 1) == -1
    assert L.rlnc_decoders_flush_gpu((vp * 1)(None), 1) == -1
    a = CoreDecoder(4)
    a.add(np.array([1, 2, 3, 4], np.uint8))
    assert L.rlnc_decoders_flush_gpu((vp * 1)(a.h.value), 0) == -1
    assert L.rlnc_decoders_flush_gpu((vp * 1)(a.h.value), 1) == -4   # no context: no device
    assert a.state() == (1, 1, 3, False)                              # and nothing changed
