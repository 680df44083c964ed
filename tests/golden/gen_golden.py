#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/.

Run in the build container (it reads the reference's Go source *as text* to
extract the literal field tables; nothing of the reference is executed):

    python tests/golden/gen_golden.py [--ref /root/reference]

Outputs (data only -- inputs and expected outputs):
  gf256_tables.json  LOG/EXP literal tables of kodr_internals/gf256/gf256.go:15-44
  kats.json          known-answer tests transcribed from
                     kodr_internals/matrix/matrix_test.go:12-109 and
                     kodr_internals/data_test.go:136-156
  vectors.json       seeded encode / recode / systematic / decode-trace / split
                     vectors computed by the pure-Python restatement below.

The restatement here is deliberately independent of oracle/kodr_oracle.c (a
second, pure-Python transcription of the same Go code), so the C oracle is
checked against it as well as against the reference's own KATs.
"""
import argparse
import json
import os
import re
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

# --------------------------------------------------------------------------
# field (gf256.go)


def parse_tables(ref):
    src = open(os.path.join(ref, "kodr_internals/gf256/gf256.go")).read()

    def grab(name):
        m = re.search(name + r"\s*=\s*\[[^\]]*\]uint8\{([^}]*)\}", src)
        return [int(t) for t in re.findall(r"\d+", m.group(1))]

    log, exp = grab("gf256_LOG_TABLE"), grab("gf256_EXP_TABLE")
    assert len(log) == 256 and len(exp) == 510
    return log, exp


def regen_tables():
    exp = [0] * 510
    log = [0] * 256
    x = 1
    for i in range(255):
        exp[i] = x
        log[x] = i
        x <<= 1
        if x & 0x100:
            x ^= 0x11D
    for i in range(255, 510):
        exp[i] = exp[i - 255]
    return log, exp


LOG, EXP = regen_tables()


def mul(a, b):  # gf256.go:109-118
    if a == 0 or b == 0:
        return 0
    return EXP[LOG[a] + LOG[b]]


def inv(a):  # gf256.go:77-86
    assert a != 0
    return EXP[255 - LOG[a]]


def div(a, b):  # gf256.go:121-127
    return mul(a, inv(b))


# --------------------------------------------------------------------------
# data.go / full / systematic / matrix


def piece_multiply(dst, src, by):  # data.go:19-29
    for i in range(len(src)):
        dst[i] ^= mul(src[i], by)


def encode(pieces, vec):  # full/encoder.go:61-71
    out = [0] * len(pieces[0])
    for i, p in enumerate(pieces):
        piece_multiply(out, p, vec[i])
    return out


def matmul(a, b):  # matrix.go:45-69
    if len(a[0]) != len(b):
        raise ValueError("ErrMatrixDimensionMismatch")
    out = [[0] * len(b[0]) for _ in a]
    for i in range(len(a)):
        for j in range(len(b[0])):
            acc = 0
            for k in range(len(a[0])):
                acc ^= mul(a[i][k], b[k][j])
            out[i][j] = acc
    return out


def recode(coded, r):  # full/recoder.go:27-46
    piece = [0] * len(coded[0][1])
    for i, (_, p) in enumerate(coded):
        piece_multiply(piece, p, r[i])
    vec = matmul([r], [list(v) for v, _ in coded])[0]
    return vec, piece


def split_by_count(n, count):  # data.go:137-166
    if count < 2:
        return ("ErrBadPieceCount", None, None)
    if count > n:
        return ("ErrPieceCountMoreThanTotalBytes", None, None)
    size = (n + count - 1) // count
    return (None, size, count * size - n)


def split_by_size(n, size):  # data.go:103-132
    if size == 0:
        return ("ErrZeroPieceSize", None, None)
    if size >= n:
        return ("ErrBadPieceCount", None, None)
    count = -(-n // size)
    return (None, count, count * size - n)


class DecoderState:  # kodr_internals/matrix/decoder_state.go
    def __init__(self, piece_count, coeffs=None, coded=None):
        self.piece_count = piece_count
        self.coeffs = [list(r) for r in (coeffs or [])]
        self.coded = [list(r) for r in (coded or [])]

    def clean_forward(self):  # :15-76
        rows, cols = len(self.coeffs), len(self.coeffs[0])
        for i in range(min(rows, cols)):
            if self.coeffs[i][i] == 0:
                pivot = next((p for p in range(i + 1, rows) if self.coeffs[p][i] != 0), None)
                if pivot is None:
                    continue
                self.coeffs[i], self.coeffs[pivot] = self.coeffs[pivot], self.coeffs[i]
                self.coded[i], self.coded[pivot] = self.coded[pivot], self.coded[i]
            for j in range(i + 1, rows):
                if self.coeffs[j][i] == 0:
                    continue
                q = div(self.coeffs[j][i], self.coeffs[i][i])
                for k in range(i, cols):
                    self.coeffs[j][k] ^= mul(self.coeffs[i][k], q)
                for k in range(len(self.coded[0])):
                    self.coded[j][k] ^= mul(self.coded[i][k], q)

    def clean_backward(self):  # :78-134
        rows, cols = len(self.coeffs), len(self.coeffs[0])
        for i in range(min(rows, cols) - 1, -1, -1):
            if self.coeffs[i][i] == 0:
                continue
            for j in range(i):
                if self.coeffs[j][i] == 0:
                    continue
                q = div(self.coeffs[j][i], self.coeffs[i][i])
                for k in range(i, cols):
                    self.coeffs[j][k] ^= mul(self.coeffs[i][k], q)
                for k in range(len(self.coded[0])):
                    self.coded[j][k] ^= mul(self.coded[i][k], q)
            if self.coeffs[i][i] == 1:
                continue
            iv = inv(self.coeffs[i][i])
            self.coeffs[i][i] = 1
            for j in range(i + 1, cols):
                if self.coeffs[i][j] != 0:
                    self.coeffs[i][j] = mul(self.coeffs[i][j], iv)
            for j in range(len(self.coded[0])):
                self.coded[i][j] = mul(self.coded[i][j], iv)

    def remove_zero_rows(self):  # :136-165
        i = 0
        while i < len(self.coeffs):
            if all(c == 0 for c in self.coeffs[i]):
                del self.coeffs[i]
                del self.coded[i]
            else:
                i += 1

    def rref(self):  # :178-182
        self.clean_forward()
        self.clean_backward()
        self.remove_zero_rows()

    def get_piece(self, idx):  # :221-261
        if idx >= self.piece_count:
            return ("ErrPieceOutOfBound", None)
        if idx >= len(self.coeffs):
            return ("ErrPieceNotDecodedYet", None)
        if len(self.coeffs) >= self.piece_count:
            return (None, list(self.coded[idx]))
        for i in range(len(self.coeffs[0])):
            if i == idx:
                if self.coeffs[idx][i] != 1:
                    return ("ErrPieceNotDecodedYet", None)
            elif self.coeffs[idx][i] == 0:
                return ("ErrPieceNotDecodedYet", None)
        return (None, list(self.coded[idx]))


class FullDecoder:  # full/decoder.go
    def __init__(self, k):
        self.expected, self.useful, self.received = k, 0, 0
        self.state = DecoderState(k)

    def is_decoded(self):
        return self.useful >= self.expected

    def add_piece(self, vec, piece):  # :50-66
        if self.is_decoded():
            return "ErrAllUsefulPiecesReceived"
        self.state.coeffs.append(list(vec))
        self.state.coded.append(list(piece))
        self.received += 1
        if not (self.received > 1):
            self.useful += 1
            return None
        self.state.rref()
        self.useful = len(self.state.coeffs)
        return None


# --------------------------------------------------------------------------


def hx(b):
    return bytes(bytearray(b)).hex()


def rng_bytes(rng, n):
    return [int(x) for x in rng.integers(0, 256, n, dtype=np.uint16)]


def decode_trace(k, stream, probe_get=True):
    """Feed (vec, piece) pairs; record the decoder's observable state."""
    dec = FullDecoder(k)
    steps = []
    for vec, piece in stream:
        err = dec.add_piece(vec, piece)
        step = {"err": err, "useful": dec.useful, "received": dec.received,
                "required": dec.expected - dec.useful, "decoded": dec.is_decoded()}
        if probe_get and not dec.is_decoded():
            gets = []
            for idx in range(k + 1):
                e, p = dec.state.get_piece(idx)
                gets.append([e, hx(p) if p is not None else None])
            step["get"] = gets
        steps.append(step)
    out = None
    if dec.is_decoded():
        out = [hx(dec.state.get_piece(i)[1]) for i in range(dec.useful)]
    return steps, out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    args = ap.parse_args()

    if os.path.isdir(args.ref):
        log, exp = parse_tables(args.ref)
        assert (log[1:], exp) == (LOG[1:], EXP), "literal tables differ from 0x11D regeneration"
        assert log[0] == 0
        with open(os.path.join(HERE, "gf256_tables.json"), "w") as f:
            json.dump({"source": "kodr_internals/gf256/gf256.go:15-44", "LOG": log, "EXP": exp}, f)

    # Known-answer tests, transcribed as data.
    kats = {
        "source": {"rref_rank": "kodr_internals/matrix/matrix_test.go:12-87",
                   "matmul": "kodr_internals/matrix/matrix_test.go:89-109",
                   "is_systematic": "kodr_internals/data_test.go:136-156"},
        "rref": [
            {"m": [[70, 137, 2, 152], [223, 92, 234, 98], [217, 141, 33, 44], [145, 135, 71, 45]],
             "rref": [[1, 0, 0, 105], [0, 1, 0, 181], [0, 0, 1, 42]], "rank": 3, "coded_cols": 4},
            {"m": [[68, 54, 6, 230], [16, 56, 215, 78], [159, 186, 146, 163], [122, 41, 205, 133]],
             "rref": [[1, 0, 0, 0], [0, 1, 0, 0], [0, 0, 1, 0], [0, 0, 0, 1]], "rank": 4, "coded_cols": 4},
            {"m": [[100, 31, 76, 199, 119], [207, 34, 207, 208, 18], [62, 20, 54, 6, 187],
                   [66, 8, 52, 73, 54], [122, 138, 247, 211, 165]],
             "rref": [[1, 0, 0, 0, 0], [0, 1, 0, 0, 0], [0, 0, 1, 0, 0], [0, 0, 0, 1, 0], [0, 0, 0, 0, 1]],
             "rank": 5, "coded_cols": 4},
        ],
        "matmul": {"a": [[102, 82, 165, 0]],
                   "b": [[157, 233, 247], [160, 28, 233], [149, 234, 117], [200, 181, 55]],
                   "expected": [[186, 23, 11]],
                   "bad_a": [[1, 2, 3]]},
        "is_systematic": [
            {"vector": [0, 1, 0, 0], "expected": True},
            {"vector": [1, 1, 0, 0], "expected": False},
            {"vector": [0, 0, 1, 0], "expected": True},
            {"vector": [0, 0, 0, 0], "expected": False},
        ],
    }
    # the restatement must reproduce every KAT before any vector is trusted
    for case in kats["rref"]:
        ds = DecoderState(len(case["m"]), case["m"], [[0] * case["coded_cols"]] * len(case["m"]))
        ds.rref()
        assert ds.coeffs == case["rref"] and len(ds.coeffs) == case["rank"], case
    assert matmul(kats["matmul"]["a"], kats["matmul"]["b"]) == kats["matmul"]["expected"]
    with open(os.path.join(HERE, "kats.json"), "w") as f:
        json.dump(kats, f, indent=1)

    rng = np.random.default_rng(0x6B6F6472)
    vec = {"seed": 0x6B6F6472, "encode": [], "recode": [], "systematic": [], "decode": [],
           "split_count": [], "split_size": []}

    # ---- encode (full/encoder.go:61-71)
    for k, L in [(2, 1), (3, 7), (4, 64), (16, 1024), (16, 4096)]:
        pieces = [rng_bytes(rng, L) for _ in range(k)]
        vecs = [rng_bytes(rng, k) for _ in range(3)]
        vecs.append([0] * k)           # all-zero vector (crypto/rand can draw it)
        vecs.append([1] * k)
        vecs.append([255] * k)
        outs = [encode(pieces, v) for v in vecs]
        vec["encode"].append({"k": k, "L": L, "pieces": [hx(p) for p in pieces],
                              "vectors": [hx(v) for v in vecs], "coded": [hx(o) for o in outs]})

    # ---- recode (full/recoder.go:27-46)
    for k, L, n in [(2, 5, 3), (4, 64, 6), (16, 512, 18)]:
        pieces = [rng_bytes(rng, L) for _ in range(k)]
        coded = []
        for _ in range(n):
            v = rng_bytes(rng, k)
            coded.append((v, encode(pieces, v)))
        rs = [rng_bytes(rng, n) for _ in range(3)]
        outs = [recode(coded, r) for r in rs]
        vec["recode"].append({"k": k, "L": L, "n": n,
                              "flat": hx(sum((list(v) + list(p) for v, p in coded), [])),
                              "r": [hx(r) for r in rs],
                              "out": [hx(list(v) + list(p)) for v, p in outs],
                              "pieces": [hx(p) for p in pieces]})

    # ---- systematic encoder (systematic/encoder.go:82-109)
    for k, L in [(4, 16), (8, 100)]:
        pieces = [rng_bytes(rng, L) for _ in range(k)]
        randv = [rng_bytes(rng, k) for _ in range(k + 3)]
        outs = []
        for cid in range(k + 3):
            if cid < k:
                v = [0] * k
                v[cid] = 1
                outs.append((v, list(pieces[cid])))
            else:
                outs.append((randv[cid], encode(pieces, randv[cid])))
        vec["systematic"].append({"k": k, "L": L, "pieces": [hx(p) for p in pieces],
                                  "random_vectors": [hx(v) for v in randv],
                                  "out": [hx(v + p) for v, p in outs]})

    # ---- decode traces (full/decoder.go:50-99 + decoder_state.go)
    def coded_stream(pieces, vectors):
        return [(v, encode(pieces, v)) for v in vectors]

    cases = []
    for k, L in [(2, 3), (4, 32), (16, 256), (32, 64)]:
        pieces = [rng_bytes(rng, L) for _ in range(k)]
        vs = [rng_bytes(rng, k) for _ in range(k + 4)]
        cases.append(("random", k, L, pieces, vs))
    # zero first vector: counted useful without RREF (full/decoder.go:58-61)
    k, L = 4, 16
    pieces = [rng_bytes(rng, L) for _ in range(k)]
    vs = [[0] * k] + [rng_bytes(rng, k) for _ in range(k + 2)]
    cases.append(("zero_first", k, L, pieces, vs))
    # duplicate / dependent vectors get removed as zero rows (:136-165)
    base = [rng_bytes(rng, k) for _ in range(3)]
    dep = [a ^ mul(7, b) for a, b in zip(base[0], base[1])]
    vs = [base[0], base[0], base[1], dep, base[2], [0] * k, rng_bytes(rng, k), rng_bytes(rng, k)]
    cases.append(("dependent", k, L, pieces, vs))
    # rank over-count quirk: off-diagonal pivots (:23-35, :86-88)
    k, L = 3, 5
    pieces = [rng_bytes(rng, L) for _ in range(k)]
    vs = [[0, 0, 1], [0, 0, 1], [0, 0, 5], [0, 3, 0], [1, 1, 1], [9, 0, 0]]
    cases.append(("offdiag_quirk", k, L, pieces, vs))
    vs = [[0, 0, 1], [0, 2, 3], [0, 0, 7], [5, 0, 0]]
    cases.append(("offdiag_quirk2", k, L, pieces, vs))
    # GetPiece before full rank succeeds only for [.. 1 at idx, every other
    # coefficient non-zero ..] (decoder_state.go:237-251); first piece skips RREF
    vs = [[1, 5, 7], [2, 3, 4], [6, 1, 9], [3, 3, 3]]
    cases.append(("partial_get", k, L, pieces, vs))
    # systematic-style stream (unit vectors + random), as systematic/decoder.go sees it
    k, L = 8, 40
    pieces = [rng_bytes(rng, L) for _ in range(k)]
    vs = []
    for i in [0, 2, 3, 5, 7]:
        v = [0] * k
        v[i] = 1
        vs.append(v)
    vs += [rng_bytes(rng, k) for _ in range(6)]
    cases.append(("systematic_mix", k, L, pieces, vs))
    # low-rank generator: pieces whose coded data is inconsistent with vectors
    # (random piece bytes), exercising T-tracking on arbitrary rows
    k, L = 5, 24
    pieces = [rng_bytes(rng, L) for _ in range(k)]
    stream = [(rng_bytes(rng, k), rng_bytes(rng, L)) for _ in range(k + 2)]
    cases.append(("arbitrary_rows", k, L, pieces, stream))

    for name, k, L, pieces, vs in cases:
        stream = vs if (vs and isinstance(vs[0], tuple)) else coded_stream(pieces, vs)
        steps, out = decode_trace(k, stream, probe_get=(k <= 16))
        vec["decode"].append({"name": name, "k": k, "L": L, "pieces": [hx(p) for p in pieces],
                              "stream": [[hx(v), hx(p)] for v, p in stream],
                              "steps": steps, "decoded": out})

    # ---- splitting (data.go:103-166)
    for n, c in [(10, 0), (10, 1), (10, 2), (10, 3), (10, 10), (10, 11), (1 << 20, 16),
                 (33554432, 256), (16777216, 128), (2049, 7), (3000, 517)]:
        e, s, p = split_by_count(n, c)
        vec["split_count"].append({"len": n, "count": c, "err": e, "piece_size": s, "padding": p})
    for n, s in [(10, 0), (10, 10), (10, 11), (10, 3), (10, 9), (2049, 64), (4096, 127), (3, 1)]:
        e, c, p = split_by_size(n, s)
        vec["split_size"].append({"len": n, "size": s, "err": e, "piece_count": c, "padding": p})

    with open(os.path.join(HERE, "vectors.json"), "w") as f:
        json.dump(vec, f)
    print("wrote", os.listdir(HERE))


if __name__ == "__main__":
    sys.exit(main())
