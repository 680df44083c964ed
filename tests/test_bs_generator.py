"""CPU checks of the bit-sliced kernel's generated code (kodr_amd/csrc/
gen_bs_bodies.py): a small interpreter runs the emitted row-prep and body
instructions on random bit-sliced blocks and compares every coefficient's
product with the oracle's GF(2^8) multiply (gf256.go:109-118)."""
import os
import re
import sys

import numpy as np
import pytest

import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "kodr_amd", "csrc"))
import gen_bs_bodies as gen  # noqa: E402


def bitslice_np(x):
    d = x.reshape(-1, 8, 4).copy().view(np.uint32).reshape(-1, 8)
    for sh, m, di in ((4, 0x0F0F0F0F, 4), (2, 0x33333333, 2), (1, 0x55555555, 1)):
        for q in range(8):
            if q & di:
                continue
            t = ((d[:, q] >> sh) ^ d[:, q + di]) & m
            d[:, q + di] ^= t
            d[:, q] ^= (t << sh).astype(np.uint32)
    return d.view(np.uint8).reshape(x.shape)


def run(lines, regs, idx=0):
    """Interpret the generator's VALU subset; idx = VGPR index (SRC0|DST)."""
    for ln in lines:
        op = ln.split()[0]
        r = [int(v) for v in re.findall(r"v\[?(\d+)", ln)]
        if op == "v_pk_mov_b32":      # v[d:d+1], v[a:a+1], v[b:b+1] op_sel:[0,1]
            assert ln.endswith("op_sel:[0,1]")
            regs[r[0]] = regs[r[1]]          # lo <- a.lo
            regs[r[0] + 1] = regs[r[2] + 1]  # hi <- b.hi
        elif op in ("v_xor_b32_e32", "v_xor_b32_e64"):
            if r[0] < gen.TL0:        # body: acc (indexed) ^= table entry
                regs[r[0] + idx] = regs[r[1] + idx] ^ regs[r[2]]
            else:                     # table build
                regs[r[0]] = regs[r[1]] ^ regs[r[2]]
        elif op == "v_bitop3_b32":
            assert ln.endswith("bitop3:0x96")
            if r[0] < gen.TL0:        # body: acc (indexed) ^= a ^ b
                regs[r[0] + idx] = regs[r[1] + idx] ^ regs[r[2]] ^ regs[r[3]]
            else:
                regs[r[0]] = regs[r[1]] ^ regs[r[2]] ^ regs[r[3]]
        elif op.startswith("s_"):
            continue
        else:
            raise AssertionError(ln)


def test_body_sizes_match_offsets():
    offs, total = gen.body_offsets()
    assert len(offs) == 256 * gen.NCOPY
    for r in range(gen.NCOPY):
        for c in range(256):
            assert len(gen.body_ops(c)) <= 8
            # an XOR3 is VOP3 (8 bytes), a single-entry XOR VOP2 (4), s_setpc 4
            assert gen.body_bytes(c) == sum(8 if lo and hi else 4 for _j, lo, hi in gen.body_ops(c)) + 4
            assert sum(8 if ln.startswith("v_bitop3") else 4 for ln in gen.body_lines(c, r)) == gen.body_bytes(c)
            nxt = offs[r * 256 + c + 1] if r * 256 + c + 1 < len(offs) else total
            assert nxt - offs[r * 256 + c] == gen.body_bytes(c)
    # every copy is laid out identically, and all of them stay within what the
    # instruction cache holds (tools/probe/dispatch.py: 4 copies fit, 8 thrash)
    assert all(offs[r * 256 + c] - offs[r * 256] == offs[c] for r in range(gen.NCOPY) for c in range(256))
    assert total < 72 * 1024


def test_registers_fit_four_waves():
    assert gen.VMAX <= 128
    assert gen.TL0 % 2 == 0 and gen.TH0 % 2 == 0 and gen.RING % 2 == 0   # v_pk_mov pairs
    used = set(range(gen.ACC, gen.ACC + 64)) | set(range(gen.TL0, gen.TL0 + 15)) | \
        set(range(gen.TH0, gen.TH0 + 15)) | set(range(gen.RING, gen.RING + 8 * gen.P)) | \
        {gen.PG, gen.PGN, gen.PL}
    assert len(used) == 64 + 30 + 8 * gen.P + 3          # no overlaps


def test_every_coefficient_body_vs_oracle():
    rng = np.random.default_rng(7)
    x = rng.integers(0, 256, 32, dtype=np.uint8)
    planes = bitslice_np(x).view(np.uint32)
    for slot in range(gen.P):
        regs = {}
        for i in range(8):
            regs[gen.RING + 8 * slot + i] = int(planes[i])
        run(gen.table_lines(slot), regs)
        for c in range(256):
            m = c % 8                                     # any accumulator row
            for j in range(8):
                regs[gen.ACC + 8 * m + j] = 0
            run(gen.body_lines(c), regs, idx=8 * m)
            out = np.array([regs[gen.ACC + 8 * m + j] for j in range(8)], np.uint32)
            got = bitslice_np(out.view(np.uint8).copy())
            exp = np.array([oracle.gf_mul(c, int(b)) for b in x], np.uint8)
            assert np.array_equal(got, exp), (slot, c)


def test_bitslice_model_is_an_involution_and_plane_layout():
    rng = np.random.default_rng(8)
    x = rng.integers(0, 256, (5, 32), dtype=np.uint8)
    assert np.array_equal(bitslice_np(bitslice_np(x)), x)
    blk = np.zeros(32, np.uint8)
    blk[17] = 1 << 5
    planes = bitslice_np(blk).view(np.uint32)
    assert [i for i in range(8) if planes[i]] == [5]


class _Wave:
    """Model of the generated main loop + threaded bodies: every SALU, VALU,
    LDS and buffer instruction the generator emits, with PC-level control flow
    (s_setpc to absolute addresses, labels, branches), VGPR index mode, and
    64-lane program chunks (v_readlane); data planes are modelled for one
    lane.  Checks the dispatch plumbing (targets, stub, returns, M0, program
    chunks) end to end on CPU, before any GPU run."""

    BASE = 0x7F12_3456_0000
    VEC = (gen.PG, gen.PGN, gen.PL)                # registers modelled per lane

    def __init__(self, X, A, nr, loop=None):
        self.X, self.A, self.nr = X, A, nr          # X: nr x 32 bytes, A: 8 x nr
        offs, _ = gen.body_offsets()
        self.code, self.addr = [], {}
        for r in range(gen.NCOPY):
            for c in range(256):
                self.addr[self.BASE + offs[r * 256 + c]] = len(self.code)
                self.code += gen.body_lines(c, r)
        self.main0 = len(self.code)
        loop = gen.main_loop(True) if loop is None else loop
        self.code += [ln.replace("_%=", "") for ln in loop] + ["END"]
        self.labels = {ln[:-1]: i for i, ln in enumerate(self.code) if ln.endswith(":")}
        for name, i in self.labels.items():          # main code at fake addresses
            self.addr[0x1000_0000 + 4 * i] = i
        self.s, self.v = {}, {}
        self.m0, self.idx_on = 0, False
        # LDS program: per row 8 absolute lo targets, body c in copy m % NCOPY
        self.lds = {}
        pl = 0x400
        for k in range(nr):
            for m in range(8):
                c = int(A[m, k])
                self.lds[pl + 4 * (8 * k + m)] = (self.BASE + offs[(m % gen.NCOPY) * 256 + c]) & 0xFFFFFFFF
        # the same program in global memory for the scalar-load variant (plus
        # one row of look-ahead past the end, as the kernel's scratch has)
        self.gmem = {0x2000_0000 + a - pl: v for a, v in self.lds.items()}
        self.ops = {"xlo": 0, "xhi": 0, "nrec": nr * 32, "roff": gen.P * 32, "ldx": 32, "ngrp": nr // 8,
                    "thi": self.BASE >> 32, "col": 0, "pglo": 0x2000_0000, "pghi": 0}
        self.pl_lanes = [pl + 4 * lane for lane in range(64)]
        for slot in range(gen.P):                      # the compiler's ring prologue
            self._load_row(gen.RING + 8 * slot, slot * 32)

    def _load_row(self, vb, off, half=None):
        row = off // 32
        planes = bitslice_np(self.X[row]).view(np.uint32) if row < self.nr else np.zeros(8, np.uint32)
        for i in range(8):
            if half is None or i // 4 == half:
                self.v[vb + i] = int(planes[i])

    def val(self, tok):
        if tok.startswith("%["):
            return self.ops[tok[2:-1]]
        if tok.startswith("s"):
            return self.s[int(tok[1:])]
        return int(tok, 0)

    def run(self):
        pc, steps = self.main0, 0
        while self.code[pc] != "END":
            steps += 1
            assert steps < 400000
            ln = self.code[pc]
            pc += 1
            if ln.endswith(":"):
                continue
            op, _, rest = ln.partition(" ")
            a = [t.strip() for t in rest.split(",")]
            r = [int(x) for x in re.findall(r"v\[?(\d+)", ln)]
            pc = self.step(ln, op, a, r, pc)
        return np.array([[self.v[gen.ACC + 8 * m + j] for j in range(8)] for m in range(8)], np.uint32)

    def step(self, ln, op, a, r, pc):
        """One instruction; returns the next pc."""
        if op == "s_getpc_b64":
            self.s[gen.GPC], self.s[gen.GPC + 1] = 0x1000_0000, 0
        elif op == "s_add_u32" and "- .Lpc" in ln:
            lab = a[2].split(" - ")[0]
            self.s[int(a[0][1:])] = 0x1000_0000 + 4 * self.labels[lab]
        elif op == "s_addc_u32":
            self.s[int(a[0][1:])] = 0
        elif op == "s_mov_b32":
            self.s[int(a[0][1:])] = self.val(a[1])
        elif op == "s_and_b32":
            self.s[int(a[0][1:])] = self.val(a[1]) & self.val(a[2])
        elif op == "s_add_u32" and a[0] == "m0":
            assert self.idx_on
            self.m0 += self.val(a[2])
        elif op == "s_add_u32":
            self.s[int(a[0][1:])] = self.val(a[1]) + self.val(a[2])
        elif op == "s_sub_u32":
            self.s[int(a[0][1:])] = self.val(a[1]) - self.val(a[2])
        elif op == "s_cmp_lg_u32":
            self.scc = self.val(a[0]) != self.val(a[1])
        elif op == "s_cbranch_scc1":
            if self.scc:
                return self.labels[a[0]]
        elif op == "s_branch":
            return self.labels[a[0]]
        elif op == "s_mov_b64":
            d, sr = [int(x) for x in re.findall(r"s\[(\d+):", ln)]
            self.s[d], self.s[d + 1] = self.s[sr], self.s[sr + 1]
        elif op == "s_load_dwordx8":
            d, sr = [int(x) for x in re.findall(r"s\[(\d+):", ln)]
            addr = (self.s[sr + 1] << 32) | self.s[sr]
            for i in range(8):
                self.s[d + i] = self.gmem.get(addr + 4 * i, 0xDEAD)
        elif op == "s_setpc_b64":
            lo = int(re.findall(r"s\[(\d+):", ln)[0])
            return self.addr[(self.s[lo + 1] << 32) | self.s[lo]]
        elif op == "s_set_gpr_idx_on":
            assert a[0] == "0"
            self.idx_on, self.m0 = True, 0
        elif op == "s_set_gpr_idx_off":
            self.idx_on = False
        elif op == "s_waitcnt":
            pass
        elif op == "v_mov_b32" and r[0] == gen.PL:
            self.v[gen.PL] = list(self.pl_lanes)
        elif op == "v_mov_b32" and r[0] in self.VEC:
            self.v[r[0]] = list(self.v[r[1]])
        elif op == "v_mov_b32":
            self.v[r[0]] = self.val(a[1])
        elif op == "v_readlane_b32":
            assert not self.idx_on
            self.s[int(a[0][1:])] = self.v[r[0]][int(a[2])]
        elif op == "v_add_u32_e32":
            assert r[0] == r[1] == gen.PL
            self.v[gen.PL] = [x + int(a[1]) for x in self.v[gen.PL]]
        elif op == "ds_read_b32":
            off = int(ln.split("offset:")[1]) if "offset:" in ln else 0
            self.v[r[0]] = [self.lds.get(x + off, 0xDEAD) for x in self.v[r[1]]]
        elif op == "buffer_load_dwordx4":
            half = 1 if "offset:16" in ln else 0
            self._load_row(r[0] - 4 * half, self.s[44], half)
        elif op == "s_setprio":  # scheduling only
            assert 0 <= int(a[0]) <= 3
        elif op in ("v_pk_mov_b32", "v_xor_b32_e32", "v_xor_b32_e64", "v_bitop3_b32"):
            idx = self.m0 if self.idx_on else 0
            run([ln], self.v, idx)
        else:
            raise AssertionError(ln)
        return pc


# the shipped loop and the tuning build's variants (gf_bs.hip MODE 10-14)
LOOPS = {"main": lambda: gen.main_loop(True),
         "noprio": lambda: gen.main_loop(True, True, None),
         "half": lambda: gen.main_loop(True, True, gen.ROW_PRIO, lambda j: (j + 2) % 4),
         "twice_readlane": lambda: gen.main_loop(True, True, gen.ROW_PRIO, None, ("readlane",)),
         "twice_table": lambda: gen.main_loop(True, True, gen.ROW_PRIO, None, ("table",)),
         "sload": lambda: gen.main_loop(True, True, gen.ROW_PRIO, None, (), True)}


@pytest.fixture
def four_copies():
    """The tuning loops written for 4 body copies (HALF, DYN)."""
    c0 = gen.NCOPY
    gen.set_ncopy(4)
    yield
    gen.set_ncopy(c0)


@pytest.mark.parametrize("ncopy", [3, 4])
@pytest.mark.parametrize("variant", sorted(LOOPS))
def test_threaded_dispatch_end_to_end_vs_oracle(variant, ncopy):
    if variant == "half" and ncopy != 4:
        pytest.skip("the half-priority stubs exist for 4 copies only")
    c0 = gen.NCOPY
    gen.set_ncopy(ncopy)
    try:
        _threaded_dispatch(variant)
    finally:
        gen.set_ncopy(c0)


def _threaded_dispatch(variant):
    rng = np.random.default_rng(11)
    for nr in (8, 16, 24):
        X = rng.integers(0, 256, (nr, 32), dtype=np.uint8)
        A = rng.integers(0, 256, (8, nr), dtype=np.uint8)
        A[0, 0], A[5, 1] = 0, 1                      # empty body, identity body
        acc = _Wave(X, A, nr, LOOPS[variant]()).run()
        for m in range(8):
            got = bitslice_np(acc[m].view(np.uint8).copy())
            exp = np.zeros(32, np.uint8)
            for k in range(nr):
                exp ^= np.array([oracle.gf_mul(int(A[m, k]), int(b)) for b in X[k]], np.uint8)
            assert np.array_equal(got, exp), (nr, m)


class _DynWave(_Wave):
    """The dynamic-row loop (gen.main_loop_dyn, gf_bs.hip MODE 20): one
    wave of a workgroup sharing the program and the row counter in `shared`.
    Rows are taken one at a time; every row must be consumed exactly once
    across the waves, whatever order they run in."""

    VEC = (gen.D_PG, gen.D_PGN, gen.PL, gen.D_VADDR, gen.D_VCNT, gen.D_VONE, gen.D_VAT)

    def __init__(self, X, A, K, w, kw, shared):
        self.X, self.A, self.nr = X, A, K
        offs, _ = gen.body_offsets()
        self.code, self.addr = [], {}
        for r in range(gen.NCOPY):
            for c in range(256):
                self.addr[self.BASE + offs[r * 256 + c]] = len(self.code)
                self.code += gen.body_lines(c, r)
        self.main0 = len(self.code)
        self.code += [ln.replace("_%=", "") for ln in gen.main_loop_dyn(True)] + ["END"]
        self.labels = {ln[:-1]: i for i, ln in enumerate(self.code) if ln.endswith(":")}
        for name, i in self.labels.items():
            self.addr[0x1000_0000 + 4 * i] = i
        self.s, self.v = {}, {}
        self.m0, self.idx_on = 0, False
        self.lds = shared                      # program at 0x400, counter at 0x40
        self.exec1 = False
        prog = 0x400
        self.ops = {"xlo": 0, "xhi": 0, "nrec": K * 32, "ldx": 32, "thi": self.BASE >> 32, "col": 0,
                    "sc": w, "sn": w + kw, "nk": K, "km1": K - 1, "r0x32": w * 32,
                    "pl": None, "cnt": 0x40}
        self.pl_lanes = [prog + 4 * (lane & 7) for lane in range(64)]
        self.rows_done = []
        self._load_row(gen.RING, w * 32)       # the compiler's first ring load (row w)

    def step(self, ln, op, a, r, pc):
        if op == "s_cmp_ge_u32":
            self.scc = self.val(a[0]) >= self.val(a[1])
            if not self.scc:
                self.rows_done.append(self.s[gen.D_SC])
        elif op == "s_mul_i32":
            self.s[int(a[0][1:])] = self.val(a[1]) * self.val(a[2])
        elif op == "s_min_u32":
            self.s[int(a[0][1:])] = min(self.val(a[1]), self.val(a[2]))
        elif op == "s_lshl_b32":
            self.s[int(a[0][1:])] = self.val(a[1]) << int(a[2])
        elif op == "v_mov_b32" and r[0] in (gen.D_VCNT, gen.D_VONE):
            self.v[r[0]] = [self.val(a[1])] * 64
        elif op == "v_add_u32_e32" and r[0] == gen.D_VADDR:
            self.v[r[0]] = [self.val(a[1]) + x for x in self.v[gen.PL]]
        elif op == "s_mov_b64" and a[0] == "exec":
            self.exec1 = a[1] == "1"
        elif op == "s_mov_b64" and a[1] == "exec":
            assert not self.exec1
        elif op == "ds_add_rtn_u32":
            assert self.exec1                 # one lane: one row per fetch
            addr = self.v[r[1]][0]
            self.v[r[0]] = [self.lds[addr]] + [0xDEAD] * 63
            self.lds[addr] += self.v[r[2]][0]
        elif op == "v_readfirstlane_b32":
            self.s[int(a[0][1:])] = self.v[r[0]][0]
        elif op == "s_cbranch_scc1":
            return self.labels[a[0]] if self.scc else pc
        else:
            return super().step(ln, op, a, r, pc)
        return pc


@pytest.mark.parametrize("K,kw", [(8, 1), (13, 2), (40, 3), (33, 4)])
def test_dynamic_rows_end_to_end_vs_oracle(K, kw, four_copies):
    rng = np.random.default_rng(100 + K)
    X = rng.integers(0, 256, (K, 32), dtype=np.uint8)
    A = rng.integers(0, 256, (8, K), dtype=np.uint8)
    A[0, 0], A[5, 1] = 0, 1
    offs, _ = gen.body_offsets()
    shared = {0x40: 2 * kw}                       # rows 0..2kw-1 are the waves' first two
    for k in range(K):
        for m in range(8):
            shared[0x400 + 4 * (8 * k + m)] = (_Wave.BASE + offs[(m & 3) * 256 + int(A[m, k])]) & 0xFFFFFFFF
    total = np.zeros((8, 8), np.uint32)
    done = []
    order = list(range(kw))[::-1] if K % 2 else list(range(kw))   # any wave order
    for w in order:
        wave = _DynWave(X, A, K, w, kw, shared)
        total ^= wave.run()
        done += wave.rows_done
    assert sorted(done) == list(range(K))         # every row exactly once
    for m in range(8):
        got = bitslice_np(total[m].view(np.uint8).copy())
        exp = np.zeros(32, np.uint8)
        for k in range(K):
            exp ^= np.array([oracle.gf_mul(int(A[m, k]), int(b)) for b in X[k]], np.uint8)
        assert np.array_equal(got, exp), (K, kw, m)


def test_two_row_ring_end_to_end_vs_oracle():
    # the grouped launches' loop (KODR_BS_MAIN_P2, gf_bs_kernel RP = 2): the
    # same interpreter with the ring two rows deep, registers still within
    # 4 waves per SIMD
    p0 = gen.P
    gen.set_ring(2)
    try:
        assert gen.VMAX <= 128 and gen.PG == gen.RING + 16

        class _Wave2(_Wave):
            VEC = (gen.PG, gen.PGN, gen.PL)

        rng = np.random.default_rng(12)
        for nr in (8, 16, 40):
            X = rng.integers(0, 256, (nr, 32), dtype=np.uint8)
            A = rng.integers(0, 256, (8, nr), dtype=np.uint8)
            A[3, 2], A[6, 0] = 0, 1
            acc = _Wave2(X, A, nr, gen.main_loop(True)).run()
            for m in range(8):
                got = bitslice_np(acc[m].view(np.uint8).copy())
                exp = np.zeros(32, np.uint8)
                for k in range(nr):
                    exp ^= np.array([oracle.gf_mul(int(A[m, k]), int(b)) for b in X[k]], np.uint8)
                assert np.array_equal(got, exp), (nr, m)
    finally:
        gen.set_ring(p0)


@pytest.mark.parametrize("ncopy", [2, 3])
@pytest.mark.parametrize("ring", [1, 2])
def test_fewer_copies_end_to_end_vs_oracle(ncopy, ring):
    # the shipped 3 copies and the 2-copy A/B build (KODR_BS_NCOPY): row
    # groups of ncopy rows joined by ceil(8/ncopy)-1 stubs, return address
    # computed per row; SGPRs stay below the kernel's budget
    c0, p0 = gen.NCOPY, gen.P
    gen.set_ncopy(ncopy)
    gen.set_ring(ring)
    try:
        assert gen.CNT <= 101 and gen.RET is None
        offs, total = gen.body_offsets()
        assert total == 16384 * ncopy

        class _WaveC(_Wave):
            VEC = (gen.PG, gen.PGN, gen.PL)

        rng = np.random.default_rng(20 + ncopy)
        for nr in (8, 24):
            X = rng.integers(0, 256, (nr, 32), dtype=np.uint8)
            A = rng.integers(0, 256, (8, nr), dtype=np.uint8)
            A[2, 0], A[7, 1] = 0, 1
            acc = _WaveC(X, A, nr, gen.main_loop(True)).run()
            for m in range(8):
                got = bitslice_np(acc[m].view(np.uint8).copy())
                exp = np.zeros(32, np.uint8)
                for k in range(nr):
                    exp ^= np.array([oracle.gf_mul(int(A[m, k]), int(b)) for b in X[k]], np.uint8)
                assert np.array_equal(got, exp), (ncopy, nr, m)
    finally:
        gen.set_ncopy(c0)
        gen.set_ring(p0)
