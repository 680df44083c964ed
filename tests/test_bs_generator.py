"""CPU checks of the bit-sliced kernel's generated code (kodr_amd/csrc/
gen_bs_bodies.py): a small interpreter runs the emitted row-prep and body
instructions on random bit-sliced blocks and compares every coefficient's
product with the oracle's GF(2^8) multiply (gf256.go:109-118)."""
import os
import re
import sys

import numpy as np

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
        elif op == "v_xor_b32_e32":
            regs[r[0]] = regs[r[1]] ^ regs[r[2]]
        elif op == "v_xor_b32_e64":   # body: acc (indexed) ^= table
            regs[r[0] + idx] = regs[r[1] + idx] ^ regs[r[2]]
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
    off = 0
    for c in range(256):
        assert len(gen.body_ops(c)) <= 8
        assert gen.body_bytes(c) == 8 * len(gen.body_ops(c)) + 4
        off += gen.body_bytes(c)
    assert off < 0xFFFF    # the LDS program stores 16-bit offsets


def test_registers_fit_four_waves():
    assert gen.VMAX <= 128
    assert gen.TL0 % 2 == 0 and gen.TH0 % 2 == 0 and gen.RING % 2 == 0   # v_pk_mov pairs
    used = set(range(gen.ACC, gen.ACC + 64)) | set(range(gen.TL0, gen.TL0 + 15)) | \
        set(range(gen.TH0, gen.TH0 + 15)) | set(range(gen.RING, gen.RING + 8 * gen.P)) | \
        set(range(gen.PR, gen.PR + 4)) | {gen.PL}
    assert len(used) == 64 + 30 + 8 * gen.P + 5          # no overlaps


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
