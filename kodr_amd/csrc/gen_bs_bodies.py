#!/usr/bin/env python3
"""Generate gf_bs_bodies.inc for the bit-sliced kernel (gf_bs.hip).

Bit-sliced layout: a 32-byte block is held as 8 dwords ("planes"); plane i
holds bit i of all 32 bytes (bitslice32 in gf_bs.hip).  Multiplying by c is
GF(2)-linear, so plane j of c*x is the XOR of the input planes i whose matrix
bit M_c[j][i] = bit j of (c * 2^i) is set (poly 0x11D, gf256.go:15-44).

Per input row the wave first builds a table of XOR combinations ("Four
Russians"): TL[s] = XOR of planes {0..3} selected by the 4-bit mask s, TH[s]
the same over planes {4..7} (30 registers, 4 moves + 22 XORs, shared by the 8
output rows).  Then every output plane needs one instruction:

    acc_j ^= TL[S_j & 15] ^ TH[S_j >> 4]        (v_bitop3_b32, XOR3)

so a coefficient's body is at most 8 VALU instructions, one per non-empty S_j.

Threaded dispatch.  A wave applies 8 coefficients per input row (output rows
m = 0..7).  The bodies exist in C = NCOPY copies (3); copy r XORs into
accumulator set r and ends with s_setpc_b64 to T[r+1], so body m jumps
straight to body m+1: one taken branch per body and no SALU inside it
(measured on gfx950: 26 SIMD-cycles per 8-XOR body against 43.6 for a
s_swappc call and return, tools/probe/dispatch.py).  Rows C..7 reuse the
copies under VGPR index mode (SRC0|DST, M0 index 8C per group): a stub
between groups advances M0 and moves the next group's targets into T[1..].
3 copies (48 KB, 2 stubs per row) measured 1-2.5 % faster than 4 (64 KB, 1
stub) at B = 64-256 and in single launches, equal at grouped B = 32; 2
copies (32 KB, 3 stubs) in between (profiles/r03/ncopy_ab/).  8 copies
thrash the instruction cache.

The bodies live in gf_bs_export_kernel, which never runs them: it only exports
their byte offsets.  Every gf_bs_kernel instance jumps into that one copy with
absolute targets that its prologue looked up per coefficient.

Usage: gen_bs_bodies.py > gf_bs_bodies.inc
"""

import os

# Register map: 128 VGPRs in all (4 waves per SIMD), the compiler keeping its
# own values in v[0..ACC).
# (KODR_BS_ACC moves the whole map: A/B builds that give the compiler fewer
# registers of its own to fit a deeper ring)
ACC = int(os.environ.get("KODR_BS_ACC", "12"))  # 8 rows x 8 planes: v[12..75]; copy r owns v[12+8r .. 19+8r]
TL0 = ACC + 64     # TL table, 15 registers v[76..90] (singles first, as aligned pairs)
PL = TL0 + 15      # LDS address of the next program quad
TH0 = PL + 1       # TH table v[92..106]
# ring depth (rows in flight per wave): 1 measured 1.5-2.5 % faster than 2 at
# B = 16-32 in single launches (profiles/r01/bs_ring.log), 2 about 1.7 %
# faster in grouped launches, whose waves stream 64 rows
# (profiles/r02/ring_ab/); the kernel carries both (KODR_BS_MAIN: P, the
# default; KODR_BS_MAIN_P2: two rows).  3 drops to 3 waves per SIMD.
P = int(os.environ.get("KODR_BS_P", "1"))
RING = TH0 + 16    # P row slots x 8 planes: v[108..123]
PG = RING + 8 * P  # program chunk: 8 rows x 8 targets, lane 8j + m (absolute lo words)
PGN = PG + 1       # the next chunk, in flight from LDS
VMAX = PGN + 1     # first VGPR not used by the asm


def set_ring(p):
    """Switch the module's ring depth (and the registers after the ring)."""
    global P, PG, PGN, VMAX
    P, PG = p, RING + 8 * p
    PGN, VMAX = PG + 1, PG + 2
# body copies: rows are taken C = NCOPY at a time (copy r for row m = r + C g,
# M0 index 8 C g), with a stub between groups.  3 (2 stubs per row, 48 KB) is
# the shipped build; 4 (1 stub, 64 KB) and 2 (3 stubs, 32 KB) are A/B builds
# (KODR_BS_NCOPY); the tuning loops HALF and DYN exist for 4 only
NCOPY = int(os.environ.get("KODR_BS_NCOPY", "3"))
assert NCOPY in (2, 3, 4)
# body start alignment in bytes (0: packed back to back); the instruction
# fetch after each s_setpc starts at the body's first byte
ALIGN = int(os.environ.get("KODR_BS_ALIGN", "0"))
# SGPRs (NCOPY = 4): T[0..4] = s[60:69] (T[0] entry, T[r+1] the tail of copy
# r), the second half's targets s[70:77], the stub s[78:79], this row's
# return address s[80:81], the 8 rows' return addresses s[82:97].  With
# fewer copies T[0..C] is shorter, the rows after the first group follow it
# (still ending at s77), the ceil(8/C)-1 stubs start at s78 and the row
# computes its return address itself (no RET table: SGPRs run out)
T0 = 60
H2 = 70
STUB = 78
RT = 80
RET = 82
CNT = 98


def set_ncopy(c):
    """Switch the module's copy count and the SGPR map that depends on it."""
    global NCOPY, H2, RT, RET, CNT
    NCOPY = c
    H2 = T0 + 2 * (c + 1)
    assert H2 + 2 * (8 - c) == STUB
    nst = n_stubs()
    RT = STUB + 2 * nst
    RET = RT + 2 if c == 4 else None
    CNT = RET + 16 if c == 4 else RT + 2


def n_stubs():
    return (8 + NCOPY - 1) // NCOPY - 1


def stub_reg(g):
    """Address register of the stub before row group g (1..)."""
    return STUB + 2 * (g - 1)


def row_target(m):
    """SGPR pair holding row m's target at dispatch: T[m] in the first group,
    the H2 block after it."""
    return T0 + 2 * m if m < NCOPY else H2 + 2 * (m - NCOPY)


def stub_label(g, label="stub"):
    return f"{label}_g{g}" if g > 1 else label


set_ncopy(NCOPY)
GPC = 56           # s_getpc scratch s[56:57]
SP = 46            # scalar-load variant: program pointer s[46:47]
SL = 48            # scalar-load variant: the next row's 8 targets s[48:55]
# table slot of subset s (1..15): the singles 1, 2, 4, 8 first so that each
# pair of them is one aligned v_pk_mov_b32, then the combinations in order
SLOT = {1: 0, 2: 1, 4: 2, 8: 3}
for _s in range(3, 16):
    if _s & (_s - 1):
        SLOT[_s] = len(SLOT)


def gmul(a, b):
    r = 0
    while b:
        if b & 1:
            r ^= a
        a <<= 1
        if a & 0x100:
            a ^= 0x11D
        b >>= 1
    return r


def tl(s):
    return TL0 + SLOT[s]


def th(s):
    return TH0 + SLOT[s]


def body_ops(c):
    """[(j, lo_mask, hi_mask)] for the non-empty output planes of body c."""
    ops = []
    for j in range(8):
        s = sum(1 << i for i in range(8) if (gmul(c, 1 << i) >> j) & 1)
        if s:
            ops.append((j, s & 15, s >> 4))
    return ops


def body_lines(c, r=0):
    """Body of coefficient c in copy r: XOR3s into v[ACC+8r+j] (indexed), then
    jump to T[r+1]."""
    out = []
    for j, lo, hi in body_ops(c):
        a = ACC + 8 * r + j
        if lo and hi:
            out.append(f"v_bitop3_b32 v{a}, v{a}, v{tl(lo)}, v{th(hi)} bitop3:0x96")
        else:  # one table entry: a 4-byte VOP2 XOR (index mode applies to src0 and vdst)
            out.append(f"v_xor_b32_e32 v{a}, v{a}, v{tl(lo) if lo else th(hi)}")
    out.append(f"s_setpc_b64 s[{T0 + 2 * (r + 1)}:{T0 + 2 * (r + 1) + 1}]")
    return out


def body_inline(c, m):
    """Body of coefficient c straight into row m's accumulators, no jump (the
    tuning loop INLINE: the dispatch-free bound of the real kernel)."""
    out = []
    for j, lo, hi in body_ops(c):
        a = ACC + 8 * m + j
        if lo and hi:
            out.append(f"v_bitop3_b32 v{a}, v{a}, v{tl(lo)}, v{th(hi)} bitop3:0x96")
        else:
            out.append(f"v_xor_b32_e32 v{a}, v{a}, v{tl(lo) if lo else th(hi)}")
    return out


def body_bytes(c):
    # v_bitop3 (VOP3) 8 bytes, v_xor_b32_e32 (VOP2) 4, s_setpc_b64 4
    return sum(8 if lo and hi else 4 for _j, lo, hi in body_ops(c)) + 4


def body_offsets():
    """Byte offset of body (r, c) from body (0, 0), index r*256 + c."""
    offs, off = [], 0
    for _r in range(NCOPY):
        for c in range(256):
            if ALIGN:
                off = (off + ALIGN - 1) // ALIGN * ALIGN
            offs.append(off)
            off += body_bytes(c)
    return offs, off


def table_lines(slot):
    """Row prep: TL/TH from ring slot `slot`: singles moved (v_pk_mov_b32),
    pairs and triples XORed straight from the ring (v_xor / v_bitop3), the
    4-subset from two pairs.  Nothing waits on the instruction before it."""
    base = RING + 8 * slot
    out = []
    for i in (0, 2):
        for half, reg in ((0, tl), (1, th)):
            src = base + 4 * half + i
            out.append(f"v_pk_mov_b32 v[{reg(1 << i)}:{reg(1 << i) + 1}], v[{src}:{src + 1}], "
                       f"v[{src}:{src + 1}] op_sel:[0,1]")
    subsets = [s_ for s_ in range(3, 16) if s_ & (s_ - 1)]
    for pop in (2, 3, 4):
        for s_ in subsets:
            if bin(s_).count("1") != pop:
                continue
            for half, reg in ((0, tl), (1, th)):
                srcs = [base + 4 * half + i for i in range(4) if s_ >> i & 1]
                if pop == 2:
                    out.append(f"v_xor_b32_e32 v{reg(s_)}, v{srcs[0]}, v{srcs[1]}")
                elif pop == 3:
                    out.append(f"v_bitop3_b32 v{reg(s_)}, v{srcs[0]}, v{srcs[1]}, v{srcs[2]} bitop3:0x96")
                else:
                    out.append(f"v_xor_b32_e32 v{reg(s_)}, v{reg(3)}, v{reg(12)}")
    return out


# Wave priority of input row j of a chunk.  Without it the SIMD's arbiter
# favours the oldest wave and the 4 waves of a SIMD finish far apart (18-35 k
# cycles, profiles/r01/bs_timeline.log), so the last rows of a launch run at
# low occupancy.  Rotating the priority with the row index lets the waves
# overtake each other: -5 % per B = 32 launch, -6 % at B = 64 (measured against
# 5 other patterns, profiles/r01/bs_prio.log).
def ROW_PRIO(j):
    return j % 4


def row_lines(j, dispatch=True, loads=True, prio=ROW_PRIO, half_prio=None, twice=(), sload=False, inline=None,
              body_prio=None):
    """Input row j (0..7) of an 8-row chunk, from ring slot j % P.  v[PG]
    holds the chunk's program: lane 8j + m = the target of output row m
    (absolute lo word; hi words preset), read with v_readlane, so no LDS round
    trip sits inside a row."""
    slot = j % P
    h = lambda i: T0 + 2 * i  # noqa: E731
    t = [f"s_setprio {prio(j)}"] if prio else []
    if sload:  # targets staged by the previous row's scalar load; fetch the next row's
        t += [f"s_waitcnt vmcnt({2 * (P - 1)}) lgkmcnt(0)"]
        t += [f"s_mov_b32 s{row_target(m)}, s{SL + m}" for m in range(8)]
        t += [f"s_load_dwordx8 s[{SL}:{SL + 7}], s[{SP}:{SP + 1}], 0x0",
              f"s_add_u32 s{SP}, s{SP}, 32", f"s_addc_u32 s{SP + 1}, s{SP + 1}, 0"]
    else:
        t += [f"s_waitcnt vmcnt({2 * (P - 1)}) lgkmcnt(1)"]
        t += [f"v_readlane_b32 s{h(m)}, v{PG}, {8 * j + m}" for m in range(NCOPY)] * (2 if "readlane" in twice else 1)
    t += table_lines(slot) * (2 if "table" in twice else 1)
    b = RING + 8 * slot
    # the row P ahead into this slot (rows past the wave's range read zero)
    if loads:
        t += [f"buffer_load_dwordx4 v[{b}:{b + 3}], %[col], s[40:43], s44 offen",
              f"buffer_load_dwordx4 v[{b + 4}:{b + 7}], %[col], s[40:43], s44 offen offset:16",
              "s_add_u32 s44, s44, s45"]
    if not sload:
        t += [f"v_readlane_b32 s{row_target(m)}, v{PG}, {8 * j + m}"
              for m in range(NCOPY, 8)] * (2 if "readlane" in twice else 1)
    if inline is not None:  # tuning: every output row's body inlined for the fixed coefficient `inline`
        for m in range(8):
            t += body_inline(inline, m)
    elif dispatch:
        C = NCOPY
        if half_prio:  # this row's own stub, which sets the second half's priority
            assert C == 4
            t += [f"s_add_u32 s{h(4)}, s{GPC}, .Lstub{j}_%= - .Lpc_%=",
                  f"s_addc_u32 s{h(4) + 1}, s{GPC + 1}, 0"]
        else:
            t += [f"s_mov_b64 s[{h(C)}:{h(C) + 1}], s[{STUB}:{STUB + 1}]"]
        if 8 % C:  # the last stub put the return address into T[8 % C]: its hi word back
            t += [f"s_mov_b32 s{h(8 % C) + 1}, %[thi]"]
        if RET is not None:
            t += [f"s_mov_b64 s[{RT}:{RT + 1}], s[{RET + 2 * j}:{RET + 2 * j + 1}]"]
        else:
            t += [f"s_add_u32 s{RT}, s{GPC}, .Lret{j}_%= - .Lpc_%=", f"s_addc_u32 s{RT + 1}, s{GPC + 1}, 0"]
        if body_prio is not None:  # tuning: another priority for the bodies than for the row's preparation
            t += [f"s_setprio {body_prio}"]
        t += ["s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)",
              f"s_setpc_b64 s[{h(0)}:{h(0) + 1}]",
              f".Lret{j}_%=:",
              "s_set_gpr_idx_off"]
    return t


def stub_lines(label="stub", prio=None):
    """Between row groups: group g (rows C g .. C g + n - 1) reuses copies
    0..n-1 at M0 index 8 C g, with targets T[1..n-1] from the later rows'
    registers and T[n] the next stub, or the row's return address after the
    last group (NCOPY = 4: one stub, rows 4..7 at index 32)."""
    h = lambda i: T0 + 2 * i  # noqa: E731
    C, ng = NCOPY, n_stubs() + 1
    t = []
    for g in range(1, ng):
        n = min(C, 8 - C * g)
        t += [f".L{stub_label(g, label)}_%=:"] + ([f"s_setprio {prio}"] if prio is not None else [])
        t += [f"s_add_u32 m0, m0, {8 * C}"]
        t += [f"s_mov_b64 s[{h(i)}:{h(i) + 1}], s[{row_target(C * g + i)}:{row_target(C * g + i) + 1}]"
              for i in range(1, n)]
        nxt = stub_reg(g + 1) if g + 1 < ng else RT
        t += [f"s_mov_b64 s[{h(n)}:{h(n) + 1}], s[{nxt}:{nxt + 1}]",
              f"s_setpc_b64 s[{row_target(C * g)}:{row_target(C * g) + 1}]"]
    return t


def prologue_lines(dispatch=True, sload=False):
    """Descriptor, stub and per-row return addresses, target hi words, the
    first two program chunks, zeroed accumulators.  SGPRs: s[40:43] X
    descriptor (num_records = end of this wave's rows), s44 row offset,
    s45 ldx."""
    pro = ["s_mov_b32 s40, %[xlo]", "s_and_b32 s41, %[xhi], 0xffff", "s_mov_b32 s42, %[nrec]",
           "s_mov_b32 s43, 0x00020000", "s_mov_b32 s44, %[roff]", "s_mov_b32 s45, %[ldx]",
           f"s_getpc_b64 s[{GPC}:{GPC + 1}]", ".Lpc_%=:"]
    if dispatch:
        regs = [(stub_reg(g), stub_label(g)) for g in range(1, n_stubs() + 1)]
        if RET is not None:
            regs += [(RET + 2 * j, f"ret{j}") for j in range(8)]
        for reg, lab in regs:
            pro += [f"s_add_u32 s{reg}, s{GPC}, .L{lab}_%= - .Lpc_%=",
                    f"s_addc_u32 s{reg + 1}, s{GPC + 1}, 0"]
    pro += [f"s_mov_b32 s{row_target(m) + 1}, %[thi]" for m in range(8)]
    if sload:  # the wave's program in global memory, one 32-byte row of targets at a time
        pro += [f"s_mov_b32 s{SP}, %[pglo]", f"s_mov_b32 s{SP + 1}, %[pghi]",
                f"s_load_dwordx8 s[{SL}:{SL + 7}], s[{SP}:{SP + 1}], 0x0",
                f"s_add_u32 s{SP}, s{SP}, 32", f"s_addc_u32 s{SP + 1}, s{SP + 1}, 0"]
    else:
        pro += [f"v_mov_b32 v{PL}, %[pl]", f"ds_read_b32 v{PG}, v{PL}", f"ds_read_b32 v{PGN}, v{PL} offset:256",
                f"v_add_u32_e32 v{PL}, 512, v{PL}"]
    pro += [f"v_mov_b32 v{ACC + r}, 0" for r in range(64)]
    pro += [f"s_mov_b32 s{CNT}, %[ngrp]"]
    return pro


def main_loop(dispatch=True, loads=True, prio=ROW_PRIO, half_prio=None, twice=(), sload=False, inline=None,
              body_prio=None):
    """Prologue, the shared stub (branched over) and the 8-row loop; the
    ring's first P rows arrive as asm operands (loaded by the compiler before
    the program build).  At the end of each iteration the next chunk moves
    into v[PG] and the one after is requested."""
    t = prologue_lines(dispatch, sload)
    if dispatch:
        t += ["s_branch .Lloop_%="] + stub_lines()
        if half_prio:
            for j in range(8):
                t += stub_lines(f"stub{j}", half_prio(j))
    t += [".Lloop_%=:"]
    for j in range(8):
        t += row_lines(j, dispatch, loads, prio, half_prio, twice, sload, inline, body_prio)
    if not sload:
        t += ["s_waitcnt lgkmcnt(0)", f"v_mov_b32 v{PG}, v{PGN}", f"ds_read_b32 v{PGN}, v{PL}",
              f"v_add_u32_e32 v{PL}, 256, v{PL}"]
    t += [f"s_sub_u32 s{CNT}, s{CNT}, 1", f"s_cmp_lg_u32 s{CNT}, 0", "s_cbranch_scc1 .Lloop_%="]
    if prio:
        t += ["s_setprio 0"]
    return t


# Dynamic rows (gf_bs.hip MODE 20): the KW waves of a workgroup share one
# program (K rows x 8 targets in LDS) and take input rows one at a time from
# an LDS counter, so a wave the SIMD's arbiter serves less takes fewer rows
# and the waves of a workgroup finish together (with a static K split they
# finished 18-35 k cycles apart, profiles/r01/bs_timeline.log).  Per row the
# wave knows its row I (SC) and its next row I' (SN); during row I it loads
# row I' (ring) and its targets (PG/PGN, alternating), and fetches the row
# after I' with one ds_add_rtn_u32 from a single lane.
D_EX = 46          # s[46:47] exec save
D_SC, D_SN, D_SK, D_SKM1, D_TMP = 48, 49, 50, 51, 52
D_VAT = RING - 1   # the fetched row index (lane 0)
D_PG, D_PGN = RING + 8 * P, RING + 8 * P + 1   # targets of the current / next row (lanes 0..7)
D_VADDR, D_VCNT, D_VONE = D_PG + 2, D_PG + 3, D_PG + 4
D_VMAX = D_VONE + 1
D_ROWS = 4         # rows per loop iteration (priority rotation j % 4, PG/PGN alternate)


def row_lines_dyn(j, dispatch=True, prio=ROW_PRIO):
    assert P == 1
    pgc, pgn = (D_PG, D_PGN) if j % 2 == 0 else (D_PGN, D_PG)
    h = lambda i: T0 + 2 * i  # noqa: E731
    t = [f"s_cmp_ge_u32 s{D_SC}, s{D_SK}", "s_cbranch_scc1 .Ldone_%="]
    t += [f"s_setprio {prio(j)}"] if prio else []
    t += ["s_waitcnt vmcnt(0)"]
    t += [f"v_readlane_b32 s{h(m)}, v{pgc}, {m}" for m in range(4)]
    t += table_lines(0)
    b = RING
    t += [f"s_mul_i32 s44, s{D_SN}, s45",
          f"buffer_load_dwordx4 v[{b}:{b + 3}], %[col], s[40:43], s44 offen",
          f"buffer_load_dwordx4 v[{b + 4}:{b + 7}], %[col], s[40:43], s44 offen offset:16"]
    t += [f"v_readlane_b32 s{H2 + 2 * m}, v{pgc}, {4 + m}" for m in range(4)]
    t += [f"s_min_u32 s{D_TMP}, s{D_SN}, s{D_SKM1}", f"s_lshl_b32 s{D_TMP}, s{D_TMP}, 5",
          f"v_add_u32_e32 v{D_VADDR}, s{D_TMP}, v{PL}", f"ds_read_b32 v{pgn}, v{D_VADDR}",
          f"s_mov_b64 s[{D_EX}:{D_EX + 1}], exec", "s_mov_b64 exec, 1",
          f"ds_add_rtn_u32 v{D_VAT}, v{D_VCNT}, v{D_VONE}", f"s_mov_b64 exec, s[{D_EX}:{D_EX + 1}]"]
    if dispatch:
        t += [f"s_mov_b64 s[{h(4)}:{h(4) + 1}], s[{STUB}:{STUB + 1}]",
              f"s_mov_b64 s[{RT}:{RT + 1}], s[{RET + 2 * j}:{RET + 2 * j + 1}]",
              "s_set_gpr_idx_on 0, gpr_idx(SRC0,DST)",
              f"s_setpc_b64 s[{h(0)}:{h(0) + 1}]",
              f".Lret{j}_%=:",
              "s_set_gpr_idx_off"]
    t += ["s_waitcnt lgkmcnt(0)", f"s_mov_b32 s{D_SC}, s{D_SN}", f"v_readfirstlane_b32 s{D_SN}, v{D_VAT}"]
    return t


def main_loop_dyn(dispatch=True, prio=ROW_PRIO):
    """Prologue (descriptor, stub/return addresses, hi words, row registers,
    the first row's targets, zeroed accumulators), the stub, and the 4-row
    loop; exits when the wave's next row is past K.  Operands: %[sc] the
    wave's first row, %[sn] its second, %[nk] K, %[km1] K - 1, %[r0x32] the
    first row * 32, %[pl] this lane's program address (program + (lane & 7) * 4),
    %[cnt] the counter's LDS address."""
    pro = ["s_mov_b32 s40, %[xlo]", "s_and_b32 s41, %[xhi], 0xffff", "s_mov_b32 s42, %[nrec]",
           "s_mov_b32 s43, 0x00020000", "s_mov_b32 s45, %[ldx]",
           f"s_getpc_b64 s[{GPC}:{GPC + 1}]", ".Lpc_%=:"]
    if dispatch:
        for reg, lab in [(STUB, "stub")] + [(RET + 2 * j, f"ret{j}") for j in range(D_ROWS)]:
            pro += [f"s_add_u32 s{reg}, s{GPC}, .L{lab}_%= - .Lpc_%=",
                    f"s_addc_u32 s{reg + 1}, s{GPC + 1}, 0"]
    pro += [f"s_mov_b32 s{T0 + 2 * i + 1}, %[thi]" for i in range(4)]
    pro += [f"s_mov_b32 s{H2 + 2 * i + 1}, %[thi]" for i in range(4)]
    pro += [f"s_mov_b32 s{D_SC}, %[sc]", f"s_mov_b32 s{D_SN}, %[sn]", f"s_mov_b32 s{D_SK}, %[nk]",
            f"s_mov_b32 s{D_SKM1}, %[km1]",
            f"v_mov_b32 v{PL}, %[pl]", f"v_mov_b32 v{D_VCNT}, %[cnt]", f"v_mov_b32 v{D_VONE}, 1",
            f"v_add_u32_e32 v{D_VADDR}, %[r0x32], v{PL}", f"ds_read_b32 v{D_PG}, v{D_VADDR}"]
    pro += [f"v_mov_b32 v{ACC + r}, 0" for r in range(64)]
    pro += ["s_waitcnt lgkmcnt(0)"]
    t = pro
    if dispatch:
        t += ["s_branch .Lloop_%="] + stub_lines()
    t += [".Lloop_%=:"]
    for j in range(D_ROWS):
        t += row_lines_dyn(j, dispatch, prio)
    t += ["s_branch .Lloop_%=", ".Ldone_%=:"]
    if prio:
        t += ["s_setprio 0"]
    return t


def dump_lines():
    """Bring-up only (MODE 9): the prologue and the first row's target reads,
    then s[60:99] and M0 stored to %[ydbg] (lane 0's values), no jump taken."""
    t = prologue_lines(True) + ["s_waitcnt lgkmcnt(0)"]
    t += [f"v_readlane_b32 s{T0 + 2 * m}, v{PG}, {m}" for m in range(4)]
    t += [f"v_readlane_b32 s{H2 + 2 * m}, v{PG}, {4 + m}" for m in range(4)]
    t += [f"v_mov_b32 v{ACC + 1}, 0"]
    for i, sg in enumerate(list(range(T0, CNT + 1)) + ["m0"]):
        src = f"s{sg}" if sg != "m0" else "m0"
        t += [f"v_mov_b32 v{ACC}, {src}",
              f"global_store_dword v{ACC + 1}, v{ACC}, %[ydbg] offset:{4 * i}"]
    t += ["s_waitcnt vmcnt(0)"]
    t += [f".L{stub_label(g)}_%=:" for g in range(1, n_stubs() + 1)]   # never jumped to
    t += [f".Lret{j}_%=:" for j in range(8)]
    return t




def emit(name, lines):
    res = [f"#define {name} \\"]
    res += [f'  "{ln}\\n\\t" \\' for ln in lines]
    res.append('  ""')
    return res


def main():
    out = ["// generated by gen_bs_bodies.py -- do not edit",
           f"// accumulators v[{ACC}..{ACC + 63}] (copy r: v[{ACC}+8r..], +32 under index mode),",
           f"// XOR tables v[{TL0}..{TH0 + 14}], row ring v[{RING}..{RING + 8 * P - 1}], "
           f"program chunks v[{PG}..{VMAX - 1}]",
           f"#define KODR_BS_VMAX {VMAX}",
           f"#define KODR_BS_P {P}",
           f"#define KODR_BS_NCOPY {NCOPY}"]
    ops = [f'"+{{v[{RING + 4 * i}:{RING + 4 * i + 3}]}}"(ring[{i}])' for i in range(2 * P)]
    out.append("#define KODR_BS_RING_OPERANDS " + ", ".join(ops))
    bodies = []
    n_inst = 0
    for r in range(NCOPY):
        for c in range(256):
            if ALIGN:
                bodies.append(f".p2align {ALIGN.bit_length() - 1}")
            bodies.append(f".Lbs_b{r}_{c}_%=:")
            lines = body_lines(c, r)
            n_inst += len(lines) - 1
            bodies += lines
    out += emit("KODR_BS_BODIES", bodies)
    offs, total = body_offsets()
    out.append(f"#define KODR_BS_CODE_BYTES {total}")
    out.append(f"#define KODR_BS_COPY_BYTES {offs[256]}u")
    out.append("static const uint32_t kBsBodyOffsets[%d] = {" % len(offs))
    for i in range(0, len(offs), 16):
        out.append("  " + ", ".join(str(o) for o in offs[i:i + 16]) + ",")
    out.append("};")
    # export: the absolute address of body (0, 0) (s_getpc) and every body's
    # offset from it, stored by lane-uniform global stores (once per process,
    # checked against kBsBodyOffsets)
    out.append("#define KODR_BS_EXPORT(VTMP, VZERO, VOFF, SOUT) \\")
    out.append('  "s_getpc_b64 s[88:89]\\n\\t" \\')
    out.append('  ".Lexpc_%=:\\n\\t" \\')
    # the bodies precede the export code: subtract with borrow (an add of the
    # negative difference would carry into the hi word)
    out.append('  "s_sub_u32 s88, s88, .Lexpc_%= - .Lbs_b0_0_%=\\n\\t" \\')
    out.append('  "s_subb_u32 s89, s89, 0\\n\\t" \\')
    out.append(f'  "v_mov_b32 " VOFF ", {4 * NCOPY * 256}\\n\\t" \\')
    out.append('  "v_mov_b32 " VTMP ", s88\\n\\t" \\')
    out.append('  "global_store_dword " VOFF ", " VTMP ", " SOUT "\\n\\t" \\')
    out.append('  "v_mov_b32 " VTMP ", s89\\n\\t" \\')
    out.append('  "global_store_dword " VOFF ", " VTMP ", " SOUT " offset:4\\n\\t" \\')
    for r in range(NCOPY):
        for c in range(256):
            i = r * 256 + c
            out.append(f'  "v_mov_b32 " VTMP ", .Lbs_b{r}_{c}_%= - .Lbs_b0_0_%=\\n\\t" \\')
            out.append(f'  "global_store_dword " VZERO ", " VTMP ", " SOUT " offset:{4 * i}\\n\\t" \\')
    out.append('  "s_waitcnt vmcnt(0)\\n\\t"')
    out += emit("KODR_BS_MAIN", main_loop(True))
    out += emit("KODR_BS_MAIN_ND", main_loop(False))
    out += emit("KODR_BS_MAIN_NL", main_loop(True, False))
    out += emit("KODR_BS_MAIN_NDNL", main_loop(False, False))
    # tuning: the loop without the priority rotation (MODE 10)
    out += emit("KODR_BS_MAIN_NOPRIO", main_loop(True, True, None))
    out += emit("KODR_BS_MAIN_HALF", main_loop(True, True, ROW_PRIO, lambda j: (j + 2) % 4) if NCOPY == 4 else [])
    # cost probes: the row's target reads or its tables issued twice (same result)
    out += emit("KODR_BS_MAIN_2RL", main_loop(True, True, ROW_PRIO, None, ("readlane",)))
    out += emit("KODR_BS_MAIN_2TB", main_loop(True, True, ROW_PRIO, None, ("table",)))
    # program through scalar loads instead of LDS + v_readlane (MODE 14)
    out += emit("KODR_BS_MAIN_SLOAD", main_loop(True, True, ROW_PRIO, None, (), True))
    out += emit("KODR_BS_DUMP", dump_lines())
    # dynamic rows (MODE 20)
    # (a one-row ring only; other ring depths build it empty, and only a
    # tuning build instantiates MODE 20)
    out += emit("KODR_BS_MAIN_DYN", main_loop_dyn(True) if P == 1 and NCOPY == 4 else [])
    out.append(f"#define KODR_BS_DYN_VMAX {D_VMAX}")
    red = [f"ds_xor_b32 %[lds], v{ACC + r} offset:{256 * r}" for r in range(64)]
    out += emit("KODR_BS_REDUCE", red)
    # the ring v[RING..RING+8P) is bound to in/out operands, not clobbered
    clob = [f'"v{r}"' for r in list(range(ACC, RING)) + list(range(RING + 8 * P, VMAX))]
    assert CNT <= 101 and GPC + 1 < T0
    clob += [f'"s{r}"' for r in list(range(40, 46)) + [GPC, GPC + 1] + list(range(T0, CNT + 1))]
    out.append("#define KODR_BS_CLOBBERS " + ", ".join(clob) + ', "scc", "memory"')
    dclob = [f'"v{r}"' for r in list(range(ACC, RING)) + list(range(RING + 8 * P, D_VMAX))]
    dclob += [f'"s{r}"' for r in list(range(40, 46)) + list(range(D_EX, D_TMP + 1)) + [GPC, GPC + 1] +
              list(range(T0, (RET or RT) + 2 * D_ROWS))]
    out.append("#define KODR_BS_CLOBBERS_DYN " + ", ".join(dclob) + ', "scc", "memory"')
    out.append("#define KODR_BS_CLOBBERS_SLOAD " + ", ".join(clob + [f'"s{r}"' for r in range(SP, SL + 8)]) +
               ', "scc", "memory"')
    # the two-row ring variant (grouped launches): main loop, ring operands,
    # clobbers, register count
    p0 = P
    set_ring(2)
    out += emit("KODR_BS_MAIN_P2", main_loop(True))
    # tuning (MODE 30): the grouped two-row loop with every body inlined for
    # one coefficient (19: eight XOR3s) -- no jumps, wrong products
    out += emit("KODR_BS_MAIN_P2_INLINE", main_loop(True, inline=19))
    # tuning (MODE 31 / 32): the grouped two-row loop without the row stream
    # (the ring's stale rows; wrong products), with threaded / inlined bodies:
    # what any load path (LDS staging, deeper prefetch) could save at most
    out += emit("KODR_BS_MAIN_P2_NL", main_loop(True, False))
    # tuning (MODE 35): the grouped two-row loop without the priority rotation
    out += emit("KODR_BS_MAIN_P2_NOPRIO", main_loop(True, True, None))
    # tuning (MODE 36): the rotation over the rows' pairs (priority j // 2 % 4)
    out += emit("KODR_BS_MAIN_P2_PRIO2", main_loop(True, True, lambda j: (j // 2) % 4))
    # tuning (MODE 37): the row's preparation (tables, targets) at priority 3,
    # its bodies at 0 (the preparation is the wave's dependency chain)
    out += emit("KODR_BS_MAIN_P2_PREP", main_loop(True, True, lambda j: 3, body_prio=0))
    out += emit("KODR_BS_MAIN_P2_INLINE_NL", main_loop(True, False, inline=19))
    ops2 = [f'"+{{v[{RING + 4 * i}:{RING + 4 * i + 3}]}}"(ring[{i}])' for i in range(2 * P)]
    out.append("#define KODR_BS_RING_OPERANDS_P2 " + ", ".join(ops2))
    clob2 = [f'"v{r}"' for r in list(range(ACC, RING)) + list(range(RING + 8 * P, VMAX))]
    clob2 += [f'"s{r}"' for r in list(range(40, 46)) + [GPC, GPC + 1] + list(range(T0, CNT + 1))]
    out.append("#define KODR_BS_CLOBBERS_P2 " + ", ".join(clob2) + ', "scc", "memory"')
    out.append(f"#define KODR_BS_VMAX_P2 {VMAX}")
    # direct variant (KW = 1, no cross-wave fold): the accumulators leave the
    # asm as outputs (early clobber: the prologue zeroes them before it reads
    # every input) and the C++ epilogue transposes and stores them
    acc_out = [f'"=&{{v[{ACC + 8 * m}:{ACC + 8 * m + 7}]}}"(acc[{m}])' for m in range(8)]
    out.append("#define KODR_BS_ACC_OUTPUTS " + ", ".join(acc_out))
    clob2d = [f'"v{r}"' for r in list(range(ACC + 64, RING)) + list(range(RING + 8 * P, VMAX))]
    clob2d += [f'"s{r}"' for r in list(range(40, 46)) + [GPC, GPC + 1] + list(range(T0, CNT + 1))]
    out.append("#define KODR_BS_CLOBBERS_P2_DIRECT " + ", ".join(clob2d) + ', "scc", "memory"')
    # the three-row ring (tuning, MODE 33: direct grouped launches), which fits
    # 4 waves per SIMD only with the map moved down (KODR_BS_ACC=4)
    set_ring(3)
    out += emit("KODR_BS_MAIN_P3", main_loop(True))
    ops3 = [f'"+{{v[{RING + 4 * i}:{RING + 4 * i + 3}]}}"(ring[{i}])' for i in range(2 * P)]
    out.append("#define KODR_BS_RING_OPERANDS_P3 " + ", ".join(ops3))
    clob3d = [f'"v{r}"' for r in list(range(ACC + 64, RING)) + list(range(RING + 8 * P, VMAX))]
    clob3d += [f'"s{r}"' for r in list(range(40, 46)) + [GPC, GPC + 1] + list(range(T0, CNT + 1))]
    out.append("#define KODR_BS_CLOBBERS_P3_DIRECT " + ", ".join(clob3d) + ', "scc", "memory"')
    out.append(f"#define KODR_BS_VMAX_P3 {VMAX}")
    set_ring(p0)
    out.append(f"// {n_inst} body instructions in {NCOPY} copies, {n_inst / 256 / NCOPY:.2f} per coefficient; "
               f"row prep {len(table_lines(0))} per row; {total} bytes of bodies")
    print("\n".join(out))


if __name__ == "__main__":
    main()
