#!/usr/bin/env python3
"""Generate gf_bs_bodies.inc for the bit-sliced kernel (gf_bs.hip).

Bit-sliced layout: a 32-byte block is held as 8 dwords ("planes"); plane i
holds bit i of all 32 bytes (bitslice32 in gf_bs.hip).  Multiplying by c is
GF(2)-linear, so plane j of c*x is the XOR of the input planes i whose matrix
bit M_c[j][i] = bit j of (c * 2^i) is set (poly 0x11D, gf256.go:15-44).

Per input row the wave first builds a table of XOR combinations ("Four
Russians"): TL[s] = XOR of planes {0..3} selected by the 4-bit mask s, TH[s]
the same over planes {4..7} (30 registers, 8 moves + 22 XORs, shared by the 8
output rows).  Then every output plane needs one instruction:

    acc_j ^= TL[S_j & 15] ^ TH[S_j >> 4]        (v_bitop3_b32, XOR3)

so a coefficient's body is at most 8 VALU instructions, one per non-empty
S_j.  Bodies address the accumulators v[ACC..ACC+7] under VGPR index mode
(SRC0|DST) so one body serves every output row m (index 8m); the table is
read through src1/src2, unindexed.  The wave reaches body[c] with s_swappc_b64
and the body returns with s_setpc_b64.

Usage: gen_bs_bodies.py > gf_bs_bodies.inc
"""

# Register map: 128 VGPRs in all (4 waves per SIMD), the compiler keeping its
# own values in v[0..ACC).
ACC = 12           # 8 rows x 8 planes: v[12..75]
TL0 = 76           # TL table, 15 registers v[76..90] (singles first, as aligned pairs)
PL = 91            # LDS address of the next program row
TH0 = 92           # TH table v[92..106]
P = 2              # ring depth (rows in flight per wave)
RING = 108         # P row slots x 8 planes: v[108..123]
PR = RING + 8 * P  # next row's packed offsets, read from the LDS program: v[124..127]
RET = 54           # return address s[54:55]
OCT = 56           # s[56:59]: this row's 8 body offsets, two 16-bit offsets per SGPR
VMAX = PR + 4      # first VGPR not used by the asm
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


def body_lines(c):
    out = []
    for j, lo, hi in body_ops(c):
        a = ACC + j
        if lo and hi:
            out.append(f"v_bitop3_b32 v{a}, v{a}, v{tl(lo)}, v{th(hi)} bitop3:0x96")
        else:
            out.append(f"v_xor_b32_e64 v{a}, v{a}, v{tl(lo) if lo else th(hi)}")
    out.append(f"s_setpc_b64 s[{RET}:{RET + 1}]")
    return out


def body_bytes(c):
    return 8 * len(body_ops(c)) + 4      # VOP3 = 8 bytes, s_setpc_b64 = 4


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


def main_loop():
    """Row macros.  The ring's first 4 rows arrive as asm inputs (loaded by the
    compiler before the program build); the program (8 body offsets per row)
    is in LDS at %[pl].  SGPRs: s[40:43] X descriptor, s44 row offset, s45
    ldx, s[50:51] body 0, s[52:53] jump target, s[56:63] this row's offsets,
    s72 group counter."""
    def row(slot, wait, loads, dispatch=True, rfl=True, prog=True):
        t = [f"s_waitcnt vmcnt({wait}) lgkmcnt(0)"]
        # this row's offsets to SGPRs, then fetch the next row's (an LDS read
        # past the last row reads unused LDS and is never consumed)
        if rfl:
            t += [f"v_readfirstlane_b32 s{OCT + i}, v{PR + i}" for i in range(4)]
        if prog:
            t += [f"ds_read_b128 v[{PR}:{PR + 3}], v{PL}", f"v_add_u32_e32 v{PL}, 16, v{PL}"]
        t += table_lines(slot)
        if loads:
            b = RING + 8 * slot
            t += [f"buffer_load_dwordx4 v[{b}:{b + 3}], %[col], s[40:43], s44 offen",
                  f"buffer_load_dwordx4 v[{b + 4}:{b + 7}], %[col], s[40:43], s44 offen offset:16",
                  "s_add_u32 s44, s44, s45"]
        for m in range(8 if dispatch else 0):
            half = (f"s_and_b32 s60, s{OCT + m // 2}, 0xffff" if m % 2 == 0
                    else f"s_lshr_b32 s60, s{OCT + m // 2}, 16")
            t += [half, "s_add_u32 s52, s50, s60", "s_addc_u32 s53, s51, 0",
                  f"s_set_gpr_idx_on {8 * m}, gpr_idx(SRC0,DST)",
                  f"s_swappc_b64 s[{RET}:{RET + 1}], s[52:53]", "s_set_gpr_idx_off"]
        return t

    pro = [f"v_mov_b32 v{PL}, %[pl]", f"ds_read_b128 v[{PR}:{PR + 3}], v{PL}", f"v_add_u32_e32 v{PL}, 16, v{PL}"]
    pro += [f"v_mov_b32 v{ACC + r}, 0" for r in range(64)]
    loop = []
    for slot in range(P):
        loop += row(slot, 2 * (P - 1), True)
    tail = []
    for slot in range(P):
        tail += row(slot, 2 * (P - 1 - slot), False)
    red = [f"ds_xor_b32 %[lds], v{ACC + r} offset:{256 * r}" for r in range(64)]
    # tuning variants (KODR_TUNE_MODES builds only): rows without body dispatch
    loop_nd, tail_nd = [], []
    for slot in range(P):
        loop_nd += row(slot, 2 * (P - 1), True, False)
        tail_nd += row(slot, 2 * (P - 1 - slot), False, False)
    loop_nl, loop_nl2, loop_nl3 = [], [], []
    for slot in range(P):
        loop_nl += row(slot, 2 * (P - 1), False, False)
        loop_nl2 += row(slot, 2 * (P - 1), False, False, rfl=False)
        loop_nl3 += row(slot, 2 * (P - 1), False, False, rfl=False, prog=False)
    return [("KODR_BS_PROLOGUE", pro), ("KODR_BS_LOOP", loop), ("KODR_BS_TAIL", tail),
            ("KODR_BS_REDUCE", red), ("KODR_BS_LOOP_ND", loop_nd), ("KODR_BS_TAIL_ND", tail_nd),
            ("KODR_BS_LOOP_NL", loop_nl), ("KODR_BS_LOOP_NL2", loop_nl2), ("KODR_BS_LOOP_NL3", loop_nl3)]


def emit(name, lines):
    res = [f"#define {name} \\"]
    res += [f'  "{l}\\n\\t" \\' for l in lines]
    res.append('  ""')
    return res


def main():
    out = ["// generated by gen_bs_bodies.py -- do not edit",
           f"// accumulators v[{ACC}..{ACC + 63}] (indexed), XOR tables v[{TL0}..{TH0 + 14}],",
           f"// row ring v[{RING}..{VMAX - 1}], return s[{RET}:{RET + 1}]",
           f"#define KODR_BS_VMAX {VMAX}",
           f"#define KODR_BS_P {P}"]
    # the ring rows enter the asm as in/out operands pinned to their slots
    ops = [f'"+{{v[{RING + 4 * i}:{RING + 4 * i + 3}]}}"(ring[{i}])' for i in range(2 * P)]
    out.append("#define KODR_BS_RING_OPERANDS " + ", ".join(ops))
    bodies = []
    n_inst = 0
    for c in range(256):
        bodies.append(f".Lbs_b{c}_%=:")
        lines = body_lines(c)
        n_inst += len(lines) - 1
        bodies += lines
    out += emit("KODR_BS_BODIES", bodies)
    # export: offsets of every body from body 0, stored by lane-uniform global
    # stores to SOUT + 4c (used once per process, checked against body_bytes)
    out.append("#define KODR_BS_EXPORT(VTMP, VZERO, SOUT) \\")
    for c in range(256):
        out.append(f'  "v_mov_b32 " VTMP ", .Lbs_b{c}_%= - .Lbs_b0_%=\\n\\t" \\')
        out.append(f'  "global_store_dword " VZERO ", " VTMP ", " SOUT " offset:{4 * c}\\n\\t" \\')
    out.append('  "s_waitcnt vmcnt(0)\\n\\t"')
    for name, lines in main_loop():
        out += emit(name, lines)
    # the ring v[RING..RING+8P) is bound to in/out operands, not clobbered
    clob = [f'"v{r}"' for r in list(range(ACC, RING)) + list(range(RING + 8 * P, VMAX))]
    clob += [f'"s{r}"' for r in list(range(40, 46)) + list(range(50, 61)) + [72, 74, 75]]
    out.append("#define KODR_BS_CLOBBERS " + ", ".join(clob) + ', "scc", "memory"')
    out.append(f"// {n_inst} body instructions, {n_inst / 256:.2f} per coefficient; "
               f"row prep {len(table_lines(0))} per row")
    print("\n".join(out))


if __name__ == "__main__":
    main()
