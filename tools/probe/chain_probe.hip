// Critical-path probe for gf_elim_mc2_kernel's chain (measurement only, not
// part of the library): one 1024-thread workgroup; chain wave 8 runs the
// owned-panel work of the kernel -- the two small products that bring a
// 16 x 16 block up to date with the previous panel, then its inversion --
// ITER times on random data staged in LDS, stamping s_memtime around each
// phase.  The other 15 waves either exit (mode 0), poll an LDS word with
// s_sleep 1 as mc2_wait does (mode 1), or run row-update work like the row
// waves' apply (mode 2, waves 0-7) while 9-15 poll (the kernel's situation).
// Variants of each phase are compared on the same inputs; S of every
// iteration is checked against a host Gauss-Jordan.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I kodr_amd/csrc tools/probe/chain_probe.hip -o tools/probe/chain_probe
#include "../../kodr_amd/csrc/gf_elim.hip"

#include <stdio.h>
#include <string.h>

#include <vector>

namespace kodr_amd {
namespace {

// The library's mc2 LDS plus the probe's scratch (the panel block and the
// split variants' partial products live here, not in the kernel).
struct ProbeLds {
  uint4 tab[256 * 2];
  uint4 itab[256 * 2];
  uint32_t rp[kMc2Slots][16][64];
  uint32_t sp[kMc2Slots][16][4];
  uint32_t mb[kMc2Slots][16][8];
  uint32_t pan[16][4];
  uint32_t ft[16][4];
  int chain_cnt;
  int fail;
};

// ---- chain variants measured here and not kept in the library ----
// mc_panel_gj's algorithm on an LDS block, S to `s_out` ([16][4]), its rows
// also kept in registers for publishing (returns false if singular)
// lane (t, d) gets dword d of block row tp: four v_readlane and a select,
// instead of a ds_bpermute round trip
__device__ __forceinline__ uint32_t row_bcast(uint32_t v, int tp, int d) {
  const uint32_t a0 = __builtin_amdgcn_readlane(v, 4 * tp), a1 = __builtin_amdgcn_readlane(v, 4 * tp + 1);
  const uint32_t a2 = __builtin_amdgcn_readlane(v, 4 * tp + 2), a3 = __builtin_amdgcn_readlane(v, 4 * tp + 3);
  return d == 0 ? a0 : d == 1 ? a1 : d == 2 ? a2 : a3;
}

template <bool RL>
__device__ __forceinline__ bool mc2_panel_gj(const uint4* tab, const uint4* itab, const uint32_t (*pan)[4],
                                             uint32_t (*s_out)[4], int lane, uint32_t* s_val, int* s_row) {
  const int t = lane >> 2, d = lane & 3;
  uint32_t P = pan[t][d], Tr = (t >> 2) == d ? 1u << (8 * (t & 3)) : 0u;
  uint32_t used = 0;
  int mycol = 0;
#pragma unroll
  for (int c = 0; c < 16; c++) {
    const int cd = c >> 2, cb = 8 * (c & 3);
    const uint32_t f = (quad_bcast(P, cd) >> cb) & 0xffu;
    const uint4 tf = tab[2 * f];
    const uint32_t tf2 = tab[2 * f + 1].x;
    const bool nz = d == 0 && f != 0u && !((used >> t) & 1u);
    const uint64_t m = __builtin_amdgcn_ballot_w64(nz);
    if (m == 0) return false;
    const int pl = __builtin_ctzll(m), tp = pl >> 2;
    const uint32_t dp = __builtin_amdgcn_readlane(f, pl);
    const uint4 ti = itab[2 * dp];
    const uint32_t ti2 = itab[2 * dp + 1].x;
    const uint32_t Pp = RL ? row_bcast(P, tp, d) : bperm(P, tp * 4 + d);
    const uint32_t Tp = RL ? row_bcast(Tr, tp, d) : bperm(Tr, tp * 4 + d);
    const uint32_t Pn = gmul4(ti, ti2, sel0(Pp), sel1(Pp), sel2(Pp));
    const uint32_t Tn = gmul4(ti, ti2, sel0(Tp), sel1(Tp), sel2(Tp));
    if (t == tp) {
      P = Pn;
      Tr = Tn;
      mycol = c;
    } else {
      P ^= gmul4(tf, tf2, sel0(Pn), sel1(Pn), sel2(Pn));
      Tr ^= gmul4(tf, tf2, sel0(Tn), sel1(Tn), sel2(Tn));
    }
    used |= 1u << tp;
  }
  s_out[mycol][d] = Tr;
  *s_val = Tr;
  *s_row = mycol;
  return true;
}

// out[t][d] = base ^ sum_c M[t][c] x X[c][d], one wave, lane (t, d): the M
// row (4 dwords, 16 bytes) and X rows (4 dwords) in LDS
__device__ __forceinline__ uint32_t mc2_small(const uint4* tab, uint32_t base, const uint32_t* mrow,
                                              const uint32_t (*x)[4], int d) {
  uint32_t acc = base;
  for (int cq = 0; cq < 4; cq++) {
    const uint32_t mw = mrow[cq];
#pragma unroll
    for (int cc = 0; cc < 4; cc++) {
      const uint32_t m = (mw >> (8 * cc)) & 0xffu;
      const uint4 t = tab[2 * m];
      const uint32_t t2 = tab[2 * m + 1].x;
      const uint32_t xv = x[4 * cq + cc][d];
      acc ^= gmul4(t, t2, sel0(xv), sel1(xv), sel2(xv));
    }
  }
  return acc;
}

// The owned block brought up to date with the previous panel in one pass, one
// wave, lane (t, d): F = M x S_{p-1} (M: the block rows' panel p - 1
// columns, `mrow` = row t's 4 dwords), then blk ^= F x R_{p-1}[:, panel p]
// (`rp` rows, dwords col0 .. col0 + 3).  Every operand load and both table
// gathers are issued before the arithmetic that waits on them; F's row goes
// to the quad by DPP, not through LDS.
__device__ __forceinline__ uint32_t mc3_block_update(const uint4* tab, uint32_t blk, const uint32_t* mrow,
                                                     const uint32_t (*sp)[4], const uint32_t (*rp)[64], int col0,
                                                     int lane) {
  const int d = lane & 3;
  uint32_t mw[4], sv[16], rv[16];
#pragma unroll
  for (int q = 0; q < 4; q++) mw[q] = mrow[q];
#pragma unroll
  for (int c = 0; c < 16; c++) {
    sv[c] = sp[c][d];
    rv[c] = rp[c][col0 + d];
  }
  uint32_t F = 0;
#pragma unroll
  for (int c = 0; c < 16; c++) {
    const uint32_t m = (mw[c >> 2] >> (8 * (c & 3))) & 0xffu;
    const uint4 tt = tab[2 * m];
    const uint32_t tt2 = tab[2 * m + 1].x;
    F ^= gmul4(tt, tt2, sel0(sv[c]), sel1(sv[c]), sel2(sv[c]));
  }
  uint32_t fw[4];
#pragma unroll
  for (int q = 0; q < 4; q++) fw[q] = quad_bcast(F, q);
  uint32_t acc = blk;
#pragma unroll
  for (int c = 0; c < 16; c++) {
    const uint32_t m = (fw[c >> 2] >> (8 * (c & 3))) & 0xffu;
    const uint4 tt = tab[2 * m];
    const uint32_t tt2 = tab[2 * m + 1].x;
    acc ^= gmul4(tt, tt2, sel0(rv[c]), sel1(rv[c]), sel2(rv[c]));
  }
  return acc;
}

// mc2_panel_gj with the block in registers (lane (t, d) = dword d of block
// row t, `P`) and the pivot's inverse tables gathered beside the row's own
// tables, before the pivot is known: lane (t, 0..3) loads the tables of f
// and inv(f) for its row's entry f in column c; the pivot lane's inverse
// tables then come by v_readlane.  One dependent LDS round trip per step
// (the gathers), no ds_bpermute.
__device__ __forceinline__ bool mc3_panel_gj(const uint4* tab, const uint4* itab, uint32_t P, int lane,
                                             uint32_t* s_val, int* s_row) {
  const int t = lane >> 2, d = lane & 3;
  uint32_t Tr = (t >> 2) == d ? 1u << (8 * (t & 3)) : 0u;
  uint32_t used = 0;
  int mycol = 0;
#pragma unroll
  for (int c = 0; c < 16; c++) {
    const uint32_t f = (quad_bcast(P, c >> 2) >> (8 * (c & 3))) & 0xffu;
    const uint4 tf = tab[2 * f];
    const uint32_t tf2 = tab[2 * f + 1].x;
    const uint4 ti = itab[2 * f];
    const uint32_t ti2 = itab[2 * f + 1].x;
    const bool nz = d == 0 && f != 0u && !((used >> t) & 1u);
    const uint64_t m = __builtin_amdgcn_ballot_w64(nz);
    if (m == 0) return false;
    const int pl = __builtin_ctzll(m), tp = pl >> 2;
    const uint32_t Pp = row_bcast(P, tp, d), Tp = row_bcast(Tr, tp, d);
    const uint4 si = make_uint4(__builtin_amdgcn_readlane(ti.x, pl), __builtin_amdgcn_readlane(ti.y, pl),
                                __builtin_amdgcn_readlane(ti.z, pl), __builtin_amdgcn_readlane(ti.w, pl));
    const uint32_t si2 = __builtin_amdgcn_readlane(ti2, pl);
    const uint32_t Pn = gmul4(si, si2, sel0(Pp), sel1(Pp), sel2(Pp));
    const uint32_t Tn = gmul4(si, si2, sel0(Tp), sel1(Tp), sel2(Tp));
    if (t == tp) {
      P = Pn;
      Tr = Tn;
      mycol = c;
    } else {
      P ^= gmul4(tf, tf2, sel0(Pn), sel1(Pn), sel2(Pn));
      Tr ^= gmul4(tf, tf2, sel0(Tn), sel1(Tn), sel2(Tn));
    }
    used |= 1u << tp;
  }
  *s_val = Tr;
  *s_row = mycol;
  return true;
}

// The block update's second product with the selectors of its data operand
// (R_{p-1}[:, panel p], known before S_{p-1}) computed ahead: r0/r1/r2[c] =
// sel0/1/2 of R[c][col0 + d]
__device__ __forceinline__ void mc3_pre_r(const uint32_t (*rp)[64], int col0, int lane, uint32_t* r0, uint32_t* r1,
                                          uint32_t* r2) {
  const int d = lane & 3;
#pragma unroll
  for (int c = 0; c < 16; c++) {
    const uint32_t x = rp[c][col0 + d];
    r0[c] = sel0(x);
    r1[c] = sel1(x);
    r2[c] = sel2(x);
  }
}
__device__ __forceinline__ uint32_t mc3_block_update_pre(const uint4* tab, uint32_t blk, const uint32_t* mrow,
                                                         const uint32_t (*sp)[4], const uint32_t* r0,
                                                         const uint32_t* r1, const uint32_t* r2, int lane) {
  const int d = lane & 3;
  uint32_t mw[4], sv[16];
#pragma unroll
  for (int q = 0; q < 4; q++) mw[q] = mrow[q];
#pragma unroll
  for (int c = 0; c < 16; c++) sv[c] = sp[c][d];
  uint32_t F = 0;
#pragma unroll
  for (int c = 0; c < 16; c++) {
    const uint32_t m = (mw[c >> 2] >> (8 * (c & 3))) & 0xffu;
    const uint4 tt = tab[2 * m];
    const uint32_t tt2 = tab[2 * m + 1].x;
    F ^= gmul4(tt, tt2, sel0(sv[c]), sel1(sv[c]), sel2(sv[c]));
  }
  uint32_t fw[4];
#pragma unroll
  for (int q = 0; q < 4; q++) fw[q] = quad_bcast(F, q);
  uint32_t acc = blk;
#pragma unroll
  for (int c = 0; c < 16; c++) {
    const uint32_t m = (fw[c >> 2] >> (8 * (c & 3))) & 0xffu;
    const uint4 tt = tab[2 * m];
    const uint32_t tt2 = tab[2 * m + 1].x;
    acc ^= gmul4(tt, tt2, r0[c], r1[c], r2[c]);
  }
  return acc;
}

// The 16 x 16 block inversion in circular form: one 16-byte row per block
// row (lane (t, d) = dword d), slot s holding the coefficient of column s
// until column s is eliminated and then T's column pi(s) (pi(s): the row that
// pivoted column s), as gf_elim_circ_kernel does for whole rows.  Step c:
// the pivot row (lowest unpicked row with slot c non-zero, entry dp) is
// normalized, Q = inv(dp) x row, whose slot c is then 1; a non-pivot row
// takes row ^= f x Q' with Q' = Q but slot c = 1 ^ inv(dp), so that its slot
// c becomes f x inv(dp) = T[t][pi(c)] (the pivot row's T column pi(c), its
// own identity, was 1); the pivot row becomes Q with slot c = inv(dp).  An
// unpicked row's own identity T[t][t] = 1 needs no slot: no pivot row has T
// column t.  At the end, S row c = the slots of row pi(c) with output byte j
// taken from slot pi^-1(j) (two v_perm per lane).  Half the row operations
// of the [block | T] form (mc2_panel_gj).
__device__ __forceinline__ bool mc3_gj_circ(const uint4* tab, const uint4* itab, uint32_t P, int lane,
                                            uint32_t* s_val, int* s_row) {
  const int t = lane >> 2, d = lane & 3;
  uint32_t used = 0, selA = 0, selB = 0, mskA = 0;
  int mycol = 0;
#pragma unroll
  for (int c = 0; c < 16; c++) {
    const int cd = c >> 2, cb = 8 * (c & 3);
    const uint32_t f = (quad_bcast(P, cd) >> cb) & 0xffu;
    const uint4 tf = tab[2 * f];
    const uint32_t tf2 = tab[2 * f + 1].x;
    const bool nz = d == 0 && f != 0u && !((used >> t) & 1u);
    const uint64_t m = __builtin_amdgcn_ballot_w64(nz);
    if (m == 0) return false;
    const int pl = __builtin_ctzll(m), tp = pl >> 2;
    const uint32_t dp = __builtin_amdgcn_readlane(f, pl);
    const uint4 ti = itab[2 * dp];
    const uint32_t ti2 = itab[2 * dp + 1].x;
    const uint32_t Pp = bperm(P, tp * 4 + d);
    const uint32_t inv = (ti.x >> 8) & 0xffu;  // T0 entry 1: inv(dp) x 1
    uint32_t Q = gmul4(ti, ti2, sel0(Pp), sel1(Pp), sel2(Pp));
    if (d == cd) Q ^= inv << cb;
    if (t == tp) {
      P = d == cd ? Q ^ (1u << cb) : Q;
      mycol = c;
    } else {
      P ^= gmul4(tf, tf2, sel0(Q), sel1(Q), sel2(Q));
    }
    used |= 1u << tp;
    if (d == (tp >> 2)) {  // output byte tp of every S row comes from slot c
      const int ob = 8 * (tp & 3);
      if (c < 8) {
        selA |= (uint32_t)c << ob;
        mskA |= 0xffu << ob;
      } else {
        selB |= (uint32_t)(c - 8) << ob;
      }
    }
  }
  const uint32_t w0 = quad_bcast(P, 0), w1 = quad_bcast(P, 1), w2 = quad_bcast(P, 2), w3 = quad_bcast(P, 3);
  *s_val = (__builtin_amdgcn_perm(w1, w0, selA) & mskA) | (__builtin_amdgcn_perm(w3, w2, selB) & ~mskA);
  *s_row = mycol;
  return true;
}

// The circular-form inversion with one block row per lane (lanes 0-15, row t
// = lane: slots in P[0..3]; lanes 16-63 carry zero rows that are never
// candidates) and no branches, so that the step's one LDS round trip -- the
// gather of the tables of f and of inv(f) for every row's entry f in column
// c -- is issued before anything waits on it:
//  * the candidates are a ballot of f != 0 under an SGPR mask of unpicked
//    rows; the pivot row's four dwords and, once the gather is back, the
//    tables of inv(dp) come by v_readlane from the pivot lane (uniform);
//  * Q = inv(dp) x pivot row with slot c = 1 ^ inv(dp); a row takes row ^=
//    f x Q, the pivot lane takes Q with slot c = inv(dp) (a select);
//  * pi^-1 is kept as sixteen 4-bit slot numbers in an SGPR pair; at the end
//    S row c = row pi(c)'s slots with output byte j from slot pi^-1(j)
//    (v_perm with uniform selectors).
// Returns false (S undefined) when a column has no candidate.  Lane t < 16
// ends holding S row *s_row in s[0..3].
__device__ __forceinline__ bool mc3_gj_rows(const uint4* tab, const uint4* itab, uint32_t* P, int lane, uint32_t* s,
                                            int* s_row) {
  uint64_t cand = 0xffffull;  // unpicked rows (lanes)
  uint64_t pinv = 0;          // slot of output byte j at bits 4j .. 4j + 3
  bool fail = false;
  int mycol = 0;
#pragma unroll
  for (int c = 0; c < 16; c++) {
    const int cq = c >> 2, cb = 8 * (c & 3);
    const uint32_t f = (P[cq] >> cb) & 0xffu;
    const uint4 tf = tab[2 * f];
    const uint32_t tf2 = tab[2 * f + 1].x;
    const uint4 ti = itab[2 * f];
    const uint32_t ti2 = itab[2 * f + 1].x;
    const uint64_t m = __builtin_amdgcn_ballot_w64(f != 0u) & cand;
    fail |= m == 0;
    const int pl = m ? __builtin_ctzll(m) : 0;
    cand &= ~(1ull << pl);
    pinv |= (uint64_t)c << (4 * pl);
    uint32_t pr[4];
#pragma unroll
    for (int q = 0; q < 4; q++) pr[q] = __builtin_amdgcn_readlane(P[q], pl);
    const uint4 si = make_uint4(__builtin_amdgcn_readlane(ti.x, pl), __builtin_amdgcn_readlane(ti.y, pl),
                                __builtin_amdgcn_readlane(ti.z, pl), __builtin_amdgcn_readlane(ti.w, pl));
    const uint32_t si2 = __builtin_amdgcn_readlane(ti2, pl);
    const uint32_t inv = (si.x >> 8) & 0xffu;
    const bool piv = lane == pl;
    mycol = piv ? c : mycol;
#pragma unroll
    for (int q = 0; q < 4; q++) {
      uint32_t Q = gmul4(si, si2, sel0(pr[q]), sel1(pr[q]), sel2(pr[q]));
      if (q == cq) Q ^= inv << cb;
      const uint32_t upd = P[q] ^ gmul4(tf, tf2, sel0(Q), sel1(Q), sel2(Q));
      P[q] = piv ? (q == cq ? Q ^ (1u << cb) : Q) : upd;
    }
  }
#pragma unroll
  for (int q = 0; q < 4; q++) {
    uint32_t sa = 0, sb = 0, ma = 0;
#pragma unroll
    for (int b = 0; b < 4; b++) {
      const uint32_t sl = (uint32_t)(pinv >> (4 * (4 * q + b))) & 15u;
      if (sl < 8) {
        sa |= sl << (8 * b);
        ma |= 0xffu << (8 * b);
      } else {
        sb |= (sl - 8) << (8 * b);
      }
    }
    s[q] = (__builtin_amdgcn_perm(P[1], P[0], sa) & ma) | (__builtin_amdgcn_perm(P[3], P[2], sb) & ~ma);
  }
  *s_row = mycol;
  return !fail;
}

// acc ^ sum over 8 terms of (tables of the multiplier bytes m[0..7]) x data
// with precomputed selectors: all 16 table reads are issued first (a
// scheduling barrier keeps the compiler from sinking each read next to its
// use, which serialises one LDS round trip per term)
__device__ __forceinline__ uint32_t mc3_dot8(const uint4* tab, uint32_t acc, const uint32_t* m, const uint32_t* s0,
                                             const uint32_t* s1, const uint32_t* s2) {
  uint4 tt[8];
  uint32_t t2[8];
#pragma unroll
  for (int c = 0; c < 8; c++) {
    tt[c] = tab[2 * m[c]];
    t2[c] = tab[2 * m[c] + 1].x;
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int c = 0; c < 8; c++) acc ^= gmul4(tt[c], t2[c], s0[c], s1[c], s2[c]);
  return acc;
}

// mc3_block_update_pre with the table reads batched (mc3_dot8): F = M x S,
// then blk ^= F x R[:, panel p] (R's selectors r0/r1/r2 computed ahead)
__device__ __forceinline__ uint32_t mc3_block_update_b(const uint4* tab, uint32_t blk, const uint32_t* mrow,
                                                       const uint32_t (*sp)[4], const uint32_t* r0,
                                                       const uint32_t* r1, const uint32_t* r2, int lane) {
  const int d = lane & 3;
  uint32_t mw[4], m[16], s0[16], s1[16], s2[16];
#pragma unroll
  for (int q = 0; q < 4; q++) mw[q] = mrow[q];
#pragma unroll
  for (int c = 0; c < 16; c++) {
    const uint32_t x = sp[c][d];
    m[c] = (mw[c >> 2] >> (8 * (c & 3))) & 0xffu;
    s0[c] = sel0(x);
    s1[c] = sel1(x);
    s2[c] = sel2(x);
  }
  uint32_t F = mc3_dot8(tab, 0u, m, s0, s1, s2);
  F = mc3_dot8(tab, F, m + 8, s0 + 8, s1 + 8, s2 + 8);
  uint32_t fw[4];
#pragma unroll
  for (int q = 0; q < 4; q++) fw[q] = quad_bcast(F, q);
#pragma unroll
  for (int c = 0; c < 16; c++) m[c] = (fw[c >> 2] >> (8 * (c & 3))) & 0xffu;
  uint32_t acc = mc3_dot8(tab, blk, m, r0, r1, r2);
  return mc3_dot8(tab, acc, m + 8, r0 + 8, r1 + 8, r2 + 8);
}



// ---- the library's inversion before round 6 (ballot on every step) ----
// The circular-form inversion ((t, d) layout as mc3_gj_circ), branch-free:
// the candidates are a ballot of f != 0 under an SGPR mask of the unpicked
// rows' lanes (t, 0); the row's own tables (of f) are read right after f,
// beside the pivot path (ballot -> s_ff1 -> v_readlane of dp -> uniform read
// of inv(dp)'s tables, and ds_bpermute of the pivot row); every row then
// computes both the pivot's and a non-pivot row's new value and selects.
__device__ __forceinline__ bool mc3_gj_v5(const uint4* tab, const uint4* itab, uint32_t P, int lane, uint32_t* s_val,
                                          int* s_row) {
  const int t = lane >> 2, d = lane & 3;
  uint64_t cand = 0x1111111111111111ull;
  uint64_t pinv = 0;  // nibble tp = the slot (column) row tp pivoted: SALU only
  bool fail = false;
#pragma unroll
  for (int c = 0; c < 16; c++) {
    const int cd = c >> 2, cb = 8 * (c & 3);
    const uint32_t f = (quad_bcast(P, cd) >> cb) & 0xffu;
    const uint4 tf = tab[2 * f];
    const uint32_t tf2 = tab[2 * f + 1].x;
    const uint64_t m = __builtin_amdgcn_ballot_w64(f != 0u) & cand;
    fail |= m == 0;
    const int pl = (int)__builtin_ctzll(m | (1ull << 60));  // a failed column picks lane 60 (result unused)
    const int tp = pl >> 2;
    cand &= ~(1ull << pl);
    pinv |= (uint64_t)c << (4 * tp);
    const uint32_t dp = __builtin_amdgcn_readlane(f, pl);
    const uint4 ti = itab[2 * dp];
    const uint32_t ti2 = itab[2 * dp + 1].x;
    const uint32_t Pp = bperm(P, pl + d);
    const uint32_t inv = (ti.x >> 8) & 0xffu;
    const uint32_t Q = gmul4(ti, ti2, sel0(Pp), sel1(Pp), sel2(Pp)) ^ (d == cd ? inv << cb : 0u);
    const uint32_t upd = P ^ gmul4(tf, tf2, sel0(Q), sel1(Q), sel2(Q));
    P = t == tp ? Q ^ (d == cd ? 1u << cb : 0u) : upd;
  }
  // S row c = the slots of row pi(c) with output byte j from slot pi^-1(j) =
  // nibble j of pinv; row t pivoted column nibble t
  uint32_t selA = 0, selB = 0, mskA = 0;
  const uint32_t pq = (uint32_t)(pinv >> (16 * d));  // nibbles 4d .. 4d + 3: this lane's output bytes
#pragma unroll
  for (int b = 0; b < 4; b++) {
    const uint32_t sl = (pq >> (4 * b)) & 15u;
    selA |= (sl & 7u) << (8 * b);
    selB |= (sl & 7u) << (8 * b);
    mskA |= sl < 8 ? 0xffu << (8 * b) : 0u;
  }
  const uint32_t w0 = quad_bcast(P, 0), w1 = quad_bcast(P, 1), w2 = quad_bcast(P, 2), w3 = quad_bcast(P, 3);
  *s_val = (__builtin_amdgcn_perm(w1, w0, selA) & mskA) | (__builtin_amdgcn_perm(w3, w2, selB) & ~mskA);
  *s_row = (int)((pinv >> (4 * t)) & 15u);
  return !fail;
}

// ---- division-free, guessed pivot (round 6: slower, more VALU per step) ----
// The same inversion (same pivots, same S), division-free, with the pivot
// row guessed before its column is known.  mc3_gj_v5's step waits on a
// chain of ballot -> s_ff1 -> v_readlane -> inverse tables -> Q -> Q's
// selectors -> the row update; here:
//  * the pivot is the lowest unpicked row when its entry a in column c is
//    non-zero (255 in 256; otherwise the ballot picks, as in v5, so the pivots
//    are v5's), its lane known from the SGPR candidate mask before the step:
//    a = one v_readlane of the previous step's P;
//  * no row is normalized: a non-pivot row becomes a x row ^ f x pivot row,
//    the pivot row stays, so the update needs a's tables (one uniform LDS
//    read) and the row's own tables of f (gathered beside it), and its
//    selectors are ready before a is;
//  * slot c (T's column pi(c) from now on) takes f x s on a non-pivot row and
//    s on the pivot row, s = the product of the pivots so far (the implicit
//    T[t][t] of every unpicked row, which every step scaled by its pivot);
//  * a row's scale dsc = its own pivot times every later one; at the end one
//    gather of inv(dsc)'s tables normalizes it: the slots equal v5's.
__device__ __forceinline__ bool mc3_gj_v6(const uint4* tab, const uint4* itab, uint32_t P, int lane, uint32_t* s_val,
                                          int* s_row) {
  const int t = lane >> 2, d = lane & 3;
  uint64_t cand = 0x1111111111111111ull;
  uint64_t pinv = 0;
  bool fail = false;
  uint32_t s = 1u, dsc = 1u;  // bytes
#pragma unroll
  for (int c = 0; c < 16; c++) {
    const int cd = c >> 2, cb = 8 * (c & 3);
    const uint32_t s0 = sel0(P), s1 = sel1(P), s2 = sel2(P);
    const uint32_t f = (quad_bcast(P, cd) >> cb) & 0xffu;
    const uint4 tf = tab[2 * f];
    const uint32_t tf2 = tab[2 * f + 1].x;
    int pl = (int)__builtin_ctzll(cand);
    uint32_t a = (__builtin_amdgcn_readlane(P, pl + cd) >> cb) & 0xffu;
    if (a == 0u) {  // the lowest unpicked row has a zero: v5's rule
      const uint64_t m = __builtin_amdgcn_ballot_w64(f != 0u) & cand;
      fail |= m == 0;
      pl = (int)__builtin_ctzll(m | (1ull << 60));  // a failed column picks lane 60 (result unused)
      a = __builtin_amdgcn_readlane(f, pl);
    }
    const int tp = pl >> 2;
    cand &= ~(1ull << pl);
    pinv |= (uint64_t)c << (4 * tp);
    const uint4 ta = tab[2 * a];
    const uint32_t ta2 = tab[2 * a + 1].x;
    const uint32_t Pp = bperm(P, pl + d);
    const uint32_t X = d == cd ? Pp ^ (s << cb) : Pp;  // slot c: a ^ s, so that a x f ^ f x (a ^ s) = f x s
    uint32_t upd = gmul4(ta, ta2, s0, s1, s2) ^ gmul4(tf, tf2, sel0(X), sel1(X), sel2(X));
    uint32_t dup = gmul4(ta, ta2, sel0(dsc), sel1(dsc), sel2(dsc));
    // (computed on every lane: left to itself the compiler sinks them into
    // exec-masked branches around the selects, which serialize the step)
    asm volatile("" : "+v"(upd), "+v"(dup));
    const bool piv = t == tp;
    P = piv ? (d == cd ? P ^ ((a ^ s) << cb) : P) : upd;
    dsc = piv ? a : dup;
    s = gmul4(ta, ta2, sel0(s), sel1(s), sel2(s));
  }
  {
    const uint4 ti = itab[2 * dsc];
    const uint32_t ti2 = itab[2 * dsc + 1].x;
    P = gmul4(ti, ti2, sel0(P), sel1(P), sel2(P));
  }
  uint32_t selA = 0, selB = 0, mskA = 0;
  const uint32_t pq = (uint32_t)(pinv >> (16 * d));
#pragma unroll
  for (int b = 0; b < 4; b++) {
    const uint32_t sl = (pq >> (4 * b)) & 15u;
    selA |= (sl & 7u) << (8 * b);
    selB |= (sl & 7u) << (8 * b);
    mskA |= sl < 8 ? 0xffu << (8 * b) : 0u;
  }
  const uint32_t w0 = quad_bcast(P, 0), w1 = quad_bcast(P, 1), w2 = quad_bcast(P, 2), w3 = quad_bcast(P, 3);
  *s_val = (__builtin_amdgcn_perm(w1, w0, selA) & mskA) | (__builtin_amdgcn_perm(w3, w2, selB) & ~mskA);
  *s_row = (int)((pinv >> (4 * t)) & 15u);
  return !fail;
}

// mc3_gj_v6 with the guessed pivot's loads (a's tables, the pivot row) issued
// before the zero check (the rare fallback reloads them); RB: the pivot row
// by four v_readlane and a select instead of ds_bpermute
template <bool RB>
__device__ __forceinline__ bool mc3_gj_v7(const uint4* tab, const uint4* itab, uint32_t P, int lane, uint32_t* s_val,
                                          int* s_row) {
  const int t = lane >> 2, d = lane & 3;
  uint64_t cand = 0x1111111111111111ull;
  uint64_t pinv = 0;
  bool fail = false;
  uint32_t s = 1u, dsc = 1u;
#pragma unroll
  for (int c = 0; c < 16; c++) {
    const int cd = c >> 2, cb = 8 * (c & 3);
    const uint32_t s0 = sel0(P), s1 = sel1(P), s2 = sel2(P);
    const uint32_t f = (quad_bcast(P, cd) >> cb) & 0xffu;
    const uint4 tf = tab[2 * f];
    const uint32_t tf2 = tab[2 * f + 1].x;
    int pl = (int)__builtin_ctzll(cand);
    uint32_t a = (__builtin_amdgcn_readlane(P, pl + cd) >> cb) & 0xffu;
    uint4 ta = tab[2 * a];
    uint32_t ta2 = tab[2 * a + 1].x;
    uint32_t Pp = RB ? row_bcast(P, pl >> 2, d) : bperm(P, pl + d);
    if (__builtin_expect(a == 0u, 0)) {
      const uint64_t m = __builtin_amdgcn_ballot_w64(f != 0u) & cand;
      fail |= m == 0;
      pl = (int)__builtin_ctzll(m | (1ull << 60));
      a = __builtin_amdgcn_readlane(f, pl);
      ta = tab[2 * a];
      ta2 = tab[2 * a + 1].x;
      Pp = RB ? row_bcast(P, pl >> 2, d) : bperm(P, pl + d);
    }
    const int tp = pl >> 2;
    cand &= ~(1ull << pl);
    pinv |= (uint64_t)c << (4 * tp);
    const uint32_t X = d == cd ? Pp ^ (s << cb) : Pp;
    uint32_t upd = gmul4(ta, ta2, s0, s1, s2) ^ gmul4(tf, tf2, sel0(X), sel1(X), sel2(X));
    uint32_t dup = gmul4(ta, ta2, sel0(dsc), sel1(dsc), sel2(dsc));
    asm volatile("" : "+v"(upd), "+v"(dup));
    const bool piv = t == tp;
    P = piv ? (d == cd ? P ^ ((a ^ s) << cb) : P) : upd;
    dsc = piv ? a : dup;
    s = gmul4(ta, ta2, sel0(s), sel1(s), sel2(s));
  }
  {
    const uint4 ti = itab[2 * dsc];
    const uint32_t ti2 = itab[2 * dsc + 1].x;
    P = gmul4(ti, ti2, sel0(P), sel1(P), sel2(P));
  }
  uint32_t selA = 0, selB = 0, mskA = 0;
  const uint32_t pq = (uint32_t)(pinv >> (16 * d));
#pragma unroll
  for (int b = 0; b < 4; b++) {
    const uint32_t sl = (pq >> (4 * b)) & 15u;
    selA |= (sl & 7u) << (8 * b);
    selB |= (sl & 7u) << (8 * b);
    mskA |= sl < 8 ? 0xffu << (8 * b) : 0u;
  }
  const uint32_t w0 = quad_bcast(P, 0), w1 = quad_bcast(P, 1), w2 = quad_bcast(P, 2), w3 = quad_bcast(P, 3);
  *s_val = (__builtin_amdgcn_perm(w1, w0, selA) & mskA) | (__builtin_amdgcn_perm(w3, w2, selB) & ~mskA);
  *s_row = (int)((pinv >> (4 * t)) & 15u);
  return !fail;
}

struct ProbeIn {  // one iteration's data (dwords)
  uint32_t mb[16][8];  // block rows: panel p - 1 columns (0-3), panel p columns (4-7)
  uint32_t sp[16][4];  // S_{p-1}
  uint32_t rp[16][64]; // R_{p-1} (p = 1: its panel p columns are dwords 4-7)
};

template <int SMV, int GJV>
__global__ __launch_bounds__(1024) void chain_probe(const uint32_t* tables, const ProbeIn* in, int iters, int mode,
                                                    unsigned long long* stats, uint32_t* s_out) {
  __shared__ ProbeLds lds;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int i = tid; i < 256 * 2; i += 1024) {
    const uint32_t* a = tables + 4 * i;
    const uint32_t* b = tables + kElimInvTables + 4 * i;
    lds.tab[i] = make_uint4(a[0], a[1], a[2], a[3]);
    lds.itab[i] = make_uint4(b[0], b[1], b[2], b[3]);
  }
  if (tid == 0) lds.fail = 0;
  if (tid == 0) lds.chain_cnt = 0;
  __syncthreads();
  if (w != 8) {
    if (mode == 0) return;
    if (mode == 2 && w < 8) {
      uint32_t R[4] = {(uint32_t)lane, (uint32_t)lane * 3u, (uint32_t)lane * 5u, (uint32_t)lane * 7u};
      uint32_t g = 0x01020304u * (uint32_t)(w + 1);
      while (__hip_atomic_load(&lds.chain_cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) {
#pragma unroll
        for (int cc = 0; cc < 16; cc++) {
          const uint32_t x = lds.rp[cc % 3][cc][lane];
          const uint32_t s0 = sel0(x), s1 = sel1(x), s2 = sel2(x);
#pragma unroll
          for (int i = 0; i < 4; i++) {
            const uint32_t f = __builtin_amdgcn_readfirstlane((g >> (8 * i)) & 0xffu);
            const uint4 t = lds.tab[2 * f];
            const uint32_t t2 = lds.tab[2 * f + 1].x;
            R[i] ^= mc_mul(t, t2, s0, s1, s2);
          }
          g = g * 1664525u + 1013904223u;
        }
      }
      if (R[0] == 0x12345678u && R[1] == R[2]) lds.fail = 7;  // keep the work
      return;
    }
    for (int spins = 0; spins < (1 << 22); spins++) {
      if (__hip_atomic_load(&lds.chain_cnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
      __builtin_amdgcn_s_sleep(1);
    }
    return;
  }
  __builtin_amdgcn_s_setprio(3);
  const int t = lane >> 2, d = lane & 3;
  unsigned long long c_small = 0, c_gj = 0;
  int fails = 0;
  const unsigned long long r0 = __builtin_amdgcn_s_memrealtime(), m0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; it++) {
    const ProbeIn& x = in[it];
    // stage: slot 1 = this block's mb, slot 0 = the previous panel's S / R
    for (int i = lane; i < 16 * 8; i += 64) lds.mb[1][i >> 3][i & 7] = x.mb[i >> 3][i & 7];
    lds.sp[0][lane >> 2][lane & 3] = x.sp[lane >> 2][lane & 3];
    for (int r = 0; r < 16; r++) lds.rp[0][r][lane] = x.rp[r][lane];
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    const int p = 1, slot = 1, ps = 0;
    uint32_t r0[16], r1[16], r2[16];  // SMV 2: R's selectors before S_{p-1} is there
    if (SMV == 2 || SMV == 3) mc3_pre_r(lds.rp[ps], 4 * p, lane, r0, r1, r2);
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long a0 = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_sched_barrier(0);
    uint32_t blk = lds.mb[slot][t][4 + d];
    if (SMV == 0) {  // as gf_elim_mc2_kernel (not split)
      lds.ft[t][d] = mc2_small(lds.tab, 0u, lds.mb[slot][t], lds.sp[ps], d);
      __builtin_amdgcn_s_waitcnt(0xc07f);
      uint32_t acc = blk;
      for (int cq = 0; cq < 4; cq++) {
        const uint32_t fw = lds.ft[t][cq];
#pragma unroll
        for (int cc = 0; cc < 4; cc++) {
          const uint32_t m = (fw >> (8 * cc)) & 0xffu;
          const uint4 tt = lds.tab[2 * m];
          const uint32_t tt2 = lds.tab[2 * m + 1].x;
          const uint32_t xv = lds.rp[ps][4 * cq + cc][4 * p + d];
          acc ^= gmul4(tt, tt2, sel0(xv), sel1(xv), sel2(xv));
        }
      }
      blk = acc;
    } else if (SMV == 1) {
      blk = mc3_block_update(lds.tab, blk, lds.mb[slot][t], lds.sp[ps], lds.rp[ps], 4 * p, lane);
    } else if (SMV == 2) {
      blk = mc3_block_update_pre(lds.tab, blk, lds.mb[slot][t], lds.sp[ps], r0, r1, r2, lane);
    } else if (SMV == 3) {
      blk = mc3_block_update_b(lds.tab, blk, lds.mb[slot][t], lds.sp[ps], r0, r1, r2, lane);
    } else {
      blk = mc3_block_update_c(lds.tab, blk, lds.mb[slot][t], lds.sp[ps], lds.rp[ps], 4 * p, lane);
    }
    lds.pan[t][d] = blk;
    __builtin_amdgcn_s_waitcnt(0xc07f);
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long a1 = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_sched_barrier(0);
    uint32_t sval = 0;
    int srow = 0;
    bool ok;
    if (GJV == 0)
      ok = mc2_panel_gj<false>(lds.tab, lds.itab, lds.pan, lds.sp[2], lane, &sval, &srow);
    else if (GJV == 1)
      ok = mc2_panel_gj<true>(lds.tab, lds.itab, lds.pan, lds.sp[2], lane, &sval, &srow);
    else if (GJV == 2)
      ok = mc3_panel_gj(lds.tab, lds.itab, blk, lane, &sval, &srow);
    else if (GJV == 3)
      ok = mc3_gj_circ(lds.tab, lds.itab, blk, lane, &sval, &srow);
    if (GJV == 5) ok = mc3_gj_v5(lds.tab, lds.itab, blk, lane, &sval, &srow);
    if (GJV == 6) ok = mc3_gj_v6(lds.tab, lds.itab, blk, lane, &sval, &srow);
    if (GJV == 7) ok = mc3_gj_v7<false>(lds.tab, lds.itab, blk, lane, &sval, &srow);
    if (GJV == 8) ok = mc3_gj_v7<true>(lds.tab, lds.itab, blk, lane, &sval, &srow);
    if (GJV == 9) ok = mc3_gj(lds.tab, lds.itab, blk, lane, &sval, &srow);
    uint32_t Pr[4], Sr[4];
    if (GJV == 4) {  // (t, d) layout -> one row per lane, then the row-form inversion
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint32_t v = bperm(blk, 4 * (lane & 15) + q);  // all lanes active: a disabled source reads 0
        Pr[q] = lane < 16 ? v : 0u;
      }
      ok = mc3_gj_rows(lds.tab, lds.itab, Pr, lane, Sr, &srow);
    }
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_sched_barrier(0);
    const unsigned long long a2 = __builtin_amdgcn_s_memtime();
    __builtin_amdgcn_sched_barrier(0);
    c_small += a1 - a0;
    c_gj += a2 - a1;
    if (!ok) fails++;
    // S by rows into s_out: lane (t, d) holds S row srow, dword d
    if (GJV == 4) {
      if (lane < 16)
        for (int q = 0; q < 4; q++) s_out[(size_t)it * 64 + srow * 4 + q] = ok ? Sr[q] : 0u;
    } else {
      s_out[(size_t)it * 64 + srow * 4 + d] = ok ? sval : 0u;
    }
    s_out[(size_t)iters * 64 + (size_t)it * 64 + lane] = blk;  // the block it inverted (host check)
  }
  const unsigned long long r1 = __builtin_amdgcn_s_memrealtime(), m1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) {
    __hip_atomic_store(&lds.chain_cnt, 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    stats[0] = c_small;
    stats[1] = c_gj;
    stats[2] = r1 - r0;
    stats[3] = m1 - m0;
    stats[4] = (unsigned long long)fails;
  }
}

}  // namespace
}  // namespace kodr_amd

using namespace kodr_amd;

static unsigned gmul(unsigned a, unsigned b) {
  unsigned r = 0;
  while (b) {
    if (b & 1) r ^= a;
    a <<= 1;
    if (a & 0x100) a ^= 0x11D;
    b >>= 1;
  }
  return r;
}
static unsigned ginv(unsigned a) {
  for (unsigned b = 1; b < 256; b++)
    if (gmul(a, b) == 1) return b;
  return 0;
}
static uint8_t byte_of(const uint32_t* row, int c) { return (uint8_t)(row[c >> 2] >> (8 * (c & 3))); }

// block_p as of p - 1 on the host: blk ^ (M x S) x R[:, panel p]
static void host_block(const ProbeIn& x, uint8_t out[16][16]) {
  for (int t = 0; t < 16; t++) {
    uint8_t F[16] = {};
    for (int u = 0; u < 16; u++) {
      unsigned a = 0;
      for (int c = 0; c < 16; c++) a ^= gmul(byte_of(x.mb[t], c), byte_of(x.sp[c], u));
      F[u] = (uint8_t)a;
    }
    for (int v = 0; v < 16; v++) {
      unsigned a = byte_of(x.mb[t], 16 + v);
      for (int c = 0; c < 16; c++) a ^= gmul(F[c], byte_of(x.rp[c], 16 + v));
      out[t][v] = (uint8_t)a;
    }
  }
}
static bool host_inv(const uint8_t in[16][16], uint8_t S[16][16]) {
  uint8_t A[16][32];
  for (int i = 0; i < 16; i++)
    for (int j = 0; j < 32; j++) A[i][j] = j < 16 ? in[i][j] : (j - 16 == i);
  for (int c = 0; c < 16; c++) {
    int p = -1;
    for (int r = c; r < 16; r++)
      if (A[r][c]) { p = r; break; }
    if (p < 0) return false;
    for (int j = 0; j < 32; j++) std::swap(A[p][j], A[c][j]);
    const unsigned iv = ginv(A[c][c]);
    for (int j = 0; j < 32; j++) A[c][j] = (uint8_t)gmul(A[c][j], iv);
    for (int r = 0; r < 16; r++)
      if (r != c && A[r][c]) {
        const unsigned f = A[r][c];
        for (int j = 0; j < 32; j++) A[r][j] ^= (uint8_t)gmul(f, A[c][j]);
      }
  }
  for (int i = 0; i < 16; i++)
    for (int j = 0; j < 16; j++) S[i][j] = A[i][16 + j];
  return true;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

template <int SMV, int GJV>
static int run(const char* name, const uint32_t* dtab, const ProbeIn* din, const std::vector<ProbeIn>& hin, int iters,
               int mode, unsigned long long* dstats, uint32_t* dS) {
  hipLaunchKernelGGL((chain_probe<SMV, GJV>), dim3(1), dim3(1024), 0, 0, dtab, din, iters, mode, dstats, dS);
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL((chain_probe<SMV, GJV>), dim3(1), dim3(1024), 0, 0, dtab, din, iters, mode, dstats, dS);
  CK(hipDeviceSynchronize());
  unsigned long long st[5];
  CK(hipMemcpy(st, dstats, sizeof st, hipMemcpyDeviceToHost));
  std::vector<uint32_t> S((size_t)iters * 128);
  CK(hipMemcpy(S.data(), dS, S.size() * 4, hipMemcpyDeviceToHost));
  int bad = 0, sing = 0;
  for (int it = 0; it < iters; it++) {
    uint8_t blk[16][16], Sh[16][16];
    host_block(hin[it], blk);
    bool blk_ok = true;
    for (int t = 0; t < 16; t++)
      for (int v = 0; v < 16; v++) blk_ok &= byte_of(&S[(size_t)iters * 64 + (size_t)it * 64 + 4 * t], v) == blk[t][v];
    if (!blk_ok) { bad++; continue; }
    if (!host_inv(blk, Sh)) { sing++; continue; }
    for (int t = 0; t < 16; t++)
      for (int v = 0; v < 16; v++)
        if (byte_of(&S[(size_t)it * 64 + 4 * t], v) != Sh[t][v]) { bad++; t = 16; break; }
  }
  const double clk = (double)st[3] / ((double)st[2] / 100.0);  // MHz
  printf("%-22s mode %d: small %7.0f cyc, gj %7.0f cyc per panel (%.2f + %.2f us at %.0f MHz), fails %llu, "
         "singular %d, wrong %d\n",
         name, mode, (double)st[0] / iters, (double)st[1] / iters, st[0] / (double)iters / clk,
         st[1] / (double)iters / clk, clk, st[4], sing, bad);
  return 0;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 512;
  std::vector<uint32_t> tabs(kElimInvTables + 256 * 8);
  elim_tables(tabs.data());
  std::vector<ProbeIn> hin(iters);
  uint64_t s = 0x6b6f6472ull;
  auto rnd = [&] { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return (uint32_t)s; };
  for (auto& x : hin) {
    for (auto& r : x.mb) for (auto& v : r) v = rnd();
    for (auto& r : x.sp) for (auto& v : r) v = rnd();
    for (auto& r : x.rp) for (auto& v : r) v = rnd();
  }
  uint32_t* dtab;
  ProbeIn* din;
  unsigned long long* dstats;
  uint32_t* dS;
  CK(hipMalloc(&dtab, tabs.size() * 4));
  CK(hipMalloc(&din, hin.size() * sizeof(ProbeIn)));
  CK(hipMalloc(&dstats, 64));
  CK(hipMalloc(&dS, (size_t)iters * 128 * 4));
  CK(hipMemcpy(dtab, tabs.data(), tabs.size() * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(din, hin.data(), hin.size() * sizeof(ProbeIn), hipMemcpyHostToDevice));
  for (int mode = 0; mode < 3; mode += 2) {
    run<0, 0>("mc2 small / gj", dtab, din, hin, iters, mode, dstats, dS);
    run<2, 3>("pre-R update / circ gj", dtab, din, hin, iters, mode, dstats, dS);
    run<3, 5>("batched update / gj v5", dtab, din, hin, iters, mode, dstats, dS);
    run<4, 5>("batched-c update / gj v5", dtab, din, hin, iters, mode, dstats, dS);
    run<4, 6>("batched-c update / gj v6", dtab, din, hin, iters, mode, dstats, dS);
    run<4, 7>("batched-c update / gj v7", dtab, din, hin, iters, mode, dstats, dS);
    run<4, 8>("batched-c update / gj v7 rb", dtab, din, hin, iters, mode, dstats, dS);
    run<4, 9>("batched-c update / gj (lib)", dtab, din, hin, iters, mode, dstats, dS);
  }
  return 0;
}
