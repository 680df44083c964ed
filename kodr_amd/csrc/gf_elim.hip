// gf_elim.hip -- kodr's decoder elimination on the GPU, one workgroup per
// generation (decoder), for batched AddPiece on fresh decoders.
//
// What kodr computes, and what the kernel may therefore compute instead.
// kodr's DecoderState (decoder_state.go:15-182) pivots on the diagonal only;
// its state keeps a zero strict lower triangle (decoder_core.cpp) and drops a
// row only when it becomes zero, which a linearly independent row never does.
// Two cases have a state that does not depend on the route:
//  * FULL: a batch of n >= k rows whose first k coding vectors C are linearly
//    independent.  kodr accepts all k (none can vanish, and rank counts kept
//    rows, so it reaches k exactly at row k - 1) and then holds an upper
//    triangular, invertible -- so diagonal -- coefficient half, which its
//    backward pass normalizes: the state is [I | C^-1], T's columns in arrival
//    order.  The kernel inverts C by Gauss-Jordan with a pivot search (the
//    lowest unused row with a non-zero entry in the column, so the clean case
//    pivots on the diagonal as kodr does); a column with no candidate means C
//    is singular and the whole batch goes back to the host (c = 0).
//  * CLEAN: fewer than k rows, all landing on their diagonals (after reduction
//    against the earlier pivots, row r has a non-zero entry in column r).
//    Then the state after c rows is the reduced row echelon form of
//    [C_c | I_c] (decoder_core.cpp add_panel), unique.  The kernel pivots on
//    the diagonal only and stops at the first zero: c = r.
// The host loads the state into DecoderCore and runs kodr's literal
// algorithm on whatever is left (decoder_core.cpp), so its quirks (zero
// diagonals with rank over-count, dependent rows) never need the GPU.  c < 2
// is reported as 0: kodr keeps the first piece unreduced until a second one
// arrives (full/decoder.go:58-61).
//
// Layout.  Row j (bytes [0, k) coefficients, [k, k + n) the transform T) lives
// in registers: wave w owns rows 16w .. 16w+15, lane l owns dwords l and
// l + 64 of each (DPL = 1 dword per lane for k <= 128, 2 for k <= 256).
//
// Multiply.  x -> f*x is GF(2)-linear, so f*x = T0[x & 7] ^ T1[(x >> 3) & 7] ^
// T2[x >> 6] with 8-, 8- and 4-entry byte tables of f (gf256.go:15-44, poly
// 0x11D), one v_perm_b32 each for 4 bytes.  The pivot row's selectors are
// computed once per step and shared by the rows each wave updates; a row's
// tables come from a table of all 256 multipliers through the scalar cache
// (the multiplier is wave-uniform).  The multiplier of row j at
// step r is byte r of row j, read wavefront-wide with v_readlane (its owner
// lane is r / 4); the pivot search takes the LDS atomic minimum of the
// waves' candidates.
//
// Sync.  Two workgroup barriers per step: after the candidates, and after the
// owner wave of the pivot has normalized it (multiplier inv(d), gf256.go:77-86)
// and published it in LDS (two buffers, alternating).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>

#include "gf_kernels.hpp"
#include "tune.hpp"

namespace kodr_amd {

namespace {

constexpr int kElimWaves = 16;
constexpr int kElimRowsPerWave = 16;   // 16 x 16 = 256 rows
constexpr int kNone = 0x7fffffff;
constexpr int kElimBlockedMinK = 32;  // below: the per-step kernel (one panel would be most of it)

// LDS: two pivot buffers [2][128] dwords, the pivot choice (three rotating
// slots, LDS atomic min of the waves' candidates), the pivot column of every
// row, the stop word.  The field tables ([256][8]
// dwords: T0 lo/hi, T1 lo/hi, T2, pad; then the 256 inverse bytes) are read
// with scalar loads: every index is wave-uniform.
struct ElimLds {
  uint32_t piv[2][128];
  int best[3];               // pivot of step r: min over the waves' candidates, slot r % 3
  int colof[256];
  int stop;
};

__device__ __forceinline__ uint32_t gmul4(const uint4& t01, uint32_t t2, uint32_t s0, uint32_t s1, uint32_t s2) {
  return __builtin_amdgcn_perm(t01.y, t01.x, s0) ^ __builtin_amdgcn_perm(t01.w, t01.z, s1) ^
         __builtin_amdgcn_perm(t2, t2, s2);
}

template <int DPL>
__global__ __launch_bounds__(64 * kElimWaves) void gf_elim_kernel(ElimArgs args) {
  __shared__ ElimLds lds;
  const int g = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave index: uniform, keep it scalar
  const int k = args.k;
  const bool full = args.n[g] >= k;
  const int n = min(args.n[g], k);
  const int j0 = w * kElimRowsPerWave;  // this wave's first row
  const uint8_t* vec = args.vecs[g];
  const size_t vp = args.vpitch;
  // [256][8] tables, then 64 dwords of inverses; constant address space, so
  // the wave-uniform reads become scalar loads through the scalar cache
  typedef const __attribute__((address_space(4))) uint32_t cu32;
  cu32* tb = (cu32*)args.tables;

  for (int i = tid; i < 256; i += 64 * kElimWaves) lds.colof[i] = -1;
  if (tid < 3) lds.best[tid] = kNone;
  if (tid == 0) lds.stop = -1;

  // rows in registers: S[i][h] = dword (h * 64 + lane) of row j0 + i
  uint32_t S[kElimRowsPerWave][DPL];
#pragma unroll
  for (int i = 0; i < kElimRowsPerWave; i++) {
    const int j = j0 + i;
#pragma unroll
    for (int h = 0; h < DPL; h++) {
      uint32_t v = 0;
      if (j < n) {
#pragma unroll
        for (int b = 0; b < 4; b++) {
          const int col = (h * 64 + lane) * 4 + b;
          uint32_t byte = 0;
          if (col < k) byte = vec[(size_t)j * vp + col];
          else if (col == k + j) byte = 1;  // T row = e_j
          v |= byte << (8 * b);
        }
      }
      S[i][h] = v;
    }
  }
  uint32_t used = 0;  // this wave's rows already chosen as pivots (bit i)
  const uint32_t live = j0 >= n ? 0u : (n - j0 >= 32 ? 0xffffffffu : (1u << (n - j0)) - 1u) & 0xffffu;
  __syncthreads();

#ifdef KODR_ELIM_TIMING
  uint64_t ts[8];  // s_memtime of step 10's phases (wave 0), written to out (tuning only)
#endif
  for (int r = 0; r < n; r++) {
#ifdef KODR_ELIM_TIMING
    if (r == 10) ts[0] = __builtin_amdgcn_s_memtime();
#endif
    const int rl = r >> 2, rb = 8 * (r & 3);  // column r: lane r / 4 of dword 0, byte r % 4
    // rows of this wave with a non-zero entry in column r (wavefront-wide
    // v_readlane of the owner lane); candidate: FULL, the lowest unused one;
    // CLEAN, row r itself
    uint32_t nz = 0;
#pragma unroll
    for (int i = 0; i < kElimRowsPerWave; i++)
      nz |= (((__builtin_amdgcn_readlane(S[i][0], rl) >> rb) & 0xffu) != 0u ? 1u : 0u) << i;
    nz &= live;
    uint32_t cm = full ? (nz & ~used) : ((r >= j0 && r < j0 + kElimRowsPerWave) ? nz & (1u << (r - j0)) : 0u);
    cm = __builtin_amdgcn_readfirstlane(cm);
    if (lane == 0 && cm) atomicMin(&lds.best[r % 3], j0 + __builtin_ctz(cm));
    if (tid == 0) lds.best[(r + 1) % 3] = kNone;  // read two steps ago, next written next step
#ifdef KODR_ELIM_TIMING
    if (r == 10) ts[1] = __builtin_amdgcn_s_memtime();
#endif
    __syncthreads();
#ifdef KODR_ELIM_TIMING
    if (r == 10) ts[2] = __builtin_amdgcn_s_memtime();
#endif
    const int p = __builtin_amdgcn_readfirstlane(lds.best[r % 3]);
    if (p == kNone) {  // FULL: C singular; CLEAN: a zero diagonal (uniform)
      if (tid == 0) lds.stop = r;
      break;
    }
    if (p >= j0 && p < j0 + kElimRowsPerWave) {  // the owner: normalize row p, publish it
      const int io = p - j0;
#pragma unroll
      for (int i = 0; i < kElimRowsPerWave; i++)
        if (i == io) {
          const uint32_t d = (__builtin_amdgcn_readlane(S[i][0], rl) >> rb) & 0xffu;
          const uint32_t inv = (tb[256 * 8 + (d >> 2)] >> (8 * (d & 3))) & 0xffu;  // gf256.go:77-86
          const uint4 t01 = {tb[inv * 8], tb[inv * 8 + 1], tb[inv * 8 + 2], tb[inv * 8 + 3]};
          const uint32_t t2 = tb[inv * 8 + 4];
#pragma unroll
          for (int h = 0; h < DPL; h++) {
            const uint32_t x = S[i][h];
            S[i][h] = gmul4(t01, t2, x & 0x07070707u, (x >> 3) & 0x07070707u, (x >> 6) & 0x03030303u);
            lds.piv[r & 1][h * 64 + lane] = S[i][h];
          }
        }
      used |= 1u << io;
      if (lane == 0) lds.colof[p] = r;
    }
#ifdef KODR_ELIM_TIMING
    if (r == 10) ts[3] = __builtin_amdgcn_s_memtime();
#endif
    __syncthreads();
#ifdef KODR_ELIM_TIMING
    if (r == 10) ts[4] = __builtin_amdgcn_s_memtime();
#endif
    uint32_t s0[DPL], s1[DPL], s2[DPL];
#pragma unroll
    for (int h = 0; h < DPL; h++) {
      const uint32_t x = lds.piv[r & 1][h * 64 + lane];
      s0[h] = x & 0x07070707u;
      s1[h] = (x >> 3) & 0x07070707u;
      s2[h] = (x >> 6) & 0x03030303u;
    }
    // eliminate column r from every other row with a non-zero entry there
    const uint32_t todo = nz & ~(p >= j0 && p < j0 + kElimRowsPerWave ? 1u << (p - j0) : 0u);
    // in groups of 8 rows: all multipliers, then all their tables (scalar
    // loads issued together, one wait), then the arithmetic; a row that must
    // not change (the pivot, a zero entry, past n) has multiplier 0, whose
    // table is all zero
    constexpr int kGroup = 8;
#pragma unroll
    for (int i0 = 0; i0 < kElimRowsPerWave; i0 += kGroup) {
      uint32_t f[kGroup];
#pragma unroll
      for (int q = 0; q < kGroup; q++) {
        const uint32_t v = (__builtin_amdgcn_readlane(S[i0 + q][0], rl) >> rb) & 0xffu;
        f[q] = ((todo >> (i0 + q)) & 1u) ? v : 0u;
      }
      uint4 a[kGroup];
      uint32_t b[kGroup];
#pragma unroll
      for (int q = 0; q < kGroup; q++) {
        a[q] = {tb[f[q] * 8], tb[f[q] * 8 + 1], tb[f[q] * 8 + 2], tb[f[q] * 8 + 3]};
        b[q] = tb[f[q] * 8 + 4];
      }
#pragma unroll
      for (int q = 0; q < kGroup; q++)
#pragma unroll
        for (int h = 0; h < DPL; h++) S[i0 + q][h] ^= gmul4(a[q], b[q], s0[h], s1[h], s2[h]);
    }
#ifdef KODR_ELIM_TIMING
    if (r == 10) ts[5] = __builtin_amdgcn_s_memtime();
    if (r == 11) ts[6] = __builtin_amdgcn_s_memtime();
#endif
  }
#ifdef KODR_ELIM_TIMING
  ts[7] = __builtin_amdgcn_s_memtime();
  if (lane == 0) {
    uint64_t* o = reinterpret_cast<uint64_t*>(args.out + (size_t)g * args.out_gen_stride) + 8 * w;
    for (int q = 0; q < 8; q++) o[q] = ts[q];
  }
  return;
#endif
  __syncthreads();
  int c = lds.stop >= 0 ? lds.stop : n;
  if (full && c < k) c = 0;  // singular: kodr's own route (host) for the whole batch
  if (c < 2) c = 0;          // the first piece stays unreduced until a second one (full/decoder.go:58-61)
  // rows in pivot order: the row that pivoted column r is row r of the state
  uint8_t* out = args.out + (size_t)g * args.out_gen_stride;
#pragma unroll
  for (int i = 0; i < kElimRowsPerWave; i++) {
    const int j = j0 + i;
    const int at = j < 256 ? lds.colof[j] : -1;
    if (at < 0 || at >= c) continue;
#pragma unroll
    for (int h = 0; h < DPL; h++)
      reinterpret_cast<uint32_t*>(out + (size_t)at * args.out_pitch)[h * 64 + lane] = S[i][h];
  }
  if (tid == 0) args.counts[g] = c;
}


// ---- FULL batches, blocked: panels of 16 columns ------------------------
// The same result as the FULL case above ([I | C^-1], T in arrival order),
// computed by a blocked Gauss-Jordan whose serial part is one small panel
// per 16 columns instead of every one of the k steps:
//  1. panel b (columns jb = 16b ..): its candidates are rows jb .. jb + 15,
//     all owned by wave b (rows picked so far are exactly rows 0 .. jb - 1, as
//     long as every panel block is invertible).  Wave b inverts the block
//     M = C'[rows jb.., cols jb..] by Gauss-Jordan with row pivoting, one
//     lane per (row, dword) of [M | I]; S = M^-1 (LDS), the candidates' old
//     rows to LDS.  A singular block stops the kernel (count 0: the host
//     takes kodr's route for the batch, as for a singular C).
//  2. all waves: the new pivot rows N = S x (candidate rows), 1-2 dwords per
//     lane, to LDS.
//  3. wave b replaces its rows with N (pivot column jb + c -> row of S's
//     column c); every other row j gets row_j ^= sum_c row_j[jb + c] * N[c]
//     (multipliers wave-uniform: tables through the scalar cache).
// Two barriers per panel, k/16 panels.
struct ElimBlkLds {
  uint4 tab[256 * 2];      // the [256][8]-dword tables as 16-byte rows: tab[2f] = T0, T1; tab[2f + 1].x = T2
  uint32_t prow[16][128];  // the panel's candidate rows before the step
  uint32_t np[16][128];    // the new pivot rows, by panel column
  uint32_t pan[16][4];     // the panel block of the candidates (owner wave scratch)
  uint32_t sd[16][4];      // S[c][u] = byte u % 4 of sd[c][u / 4]
  int colof[256];          // pivot column of each row
  int fail;
};

__device__ __forceinline__ uint32_t sel0(uint32_t x) { return x & 0x07070707u; }
__device__ __forceinline__ uint32_t sel1(uint32_t x) { return (x >> 3) & 0x07070707u; }
__device__ __forceinline__ uint32_t sel2(uint32_t x) { return (x >> 6) & 0x03030303u; }
__device__ __forceinline__ uint32_t bperm(uint32_t v, int src_lane) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute(src_lane << 2, (int)v);
}

// The panel block's Gauss-Jordan, by one wave (all 64 lanes active): the
// candidates' panel dwords pan[t][d] (written by this wave) -> S in sd, the
// pivot column of each candidate row jb + t in colof, or fail.
typedef const __attribute__((address_space(4))) uint32_t cu32;
__device__ __forceinline__ void panel_gj(ElimBlkLds& lds, int jb, int nb, cu32* tb, int lane) {
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's own LDS writes land first
  const int t = lane >> 2, d = lane & 3;
  uint32_t P = lds.pan[t][d], Tr = 0;
#pragma unroll
  for (int e = 0; e < 4; e++)
    if (4 * d + e >= nb) P &= ~(0xffu << (8 * e));  // columns past the panel (the last one)
  if (t < nb && (t >> 2) == d) Tr = 1u << (8 * (t & 3));
  if (t >= nb) P = 0;
  uint32_t used = (0xffffu << nb) & 0xffffu;  // rows past k are not candidates
  int mycol = -1;
  bool ok = true;
  for (int c = 0; c < nb; c++) {
    const int cd = c >> 2, cb = 8 * (c & 3);
    const bool nz = (d == cd) && ((P >> cb) & 0xffu) != 0u && !((used >> t) & 1u);
    const uint64_t m = __builtin_amdgcn_ballot_w64(nz);
    if (m == 0) {
      ok = false;
      break;
    }
    const int pl = __builtin_ctzll(m), tp = pl >> 2;
    const uint32_t dp = (__builtin_amdgcn_readlane(P, pl) >> cb) & 0xffu;
    cu32* tinv = tb + kElimInvTables + dp * 8;  // tables of inv(dp) (gf256.go:77-86)
    const uint4 ti = {tinv[0], tinv[1], tinv[2], tinv[3]};
    const uint32_t ti2 = tinv[4];
    if (t == tp) {
      P = gmul4(ti, ti2, sel0(P), sel1(P), sel2(P));
      Tr = gmul4(ti, ti2, sel0(Tr), sel1(Tr), sel2(Tr));
      mycol = c;
    }
    const uint32_t Pp = bperm(P, tp * 4 + d), Tp = bperm(Tr, tp * 4 + d);
    uint32_t f = (bperm(P, t * 4 + cd) >> cb) & 0xffu;
    if (t == tp) f = 0u;
    const uint4 tf = lds.tab[2 * f];  // one ds_read_b128 + one ds_read_b32
    const uint32_t tf2 = lds.tab[2 * f + 1].x;
    P ^= gmul4(tf, tf2, sel0(Pp), sel1(Pp), sel2(Pp));
    Tr ^= gmul4(tf, tf2, sel0(Tp), sel1(Tp), sel2(Tp));
    used |= 1u << tp;
  }
  if (!ok) {
    if (lane == 0) lds.fail = 1;
  } else if (t < nb) {
    lds.sd[mycol][d] = Tr;
    if (d == 0) lds.colof[jb + t] = jb + mycol;
  }
}

template <int DPL>
__global__ __launch_bounds__(64 * kElimWaves) void gf_elim_blocked_kernel(ElimArgs args) {
  __shared__ ElimBlkLds lds;
  const int g = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int k = args.k;
  const int j0 = w * kElimRowsPerWave;
  const uint8_t* vec = args.vecs[g];
  const size_t vp = args.vpitch;
  typedef const __attribute__((address_space(4))) uint32_t cu32;
  cu32* tb = (cu32*)args.tables;

  for (int i = tid; i < 256 * 2; i += 64 * kElimWaves)
    lds.tab[i] = make_uint4(args.tables[4 * i], args.tables[4 * i + 1], args.tables[4 * i + 2], args.tables[4 * i + 3]);
  for (int i = tid; i < 256; i += 64 * kElimWaves) lds.colof[i] = -1;
  if (tid == 0) lds.fail = 0;

  // rows [C | I] in registers, as gf_elim_kernel
  uint32_t R[kElimRowsPerWave][DPL];
#pragma unroll
  for (int i = 0; i < kElimRowsPerWave; i++) {
    const int j = j0 + i;
#pragma unroll
    for (int h = 0; h < DPL; h++) {
      uint32_t v = 0;
      if (j < k) {
#pragma unroll
        for (int b = 0; b < 4; b++) {
          const int col = (h * 64 + lane) * 4 + b;
          uint32_t byte = 0;
          if (col < k) byte = vec[(size_t)j * vp + col];
          else if (col == k + j) byte = 1;
          v |= byte << (8 * b);
        }
      }
      R[i][h] = v;
    }
  }
  __syncthreads();

  const int npanels = (k + 15) / 16;
#ifdef KODR_ELIM_TIMING
  uint64_t tacc[6] = {0, 0, 0, 0, 0, 0};  // owner panel, barrier 1, pivot rows, barrier 2, row update
  uint64_t tq = __builtin_amdgcn_s_memtime(), tstart = tq;
#define KODR_STAMP(i)                              \
  do {                                             \
    const uint64_t tn = __builtin_amdgcn_s_memtime(); \
    tacc[i] += tn - tq;                            \
    tq = tn;                                       \
  } while (0)
#else
#define KODR_STAMP(i) \
  do {                \
  } while (0)
#endif
  for (int pb = 0; pb < npanels; pb++) {
    const int jb = pb * 16, nb = min(16, k - jb);
    const int pl0 = jb >> 2;  // lane of the panel's first dword (h = 0)
    if (w == pb) {
      // ---- 1. the owner: old rows out, panel block inverted ----
#pragma unroll
      for (int i = 0; i < kElimRowsPerWave; i++) {
#pragma unroll
        for (int h = 0; h < DPL; h++) lds.prow[i][h * 64 + lane] = R[i][h];
        if (lane >= pl0 && lane < pl0 + 4) lds.pan[i][lane - pl0] = R[i][0];
      }
      panel_gj(lds, jb, nb, tb, lane);
    }
    KODR_STAMP(0);
    __syncthreads();
    KODR_STAMP(1);
    if (lds.fail) break;  // uniform
    // ---- 2. the new pivot rows, spread over the workgroup ----
#pragma unroll
    for (int r = 0; r < DPL; r++) {
      const int idx = tid + r * 64 * kElimWaves;
      const int c = __builtin_amdgcn_readfirstlane(idx / (64 * DPL)), dw = idx % (64 * DPL);
      if (c < nb) {
        uint32_t acc = 0;
        for (int u4 = 0; u4 < 4; u4++) {  // S[c][4 u4 .. 4 u4 + 3]: one dword, four tables in flight
          const uint32_t sw = __builtin_amdgcn_readfirstlane(lds.sd[c][u4]);
          uint32_t x[4];
#pragma unroll
          for (int e = 0; e < 4; e++) x[e] = lds.prow[4 * u4 + e][dw];
#pragma unroll
          for (int e = 0; e < 4; e++) {
            const uint32_t su = (sw >> (8 * e)) & 0xffu;  // 0 past nb (S rows are zero there)
            const uint4 ts = {tb[su * 8], tb[su * 8 + 1], tb[su * 8 + 2], tb[su * 8 + 3]};
            const uint32_t ts2 = tb[su * 8 + 4];
            acc ^= gmul4(ts, ts2, sel0(x[e]), sel1(x[e]), sel2(x[e]));
          }
        }
        lds.np[c][dw] = acc;
      }
    }
    KODR_STAMP(2);
    __syncthreads();
    KODR_STAMP(3);
    // ---- 3. rows: the owner's become the pivot rows, the others drop the panel ----
    if (w == pb) {
#pragma unroll
      for (int i = 0; i < kElimRowsPerWave; i++)
        if (i < nb) {
          const int c = __builtin_amdgcn_readfirstlane(lds.colof[jb + i]) - jb;
#pragma unroll
          for (int h = 0; h < DPL; h++) R[i][h] = lds.np[c][h * 64 + lane];
        }
    } else if (j0 < k) {
      // one panel column c at a time: its pivot row's selectors, then every
      // row's multiplier table (the row's panel byte c: wave-uniform) read
      // from LDS one row ahead, so no row waits for its own table
      for (int c = 0; c < nb; c++) {
        uint32_t s0[DPL], s1[DPL], s2[DPL];
#pragma unroll
        for (int h = 0; h < DPL; h++) {
          const uint32_t x = lds.np[c][h * 64 + lane];
          s0[h] = sel0(x);
          s1[h] = sel1(x);
          s2[h] = sel2(x);
        }
        const int ql = pl0 + (c >> 2), qs = 8 * (c & 3);
        auto fetch = [&](int i, uint4& t, uint32_t& t2) {
          const uint32_t f = (__builtin_amdgcn_readlane(R[i][0], ql) >> qs) & 0xffu;
          t = lds.tab[2 * f];
          t2 = lds.tab[2 * f + 1].x;
        };
        // two rows ahead: a row's LDS reads have two rows of arithmetic to land
        uint4 ta, tb1, tn;
        uint32_t ta2, tb2, tn2;
        fetch(0, ta, ta2);
        fetch(1, tb1, tb2);
#pragma unroll
        for (int i = 0; i < kElimRowsPerWave; i++) {
          if (i + 2 < kElimRowsPerWave) fetch(i + 2, tn, tn2);
#pragma unroll
          for (int h = 0; h < DPL; h++) {
            const uint32_t p0 = __builtin_amdgcn_perm(ta.y, ta.x, s0[h]);
            const uint32_t p1 = __builtin_amdgcn_perm(ta.w, ta.z, s1[h]);
            const uint32_t p2 = __builtin_amdgcn_perm(ta2, ta2, s2[h]);
            R[i][h] = __builtin_amdgcn_bitop3_b32(R[i][h], p0, p1, 0x96) ^ p2;
          }
          ta = tb1;
          ta2 = tb2;
          tb1 = tn;
          tb2 = tn2;
        }
      }
    }
    KODR_STAMP(4);
  }
#ifdef KODR_ELIM_TIMING
  tacc[5] = __builtin_amdgcn_s_memtime() - tstart;
  if (lane == 0) {
    uint64_t* o = reinterpret_cast<uint64_t*>(args.out + (size_t)g * args.out_gen_stride) + 8 * w;
    for (int q = 0; q < 6; q++) o[q] = tacc[q];
  }
  if (tid == 0) args.counts[g] = 0;
  return;
#endif
#undef KODR_STAMP
  __syncthreads();
  const int c = lds.fail ? 0 : k;
  uint8_t* out = args.out + (size_t)g * args.out_gen_stride;
  if (c) {
#pragma unroll
    for (int i = 0; i < kElimRowsPerWave; i++) {
      const int j = j0 + i;
      if (j >= k) continue;
      const int at = lds.colof[j];
#pragma unroll
      for (int h = 0; h < DPL; h++)
        reinterpret_cast<uint32_t*>(out + (size_t)at * args.out_pitch)[h * 64 + lane] = R[i][h];
    }
  }
  if (tid == 0) args.counts[g] = c;
}


// ---- FULL batches, blocked, one dword per lane: the "circular" row -------
// The same panels as gf_elim_blocked_kernel, on half the bytes.  At any panel
// boundary a row's coefficient byte s and its T byte s are never both in
// play except where the row's own identity sits: coefficient columns [0, jb)
// are eliminated (zero) exactly where T columns [0, jb) can be non-zero, and
// an unpicked row j has T = e_j + (columns < jb).  So slot s (s < k) holds
// coefficient[s] XOR T[s], 64 lanes x 4 slots cover k <= 256 (against
// 2 dwords per lane for [C | T] at k > 128), and every step stays linear:
//  * a candidate's panel block is its slots with its identity XORed out;
//  * a new pivot row N[c] = S x (candidate rows) is the same combination of
//    slots (coefficient part e_(jb+c) + columns >= jb + 16, T part columns
//    < jb + 16, both in the panel's slots);
//  * a non-candidate row's panel slots are pure coefficients (its T is zero
//    there), so its multipliers read as before, and row ^= sum f_c N[c]
//    leaves 0 ^ T in those slots: f_c ^ f_c from N's identity.
// At the end the pivot row of column col holds e_col ^ T: T is its slots
// with byte col flipped.  The output is the blocked kernel's: [I | C^-1] at
// out_pitch, T from byte k.
__global__ __launch_bounds__(64 * kElimWaves) void gf_elim_circ_kernel(ElimArgs args) {
  __shared__ ElimBlkLds lds;
  const int g = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int k = args.k;
  const int j0 = w * kElimRowsPerWave;
  const uint8_t* vec = args.vecs[g];
  const size_t vp = args.vpitch;
  typedef const __attribute__((address_space(4))) uint32_t cu32;
  cu32* tb = (cu32*)args.tables;

  for (int i = tid; i < 256 * 2; i += 64 * kElimWaves)
    lds.tab[i] = make_uint4(args.tables[4 * i], args.tables[4 * i + 1], args.tables[4 * i + 2], args.tables[4 * i + 3]);
  for (int i = tid; i < 256; i += 64 * kElimWaves) lds.colof[i] = -1;
  if (tid == 0) lds.fail = 0;

  // slots of rows j0 .. j0 + 15: C[j] ^ e_j (slots >= k zero)
  uint32_t R[kElimRowsPerWave];
#pragma unroll
  for (int i = 0; i < kElimRowsPerWave; i++) {
    const int j = j0 + i;
    uint32_t v = 0;
    if (j < k) {
#pragma unroll
      for (int b = 0; b < 4; b++) {
        const int col = lane * 4 + b;
        uint32_t byte = col < k ? vec[(size_t)j * vp + col] : 0u;
        if (col == j) byte ^= 1u;
        v |= byte << (8 * b);
      }
    }
    R[i] = v;
  }
  __syncthreads();

  const int npanels = (k + 15) / 16;
#ifdef KODR_ELIM_TIMING
  uint64_t tacc[6] = {0, 0, 0, 0, 0, 0};  // owner panel, barrier 1, pivot rows, barrier 2, row update
  uint64_t tq = __builtin_amdgcn_s_memtime(), tstart = tq;
#define KODR_STAMP(i)                                 \
  do {                                                \
    const uint64_t tn = __builtin_amdgcn_s_memtime(); \
    tacc[i] += tn - tq;                               \
    tq = tn;                                          \
  } while (0)
#else
#define KODR_STAMP(i) \
  do {                \
  } while (0)
#endif
  for (int pb = 0; pb < npanels; pb++) {
    const int jb = pb * 16, nb = min(16, k - jb);
    const int pl0 = jb >> 2;  // lane of the panel's first slot
    if (w == pb) {
      // ---- 1. the owner: old rows out, panel block (identity removed) inverted ----
#pragma unroll
      for (int i = 0; i < kElimRowsPerWave; i++) {
        lds.prow[i][lane] = R[i];
        if (lane >= pl0 && lane < pl0 + 4) {
          uint32_t blk = R[i];
          if (i < nb && lane == pl0 + (i >> 2)) blk ^= 1u << (8 * (i & 3));  // row jb + i's own T byte
          lds.pan[i][lane - pl0] = blk;
        }
      }
      panel_gj(lds, jb, nb, tb, lane);
    }
    KODR_STAMP(0);
    __syncthreads();
    KODR_STAMP(1);
    if (lds.fail) break;  // uniform
    // ---- 2. the new pivot rows: one (panel column, slot dword) per thread ----
    {
      const int c = __builtin_amdgcn_readfirstlane(tid >> 6), dw = lane;
      if (c < nb) {
        uint32_t acc = 0;
        for (int u4 = 0; u4 < 4; u4++) {
          const uint32_t sw = __builtin_amdgcn_readfirstlane(lds.sd[c][u4]);
          uint32_t x[4];
#pragma unroll
          for (int e = 0; e < 4; e++) x[e] = lds.prow[4 * u4 + e][dw];
#pragma unroll
          for (int e = 0; e < 4; e++) {
            const uint32_t su = (sw >> (8 * e)) & 0xffu;
            const uint4 ts = {tb[su * 8], tb[su * 8 + 1], tb[su * 8 + 2], tb[su * 8 + 3]};
            const uint32_t ts2 = tb[su * 8 + 4];
            acc ^= gmul4(ts, ts2, sel0(x[e]), sel1(x[e]), sel2(x[e]));
          }
        }
        lds.np[c][dw] = acc;
      }
    }
    KODR_STAMP(2);
    __syncthreads();
    KODR_STAMP(3);
    // ---- 3. the owner's rows become the pivot rows, the others drop the panel ----
    if (w == pb) {
#pragma unroll
      for (int i = 0; i < kElimRowsPerWave; i++)
        if (i < nb) {
          const int c = __builtin_amdgcn_readfirstlane(lds.colof[jb + i]) - jb;
          R[i] = lds.np[c][lane];
        }
    } else if (j0 < k) {
      // every multiplier first: N[c]'s panel slots carry T bytes, so applying
      // N[c] changes the row's later panel slots (unlike [C | T], where they
      // hold the zero coefficients of N's identity block)
      uint32_t F[kElimRowsPerWave][4];
#pragma unroll
      for (int i = 0; i < kElimRowsPerWave; i++)
#pragma unroll
        for (int q = 0; q < 4; q++) F[i][q] = __builtin_amdgcn_readlane(R[i], pl0 + q);
      // (all 16 columns, unrolled, so that F is indexed by constants only and
      // stays in registers; past nb, in the last panel, every multiplier is
      // a slot >= k, zero in every row, so the stale N[c] adds nothing)
#pragma unroll
      for (int c = 0; c < 16; c++) {
        const uint32_t x = lds.np[c][lane];
        const uint32_t s0 = sel0(x), s1 = sel1(x), s2 = sel2(x);
        const int qd = c >> 2, qs = 8 * (c & 3);
        auto fetch = [&](int i, uint4& t, uint32_t& t2) {
          const uint32_t f = (F[i][qd] >> qs) & 0xffu;
          t = lds.tab[2 * f];  // (scalar loads of tb instead: 384 vs 368 us, profiles/r03/elim_circ/)
          t2 = lds.tab[2 * f + 1].x;
        };
        uint4 ta, tb1, tn;
        uint32_t ta2, tb2, tn2;
        fetch(0, ta, ta2);
        fetch(1, tb1, tb2);
#pragma unroll
        for (int i = 0; i < kElimRowsPerWave; i++) {
          if (i + 2 < kElimRowsPerWave) fetch(i + 2, tn, tn2);
          const uint32_t p0 = __builtin_amdgcn_perm(ta.y, ta.x, s0);
          const uint32_t p1 = __builtin_amdgcn_perm(ta.w, ta.z, s1);
          const uint32_t p2 = __builtin_amdgcn_perm(ta2, ta2, s2);
          R[i] = __builtin_amdgcn_bitop3_b32(R[i], p0, p1, 0x96) ^ p2;
          ta = tb1;
          ta2 = tb2;
          tb1 = tn;
          tb2 = tn2;
        }
      }
    }
    KODR_STAMP(4);
  }
#ifdef KODR_ELIM_TIMING
  tacc[5] = __builtin_amdgcn_s_memtime() - tstart;
  if (lane == 0) {
    uint64_t* o = reinterpret_cast<uint64_t*>(args.out + (size_t)g * args.out_gen_stride) + 8 * w;
    for (int q = 0; q < 6; q++) o[q] = tacc[q];
  }
  if (tid == 0) args.counts[g] = 0;
  return;
#endif
#undef KODR_STAMP
  __syncthreads();
  const int c = lds.fail ? 0 : k;
  uint8_t* out = args.out + (size_t)g * args.out_gen_stride;
  if (c) {
#pragma unroll
    for (int i = 0; i < kElimRowsPerWave; i++) {
      const int j = j0 + i;
      if (j >= k) continue;
      const int at = lds.colof[j];
      uint8_t* row = out + (size_t)at * args.out_pitch;
      uint32_t e = 0;  // e_at in this lane's 4 slots
      if (at >= 4 * lane && at < 4 * lane + 4) e = 1u << (8 * (at - 4 * lane));
      const uint32_t t = R[i] ^ e;
#pragma unroll
      for (int b = 0; b < 4; b++)
        if (4 * lane + b < k) {
          row[4 * lane + b] = (uint8_t)(e >> (8 * b));      // [I]
          row[k + 4 * lane + b] = (uint8_t)(t >> (8 * b));  // [C^-1]
        }
    }
  }
  if (tid == 0) args.counts[g] = c;
}

// ---- FULL batches on several workgroups per decoder (mc2, mc4) -----------
// One decoder's inversion split over several workgroups (below: mc2, the
// chain and the rows of 32-row groups in one workgroup each; mc4, the chain
// on a workgroup of its own beside 8-row row workgroups).  Both hand data
// between workgroups the same way (MI355X_MICROARCH.md, hand-off price list,
// granule form R2): 8-byte {data, tag} granules, each ONE agent-scope
// relaxed store (global_store_dwordx2 sc1); a consumer re-reads its granules
// with sc1 loads until every tag is this launch's epoch.  No fence, no flag.
// A singular panel block publishes FAIL; a workgroup that sees one publishes
// FAIL on what it still owes and stops, so every workgroup ends; spins are
// bounded.  Every workgroup writes its status word last.  All of a launch's
// workgroups must be resident at once (kElimMcMaxBlocks).  (Round 4's first
// multi-workgroup kernel, 32-row groups handing finished pivot rows to each
// other with no overlap between groups, is superseded by these two: 200 vs
// 153 (mc2) and 59 (mc4) us for one k = 256 decoder.)
constexpr uint32_t kMcFail = 0x80000000u;
// A launch owns kMcAttempts consecutive tags, args.epoch .. args.epoch + 3, one
// per attempt.  Attempt a inverts the rows rotated by mc_rot(a): when a panel's
// 16 x 16 block is singular although C may not be (pivots stay inside the
// panel's 16 rows, so a singular leading 16j x 16j block of C fails the
// attempt: about 6 % of uniform k = 256 batches), every workgroup starts the
// next attempt from the rows in another order.  FAIL granules carry the
// reason in their data: 0 this attempt failed, kMcAbort the launch stops (a
// singular last panel, which means C itself is singular; a panel block with
// a zero column, which means a structured -- systematic -- batch no row order
// fixes; a timeout; or the last attempt).  An abort is published with the
// last tag, so that a consumer in any attempt sees it.
constexpr int kMcAttempts = 4;
constexpr uint32_t kMcAbort = 1u;
// the longest a workgroup waits on one hand-off before it gives up (a
// workgroup of the launch that is not resident, e.g. behind another kernel;
// the host then takes kodr's route), in polls: a global poll (an agent-scope
// round trip, >= ~0.3 us, and s_sleep) 8192 times is >= ~2 ms, an LDS counter
// (>= ~50 cycles) 2^17 times >= ~3 ms.  Counted, not timed: a clock read in
// the poll loops (s_memrealtime) slowed the chain by ~13 % (58 -> 66 us).
constexpr int kMcPollSpins = 1 << 13;
constexpr int kMcLdsSpins = 1 << 17;

typedef __attribute__((address_space(1))) unsigned long long gu64;

#ifdef KODR_MC_CHECK
// Tuning build (round 6, the round-5 mc4 fault): every global access of mc2 /
// mc4 is checked against the allocations the host sized for the launch
// (gf_elim sets them before each launch); an access outside is printed and
// skipped instead of issued.
struct McBounds {
  const uint8_t *pub, *out, *cnt, *odev, *tab;
  uint64_t pub_bytes, out_bytes, cnt_bytes, odev_bytes, tab_bytes;
};
__device__ McBounds g_mcb;
__device__ __forceinline__ bool mc_in(const void* p, size_t len, const uint8_t* base, uint64_t bytes) {
  const uintptr_t a = (uintptr_t)p, b = (uintptr_t)base;
  return base && a >= b && a + len <= b + bytes;
}
__device__ __noinline__ void mc_report(int site, const void* p) {
  printf("KODR_MC_CHECK site %d block (%d,%d) thread %d addr %p pub %p+%lu out %p+%lu cnt %p+%lu odev %p+%lu\n",
         site, (int)blockIdx.x, (int)blockIdx.y, (int)threadIdx.x, p, g_mcb.pub, (unsigned long)g_mcb.pub_bytes,
         g_mcb.out, (unsigned long)g_mcb.out_bytes, g_mcb.cnt, (unsigned long)g_mcb.cnt_bytes, g_mcb.odev,
         (unsigned long)g_mcb.odev_bytes);
}
#define MC_CK(p, len, base, bytes, site)                                                          \
  (mc_in((const void*)(uintptr_t)(p), (len), (base), (bytes)) ||                                  \
   (mc_report((site), (const void*)(uintptr_t)(p)), false))
#define MC_CK_PUB(p, site) MC_CK((p), 8, g_mcb.pub, g_mcb.pub_bytes, site)
#else
#define MC_CK(p, len, base, bytes, site) true
#define MC_CK_PUB(p, site) true
#endif

// input row of row i < k in attempt att: (i + s) mod k, s = 0, k/2, k/4, 3k/4
__device__ __forceinline__ int mc_rot(int att, int k) {
  return att == 0 ? 0 : att == 1 ? k / 2 : att == 2 ? k / 4 : (3 * k) / 4;
}
__device__ __forceinline__ int mc_src_row(int gr, int k, int rot) {
  const int r = gr + rot;
  return r >= k ? r - k : r;
}

// a hand-off granule seen by attempt `tag` of a launch whose last tag is tlast:
// 0 this attempt's value, 1 this attempt failed (its FAIL, or a later attempt's
// value or FAIL: the producer has moved on), 2 abort, -1 not there yet
// (branch-free: a branch per granule made the compiler wait for each poll
// load before issuing the next, 4x the hand-off latency)
__device__ __forceinline__ int mc_tag_state(uint64_t x, uint32_t tag, uint32_t tlast) {
  const uint32_t tg = (uint32_t)(x >> 32), t = tg & ~kMcFail;
  const int failed = (tg & kMcFail) && ((uint32_t)x & kMcAbort) ? 2 : 1;
  const int later = t >= tag && t <= tlast ? failed : -1;
  return tg == tag ? 0 : later;
}


// the workgroup's fail word: the largest reason any wave saw (1 this attempt, 2 abort)
__device__ __forceinline__ void mc_set_fail(int* lfail, int why) {
  __hip_atomic_fetch_max(lfail, why, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

__device__ __forceinline__ void mc_put(gu64* dst, uint32_t tag, uint32_t v) {
  if (!MC_CK_PUB(dst, 1)) return;
  __hip_atomic_store(dst, ((unsigned long long)tag << 32) | v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// FAIL for attempt `tag` (why 1) or an abort for every attempt (why 2)
__device__ __forceinline__ void mc_put_fail(gu64* dst, uint32_t tag, uint32_t tlast, int why) {
  if (!MC_CK_PUB(dst, 2)) return;
  const uint32_t t = why >= 2 ? tlast : tag;
  __hip_atomic_store(dst, ((unsigned long long)(t | kMcFail) << 32) | (why >= 2 ? kMcAbort : 0u), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// why a singular panel block fails the launch: 2 (abort) when it is the last
// panel with rows of C (every block before it was invertible, so C is
// singular) or when a column of the block is zero in all 16 rows (a
// structured batch: random rows make that a 256^-16 event), else 1 (retry)
__device__ __forceinline__ int mc_singular_why(uint32_t blk, int lane, int p, int k) {
  if (p == (k - 1) / 16) return 2;
  uint32_t o = blk;  // OR over the 16 rows (t = lane / 4) of each dword d = lane % 4
  o |= bperm(o, lane ^ 4);
  o |= bperm(o, lane ^ 8);
  o |= bperm(o, lane ^ 16);
  o |= bperm(o, lane ^ 32);
  const bool zero = lane < 4 && ((o - 0x01010101u) & ~o & 0x80808080u) != 0;
  return __builtin_amdgcn_ballot_w64(zero) ? 2 : 1;
}

// byte j of a T row from the row attempt rotation s computed (T = T' Pi with
// (Pi C)_i = C_{(i + s) mod k}, so T[j] = T'[(j - s) mod k]); scr: this
// wave's 256 bytes of LDS
__device__ __forceinline__ uint32_t mc_unrotate(uint32_t v, uint32_t* scr, int lane, int k, int s) {
  scr[lane] = v;
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the wave's writes land before its reads
  const volatile uint8_t* b = reinterpret_cast<const volatile uint8_t*>(scr);
  uint32_t o = 0;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const int j = 4 * lane + q;
    if (j < k) {
      const int src = j - s < 0 ? j - s + k : j - s;
      o |= (uint32_t)b[src] << (8 * q);
    }
  }
  __builtin_amdgcn_s_waitcnt(0xc07f);  // ... and the reads before the next row's writes
  return o;
}

__device__ __forceinline__ uint32_t mc_mul(const uint4& t, uint32_t t2, uint32_t s0, uint32_t s1, uint32_t s2) {
  return __builtin_amdgcn_perm(t.y, t.x, s0) ^ __builtin_amdgcn_perm(t.w, t.z, s1) ^
         __builtin_amdgcn_perm(t2, t2, s2);
}

// lane v gets the value of lane 4 (v / 4) + cd (a quad broadcast, DPP)
__device__ __forceinline__ uint32_t quad_bcast(uint32_t v, int cd) {
  switch (cd) {
    case 0: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x00, 0xf, 0xf, false);
    case 1: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x55, 0xf, 0xf, false);
    case 2: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xaa, 0xf, 0xf, false);
    default: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xff, 0xf, 0xf, false);
  }
}

// one state row's bytes [0, k) from a row register (lane = dword): a dword
// store where the row is 4-byte aligned and the dword lies below k (pinned
// host memory takes whole coalesced writes), bytes otherwise
__device__ __forceinline__ void mc_store_row(uint8_t* row, uint32_t v, int lane, int k) {
#ifdef KODR_MC_CHECK
  if (4 * lane < k) {
    const int n = k - 4 * lane < 4 ? k - 4 * lane : 4;
    if (!mc_in(row + 4 * lane, n, g_mcb.out, g_mcb.out_bytes) && !mc_in(row + 4 * lane, n, g_mcb.odev, g_mcb.odev_bytes)) {
      mc_report(3, row + 4 * lane);
      return;
    }
  }
#endif
  if (((uintptr_t)row & 3) == 0 && 4 * lane + 3 < k) {
    *reinterpret_cast<uint32_t*>(row + 4 * lane) = v;
    return;
  }
#pragma unroll
  for (int b = 0; b < 4; b++)
    if (4 * lane + b < k) row[4 * lane + b] = (uint8_t)(v >> (8 * b));
}

// row gr of the launch's matrix in attempt rotation rot, lane = dword (rows
// past k: identity padding, the matrix stays [[C, 0], [0, I]])
__device__ __forceinline__ uint32_t mc_load_row(const ElimArgs& args, int g, int gr, int rot, int lane) {
  const int k = args.k;
  if (gr >= k) return gr >> 2 == lane ? 1u << (8 * (gr & 3)) : 0u;
  const uint8_t* src = args.vecs[g] + (size_t)mc_src_row(gr, k, rot) * args.vpitch;
  if (!MC_CK(src, k, args.vecs[g], (uint64_t)(args.n[g] - 1) * args.vpitch + k, 5)) return 0u;
  uint32_t v = 0;
#pragma unroll
  for (int b = 0; b < 4; b++)
    if (4 * lane + b < k) v |= (uint32_t)src[4 * lane + b] << (8 * b);
  return v;
}

// v, opaque to the compiler: an attempt's body takes its indices through
// these, so that nothing computed from them is hoisted out of the attempt
// loop (hoisted addresses stayed live through both roles and spilled)
__device__ __forceinline__ int mc_opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}
__device__ __forceinline__ int mc_opaque_s(int v) {
  asm volatile("" : "+s"(v));
  return v;
}
__device__ __forceinline__ gu64* mc_opaque_s(gu64* v) {
  asm volatile("" : "+s"(v));
  return v;
}

// A workgroup that starts after its decoder's launch was given up (an abort
// in the decoder's abort granule, written before any failed status word)
// reads no input at all: the host may already have handed the rows back to
// their owner.  (The granule's read is issued beside the table loads.)

// ---- mc2: the same inversion, pipelined inside each workgroup -------------
// Panels of 16 columns (NP = 2P); workgroup q owns panels 2q ("A rows", its
// local rows 0-15) and 2q + 1 ("B rows", 16-31).  In-place block
// Gauss-Jordan in "L form": panel p publishes R_p (its 16 rows as they are
// before its step) and S_p = (R_p's 16 x 16 block)^-1; a row i outside the
// panel takes F_i = row_i[panel] x S_p, then row_i ^= F_i x R_p and
// row_i[panel] = F_i; the panel's own rows become S_p x R_p with S_p in the
// panel columns (both: new = base ^ G x R_p, then the panel columns := G,
// with G = F_i, base = row_i or G = row of S_p, base = 0).
// Two roles per workgroup, synchronised through LDS counters, not barriers:
//  * row waves 0-7 hold the 32 rows (4 per wave, lane = dword) and apply
//    every panel in order, one panel behind the chain;
//  * chain waves 8-15 run the critical path: for an owned panel p, wave 8
//    brings the 16 x 16 block up to date with panel p - 1 (two small products
//    from rows as of panel p - 2, so it does not wait for the row waves'
//    apply of p - 1), inverts it (mc2_panel_gj) and publishes S_p; for any
//    other panel the chain waves poll R_p and S_p into LDS.
// Hand-offs between workgroups as described above (granules tagged with
// the attempt's tag, FAIL bit; bounded waits); three LDS slots per panel
// buffer so a slot is rewritten only after both roles are two panels on.
constexpr int kMc2Slots = 3;
constexpr int kMc2ApplyCols = 4;  // columns per operand batch in the row apply
constexpr int kMc2PanelGran = 16 * 64 + 64;  // granules per panel: R_p rows, then S_p

struct ElimMc2Lds {
  uint4 tab[256 * 2];
  uint4 itab[256 * 2];
  uint32_t rp[kMc2Slots][16][64];  // R_p by slot p % 3
  uint32_t sp[kMc2Slots][16][4];   // S_p by rows: S[c][u] = byte u % 4 of sp[c][u / 4]
  uint32_t mb[kMc2Slots][16][8];   // owned panel p: its rows' panel p - 1 (dwords 0-3) and panel p (4-7) columns, as of panel p - 2
  uint32_t mw[8][4][4];            // row wave w: its rows' columns of the panel it applies (the multipliers)
  uint32_t fw[8][4][4];            // row wave w: G of its rows
  int rows_done;                   // row-wave iterations finished (8 per panel, 8 for the start)
  int chain_cnt;                   // chain-wave iterations finished (8 per panel)
  int fail;                        // this attempt: 1 failed, 2 abort
  int late;                        // the launch was aborted before this workgroup started
};

__device__ __forceinline__ bool mc2_wait(ElimMc2Lds& lds, int* ctr, int target) {
  for (int spins = 0;; spins++) {
    if (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) return true;
    if (__hip_atomic_load(&lds.fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return false;
    if (spins > kMcLdsSpins) {
      mc_set_fail(&lds.fail, 2);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}
// this wave's LDS writes first, then one count
__device__ __forceinline__ void mc2_signal(int* ctr, int lane) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
  if (lane == 0) __hip_atomic_fetch_add(ctr, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// acc ^ sum over 8 terms of (tables of m[c]) x x[c], both the tables and the
// data read from LDS first (x: 8 dwords at stride `xs` from `xp`), then the
// arithmetic (selectors computed after the reads)
// (m: the 8 multipliers packed 4 per dword, mw[0..1])
__device__ __forceinline__ uint32_t mc3_dot8x(const uint4* tab, uint32_t acc, const uint32_t* mw, const uint32_t* xp,
                                              int xs) {
  uint4 tt[8];
  uint32_t t2[8], x[8];
#pragma unroll
  for (int c = 0; c < 8; c++) {
    const uint32_t m = (mw[c >> 2] >> (8 * (c & 3))) & 0xffu;
    tt[c] = tab[2 * m];
    t2[c] = tab[2 * m + 1].x;
    x[c] = xp[c * xs];
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int c = 0; c < 8; c++) acc ^= gmul4(tt[c], t2[c], sel0(x[c]), sel1(x[c]), sel2(x[c]));
  return acc;
}

// the block update (F = M x S, blk ^= F x R[:, panel p]) in batches of 8
// terms, operands read per batch (no registers held across the wait)
__device__ __forceinline__ uint32_t mc3_block_update_c(const uint4* tab, uint32_t blk, const uint32_t* mrow,
                                                       const uint32_t (*sp)[4], const uint32_t (*rp)[64], int col0,
                                                       int lane) {
  const int d = lane & 3;
  uint32_t mw[4];
#pragma unroll
  for (int q = 0; q < 4; q++) mw[q] = mrow[q];
  uint32_t F = mc3_dot8x(tab, 0u, mw, &sp[0][d], 4);
  F = mc3_dot8x(tab, F, mw + 2, &sp[8][d], 4);
  uint32_t fw[4];
#pragma unroll
  for (int q = 0; q < 4; q++) fw[q] = quad_bcast(F, q);
  const uint32_t acc = mc3_dot8x(tab, blk, fw, &rp[0][col0 + d], 64);
  return mc3_dot8x(tab, acc, fw + 2, &rp[8][col0 + d], 64);
}

// The circular-form inversion ((t, d) layout as mc3_gj_circ), branch-free
// in the common case.  The pivot of column c is the lowest unpicked row whose
// entry is non-zero; the step guesses the lowest unpicked row (its lane is
// known from the SGPR candidate mask before the step) and reads its entry dp
// with one v_readlane of P, then the uniform read of inv(dp)'s tables and the
// ds_bpermute of the pivot row go out at once; only when dp is zero (1 in
// 256) does it take the ballot of f != 0 under the mask (the same rule, so
// the same pivots).  The row's own tables (of f) are read right after f,
// beside the pivot path; every row computes both the pivot's and a non-pivot
// row's new value and selects.  (Before round 6 the ballot -> s_ff1 ->
// v_readlane of dp ran on every step: 5,258 against 4,927 cycles per panel,
// tools/probe/chain_probe.hip, profiles/r06/chain/.)
__device__ __forceinline__ bool mc3_gj(const uint4* tab, const uint4* itab, uint32_t P, int lane, uint32_t* s_val,
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
    int pl = (int)__builtin_ctzll(cand);
    uint32_t dp = (__builtin_amdgcn_readlane(P, pl + cd) >> cb) & 0xffu;
    uint4 ti = itab[2 * dp];
    uint32_t ti2 = itab[2 * dp + 1].x;
    uint32_t Pp = bperm(P, pl + d);
    if (__builtin_expect(dp == 0u, 0)) {
      const uint64_t m = __builtin_amdgcn_ballot_w64(f != 0u) & cand;
      fail |= m == 0;
      pl = (int)__builtin_ctzll(m | (1ull << 60));  // a failed column picks lane 60 (result unused)
      dp = __builtin_amdgcn_readlane(f, pl);
      ti = itab[2 * dp];
      ti2 = itab[2 * dp + 1].x;
      Pp = bperm(P, pl + d);
    }
    const int tp = pl >> 2;
    cand &= ~(1ull << pl);
    pinv |= (uint64_t)c << (4 * tp);
    const uint32_t inv = (ti.x >> 8) & 0xffu;
    const uint32_t Q = gmul4(ti, ti2, sel0(Pp), sel1(Pp), sel2(Pp)) ^ (d == cd ? inv << cb : 0u);
    uint32_t upd = P ^ gmul4(tf, tf2, sel0(Q), sel1(Q), sel2(Q));
    asm volatile("" : "+v"(upd));  // (on every lane: not sunk into an exec-masked branch)
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

// the chain waves' sleep between hand-off polls: 8 and 32 measured the same
// beside the pipelined encode (3.334-3.358 against 3.337-3.352 ms per step)
// and alone (mc2 16 decoders 188.7 / 192.5 against 188.4 us), so the polls'
// agent-scope traffic is not what slows the encode beside it
// (tools/gpu_r6_p.sh, profiles/r06/poll_sleep/)
#ifndef KODR_MC2_POLL_SLEEP
#define KODR_MC2_POLL_SLEEP 2
#endif
#ifdef KODR_MC2_WAVES_PER_EU  // (tuning builds only: mc2's register cap, tools/gpu_r6_i.sh)
#define KODR_MC2_ATTR __attribute__((amdgpu_waves_per_eu(KODR_MC2_WAVES_PER_EU)))
#else
#define KODR_MC2_ATTR
#endif
__global__ __launch_bounds__(1024) KODR_MC2_ATTR void gf_elim_mc2_kernel(ElimArgs args) {
  __shared__ ElimMc2Lds lds;
  const int q = blockIdx.x, g = blockIdx.y, P = gridDim.x, NP = 2 * gridDim.x;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int k = args.k;
  const uint32_t tag0 = args.epoch, tlast = tag0 + kMcAttempts - 1;
  gu64* const pub = (gu64*)args.pub + (size_t)g * NP * kMc2PanelGran;
  gu64* const pubA = (gu64*)args.pub + (size_t)gridDim.y * NP * kMc2PanelGran + g;  // the decoder's abort granule
#ifdef KODR_ELIM_TIMING
  // tuning build: s_memrealtime (100 MHz) stamps by lane 0 of row wave 0 and
  // chain wave 0, into this workgroup's 1 KiB of the T region (no result):
  // chain [4 p + j]: panel p's start, rows ready / polled, small products
  // done / slot free, end; row wave [64 + p] iteration p done, [80] entry,
  // [81] rows loaded, [82] last apply done, [83] rows out
  gu64* const tsout = (gu64*)(args.out + (size_t)g * args.out_gen_stride + (size_t)q * 1024);
#define MC2_STAMP(i)                                                                                \
  do {                                                                                              \
    if (lane == 0)                                                                                  \
      __hip_atomic_store(tsout + (i), (unsigned long long)__builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED, \
                         __HIP_MEMORY_SCOPE_SYSTEM);                                                \
  } while (0)
#else
#define MC2_STAMP(i) \
  do {               \
  } while (0)
#endif
  if (w == 0) MC2_STAMP(80);

  const uint64_t ab = tid == 0 ? __hip_atomic_load(pubA, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
  for (int i = tid; i < 256 * 2; i += 1024) {
    const uint32_t* a = args.tables + 4 * i;
    const uint32_t* b = args.tables + kElimInvTables + 4 * i;
    lds.tab[i] = make_uint4(a[0], a[1], a[2], a[3]);
    lds.itab[i] = make_uint4(b[0], b[1], b[2], b[3]);
  }
  if (tid == 0) lds.late = mc_tag_state(ab, tag0, tlast) == 2;
  __syncthreads();
  const bool late = __builtin_amdgcn_readfirstlane(lds.late) != 0;

  // row waves: T rows 32 q + 4 w + i of the successful attempt (assigned only
  // on the way out of the loop, so nothing is carried through the chain's path)
  uint32_t Tout[4];
  int fail = late ? 2 : 0, att = 0;
  for (; !late; att++) {
    const uint32_t tag = tag0 + att;
    const int rot = mc_rot(att, k);
    if (tid == 0) {  // (separate stores: a merged one kept a vector of zeros live through the kernel)
      __hip_atomic_store(&lds.rows_done, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_store(&lds.chain_cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_store(&lds.fail, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __syncthreads();
    // the attempt, on opaque copies of the indices (mc_opaque)
    auto attempt = [&](const int q, const int w, const int lane, gu64* const pub) {
    int unpublished = 2 * q;  // chain wave 0: the first owned panel whose S_p is not out yet
    uint32_t R[4] = {0u, 0u, 0u, 0u};  // row waves: rows 32 q + 4 w + i
    if (w < 8) {
      // ================= row waves: rows 4w .. 4w + 3 =================
      const int half = w >> 2;  // 0: panel 2q's rows, 1: panel 2q + 1's
#pragma unroll
      for (int i = 0; i < 4; i++) R[i] = mc_load_row(args, g, 32 * q + 4 * w + i, rot, lane);
      // workgroup 0's first panel: its block for the chain (no earlier panel)
      if (q == 0 && half == 0 && lane < 4)
#pragma unroll
        for (int i = 0; i < 4; i++) lds.mb[0][4 * w + i][4 + lane] = R[i];
      mc2_signal(&lds.rows_done, lane);
      if (w == 0) MC2_STAMP(81);

      auto apply = [&](int pa) {
        const int slot = pa % kMc2Slots, db = 4 * pa;
        const bool own = (pa >> 1) == q && (pa & 1) == half;
        // G of the 4 rows: the panel's S rows (own) or F (in lds.fw)
        const uint32_t(*Gp)[4] = own ? &lds.sp[slot][4 * (w & 3)] : lds.fw[w];
        if (!own) {
          // F of the 4 rows: lane (cg, i, u) sums c = 4 cg .. 4 cg + 3, then
          // the four groups are folded (lanes 16 and 32 apart)
          if (lane >= db && lane < db + 4)
#pragma unroll
            for (int i = 0; i < 4; i++) lds.mw[w][i][lane - db] = R[i];
          __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's writes land first
          const int cg = lane >> 4, i = (lane >> 2) & 3, u = lane & 3;
          const uint32_t mwd = lds.mw[w][i][cg];
          uint32_t acc = 0;
#pragma unroll
          for (int cc = 0; cc < 4; cc++) {
            const uint32_t m = (mwd >> (8 * cc)) & 0xffu;
            const uint4 t = lds.tab[2 * m];
            const uint32_t t2 = lds.tab[2 * m + 1].x;
            const uint32_t xv = lds.sp[slot][4 * cg + cc][u];
            acc ^= gmul4(t, t2, sel0(xv), sel1(xv), sel2(xv));
          }
          acc ^= bperm(acc, lane ^ 16);
          acc ^= bperm(acc, lane ^ 32);
          if (lane < 16) lds.fw[w][i][u] = acc;
          __builtin_amdgcn_s_waitcnt(0xc07f);
        }
        if (w == 0) MC2_STAMP(112 + pa);  // F of the rows known (pa <= 15: index <= 127)
        uint32_t acc[4];
#pragma unroll
        for (int i = 0; i < 4; i++) acc[i] = own ? 0u : R[i];
        // kMc2ApplyCols columns per batch, one batch live at a time (the whole
        // loop unrolled spilled 513 VGPRs).  The kernel holds ~113 VGPRs, all of
        // a SIMD's file at 4 waves, so the row copies launched beside it cannot
        // share its CUs; capped at 96 (waves_per_eu 5, a few bytes spilled) with
        // the copies at 2 or 4 loads per lane, the round trip measured slower
        // (238-241 against 230-235, 235-236 against 228-230 us per generation,
        // profiles/r04/var_ab/); in the pipelined round trip (round 6, encode
        // waves beside it) 96 VGPRs measured the same as 128 (3.336-3.355 ms
        // per step both), 80 and 64 slower (3.39-3.48: spills),
        // profiles/r06/mc2_vgpr/
#pragma unroll 1
        for (int cb = 0; cb < 16; cb += kMc2ApplyCols) {
          uint32_t gw[4];  // the bytes of columns cb .. of each row's G (wave-uniform)
#pragma unroll
          for (int i = 0; i < 4; i++) gw[i] = __builtin_amdgcn_readfirstlane(Gp[i][cb >> 2]) >> (8 * (cb & 3));
          // the (uniform) table reads and the data reads of these columns
          // first, then the arithmetic: one LDS round trip per batch (sinking
          // each read next to its use cost one round trip per term)
          uint4 tt[kMc2ApplyCols][4];
          uint32_t t2[kMc2ApplyCols][4], xs[kMc2ApplyCols];
#pragma unroll
          for (int cc = 0; cc < kMc2ApplyCols; cc++) {
            xs[cc] = lds.rp[slot][cb + cc][lane];
#pragma unroll
            for (int i = 0; i < 4; i++) {
              const uint32_t f = (gw[i] >> (8 * cc)) & 0xffu;
              tt[cc][i] = lds.tab[2 * f];
              t2[cc][i] = lds.tab[2 * f + 1].x;
            }
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int cc = 0; cc < kMc2ApplyCols; cc++) {
            const uint32_t s0 = sel0(xs[cc]), s1 = sel1(xs[cc]), s2 = sel2(xs[cc]);
#pragma unroll
            for (int i = 0; i < 4; i++) acc[i] ^= mc_mul(tt[cc][i], t2[cc][i], s0, s1, s2);
          }
        }
        const int u = lane - db;  // the panel columns take G
#pragma unroll
        for (int i = 0; i < 4; i++) R[i] = (u >= 0 && u < 4) ? Gp[i][u & 3] : acc[i];
      };

      for (int p = 0; p < NP; p++) {
        if (!mc2_wait(lds, &lds.rows_done, 8 * (p + 1)) || !mc2_wait(lds, &lds.chain_cnt, 8 * p)) break;
        if (w == 0) MC2_STAMP(96 + p);
        if (p >= 1) apply(p - 1);
        if ((p >> 1) == q && (p & 1) == half) {  // my rows are panel p's: R_p out
          const int slot = p % kMc2Slots;
          gu64* dst = pub + (size_t)p * kMc2PanelGran;
#pragma unroll
          for (int i = 0; i < 4; i++) {
            const int r = 4 * (w & 3) + i;
            lds.rp[slot][r][lane] = R[i];
            mc_put(dst + r * 64 + lane, tag, R[i]);
          }
        }
        const int pn = p + 1;
        if (pn < NP && (pn >> 1) == q && (pn & 1) == half) {  // next panel's block for the chain
          const int slot = pn % kMc2Slots;
#pragma unroll
          for (int i = 0; i < 4; i++) {
            const int r = 4 * (w & 3) + i;
            if (lane >= 4 * p && lane < 4 * p + 4) lds.mb[slot][r][lane - 4 * p] = R[i];
            if (lane >= 4 * pn && lane < 4 * pn + 4) lds.mb[slot][r][4 + lane - 4 * pn] = R[i];
          }
        }
        mc2_signal(&lds.rows_done, lane);
        if (w == 0) MC2_STAMP(64 + p);
      }
      if (mc2_wait(lds, &lds.chain_cnt, 8 * NP) && mc2_wait(lds, &lds.rows_done, 8 * (NP + 1))) {
        apply(NP - 1);
        if (w == 0) MC2_STAMP(82);
      }
    } else {
      // ================= chain waves =================
      const int cw = w - 8;
      if (cw == 0) __builtin_amdgcn_s_setprio(3);
      for (int p = 0; p < NP; p++) {
        const int slot = p % kMc2Slots;
        gu64* base = pub + (size_t)p * kMc2PanelGran;
        // every chain wave finished panel p - 1 (no wave runs ahead: the count
        // then means exactly that)
        if (!mc2_wait(lds, &lds.chain_cnt, 8 * p)) break;
        if (cw == 0) MC2_STAMP(4 * p);
        if ((p >> 1) == q) {
          if (!mc2_wait(lds, &lds.rows_done, 8 * (p + 1))) break;
          if (cw == 0) MC2_STAMP(4 * p + 1);
          if (cw == 0) {
            // the block brought up to date with panel p - 1 (two 16-term
            // products, operand reads batched), then inverted in registers
            const int t = lane >> 2, d = lane & 3;
            uint32_t blk = lds.mb[slot][t][4 + d];
            if (p >= 1) {
              const int ps = (p - 1) % kMc2Slots;
              blk = mc3_block_update_c(lds.tab, blk, lds.mb[slot][t], lds.sp[ps], lds.rp[ps], 4 * p, lane);
            }
            MC2_STAMP(4 * p + 2);
            uint32_t sval = 0;
            int srow = 0;
            const bool inv_ok = mc3_gj(lds.tab, lds.itab, blk, lane, &sval, &srow);
            if (inv_ok) {
              lds.sp[slot][srow][d] = sval;
              mc_put(base + 16 * 64 + srow * 4 + d, tag, sval);
              unpublished = p + 1;
            } else {
              mc_set_fail(&lds.fail, mc_singular_why(blk, lane, p, k));
            }
            MC2_STAMP(4 * p + 3);
          }
          if (__hip_atomic_load(&lds.fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
          mc2_signal(&lds.chain_cnt, lane);
        } else {
          // another workgroup's panel: R_p (rows 2cw, 2cw + 1) and S_p (wave 0) into LDS
          const gu64* src = base + (size_t)(2 * cw) * 64 + lane;
          uint64_t a = 0, b = 0, s = 0;
          int why = 0;
          for (int spins = 0;; spins++) {
            a = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            b = __hip_atomic_load(src + 64, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (cw == 0) s = __hip_atomic_load(base + 16 * 64 + lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int sa = mc_tag_state(a, tag, tlast), sb = mc_tag_state(b, tag, tlast);
            const int ss = cw == 0 ? mc_tag_state(s, tag, tlast) : 0;
            if (__builtin_amdgcn_ballot_w64(sa == 2 || sb == 2 || ss == 2)) {
              why = 2;
              break;
            }
            if (__builtin_amdgcn_ballot_w64(sa == 1 || sb == 1 || ss == 1)) {
              why = 1;
              break;
            }
            if (__builtin_amdgcn_ballot_w64(sa != 0 || sb != 0 || ss != 0) == 0) break;
            if (const int lf = __hip_atomic_load(&lds.fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
              why = lf;
              break;
            }
            if (spins > kMcPollSpins) {
              why = 2;
              break;
            }
            __builtin_amdgcn_s_sleep(KODR_MC2_POLL_SLEEP);
          }
          if (why) {
            mc_set_fail(&lds.fail, why);
            break;
          }
          if (cw == 0) MC2_STAMP(4 * p + 1);
          if (!mc2_wait(lds, &lds.rows_done, 8 * p)) break;  // the slot's last readers are done
          if (cw == 0) MC2_STAMP(4 * p + 2);
          lds.rp[slot][2 * cw][lane] = (uint32_t)a;
          lds.rp[slot][2 * cw + 1][lane] = (uint32_t)b;
          if (cw == 0) lds.sp[slot][lane >> 2][lane & 3] = (uint32_t)s;
          mc2_signal(&lds.chain_cnt, lane);
          if (cw == 0) MC2_STAMP(4 * p + 3);
        }
      }
      if (cw == 0) __builtin_amdgcn_s_setprio(0);
    }
    __syncthreads();
    fail = lds.fail;
#ifdef KODR_ELIM_TIMING
    if (!fail) fail = 2;  // the stamps overwrite T: kodr's route on the host
#endif
    if (fail && w == 8) {
      // owned panels whose S_p is not out (an abort: every owned panel): FAIL
      // on R_p and S_p, so that every later workgroup stops too
      for (int p = fail >= 2 ? 2 * q : unpublished; p < 2 * q + 2 && p < NP; p++) {
        gu64* base = pub + (size_t)p * kMc2PanelGran;
        for (int r = 0; r < 17; r++) mc_put_fail(base + r * 64 + lane, tag, tlast, fail);
      }
      // the FAILs reach L2 before the row waves' stores of the next attempt
      // to the same R_p slots (another wave: the barrier alone does not order them)
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    }
    if (!fail && w < 8) {
      // T = T' Pi: the rotation undone (through a slot no wave reads any more)
      uint32_t* scr = &lds.rp[NP % kMc2Slots][0][0] + 64 * w;
      uint8_t* out = args.out + (size_t)g * args.out_gen_stride;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        Tout[i] = rot ? mc_unrotate(R[i], scr, lane, k, rot) : R[i];
        const int gr = 32 * q + 4 * w + i;
        if (gr < k) mc_store_row(out + (size_t)gr * args.out_pitch + (args.direct ? 0 : k), Tout[i], lane, k);
      }
    }
    };
    attempt(mc_opaque_s(q), mc_opaque_s(w), mc_opaque(lane), mc_opaque_s(pub));
    __syncthreads();  // every wave read lds.fail before the next attempt resets it
    if (fail != 1 || att + 1 == kMcAttempts) break;
  }
  const bool ok = fail == 0;
  if (w == 0) MC2_STAMP(83);
#undef MC2_STAMP
  if (!ok && tid == 0) mc_put_fail(pubA, tag0, tlast, 2);  // late workgroups read no input
  if (args.direct) __atomic_thread_fence(__ATOMIC_RELEASE);  // this wave's T rows reach (host) memory first
  __syncthreads();
  if (tid == 0) {
    const uint32_t tg = late ? tlast : tag0 + att;
    if (args.direct) {
      __atomic_thread_fence(__ATOMIC_RELEASE);
      __hip_atomic_store(&args.counts[g * P + q], (int)(ok ? tg : tg | kMcFail), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    } else {
      args.counts[g * P + q] = ok ? 1 : 0;
    }
  }
  // the device copy of T after the system-scope release (as in mc4)
  if (w < 8 && args.out_dev && ok)
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int gr = 32 * q + 4 * w + i;
      if (gr < k) mc_store_row(args.out_dev + ((size_t)g * k + gr) * k, Tout[i], lane, k);
    }
}

// ---- mc4: a chain workgroup beside one row workgroup per 16-row panel ------
// The same block Gauss-Jordan in L form as gf_elim_mc2_kernel, with the two
// roles on different CUs, so that the critical path -- bring panel p's 16 x
// 16 block up to date with panel p - 1, invert it -- never leaves one
// workgroup and never shares a SIMD with the row updates:
//  * row workgroup r (blockIdx.x = r < NP) holds rows 16 r .. 16 r + 15
//    (4 waves x 4 rows, lane = dword) and applies every panel j in order
//    from S_j (the chain's) and R_j (panel j's rows as of j - 1, from row
//    workgroup j; its own when r = j); after apply(j) it publishes R_r when
//    r = j + 1 and MB_r = its rows' columns of panels r - 1 and r when
//    r = j + 2 (both "as of r - 1 / r - 2", what the chain and the other
//    row workgroups need next);
//  * the chain workgroup (blockIdx.x = NP): wave 1 stages MB_p and R_{p-1}'s
//    panel-p columns (both as of p - 2) into LDS as they appear; wave 0 updates
//    the block with S_{p-1} (two 16-term products, mc4_block_update), inverts
//    it (mc3_gj) and publishes S_p.
// The row data the chain needs for panel p leaves the row workgroups one
// panel earlier (after apply(p - 2)), so the chain waits on them only when a
// row workgroup's hand-off and apply take longer than one chain step.
// Hand-offs are 8-byte {data, tag} granules (agent-scope relaxed stores,
// polled with agent-scope loads), as in mc2; a singular block publishes
// FAIL on every later S_p, and a workgroup that sees FAIL publishes FAIL on
// its own slots and starts the next attempt (or stops), so every workgroup
// ends; waits are bounded.
// Results are direct only: T rows into out (pinned host memory) and one
// status word per workgroup, counts[g * (NP + 1) + x].
constexpr int kMc4Threads = 256;
constexpr int kMc4SGran = 64, kMc4RGran = 16 * 64, kMc4MGran = 16 * 8;

struct ElimMc4Lds {
  uint4 tab[256 * 2];
  uint4 itab[256 * 2];      // chain only
  uint32_t rp[16][64];      // row workgroup: R_j
  uint32_t sp[16][4];       // row workgroup: S_j
  uint32_t mw[4][4][4];     // row wave w: its rows' panel-j columns (multipliers)
  uint32_t fw[4][4][4];     // row wave w: F of its rows
  uint32_t cmb[2][16][8];   // chain: MB_p by slot p % 2 (M: dwords 0-3, X: 4-7)
  uint32_t crq[2][16][4];   // chain: R_{p-1}'s panel-p columns
  uint4 csel[2][16][4];     // chain: selectors (sel0, sel1, sel2) of S_p's dwords, slot p % 2
  uint4 crsel[2][16][4];    // chain: selectors of the staged R_{p-1} columns
  int staged, consumed, fail, late;
};

__device__ __forceinline__ size_t mc4_pub_words(int NP) {
  return (size_t)NP * (kMc4SGran + kMc4RGran + kMc4MGran);
}

// polls N granules per lane (at src[i * stride]) until every tag is this
// attempt's: 0 (values in v), 1 this attempt failed (a FAIL or a later tag
// seen, or the workgroup's fail word 1), 2 abort (an abort, a timeout, or
// the fail word 2)
template <int N>
__device__ __forceinline__ int mc4_poll(const gu64* src, int stride, uint32_t tag, uint32_t tlast, uint32_t* v,
                                        const int* lfail) {
  for (int spins = 0;; spins++) {
    bool okv = true, f1 = false, f2 = false;
    uint64_t x[N];
#pragma unroll
    for (int i = 0; i < N; i++)  // every load in flight before the first wait
      x[i] = MC_CK_PUB(src + (size_t)i * stride, 6)
                 ? __hip_atomic_load(src + (size_t)i * stride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                 : 0ull;
#pragma unroll
    for (int i = 0; i < N; i++) {
      const int s = mc_tag_state(x[i], tag, tlast);
      okv = okv && s == 0;
      f1 = f1 || s == 1;
      f2 = f2 || s == 2;
      v[i] = (uint32_t)x[i];
    }
    if (__builtin_amdgcn_ballot_w64(f2)) return 2;
    if (__builtin_amdgcn_ballot_w64(f1)) return 1;
    if (__builtin_amdgcn_ballot_w64(!okv) == 0) return 0;
    if (lfail)
      if (const int lf = __hip_atomic_load(lfail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return lf;
    if (spins > kMcPollSpins) return 2;
    __builtin_amdgcn_s_sleep(1);
#if defined(KODR_TUNE) && defined(KODR_MC_PROBE)
    // tuning build (round 5's measurement, rebuilt for the fault check of
    // round 6): not there yet -- wait on lane 0's first granule alone (one
    // address for the wave) before the next full poll
    if (__builtin_amdgcn_readfirstlane(mc_tag_state(x[0], tag, tlast)) < 0) {
      const uint64_t pa = reinterpret_cast<uint64_t>(src);
      const gu64* p0 = reinterpret_cast<const gu64*>(
          ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(pa >> 32)) << 32) |
          __builtin_amdgcn_readfirstlane((uint32_t)pa));
      for (;; spins++) {
        const uint64_t y =
            MC_CK_PUB(p0, 11) ? __hip_atomic_load(p0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0ull;
        if (__builtin_amdgcn_readfirstlane(mc_tag_state(y, tag, tlast)) >= 0 || spins > kMcPollSpins) break;
        if (lfail && __hip_atomic_load(lfail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
        __builtin_amdgcn_s_sleep(1);
      }
    }
#endif
  }
}

// waits for an LDS counter of the mc4 chain workgroup (bounded; false on a
// fail word or a timeout)
__device__ __forceinline__ bool mc4_wait(int* ctr, int target, int* lfail) {
  for (int spins = 0;; spins++) {
    if (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) >= target) return true;
    if (__hip_atomic_load(lfail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) return false;
    if (spins > kMcLdsSpins) {
      mc_set_fail(lfail, 2);
      return false;
    }
  }
}

// acc ^ sum over 8 terms of (tables of m[c]) x data whose selectors are
// precomputed (sp[c * ss] = {sel0, sel1, sel2, -}): three LDS reads and five
// VALU per term
__device__ __forceinline__ uint32_t mc4_dot8s(const uint4* tab, uint32_t acc, const uint32_t* m, const uint4* sp,
                                              int ss) {
  uint4 tt[8], sv[8];
  uint32_t t2[8];
#pragma unroll
  for (int c = 0; c < 8; c++) {
    tt[c] = tab[2 * m[c]];
    t2[c] = tab[2 * m[c] + 1].x;
    sv[c] = sp[c * ss];
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int c = 0; c < 8; c++) acc ^= gmul4(tt[c], t2[c], sv[c].x, sv[c].y, sv[c].z);
  return acc;
}
__device__ __forceinline__ uint4 mc4_sel(uint32_t v) { return make_uint4(sel0(v), sel1(v), sel2(v), 0u); }

// the chain's block update from precomputed selectors of S_{p-1} (ssel) and
// of R_{p-1}'s panel-p columns (rsel), both [16][4]
__device__ __forceinline__ uint32_t mc4_block_update_s(const uint4* tab, uint32_t blk, const uint32_t* mrow,
                                                       const uint4 (*ssel)[4], const uint4 (*rsel)[4], int lane) {
  const int d = lane & 3;
  uint32_t mw[4], m[16];
#pragma unroll
  for (int q = 0; q < 4; q++) mw[q] = mrow[q];
#pragma unroll
  for (int c = 0; c < 16; c++) m[c] = (mw[c >> 2] >> (8 * (c & 3))) & 0xffu;
  uint32_t F = mc4_dot8s(tab, 0u, m, &ssel[0][d], 4);
  F = mc4_dot8s(tab, F, m + 8, &ssel[8][d], 4);
  uint32_t fw[4];
#pragma unroll
  for (int q = 0; q < 4; q++) fw[q] = quad_bcast(F, q);
#pragma unroll
  for (int c = 0; c < 16; c++) m[c] = (fw[c >> 2] >> (8 * (c & 3))) & 0xffu;
  const uint32_t acc = mc4_dot8s(tab, blk, m, &rsel[0][d], 4);
  return mc4_dot8s(tab, acc, m + 8, &rsel[8][d], 4);
}

// RPW rows per row wave (4 waves per workgroup): 16 or 8 rows per row
// workgroup; gridDim.x = NP * 16 / (4 RPW) row workgroups + the chain
template <int RPW>
__global__ __launch_bounds__(kMc4Threads) void gf_elim_mc4_kernel(ElimArgs args) {
  __shared__ ElimMc4Lds lds;
  constexpr int RW = 4 * RPW;
  const int x = blockIdx.x, g = blockIdx.y, NRW = gridDim.x - 1, NP = NRW * RW / 16;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int k = args.k;
  const uint32_t tag0 = args.epoch, tlast = tag0 + kMcAttempts - 1;
  gu64* const pubS = (gu64*)args.pub + (size_t)g * mc4_pub_words(NP);  // then R and M slots (attempt)
  gu64* const pubA = (gu64*)args.pub + (size_t)gridDim.y * mc4_pub_words(NP) + g;  // the decoder's abort granule
  const bool chain = x == NRW;
#ifdef KODR_ELIM_TIMING
  // tuning build: s_memrealtime stamps by lane 0 into workgroup x's 1 KiB of
  // the T region (no result): chain [p] staged, [16 + p] block updated,
  // [32 + p] S_p out, staging wave [48 + p]; row workgroup [j] R_j / S_j in
  // LDS, [16 + j] apply(j) done; [96] entry, [97] tables in LDS
  gu64* const tsout = (gu64*)(args.out + (size_t)g * args.out_gen_stride + (size_t)x * 1024);
#define MC4_STAMP(i)                                                                                          \
  do {                                                                                                        \
    if (lane == 0)                                                                                            \
      __hip_atomic_store(tsout + (i), (unsigned long long)__builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,  \
                         __HIP_MEMORY_SCOPE_SYSTEM);                                                          \
  } while (0)
#else
#define MC4_STAMP(i) \
  do {               \
  } while (0)
#endif
  if (w == 0) MC4_STAMP(96);
  const uint64_t ab =
      tid == 0 && MC_CK_PUB(pubA, 7) ? __hip_atomic_load(pubA, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
#ifdef KODR_MC_CHECK
  if (!mc_in(args.tables + kElimInvTables + 4 * (256 * 2 - 1), 16, g_mcb.tab, g_mcb.tab_bytes)) mc_report(8, args.tables);
  if (!mc_in(&args.counts[g * (gridDim.x) + x], 4, g_mcb.cnt, g_mcb.cnt_bytes)) mc_report(10, &args.counts[g * gridDim.x + x]);
#endif
  for (int i = tid; i < 256 * 2; i += kMc4Threads) {
    const uint32_t* a = args.tables + 4 * i;
    lds.tab[i] = make_uint4(a[0], a[1], a[2], a[3]);
    if (chain) {
      const uint32_t* b = args.tables + kElimInvTables + 4 * i;
      lds.itab[i] = make_uint4(b[0], b[1], b[2], b[3]);
    }
  }
  if (tid == 0) lds.late = mc_tag_state(ab, tag0, tlast) == 2;
  __syncthreads();
  const bool late = __builtin_amdgcn_readfirstlane(lds.late) != 0;
  if (w == 0) MC4_STAMP(97);

  const int row0 = RW * x, pr = row0 / 16, lo = row0 - 16 * pr;  // row workgroup: its panel, offset in it
  uint32_t Tout[RPW];  // row workgroup: T rows of the successful attempt (assigned on the way out)
  int fail = late ? 2 : 0, att = 0;
  for (; !late; att++) {
    const uint32_t tag = tag0 + att;
    const int rot = mc_rot(att, k);
    if (tid == 0) {
      __hip_atomic_store(&lds.staged, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_store(&lds.consumed, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      __hip_atomic_store(&lds.fail, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    __syncthreads();
    // the attempt, on opaque copies of the indices (mc_opaque)
    auto attempt = [&](const int g, const int w, const int lane, gu64* const pubS) {
    gu64* const pubR = pubS + (size_t)NP * kMc4SGran;
    gu64* const pubM = pubR + (size_t)NP * kMc4RGran;
    int pfail = NP;  // chain wave 0: the first S_p not published
    uint32_t R[RPW];
#pragma unroll
    for (int i = 0; i < RPW; i++) R[i] = 0u;
    if (chain) {
      const int t = lane >> 2, d = lane & 3;
      if (w == 1) {
        // ---- staging wave: MB_p and R_{p-1}'s panel-p columns into LDS ----
        for (int p = 0; p < NP; p++) {
          const int slot = p & 1;
          if (p >= 2 && !mc4_wait(&lds.consumed, p - 1, &lds.fail)) break;  // the slot's last readers are done
          uint32_t v[2];
          int st = 0;
          // dword dw of row gr (rows past k: identity padding)
          auto orig = [&](int gr, int dw) -> uint32_t {
            if (gr >= k) return gr >> 2 == dw ? 1u << (8 * (gr & 3)) : 0u;
            const uint8_t* src = args.vecs[g] + (size_t)mc_src_row(gr, k, rot) * args.vpitch;
            if (!MC_CK(src, k, args.vecs[g], (uint64_t)(args.n[g] - 1) * args.vpitch + k, 9)) return 0u;
            uint32_t o = 0;
#pragma unroll
            for (int b = 0; b < 4; b++)
              if (4 * dw + b < k) o |= (uint32_t)src[4 * dw + b] << (8 * b);
            return o;
          };
          if (p == 0) {  // panels 0 and 1 start from the input rows ("as of -1"): no hand-off
            lds.cmb[slot][t][4 + d] = orig(t, d);
          } else if (p == 1) {
            lds.cmb[slot][t][d] = orig(16 + t, d);
            lds.cmb[slot][t][4 + d] = orig(16 + t, 4 + d);
            const uint32_t rq = orig(t, 4 + d);
            lds.crq[slot][t][d] = rq;
            lds.crsel[slot][t][d] = mc4_sel(rq);
          } else {
            const gu64* mb = pubM + (size_t)p * kMc4MGran + t * 8 + d;
            st = mc4_poll<2>(mb, 4, tag, tlast, v, &lds.fail);
            if (st == 0) {
              lds.cmb[slot][t][d] = v[0];
              lds.cmb[slot][t][4 + d] = v[1];
              st = mc4_poll<1>(pubR + (size_t)(p - 1) * kMc4RGran + t * 64 + 4 * p + d, 0, tag, tlast, v,
                               &lds.fail);
              if (st == 0) {
                lds.crq[slot][t][d] = v[0];
                lds.crsel[slot][t][d] = mc4_sel(v[0]);
              }
            }
          }
          if (st) {
            mc_set_fail(&lds.fail, st);
            break;
          }
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
          if (lane == 0) __hip_atomic_store(&lds.staged, p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          MC4_STAMP(48 + p);
        }
      } else if (w == 0) {
        // ---- wave 0: update the block, invert it, publish S_p ----
        __builtin_amdgcn_s_setprio(3);
        int p = 0;
        for (; p < NP; p++) {
          const int slot = p & 1;
          if (!mc4_wait(&lds.staged, p + 1, &lds.fail)) break;
          MC4_STAMP(p);
          uint32_t blk = lds.cmb[slot][t][4 + d];
          if (p >= 1)
            blk = mc4_block_update_s(lds.tab, blk, lds.cmb[slot][t], lds.csel[slot ^ 1], lds.crsel[slot], lane);
          MC4_STAMP(16 + p);
          uint32_t sval = 0;
          int srow = 0;
          if (!mc3_gj(lds.tab, lds.itab, blk, lane, &sval, &srow)) {
            mc_set_fail(&lds.fail, mc_singular_why(blk, lane, p, k));
            break;
          }
          mc_put(pubS + (size_t)p * kMc4SGran + 4 * srow + d, tag, sval);
          lds.csel[slot][srow][d] = mc4_sel(sval);
          MC4_STAMP(32 + p);
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
          if (lane == 0) __hip_atomic_store(&lds.consumed, p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
        pfail = p;
        __builtin_amdgcn_s_setprio(0);
      }
    } else {
      // ================= row workgroup x: rows RW x + RPW w + i =================
#pragma unroll
      for (int i = 0; i < RPW; i++) R[i] = mc_load_row(args, g, row0 + RPW * w + i, rot, lane);
      // what the workgroup owes after apply(j) (j = -1: the loaded rows)
      auto publish = [&](int j) {
        const int lr = lo + RPW * w;  // local row (in the panel) of R[0]
        if (pr == j + 1) {  // R_pr: the panel's rows as of pr - 1
          gu64* dst = pubR + (size_t)pr * kMc4RGran + lr * 64 + lane;
#pragma unroll
          for (int i = 0; i < RPW; i++) mc_put(dst + i * 64, tag, R[i]);
        }
        if (pr == j + 2) {  // MB_pr: columns of panels pr - 1 and pr as of pr - 2
          const int u = lane - 4 * (pr - 1);
          if (u >= 0 && u < 8) {
            gu64* dst = pubM + (size_t)pr * kMc4MGran + lr * 8 + u;
#pragma unroll
            for (int i = 0; i < RPW; i++) mc_put(dst + i * 8, tag, R[i]);
          }
        }
      };
      publish(-1);
      for (int j = 0; j < NP; j++) {
        // R_j (all 16 rows, from the hand-off slots, this workgroup's own
        // included) and S_j into LDS: wave w polls rows 4 w .. 4 w + 3, wave 0 S_j
        {
          uint32_t v[4];
          const int st =
              mc4_poll<4>(pubR + (size_t)j * kMc4RGran + (4 * w) * 64 + lane, 64, tag, tlast, v, &lds.fail);
          if (st) {
            mc_set_fail(&lds.fail, st);
          } else {
#pragma unroll
            for (int i = 0; i < 4; i++) lds.rp[4 * w + i][lane] = v[i];
          }
        }
        if (w == 0) {
          uint32_t v[1];
          const int st = mc4_poll<1>(pubS + (size_t)j * kMc4SGran + lane, 0, tag, tlast, v, &lds.fail);
          if (st)
            mc_set_fail(&lds.fail, st);
          else
            lds.sp[lane >> 2][lane & 3] = v[0];
        }
        __syncthreads();
        if (__hip_atomic_load(&lds.fail, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
        if (w == 0) MC4_STAMP(j);
        // apply(j): the panel's own rows become S_j x R_j with S_j in the panel
        // columns; the others take F = (panel-j bytes) x S_j, row ^= F x R_j,
        // panel columns := F
        const int db = 4 * j;
        const bool own = pr == j;
        const uint32_t(*Gp)[4] = own ? &lds.sp[lo + RPW * w] : lds.fw[w];
        if (!own) {
          // F of the RPW rows: lane (cg, i, u) sums terms c in group cg (16 / G
          // of them), the G groups folded by ds_bpermute
          constexpr int G = 16 / RPW, TPG = 16 / G;  // groups, terms per group
          if (lane >= db && lane < db + 4)
#pragma unroll
            for (int i = 0; i < RPW; i++) lds.mw[w][i][lane - db] = R[i];
          __builtin_amdgcn_s_waitcnt(0xc07f);
          const int u = lane & 3, i = (lane >> 2) % RPW, cg = (lane >> 2) / RPW;
          uint32_t acc = 0;
#pragma unroll
          for (int cc = 0; cc < TPG; cc++) {
            const int c = TPG * cg + cc;
            const uint32_t m = (lds.mw[w][i][c >> 2] >> (8 * (c & 3))) & 0xffu;
            const uint4 tt = lds.tab[2 * m];
            const uint32_t tt2 = lds.tab[2 * m + 1].x;
            const uint32_t xv = lds.sp[c][u];
            acc ^= gmul4(tt, tt2, sel0(xv), sel1(xv), sel2(xv));
          }
#pragma unroll
          for (int sft = 4 * RPW; sft < 64; sft <<= 1) acc ^= bperm(acc, lane ^ sft);
          if (lane < 4 * RPW) lds.fw[w][i][u] = acc;
          __builtin_amdgcn_s_waitcnt(0xc07f);
        }
        uint32_t acc[RPW];
#pragma unroll
        for (int i = 0; i < RPW; i++) acc[i] = own ? 0u : R[i];
#pragma unroll
        for (int cq = 0; cq < 4; cq++) {
          uint32_t gw[RPW];
#pragma unroll
          for (int i = 0; i < RPW; i++) gw[i] = __builtin_amdgcn_readfirstlane(Gp[i][cq]);
          uint4 tt[4][RPW];
          uint32_t t2[4][RPW], xs[4];
#pragma unroll
          for (int cc = 0; cc < 4; cc++) {
            xs[cc] = lds.rp[4 * cq + cc][lane];
#pragma unroll
            for (int i = 0; i < RPW; i++) {
              const uint32_t f = (gw[i] >> (8 * cc)) & 0xffu;
              tt[cc][i] = lds.tab[2 * f];
              t2[cc][i] = lds.tab[2 * f + 1].x;
            }
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int cc = 0; cc < 4; cc++) {
            const uint32_t s0 = sel0(xs[cc]), s1 = sel1(xs[cc]), s2 = sel2(xs[cc]);
#pragma unroll
            for (int i = 0; i < RPW; i++) acc[i] ^= mc_mul(tt[cc][i], t2[cc][i], s0, s1, s2);
          }
        }
        const int u = lane - db;
#pragma unroll
        for (int i = 0; i < RPW; i++) R[i] = (u >= 0 && u < 4) ? Gp[i][u & 3] : acc[i];
        publish(j);
        if (w == 0) MC4_STAMP(16 + j);
        __syncthreads();  // rp / sp / mw / fw are rewritten next iteration
      }
    }
    __syncthreads();
    fail = lds.fail;
#ifdef KODR_ELIM_TIMING
    if (!fail) fail = 2;  // the stamps overwrote T: report failure, kodr's route on the host
#endif
    if (fail) {
      if (chain) {
        // every S_p not out yet (an abort: all of them), so that every row workgroup stops
        if (w == 0)
          for (int p = fail >= 2 ? 0 : pfail; p < NP; p++) mc_put_fail(pubS + (size_t)p * kMc4SGran + lane, tag, tlast, fail);
      } else {
        // every slot this workgroup owes (or has put) gets FAIL, so its consumers stop
        const int lr = lo + RPW * w;
        for (int i = 0; i < RPW; i++)
          mc_put_fail(pubR + (size_t)pr * kMc4RGran + (lr + i) * 64 + lane, tag, tlast, fail);
        if (pr >= 1 && lane < 8)
          for (int i = 0; i < RPW; i++) mc_put_fail(pubM + (size_t)pr * kMc4MGran + (lr + i) * 8 + lane, tag, tlast, fail);
      }
      // the FAILs reach L2 before any store of the next attempt to the same slots
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    }
    if (!fail && !chain) {
      // T = T' Pi: the rotation undone (lds.rp is free after the last barrier)
      uint8_t* out = args.out + (size_t)g * args.out_gen_stride;
#pragma unroll
      for (int i = 0; i < RPW; i++) {
        Tout[i] = rot ? mc_unrotate(R[i], &lds.rp[w][0], lane, k, rot) : R[i];
        const int gr = row0 + RPW * w + i;
        if (gr < k) mc_store_row(out + (size_t)gr * args.out_pitch, Tout[i], lane, k);
      }
    }
    };
    attempt(mc_opaque_s(g), mc_opaque_s(w), mc_opaque(lane), mc_opaque_s(pubS));
    __syncthreads();  // every wave read lds.fail before the next attempt resets it
    if (fail != 1 || att + 1 == kMcAttempts) break;
  }
  const bool ok = fail == 0;
  if (!ok && tid == 0) mc_put_fail(pubA, tag0, tlast, 2);  // late workgroups read no input
  __atomic_thread_fence(__ATOMIC_RELEASE);  // this wave's T rows reach (host) memory first
  __syncthreads();
  if (tid == 0) {
    const uint32_t tg = late ? tlast : tag0 + att;
    __atomic_thread_fence(__ATOMIC_RELEASE);
    __hip_atomic_store(&args.counts[g * (NRW + 1) + x], (int)(ok ? tg : tg | kMcFail), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // the device copy of T after the system-scope releases: written before
  // them, its dirty lines made every wave's release write back L2 (mc2 with
  // 16 decoders 280 -> 890 us); later kernels see it at the launch boundary
  if (ok && !chain && args.out_dev)
#pragma unroll
    for (int i = 0; i < RPW; i++) {
      const int gr = row0 + RPW * w + i;
      if (gr < k) mc_store_row(args.out_dev + ((size_t)g * k + gr) * k, Tout[i], lane, k);
    }
#undef MC4_STAMP
}

}  // namespace

void elim_tables(uint32_t* host_out) {
  // [256][8] dwords: T0 = f*{0..7}, T1 = f*({0..7} << 3), T2 = f*({0..3} << 6)
  // as little-endian byte tables for v_perm (lo dword = entries 0..3); then
  // the 256 inverse bytes (gf256.go:77-86; inv(0) unused)
  auto mul = [](unsigned a, unsigned b) {
    unsigned r = 0;
    while (b) {
      if (b & 1) r ^= a;
      a <<= 1;
      if (a & 0x100) a ^= 0x11D;
      b >>= 1;
    }
    return r;
  };
  for (unsigned f = 0; f < 256; f++) {
    uint8_t t[20] = {};
    for (unsigned i = 0; i < 8; i++) {
      t[i] = (uint8_t)mul(f, i);
      t[8 + i] = (uint8_t)mul(f, i << 3);
    }
    for (unsigned i = 0; i < 4; i++) t[16 + i] = (uint8_t)mul(f, i << 6);
    for (int q = 0; q < 8; q++) {
      uint32_t v = 0;
      if (q < 5)
        for (int b = 0; b < 4; b++) v |= (uint32_t)t[q * 4 + b] << (8 * b);
      host_out[f * 8 + q] = v;
    }
  }
  uint8_t inv[256] = {};
  for (unsigned a = 1; a < 256; a++)
    for (unsigned b = 1; b < 256; b++)
      if (mul(a, b) == 1) {
        inv[a] = (uint8_t)b;
        break;
      }
  for (int i = 0; i < 64; i++)
    host_out[256 * 8 + i] = (uint32_t)inv[4 * i] | ((uint32_t)inv[4 * i + 1] << 8) |
                            ((uint32_t)inv[4 * i + 2] << 16) | ((uint32_t)inv[4 * i + 3] << 24);
  // tables of inv(f), so a pivot's normalization is one dependent load
  for (unsigned f = 0; f < 256; f++)
    for (int q = 0; q < 8; q++) host_out[kElimInvTables + f * 8 + q] = f ? host_out[inv[f] * 8 + q] : 0u;
}

bool gf_elim_blocked(const ElimArgs& args, int G) {
  // every batch full (n >= k) and k large enough for panels to pay
  bool full = args.k >= kElimBlockedMinK;
  for (int i = 0; i < G && full; i++) full = args.n[i] >= args.k;
  if (const char* e = tune_env("KODR_ELIM_BLOCKED")) full = full && atoi(e) != 0;  // A/B measurements
  return full;
}

// KODR_ELIM_MC: 0 one workgroup per decoder, 2 mc2, 4 mc4, 3 (default) mc4
// when the launch's decoders fit it
// (G * groups <= kElimMcMaxBlocks: one decoder at k = 256 takes 33
// workgroups) else mc2 (measured: profiles/r04/elim_modes/)
static int elim_mc_mode() {
  static const int mc = [] {
    const int m = tune_env("KODR_ELIM_MC") ? atoi(tune_env("KODR_ELIM_MC")) : 3;
    return m == 0 || m == 2 || m == 4 ? m : 3;
  }();
  return mc;
}

// mc4 rows per row wave (KODR_MC4_RPW: 4 = 16 rows per row workgroup, 2
// (default) = 8)
static int mc4_rows_per_wave() {
  static const int rpw = tune_env("KODR_MC4_RPW") && atoi(tune_env("KODR_MC4_RPW")) == 4 ? 4 : 2;
  return rpw;
}
static int mc4_groups(int k) { return (k + 15) / 16 * (16 / (4 * mc4_rows_per_wave())) + 1; }
static int mc2_groups(int k) { return (k + 31) / 32; }

// the multi-workgroup kernel a launch of G decoders takes (0: none)
static int mc_kernel_for(int k, int G) {
  const int m = elim_mc_mode();
  if (m == 3) return G * mc4_groups(k) <= kElimMcMaxBlocks ? 4 : 2;
  return m;
}

int gf_elim_mc_groups(int k, int G) { return mc_kernel_for(k, G) == 4 ? mc4_groups(k) : mc2_groups(k); }

int gf_elim_mc_max_gens(int k) { return std::max(1, kElimMcMaxBlocks / mc2_groups(k)); }

bool gf_elim_mc_taken(const ElimArgs& args, int G) {
  return elim_mc_mode() && args.pub && args.epoch && args.epoch < kMcFail && gf_elim_blocked(args, G) &&
         G * gf_elim_mc_groups(args.k, G) <= kElimMcMaxBlocks;
}

bool gf_elim_mc_enabled() { return elim_mc_mode() != 0; }

bool gf_elim_mc_direct(const ElimArgs& args, int G) {
  const int m = mc_kernel_for(args.k, G);
  return gf_elim_mc_taken(args, G) && (m == 2 || m == 4);
}

// the hand-off granules of G decoders, then one abort granule per decoder
size_t gf_elim_mc_pub_bytes(int k, int G) {
  if (mc_kernel_for(k, G) == 4)
    return ((size_t)G * (size_t)((k + 15) / 16) * (kMc4SGran + kMc4RGran + kMc4MGran) + (size_t)G) * 8;
  const size_t P = (size_t)mc2_groups(k);
  return ((size_t)G * 2 * P * kMc2PanelGran + (size_t)G) * 8;
}
int gf_elim_mc_attempts() { return kMcAttempts; }

#ifdef KODR_MC_CHECK
// the allocation that holds p (hipMemGetAddressRange), else [p, p + fallback)
static void mc_alloc_range(const void* p, size_t fallback, const uint8_t** base, uint64_t* bytes) {
  hipDeviceptr_t b = nullptr;
  size_t n = 0;
  if (p && hipMemGetAddressRange(&b, &n, (hipDeviceptr_t)p) == hipSuccess && b) {
    *base = reinterpret_cast<const uint8_t*>(b);
    *bytes = n;
  } else {
    (void)hipGetLastError();
    *base = reinterpret_cast<const uint8_t*>(p);
    *bytes = p ? fallback : 0;
  }
}
#endif

hipError_t gf_elim(const ElimArgs& args, int G, hipStream_t stream) {
  if (G <= 0) return hipSuccess;
  if (G <= kElimMaxGens && args.k >= 2 && args.k <= 256 && gf_elim_mc_taken(args, G)) {
    const int m = mc_kernel_for(args.k, G);
    const dim3 grid(gf_elim_mc_groups(args.k, G), G);
#ifdef KODR_MC_CHECK
    {  // the launch's bounds: the hand-off layout the host sized, the real allocations of the rest
      McBounds mb = {};
      mb.pub = reinterpret_cast<const uint8_t*>(args.pub);
      mb.pub_bytes = gf_elim_mc_pub_bytes(args.k, G);
      const size_t k = (size_t)args.k;
      mc_alloc_range(args.out, (size_t)G * k * k, &mb.out, &mb.out_bytes);
      mc_alloc_range(args.counts, 4 * (size_t)kElimMcMaxBlocks, &mb.cnt, &mb.cnt_bytes);
      mc_alloc_range(args.out_dev, (size_t)G * k * k, &mb.odev, &mb.odev_bytes);
      mc_alloc_range(args.tables, kElimTableWords * 4, &mb.tab, &mb.tab_bytes);
      fprintf(stderr, "KODR_MC_CHECK launch mc%d G %d grid %d x %d: pub %p+%lu out %p+%lu cnt %p+%lu odev %p+%lu\n", m,
              G, (int)grid.x, (int)grid.y, (const void*)mb.pub, (unsigned long)mb.pub_bytes, (const void*)mb.out,
              (unsigned long)mb.out_bytes, (const void*)mb.cnt, (unsigned long)mb.cnt_bytes, (const void*)mb.odev,
              (unsigned long)mb.odev_bytes);
      const hipError_t e = hipMemcpyToSymbolAsync(HIP_SYMBOL(g_mcb), &mb, sizeof(mb), 0, hipMemcpyHostToDevice, stream);
      if (e != hipSuccess) return e;
      (void)hipStreamSynchronize(stream);  // (mb is on this stack frame)
    }
#endif
    if (m == 4) {
      if (!args.direct) return hipErrorInvalidValue;  // mc4 reports directly only
#ifdef KODR_TUNE
      if (mc4_rows_per_wave() == 4)
        hipLaunchKernelGGL(gf_elim_mc4_kernel<4>, grid, dim3(kMc4Threads), 0, stream, args);
      else
#endif
        hipLaunchKernelGGL(gf_elim_mc4_kernel<2>, grid, dim3(kMc4Threads), 0, stream, args);
    } else {
      hipLaunchKernelGGL(gf_elim_mc2_kernel, grid, dim3(1024), 0, stream, args);
    }
    return hipGetLastError();
  }
  if (G > kElimMaxGens || args.k < 2 || args.k > 256 || args.out_pitch % 4 ||
      args.out_pitch < (size_t)(args.k <= 128 ? 256 : 512))
    return hipErrorInvalidValue;
  const bool full = gf_elim_blocked(args, G);
  // (a panel step with DPP/readlane broadcasts instead of ds_bpermute measured
  // slower: 520 vs 493 us at k = 256, profiles/r02/elim/elim_gj_ab.log)
  // (a row-per-lane layout of the same algorithm -- one LDS gather per
  // multiplier serving 64 rows, pivot rows as scalars -- measured slower too:
  // 536 vs 493 us at k = 256, profiles/r02/elim/elim_rows_ab.log)
  static const int circ = tune_env("KODR_ELIM_CIRC") ? atoi(tune_env("KODR_ELIM_CIRC")) : 1;
  if (full && circ)
    hipLaunchKernelGGL(gf_elim_circ_kernel, dim3(G), dim3(64 * kElimWaves), 0, stream, args);
  else if (full && args.k <= 128)
    hipLaunchKernelGGL(gf_elim_blocked_kernel<1>, dim3(G), dim3(64 * kElimWaves), 0, stream, args);
  else if (full)
    hipLaunchKernelGGL(gf_elim_blocked_kernel<2>, dim3(G), dim3(64 * kElimWaves), 0, stream, args);
  else if (args.k <= 128)
    hipLaunchKernelGGL(gf_elim_kernel<1>, dim3(G), dim3(64 * kElimWaves), 0, stream, args);
  else
    hipLaunchKernelGGL(gf_elim_kernel<2>, dim3(G), dim3(64 * kElimWaves), 0, stream, args);
  return hipGetLastError();
}

}  // namespace kodr_amd
