// gf_bs.hip -- bit-sliced GF(2^8) product for gfx950: Y = A (x) X with X held
// in bit-sliced blocks (see DESIGN.md "Bit-sliced kernel").
//
// Layout.  X rows are cut into 32-byte blocks; bitslice32 turns a block's 8
// dwords into 8 planes, plane i = bit i of all 32 bytes (it is an involution,
// so the same transform converts back).  In that layout multiplying by a
// coefficient c is GF(2)-linear on the planes: out plane j = XOR of the input
// planes i with bit j of c*2^i set (gf256.go:15-44, poly 0x11D).  Per input
// row the wave tabulates the XORs of every subset of planes 0-3 and of planes
// 4-7 (30 registers, 26 VALU shared by 8 output rows); then each output plane
// is one XOR3, at most 8 instructions per coefficient per 32 bytes, against 36
// for the 3x v_perm lookup formulation of gf_gemm_kernel.
//
// Code.  The XOR pattern depends on c, which is wave-uniform, so each of the
// 256 patterns is a straight-line body (generated: gen_bs_bodies.py).  The
// bodies are threaded: 4 copies, copy r XORing into accumulator set r and
// ending with a jump to the next output row's body, so the 8 coefficients of
// an input row cost 8 bodies and one taken branch each (rows 4..7 reuse the
// copies under VGPR index mode).  They live in gf_bs_export_kernel, which
// exports their addresses once; no LDS tables, no lookups, no per-lane
// branches.
//
// Work split.  A wave owns 8 output rows x 64 blocks (2 KiB of columns) x a
// range of at most rpw input rows; the KW waves of a workgroup split K and are
// XOR-reduced in LDS.  Per wave, the absolute body targets for its (row, k)
// pairs are built once into LDS ("program") and moved to SGPRs with
// v_readlane within the row.  X rows stream through a P-deep register ring of
// buffer loads (rows past the wave's range are outside num_records and read
// as zero); the first P are in flight while the program is built.  Each input
// row starts with s_setprio (row mod 4) so the 4 waves of a SIMD take turns
// instead of finishing oldest-first.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdlib.h>

#include <algorithm>
#include <mutex>

#include "gf_device.hpp"
#include "gf_kernels.hpp"
// generated: bodies, row loop, register map (gen_bs_bodies.py)
#include "gf_bs_bodies.inc"
#include "tune.hpp"

namespace kodr_amd {

namespace {

constexpr int kBsRows = 8;     // output rows per wave
constexpr int kBsBlock = 32;   // bytes per bit-sliced block
constexpr int kBsWaveCols = 64 * kBsBlock;
constexpr int kBsChunk = 8;    // input rows per program chunk (one VGPR of targets)

// 8x8 bit-matrix transpose inside each byte lane of 8 dwords: afterwards
// dword i holds bit i of all 32 bytes.  Self-inverse.
__device__ __forceinline__ void bitslice32(uint32_t (&d)[8]) {
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const uint32_t t = ((d[q] >> 4) ^ d[q + 4]) & 0x0F0F0F0Fu;
    d[q + 4] ^= t;
    d[q] ^= t << 4;
  }
#pragma unroll
  for (int q = 0; q < 8; q++) {
    if (q & 2) continue;
    const uint32_t t = ((d[q] >> 2) ^ d[q + 2]) & 0x33333333u;
    d[q + 2] ^= t;
    d[q] ^= t << 2;
  }
#pragma unroll
  for (int q = 0; q < 8; q += 2) {
    const uint32_t t = ((d[q] >> 1) ^ d[q + 1]) & 0x55555555u;
    d[q + 1] ^= t;
    d[q] ^= t << 1;
  }
}

// src may equal dst (in place): each thread reads its block before writing it
__global__ __launch_bounds__(256) void bitslice_kernel(const uint8_t* src, uint8_t* dst, size_t ldx, int rows,
                                                      int nblk) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const int r = (int)(i / (size_t)nblk), b = (int)(i % (size_t)nblk);
  if (r >= rows) return;
  const size_t off = (size_t)r * ldx + (size_t)b * kBsBlock;
  const uint4* q = reinterpret_cast<const uint4*>(src + off);
  uint4* p = reinterpret_cast<uint4*>(dst + off);
  const uint4 a = q[0], c = q[1];
  uint32_t d[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
  bitslice32(d);
  p[0] = make_uint4(d[0], d[1], d[2], d[3]);
  p[1] = make_uint4(d[4], d[5], d[6], d[7]);
}

// bitslice_kernel with separate source and destination pitches (the piece
// columns of a recoder's wire rows into a twin of their own)
__global__ __launch_bounds__(256) void bitslice_pitched_kernel(const uint8_t* __restrict__ src, size_t spitch,
                                                              uint8_t* __restrict__ dst, size_t dpitch, int rows,
                                                              int nblk) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const int r = (int)(i / (size_t)nblk), b = (int)(i % (size_t)nblk);
  if (r >= rows) return;
  const uint4* q = reinterpret_cast<const uint4*>(src + (size_t)r * spitch + (size_t)b * kBsBlock);
  const uint4 a = q[0], c = q[1];
  uint32_t d[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
  bitslice32(d);
  uint4* p = reinterpret_cast<uint4*>(dst + (size_t)r * dpitch + (size_t)b * kBsBlock);
  p[0] = make_uint4(d[0], d[1], d[2], d[3]);
  p[1] = make_uint4(d[4], d[5], d[6], d[7]);
}

// dst row r = src row r (bytes [0, nblk * 32)), and dst_bs row r = its
// bit-sliced form: one read of the source for both, for the decoder's
// received rows (plain rows for the GetPiece paths, the twin for T x R);
// dst == nullptr writes the twin only (a compact decoder's rows).
// src, spitch, dpitch: multiples of 16 (checked by the host).
__global__ __launch_bounds__(256) void copy_bitslice_kernel(const uint8_t* __restrict__ src, size_t spitch,
                                                           uint8_t* __restrict__ dst, uint8_t* __restrict__ dst_bs,
                                                           size_t dpitch, int rows, int nblk) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const int r = (int)(i / (size_t)nblk), b = (int)(i % (size_t)nblk);
  if (r >= rows) return;
  const uint4* q = reinterpret_cast<const uint4*>(src + (size_t)r * spitch + (size_t)b * kBsBlock);
  const size_t off = (size_t)r * dpitch + (size_t)b * kBsBlock;
  const uint4 a = q[0], c = q[1];
  if (dst) {
    uint4* p = reinterpret_cast<uint4*>(dst + off);
    p[0] = a;
    p[1] = c;
  }
  uint32_t d[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
  bitslice32(d);
  uint4* t = reinterpret_cast<uint4*>(dst_bs + off);
  t[0] = make_uint4(d[0], d[1], d[2], d[3]);
  t[1] = make_uint4(d[4], d[5], d[6], d[7]);
}

// copy_bitslice_kernel over several row sets at once (blockIdx.y = set), two
// lanes per 32-byte block: lane pair (2j, 2j + 1) reads and writes its
// block's halves (16 bytes per lane, contiguous over the wave: one 1 KiB
// request per instruction instead of two half-used ones) and swaps them by
// DPP; each lane then computes only the four planes it stores
// (bitslice32_half: the first butterfly stage pairs dwords across the halves,
// the other two stay inside one).  Grid-stride over a capped grid
// (copy_bitslice_rows_grouped): the copies run beside the elimination kernel,
// whose workgroups must find free wave slots even when the copies reach the
// CUs first (a grid of one lane per half-block filled every CU, and the
// elimination's workgroups waited behind it).  The copy is bound by what one
// CU moves (~23 GB/s per CU alone and beside the elimination), so its VALU
// work per byte counts: no division per item (the row and half-block advance
// by the grid stride's quotient and remainder), half the butterfly per lane.
constexpr int kCopyUnroll = 4;
// The copy streams its rows and the twin past the caches (nontemporal loads
// and stores: nothing of either is read again before it has left L2), so
// beside the pipelined encode it leaves the encode's column chunks in L2:
// the AddPiece leg alone 362-370 against 371-384 us, the pipelined step
// 3.336-3.350 against 3.342-3.356 ms (tools/gpu_r6_m.sh, profiles/r06/copy_nt/).
// KODR_COPY_NT=0 builds the cached variant (A/B).
#ifndef KODR_COPY_NT
#define KODR_COPY_NT 1
#endif
typedef uint32_t cp_u32x4 __attribute__((ext_vector_type(4)));

// one 32-byte block of a product's output rows.  KODR_BS_NT_STORE=1 streams
// them past the caches: measured no faster (3.312-3.317 against 3.305-3.317 ms
// per round-trip step), and the twin copy that reads the encode's rows next
// then takes them from HBM (tools/gpu_r6_n.sh, profiles/r06/store_nt/)
#ifndef KODR_BS_NT_STORE
#define KODR_BS_NT_STORE 0
#endif
__device__ __forceinline__ void bs_store32(uint8_t* dst, const uint4& v0, const uint4& v1) {
#if KODR_BS_NT_STORE
  __builtin_nontemporal_store(cp_u32x4{v0.x, v0.y, v0.z, v0.w}, reinterpret_cast<cp_u32x4*>(dst));
  __builtin_nontemporal_store(cp_u32x4{v1.x, v1.y, v1.z, v1.w}, reinterpret_cast<cp_u32x4*>(dst) + 1);
#else
  reinterpret_cast<uint4*>(dst)[0] = v0;
  reinterpret_cast<uint4*>(dst)[1] = v1;
#endif
}

// planes of the 32-byte block whose dwords d[0..3] are in the lower lane of a
// pair and d[4..7] in the upper one: h = this lane's four, p = the partner's;
// on return h = planes 0..3 (lower lane) or 4..7 (upper), as bitslice32 leaves
// d[0..3] / d[4..7]
__device__ __forceinline__ void bitslice32_half(uint32_t (&h)[4], const uint32_t (&p)[4], bool lo) {
#pragma unroll
  for (int q = 0; q < 4; q++) {  // (q, q + 4)
    const uint32_t a = lo ? h[q] : p[q], b = lo ? p[q] : h[q];
    const uint32_t t = ((a >> 4) ^ b) & 0x0F0F0F0Fu;
    h[q] = lo ? a ^ (t << 4) : b ^ t;
  }
#pragma unroll
  for (int q = 0; q < 2; q++) {  // (q, q + 2)
    const uint32_t t = ((h[q] >> 2) ^ h[q + 2]) & 0x33333333u;
    h[q + 2] ^= t;
    h[q] ^= t << 2;
  }
#pragma unroll
  for (int q = 0; q < 4; q += 2) {  // (q, q + 1)
    const uint32_t t = ((h[q] >> 1) ^ h[q + 1]) & 0x55555555u;
    h[q + 1] ^= t;
    h[q] ^= t << 1;
  }
}

__device__ __forceinline__ void copy_bs_pair(const CopyGroup& g, int y, uint32_t r, uint32_t hi, size_t dpitch,
                                             const uint4& a) {
  const uint32_t p[4] = {(uint32_t)__builtin_amdgcn_mov_dpp((int)a.x, 0xb1, 0xf, 0xf, false),
                         (uint32_t)__builtin_amdgcn_mov_dpp((int)a.y, 0xb1, 0xf, 0xf, false),
                         (uint32_t)__builtin_amdgcn_mov_dpp((int)a.z, 0xb1, 0xf, 0xf, false),
                         (uint32_t)__builtin_amdgcn_mov_dpp((int)a.w, 0xb1, 0xf, 0xf, false)};
  const size_t off = (size_t)r * dpitch + (size_t)hi * 16;
  uint32_t h[4] = {a.x, a.y, a.z, a.w};
  bitslice32_half(h, p, (hi & 1) == 0);
#if KODR_COPY_NT
  if (g.dst[y]) __builtin_nontemporal_store(cp_u32x4{a.x, a.y, a.z, a.w}, reinterpret_cast<cp_u32x4*>(g.dst[y] + off));
  __builtin_nontemporal_store(cp_u32x4{h[0], h[1], h[2], h[3]}, reinterpret_cast<cp_u32x4*>(g.dbs[y] + off));
#else
  if (g.dst[y]) *reinterpret_cast<uint4*>(g.dst[y] + off) = a;  // (null: twin only)
  *reinterpret_cast<uint4*>(g.dbs[y] + off) = make_uint4(h[0], h[1], h[2], h[3]);
#endif
}

__global__ __launch_bounds__(256) void copy_bitslice_grouped_kernel(CopyGroup g, size_t spitch, size_t dpitch,
                                                                   int nblk) {
  const int y = blockIdx.y;
  const uint32_t hb = (uint32_t)nblk * 2;  // half-blocks per row (< 2^31: copy_bitslice_ok)
  const uint32_t rows = (uint32_t)g.rows[y];
  const size_t stride = (size_t)gridDim.x * 256;
  // item i = (row r, half-block h) = (i / hb, i % hb); a step of `stride`
  // items adds (sr, sh) with a carry
  const uint32_t sr = (uint32_t)(stride / hb), sh = (uint32_t)(stride % hb);
  const size_t i0 = (size_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t r = (uint32_t)(i0 / hb), h = (uint32_t)(i0 % hb);
  const auto step = [&](uint32_t& rr, uint32_t& hh) {
    hh += sh;
    rr += sr;
    if (hh >= hb) {
      hh -= hb;
      rr++;
    }
  };
  // kCopyUnroll half-blocks per lane per trip, every load in flight before
  // the stores (the capped grid holds fewer loads in flight than one lane
  // per half-block did); rows is even per pair: a lane pair is live or done
  // together (hb is even)
  constexpr int U = kCopyUnroll;
  while (r < rows) {
    uint32_t ru[U], hu[U];
    uint4 a[U];
    uint32_t rr = r, hh = h;
#pragma unroll
    for (int u = 0; u < U; u++) {
      ru[u] = rr;
      hu[u] = hh;
      a[u] = make_uint4(0u, 0u, 0u, 0u);
#if KODR_COPY_NT
      if (rr < rows) {
        const cp_u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const cp_u32x4*>(g.src[y] + (size_t)rr * spitch + (size_t)hh * 16));
        a[u] = make_uint4(v.x, v.y, v.z, v.w);
      }
#else
      if (rr < rows) a[u] = *reinterpret_cast<const uint4*>(g.src[y] + (size_t)rr * spitch + (size_t)hh * 16);
#endif
      step(rr, hh);
    }
#pragma unroll
    for (int u = 0; u < U; u++)
      if (ru[u] < rows) copy_bs_pair(g, y, ru[u], hu[u], dpitch, a[u]);
    r = rr;
    h = hh;
  }
}

// The bodies' only home: this kernel exports the absolute address of body
// (0, 0) and every body's offset from it (out[i] for body i = copy * 256 + c,
// out[1024] lo, out[1025] hi) and never runs them; gf_bs_kernel jumps here.
__global__ __launch_bounds__(64) void gf_bs_export_kernel(uint32_t* out) {
  asm volatile(
      "s_branch .Lexp_%=\n\t"
      KODR_BS_BODIES
      ".Lexp_%=:\n\t"
      KODR_BS_EXPORT("v24", "%[z]", "v25", "%[out]")
      :
      : [z] "v"(0u), [out] "s"(out)
      : "v24", "v25", "s88", "s89", "memory");
}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x8 __attribute__((ext_vector_type(8)));

// MODE (tuning builds only, -DKODR_TUNE_MODES): 3 = the row stream, table
// prep and program reads without dispatching bodies, 4 = as 3 without the
// row stream, 5 = no main loop (prologue, reduction and store only), 6 = the
// full loop without the row stream (stale rows), 8 = s_memtime timeline,
// 9 = register dump before the first jump.
#ifdef KODR_TUNE_MODES
__device__ uint32_t* g_bs_prog = nullptr;  // MODE 14's program scratch (tuning builds only)
#endif

// Products of one shape over several resident generations in one launch
// (GRP): blockIdx.y = generation g reads X = x[g], A + g * a_stride and
// writes Y + g * y_stride.
struct BsGroupK {
  const uint8_t* x[kGemmGroupMax];
  size_t a_stride, y_stride;
};

// Side product of a single launch (BsSideK, ncols > 0): Y2 = A x X2 over
// plain rows X2 of a few hundred columns -- the recoded coding vectors r x C
// next to the recoded pieces (full/recoder.go:32-40), otherwise a gf_gemm
// launch of their own (~5 us at B = 32).  The work is spread over every
// workgroup of the launch, so that none of them finishes late: a unit is one
// output row x 16 bytes, block b owns units [b U / nb, (b + 1) U / nb) of
// U = M x ceil(ncols / 16); thread t owns dword t % 4 of the unit and the
// input rows k = t / 4 + j x 16 KW, multiplies by v_perm tables
// (gf_make_tables), and the block folds through lane shuffles and LDS.  Up to
// kSideUnits units x kSidePass row steps are loaded in the prologue, ahead of
// the row ring, and multiplied while the ring's rows are in flight; blocks
// with more run their units after the store.
struct BsSideK {
  const uint8_t* x;
  uint8_t* y;
  uint32_t ldx, ldy;
  int ncols;  // 0: no side product
};
constexpr int kSideUnits = 2, kSidePass = 4;

// XOR over the 16 lanes of a wave that share lane % 4 (lane ^ 4 ... ^ 32)
__device__ __forceinline__ uint32_t side_fold16(uint32_t v) {
  v ^= __shfl_xor(v, 4);
  v ^= __shfl_xor(v, 8);
  {
    const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);  // lane ^ 16
    v = r[0] ^ r[1];
  }
  const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);    // lane ^ 32
  return r[0] ^ r[1];
}

// dword d of unit u from the KW waves' partial sums part[w * 4 + d]
__device__ __forceinline__ void side_store_dword(const uint32_t* part, int kw, const BsSideK& sd, int n16, int u,
                                                 int d) {
  uint32_t v = 0;
  for (int w = 0; w < kw; w++) v ^= part[w * 4 + d];
  const int row = u / n16, col = (u - row * n16) * 16 + d * 4;
  if (col >= sd.ncols) return;
  uint8_t* dst = sd.y + (size_t)row * sd.ldy + col;
  if (col + 4 <= sd.ncols) {
    *reinterpret_cast<uint32_t*>(dst) = v;
  } else {
    for (int i = 0; col + i < sd.ncols; i++) dst[i] = (uint8_t)(v >> (8 * i));
  }
}

// the block's units [u0, u1) outside the prologue (blocks past the column
// chunks, or more units or row steps than the prologue holds)
template <int KW>
__device__ void bs_side_rest(const uint8_t* __restrict__ A, int lda, int K, const BsSideK& sd, uint32_t* part,
                             int u0, int u1) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, d = tid & 3, kt = tid >> 2;
  const int n16 = (sd.ncols + 15) >> 4;
  for (int u = u0; u < u1; u++) {
    const int row = u / n16, col = (u - row * n16) * 16 + d * 4;
    uint32_t acc = 0;
    for (int k = kt; k < K; k += 16 * KW) {
      const uint32_t x = col < sd.ncols ? *reinterpret_cast<const uint32_t*>(sd.x + (size_t)k * sd.ldx + col) : 0u;
      uint4 t01;
      uint32_t t2;
      gf_make_tables(A[(size_t)row * lda + k], t01, t2);
      acc = gf_mul_acc4(acc, x, t01, t2);
    }
    acc = side_fold16(acc);
    __syncthreads();  // the previous unit's (or the main product's) LDS reads are done
    if (lane < 4) part[w * 4 + lane] = acc;
    __syncthreads();
    if (tid < 4) side_store_dword(part, KW, sd, n16, u, tid);
  }
}

// RP: rows in flight per wave in the row ring (KODR_BS_P, one, for single
// launches; two for grouped launches, whose waves stream long row ranges:
// DESIGN.md, grouped bit-sliced encode).  Both fit 4 waves per SIMD.
static_assert(512 / KODR_BS_VMAX == 512 / KODR_BS_VMAX_P2, "ring variants differ in occupancy");

template <int KW, int MODE = 0, bool GRP = false, int RP = KODR_BS_P>
__global__ __launch_bounds__(64 * KW) __attribute__((amdgpu_waves_per_eu(512 / KODR_BS_VMAX))) void gf_bs_kernel(
    const uint8_t* __restrict__ A, int lda, int M, int K, const uint8_t* __restrict__ X, int ldx,
    uint8_t* __restrict__ Y, size_t ldy, int ncols, int rpw, int ncx, int nrg,
    const uint32_t* __restrict__ tgt, uint32_t thi, int accum, const BsGroupK grp, const BsSideK side) {
  // LDS: [0, 16 KiB) per-row XOR sums [8 rows x 8 planes][64 lanes];
  // [16, 17 KiB) the body target table (absolute lo words of copy 0; copy r
  // is r * KODR_BS_COPY_BYTES further); then each wave's program: per input
  // row the targets of output rows 0..7
  extern __shared__ uint32_t lds[];
  uint64_t stamp[4] = {0, 0, 0, 0};  // MODE 8: s_memtime per phase (timeline)
  if constexpr (MODE == 8) stamp[0] = __builtin_amdgcn_s_memtime();
  if (ncols < 0) {  // bs_init's cross-check: where this kernel's code runs
    const uint64_t pc = __builtin_amdgcn_s_getpc();
    if (threadIdx.x == 0) {
      reinterpret_cast<uint32_t*>(Y)[0] = (uint32_t)pc;
      reinterpret_cast<uint32_t*>(Y)[1] = (uint32_t)(pc >> 32);
    }
    return;
  }
  // DIRECT (one wave per workgroup in a grouped launch): the wave runs all K
  // rows of its task, so there is no cross-wave fold; its accumulators leave
  // the asm in registers and are transposed and stored straight from there
  // (no 16 KiB LDS sum buffer, no barrier: 16 workgroups per CU fit)
  constexpr bool DIRECT = KW == 1 && GRP && (MODE == 0 || (MODE >= 30 && MODE <= 38)) &&
                         (RP == 2 || RP == 3);
  // A direct launch whose grid is resident at once (<= 16 workgroups per CU
  // on 256 CUs: blocks L, L + 256, ... land on CU L mod 256) puts the row
  // groups of one (generation, column chunk) on one CU, which then share the
  // rows through its L1 instead of re-reading them from L2: the B = 32 x 16
  // generation launch 228-229 -> 222-223 us at 2,262 -> 2,302 MHz
  // (profiles/r05/cumap/).  Launches of several rounds keep the XCD order
  // below (co-located there: +4.5 % at B = 256, the placement of later rounds
  // is the dispatcher's).  MODE 34 (tuning) co-locates in any launch.
  int cm_g = blockIdx.y, cm_rg = -1, cm_cx = -1;
  if constexpr (DIRECT) {
    const int S = nrg < 16 ? nrg : 16;
    const long nb = gridDim.x, T = nb * gridDim.y;
    if ((MODE == 34 || T <= 256L * 16) && 16 % S == 0 && nrg % S == 0 && nb % nrg == 0 && T % (256L * S) == 0) {
      const long L = (long)blockIdx.y * nb + blockIdx.x;
      const long c = L & 255, q = L >> 8;
      const long u = (q / S) * 256 + c;
      const int nhi = nrg / S, ncxp = (int)(nb / nrg);
      const long t = u / nhi;
      cm_rg = (int)(u % nhi) * S + (int)(q % S);
      cm_cx = (int)(t % ncxp);
      cm_g = (int)(t / ncxp);
    }
  }
  if constexpr (GRP) {
    const int g = cm_g;
    A += (size_t)g * grp.a_stride;
    X = grp.x[g];
    Y += (size_t)g * grp.y_stride;
  }
  uint32_t* red = lds;
  uint32_t* tgt_l = DIRECT ? lds : lds + 64 * 64;
  uint32_t* prog_l = tgt_l + 256;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  if constexpr (MODE == 20) {
    // Dynamic rows: one program for the workgroup (K rows x 8 targets) and
    // a row counter after it; wave w starts on rows w and w + KW and then
    // takes rows one at a time (gen_bs_bodies.py main_loop_dyn).
    const int b = blockIdx.x;
    const int rg = (b >> 3) % nrg;
    const int cx = (b / (8 * nrg)) * 8 + (b & 7);
    if (cx >= ncx) return;
    const int m0 = rg * kBsRows;
    const int kpad = (K + kBsChunk - 1) / kBsChunk * kBsChunk;
    uint32_t* cnt = prog_l + kpad * kBsRows;
    constexpr int kTgt = 256;
    uint32_t ot[(kTgt + 63) / 64];
#pragma unroll
    for (int j = 0; j < (kTgt + 63) / 64; j++) {
      const int i = tid + j * 64 * KW;
      ot[j] = i < kTgt ? tgt[i] : 0u;
    }
    const int ne = kpad * kBsRows;
    auto coef = [&](int e) -> uint32_t {
      const int k = e >> 3, row = m0 + (e & 7);
      return (e < ne && k < K && row < M) ? (uint32_t)A[(size_t)row * lda + k] : 0u;
    };
    uint32_t c[4];
#pragma unroll
    for (int j = 0; j < 4; j++) c[j] = coef(tid + j * 64 * KW);
    const uint32_t col = (uint32_t)(cx * 64 + lane) * kBsBlock;
    const uint32_t nrec = __builtin_amdgcn_readfirstlane((uint32_t)K * (uint32_t)ldx);
    const uint32_t sldx = __builtin_amdgcn_readfirstlane((uint32_t)ldx);
    const __amdgpu_buffer_rsrc_t xr =
        __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, (int)nrec, 0x00020000);
    u32x4 ring[2 * KODR_BS_P];
    ring[0] = __builtin_amdgcn_raw_buffer_load_b128(xr, col, (uint32_t)w * sldx, 0);
    ring[1] = __builtin_amdgcn_raw_buffer_load_b128(xr, col + 16, (uint32_t)w * sldx, 0);
#pragma unroll
    for (int j = 0; j < (kTgt + 63) / 64; j++) {
      const int i = tid + j * 64 * KW;
      if (i < kTgt) tgt_l[i] = ot[j];
    }
    for (int i = tid; i < 64 * 64; i += 64 * KW) red[i] = 0u;
    if (tid == 0) *cnt = 2u * KW;
    __syncthreads();
    for (int e0 = 0; e0 < ne; e0 += 4 * 64 * KW) {
      if (e0) {
#pragma unroll
        for (int j = 0; j < 4; j++) c[j] = coef(e0 + tid + j * 64 * KW);
      }
#pragma unroll
      for (int j = 0; j < 4; j++) {
        const int e = e0 + tid + j * 64 * KW;
        if (e < ne) prog_l[e] = tgt_l[c[j]] + (uint32_t)((e & 7) % KODR_BS_NCOPY) * KODR_BS_COPY_BYTES;
      }
    }
    __syncthreads();
    const uint64_t xa = reinterpret_cast<uint64_t>(X);
    const uint32_t xlo = __builtin_amdgcn_readfirstlane((uint32_t)xa);
    const uint32_t xhi = __builtin_amdgcn_readfirstlane((uint32_t)(xa >> 32));
    const uint32_t sthi = __builtin_amdgcn_readfirstlane(thi);
    const uint32_t sc = __builtin_amdgcn_readfirstlane((uint32_t)w);
    const uint32_t sn = __builtin_amdgcn_readfirstlane((uint32_t)(w + KW));
    const uint32_t nk = __builtin_amdgcn_readfirstlane((uint32_t)K);
    const uint32_t km1 = __builtin_amdgcn_readfirstlane((uint32_t)max(K - 1, 0));
    const uint32_t r0x32 = __builtin_amdgcn_readfirstlane((uint32_t)w * 32u);
    const uint32_t pl = (uint32_t)reinterpret_cast<uintptr_t>(prog_l) + (uint32_t)(lane & 7) * 4u;
    const uint32_t cnta = (uint32_t)reinterpret_cast<uintptr_t>(cnt);
    if (K > 0) {
      asm volatile(KODR_BS_MAIN_DYN KODR_BS_REDUCE "s_waitcnt lgkmcnt(0)\n\t"
                   : KODR_BS_RING_OPERANDS
                   : [xlo] "s"(xlo), [xhi] "s"(xhi), [nrec] "s"(nrec), [ldx] "s"(sldx), [thi] "s"(sthi),
                     [col] "v"(col), [lds] "v"((uint32_t)reinterpret_cast<uintptr_t>(red) + (uint32_t)lane * 4u),
                     [sc] "s"(sc), [sn] "s"(sn), [nk] "s"(nk), [km1] "s"(km1), [r0x32] "s"(r0x32), [pl] "v"(pl),
                     [cnt] "v"(cnta)
                   : KODR_BS_CLOBBERS_DYN);
    }
    __syncthreads();
    for (int it = tid; it < kBsRows * 64; it += 64 * KW) {
      const int m = it >> 6, l = it & 63;
      const int row = m0 + m;
      const int cc = (cx * 64 + l) * kBsBlock;
      if (row >= M || cc >= ncols) continue;
      uint32_t d[8];
#pragma unroll
      for (int p = 0; p < 8; p++) d[p] = red[(m * 8 + p) * 64 + l];
      bitslice32(d);
      uint8_t* dst = Y + (size_t)row * ldy + cc;
      if (cc + kBsBlock <= ncols) {
        uint4 v0 = make_uint4(d[0], d[1], d[2], d[3]), v1 = make_uint4(d[4], d[5], d[6], d[7]);
        if (accum) {
          const uint4 o0 = reinterpret_cast<const uint4*>(dst)[0], o1 = reinterpret_cast<const uint4*>(dst)[1];
          v0 = make_uint4(v0.x ^ o0.x, v0.y ^ o0.y, v0.z ^ o0.z, v0.w ^ o0.w);
          v1 = make_uint4(v1.x ^ o1.x, v1.y ^ o1.y, v1.z ^ o1.z, v1.w ^ o1.w);
        }
        bs_store32(dst, v0, v1);
      } else {
        for (int i = 0; cc + i < ncols; i++)
          dst[i] = (uint8_t)(d[i >> 2] >> (8 * (i & 3))) ^ (accum ? dst[i] : (uint8_t)0);
      }
    }
    return;
  }
  // XCD-aware order: the nrg row groups of one column chunk go to blocks
  // b, b+8, ... (one XCD) and re-read that chunk from its L2.  Speed only.
  // (row groups past 32 in bands of 32, each band in this order over its own
  // blocks, measured the same at B = 258: profiles/r06/tail/)
  const int b = blockIdx.x;
  const int rg = cm_rg >= 0 ? cm_rg : (b >> 3) % nrg;
  const int cx = cm_cx >= 0 ? cm_cx : (b / (8 * nrg)) * 8 + (b & 7);
  // the side product's partial sums: past the programs (bs_lds_bytes)
  constexpr bool SIDE = !GRP && MODE == 0;
  uint32_t* side_part = lds + 64 * 64 + 256 + KW * rpw * kBsRows + 4;
  const int s_n16 = (side.ncols + 15) >> 4;
  const long s_U = (long)M * s_n16;
  const int s_u0 = (int)((long)blockIdx.x * s_U / gridDim.x), s_u1 = (int)((long)(blockIdx.x + 1) * s_U / gridDim.x);
  if (cx >= ncx) {
    if constexpr (SIDE)
      if (side.ncols > 0) bs_side_rest<KW>(A, lda, K, side, side_part, s_u0, s_u1);
    return;
  }
  const int m0 = rg * kBsRows, kb = w * rpw;
  if constexpr (MODE == 38)  // tuning: a last row group with fewer than 8 rows does nothing (wrong products)
    if (m0 + kBsRows > M) return;
  // this wave's input rows: [kb, kb + nr), nr a multiple of the 8-row
  // program chunk (rows >= K read zero and have coefficient 0)
  const int kpad = (K + kBsChunk - 1) / kBsChunk * kBsChunk;
  const int nr = __builtin_amdgcn_readfirstlane(max(0, min(rpw, kpad - kb)));

  // Prologue loads in retirement order (vmcnt counts in issue order): the
  // target table and this wave's coefficients (all of them up to K = 256:
  // kPre per lane), then the ring's first rows, so the program build waits
  // only for the former while the rows' HBM latency overlaps it.  (With 8
  // per lane, a one-wave task of 256 rows loaded the rest in three more
  // rounds, each behind the ring's rows in the vmcnt order.)
  const int ne = nr * kBsRows;
  auto coef = [&](int e) -> uint32_t {
    const int k = kb + (e >> 3), row = m0 + (e & 7);
    return (e < ne && k < K && row < M) ? (uint32_t)A[(size_t)row * lda + k] : 0u;
  };
  constexpr int kTgt = 256;
  uint32_t ot[(kTgt + 63) / 64];
#pragma unroll
  for (int j = 0; j < (kTgt + 63) / 64; j++) {
    const int i = tid + j * 64 * KW;
    ot[j] = i < kTgt ? tgt[i] : 0u;
  }
  constexpr int kPre = KW == 1 ? 32 : KW == 2 ? 16 : KW == 3 ? 12 : 8;  // ceil(256 / KW) rows x 8 / 64 lanes
  uint32_t c[kPre];
#pragma unroll
  for (int j = 0; j < kPre; j++) c[j] = coef(j * 64 + lane);

  // side product: this block's units, loaded ahead of the row ring (vmcnt
  // retires in issue order) through descriptors that read zero past K
  const int s_d = tid & 3, s_kt = tid >> 2;
  const int s_nu = s_u1 - s_u0, s_np = (K + 16 * KW - 1) / (16 * KW);
  const bool side_fast = SIDE && side.ncols > 0 && s_nu <= kSideUnits && s_np <= kSidePass;
  uint32_t s_x[kSideUnits][kSidePass], s_c[kSideUnits][kSidePass];
  if constexpr (SIDE) {
#pragma unroll
    for (int j = 0; j < kSideUnits; j++) {
      const bool on = side_fast && j < s_nu;
      const int u = s_u0 + j, row = on ? u / s_n16 : 0, col = on ? (u - row * s_n16) * 16 + s_d * 4 : 0;
      const __amdgpu_buffer_rsrc_t xr2 = __builtin_amdgcn_make_buffer_rsrc(
          (void*)side.x, (short)0, on ? (int)((uint32_t)K * side.ldx) : 0, 0x00020000);
      const __amdgpu_buffer_rsrc_t ar2 = __builtin_amdgcn_make_buffer_rsrc(
          (void*)(A + (size_t)row * lda), (short)0, on ? K : 0, 0x00020000);
#pragma unroll
      for (int p = 0; p < kSidePass; p++) {
        const uint32_t k = (uint32_t)(s_kt + p * 16 * KW);
        s_c[j][p] = __builtin_amdgcn_raw_buffer_load_b8(ar2, k, 0, 0);
        s_x[j][p] = __builtin_amdgcn_raw_buffer_load_b32(xr2, k * side.ldx + (uint32_t)col, 0, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);  // keep them ahead of the ring loads
  }

  const uint32_t col = (uint32_t)(cx * 64 + lane) * kBsBlock;
  // rows past this wave's range read zero, so the look-ahead loads of its
  // last P rows move no data
  const uint32_t kend = (uint32_t)max(0, min(K, kb + nr));
  const uint32_t nrec = __builtin_amdgcn_readfirstlane(kend * (uint32_t)ldx);
  const uint32_t sldx = __builtin_amdgcn_readfirstlane((uint32_t)ldx);
  const uint32_t kboff = __builtin_amdgcn_readfirstlane((uint32_t)kb * (uint32_t)ldx);
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, (int)nrec, 0x00020000);
  // (unconditional: a wave past K reads zeros, and a branch here would make
  // the compiler's waitcnt pass drain these loads at the next LDS write)
  u32x4 ring[2 * RP];
#pragma unroll
  for (int i = 0; i < RP; i++) {
    ring[2 * i] = __builtin_amdgcn_raw_buffer_load_b128(xr, col, kboff + i * sldx, 0);
    ring[2 * i + 1] = __builtin_amdgcn_raw_buffer_load_b128(xr, col + 16, kboff + i * sldx, 0);
  }

#pragma unroll
  for (int j = 0; j < (kTgt + 63) / 64; j++) {
    const int i = tid + j * 64 * KW;
    if (i < kTgt) tgt_l[i] = ot[j];
  }
  if constexpr (!DIRECT)
    for (int i = tid; i < 64 * 64; i += 64 * KW) red[i] = 0u;
  __syncthreads();
  // program: entry e = the target of (output row m0 + e%8, input row kb + e/8):
  // body c in copy (e%8) % KODR_BS_NCOPY
  uint32_t* wp = prog_l + w * rpw * kBsRows;
#pragma unroll
  for (int j = 0; j < kPre; j++) {
    const int e = j * 64 + lane;
    if (e < ne) wp[e] = tgt_l[c[j]] + (uint32_t)((e & 7) % KODR_BS_NCOPY) * KODR_BS_COPY_BYTES;
  }
  for (int e0 = kPre * 64; e0 < ne; e0 += 64 * 8) {  // K > 256: the rest in rounds of 8 per lane
    uint32_t cc[8];
#pragma unroll
    for (int j = 0; j < 8; j++) cc[j] = coef(e0 + j * 64 + lane);
#pragma unroll
    for (int j = 0; j < 8; j++) {
      const int e = e0 + j * 64 + lane;
      if (e < ne) wp[e] = tgt_l[cc[j]] + (uint32_t)((e & 7) % KODR_BS_NCOPY) * KODR_BS_COPY_BYTES;
    }
  }
#ifdef KODR_TUNE_MODES
  // MODE 14: the program also in global memory, read by the asm with scalar
  // loads (the compiler waits for these stores with the ring loads before the asm)
  uint32_t* progw = nullptr;
  if constexpr (MODE == 14) {
    progw = g_bs_prog + ((size_t)blockIdx.x * KW + w) * (size_t)rpw * kBsRows;
    for (int e = lane; e < ne; e += 64) progw[e] = wp[e];
  }
#else
  uint32_t* progw = nullptr;
#endif
  if constexpr (SIDE) {
    if (side_fast) {
#pragma unroll
      for (int j = 0; j < kSideUnits; j++) {
        if (j < s_nu) {
          uint32_t acc = 0;
#pragma unroll
          for (int p = 0; p < kSidePass; p++) {
            if (p < s_np) {  // row steps past K: nothing to add
              uint4 t01;
              uint32_t t2;
              gf_make_tables(s_c[j][p], t01, t2);
              acc = gf_mul_acc4(acc, s_x[j][p], t01, t2);
            }
          }
          acc = side_fold16(acc);
          if (lane < 4) side_part[(j * KW + w) * 4 + lane] = acc;
        }
      }
    }
  }
  // (the stores wait for the block's own: a store before the main loop
  // would make the compiler wait for it, vmcnt(0), at the loop's asm)
  __syncthreads();

  const uint32_t ngrp = __builtin_amdgcn_readfirstlane((uint32_t)(nr / kBsChunk));
  const uint64_t xa = reinterpret_cast<uint64_t>(X);
  const uint32_t xlo = __builtin_amdgcn_readfirstlane((uint32_t)xa);
  const uint32_t xhi = __builtin_amdgcn_readfirstlane((uint32_t)(xa >> 32));
  const uint32_t roff = kboff + RP * sldx;  // the asm streams from row kb + RP
  // this lane's program word in LDS (chunk lane 8j + m: row j, output row m)
  const uint32_t pl = (uint32_t)(reinterpret_cast<uintptr_t>(wp)) + (uint32_t)lane * 4u;
  const uint32_t sthi = __builtin_amdgcn_readfirstlane(thi);
  if constexpr (MODE == 8) stamp[1] = __builtin_amdgcn_s_memtime();
  const uint64_t pga = reinterpret_cast<uint64_t>(progw);
  const uint32_t pglo = __builtin_amdgcn_readfirstlane((uint32_t)pga);
  const uint32_t pghi = __builtin_amdgcn_readfirstlane((uint32_t)(pga >> 32));
#define KODR_BS_ASM_INPUTS                                                                          \
  [xlo] "s"(xlo), [xhi] "s"(xhi), [nrec] "s"(nrec), [roff] "s"(roff), [ldx] "s"(sldx), [ngrp] "s"(ngrp),  \
      [thi] "s"(sthi), [col] "v"(col), [lds] "v"((uint32_t)reinterpret_cast<uintptr_t>(red) + (uint32_t)lane * 4u), \
      [pl] "v"(pl), [ydbg] "s"(Y), [pglo] "s"(pglo), [pghi] "s"(pghi)
#define KODR_BS_ASM2(MAIN, CLOB)                                                                    \
  asm volatile(MAIN KODR_BS_REDUCE "s_waitcnt lgkmcnt(0)\n\t" : KODR_BS_RING_OPERANDS : KODR_BS_ASM_INPUTS : CLOB)
#define KODR_BS_ASM(MAIN) KODR_BS_ASM2(MAIN, KODR_BS_CLOBBERS)
  if constexpr (DIRECT) {
    u32x8 acc[8];
    if (nr > 0 && MODE == 30) {  // tuning: bodies inlined for one coefficient (no jumps, wrong products)
      asm volatile(KODR_BS_MAIN_P2_INLINE "s_waitcnt lgkmcnt(0)\n\t"
                   : KODR_BS_RING_OPERANDS_P2, KODR_BS_ACC_OUTPUTS
                   : KODR_BS_ASM_INPUTS
                   : KODR_BS_CLOBBERS_P2_DIRECT);
    } else if (nr > 0 && MODE == 31) {  // tuning: no row stream (stale rows, wrong products)
      asm volatile(KODR_BS_MAIN_P2_NL "s_waitcnt lgkmcnt(0)\n\t"
                   : KODR_BS_RING_OPERANDS_P2, KODR_BS_ACC_OUTPUTS
                   : KODR_BS_ASM_INPUTS
                   : KODR_BS_CLOBBERS_P2_DIRECT);
    } else if (nr > 0 && MODE == 32) {  // tuning: neither jumps nor row stream
      asm volatile(KODR_BS_MAIN_P2_INLINE_NL "s_waitcnt lgkmcnt(0)\n\t"
                   : KODR_BS_RING_OPERANDS_P2, KODR_BS_ACC_OUTPUTS
                   : KODR_BS_ASM_INPUTS
                   : KODR_BS_CLOBBERS_P2_DIRECT);
#ifdef KODR_TUNE_MODES
    } else if (nr > 0 && MODE == 35) {  // tuning: no priority rotation
      asm volatile(KODR_BS_MAIN_P2_NOPRIO "s_waitcnt lgkmcnt(0)\n\t"
                   : KODR_BS_RING_OPERANDS_P2, KODR_BS_ACC_OUTPUTS
                   : KODR_BS_ASM_INPUTS
                   : KODR_BS_CLOBBERS_P2_DIRECT);
    } else if (nr > 0 && MODE == 37) {  // tuning: preparation at priority 3, bodies at 0
      asm volatile(KODR_BS_MAIN_P2_PREP "s_waitcnt lgkmcnt(0)\n\t"
                   : KODR_BS_RING_OPERANDS_P2, KODR_BS_ACC_OUTPUTS
                   : KODR_BS_ASM_INPUTS
                   : KODR_BS_CLOBBERS_P2_DIRECT);
    } else if (nr > 0 && MODE == 36) {  // tuning: the rotation over row pairs
      asm volatile(KODR_BS_MAIN_P2_PRIO2 "s_waitcnt lgkmcnt(0)\n\t"
                   : KODR_BS_RING_OPERANDS_P2, KODR_BS_ACC_OUTPUTS
                   : KODR_BS_ASM_INPUTS
                   : KODR_BS_CLOBBERS_P2_DIRECT);
    } else if (nr > 0 && RP == 3) {  // tuning: three rows in flight (a build with the map moved down)
      asm volatile(KODR_BS_MAIN_P3 "s_waitcnt lgkmcnt(0)\n\t"
                   : KODR_BS_RING_OPERANDS_P3, KODR_BS_ACC_OUTPUTS
                   : KODR_BS_ASM_INPUTS
                   : KODR_BS_CLOBBERS_P3_DIRECT);
#endif
    } else if (nr > 0) {
      asm volatile(KODR_BS_MAIN_P2 "s_waitcnt lgkmcnt(0)\n\t"
                   : KODR_BS_RING_OPERANDS_P2, KODR_BS_ACC_OUTPUTS
                   : KODR_BS_ASM_INPUTS
                   : KODR_BS_CLOBBERS_P2_DIRECT);
    } else {
#pragma unroll
      for (int m = 0; m < kBsRows; m++) acc[m] = u32x8{0, 0, 0, 0, 0, 0, 0, 0};
    }
    // rows m0..m0+7 of this lane's 32-byte block: planes -> bytes, store
    const int cc = (cx * 64 + lane) * kBsBlock;
#pragma unroll
    for (int m = 0; m < kBsRows; m++) {
      const int row = m0 + m;
      if (row >= M || cc >= ncols) continue;
      uint32_t d[8] = {acc[m][0], acc[m][1], acc[m][2], acc[m][3], acc[m][4], acc[m][5], acc[m][6], acc[m][7]};
      bitslice32(d);
      uint8_t* dst = Y + (size_t)row * ldy + cc;
      if (cc + kBsBlock <= ncols) {
        uint4 v0 = make_uint4(d[0], d[1], d[2], d[3]), v1 = make_uint4(d[4], d[5], d[6], d[7]);
        if (accum) {
          const uint4 o0 = reinterpret_cast<const uint4*>(dst)[0], o1 = reinterpret_cast<const uint4*>(dst)[1];
          v0 = make_uint4(v0.x ^ o0.x, v0.y ^ o0.y, v0.z ^ o0.z, v0.w ^ o0.w);
          v1 = make_uint4(v1.x ^ o1.x, v1.y ^ o1.y, v1.z ^ o1.z, v1.w ^ o1.w);
        }
        bs_store32(dst, v0, v1);
      } else {
        for (int i = 0; cc + i < ncols; i++)
          dst[i] = (uint8_t)(d[i >> 2] >> (8 * (i & 3))) ^ (accum ? dst[i] : (uint8_t)0);
      }
    }
    return;
  }
  if (nr > 0 && MODE != 5) {
    if constexpr (RP != KODR_BS_P) {
      static_assert(DIRECT || (RP == 2 && (MODE == 0 || MODE >= 30)), "the two-row ring variant has the plain main loop only");
      asm volatile(KODR_BS_MAIN_P2 KODR_BS_REDUCE "s_waitcnt lgkmcnt(0)\n\t"
                   : KODR_BS_RING_OPERANDS_P2
                   : KODR_BS_ASM_INPUTS
                   : KODR_BS_CLOBBERS_P2);
    } else if constexpr (MODE == 9) {
      if (blockIdx.x == 0 && w == 0) {
        KODR_BS_ASM(KODR_BS_DUMP);
        uint32_t* yd = reinterpret_cast<uint32_t*>(Y) + 64;
        if (lane == 0) {
          yd[0] = pl;
          for (int i = 0; i < 16; i++) yd[1 + i] = wp[i];
          for (int i = 0; i < 8; i++) yd[17 + i] = tgt_l[i];
          for (int i = 0; i < 4; i++) yd[25 + i] = tgt[i];
          yd[29] = (uint32_t)ne;
          yd[30] = (uint32_t)c[0];
        }
      }
      return;
    } else if constexpr (MODE == 3) {
      KODR_BS_ASM(KODR_BS_MAIN_ND);
    } else if constexpr (MODE == 4) {
      KODR_BS_ASM(KODR_BS_MAIN_NDNL);
    } else if constexpr (MODE == 10) {
      KODR_BS_ASM(KODR_BS_MAIN_NOPRIO);
    } else if constexpr (MODE == 11) {
      KODR_BS_ASM(KODR_BS_MAIN_HALF);
    } else if constexpr (MODE == 12) {
      KODR_BS_ASM(KODR_BS_MAIN_2RL);
    } else if constexpr (MODE == 13) {
      KODR_BS_ASM(KODR_BS_MAIN_2TB);
#ifdef KODR_TUNE_MODES
    } else if constexpr (MODE == 14) {
      KODR_BS_ASM2(KODR_BS_MAIN_SLOAD, KODR_BS_CLOBBERS_SLOAD);
#endif
    } else if constexpr (MODE == 6) {
      KODR_BS_ASM(KODR_BS_MAIN_NL);
    } else {
      KODR_BS_ASM(KODR_BS_MAIN);
    }
  }
#undef KODR_BS_ASM
#undef KODR_BS_ASM2
#undef KODR_BS_ASM_INPUTS
  if constexpr (MODE == 8) stamp[2] = __builtin_amdgcn_s_memtime();
  __syncthreads();

  // rows m0..m0+7 of this column chunk: planes -> bytes, store
  for (int it = tid; it < kBsRows * 64; it += 64 * KW) {
    const int m = it >> 6, l = it & 63;
    const int row = m0 + m;
    const int cc = (cx * 64 + l) * kBsBlock;
    if (row >= M || cc >= ncols) continue;
    uint32_t d[8];
#pragma unroll
    for (int p = 0; p < 8; p++) d[p] = red[(m * 8 + p) * 64 + l];
    bitslice32(d);
    uint8_t* dst = Y + (size_t)row * ldy + cc;
    if (cc + kBsBlock <= ncols) {
      uint4 v0 = make_uint4(d[0], d[1], d[2], d[3]), v1 = make_uint4(d[4], d[5], d[6], d[7]);
      if (accum) {  // a later row chunk of a K-split product: Y ^= this chunk's part
        const uint4 o0 = reinterpret_cast<const uint4*>(dst)[0], o1 = reinterpret_cast<const uint4*>(dst)[1];
        v0 = make_uint4(v0.x ^ o0.x, v0.y ^ o0.y, v0.z ^ o0.z, v0.w ^ o0.w);
        v1 = make_uint4(v1.x ^ o1.x, v1.y ^ o1.y, v1.z ^ o1.z, v1.w ^ o1.w);
      }
      bs_store32(dst, v0, v1);
    } else {
      for (int i = 0; cc + i < ncols; i++)
        dst[i] = (uint8_t)(d[i >> 2] >> (8 * (i & 3))) ^ (accum ? dst[i] : (uint8_t)0);
    }
  }
  if constexpr (SIDE) {
    if (side_fast && tid < 4 * s_nu)  // the prologue's sums, still in LDS
      side_store_dword(side_part + (tid >> 2) * KW * 4, KW, side, s_n16, s_u0 + (tid >> 2), tid & 3);
    if (side.ncols > 0 && !side_fast) bs_side_rest<KW>(A, lda, K, side, side_part, s_u0, s_u1);
  }
  if constexpr (MODE == 8) {  // timeline build: stamps past the M output rows (the caller sizes Y)
    __syncthreads();
    stamp[3] = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
      uint64_t* t = reinterpret_cast<uint64_t*>(Y + (size_t)M * ldy) + ((size_t)blockIdx.x * KW + w) * 5;
      for (int i = 0; i < 4; i++) t[i] = stamp[i];
      t[4] = __builtin_amdgcn_s_memrealtime();
    }
  }
}

struct BsDevice {
  uint32_t* tgt = nullptr;  // absolute lo words of the 256 bodies of copy 0
  uint32_t thi = 0;         // their common hi word
  uint32_t offs[256 * KODR_BS_NCOPY] = {};
  bool ready = false, ok = false;
};
std::mutex g_bs_mu;
BsDevice g_bs[64];

// Once per device: export the bodies' addresses, check them against the
// generator's layout and that all share one hi word (the kernel jumps to
// hi:lo with a fixed hi).  ok = false leaves the bit-sliced path unused
// (callers fall back to gf_gemm); the error return is for HIP failures.
hipError_t bs_init(int dev, const BsDevice** out) {
  std::lock_guard<std::mutex> lk(g_bs_mu);
  if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
  BsDevice& d = g_bs[dev];
  if (!d.ready) {
    constexpr int n = 256 * KODR_BS_NCOPY;
    uint32_t* buf = nullptr;
    hipError_t e = hipMalloc((void**)&buf, (n + 2) * sizeof(uint32_t));
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(gf_bs_export_kernel, dim3(1), dim3(64), 0, 0, buf);
    if ((e = hipGetLastError()) == hipSuccess) e = hipDeviceSynchronize();
    static uint32_t h[n + 2];
    if (e == hipSuccess) e = hipMemcpy(h, buf, sizeof(h), hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
      (void)hipFree(buf);
      return e;
    }
    const uint64_t base = (uint64_t)h[n] | ((uint64_t)h[n + 1] << 32);
    // the bodies and gf_bs_kernel are in one code object: a base far from
    // where gf_bs_kernel runs means the export is wrong, and jumping there
    // would fault
    hipLaunchKernelGGL((gf_bs_kernel<1, 0>), dim3(1), dim3(64), 0, 0, nullptr, 0, 0, 0, nullptr, 0,
                       reinterpret_cast<uint8_t*>(buf), (size_t)0, -1, 0, 0, 0, nullptr, 0u, 0, BsGroupK{}, BsSideK{});
    if ((e = hipGetLastError()) == hipSuccess) e = hipDeviceSynchronize();
    uint32_t kpc[2] = {0, 0};
    if (e == hipSuccess) e = hipMemcpy(kpc, buf, sizeof(kpc), hipMemcpyDeviceToHost);
    if (e != hipSuccess) {
      (void)hipFree(buf);
      return e;
    }
    const uint64_t kernel_pc = (uint64_t)kpc[0] | ((uint64_t)kpc[1] << 32);
    const uint64_t dist = kernel_pc > base ? kernel_pc - base : base - kernel_pc;
    bool ok = dist < ((uint64_t)64 << 20) && (base >> 32) == ((base + KODR_BS_CODE_BYTES) >> 32);
    for (int i = 0; i < n; i++) {
      d.offs[i] = h[i];
      ok = ok && h[i] == kBsBodyOffsets[i] && h[i] == d.offs[i % 256] + (uint32_t)(i / 256) * KODR_BS_COPY_BYTES;
      h[i] = (uint32_t)(base + h[i]);
    }
    if (ok) e = hipMemcpy(buf, h, 256 * sizeof(uint32_t), hipMemcpyHostToDevice);
    if (e != hipSuccess || !ok) {
      (void)hipFree(buf);
      buf = nullptr;
    }
    if (e != hipSuccess) return e;
    d.tgt = buf;
    d.thi = (uint32_t)(base >> 32);
    d.ok = ok;
    d.ready = true;
  }
  *out = &d;
  return hipSuccess;
}

template <int KW, int MODE = 0>
hipError_t bs_launch(const uint8_t* A, int lda, int M, int K, const uint8_t* X, int ldx, uint8_t* Y,
                     size_t ldy, int ncols, int rpw, int ncx, int nrg, size_t lds_bytes, const BsDevice* bd,
                     hipStream_t st, int accum, const GemmGroupArgs* group, const BsSideK& side) {
  const int nb = (ncx + 7) / 8 * 8 * nrg;
  BsGroupK g{};
  if (group) {
    for (int i = 0; i < group->n; i++) g.x[i] = group->x[i];
    g.a_stride = group->a_stride;
    g.y_stride = group->y_stride;
    // gridDim.x is a multiple of 8, so the XCD order of each generation's
    // blocks is the single-generation one; the two-row ring (plain loop only)
    constexpr int rp = MODE == 33 ? (KW == 1 ? 3 : 2) : MODE == 0 || (MODE >= 30 && MODE <= 38) ? 2 : KODR_BS_P;
    hipLaunchKernelGGL((gf_bs_kernel<KW, MODE, true, rp>), dim3(nb, group->n), dim3(64 * KW), lds_bytes, st, A,
                       lda, M, K, X, ldx, Y, ldy, ncols, rpw, ncx, nrg, bd->tgt, bd->thi, accum, g, BsSideK{});
    last_launch_plan() = LaunchPlan{2, kBsRows, KW, 1, rp, rpw, group->n, nb};
  } else {
    hipLaunchKernelGGL((gf_bs_kernel<KW, MODE>), dim3(nb), dim3(64 * KW), lds_bytes, st, A, lda, M, K, X, ldx, Y,
                       ldy, ncols, rpw, ncx, nrg, bd->tgt, bd->thi, accum, g, side);
    last_launch_plan() = LaunchPlan{2, kBsRows, KW, 1, KODR_BS_P, rpw, 1, nb};
  }
  return hipGetLastError();
}

}  // namespace

hipError_t bs_body_offsets(int device, uint32_t* host_out) {
  const BsDevice* bd = nullptr;
  hipError_t e = bs_init(device, &bd);
  if (e != hipSuccess) return e;
  for (int c = 0; c < 256; c++) host_out[c] = bd->offs[c];
  return hipSuccess;
}

bool bs_ready(int device) {
  const BsDevice* bd = nullptr;
  return bs_init(device, &bd) == hipSuccess && bd->ok;
}

hipError_t copy_bitslice_rows(const uint8_t* src, size_t spitch, uint8_t* dst, uint8_t* dst_bs, size_t dpitch,
                              size_t rows, size_t ncols, hipStream_t stream) {
  if (!rows || !ncols) return hipSuccess;
  if (ncols % kBsBlock || dpitch % kBsBlock || dpitch < ncols || (uintptr_t)src % 16 || spitch % 16 ||
      (uintptr_t)dst % 16 || !dst_bs || (uintptr_t)dst_bs % 16)
    return hipErrorInvalidValue;
  const size_t nblk = ncols / kBsBlock;
  const size_t total = rows * nblk;
  if (rows > 0x7fffffff || nblk > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(copy_bitslice_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, src,
                     spitch, dst, dst_bs, dpitch, (int)rows, (int)nblk);
  return hipGetLastError();
}

bool copy_bitslice_ok(const uint8_t* src, size_t spitch, const uint8_t* dst, const uint8_t* dst_bs, size_t dpitch,
                      size_t ncols) {
  return ncols && ncols % kBsBlock == 0 && dpitch % kBsBlock == 0 && dpitch >= ncols && (uintptr_t)src % 16 == 0 &&
         spitch % 16 == 0 && (uintptr_t)dst % 16 == 0 && dst_bs && (uintptr_t)dst_bs % 16 == 0 &&
         ncols / kBsBlock <= 0x7fffffff;
}

// copy workgroups per CU over the launch beside the elimination (16 of a
// CU's 32 wave slots: room for an elimination workgroup of 16 waves), and
// alone (after it: 187 against 198 us for the round trip's 16 generations at
// 4, profiles/r05/copy_order/)
constexpr int kCopyWgPerCu = 4, kCopyWgPerCuAlone = 16;

hipError_t copy_bitslice_rows_grouped(const CopyGroup& g, int n, size_t spitch, size_t dpitch, size_t ncols,
                                      hipStream_t stream, bool beside) {
  if (n <= 0) return hipSuccess;
  if (n > kCopyGroupMax) return hipErrorInvalidValue;
  int maxr = 0;
  for (int i = 0; i < n; i++) {
    if (g.rows[i] < 0 || !copy_bitslice_ok(g.src[i], spitch, g.dst[i], g.dbs[i], dpitch, ncols))
      return hipErrorInvalidValue;
    maxr = g.rows[i] > maxr ? g.rows[i] : maxr;
  }
  const size_t nblk = ncols / kBsBlock, total = (size_t)maxr * nblk * 2;  // two lanes per block
  if (!total) return hipSuccess;
  // at most kCopyWgPerCu workgroups (4 waves each) per CU over the launch
  static const int wg_tune = tune_env("KODR_COPY_WG_PER_CU") ? atoi(tune_env("KODR_COPY_WG_PER_CU")) : 0;
  const int wg_per_cu = wg_tune ? wg_tune : beside ? kCopyWgPerCu : kCopyWgPerCuAlone;
  const size_t cap = std::max<size_t>(1, (size_t)std::max(wg_per_cu, 1) * 256 / (size_t)n);
  const size_t gx = std::min<size_t>((total + 255) / 256, cap);
  hipLaunchKernelGGL(copy_bitslice_grouped_kernel, dim3((unsigned)gx, (unsigned)n), dim3(256), 0, stream, g, spitch,
                     dpitch, (int)nblk);
  return hipGetLastError();
}

hipError_t bitslice_rows_pitched(const uint8_t* src, size_t spitch, uint8_t* dst, size_t dpitch, size_t rows,
                                 size_t ncols, hipStream_t stream) {
  if (!rows || !ncols) return hipSuccess;
  const size_t nblk = (ncols + kBsBlock - 1) / kBsBlock;
  if ((uintptr_t)src % 16 || spitch % 16 || dpitch % kBsBlock || dpitch < nblk * kBsBlock) return hipErrorInvalidValue;
  const size_t total = rows * nblk;
  if (rows > 0x7fffffff || nblk > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(bitslice_pitched_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, src,
                     spitch, dst, dpitch, (int)rows, (int)nblk);
  return hipGetLastError();
}

hipError_t bitslice_rows(const uint8_t* src, uint8_t* dst, size_t ldx, size_t rows, size_t ncols,
                         hipStream_t stream) {
  if (!rows || !ncols) return hipSuccess;
  if (ldx % kBsBlock || ldx < (ncols + kBsBlock - 1) / kBsBlock * kBsBlock) return hipErrorInvalidValue;
  const size_t nblk = (ncols + kBsBlock - 1) / kBsBlock;
  const size_t total = rows * nblk;
  if (rows > 0x7fffffff || nblk > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(bitslice_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, src, dst,
                     ldx, (int)rows, (int)nblk);
  return hipGetLastError();
}

namespace {

// Waves per SIMD the kernel's VGPR budget allows (gen_bs_bodies.py: VMAX
// registers plus the compiler's own below v24, rounded to 8).
constexpr int kBsWavesPerSimd = 512 / ((KODR_BS_VMAX + 7) / 8 * 8);
constexpr int kBsKw[] = {1, 2, 3, 4, 6, 8, 16};
constexpr size_t kLdsPerCu = 160 * 1024;

// row sums, the body target table, and KW programs of rpw rows x 8 targets;
// the direct variant (KW = 1 in a grouped launch) has no row sums
size_t bs_lds_bytes(int kw, int rpw, bool direct = false) {
  return (direct ? 256 : 64 * 64 + 256) * 4 + (size_t)kw * rpw * kBsRows * 4 + 16;  // + the dynamic rows' counter
}

// Grouped launches may plan the direct variant (one wave per workgroup, no
// fold): equal at B = 32-64, 2.4 % faster at B = 256 (profiles/r03/direct_ab/).
// KODR_BS_DIRECT=0 keeps the folded plans (A/B measurements).
bool bs_direct_allowed() {
  static const bool v = tune_env("KODR_BS_DIRECT") ? atoi(tune_env("KODR_BS_DIRECT")) != 0 : true;
  return v;
}

}  // namespace

bool side_ok(const BsSide& sd, size_t K) {
  return sd.x && sd.y && (uintptr_t)sd.x % 16 == 0 && (uintptr_t)sd.y % 16 == 0 && sd.ldx % 16 == 0 &&
         sd.ldy % 16 == 0 && sd.ldx >= (sd.ncols + 15) / 16 * 16 && sd.ldy >= sd.ncols && K * sd.ldx < ((size_t)1 << 31) &&
         sd.ldy <= 0xffffffffu && sd.ncols <= 0x7fffffff;
}

BsPlan plan_gemm_bs(size_t M, size_t K, size_t ncols, int groups, bool grouped) {
  BsPlan p;
  p.ncx = (int)((ncols + kBsWaveCols - 1) / kBsWaveCols);
  p.nrg = (int)((M + kBsRows - 1) / kBsRows);
  const long tasks = (long)p.ncx * p.nrg * std::max(groups, 1);
  constexpr long P = kBsChunk;  // rows per wave: whole program chunks
  const long kpad = ((long)K + P - 1) / P * P;
  // cost model in row-units: rounds of resident waves x (rows per wave + the
  // per-wave fixed cost of program build, reduction and store, ~6 rows)
  double best = 1e300;
  for (int kw : kBsKw) {
    if (kw > 4 * kBsWavesPerSimd) continue;  // one workgroup must fit a CU
    const long rpw = ((kpad + kw - 1) / kw + P - 1) / P * P;
    const size_t lds = bs_lds_bytes(kw, (int)rpw, grouped && kw == 1 && bs_direct_allowed());
    if (lds > kLdsPerCu) continue;
    const long wg_per_cu = std::min<long>((4L * kBsWavesPerSimd) / kw, (long)(kLdsPerCu / lds));
    const long slots = 256L * wg_per_cu * kw;  // waves resident at once
    const long waves = tasks * kw;
    const long rounds = (waves + slots - 1) / slots;
    const double cost = (double)rounds * (double)(rpw + 6);
    if (cost < best - 1e-9) {
      best = cost;
      p.kw = kw;
      p.rpw = (int)rpw;
      p.lds_bytes = lds;
    }
  }
  p.blocks = (p.ncx + 7) / 8 * 8 * p.nrg;
  p.ok = best < 1e299;
  return p;
}

hipError_t gf_gemm_bs(const uint8_t* dA, size_t lda, size_t M, size_t K, const uint8_t* dXbs, size_t ldx,
                      uint8_t* dY, size_t ldy, size_t ncols, int device, hipStream_t stream, bool accumulate,
                      const GemmGroupArgs* group, const BsSide* side) {
  if (M == 0 || ncols == 0 || (group && group->n <= 0)) return hipSuccess;
  if (group && group->n > kGemmGroupMax) return hipErrorInvalidValue;
  BsSideK sk{};
  if (side && side->ncols) {
    if (group || accumulate || !side_ok(*side, K)) return hipErrorInvalidValue;
    sk = BsSideK{side->x, side->y, (uint32_t)side->ldx, (uint32_t)side->ldy, (int)side->ncols};
  }
  if (ldx % kBsBlock || ldy % 16 || (size_t)K * ldx >= ((size_t)1 << 32) || ldx > 0x7fffffff ||
      lda > 0x7fffffff || M > 0x7fffffff)
    return hipErrorInvalidValue;
  BsPlan p = plan_gemm_bs(M, K, ncols, group ? group->n : 1, group != nullptr);
  if (!p.ok) return hipErrorInvalidValue;
#ifdef KODR_TUNE_MODES
  if (const char* env = tune_env("KODR_BS_KW")) {  // force the waves per workgroup
    const int kw = atoi(env);
    const long kpad = ((long)K + kBsChunk - 1) / kBsChunk * kBsChunk;
    p.kw = kw;
    p.rpw = (int)(((kpad + kw - 1) / kw + kBsChunk - 1) / kBsChunk * kBsChunk);
    p.lds_bytes = bs_lds_bytes(kw, p.rpw, group && kw == 1 && bs_direct_allowed());
  }
  if (const char* env = tune_env("KODR_BS_WG_PER_CU")) {  // occupancy probe: LDS padding caps workgroups per CU
    const size_t n = (size_t)std::max(1, atoi(env));
    p.lds_bytes = std::max(p.lds_bytes, kLdsPerCu / n - 64);
  }
#endif
  // the side product's partial sums: kSideUnits x KW dwords x 4
  const size_t side_lds = sk.ncols ? (size_t)kSideUnits * p.kw * 16 : 0;
  if (p.lds_bytes + side_lds > kLdsPerCu) return hipErrorInvalidValue;
  const BsDevice* bd = nullptr;
  hipError_t e = bs_init(device, &bd);
  if (e != hipSuccess) return e;
  if (!bd->ok) return hipErrorNotSupported;
  const int iM = (int)M, iK = (int)K, ild = (int)lda, ilx = (int)ldx, inc = (int)ncols;
  int mode = 0;
  (void)mode;
#ifdef KODR_TUNE_MODES
  if (const char* env = tune_env("KODR_BS_MODE")) mode = atoi(env);
  if (mode == 14) {  // program scratch for the scalar-load variant, with look-ahead slack
    static uint32_t* scratch = nullptr;
    constexpr size_t kScratch = (size_t)64 << 20;
    const size_t need = (size_t)p.blocks * p.kw * p.rpw * kBsRows * 4 + 256;
    if (need > kScratch) return hipErrorInvalidValue;
    if (!scratch) {
      if ((e = hipMalloc((void**)&scratch, kScratch)) != hipSuccess) return e;
      if ((e = hipMemcpyToSymbol(HIP_SYMBOL(g_bs_prog), &scratch, sizeof(scratch))) != hipSuccess) return e;
    }
  }
#endif
#define KODR_BS_CALL(KW_, MODE_)                                                                  \
  bs_launch<KW_, MODE_>(dA, ild, iM, iK, dXbs, ilx, dY, ldy, inc, p.rpw, p.ncx, p.nrg,                 \
                        p.lds_bytes + side_lds, bd, stream, accumulate ? 1 : 0,                         \
                        group, sk)
#ifdef KODR_TUNE_MODES
#define KODR_BS_CASE(KW_)                                                                         \
  case KW_:                                                                                       \
    return mode == 3 ? KODR_BS_CALL(KW_, 3) : mode == 5 ? KODR_BS_CALL(KW_, 5)                    \
         : mode == 4 ? KODR_BS_CALL(KW_, 4) : mode == 6 ? KODR_BS_CALL(KW_, 6)                    \
         : mode == 8 ? KODR_BS_CALL(KW_, 8) : mode == 9 ? KODR_BS_CALL(KW_, 9)                    \
         : mode == 10 ? KODR_BS_CALL(KW_, 10) : mode == 11 ? KODR_BS_CALL(KW_, 11)                \
         : mode == 12 ? KODR_BS_CALL(KW_, 12) : mode == 13 ? KODR_BS_CALL(KW_, 13)                \
         : mode == 14 ? KODR_BS_CALL(KW_, 14) : mode == 20 ? KODR_BS_CALL(KW_, 20)           \
         : mode == 30 ? KODR_BS_CALL(KW_, 30) : mode == 31 ? KODR_BS_CALL(KW_, 31)           \
         : mode == 32 ? KODR_BS_CALL(KW_, 32) : mode == 33 ? KODR_BS_CALL(KW_, 33)           \
         : mode == 34 ? KODR_BS_CALL(KW_, 34) : mode == 35 ? KODR_BS_CALL(KW_, 35)           \
         : mode == 36 ? KODR_BS_CALL(KW_, 36) : mode == 37 ? KODR_BS_CALL(KW_, 37)           \
         : mode == 38 ? KODR_BS_CALL(KW_, 38)                                                    \
                                               : KODR_BS_CALL(KW_, 0);
#else
#define KODR_BS_CASE(KW_) \
  case KW_:               \
    return KODR_BS_CALL(KW_, 0);
#endif
  switch (p.kw) {
    KODR_BS_CASE(1)
    KODR_BS_CASE(2)
    KODR_BS_CASE(3)
    KODR_BS_CASE(4)
    KODR_BS_CASE(6)
    KODR_BS_CASE(8)
    KODR_BS_CASE(16)
    default: return hipErrorInvalidValue;
  }
#undef KODR_BS_CASE
#undef KODR_BS_CALL
}

}  // namespace kodr_amd
