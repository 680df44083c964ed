// gf_kernels.hip -- GF(2^8) "GEMM" for gfx950 (CDNA4): Y = A (x) X.
//
//   Y[m][j] = XOR_k  A[m][k] * X[k][j]        (GF(2^8), poly 0x11D)
//
// This one kernel is every data-plane operation of the engine:
//   encode  (full/encoder.go:61-71)   A = B coding vectors (B x k), X = the k
//                                     original pieces, Y = B coded pieces
//   recode  (full/recoder.go:27-46)   A = B recoding vectors (B x n), X = the
//                                     n held coded pieces in wire layout, so the
//                                     vector columns come out as r x C
//                                     (matrix.go:45-69) in the same pass
//   decode  (decoder_state.go:66-73,105-112,130-132)  A = the transform T that
//                                     the host mirror of kodr's elimination
//                                     tracks, X = the received pieces
// It is column-separable (byte j of Y depends only on byte j of X), which is
// what makes the coalesced byte-stream layout and the column sharding work.
//
// Multiply by a coefficient c is GF(2)-linear in x, so c*x = T0[x&7] ^
// T1[(x>>3)&7] ^ T2[x>>6] with three 8/8/4-entry tables of c-multiples.  Each
// table fits in the 8-byte window of v_perm_b32, which looks up 4 bytes per
// instruction: per data dword and coefficient that is 3 v_perm + 2 XOR, and the
// selectors (x&7, x>>3&7, x>>6) are computed once per data dword and shared by
// every output row m.  The tables are built per workgroup into LDS and read as
// wave-uniform broadcasts.  No MFMA: this is byte-field arithmetic.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "gf_device.hpp"
#include "gf_kernels.hpp"
#include "tune.hpp"

namespace kodr_amd {

LaunchPlan& last_launch_plan() {
  static thread_local LaunchPlan p;
  return p;
}

namespace {

constexpr int kLaneBytes = 16;  // one dwordx4 per lane per row
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// Workgroup barrier that waits only for LDS traffic: HIP's __syncthreads()
// also drains vmcnt, which would empty the row-prefetch ring at every K-chunk.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

// Tile: MT output rows x one column chunk of CB = 1024/S bytes per workgroup.
//  - The KW waves of a workgroup split K; each K-chunk of KC = KW*RC rows gives
//    wave w the rows [w*RC, (w+1)*RC).
//  - Inside a wave the 64 lanes form S groups of 64/S lanes; in one row-step
//    group g reads row (base + g) over the chunk, so every load is still a
//    16-byte-per-lane dwordx4 while the chunk narrows to 1024/S bytes (more
//    workgroups, all CUs streaming, nothing read twice).
//  - Partial sums: across the S lane groups by __shfl_xor, across the KW waves
//    by ds_xor in LDS.
// Coefficient tables for (MT x KC) are staged per K-chunk into LDS
// (double-buffered when K > KC) and read back as (S-way) broadcasts.  Rows are
// streamed through a P-deep ring of loads that runs across K-chunk barriers.
//
// Grouped launch (gridDim.y > 1): workgroup row y works on generation y of a
// group of independent products that share M, K, ncols and the pitches --
// X = xg.x[y], A and Y advanced by y strides -- so one launch streams G
// resident generations (full/encoder.go:61-71 once per generation) and pays
// the launch and ramp once.  AUX is the buffer loads' cache policy (2 = nt,
// for rows read once per launch).
template <int MT, int KW, int S, int RC, int P, int MODE = 0, int AUX = 0>
__global__ __launch_bounds__(64 * KW) void gf_gemm_kernel(
    const uint8_t* __restrict__ A, int lda, int M, int K,
    const uint8_t* __restrict__ X, size_t ldx,
    uint8_t* __restrict__ Y, size_t ldy, int ncols, int nx, int ny, int nbuf, int accum,
    GemmGroup xg, size_t a_gstride, size_t y_gstride) {
  static_assert(S == 1 || S == 2 || S == 4, "lane groups");
  static_assert(RC % (S * P) == 0, "ring: P row-steps of S rows must divide RC");
  constexpr int KC = KW * RC;
  constexpr int NT = 64 * KW;
  constexpr int GL = 64 / S;             // lanes per group
  constexpr int CB = GL * kLaneBytes;    // chunk bytes
  constexpr int STEPS = RC / S;          // row-steps per wave per K-chunk
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint4* tab01 = reinterpret_cast<uint4*>(smem);                         // [nbuf][KC][MT]
  uint32_t* tab2 = reinterpret_cast<uint32_t*>(tab01 + nbuf * KC * MT);  // [nbuf][KC][MT]
  uint32_t* red = tab2 + nbuf * KC * MT;                                  // [MT][4][GL]

  // XCD-aware block order: blocks b and b+8 share an XCD under round-robin
  // dispatch, so the ny row-tiles of one column chunk are dealt to one XCD
  // back to back and re-read that chunk from its L2.  Speed only.
  const int b = blockIdx.x;
  const int ty = (b >> 3) % ny;
  const int tx = (b / (8 * ny)) * 8 + (b & 7);
  if (tx >= nx) return;
  const int m0 = ty * MT;
  if (gridDim.y > 1) {
    const int gi = blockIdx.y;
    X = xg.x[gi];
    A += (size_t)gi * a_gstride;
    Y += (size_t)gi * y_gstride;
  }

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int g = lane / GL;
  const int li = lane % GL;
  const int col = tx * CB + li * kLaneBytes;

  // X through a buffer descriptor: rows k >= K lie outside num_records and
  // load as zero, so the stream needs no branches (columns >= ncols are
  // loaded but never stored).
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, (int)((size_t)K * ldx), 0x00020000);
  const int ildx = (int)ldx;
  // row-step q of this wave (flat over K-chunks) -> row index of group g
  auto row_of = [&](int q) { return (q / STEPS) * KC + w * RC + (q % STEPS) * S + g; };
  auto load_step = [&](int q) -> uint4 {
    if (MODE == 2) {  // tuning: no memory traffic
      const uint32_t h = (uint32_t)(row_of(q) * 0x9E3779B1u) ^ (uint32_t)col;
      return make_uint4(h, h * 3u, h * 5u, h * 7u);
    }
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(xr, row_of(q) * ildx + col, 0, AUX);
    return make_uint4(v[0], v[1], v[2], v[3]);
  };

  // Coefficient tables of one K-chunk: thread t builds entries t + j*NT of the
  // (KC x MT) chunk.  Loading and building are split so that chunk 0's
  // coefficient bytes are requested BEFORE the row ring: vmcnt retires loads
  // in issue order, so waiting for the coefficients then does not wait for the
  // HBM-latency rows, and table building overlaps the row stream.
  constexpr int NB = (KC * MT + NT - 1) / NT;
  auto load_coefs = [&](int c, uint32_t (&cf)[NB]) {
#pragma unroll
    for (int j = 0; j < NB; j++) {
      const int idx = tid + j * NT;
      const int kk = idx / MT, m = idx % MT;
      const int k = c * KC + kk, mm = m0 + m;
      cf[j] = (idx < KC * MT && k < K && mm < M) ? A[(size_t)mm * lda + k] : 0u;
    }
  };
  auto store_tables = [&](int buf, const uint32_t (&cf)[NB]) {
#pragma unroll
    for (int j = 0; j < NB; j++) {
      const int idx = tid + j * NT;
      if (idx < KC * MT) {
        uint4 t01;
        uint32_t t2;
        gf_make_tables(cf[j], t01, t2);
        tab01[buf * KC * MT + idx] = t01;
        tab2[buf * KC * MT + idx] = t2;
      }
    }
  };

  uint32_t cf[NB];
  load_coefs(0, cf);
  __builtin_amdgcn_sched_barrier(0);
  uint4 ring[P];
#pragma unroll
  for (int j = 0; j < P; j++) ring[j] = load_step(j);
  __builtin_amdgcn_sched_barrier(0);
  store_tables(0, cf);
  if (KW > 1)
    for (int i = tid; i < MT * 4 * GL; i += NT) red[i] = 0u;

  uint32_t acc[MT][4];
#pragma unroll
  for (int m = 0; m < MT; m++)
#pragma unroll
    for (int d = 0; d < 4; d++) acc[m][d] = 0u;

  const int nchunks = (K + KC - 1) / KC;
  lds_barrier();

  for (int c = 0; c < nchunks; c++) {
    if (c + 1 < nchunks) {
      uint32_t cn[NB];
      load_coefs(c + 1, cn);
      store_tables((c + 1) % nbuf, cn);
    }
    const uint4* t01c = tab01 + (c % nbuf) * KC * MT;
    const uint32_t* t2c = tab2 + (c % nbuf) * KC * MT;
    for (int jj = 0; jj < STEPS; jj += P) {
#pragma unroll
      for (int j = 0; j < P; j += 2) {
        // two row-steps per iteration so every v_bitop3 (XOR3) absorbs two products
        const int q = c * STEPS + jj + j;
        const uint4 xa = ring[j], xb = ring[j + 1];
        ring[j] = load_step(q + P);
        ring[j + 1] = load_step(q + 1 + P);
        if (MODE == 1) {  // tuning: no GF arithmetic
          acc[0][0] ^= xa.x ^ xb.x;
          acc[0][1] ^= xa.y ^ xb.y;
          acc[0][2] ^= xa.z ^ xb.z;
          acc[0][3] ^= xa.w ^ xb.w;
          continue;
        }
        const uint32_t x[8] = {xa.x, xa.y, xa.z, xa.w, xb.x, xb.y, xb.z, xb.w};
        uint32_t s0[8], s1[8], s2[8];
#pragma unroll
        for (int d = 0; d < 8; d++) {
          s0[d] = x[d] & 0x07070707u;
          s1[d] = (x[d] >> 3) & 0x07070707u;
          s2[d] = (x[d] >> 6) & 0x03030303u;
        }
        const int kka = w * RC + (jj + j) * S + g;
        const int kkb = kka + S;
#pragma unroll
        for (int m = 0; m < MT; m++) {
          const uint4 ta = t01c[kka * MT + m];
          const uint32_t ta2 = t2c[kka * MT + m];
          const uint4 tb = t01c[kkb * MT + m];
          const uint32_t tb2 = t2c[kkb * MT + m];
#pragma unroll
          for (int d = 0; d < 4; d++) {
            const uint32_t a0 = __builtin_amdgcn_perm(ta.y, ta.x, s0[d]);
            const uint32_t a1 = __builtin_amdgcn_perm(ta.w, ta.z, s1[d]);
            const uint32_t a2 = __builtin_amdgcn_perm(ta2, ta2, s2[d]);
            const uint32_t b0 = __builtin_amdgcn_perm(tb.y, tb.x, s0[d + 4]);
            const uint32_t b1 = __builtin_amdgcn_perm(tb.w, tb.z, s1[d + 4]);
            const uint32_t b2 = __builtin_amdgcn_perm(tb2, tb2, s2[d + 4]);
            uint32_t a = __builtin_amdgcn_bitop3_b32(acc[m][d], a0, a1, 0x96);
            a = __builtin_amdgcn_bitop3_b32(a, a2, b0, 0x96);
            acc[m][d] = __builtin_amdgcn_bitop3_b32(a, b1, b2, 0x96);
          }
        }
      }
    }
    lds_barrier();  // (a conditional barrier here makes hipcc spill heavily)
  }

  // reduce across the S lane groups (each holds other rows of the same columns)
  if (S > 1) {
#pragma unroll
    for (int m = 0; m < MT; m++)
#pragma unroll
      for (int d = 0; d < 4; d++) {
        uint32_t v = acc[m][d];
        if (S >= 4) {
          const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);  // lane ^ 16
          v = r[0] ^ r[1];
        }
        const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);    // lane ^ 32
        acc[m][d] = r[0] ^ r[1];
      }
  }

  auto store16 = [&](int row, int cc, uint4 v) {
    if (row >= M || cc >= ncols) return;
    uint8_t* dst = Y + (size_t)row * ldy + cc;
    if (cc + kLaneBytes <= ncols) {
      if (accum) {  // a later row chunk of a K-split product: Y ^= this chunk's part
        const uint4 o = *reinterpret_cast<const uint4*>(dst);
        v = make_uint4(v.x ^ o.x, v.y ^ o.y, v.z ^ o.z, v.w ^ o.w);
      }
      *reinterpret_cast<uint4*>(dst) = v;
    } else {
      const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
      for (int i = 0; cc + i < ncols; i++)
        dst[i] = (uint8_t)(vv[i >> 2] >> (8 * (i & 3))) ^ (accum ? dst[i] : (uint8_t)0);
    }
  };

  if (KW == 1) {
    if (g == 0) {
#pragma unroll
      for (int m = 0; m < MT; m++)
        store16(m0 + m, col, make_uint4(acc[m][0], acc[m][1], acc[m][2], acc[m][3]));
    }
    return;
  }

  // XOR-reduce the KW per-wave partial sums of each (m, column) in LDS
  if (g == 0) {
#pragma unroll
    for (int m = 0; m < MT; m++)
#pragma unroll
      for (int d = 0; d < 4; d++) atomicXor(&red[(m * 4 + d) * GL + li], acc[m][d]);
  }
  lds_barrier();
  for (int i = tid; i < MT * GL; i += NT) {
    const int m = i / GL, l = i % GL;
    const uint4 v = make_uint4(red[(m * 4 + 0) * GL + l], red[(m * 4 + 1) * GL + l],
                               red[(m * 4 + 2) * GL + l], red[(m * 4 + 3) * GL + l]);
    store16(m0 + m, tx * CB + l * kLaneBytes, v);
  }
}

// One coded piece per launch (M = 1: full/encoder.go:61-71 called once), the
// streaming shape.  A workgroup owns one column chunk (S lane groups of 64/S
// lanes x 16 B, each group reading its own row per step: a 1024/S-byte chunk)
// and all K rows, split over KW waves of RPW rows; the coefficient and then
// every row load of a wave are issued before anything else.  Unlike
// gf_gemm_kernel there are no LDS tables and no barrier before the first
// multiply: the tables are built in registers from the coefficients while the
// rows are in flight (SHT: lane r for row r, fetched per step by ds_bpermute),
// so a step costs only its multiply once its row lands, and the tail after
// the last row is short.
// Partial sums: lane groups by v_permlane16/32_swap, waves through one LDS
// slot each and a single barrier (no atomics, nothing to zero).
// SHT: the tables are built once per row, by the lane that holds the row's
// coefficient, and each lane group fetches its row's five table dwords with
// ds_bpermute (5 crossbar reads per step instead of ~45 VALU per row per lane).
template <int KW, int RPW, int S, int AUX = 0, bool SHT = false>
__global__ __launch_bounds__(64 * KW) void gf_gemv_kernel(const uint8_t* __restrict__ A, int K,
                                                          const uint8_t* __restrict__ X, size_t ldx,
                                                          uint8_t* __restrict__ Y, int ncols, int accum) {
  static_assert(RPW % S == 0 && (S == 2 || S == 4), "S rows per step");
  constexpr int STEPS = RPW / S;
  constexpr int GL = 64 / S;              // lanes per group
  constexpr int CB = GL * kLaneBytes;     // chunk bytes
  __shared__ uint4 part[KW][GL];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane / GL, li = lane % GL;
  const int col = blockIdx.x * CB + li * kLaneBytes;
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, (int)((size_t)K * ldx), 0x00020000);
  const int ildx = (int)ldx;
  const int r0 = w * RPW;
  // lane i < RPW holds the coefficient of row r0 + i (0 past K), requested
  // first: vmcnt retires in issue order, so the tables wait for it alone
  const uint32_t cv = (lane < RPW && r0 + lane < K) ? (uint32_t)A[r0 + lane] : 0u;
  __builtin_amdgcn_sched_barrier(0);
  u32x4 ring[STEPS];
#pragma unroll
  for (int j = 0; j < STEPS; j++)
    ring[j] = __builtin_amdgcn_raw_buffer_load_b128(xr, (r0 + S * j + g) * ildx + col, 0, AUX);
  __builtin_amdgcn_sched_barrier(0);
  uint4 t01[STEPS];
  uint32_t t2[STEPS];
  if constexpr (SHT) {
    uint4 m01;
    uint32_t m2;
    gf_make_tables(cv, m01, m2);  // lane r: row r0 + r (zero tables past K and RPW)
#pragma unroll
    for (int j = 0; j < STEPS; j++) {
      const int src = (S * j + g) * 4;  // byte address of the lane holding row S j + g
      t01[j].x = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)m01.x);
      t01[j].y = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)m01.y);
      t01[j].z = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)m01.z);
      t01[j].w = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)m01.w);
      t2[j] = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)m2);
    }
  } else {
#pragma unroll
    for (int j = 0; j < STEPS; j++) {
      uint32_t c = __builtin_amdgcn_readlane(cv, S * j);
#pragma unroll
      for (int q = 1; q < S; q++) c = g == q ? __builtin_amdgcn_readlane(cv, S * j + q) : c;
      gf_make_tables(c, t01[j], t2[j]);
    }
  }
  // every table before the first row wait: otherwise the scheduler mixes the
  // first steps' multiplies into the table build and waits for rows 0 and 1
  // before building the rest (~400 VALU on the critical path)
  __builtin_amdgcn_sched_barrier(0);
  uint32_t acc[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int j = 0; j < STEPS; j++) {
    const u32x4 x = ring[j];
#pragma unroll
    for (int d = 0; d < 4; d++) {
      const uint32_t s0 = x[d] & 0x07070707u, s1 = (x[d] >> 3) & 0x07070707u, s2 = (x[d] >> 6) & 0x03030303u;
      const uint32_t a0 = __builtin_amdgcn_perm(t01[j].y, t01[j].x, s0);
      const uint32_t a1 = __builtin_amdgcn_perm(t01[j].w, t01[j].z, s1);
      const uint32_t a2 = __builtin_amdgcn_perm(t2[j], t2[j], s2);
      acc[d] = __builtin_amdgcn_bitop3_b32(acc[d], a0, a1, 0x96) ^ a2;
    }
  }
#pragma unroll
  for (int d = 0; d < 4; d++) {
    uint32_t v = acc[d];
    if (S == 4) {
      const auto r = __builtin_amdgcn_permlane16_swap(v, v, false, false);  // lane ^ 16
      v = r[0] ^ r[1];
    }
    const auto r = __builtin_amdgcn_permlane32_swap(v, v, false, false);    // lane ^ 32
    acc[d] = r[0] ^ r[1];
  }
  if (g == 0) part[w][li] = make_uint4(acc[0], acc[1], acc[2], acc[3]);
  __syncthreads();
  if (tid >= GL) return;
  uint4 v = part[0][tid];
#pragma unroll
  for (int q = 1; q < KW; q++) {
    const uint4 p = part[q][tid];
    v = make_uint4(v.x ^ p.x, v.y ^ p.y, v.z ^ p.z, v.w ^ p.w);
  }
  const int cc = blockIdx.x * CB + tid * kLaneBytes;
  if (cc >= ncols) return;
  uint8_t* dst = Y + cc;
  if (cc + kLaneBytes <= ncols) {
    if (accum) {
      const uint4 o = *reinterpret_cast<const uint4*>(dst);
      v = make_uint4(v.x ^ o.x, v.y ^ o.y, v.z ^ o.z, v.w ^ o.w);
    }
    *reinterpret_cast<uint4*>(dst) = v;
  } else {
    const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
    for (int i = 0; cc + i < ncols; i++) dst[i] = (uint8_t)(vv[i >> 2] >> (8 * (i & 3))) ^ (accum ? dst[i] : (uint8_t)0);
  }
}

// gf_gemv_kernel for M <= MT output rows (two coded pieces of one generation
// per call; MT = 2 is the instance used): the same stream -- 16 waves x 16 rows, every row load
// issued first -- and the same shared tables, one set per output row: lane r
// builds the MT table sets of row r0 + r, each step fetches its MT sets by
// ds_bpermute, and a data dword's selectors serve all MT rows.  Rows >= M
// have coefficient 0 and are not stored.
template <int MT>
__global__ __launch_bounds__(1024) void gf_gemv_multi_kernel(const uint8_t* __restrict__ A, int lda, int M, int K,
                                                             const uint8_t* __restrict__ X, size_t ldx,
                                                             uint8_t* __restrict__ Y, size_t ldy, int ncols,
                                                             int accum) {
  constexpr int KW = 16, RPW = 16, S = 2, STEPS = RPW / S, GL = 64 / S, CB = GL * kLaneBytes;
  __shared__ uint4 part[KW][MT][GL];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int g = lane / GL, li = lane % GL;
  const int col = blockIdx.x * CB + li * kLaneBytes;
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, (int)((size_t)K * ldx), 0x00020000);
  const int ildx = (int)ldx;
  const int r0 = w * RPW;
  uint32_t cv[MT];
#pragma unroll
  for (int m = 0; m < MT; m++)
    cv[m] = (lane < RPW && r0 + lane < K && m < M) ? (uint32_t)A[(size_t)m * lda + r0 + lane] : 0u;
  __builtin_amdgcn_sched_barrier(0);
  u32x4 ring[STEPS];
#pragma unroll
  for (int j = 0; j < STEPS; j++)
    ring[j] = __builtin_amdgcn_raw_buffer_load_b128(xr, (r0 + S * j + g) * ildx + col, 0, 0);
  __builtin_amdgcn_sched_barrier(0);
  uint4 m01[MT];
  uint32_t m2[MT];
#pragma unroll
  for (int m = 0; m < MT; m++) gf_make_tables(cv[m], m01[m], m2[m]);
  __builtin_amdgcn_sched_barrier(0);
  uint32_t acc[MT][4];
#pragma unroll
  for (int m = 0; m < MT; m++)
#pragma unroll
    for (int d = 0; d < 4; d++) acc[m][d] = 0u;
#pragma unroll
  for (int j = 0; j < STEPS; j++) {
    const int src = (S * j + g) * 4;
    uint4 t01[MT];
    uint32_t t2[MT];
#pragma unroll
    for (int m = 0; m < MT; m++) {
      t01[m].x = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)m01[m].x);
      t01[m].y = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)m01[m].y);
      t01[m].z = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)m01[m].z);
      t01[m].w = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)m01[m].w);
      t2[m] = (uint32_t)__builtin_amdgcn_ds_bpermute(src, (int)m2[m]);
    }
    const u32x4 x = ring[j];
#pragma unroll
    for (int d = 0; d < 4; d++) {
      const uint32_t s0 = x[d] & 0x07070707u, s1 = (x[d] >> 3) & 0x07070707u, s2 = (x[d] >> 6) & 0x03030303u;
#pragma unroll
      for (int m = 0; m < MT; m++) {
        const uint32_t a0 = __builtin_amdgcn_perm(t01[m].y, t01[m].x, s0);
        const uint32_t a1 = __builtin_amdgcn_perm(t01[m].w, t01[m].z, s1);
        const uint32_t a2 = __builtin_amdgcn_perm(t2[m], t2[m], s2);
        acc[m][d] = __builtin_amdgcn_bitop3_b32(acc[m][d], a0, a1, 0x96) ^ a2;
      }
    }
  }
#pragma unroll
  for (int m = 0; m < MT; m++)
#pragma unroll
    for (int d = 0; d < 4; d++) {
      const auto r = __builtin_amdgcn_permlane32_swap(acc[m][d], acc[m][d], false, false);  // lane ^ 32
      acc[m][d] = r[0] ^ r[1];
    }
  if (g == 0)
#pragma unroll
    for (int m = 0; m < MT; m++) part[w][m][li] = make_uint4(acc[m][0], acc[m][1], acc[m][2], acc[m][3]);
  __syncthreads();
  if (tid >= MT * GL) return;
  const int m = tid / GL, l = tid % GL;
  if (m >= M) return;
  uint4 v = part[0][m][l];
#pragma unroll
  for (int q = 1; q < KW; q++) {
    const uint4 p = part[q][m][l];
    v = make_uint4(v.x ^ p.x, v.y ^ p.y, v.z ^ p.z, v.w ^ p.w);
  }
  const int cc = blockIdx.x * CB + l * kLaneBytes;
  if (cc >= ncols) return;
  uint8_t* dst = Y + (size_t)m * ldy + cc;
  if (cc + kLaneBytes <= ncols) {
    if (accum) {
      const uint4 o = *reinterpret_cast<const uint4*>(dst);
      v = make_uint4(v.x ^ o.x, v.y ^ o.y, v.z ^ o.z, v.w ^ o.w);
    }
    *reinterpret_cast<uint4*>(dst) = v;
  } else {
    const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
    for (int i = 0; cc + i < ncols; i++) dst[i] = (uint8_t)(vv[i >> 2] >> (8 * (i & 3))) ^ (accum ? dst[i] : (uint8_t)0);
  }
}

// One product, or (grp != nullptr) grp->n products of the same shape in one launch.
template <int MT, int KW, int S, int RC, int P, int MODE = 0, int AUX = 0>
hipError_t launch(const uint8_t* A, int lda, int M, int K, const uint8_t* X, size_t ldx,
                  uint8_t* Y, size_t ldy, int ncols, hipStream_t stream, int accum = 0,
                  const GemmGroupArgs* grp = nullptr) {
  constexpr int KC = KW * RC;
  constexpr int CB = 1024 / S;
  const int nx = (ncols + CB - 1) / CB;
  const int ny = (M + MT - 1) / MT;
  const int nbuf = K > KC ? 2 : 1;
  const int nx8 = (nx + 7) / 8 * 8;
  const size_t lds = (size_t)nbuf * KC * MT * (16 + 4) + (KW > 1 ? (size_t)MT * 4 * (64 / S) * 4 : 0);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  GemmGroup xg{};
  size_t as = 0, ys = 0;
  unsigned ng = 1;
  if (grp) {
    if (grp->n < 1 || grp->n > kGemmGroupMax) return hipErrorInvalidValue;
    for (int i = 0; i < grp->n; i++) xg.x[i] = grp->x[i];
    as = grp->a_stride;
    ys = grp->y_stride;
    ng = (unsigned)grp->n;
  }
  hipLaunchKernelGGL((gf_gemm_kernel<MT, KW, S, RC, P, MODE, AUX>), dim3(nx8 * ny, ng), dim3(64 * KW), lds, stream,
                     A, lda, M, K, X, ldx, Y, ldy, ncols, nx, ny, nbuf, accum, xg, as, ys);
  last_launch_plan() = LaunchPlan{1, MT, KW, S, P, RC, (int)ng, nx8 * ny};
  return hipGetLastError();
}

// dst row r = bytes [0, ncols) of the device row src[r] (16-byte aligned rows);
// dst row r is dtab[r] when a destination table is given (a scatter into the
// caller's generation buffer), else dst + r * dpitch.  Used where a row of the
// product is a plain copy: unit rows of the decode transform (systematic
// pieces) and gathers of GEMM scratch rows.
// 8x8 bit transpose inside each byte lane of 8 dwords (gf_bs.hip bitslice32:
// the bit-sliced twin <-> plain bytes, an involution)
__device__ __forceinline__ void unslice32(uint32_t (&d)[8]) {
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

// A source pointer with bit 0 set names a row of a bit-sliced twin (a compact
// decoder's received row, 32-byte blocks, ncols a multiple of 32): the lane
// pair of each block swaps halves (DPP), un-slices the block and stores its
// half of the plain bytes.  The tag is per row (blockIdx.y): uniform.
__global__ __launch_bounds__(256) void gather_rows_kernel(const uint8_t* const* __restrict__ src,
                                                         uint8_t* const* __restrict__ dtab,
                                                         uint8_t* __restrict__ dst, size_t dpitch,
                                                         int ncols) {
  const int r = blockIdx.y;
  const int c = (blockIdx.x * 256 + threadIdx.x) * kLaneBytes;
  if (c >= ncols) return;
  const uintptr_t sp = reinterpret_cast<uintptr_t>(src[r]);
  const uint8_t* s = reinterpret_cast<const uint8_t*>(sp & ~(uintptr_t)1) + c;
  uint8_t* d = (dtab ? dtab[r] : dst + (size_t)r * dpitch) + c;
  if (sp & 1) {  // twin row: both lanes of a block are live (ncols % 32 == 0)
    const uint4 a = *reinterpret_cast<const uint4*>(s);
    const uint32_t ox = (uint32_t)__builtin_amdgcn_mov_dpp((int)a.x, 0xb1, 0xf, 0xf, false);
    const uint32_t oy = (uint32_t)__builtin_amdgcn_mov_dpp((int)a.y, 0xb1, 0xf, 0xf, false);
    const uint32_t oz = (uint32_t)__builtin_amdgcn_mov_dpp((int)a.z, 0xb1, 0xf, 0xf, false);
    const uint32_t ow = (uint32_t)__builtin_amdgcn_mov_dpp((int)a.w, 0xb1, 0xf, 0xf, false);
    const bool lo = ((c / kLaneBytes) & 1) == 0;
    uint32_t v[8];
    if (lo) {
      v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = ox; v[5] = oy; v[6] = oz; v[7] = ow;
    } else {
      v[0] = ox; v[1] = oy; v[2] = oz; v[3] = ow; v[4] = a.x; v[5] = a.y; v[6] = a.z; v[7] = a.w;
    }
    unslice32(v);
    *reinterpret_cast<uint4*>(d) = lo ? make_uint4(v[0], v[1], v[2], v[3]) : make_uint4(v[4], v[5], v[6], v[7]);
    return;
  }
  if (c + kLaneBytes <= ncols) {
    *reinterpret_cast<uint4*>(d) = *reinterpret_cast<const uint4*>(s);
  } else {
    for (int i = 0; c + i < ncols; i++) d[i] = s[i];
  }
}

}  // namespace

namespace {

// dst (pitch dpitch) = width x rows bytes read straight from host-mapped
// pinned memory (contiguous rows).  Small uploads only: a kernel's reads over
// PCIe start with the dispatch, where a DMA engine's copy is followed by a
// ~11 us cross-engine wait before the next kernel (profiles/r01/upload.log).
__global__ __launch_bounds__(256) void upload_small_kernel(const uint8_t* __restrict__ src,
                                                          uint8_t* __restrict__ dst, size_t dpitch,
                                                          int width, int total) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int r = i / width, c = i - r * width;
  dst[(size_t)r * dpitch + c] = src[i];
}

// the reverse: dst (host-mapped pinned, contiguous rows) = width x rows bytes
// of device memory at pitch spitch
__global__ __launch_bounds__(256) void download_small_kernel(const uint8_t* __restrict__ src, size_t spitch,
                                                            uint8_t* __restrict__ dst, int width, int total) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= total) return;
  const int r = i / width, c = i - r * width;
  dst[i] = src[(size_t)r * spitch + c];
}

}  // namespace

hipError_t download_small(const uint8_t* src, size_t spitch, uint8_t* dst_mapped, size_t width, size_t rows,
                          hipStream_t stream) {
  if (!width || !rows) return hipSuccess;
  const size_t total = width * rows;
  if (total > kDownloadSmallMax) return hipErrorInvalidValue;
  hipLaunchKernelGGL(download_small_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, src,
                     spitch, dst_mapped, (int)width, (int)total);
  return hipGetLastError();
}

hipError_t upload_small(const uint8_t* src_mapped, uint8_t* dst, size_t dpitch, size_t width, size_t rows,
                        hipStream_t stream) {
  if (!width || !rows) return hipSuccess;
  const size_t total = width * rows;
  if (total > kUploadSmallMax) return hipErrorInvalidValue;
  hipLaunchKernelGGL(upload_small_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, src_mapped,
                     dst, dpitch, (int)width, (int)total);
  return hipGetLastError();
}

namespace {

// dst row r = bytes [0, ncols) of src row r (both device, any pitch): 16 B
// per lane where both rows allow it, bytes otherwise
__global__ __launch_bounds__(256) void copy_rows_kernel(const uint8_t* __restrict__ src, size_t spitch,
                                                       uint8_t* __restrict__ dst, size_t dpitch, int ncols,
                                                       int vec) {
  const int r = blockIdx.y;
  const int c = (blockIdx.x * 256 + threadIdx.x) * kLaneBytes;
  if (c >= ncols) return;
  const uint8_t* s = src + (size_t)r * spitch + c;
  uint8_t* d = dst + (size_t)r * dpitch + c;
  if (vec && c + kLaneBytes <= ncols) {
    *reinterpret_cast<uint4*>(d) = *reinterpret_cast<const uint4*>(s);
  } else {
    for (int i = 0; i < kLaneBytes && c + i < ncols; i++) d[i] = s[i];
  }
}

}  // namespace

hipError_t copy_rows(const uint8_t* src, size_t spitch, uint8_t* dst, size_t dpitch, size_t rows, size_t ncols,
                     hipStream_t stream) {
  if (!rows || !ncols) return hipSuccess;
  if (rows > 65535 || ncols > 0x7fffffff) return hipErrorInvalidValue;
  const int vec = ((uintptr_t)src % 16 == 0 && (uintptr_t)dst % 16 == 0 && spitch % 16 == 0 && dpitch % 16 == 0);
  const unsigned gx = (unsigned)((ncols + 256 * kLaneBytes - 1) / (256 * kLaneBytes));
  hipLaunchKernelGGL(copy_rows_kernel, dim3(gx, (unsigned)rows), dim3(256), 0, stream, src, spitch, dst, dpitch,
                     (int)ncols, vec);
  return hipGetLastError();
}

hipError_t gather_rows(const uint8_t* const* d_src, uint8_t* dY, size_t ldy, size_t rows, size_t ncols,
                       hipStream_t stream, uint8_t* const* d_dst) {
  if (!rows || !ncols) return hipSuccess;
  if (rows > 65535) return hipErrorInvalidValue;
  const unsigned gx = (unsigned)((ncols + 256 * kLaneBytes - 1) / (256 * kLaneBytes));
  hipLaunchKernelGGL(gather_rows_kernel, dim3(gx, (unsigned)rows), dim3(256), 0, stream, d_src, d_dst, dY,
                     ldy, (int)ncols);
  return hipGetLastError();
}

namespace {

// Coding vectors drawn on the device: byte j of vector row r is
// the low byte of splitmix64(seed + (row0 + r) * 2^32 + j); rows r < n_sys are
// the unit vectors e_(sys_first + r) of a systematic encoder's first k pieces
// (systematic/encoder.go:60-68).  Uniform bytes, zeros allowed, like
// GenerateCodingVector (data.go:90-95); not a cryptographic generator.
__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(256) void fill_vectors_kernel(uint8_t* __restrict__ V, size_t ldv, int k,
                                                          uint64_t seed, uint64_t row0, int n_sys,
                                                          int sys_first) {
  const int r = blockIdx.y;
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= k) return;
  uint8_t b;
  if (r < n_sys) b = (j == sys_first + r) ? 1 : 0;
  else b = (uint8_t)splitmix64(seed + ((row0 + (uint64_t)r) << 32) + (uint64_t)j);
  V[(size_t)r * ldv + j] = b;
}

// fill_vectors_kernel for several encoders at once (blockIdx.z = encoder)
__global__ __launch_bounds__(256) void fill_vectors_grouped_kernel(VectorGroup g, size_t ldv, int k) {
  const int e = blockIdx.z, r = blockIdx.y;
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= k) return;
  uint8_t b;
  if (r < g.n_sys[e]) b = (j == g.sys_first[e] + r) ? 1 : 0;
  else b = (uint8_t)splitmix64(g.seed[e] + ((g.row0[e] + (uint64_t)r) << 32) + (uint64_t)j);
  g.v[e][(size_t)r * ldv + j] = b;
}

}  // namespace

hipError_t fill_vectors_grouped(const VectorGroup& g, int n, size_t ldv, size_t rows, size_t k, hipStream_t stream) {
  if (!rows || !k || n <= 0) return hipSuccess;
  if (n > kGemmGroupMax || rows > 65535 || k > (1u << 30)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(fill_vectors_grouped_kernel, dim3((unsigned)((k + 255) / 256), (unsigned)rows, (unsigned)n),
                     dim3(256), 0, stream, g, ldv, (int)k);
  return hipGetLastError();
}

hipError_t fill_vectors(uint8_t* dV, size_t ldv, size_t rows, size_t k, uint64_t seed, uint64_t row0,
                        size_t n_sys, size_t sys_first, hipStream_t stream) {
  if (!rows || !k) return hipSuccess;
  if (rows > 65535 || k > (1u << 30)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(fill_vectors_kernel, dim3((unsigned)((k + 255) / 256), (unsigned)rows), dim3(256), 0,
                     stream, dV, ldv, (int)k, seed, row0, (int)n_sys, (int)sys_first);
  return hipGetLastError();
}

namespace {

}  // namespace

// Tiles measured on MI355X at K = 256, ncols = 128 KiB (tools/tune_gemm.py).
// Every tile stages K-chunks of 256 rows; for K > 256 the tables are
// double-buffered (2 x 256 x MT x 20 B of LDS), which rules out MT = 16.
GemmConfig choose_gemm_config(size_t M, size_t K, size_t ncols) {
  // Few rows of X: the K-splitting tiles below give each of their waves 16-32
  // rows, so with small K most waves of a workgroup idle.  One wave per
  // workgroup running all K rows wastes nothing but needs many column chunks
  // (512 B each) to fill the chip; output rows are split over row tiles until
  // there are >= 1024 workgroups.  Where each side wins was measured over
  // K = 16-200, L = 64 KiB-4 MiB, M = 1-8 (tools/sweep_fewrows*.sh,
  // profiles/r01/sweep_fewrows*.log): K <= 32 always; K <= 64 from 128 KiB
  // rows (from 64 KiB for M >= 4); K <= 128 from 256 KiB rows; not at K = 200.
  // The rule also takes more than 8 output rows (8-row tiles, each re-reading
  // X from L2).  Timed there only at M <= 32, K = 16-128, 128 KiB and 1 MiB
  // rows (tools/bs_vs_gemm_small_k.py, profiles/r01/bs_vs_gemm_small_k.log);
  // callers with M >= 9 normally take the bit-sliced kernel instead
  // (capi_internal.hpp kBsMinRows, few_narrow_rows), so larger M reaches this only
  // where that kernel cannot take the shape.
  const size_t nxc = (ncols + 511) / 512;
  if (K <= 32 || (K <= 64 && (M >= 4 || nxc >= 256)) || (K <= 128 && nxc >= 512)) {
    int mt = M <= 1 ? 1 : M <= 2 ? 2 : M <= 4 ? 4 : 8;
    while (mt > 1 && nxc * ((M + mt - 1) / mt) < 1024) mt /= 2;
    return {mt, 1, 2, 8};
  }
  // Narrow products (a recoder's coding-vector columns r x C, ncols = k):
  // 256-byte column chunks (S = 4) with 16 waves splitting K, output rows
  // split over row tiles until there are >= 128 workgroups.  The wide-row
  // tiles below would leave one or two workgroups per 8 output rows running
  // all of K (M = 32, K = 256, 256 columns: ~25 us).
  if (ncols <= 1024 && K >= 64) {
    const size_t nx = (ncols + 255) / 256;
    int mt = 8;
    while (mt > 1 && nx * ((M + mt - 1) / mt) < 128) mt /= 2;
    return {mt, 16, 4, 4};
  }
  if (K > 256 && M > 8 && M <= 16) return {8, 16, 2, 2};
  if (M <= 1) return {1, 16, 2, 0};
  if (M <= 2) return {2, 16, 2, 0};
  if (M <= 4) return {4, 8, 2, 4};
  if (M <= 8) return {8, 16, 2, 2};
  if (M <= 16) return {16, 8, 2, 2};
  return {8, 4, 1, 4};
}

// Grouped launches (G generations of one shape per launch) stream: every
// workgroup owns a 1 KiB column chunk of one generation and its waves run long
// row sequences through a deep ring of nt loads.  Measured at K = 256, 128 KiB
// rows (tools/group_sweep.py, profiles/r02/group_sweep*.log): one coded piece
// per generation 5.3-5.5 us per 32 MiB generation (6.1-6.3 TB/s) with one wave
// per workgroup for G >= 8, 5.5 us with 8 waves splitting K for G = 4, against
// 6.4-6.9 us on the single-launch tile {1, 16, 2}; 2-8 pieces per generation
// 10-30 % faster on 4-wave tiles.
GemmConfig choose_group_config(size_t M, size_t K, size_t ncols, size_t G) {
  if (K < 64) return choose_gemm_config(M, K, ncols);
  if (M <= 1) return G >= 8 ? GemmConfig{1, 1, 1, 16} : GemmConfig{1, 8, 1, 8};
  if (M <= 2) return {2, 4, 1, 8};
  if (M <= 4) return {4, 4, 1, 8};
  if (M <= 8) return {8, 4, 1, 8};
  return choose_gemm_config(M, K, ncols);
}

// KODR_GEMM_CFG="mt,kw,s" forces a tile (tuning runs only; see tools/tune_gemm.py)
static bool env_config(GemmConfig* g) {
  const char* s = tune_env("KODR_GEMM_CFG");
  if (!s || !*s) return false;
  g->p = 0;
  return sscanf(s, "%d,%d,%d,%d", &g->mt, &g->kw, &g->s, &g->p) >= 3;
}

// One-row products of 129..256 input rows take gf_gemv_kernel (two lane
// groups, tables shared through ds_bpermute): 7.56 us per 32 MiB/256 coded
// piece in rocprof against 8.20 with per-lane tables and 9.4 on
// gf_gemm_kernel<1, 16, 2> (profiles/r03/b1/, profiles/r03/gemv_ab/); 512
// workgroups of 8 waves (four lane groups) or 256 of 8 waves (16 rows in
// flight per lane) measured 7.88 / 8.80.  KODR_GEMV=0 selects gf_gemm_kernel,
// 1 the per-lane tables (A/B measurements).
static int gemv_enabled() {
  static const int v = tune_env("KODR_GEMV") ? atoi(tune_env("KODR_GEMV")) : 2;
  return v;
}

// Two rows on gf_gemv_multi_kernel: 9.1 against 10.4 us at 32 MiB/256
// (profiles/r03/gemv_multi_ab/); four measured 11.8 against 11.0 on
// gf_gemm_kernel (20 ds_bpermute per step), so 3-8 rows stay there.
// KODR_GEMV_MULTI=0 keeps gf_gemm_kernel for two rows too (A/B).
static bool gemv_multi_enabled() {
  static const bool v = tune_env("KODR_GEMV_MULTI") ? atoi(tune_env("KODR_GEMV_MULTI")) != 0 : true;
  return v;
}

hipError_t gf_gemm(const uint8_t* dA, size_t lda, size_t M, size_t K, const uint8_t* dX,
                   size_t ldx, uint8_t* dY, size_t ldy, size_t ncols, hipStream_t stream,
                   const GemmConfig* force, bool accumulate, const GemmGroupArgs* grp) {
  const int acc = accumulate ? 1 : 0;
  if (M == 0 || ncols == 0) return hipSuccess;
  // one coded piece of a generation of up to 256 rows, wide rows: the
  // streaming kernel (row offsets of all 256 lanes' rows fit 31 bits)
  constexpr int kGemvKW = 16, kGemvRPW = 16;
  const int gemv = gemv_enabled();
  if (M == 2 && !grp && !force && K > (size_t)kGemvKW * kGemvRPW / 2 && K <= (size_t)kGemvKW * kGemvRPW &&
      ncols >= 16384 && (size_t)kGemvKW * kGemvRPW * ldx < ((size_t)1 << 31) && gemv_multi_enabled()) {
    const int nx = (int)((ncols + 511) / 512);
    hipLaunchKernelGGL(gf_gemv_multi_kernel<2>, dim3(nx), dim3(1024), 0, stream, dA, (int)lda, (int)M, (int)K, dX,
                       ldx, dY, ldy, (int)ncols, acc);
    last_launch_plan() = LaunchPlan{3, 2, kGemvKW, 2, kGemvRPW / 2, kGemvRPW, 1, nx};
    return hipGetLastError();
  }
  if (M == 1 && !grp && !force && K > (size_t)kGemvKW * kGemvRPW / 2 && K <= (size_t)kGemvKW * kGemvRPW &&
      ncols >= 16384 &&
      (size_t)kGemvKW * kGemvRPW * ldx < ((size_t)1 << 31) && gemv) {
    const int nx = (int)((ncols + 511) / 512);
    if (gemv == 1)
      hipLaunchKernelGGL((gf_gemv_kernel<kGemvKW, kGemvRPW, 2>), dim3(nx), dim3(64 * kGemvKW), 0, stream, dA, (int)K,
                         dX, ldx, dY, (int)ncols, acc);
    else
      hipLaunchKernelGGL((gf_gemv_kernel<kGemvKW, kGemvRPW, 2, 0, true>), dim3(nx), dim3(64 * kGemvKW), 0, stream, dA,
                         (int)K, dX, ldx, dY, (int)ncols, acc);
    last_launch_plan() = LaunchPlan{3, 1, kGemvKW, 2, kGemvRPW / 2, kGemvRPW, 1, nx};
    return hipGetLastError();
  }
  GemmConfig g = force ? *force : grp ? choose_group_config(M, K, ncols, (size_t)grp->n)
                                      : choose_gemm_config(M, K, ncols);
  GemmConfig ge;
  if (!force && env_config(&ge)) g = ge;
  const int iM = (int)M, iK = (int)K, ild = (int)lda, inc = (int)ncols;
  int mode = 0;
#ifdef KODR_TUNE_MODES
  if (const char* e = tune_env("KODR_GEMM_MODE")) mode = atoi(e);
  if (mode == 1 && g.mt == 8 && g.kw == 16 && g.s == 2)
    return launch<8, 16, 2, 16, 2, 1>(dA, ild, iM, iK, dX, ldx, dY, ldy, inc, stream);
  if (mode == 2 && g.mt == 8 && g.kw == 16 && g.s == 2)
    return launch<8, 16, 2, 16, 2, 2>(dA, ild, iM, iK, dX, ldx, dY, ldy, inc, stream);
  if (mode == 1 && g.mt == 4 && g.kw == 8 && g.s == 2)
    return launch<4, 8, 2, 32, 8, 1>(dA, ild, iM, iK, dX, ldx, dY, ldy, inc, stream);
  if (mode == 2 && g.mt == 4 && g.kw == 8 && g.s == 2)
    return launch<4, 8, 2, 32, 8, 2>(dA, ild, iM, iK, dX, ldx, dY, ldy, inc, stream);
  if (mode == 2 && g.mt == 8 && g.kw == 4 && g.s == 1)
    return launch<8, 4, 1, 64, 8, 2>(dA, ild, iM, iK, dX, ldx, dY, ldy, inc, stream);
  if (mode == 1 && g.mt == 1 && g.kw == 16 && g.s == 2)
    return launch<1, 16, 2, 16, 8, 1>(dA, ild, iM, iK, dX, ldx, dY, ldy, inc, stream);
  if (mode == 2 && g.mt == 1 && g.kw == 16 && g.s == 2)
    return launch<1, 16, 2, 16, 8, 2>(dA, ild, iM, iK, dX, ldx, dY, ldy, inc, stream);
#endif
  (void)mode;
  // grouped launches stream G generations once each per launch: nt loads
  // (KODR_GROUP_AUX in tuning builds)
  int aux = grp ? kGroupAux : 0;
#ifdef KODR_TUNE_MODES
  if (const char* e = tune_env("KODR_GROUP_AUX")) aux = atoi(e);
#endif
#define KODR_TRY(MT_, KW_, S_, RC_, P_)                                                         \
  if (g.mt == MT_ && g.kw == KW_ && g.s == S_ && (g.p == 0 || g.p == P_))                       \
    return aux == 2 ? launch<MT_, KW_, S_, RC_, P_, 0, 2>(dA, ild, iM, iK, dX, ldx, dY, ldy, inc, stream, acc, grp) \
                    : launch<MT_, KW_, S_, RC_, P_>(dA, ild, iM, iK, dX, ldx, dY, ldy, inc, stream, acc, grp);
  // streaming tiles for grouped launches of few rows (one 1 KiB column chunk
  // per workgroup, long per-wave row runs through a deep ring)
  KODR_TRY(1, 4, 1, 64, 8)
  KODR_TRY(1, 4, 1, 64, 16)
  KODR_TRY(1, 2, 1, 128, 16)
  KODR_TRY(1, 1, 1, 256, 16)
  KODR_TRY(1, 8, 1, 32, 8)
  KODR_TRY(1, 8, 2, 32, 16)
  KODR_TRY(2, 4, 1, 64, 8)
  KODR_TRY(4, 4, 1, 64, 8)
  KODR_TRY(1, 1, 2, 16, 8)
  KODR_TRY(2, 1, 2, 16, 8)
  KODR_TRY(4, 1, 2, 16, 8)
  KODR_TRY(8, 1, 2, 16, 8)
  KODR_TRY(1, 16, 4, 16, 4)
  KODR_TRY(1, 16, 2, 16, 8)
  KODR_TRY(1, 16, 1, 16, 8)
  KODR_TRY(2, 16, 4, 16, 4)
  KODR_TRY(2, 16, 2, 16, 8)
  KODR_TRY(4, 16, 4, 16, 4)
  KODR_TRY(4, 16, 2, 16, 8)
  KODR_TRY(4, 16, 1, 16, 8)
  KODR_TRY(8, 16, 4, 16, 4)
  KODR_TRY(8, 16, 2, 16, 8)
  KODR_TRY(8, 8, 2, 32, 8)
  KODR_TRY(8, 8, 2, 32, 4)
  KODR_TRY(8, 8, 2, 32, 2)
  KODR_TRY(8, 16, 2, 16, 4)
  KODR_TRY(8, 16, 2, 16, 2)
  KODR_TRY(8, 16, 4, 16, 2)
  KODR_TRY(8, 8, 4, 32, 4)
  KODR_TRY(4, 8, 2, 32, 4)
  KODR_TRY(16, 8, 2, 32, 2)
  KODR_TRY(8, 4, 1, 64, 4)
  KODR_TRY(4, 8, 2, 32, 8)
  KODR_TRY(8, 8, 4, 32, 8)
  KODR_TRY(16, 8, 2, 32, 4)
  KODR_TRY(8, 4, 1, 64, 8)
  KODR_TRY(16, 4, 1, 64, 4)
  KODR_TRY(8, 4, 2, 64, 8)
  KODR_TRY(16, 4, 2, 64, 4)
#undef KODR_TRY
  return hipErrorInvalidValue;
}

}  // namespace kodr_amd
