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

#include "gf_kernels.hpp"

namespace kodr_amd {

namespace {

__device__ __forceinline__ uint32_t xt(uint32_t c) {  // multiply by x (=2) mod 0x11D
  return ((c << 1) ^ ((c & 0x80u) ? 0x1Du : 0u)) & 0xFFu;
}

// T0 = c*{0..7}, T1 = c*{0..7}<<3, T2 = c*{0..3}<<6, little-endian bytes.
__device__ __forceinline__ void make_tables(uint32_t c, uint4& t01, uint32_t& t2) {
  const uint32_t c1 = c, c2 = xt(c1), c4 = xt(c2), c8 = xt(c4);
  const uint32_t c16 = xt(c8), c32 = xt(c16), c64 = xt(c32), c128 = xt(c64);
  const uint32_t lo0 = (c1 << 8) | (c2 << 16) | ((c1 ^ c2) << 24);
  const uint32_t lo1 = (c8 << 8) | (c16 << 16) | ((c8 ^ c16) << 24);
  t01.x = lo0;
  t01.y = lo0 ^ (c4 * 0x01010101u);
  t01.z = lo1;
  t01.w = lo1 ^ (c32 * 0x01010101u);
  t2 = (c64 << 8) | (c128 << 16) | ((c64 ^ c128) << 24);
}

constexpr int kLanes = 64;
constexpr int kLaneBytes = 16;                    // one dwordx4 per lane per row
constexpr int kChunkBytes = kLanes * kLaneBytes;  // 1 KiB of columns per wave

// Workgroup barrier that waits only for LDS traffic: HIP's __syncthreads()
// also drains vmcnt, which would empty the row-prefetch ring at every K-chunk.
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

__device__ __forceinline__ uint4 zero4() { return make_uint4(0u, 0u, 0u, 0u); }

// One workgroup = CW column chunks x KW K-slices, one wave each, MT output rows.
//  - KW > 1 (encode/recode, small M): KW waves share one 1 KiB column chunk and
//    split every K-chunk of KC = KW*RC rows; partial sums are XOR-reduced in LDS.
//  - CW > 1 (decode, large M): CW waves own CW adjacent column chunks and
//    share the coefficient tables of the MT rows.
// Coefficient tables are staged per K-chunk into LDS (double-buffered when
// K > KC) and read back as wave-uniform broadcasts.  Each wave streams its rows
// through a P-deep ring of dwordx4 loads that runs across K-chunk barriers.
template <int MT, int KW, int CW, int RC, int P>
__global__ __launch_bounds__(64 * KW * CW) void gf_gemm_kernel(
    const uint8_t* __restrict__ A, int lda, int M, int K,
    const uint8_t* __restrict__ X, size_t ldx,
    uint8_t* __restrict__ Y, size_t ldy, int ncols, int nx, int ny, int nbuf) {
  static_assert(KW == 1 || CW == 1, "split K or columns, not both");
  static_assert(RC % P == 0 && P % 2 == 0, "ring depth: even, divides rows per chunk");
  constexpr int KC = KW * RC;
  constexpr int NT = 64 * KW * CW;
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint4* tab01 = reinterpret_cast<uint4*>(smem);                         // [nbuf][KC][MT]
  uint32_t* tab2 = reinterpret_cast<uint32_t*>(tab01 + nbuf * KC * MT);  // [nbuf][KC][MT]
  uint32_t* red = tab2 + nbuf * KC * MT;                                  // [MT][4][64]

  // XCD-aware block order: blocks b and b+8 share an XCD under round-robin
  // dispatch, so the ny row-tiles of one column group are dealt to one XCD
  // back to back and re-read those columns from its L2.  Speed only.
  const int b = blockIdx.x;
  const int ty = (b >> 3) % ny;
  const int tx = (b / (8 * ny)) * 8 + (b & 7);
  if (tx >= nx) return;
  const int m0 = ty * MT;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int w = tid >> 6;
  const int kw = (KW > 1) ? w : 0;
  const int cw = (CW > 1) ? w : 0;
  const int col = (tx * CW + cw) * kChunkBytes + lane * kLaneBytes;

  auto build = [&](int c, int buf) {
    for (int idx = tid; idx < KC * MT; idx += NT) {
      const int kk = idx / MT, m = idx - kk * MT;
      const int k = c * KC + kk, mm = m0 + m;
      const uint32_t coef = (k < K && mm < M) ? A[(size_t)mm * lda + k] : 0u;
      uint4 t01;
      uint32_t t2;
      make_tables(coef, t01, t2);
      tab01[(buf * KC + kk) * MT + m] = t01;
      tab2[(buf * KC + kk) * MT + m] = t2;
    }
  };
  // row q of this wave's flat sequence -> matrix row k.  X is read through a
  // buffer descriptor: rows k >= K fall outside num_records and load as zero,
  // so the stream needs no branches (columns >= ncols are loaded but never
  // stored).
  const __amdgpu_buffer_rsrc_t xr =
      __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, (int)((size_t)K * ldx), 0x00020000);
  const int ildx = (int)ldx;
  auto load_row = [&](int q) -> uint4 {
    const int k = (q / RC) * KC + kw * RC + (q % RC);
    const auto v = __builtin_amdgcn_raw_buffer_load_b128(xr, k * ildx + col, 0, 0);
    return make_uint4(v[0], v[1], v[2], v[3]);
  };

  uint32_t acc[MT][4];
#pragma unroll
  for (int m = 0; m < MT; m++)
#pragma unroll
    for (int d = 0; d < 4; d++) acc[m][d] = 0u;

  if (KW > 1)
    for (int i = tid; i < MT * 4 * 64; i += NT) red[i] = 0u;

  const int nchunks = (K + KC - 1) / KC;
  uint4 ring[P];
#pragma unroll
  for (int j = 0; j < P; j++) ring[j] = load_row(j);
  build(0, 0);
  lds_barrier();

  for (int c = 0; c < nchunks; c++) {
    if (c + 1 < nchunks) build(c + 1, (c + 1) % nbuf);
    const uint4* t01c = tab01 + (c % nbuf) * KC * MT;
    const uint32_t* t2c = tab2 + (c % nbuf) * KC * MT;
    for (int jj = 0; jj < RC; jj += P) {
#pragma unroll
      for (int j = 0; j < P; j += 2) {
        // two rows per step so every v_bitop3 (XOR3) absorbs two products
        const int q = c * RC + jj + j;
        const uint4 xa = ring[j], xb = ring[j + 1];
        ring[j] = load_row(q + P);
        ring[j + 1] = load_row(q + 1 + P);
        const uint32_t x[8] = {xa.x, xa.y, xa.z, xa.w, xb.x, xb.y, xb.z, xb.w};
        uint32_t s0[8], s1[8], s2[8];
#pragma unroll
        for (int d = 0; d < 8; d++) {
          s0[d] = x[d] & 0x07070707u;
          s1[d] = (x[d] >> 3) & 0x07070707u;
          s2[d] = (x[d] >> 6) & 0x03030303u;
        }
        const int kk = kw * RC + jj + j;
#pragma unroll
        for (int m = 0; m < MT; m++) {
          const uint4 ta = t01c[kk * MT + m];
          const uint32_t ta2 = t2c[kk * MT + m];
          const uint4 tb = t01c[(kk + 1) * MT + m];
          const uint32_t tb2 = t2c[(kk + 1) * MT + m];
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
    lds_barrier();
  }

  auto store16 = [&](int row, int cc, uint4 v) {
    if (row >= M || cc >= ncols) return;
    uint8_t* dst = Y + (size_t)row * ldy + cc;
    if (cc + kLaneBytes <= ncols) {
      *reinterpret_cast<uint4*>(dst) = v;
    } else {
      const uint32_t vv[4] = {v.x, v.y, v.z, v.w};
      for (int i = 0; cc + i < ncols; i++) dst[i] = (uint8_t)(vv[i >> 2] >> (8 * (i & 3)));
    }
  };

  if (KW == 1) {
#pragma unroll
    for (int m = 0; m < MT; m++)
      store16(m0 + m, col, make_uint4(acc[m][0], acc[m][1], acc[m][2], acc[m][3]));
    return;
  }

  // XOR-reduce the KW partial sums of each (m, lane) in LDS.
#pragma unroll
  for (int m = 0; m < MT; m++)
#pragma unroll
    for (int d = 0; d < 4; d++) atomicXor(&red[(m * 4 + d) * 64 + lane], acc[m][d]);
  lds_barrier();
  for (int i = tid; i < MT * 64; i += NT) {
    const int m = i >> 6, l = i & 63;
    const uint4 v = make_uint4(red[(m * 4 + 0) * 64 + l], red[(m * 4 + 1) * 64 + l],
                               red[(m * 4 + 2) * 64 + l], red[(m * 4 + 3) * 64 + l]);
    store16(m0 + m, tx * kChunkBytes + l * kLaneBytes, v);
  }
}

template <int MT, int KW, int CW, int RC, int P>
hipError_t launch(const uint8_t* A, int lda, int M, int K, const uint8_t* X, size_t ldx,
                  uint8_t* Y, size_t ldy, int ncols, hipStream_t stream) {
  constexpr int KC = KW * RC;
  const int nchunk = (ncols + kChunkBytes - 1) / kChunkBytes;
  const int nx = (nchunk + CW - 1) / CW;
  const int ny = (M + MT - 1) / MT;
  const int nbuf = K > KC ? 2 : 1;
  const int nx8 = (nx + 7) / 8 * 8;
  const size_t lds = (size_t)nbuf * KC * MT * (16 + 4) + (KW > 1 ? (size_t)MT * 4 * 64 * 4 : 0);
  hipLaunchKernelGGL((gf_gemm_kernel<MT, KW, CW, RC, P>), dim3(nx8 * ny), dim3(64 * KW * CW), lds,
                     stream, A, lda, M, K, X, ldx, Y, ldy, ncols, nx, ny, nbuf);
  return hipGetLastError();
}

}  // namespace

GemmConfig choose_gemm_config(size_t M, size_t K, size_t ncols) {
  (void)K;
  (void)ncols;
  if (M <= 1) return {1, 16, 1};
  if (M <= 2) return {2, 16, 1};
  if (M <= 4) return {4, 16, 1};
  if (M <= 8) return {4, 16, 1};
  if (M <= 16) return {8, 16, 1};
  return {16, 1, 4};
}

hipError_t gf_gemm(const uint8_t* dA, size_t lda, size_t M, size_t K, const uint8_t* dX,
                   size_t ldx, uint8_t* dY, size_t ldy, size_t ncols, hipStream_t stream,
                   const GemmConfig* force) {
  if (M == 0 || ncols == 0) return hipSuccess;
  const GemmConfig g = force ? *force : choose_gemm_config(M, K, ncols);
  const int iM = (int)M, iK = (int)K, ild = (int)lda, inc = (int)ncols;
#define KODR_TRY(MT_, KW_, CW_, RC_, P_)                                              \
  if (g.mt == MT_ && g.kw == KW_ && g.cw == CW_)                                      \
    return launch<MT_, KW_, CW_, RC_, P_>(dA, ild, iM, iK, dX, ldx, dY, ldy, inc, stream);
  KODR_TRY(1, 16, 1, 16, 8)
  KODR_TRY(2, 16, 1, 16, 8)
  KODR_TRY(4, 16, 1, 16, 8)
  KODR_TRY(8, 16, 1, 16, 8)
  KODR_TRY(4, 4, 1, 16, 8)
  KODR_TRY(8, 1, 4, 32, 4)
  KODR_TRY(16, 1, 4, 32, 4)
#undef KODR_TRY
  return hipErrorInvalidValue;
}

}  // namespace kodr_amd
