// host_gf.hpp -- GF(2^8) row operations on the host, used only on the
// coefficient side of the decoder (k x (k + received) bytes: the small matrix
// whose elimination decides pivots; piece data never goes through here).
// Field: kodr's gf256.go:15-44 (poly 0x11D, generator 2).
#pragma once
#include <stddef.h>
#include <stdint.h>
#include <string.h>

#if defined(__x86_64__)
#include <immintrin.h>
#endif

namespace kodr_amd {
namespace hostgf {

struct Tables {
  uint8_t log[256];
  uint8_t exp[512];
  uint8_t mul_lo[256][16];  // c * n       for nibble n (pshufb table)
  uint8_t mul_hi[256][16];  // c * (n<<4)
  uint64_t affine[256];     // GF2P8AFFINEQB bit-matrix of x -> c * x (poly 0x11D)
  Tables() {
    unsigned x = 1;
    for (int i = 0; i < 255; i++) {
      exp[i] = (uint8_t)x;
      log[x] = (uint8_t)i;
      x <<= 1;
      if (x & 0x100) x ^= 0x11D;
    }
    for (int i = 255; i < 512; i++) exp[i] = exp[i - 255];
    log[0] = 0;
    for (int c = 0; c < 256; c++)
      for (int n = 0; n < 16; n++) {
        mul_lo[c][n] = mul(c, n);
        mul_hi[c][n] = mul(c, n << 4);
      }
    // affine: result bit i = parity(matrix.byte[7 - i] & x); multiply-by-c is
    // GF(2)-linear, column j of its matrix is c * 2^j
    for (int c = 0; c < 256; c++) {
      uint64_t m = 0;
      for (int i = 0; i < 8; i++) {
        unsigned row = 0;
        for (int j = 0; j < 8; j++)
          if (mul(c, 1u << j) & (1u << i)) row |= 1u << j;
        m |= (uint64_t)row << (8 * (7 - i));
      }
      affine[c] = m;
    }
  }
  uint8_t mul(unsigned a, unsigned b) const {  // gf256.go:109-118
    if (a == 0 || b == 0) return 0;
    return exp[log[a] + log[b]];
  }
  uint8_t inv(unsigned a) const { return exp[255 - log[a]]; }  // gf256.go:77-86, a != 0
  uint8_t div(unsigned a, unsigned b) const { return mul(a, inv(b)); }  // gf256.go:121-127
};

inline const Tables& T() {
  static const Tables t;
  return t;
}

#if defined(__x86_64__)
__attribute__((target("avx2"))) inline void axpy_avx2(uint8_t* dst, const uint8_t* src, size_t n,
                                                       uint8_t q) {
  const Tables& t = T();
  const __m256i lo = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i*)t.mul_lo[q]));
  const __m256i hi = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i*)t.mul_hi[q]));
  const __m256i m = _mm256_set1_epi8(0x0f);
  size_t i = 0;
  for (; i + 32 <= n; i += 32) {
    const __m256i x = _mm256_loadu_si256((const __m256i*)(src + i));
    const __m256i p = _mm256_xor_si256(_mm256_shuffle_epi8(lo, _mm256_and_si256(x, m)),
                                       _mm256_shuffle_epi8(hi, _mm256_and_si256(_mm256_srli_epi16(x, 4), m)));
    _mm256_storeu_si256((__m256i*)(dst + i),
                        _mm256_xor_si256(_mm256_loadu_si256((const __m256i*)(dst + i)), p));
  }
  for (; i < n; i++) dst[i] ^= t.mul(src[i], q);
}
__attribute__((target("avx2"))) inline void scale_avx2(uint8_t* row, size_t n, uint8_t q) {
  const Tables& t = T();
  const __m256i lo = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i*)t.mul_lo[q]));
  const __m256i hi = _mm256_broadcastsi128_si256(_mm_loadu_si128((const __m128i*)t.mul_hi[q]));
  const __m256i m = _mm256_set1_epi8(0x0f);
  size_t i = 0;
  for (; i + 32 <= n; i += 32) {
    const __m256i x = _mm256_loadu_si256((const __m256i*)(row + i));
    _mm256_storeu_si256((__m256i*)(row + i),
                        _mm256_xor_si256(_mm256_shuffle_epi8(lo, _mm256_and_si256(x, m)),
                                         _mm256_shuffle_epi8(hi, _mm256_and_si256(_mm256_srli_epi16(x, 4), m))));
  }
  for (; i < n; i++) row[i] = t.mul(row[i], q);
}
inline bool have_avx2() {
  static const bool h = __builtin_cpu_supports("avx2");
  return h;
}
// GFNI + AVX-512: one vgf2p8affineqb multiplies 64 bytes by a constant
__attribute__((target("avx512f,avx512bw,gfni"))) inline void axpy_gfni512(uint8_t* dst, const uint8_t* src,
                                                                         size_t n, uint8_t q) {
  const __m512i A = _mm512_set1_epi64((long long)T().affine[q]);
  size_t i = 0;
  for (; i + 64 <= n; i += 64) {
    const __m512i x = _mm512_loadu_si512((const void*)(src + i));
    const __m512i p = _mm512_gf2p8affine_epi64_epi8(x, A, 0);
    _mm512_storeu_si512((void*)(dst + i), _mm512_xor_si512(_mm512_loadu_si512((const void*)(dst + i)), p));
  }
  if (i < n) {
    const __mmask64 k = (__mmask64)(~0ULL >> (64 - (n - i)));
    const __m512i x = _mm512_maskz_loadu_epi8(k, src + i);
    const __m512i d = _mm512_maskz_loadu_epi8(k, dst + i);
    _mm512_mask_storeu_epi8(dst + i, k, _mm512_xor_si512(d, _mm512_gf2p8affine_epi64_epi8(x, A, 0)));
  }
}
__attribute__((target("avx512f,avx512bw,gfni"))) inline void scale_gfni512(uint8_t* row, size_t n, uint8_t q) {
  const __m512i A = _mm512_set1_epi64((long long)T().affine[q]);
  size_t i = 0;
  for (; i + 64 <= n; i += 64)
    _mm512_storeu_si512((void*)(row + i),
                        _mm512_gf2p8affine_epi64_epi8(_mm512_loadu_si512((const void*)(row + i)), A, 0));
  if (i < n) {
    const __mmask64 k = (__mmask64)(~0ULL >> (64 - (n - i)));
    _mm512_mask_storeu_epi8(row + i, k, _mm512_gf2p8affine_epi64_epi8(_mm512_maskz_loadu_epi8(k, row + i), A, 0));
  }
}
__attribute__((target("avx512f,avx512bw"))) inline bool all_zero512(const uint8_t* p, size_t n) {
  __m512i acc = _mm512_setzero_si512();
  size_t i = 0;
  for (; i + 64 <= n; i += 64) acc = _mm512_or_si512(acc, _mm512_loadu_si512((const void*)(p + i)));
  if (i < n) acc = _mm512_or_si512(acc, _mm512_maskz_loadu_epi8((__mmask64)(~0ULL >> (64 - (n - i))), p + i));
  return _mm512_test_epi64_mask(acc, acc) == 0;
}
inline bool have_gfni512() {
  static const bool h = __builtin_cpu_supports("gfni") && __builtin_cpu_supports("avx512bw") &&
                        __builtin_cpu_supports("avx512f");
  return h;
}
#endif

#if defined(__x86_64__)
// v[0..n) ^= XOR_i q[i] * rows[i][0..n): up to 8 x 64 B of v stay in
// registers while every contributing row streams through once
template <int NB>
__attribute__((target("avx512f,avx512bw,gfni"))) inline void accumulate_blk(
    uint8_t* v, const uint8_t* const* rows, const uint8_t* q, size_t nrows, size_t off, size_t w) {
  const Tables& t = T();
  __m512i acc[NB];
  __mmask64 km[NB];
#pragma GCC unroll 8
  for (int b = 0; b < NB; b++) {
    const size_t o = (size_t)b * 64, ww = w - o < 64 ? w - o : 64;
    km[b] = (__mmask64)(~0ULL >> (64 - ww));
    acc[b] = _mm512_maskz_loadu_epi8(km[b], v + off + o);
  }
  for (size_t r = 0; r < nrows; r++) {
    if (!q[r]) continue;
    const __m512i A = _mm512_set1_epi64((long long)t.affine[q[r]]);
    const uint8_t* src = rows[r] + off;
#pragma GCC unroll 8
    for (int b = 0; b < NB; b++)
      acc[b] = _mm512_xor_si512(acc[b], _mm512_gf2p8affine_epi64_epi8(
                                            _mm512_maskz_loadu_epi8(km[b], src + b * 64), A, 0));
  }
#pragma GCC unroll 8
  for (int b = 0; b < NB; b++) _mm512_mask_storeu_epi8(v + off + b * 64, km[b], acc[b]);
}
inline void accumulate_gfni512(uint8_t* v, const uint8_t* const* rows, const uint8_t* q, size_t nrows,
                               size_t n) {
  for (size_t off = 0; off < n; off += 512) {
    const size_t w = n - off < 512 ? n - off : 512;
    switch ((w + 63) / 64) {
      case 1: accumulate_blk<1>(v, rows, q, nrows, off, w); break;
      case 2: accumulate_blk<2>(v, rows, q, nrows, off, w); break;
      case 3: accumulate_blk<3>(v, rows, q, nrows, off, w); break;
      case 4: accumulate_blk<4>(v, rows, q, nrows, off, w); break;
      case 5: accumulate_blk<5>(v, rows, q, nrows, off, w); break;
      case 6: accumulate_blk<6>(v, rows, q, nrows, off, w); break;
      case 7: accumulate_blk<7>(v, rows, q, nrows, off, w); break;
      default: accumulate_blk<8>(v, rows, q, nrows, off, w); break;
    }
  }
}

// rows[j][0..n) ^= q[j] * v[0..n) for every j (rank-1 update); v is held in
// registers, one pass over each row
__attribute__((target("avx512f,avx512bw,gfni"))) inline void rank1_gfni512(
    uint8_t* const* rows, const uint8_t* q, size_t nrows, const uint8_t* v, size_t n) {
  const Tables& t = T();
  for (size_t i0 = 0; i0 < n; i0 += 256) {  // 4 registers of v at a time
    const size_t w = n - i0 < 256 ? n - i0 : 256;
    __mmask64 km[4];
    __m512i vb[4];
    for (int b = 0; b < 4; b++) {
      const size_t o = (size_t)b * 64;
      const size_t ww = w > o ? (w - o < 64 ? w - o : 64) : 0;
      km[b] = ww ? (__mmask64)(~0ULL >> (64 - ww)) : (__mmask64)0;
      vb[b] = _mm512_maskz_loadu_epi8(km[b], v + i0 + o);
    }
    for (size_t r = 0; r < nrows; r++) {
      if (!q[r]) continue;
      const __m512i A = _mm512_set1_epi64((long long)t.affine[q[r]]);
      uint8_t* dst = rows[r] + i0;
      for (int b = 0; b < 4; b++) {
        if (!km[b]) break;
        const __m512i d = _mm512_maskz_loadu_epi8(km[b], dst + b * 64);
        _mm512_mask_storeu_epi8(dst + b * 64, km[b],
                                _mm512_xor_si512(d, _mm512_gf2p8affine_epi64_epi8(vb[b], A, 0)));
      }
    }
  }
}
#endif

#if defined(__x86_64__)
// v[p][0..n) ^= XOR_i q[p * ldq + i] * rows[i][0..n) for p < P: every block of
// a source row is loaded once for all P outputs (256 B of each output in
// registers at a time)
template <int P>
__attribute__((target("avx512f,avx512bw,gfni"))) inline void accumulate_multi_gfni512(
    uint8_t* const* v, const uint8_t* const* rows, const uint8_t* q, size_t ldq, size_t nrows, size_t n) {
  const Tables& t = T();
  for (size_t i0 = 0; i0 < n; i0 += 256) {
    __mmask64 km[4];
    for (int b = 0; b < 4; b++) {
      const size_t o = i0 + (size_t)b * 64;
      km[b] = o >= n ? (__mmask64)0 : (__mmask64)(~0ULL >> (64 - (n - o < 64 ? n - o : 64)));
    }
    __m512i acc[P][4];
#pragma GCC unroll 4
    for (int p = 0; p < P; p++)
#pragma GCC unroll 4
      for (int b = 0; b < 4; b++) acc[p][b] = _mm512_maskz_loadu_epi8(km[b], v[p] + i0 + b * 64);
    for (size_t r = 0; r < nrows; r++) {
      const uint8_t* src = rows[r] + i0;
      __m512i x[4];
#pragma GCC unroll 4
      for (int b = 0; b < 4; b++) x[b] = _mm512_maskz_loadu_epi8(km[b], src + b * 64);
#pragma GCC unroll 4
      for (int p = 0; p < P; p++) {
        const uint8_t c = q[p * ldq + r];
        if (!c) continue;
        const __m512i A = _mm512_set1_epi64((long long)t.affine[c]);
#pragma GCC unroll 4
        for (int b = 0; b < 4; b++) acc[p][b] = _mm512_xor_si512(acc[p][b], _mm512_gf2p8affine_epi64_epi8(x[b], A, 0));
      }
    }
#pragma GCC unroll 4
    for (int p = 0; p < P; p++)
#pragma GCC unroll 4
      for (int b = 0; b < 4; b++) _mm512_mask_storeu_epi8(v[p] + i0 + b * 64, km[b], acc[p][b]);
  }
}

// rows[j][0..n) ^= XOR_p q[j * P + p] * v[p][0..n) for every j (rank-P
// update): each destination block is loaded and stored once for all P sources
template <int P>
__attribute__((target("avx512f,avx512bw,gfni"))) inline void rank_multi_gfni512(
    uint8_t* const* rows, const uint8_t* q, size_t nrows, const uint8_t* const* v, size_t n) {
  const Tables& t = T();
  for (size_t i0 = 0; i0 < n; i0 += 256) {
    __mmask64 km[4];
    for (int b = 0; b < 4; b++) {
      const size_t o = i0 + (size_t)b * 64;
      km[b] = o >= n ? (__mmask64)0 : (__mmask64)(~0ULL >> (64 - (n - o < 64 ? n - o : 64)));
    }
    __m512i vb[P][4];
#pragma GCC unroll 4
    for (int p = 0; p < P; p++)
#pragma GCC unroll 4
      for (int b = 0; b < 4; b++) vb[p][b] = _mm512_maskz_loadu_epi8(km[b], v[p] + i0 + b * 64);
    for (size_t j = 0; j < nrows; j++) {
      const uint8_t* qj = q + j * P;
      bool any = false;
      __m512i A[P];
#pragma GCC unroll 4
      for (int p = 0; p < P; p++) {
        A[p] = _mm512_set1_epi64((long long)t.affine[qj[p]]);  // affine[0] = 0: a zero term
        any = any || qj[p];
      }
      if (!any) continue;
      uint8_t* dst = rows[j] + i0;
#pragma GCC unroll 4
      for (int b = 0; b < 4; b++) {
        if (!km[b]) break;
        __m512i d = _mm512_maskz_loadu_epi8(km[b], dst + b * 64);
#pragma GCC unroll 4
        for (int p = 0; p < P; p++) d = _mm512_xor_si512(d, _mm512_gf2p8affine_epi64_epi8(vb[p][b], A[p], 0));
        _mm512_mask_storeu_epi8(dst + b * 64, km[b], d);
      }
    }
  }
}

// 32-byte vectors (the panel pivot search of solve_full_batch)
__attribute__((target("avx2,gfni"))) inline void axpy32(uint8_t* dst, const uint8_t* src, uint8_t q) {
  const __m256i A = _mm256_set1_epi64x((long long)T().affine[q]);
  const __m256i x = _mm256_loadu_si256((const __m256i*)src);
  _mm256_storeu_si256((__m256i*)dst, _mm256_xor_si256(_mm256_loadu_si256((const __m256i*)dst),
                                                      _mm256_gf2p8affine_epi64_epi8(x, A, 0)));
}
__attribute__((target("avx2,gfni"))) inline void scale32(uint8_t* v, uint8_t q) {
  const __m256i A = _mm256_set1_epi64x((long long)T().affine[q]);
  _mm256_storeu_si256((__m256i*)v, _mm256_gf2p8affine_epi64_epi8(_mm256_loadu_si256((const __m256i*)v), A, 0));
}

// One 64-byte column chunk [o, o + w) of a blocked Gauss-Jordan step
// (decoder_core.cpp, solve_full_batch): the nb picked rows brow[q] become
// N[bpiv[q]] = sum_u S[q][u] * (picked row u), and every row i that is not
// picked (cur[i] < 0) gets row_i ^= sum_c row_i[jb + c] * N[c] (the panel
// bytes at jb, left of every chunk the caller passes, are read here and never
// written).  N stays in registers; the multiply-by-q matrices are broadcast
// from the table (on the box's EPYC this chunk-by-chunk order beat a
// row-by-row one with the matrices in registers and N in memory: 80 vs
// 91 us at k = 256).
template <int NB>
__attribute__((target("avx512f,avx512bw,gfni"))) inline void panel_update(
    uint8_t* const* rows, size_t k, size_t o, size_t w, size_t jb, const int32_t* brow, const int* bpiv,
    const uint8_t (*S)[NB], int nb, const int16_t* cur) {
  const Tables& t = T();
  const __mmask64 km = (__mmask64)(~0ULL >> (64 - w));
  __m512i P[NB];
  alignas(64) __m512i Nm[NB];
  for (int q = 0; q < nb; q++) P[q] = _mm512_maskz_loadu_epi8(km, rows[brow[q]] + o);
  for (int c = 0; c < NB; c++) Nm[c] = _mm512_setzero_si512();
  for (int q = 0; q < nb; q++) {
    __m512i acc = _mm512_setzero_si512();
    for (int u = 0; u < nb; u++)
      if (S[q][u])
        acc = _mm512_xor_si512(acc, _mm512_gf2p8affine_epi64_epi8(P[u], _mm512_set1_epi64((long long)t.affine[S[q][u]]), 0));
    Nm[bpiv[q]] = acc;
  }
  __m512i N[NB];
#pragma GCC unroll 16
  for (int c = 0; c < NB; c++) N[c] = Nm[c];
  const uint64_t* aff = t.affine;
  for (size_t i = 0; i < k; i++) {
    if (cur[i] >= 0) continue;
    uint8_t* row = rows[i];
    const uint8_t* qi = row + jb;
    uint8_t* dst = row + o;
    __m512i d0 = _mm512_maskz_loadu_epi8(km, dst), d1 = _mm512_setzero_si512();
#pragma GCC unroll 16
    for (int c = 0; c < NB; c += 2) {
      const __m512i a0 = _mm512_gf2p8affine_epi64_epi8(N[c], _mm512_set1_epi64((long long)aff[qi[c]]), 0);
      const __m512i a1 = _mm512_gf2p8affine_epi64_epi8(N[c + 1], _mm512_set1_epi64((long long)aff[qi[c + 1]]), 0);
      if (c & 2) d1 = _mm512_ternarylogic_epi64(d1, a0, a1, 0x96);
      else d0 = _mm512_ternarylogic_epi64(d0, a0, a1, 0x96);
    }
    _mm512_mask_storeu_epi8(dst, km, _mm512_xor_si512(d0, d1));
  }
  for (int q = 0; q < nb; q++) _mm512_mask_storeu_epi8(rows[brow[q]] + o, km, Nm[bpiv[q]]);
}
#endif

// dst[0..n) ^= q * src[0..n)
inline void axpy(uint8_t* dst, const uint8_t* src, size_t n, uint8_t q) {
  if (q == 0 || n == 0) return;
#if defined(__x86_64__)
  if (have_gfni512()) return axpy_gfni512(dst, src, n, q);
  if (have_avx2()) return axpy_avx2(dst, src, n, q);
#endif
  const Tables& t = T();
  for (size_t i = 0; i < n; i++) dst[i] ^= t.mul(src[i], q);
}

// row[0..n) *= q
inline void scale(uint8_t* row, size_t n, uint8_t q) {
#if defined(__x86_64__)
  if (have_gfni512()) return scale_gfni512(row, n, q);
  if (have_avx2()) return scale_avx2(row, n, q);
#endif
  const Tables& t = T();
  for (size_t i = 0; i < n; i++) row[i] = t.mul(row[i], q);
}

// v[0..n) ^= XOR_i q[i] * rows[i][0..n)
inline void accumulate(uint8_t* v, const uint8_t* const* rows, const uint8_t* q, size_t nrows, size_t n) {
#if defined(__x86_64__)
  if (have_gfni512()) return accumulate_gfni512(v, rows, q, nrows, n);
#endif
  for (size_t r = 0; r < nrows; r++) axpy(v, rows[r], n, q[r]);
}

// rows[j][0..n) ^= q[j] * v[0..n)
inline void rank1(uint8_t* const* rows, const uint8_t* q, size_t nrows, const uint8_t* v, size_t n) {
#if defined(__x86_64__)
  if (have_gfni512()) return rank1_gfni512(rows, q, nrows, v, n);
#endif
  for (size_t r = 0; r < nrows; r++) axpy(rows[r], v, n, q[r]);
}

// v[p][0..n) ^= XOR_i q[p * ldq + i] * rows[i][0..n), p < np (np <= 4)
inline void accumulate_multi(uint8_t* const* v, size_t np, const uint8_t* const* rows, const uint8_t* q,
                             size_t ldq, size_t nrows, size_t n) {
#if defined(__x86_64__)
  if (have_gfni512()) {
    switch (np) {
      case 1: return accumulate_multi_gfni512<1>(v, rows, q, ldq, nrows, n);
      case 2: return accumulate_multi_gfni512<2>(v, rows, q, ldq, nrows, n);
      case 3: return accumulate_multi_gfni512<3>(v, rows, q, ldq, nrows, n);
      case 4: return accumulate_multi_gfni512<4>(v, rows, q, ldq, nrows, n);
    }
  }
#endif
  for (size_t p = 0; p < np; p++) accumulate(v[p], rows, q + p * ldq, nrows, n);
}

// rows[j][0..n) ^= XOR_p q[j * np + p] * v[p][0..n) for every j (np <= 4)
inline void rank_multi(uint8_t* const* rows, const uint8_t* q, size_t nrows, const uint8_t* const* v, size_t np,
                       size_t n) {
#if defined(__x86_64__)
  if (have_gfni512()) {
    switch (np) {
      case 1: return rank_multi_gfni512<1>(rows, q, nrows, v, n);
      case 2: return rank_multi_gfni512<2>(rows, q, nrows, v, n);
      case 3: return rank_multi_gfni512<3>(rows, q, nrows, v, n);
      case 4: return rank_multi_gfni512<4>(rows, q, nrows, v, n);
    }
  }
#endif
  for (size_t j = 0; j < nrows; j++)
    for (size_t p = 0; p < np; p++) axpy(rows[j], v[p], n, q[j * np + p]);
}

inline bool all_zero(const uint8_t* p, size_t n) {
#if defined(__x86_64__)
  if (have_gfni512()) return all_zero512(p, n);
#endif
  size_t i = 0;
  uint64_t acc = 0;
  for (; i + 8 <= n; i += 8) {
    uint64_t w;
    memcpy(&w, p + i, 8);
    acc |= w;
  }
  for (; i < n; i++) acc |= p[i];
  return acc == 0;
}

}  // namespace hostgf
}  // namespace kodr_amd
