// Host GFNI throughput probe (CPU only): ns per vgf2p8affineqb on zmm/ymm for
// independent streams (throughput) and one dependent chain (latency), and
// the row-update loop shape of panel_update (16 affines per 64-byte chunk
// with broadcast matrices).  gcc -O2 -mavx512f -mavx512bw -mgfni tools/probe/gfni_tput.c
#include <immintrin.h>
#include <stdint.h>
#include <stdio.h>
#include <time.h>

static volatile uint64_t sink;
static double now(void) {
  struct timespec t;
  clock_gettime(CLOCK_MONOTONIC, &t);
  return t.tv_sec + t.tv_nsec * 1e-9;
}

int main(void) {
  const long N = 50000000;
  __m512i a[8], A = _mm512_set1_epi64(0x0102040810204080LL);
  for (int i = 0; i < 8; i++) a[i] = _mm512_set1_epi32(i * 77 + 1);
  double t0 = now();
  for (long n = 0; n < N; n++) {
#pragma GCC unroll 8
    for (int i = 0; i < 8; i++) a[i] = _mm512_gf2p8affine_epi64_epi8(a[i], A, 1);
    __asm__ volatile("" : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7]));
  }
  double t1 = now();
  __m512i s = a[0];
  for (int i = 1; i < 8; i++) s = _mm512_xor_si512(s, a[i]);
  printf("zmm affine, 8 independent chains: %.3f ns/op\n", (t1 - t0) / (N * 8.0) * 1e9);
  __m512i c = s;
  t0 = now();
  for (long n = 0; n < N; n++) {
    c = _mm512_gf2p8affine_epi64_epi8(c, A, 1);
    __asm__ volatile("" : "+v"(c));
  }
  t1 = now();
  printf("zmm affine, one dependent chain:  %.3f ns/op\n", (t1 - t0) / N * 1e9);
  sink ^= (uint64_t)_mm_cvtsi128_si64(_mm512_castsi512_si128(_mm512_xor_si512(c, s)));
  __m256i b[8], B = _mm256_set1_epi64x(0x0102040810204080LL);
  for (int i = 0; i < 8; i++) b[i] = _mm256_set1_epi32(i * 77 + 1);
  t0 = now();
  for (long n = 0; n < N; n++) {
#pragma GCC unroll 8
    for (int i = 0; i < 8; i++) b[i] = _mm256_gf2p8affine_epi64_epi8(b[i], B, 1);
    __asm__ volatile("" : "+v"(b[0]), "+v"(b[1]), "+v"(b[2]), "+v"(b[3]), "+v"(b[4]), "+v"(b[5]), "+v"(b[6]), "+v"(b[7]));
  }
  t1 = now();
  printf("ymm affine, 8 independent chains: %.3f ns/op\n", (t1 - t0) / (N * 8.0) * 1e9);
  for (int i = 0; i < 8; i++) sink ^= (uint64_t)_mm_cvtsi128_si64(_mm256_castsi256_si128(b[i]));
  // the panel_update row shape: d ^= sum_c affine(N[c], bcast(tab[q[c]]))
  static uint64_t tab[256];
  static uint8_t rows[4096][64] __attribute__((aligned(64)));
  static uint8_t q[4096][16];
  for (int i = 0; i < 256; i++) tab[i] = 0x0102040810204080ULL * (i | 1);
  for (int i = 0; i < 4096; i++)
    for (int j = 0; j < 16; j++) q[i][j] = (uint8_t)(i * 31 + j * 7);
  __m512i Nr[16];
  for (int c = 0; c < 16; c++) Nr[c] = _mm512_set1_epi32(c * 13 + 5);
  const int R = 2000;
  t0 = now();
  for (int r = 0; r < R; r++)
    for (int i = 0; i < 4096; i++) {
      __m512i d0 = _mm512_load_si512(rows[i]), d1 = _mm512_setzero_si512();
#pragma GCC unroll 16
      for (int cc = 0; cc < 16; cc += 2) {
        const __m512i x0 = _mm512_gf2p8affine_epi64_epi8(Nr[cc], _mm512_set1_epi64((long long)tab[q[i][cc]]), 0);
        const __m512i x1 = _mm512_gf2p8affine_epi64_epi8(Nr[cc + 1], _mm512_set1_epi64((long long)tab[q[i][cc + 1]]), 0);
        if (cc & 2) d1 = _mm512_ternarylogic_epi64(d1, x0, x1, 0x96);
        else d0 = _mm512_ternarylogic_epi64(d0, x0, x1, 0x96);
      }
      _mm512_store_si512(rows[i], _mm512_xor_si512(d0, d1));
    }
  t1 = now();
  printf("row update (16 affines per 64 B chunk): %.3f ns/affine\n", (t1 - t0) / (R * 4096.0 * 16) * 1e9);
  return rows[5][3] == 0x5a;
}
