// Device helpers shared by the GF(2^8) kernels (gf_kernels.hip, gf_bs.hip).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace kodr_amd {

__device__ __forceinline__ uint32_t gf_xt(uint32_t c) {  // multiply by x (=2) mod 0x11D (gf256.go:15-44)
  return ((c << 1) ^ ((c & 0x80u) ? 0x1Du : 0u)) & 0xFFu;
}

// Product tables of one coefficient c for v_perm lookups, little-endian
// bytes: T0 = c*{0..7}, T1 = c*{0..7}<<3, T2 = c*{0..3}<<6.
__device__ __forceinline__ void gf_make_tables(uint32_t c, uint4& t01, uint32_t& t2) {
  const uint32_t c1 = c, c2 = gf_xt(c1), c4 = gf_xt(c2), c8 = gf_xt(c4);
  const uint32_t c16 = gf_xt(c8), c32 = gf_xt(c16), c64 = gf_xt(c32), c128 = gf_xt(c64);
  const uint32_t lo0 = (c1 << 8) | (c2 << 16) | ((c1 ^ c2) << 24);
  const uint32_t lo1 = (c8 << 8) | (c16 << 16) | ((c8 ^ c16) << 24);
  // byte broadcasts by v_perm (selector 0: byte 0 of the second source in
  // every byte), not a quarter-rate 32-bit multiply
  t01.x = lo0;
  t01.y = lo0 ^ __builtin_amdgcn_perm(0u, c4, 0u);
  t01.z = lo1;
  t01.w = lo1 ^ __builtin_amdgcn_perm(0u, c32, 0u);
  t2 = (c64 << 8) | (c128 << 16) | ((c64 ^ c128) << 24);
}

// acc ^= c * x for the 4 bytes of x (tables of c from gf_make_tables)
__device__ __forceinline__ uint32_t gf_mul_acc4(uint32_t acc, uint32_t x, const uint4& t01, uint32_t t2) {
  const uint32_t s0 = x & 0x07070707u, s1 = (x >> 3) & 0x07070707u, s2 = (x >> 6) & 0x03030303u;
  const uint32_t a0 = __builtin_amdgcn_perm(t01.y, t01.x, s0);
  const uint32_t a1 = __builtin_amdgcn_perm(t01.w, t01.z, s1);
  const uint32_t a2 = __builtin_amdgcn_perm(t2, t2, s2);
  return __builtin_amdgcn_bitop3_b32(acc, a0, a1, 0x96) ^ a2;
}

}  // namespace kodr_amd
