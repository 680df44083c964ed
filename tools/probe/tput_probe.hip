// VALU issue cost on gfx950 for the elimination's instruction mix
// (measurement only, not part of the library): 8 independent v_perm_b32
// chains, 8 independent v_xor_b32 chains, and the gmul4 body (3 v_perm + 2
// xor + 3 selector ops), per wave, with W waves per workgroup (W / 4 per SIMD).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probe/tput_probe.hip -o tools/probe/tput_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int N = 1024;

template <int K>
__global__ void tput(const uint32_t* in, unsigned long long* out, uint32_t* sink) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t a[8], x = in[lane], s = in[lane + 64] & 0x07070707u;
#pragma unroll
  for (int j = 0; j < 8; j++) a[j] = in[lane + 128 + 64 * j];
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N; i++) {
#pragma unroll
    for (int j = 0; j < 8; j++) {
      if (K == 0) a[j] = __builtin_amdgcn_perm(a[j], x, s);
      if (K == 1) a[j] = (a[j] ^ x) + 0;
      if (K == 2) {  // gmul4 of data a[j] with tables (x, s, x ^ s, ...)
        const uint32_t s0 = a[j] & 0x07070707u, s1 = (a[j] >> 3) & 0x07070707u, s2 = (a[j] >> 6) & 0x03030303u;
        a[j] = __builtin_amdgcn_perm(x, s, s0) ^ __builtin_amdgcn_perm(s, x, s1) ^ __builtin_amdgcn_perm(x, x, s2);
      }
    }
    x += 0x01010101u;
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) r ^= a[j];
  sink[threadIdx.x] = r;
  if (lane == 0) out[w] = t1 - t0;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
  uint32_t *din, *sink;
  unsigned long long* dout;
  CK(hipMalloc(&din, 4096 * 4));
  CK(hipMalloc(&sink, 1024 * 4));
  CK(hipMalloc(&dout, 64 * 8));
  uint32_t h[4096];
  uint32_t s = 7;
  for (auto& v : h) v = (s = s * 1664525u + 1013904223u);
  CK(hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice));
  const char* names[] = {"v_perm (8 chains)", "v_xor (8 chains)", "gmul4 body (8 chains)"};
  const int insts[] = {1, 1, 8};
  for (int k = 0; k < 3; k++)
    for (int W : {1, 4, 8, 12, 16}) {
      unsigned long long o[16];
      for (int rep = 0; rep < 2; rep++) {
        if (k == 0) hipLaunchKernelGGL(tput<0>, 1, 64 * W, 0, 0, din, dout, sink);
        if (k == 1) hipLaunchKernelGGL(tput<1>, 1, 64 * W, 0, 0, din, dout, sink);
        if (k == 2) hipLaunchKernelGGL(tput<2>, 1, 64 * W, 0, 0, din, dout, sink);
        CK(hipDeviceSynchronize());
      }
      CK(hipMemcpy(o, dout, 8 * W, hipMemcpyDeviceToHost));
      double mx = 0;
      for (int i = 0; i < W; i++) mx = o[i] > mx ? o[i] : mx;
      printf("%-24s W=%2d (%.2f waves/SIMD): %.2f cyc per wave-instruction per wave, %.2f per SIMD\n", names[k], W,
             W / 4.0, mx / (N * 8.0 * insts[k]), mx / (N * 8.0 * insts[k]) / (W < 4 ? 1 : W / 4.0));
    }
  return 0;
}
