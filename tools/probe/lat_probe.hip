// Latency of the primitives on the elimination chain's critical path, one
// wave, dependent chains of N links (measurement only, not part of the
// library): DPP quad broadcast, ds_read_b32 / b128 gathers with a
// data-dependent address, ds_bpermute, ballot -> s_ff1 -> v_readlane, a
// readlane-based uniform LDS read, v_perm, and whole GF multiplies.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probe/lat_probe.hip -o tools/probe/lat_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int N = 256;

__device__ __forceinline__ uint32_t qb(uint32_t v, int cd) {
  switch (cd & 3) {
    case 0: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x00, 0xf, 0xf, false);
    case 1: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x55, 0xf, 0xf, false);
    case 2: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xaa, 0xf, 0xf, false);
    default: return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xff, 0xf, 0xf, false);
  }
}

template <int K>
__global__ __launch_bounds__(64) void lat(const uint32_t* in, unsigned long long* out, uint32_t* sink) {
  __shared__ uint32_t lds[2048];
  __shared__ uint4 tab[512];
  const int lane = threadIdx.x;
  for (int i = lane; i < 2048; i += 64) lds[i] = in[i] & 0x1ff;
  for (int i = lane; i < 512; i += 64) tab[i] = make_uint4(in[4 * i] & 0x1ff, in[4 * i + 1], in[4 * i + 2], in[4 * i + 3]);
  __syncthreads();
  uint32_t v = in[lane] & 0xff;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 16
  for (int i = 0; i < N; i++) {
    if (K == 0) {  // DPP quad broadcast + bfe
      v = (qb(v, i) >> 8) & 0x1ffu;
      v += 1;
    } else if (K == 1) {  // ds_read_b32 gather
      v = lds[v & 0x7ff];
    } else if (K == 2) {  // ds_read_b128 gather (table row)
      const uint4 t = tab[v & 0x1ff];
      v = t.x ^ (t.y & 0);
    } else if (K == 3) {  // ds_bpermute
      v = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((v & 63) << 2), (int)v) + 1;
    } else if (K == 4) {  // ballot -> ff1 -> readlane
      const uint64_t m = __builtin_amdgcn_ballot_w64((v & 1) != 0) | 1ull << 63;
      const int pl = __builtin_ctzll(m);
      v = __builtin_amdgcn_readlane(v, pl) + (uint32_t)lane;
    } else if (K == 5) {  // readlane -> uniform ds_read (address from an SGPR)
      const uint32_t u = __builtin_amdgcn_readfirstlane(v);
      v = lds[u & 0x7ff] + (uint32_t)lane;
    } else if (K == 6) {  // v_perm chain
      v = __builtin_amdgcn_perm(v, v * 3u, v & 0x07070707u);
    } else if (K == 7) {  // a VALU xor/shift chain (reference, not foldable)
      v = (v ^ (v >> 3)) + (uint32_t)lane;
    } else if (K == 8) {  // v_readlane (constant lane) -> VALU use
      v = __builtin_amdgcn_readlane(v, 5) + (uint32_t)lane;
    } else if (K == 9) {  // four independent readlanes (constant lanes) -> one select
      const uint32_t a = __builtin_amdgcn_readlane(v, 4), b = __builtin_amdgcn_readlane(v, 5);
      const uint32_t c2 = __builtin_amdgcn_readlane(v, 6), e = __builtin_amdgcn_readlane(v, 7);
      const int d = lane & 3;
      v = (d == 0 ? a : d == 1 ? b : d == 2 ? c2 : e) + (uint32_t)lane;
    } else if (K == 10) {  // readlane with an SALU-computed lane -> VALU
      const uint32_t u = __builtin_amdgcn_readfirstlane(v);
      v = __builtin_amdgcn_readlane(v, (int)(u & 63)) + (uint32_t)lane;
    } else if (K == 11) {  // v_cmp -> ballot -> s_ff1 -> v_mov (SALU result back in a VGPR)
      const uint64_t m = __builtin_amdgcn_ballot_w64((v & 4) != 0) | 1ull << 63;
      v = (uint32_t)__builtin_ctzll(m) + v + 1u;
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  sink[lane] = v;
  if (lane == 0) out[K] = t1 - t0;
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
  uint32_t* din;
  unsigned long long* dout;
  uint32_t* sink;
  CK(hipMalloc(&din, 2048 * 4 * 4));
  CK(hipMalloc(&dout, 64 * 8));
  CK(hipMalloc(&sink, 64 * 4));
  uint32_t h[8192];
  uint32_t s = 12345;
  for (auto& x : h) x = (s = s * 1664525u + 1013904223u) >> 8;
  CK(hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice));
  const char* names[] = {"dpp quad bcast + bfe + add", "ds_read_b32 gather", "ds_read_b128 gather",
                         "ds_bpermute + add", "ballot + ff1 + readlane + add", "readfirstlane + uniform ds_read + add",
                         "v_perm (+ and)", "xor/shift + add", "readlane const -> add", "4 readlanes + select + add",
                         "readfirstlane -> readlane(dyn) -> add", "ballot -> ff1 -> VALU"};
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(lat<0>, 1, 64, 0, 0, din, dout, sink);
    hipLaunchKernelGGL(lat<1>, 1, 64, 0, 0, din, dout, sink);
    hipLaunchKernelGGL(lat<2>, 1, 64, 0, 0, din, dout, sink);
    hipLaunchKernelGGL(lat<3>, 1, 64, 0, 0, din, dout, sink);
    hipLaunchKernelGGL(lat<4>, 1, 64, 0, 0, din, dout, sink);
    hipLaunchKernelGGL(lat<5>, 1, 64, 0, 0, din, dout, sink);
    hipLaunchKernelGGL(lat<6>, 1, 64, 0, 0, din, dout, sink);
    hipLaunchKernelGGL(lat<7>, 1, 64, 0, 0, din, dout, sink);
    hipLaunchKernelGGL(lat<8>, 1, 64, 0, 0, din, dout, sink);
    hipLaunchKernelGGL(lat<9>, 1, 64, 0, 0, din, dout, sink);
    hipLaunchKernelGGL(lat<10>, 1, 64, 0, 0, din, dout, sink);
    hipLaunchKernelGGL(lat<11>, 1, 64, 0, 0, din, dout, sink);
    CK(hipDeviceSynchronize());
  }
  unsigned long long o[12];
  CK(hipMemcpy(o, dout, sizeof o, hipMemcpyDeviceToHost));
  for (int k = 0; k < 12; k++) printf("%-40s %6.1f cyc per link\n", names[k], (double)o[k] / N);
  return 0;
}
