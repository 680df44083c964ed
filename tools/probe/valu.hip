// VALU throughput probe (measurement only): independent chains of one opcode.
#include <hip/hip_runtime.h>
#include <stdint.h>

template <int OP>
__global__ __launch_bounds__(256) void valu_loop(uint32_t* out, uint32_t seed, int iters) {
  uint32_t a[8], t0 = seed * 0x9E3779B9u + threadIdx.x, t1 = seed ^ 0x12345678u, sel = threadIdx.x & 0x07070707u;
#pragma unroll
  for (int i = 0; i < 8; i++) a[i] = t0 + i * 0x01010101u;
  for (int it = 0; it < iters; it++) {
#pragma unroll
    for (int r = 0; r < 16; r++) {
#pragma unroll
      for (int i = 0; i < 8; i++) {
        if (OP == 0) a[i] = __builtin_amdgcn_perm(t0, t1, a[i] & 0x07070707u);
        if (OP == 1) a[i] = __builtin_amdgcn_perm(a[i], t1, sel);
        if (OP == 2) a[i] = __builtin_amdgcn_bitop3_b32(a[i], t0, t1, 0x96);
        if (OP == 3) a[i] = a[i] ^ (t1 + i);
        if (OP == 4) a[i] = __builtin_amdgcn_perm(t0, t1, a[i]);
      }
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) s ^= a[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

extern "C" int probe_valu(int op, void* out, int blocks, int iters, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (op == 0) hipLaunchKernelGGL(valu_loop<0>, dim3(blocks), dim3(256), 0, st, (uint32_t*)out, 1u, iters);
  if (op == 1) hipLaunchKernelGGL(valu_loop<1>, dim3(blocks), dim3(256), 0, st, (uint32_t*)out, 1u, iters);
  if (op == 2) hipLaunchKernelGGL(valu_loop<2>, dim3(blocks), dim3(256), 0, st, (uint32_t*)out, 1u, iters);
  if (op == 3) hipLaunchKernelGGL(valu_loop<3>, dim3(blocks), dim3(256), 0, st, (uint32_t*)out, 1u, iters);
  if (op == 4) hipLaunchKernelGGL(valu_loop<4>, dim3(blocks), dim3(256), 0, st, (uint32_t*)out, 1u, iters);
  return (int)hipGetLastError();
}
