// What does M0 hold in VGPR index mode on gfx950?  (measurement only)
#include <hip/hip_runtime.h>
#include <stdint.h>
__global__ void m0_probe(uint32_t* out) {
  uint32_t a, b, c;
  asm volatile(
      "s_mov_b32 m0, 0\n\t"
      "s_set_gpr_idx_on 8, gpr_idx(SRC0,DST)\n\t"
      "s_mov_b32 %0, m0\n\t"
      "s_add_u32 m0, m0, 8\n\t"
      "s_mov_b32 %1, m0\n\t"
      "s_set_gpr_idx_off\n\t"
      "s_mov_b32 %2, m0\n\t"
      : "=s"(a), "=s"(b), "=s"(c)
      :
      : "m0");
  if (threadIdx.x == 0) {
    out[0] = a;
    out[1] = b;
    out[2] = c;
  }
}
extern "C" int m0_run(void* out, void* st) {
  hipLaunchKernelGGL(m0_probe, dim3(1), dim3(64), 0, (hipStream_t)st, (uint32_t*)out);
  return (int)hipGetLastError();
}
