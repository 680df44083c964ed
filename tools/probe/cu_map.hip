// Where the workgroups of a grouped-launch-shaped grid land: for a 1-D grid
// of NB one-wave workgroups with the direct variant's LDS (so 16 fit a CU),
// each records its XCC, SE, CU and SIMD (s_getreg HW_ID / XCC_ID) and
// s_memrealtime at start and end; it then spins ~20 us so the whole grid is
// resident at once, as in the real launch.  Prints one line per block:
// block xcc hw_id cu simd t0 t1.  Used to pick a block -> task mapping that
// puts workgroups with the same coefficient sequence on one CU.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

#define GETREG(SZ, OFF, REG) (((SZ - 1) << 11) | ((OFF) << 6) | (REG))

__global__ __launch_bounds__(64) void probe(uint32_t* out, int spin) {
  extern __shared__ uint32_t lds[];
  const uint32_t hw = __builtin_amdgcn_s_getreg(GETREG(32, 0, 4));
  const uint32_t xcc = __builtin_amdgcn_s_getreg(GETREG(4, 0, 20));
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  lds[threadIdx.x] = hw;
  uint64_t t1 = t0;
  while (t1 - t0 < (uint64_t)spin) t1 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    uint32_t* o = out + blockIdx.x * 6;
    o[0] = xcc;
    o[1] = hw;                // raw HW_ID: SIMD 5:4, CU 11:8, SH 12, SE 15:13
    o[2] = (hw >> 8) & 31;    // CU_ID with SH_ID
    o[3] = (hw >> 4) & 3;     // SIMD_ID
    o[4] = (uint32_t)t0 + lds[1] * 0;
    o[5] = (uint32_t)t1;
  }
}

int main(int argc, char** argv) {
  const int nb = argc > 1 ? atoi(argv[1]) : 4096;
  const int lds = argc > 2 ? atoi(argv[2]) : 9 * 1024 + 64;
  uint32_t* d = nullptr;
  if (hipMalloc(&d, (size_t)nb * 6 * 4) != hipSuccess) return 1;
  for (int rep = 0; rep < 2; rep++) {
    hipLaunchKernelGGL(probe, dim3(nb), dim3(64), lds, 0, d, 2000);  // 100 MHz clock: 20 us
    if (hipDeviceSynchronize() != hipSuccess) return 2;
  }
  std::vector<uint32_t> h((size_t)nb * 6);
  if (hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost) != hipSuccess) return 3;
  for (int b = 0; b < nb; b++)
    printf("%d %u %u %u %u %u %u\n", b, h[b * 6], h[b * 6 + 1], h[b * 6 + 2], h[b * 6 + 3], h[b * 6 + 4], h[b * 6 + 5]);
  (void)hipFree(d);
  return 0;
}
