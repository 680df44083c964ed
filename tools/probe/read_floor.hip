// Floor of one launch that reads a 32 MiB generation once (measurement only,
// not part of the library): every lane issues all of its dwordx4 loads up
// front, XOR-folds them and stores one dword, like gf_gemv_kernel without the
// multiply.  16 rotating 32 MiB buffers (512 MiB, beyond the MALL), back-to-back
// launches timed with HIP events; run under rocprofv3 --kernel-trace for the
// kernel durations.  Shapes: workgroups x threads x loads per lane.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int NL>
__global__ void read_upfront(const uint8_t* __restrict__ X, uint32_t* out) {
  // lane t of block b reads 16 B at (b * NL + j) * blockDim * 16 + t * 16 for j < NL
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, 0x7fffffff, 0x00020000);
  const uint32_t base = (uint32_t)blockIdx.x * NL * blockDim.x * 16u + threadIdx.x * 16u;
  u32x4 v[NL];
#pragma unroll
  for (int j = 0; j < NL; j++) v[j] = __builtin_amdgcn_raw_buffer_load_b128(xr, base + j * blockDim.x * 16u, 0, 0);
  uint32_t acc = 0;
#pragma unroll
  for (int j = 0; j < NL; j++) acc ^= v[j][0] ^ v[j][1] ^ v[j][2] ^ v[j][3];
  if (acc == 0x12345679u) out[blockIdx.x * blockDim.x + threadIdx.x] = acc;  // keeps the loads live
}

// gf_gemv_kernel's access pattern without the multiply: a workgroup of 16
// waves owns a 512-byte column chunk of a 256 x 131072 generation, wave w rows
// [16w, 16w + 16), lane group g (32 lanes x 16 B) row 16w + 2j + g.  STORE: the
// kernel's tail as well (lane-group fold, one LDS slot per wave, a barrier,
// wave 0 XORs the 16 slots and stores 512 B); otherwise no store.
template <bool STORE>
__global__ __launch_bounds__(1024) void read_gemv_shape(const uint8_t* __restrict__ X, uint32_t* out) {
  __shared__ u32x4 part[16][32];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, g = lane >> 5, li = lane & 31;
  const int col = blockIdx.x * 512 + li * 16;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, 0x7fffffff, 0x00020000);
  u32x4 v[8];
#pragma unroll
  for (int j = 0; j < 8; j++) v[j] = __builtin_amdgcn_raw_buffer_load_b128(xr, (w * 16 + 2 * j + g) * 131072 + col, 0, 0);
  u32x4 acc = v[0];
#pragma unroll
  for (int j = 1; j < 8; j++) acc ^= v[j];
  if (!STORE) {
    if (acc[0] == 0x12345679u) out[blockIdx.x * 1024 + tid] = acc[1];
    return;
  }
#pragma unroll
  for (int d = 0; d < 4; d++) {
    const auto r = __builtin_amdgcn_permlane32_swap(acc[d], acc[d], false, false);
    acc[d] = r[0] ^ r[1];
  }
  if (g == 0) part[w][li] = acc;
  __syncthreads();
  if (tid >= 32) return;
  u32x4 s = part[0][tid];
#pragma unroll
  for (int q = 1; q < 16; q++) s ^= part[q][tid];
  reinterpret_cast<u32x4*>(out)[blockIdx.x * 32 + tid] = s;
}

template <bool STORE>
int run_gemv_shape(uint8_t** bufs, uint32_t* out, hipStream_t st, hipEvent_t a, hipEvent_t b);

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

template <int NL>
int run(uint8_t** bufs, uint32_t* out, int threads, hipStream_t st, hipEvent_t a, hipEvent_t b) {
  const size_t bytes = (size_t)32 << 20;
  const int blocks = (int)(bytes / ((size_t)NL * threads * 16));
  for (int i = 0; i < 64; i++) hipLaunchKernelGGL(read_upfront<NL>, dim3(blocks), dim3(threads), 0, st, bufs[i % 16], out);
  CK(hipStreamSynchronize(st));
  float best = 1e9;
  for (int rep = 0; rep < 5; rep++) {
    CK(hipEventRecord(a, st));
    for (int i = 0; i < 400; i++) hipLaunchKernelGGL(read_upfront<NL>, dim3(blocks), dim3(threads), 0, st, bufs[i % 16], out);
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    best = ms < best ? ms : best;
  }
  const double us = best * 1e3 / 400;
  printf("read 32 MiB: blocks=%5d threads=%5d loads/lane=%2d: %.3f us per launch (events, best of 5 x 400), %.2f TB/s\n",
         blocks, threads, NL, us, bytes / us / 1e6);
  return 0;
}

template <bool STORE>
int run_gemv_shape(uint8_t** bufs, uint32_t* out, hipStream_t st, hipEvent_t a, hipEvent_t b) {
  for (int i = 0; i < 64; i++) hipLaunchKernelGGL(read_gemv_shape<STORE>, dim3(256), dim3(1024), 0, st, bufs[i % 16], out);
  CK(hipStreamSynchronize(st));
  float best = 1e9;
  for (int rep = 0; rep < 5; rep++) {
    CK(hipEventRecord(a, st));
    for (int i = 0; i < 400; i++) hipLaunchKernelGGL(read_gemv_shape<STORE>, dim3(256), dim3(1024), 0, st, bufs[i % 16], out);
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    best = ms < best ? ms : best;
  }
  printf("read 32 MiB in gf_gemv_kernel's shape%s: %.3f us per launch (events, best of 5 x 400)\n",
         STORE ? " with its fold and store" : "", best * 1e3 / 400);
  return 0;
}

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  uint8_t* bufs[16];
  for (int i = 0; i < 16; i++) {
    CK(hipMalloc((void**)&bufs[i], (size_t)32 << 20));
    CK(hipMemset(bufs[i], i, (size_t)32 << 20));
  }
  uint32_t* out;
  CK(hipMalloc((void**)&out, (size_t)64 << 20));
  int rc = 0;
  rc |= run<8>(bufs, out, 1024, st, a, b);   // gf_gemv_kernel's shape: 256 x 1024, 8 loads
  rc |= run<16>(bufs, out, 512, st, a, b);   // 256 x 512
  rc |= run<32>(bufs, out, 256, st, a, b);   // 256 x 256
  rc |= run<8>(bufs, out, 512, st, a, b);    // 512 x 512
  rc |= run<16>(bufs, out, 256, st, a, b);   // 512 x 256
  rc |= run<8>(bufs, out, 256, st, a, b);    // 1024 x 256
  rc |= run<4>(bufs, out, 256, st, a, b);    // 2048 x 256
  rc |= run<4>(bufs, out, 1024, st, a, b);   // 512 x 1024
  rc |= run<2>(bufs, out, 1024, st, a, b);   // 1024 x 1024
  rc |= run_gemv_shape<false>(bufs, out, st, a, b);
  rc |= run_gemv_shape<true>(bufs, out, st, a, b);
  return rc;
}
