// Calibration kernels (measurement only, not part of the engine): how fast can
// one launch stream a 32 MiB generation on this GPU with the engine's access
// shapes but no GF arithmetic?
#include <hip/hip_runtime.h>
#include <stdint.h>

// grid-stride dwordx4 read of `bytes`, XOR-folded to one dword per thread
__global__ void read_stream(const uint4* __restrict__ src, size_t n16, uint32_t* out) {
  uint32_t acc = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
    uint4 v = src[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

// the engine's shape: K rows x ncols, workgroup = 16 waves over one column
// chunk of 1024/S bytes, wave w reads rows [16w, 16w+16), lane group g row +g
template <int S>
__global__ __launch_bounds__(1024) void read_tiles(const uint8_t* X, int K, int ldx, uint32_t* out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int GL = 64 / S;
  const int g = lane / GL, li = lane % GL;
  const int col = blockIdx.x * GL * 16 + li * 16;
  const int rows_per_wave = K / 16;
  uint32_t acc = 0;
  for (int r = 0; r < rows_per_wave; r += S) {
    const int k = w * rows_per_wave + r + g;
    uint4 v = *reinterpret_cast<const uint4*>(X + (size_t)k * ldx + col);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  out[blockIdx.x * 1024 + threadIdx.x] = acc;
}

extern "C" int probe_read(const void* src, size_t bytes, void* out, int blocks, int threads, void* stream) {
  hipLaunchKernelGGL(read_stream, dim3(blocks), dim3(threads), 0, (hipStream_t)stream,
                     (const uint4*)src, bytes / 16, (uint32_t*)out);
  return (int)hipGetLastError();
}

extern "C" int probe_tiles(const void* X, int K, int ldx, int ncols, int S, void* out, void* stream) {
  const int nb = ncols / (1024 / S);
  if (S == 1) hipLaunchKernelGGL(read_tiles<1>, dim3(nb), dim3(1024), 0, (hipStream_t)stream, (const uint8_t*)X, K, ldx, (uint32_t*)out);
  if (S == 2) hipLaunchKernelGGL(read_tiles<2>, dim3(nb), dim3(1024), 0, (hipStream_t)stream, (const uint8_t*)X, K, ldx, (uint32_t*)out);
  if (S == 4) hipLaunchKernelGGL(read_tiles<4>, dim3(nb), dim3(1024), 0, (hipStream_t)stream, (const uint8_t*)X, K, ldx, (uint32_t*)out);
  return (int)hipGetLastError();
}
