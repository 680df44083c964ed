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

// read_tiles<2> with the gemm kernel's extra phases switched on one at a time
// (B = 1 gap hunt): V & 1 a coefficient byte per thread < 256 through LDS and a
// barrier before the loop, V & 2 the 16-wave ds_xor fold + barrier + 512 B of
// stores instead of 4 KiB, V & 4 buffer loads instead of global loads.
template <int V>
__global__ __launch_bounds__(1024) void read_tiles_v(const uint8_t* X, int K, int ldx, uint32_t* out,
                                                     const uint8_t* coef) {
  __shared__ uint32_t tab[256];
  __shared__ uint32_t red[4 * 32];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  constexpr int S = 2, GL = 32;
  const int g = lane / GL, li = lane % GL;
  const int col = blockIdx.x * GL * 16 + li * 16;
  const int rows_per_wave = K / 16;
  uint32_t cf = 0;
  if (V & 1) {
    if (threadIdx.x < 256) cf = coef[threadIdx.x];
  }
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)X, (short)0, K * ldx, 0x00020000);
  uint4 v[8];
#pragma unroll
  for (int r = 0; r < 8; r++) {
    const int k = w * rows_per_wave + 2 * r + g;
    if (V & 4) {
      const auto t = __builtin_amdgcn_raw_buffer_load_b128(xr, k * ldx + col, 0, 0);
      v[r] = make_uint4(t[0], t[1], t[2], t[3]);
    } else {
      v[r] = *reinterpret_cast<const uint4*>(X + (size_t)k * ldx + col);
    }
  }
  if (V & 1) {
    if (threadIdx.x < 256) tab[threadIdx.x] = cf * 0x01010101u;
    if (threadIdx.x < 128) red[threadIdx.x] = 0;
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  }
  uint32_t acc[4] = {0, 0, 0, 0};
#pragma unroll
  for (int r = 0; r < 8; r++) {
    const uint32_t m = (V & 1) ? tab[w * 16 + 2 * r + g] : 1u;
    acc[0] ^= v[r].x * m;
    acc[1] ^= v[r].y * m;
    acc[2] ^= v[r].z * m;
    acc[3] ^= v[r].w * m;
  }
  if (V & 2) {
    if (!(V & 1)) {
      if (threadIdx.x < 128) red[threadIdx.x] = 0;
      __syncthreads();
    }
#pragma unroll
    for (int d = 0; d < 4; d++) {
      const auto r = __builtin_amdgcn_permlane32_swap(acc[d], acc[d], false, false);
      acc[d] = r[0] ^ r[1];
    }
    if (g == 0)
      for (int d = 0; d < 4; d++) atomicXor(&red[d * 32 + li], acc[d]);
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (threadIdx.x < 32)
      reinterpret_cast<uint4*>(out)[blockIdx.x * 32 + threadIdx.x] =
          make_uint4(red[threadIdx.x], red[32 + threadIdx.x], red[64 + threadIdx.x], red[96 + threadIdx.x]);
  } else {
    out[blockIdx.x * 1024 + threadIdx.x] = acc[0] ^ acc[1] ^ acc[2] ^ acc[3];
  }
}

extern "C" int probe_tiles_v(const void* X, int K, int ldx, int ncols, int V, void* out, const void* coef,
                             void* stream) {
  const int nb = ncols / 512;
  if (K != 256) return -1;
  const uint8_t* x = (const uint8_t*)X;
  const uint8_t* c = (const uint8_t*)coef;
  uint32_t* o = (uint32_t*)out;
  hipStream_t s = (hipStream_t)stream;
  switch (V) {
    case 0: hipLaunchKernelGGL(read_tiles_v<0>, dim3(nb), dim3(1024), 0, s, x, K, ldx, o, c); break;
    case 1: hipLaunchKernelGGL(read_tiles_v<1>, dim3(nb), dim3(1024), 0, s, x, K, ldx, o, c); break;
    case 2: hipLaunchKernelGGL(read_tiles_v<2>, dim3(nb), dim3(1024), 0, s, x, K, ldx, o, c); break;
    case 3: hipLaunchKernelGGL(read_tiles_v<3>, dim3(nb), dim3(1024), 0, s, x, K, ldx, o, c); break;
    case 4: hipLaunchKernelGGL(read_tiles_v<4>, dim3(nb), dim3(1024), 0, s, x, K, ldx, o, c); break;
    case 5: hipLaunchKernelGGL(read_tiles_v<5>, dim3(nb), dim3(1024), 0, s, x, K, ldx, o, c); break;
    case 6: hipLaunchKernelGGL(read_tiles_v<6>, dim3(nb), dim3(1024), 0, s, x, K, ldx, o, c); break;
    case 7: hipLaunchKernelGGL(read_tiles_v<7>, dim3(nb), dim3(1024), 0, s, x, K, ldx, o, c); break;
    default: return -1;
  }
  return (int)hipGetLastError();
}
