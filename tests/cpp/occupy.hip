// Test infrastructure (tests/test_gpu_coresidency.py): a kernel that holds
// n workgroups resident for a fixed time, each with 1024 threads and most of
// a CU's LDS, so that no workgroup of another kernel fits beside it -- the
// multi-workgroup elimination launched meanwhile finds only the CUs left
// free.  Spins on s_memrealtime (100 MHz) with s_sleep; every wave ends.
#include <hip/hip_runtime.h>
#include <stdint.h>

extern "C" {

__global__ __launch_bounds__(1024) void kodr_occupy_kernel(uint64_t ticks, uint32_t* sink) {
  extern __shared__ uint32_t lds[];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  lds[threadIdx.x] = threadIdx.x;
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
  __syncthreads();
  if (threadIdx.x == 0 && lds[1023] != 1023u) sink[0] = 1u;  // (never: keeps the LDS allocation live)
}

int kodr_test_cu_count(int device) {
  hipDeviceProp_t p;
  return hipGetDeviceProperties(&p, device) == hipSuccess ? p.multiProcessorCount : -1;
}

void* kodr_test_stream_create(int device) {
  hipStream_t s = nullptr;
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  return hipStreamCreateWithFlags(&s, hipStreamNonBlocking) == hipSuccess ? (void*)s : nullptr;
}

// a stream at the device's highest priority (its own hardware queue pool)
void* kodr_test_stream_create_high(int device) {
  hipStream_t s = nullptr;
  int least = 0, greatest = 0;
  if (hipSetDevice(device) != hipSuccess || hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess)
    return nullptr;
  return hipStreamCreateWithPriority(&s, hipStreamNonBlocking, greatest) == hipSuccess ? (void*)s : nullptr;
}

int kodr_test_stream_priority_range(int device, int* least, int* greatest) {
  if (hipSetDevice(device) != hipSuccess) return -1;
  return hipDeviceGetStreamPriorityRange(least, greatest) == hipSuccess ? 0 : -1;
}

int kodr_test_stream_destroy(void* s) { return hipStreamDestroy((hipStream_t)s) == hipSuccess ? 0 : -1; }

int kodr_test_stream_sync(void* s) { return hipStreamSynchronize((hipStream_t)s) == hipSuccess ? 0 : -1; }

// n workgroups of 1024 threads holding lds_bytes of LDS each for `ms`
// milliseconds on `stream`
int kodr_test_occupy(void* stream, int n, double ms, int lds_bytes) {
  static uint32_t* sink = nullptr;
  if (!sink && hipMalloc((void**)&sink, 4) != hipSuccess) return -1;
  if (hipFuncSetAttribute((const void*)kodr_occupy_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                          lds_bytes) != hipSuccess)
    return -2;
  const uint64_t ticks = (uint64_t)(ms * 1e5);
  hipLaunchKernelGGL(kodr_occupy_kernel, dim3(n), dim3(1024), lds_bytes, (hipStream_t)stream, ticks, sink);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // extern "C"
