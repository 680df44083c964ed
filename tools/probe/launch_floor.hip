// Launch floor on one stream, from C++ (no Python in the loop): back-to-back
// empty launches timed with HIP events and with the host clock, at two grid
// shapes.  Run under rocprofv3 --kernel-trace to read the start-to-start gaps.
// Measurement only; not part of the library.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <chrono>

__global__ void empty_kernel(int* p) {
  if (p && threadIdx.x == 1023) p[0] = 1;  // never taken (p is null): keeps the kernel non-trivial
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  const int N = 2000;
  struct Shape { int blocks, threads; } shapes[] = {{1, 64}, {256, 64}, {256, 1024}, {1024, 256}, {4096, 64}};
  for (auto sh : shapes) {
    for (int i = 0; i < 200; i++) hipLaunchKernelGGL(empty_kernel, dim3(sh.blocks), dim3(sh.threads), 0, st, nullptr);
    CK(hipStreamSynchronize(st));
    CK(hipEventRecord(a, st));
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < N; i++) hipLaunchKernelGGL(empty_kernel, dim3(sh.blocks), dim3(sh.threads), 0, st, nullptr);
    auto t1 = std::chrono::steady_clock::now();
    CK(hipEventRecord(b, st));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    const double host_us = std::chrono::duration<double, std::micro>(t1 - t0).count() / N;
    printf("empty blocks=%5d threads=%5d: %.3f us per launch (events, back to back), host submit %.3f us per call\n",
           sh.blocks, sh.threads, ms * 1e3 / N, host_us);
  }
  // one launch at a time from an idle stream (submit + run + sync)
  double tot = 0;
  for (int i = 0; i < 200; i++) {
    auto t0 = std::chrono::steady_clock::now();
    hipLaunchKernelGGL(empty_kernel, dim3(256), dim3(1024), 0, st, nullptr);
    CK(hipStreamSynchronize(st));
    tot += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  }
  printf("single launch + sync from idle: %.3f us\n", tot / 200);
  return 0;
}
