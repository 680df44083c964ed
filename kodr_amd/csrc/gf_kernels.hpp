// gf_kernels.hpp -- device entry points of the engine (see gf_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace kodr_amd {

// Instantiated tiles of gf_gemm_kernel: mt output rows per workgroup, kw waves
// splitting K over one column chunk, s lane groups per wave (chunk = 1024/s B),
// p row-steps in flight per wave (0 = the tile's default).
struct GemmConfig {
  int mt, kw, s, p;
};

GemmConfig choose_gemm_config(size_t M, size_t K, size_t ncols);

// Y[m][j] = XOR_k A[m][k] * X[k][j], m < M, j < ncols.  All pointers device.
// ldx/ldy multiples of 16 and >= ncols; X rows readable up to round_up(ncols,16).
hipError_t gf_gemm(const uint8_t* dA, size_t lda, size_t M, size_t K, const uint8_t* dX,
                   size_t ldx, uint8_t* dY, size_t ldy, size_t ncols, hipStream_t stream,
                   const GemmConfig* force = nullptr);

}  // namespace kodr_amd
