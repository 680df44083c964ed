// gf_bs.hip -- bit-sliced GF(2^8) product for gfx950: Y = A (x) X with X held
// in bit-sliced blocks (see DESIGN.md "Bit-sliced kernel").
//
// Layout.  X rows are cut into 32-byte blocks; bitslice32 turns a block's 8
// dwords into 8 planes, plane i = bit i of all 32 bytes (it is an involution,
// so the same transform converts back).  In that layout multiplying by a
// coefficient c is GF(2)-linear on the planes: out plane j = XOR of the input
// planes i with bit j of c*2^i set (gf256.go:15-44, poly 0x11D).  That is about
// 18 XOR3 instructions per coefficient per 32 bytes, against 36 for the
// 3x v_perm lookup formulation of gf_gemm_kernel.
//
// Code.  The XOR pattern depends on c, which is wave-uniform, so each of the
// 256 patterns is a straight-line body (generated: gen_bs_bodies.py) and the
// wave jumps to body[c] with s_swappc_b64.  The bodies address the 8
// accumulator planes through VGPR index mode, so one body serves all 8 output
// rows of a wave (index 8m).  No LDS tables, no lookups, no per-lane branches.
//
// Work split.  A wave owns 8 output rows x 64 blocks (2 KiB of columns) x a
// range of rpw input rows; the KW waves of a workgroup split K and are XOR-
// reduced in LDS.  Per wave, the body offsets for its (row, k) pairs are built
// once into a private scratch slab ("program") and streamed into SGPRs with
// s_load_dwordx8, one row ahead.  X rows stream through a 4-deep register ring
// of buffer loads (rows >= K are outside num_records and read as zero).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <mutex>

#include "gf_kernels.hpp"
// accumulators v[24..87] (8 rows x 8 planes), inputs v[88..95], return s[54:55]
#include "gf_bs_bodies.inc"

namespace kodr_amd {

namespace {

constexpr int kBsRows = 8;     // output rows per wave
constexpr int kBsBlock = 32;   // bytes per bit-sliced block
constexpr int kBsWaveCols = 64 * kBsBlock;

// 8x8 bit-matrix transpose inside each byte lane of 8 dwords: afterwards
// dword i holds bit i of all 32 bytes.  Self-inverse.
__device__ __forceinline__ void bitslice32(uint32_t (&d)[8]) {
#pragma unroll
  for (int q = 0; q < 4; q++) {
    const uint32_t t = ((d[q] >> 4) ^ d[q + 4]) & 0x0F0F0F0Fu;
    d[q + 4] ^= t;
    d[q] ^= t << 4;
  }
#pragma unroll
  for (int q = 0; q < 8; q++) {
    if (q & 2) continue;
    const uint32_t t = ((d[q] >> 2) ^ d[q + 2]) & 0x33333333u;
    d[q + 2] ^= t;
    d[q] ^= t << 2;
  }
#pragma unroll
  for (int q = 0; q < 8; q += 2) {
    const uint32_t t = ((d[q] >> 1) ^ d[q + 1]) & 0x55555555u;
    d[q + 1] ^= t;
    d[q] ^= t << 1;
  }
}

__global__ __launch_bounds__(256) void bitslice_kernel(uint8_t* __restrict__ X, size_t ldx, int rows,
                                                      int nblk) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  const int r = (int)(i / (size_t)nblk), b = (int)(i % (size_t)nblk);
  if (r >= rows) return;
  uint4* p = reinterpret_cast<uint4*>(X + (size_t)r * ldx + (size_t)b * kBsBlock);
  const uint4 a = p[0], c = p[1];
  uint32_t d[8] = {a.x, a.y, a.z, a.w, c.x, c.y, c.z, c.w};
  bitslice32(d);
  p[0] = make_uint4(d[0], d[1], d[2], d[3]);
  p[1] = make_uint4(d[4], d[5], d[6], d[7]);
}

#define KODR_BS_CLOBBERS                                                                     \
  "v24", "v25", "v26", "v27", "v28", "v29", "v30", "v31", "v32", "v33", "v34", "v35", "v36", \
  "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", \
  "v50", "v51", "v52", "v53", "v54", "v55", "v56", "v57", "v58", "v59", "v60", "v61", "v62", \
  "v63", "v64", "v65", "v66", "v67", "v68", "v69", "v70", "v71", "v72", "v73", "v74", "v75", \
  "v76", "v77", "v78", "v79", "v80", "v81", "v82", "v83", "v84", "v85", "v86", "v87", "v88", \
  "v89", "v90", "v91", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100",       \
  "v101", "v102", "v103", "v104", "v105", "v106", "v107", "v108", "v109", "v110", "v111",    \
  "v112", "v113", "v114", "v115", "v116", "v117", "v118", "v119", "v120", "v121", "v122",    \
  "v123", "v124", "v125", "v126", "v127", "s40", "s41", "s42", "s43", "s44", "s45", "s46",   \
  "s47", "s48", "s50", "s51", "s52", "s53", "s54", "s55", "s56", "s57", "s58", "s59", "s60", \
  "s61", "s62", "s63", "s64", "s65", "s66", "s67", "s68", "s69", "s70", "s71", "s72", "s74", \
  "s75", "scc", "memory"

// Writes the 256 body offsets (bytes from body 0) to offs; run once per device.
__global__ __launch_bounds__(64) void gf_bs_export_kernel(uint32_t* offs) {
  asm volatile(
      "s_branch .Lexp_%=\n\t"
      KODR_BS_BODIES
      ".Lexp_%=:\n\t"
      KODR_BS_EXPORT("v24", "%[z]", "%[out]")
      :
      : [z] "v"(0u), [out] "s"(offs)
      : "v24", "memory");
}

template <int KW>
__global__ __launch_bounds__(64 * KW) void gf_bs_kernel(
    const uint8_t* __restrict__ A, int lda, int M, int K, const uint8_t* __restrict__ X, int ldx,
    uint8_t* __restrict__ Y, size_t ldy, int ncols, int rpw, int ncx, int nrg,
    uint32_t* __restrict__ prog, const uint32_t* __restrict__ offs) {
  extern __shared__ uint32_t red[];  // [8 rows x 8 planes][64 lanes]
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  // XCD-aware order: the nrg row groups of one column chunk go to blocks
  // b, b+8, ... (one XCD) and re-read that chunk from its L2.  Speed only.
  const int b = blockIdx.x;
  const int rg = (b >> 3) % nrg;
  const int cx = (b / (8 * nrg)) * 8 + (b & 7);
  if (cx >= ncx) return;
  const int m0 = rg * kBsRows, kb = w * rpw;

  // program: body offset for (row m0 + e%8, input row kb + e/8)
  uint32_t* wp = prog + ((size_t)b * KW + w) * (size_t)rpw * kBsRows;
  for (int e = lane; e < rpw * kBsRows; e += 64) {
    const int k = kb + (e >> 3), row = m0 + (e & 7);
    const uint32_t c = (k < K && row < M) ? A[(size_t)row * lda + k] : 0u;
    wp[e] = offs[c];
  }
  for (int i = tid; i < 64 * 64; i += 64 * KW) red[i] = 0u;
  __syncthreads();

  const uint32_t col = (uint32_t)(cx * 64 + lane) * kBsBlock;
  // wave-uniform values the asm reads from SGPRs
  const uint64_t xa = reinterpret_cast<uint64_t>(X), pa = reinterpret_cast<uint64_t>(wp);
  const uint32_t nrec = __builtin_amdgcn_readfirstlane((uint32_t)K * (uint32_t)ldx);
  const uint32_t kboff = __builtin_amdgcn_readfirstlane((uint32_t)kb * (uint32_t)ldx);
  const uint32_t ngrp = __builtin_amdgcn_readfirstlane((uint32_t)(rpw / 4 - 1));
  const uint32_t xlo = __builtin_amdgcn_readfirstlane((uint32_t)xa);
  const uint32_t xhi = __builtin_amdgcn_readfirstlane((uint32_t)(xa >> 32));
  const uint32_t plo = __builtin_amdgcn_readfirstlane((uint32_t)pa);
  const uint32_t phi = __builtin_amdgcn_readfirstlane((uint32_t)(pa >> 32));
  const uint32_t sldx = __builtin_amdgcn_readfirstlane((uint32_t)ldx);
  asm volatile(
      "s_waitcnt vmcnt(0)\n\t"  // program stores have reached L2
      "s_dcache_inv\n\t"
      "s_mov_b32 s40, %[xlo]\n\t"
      "s_and_b32 s41, %[xhi], 0xffff\n\t"
      "s_mov_b32 s42, %[nrec]\n\t"
      "s_mov_b32 s43, 0x00020000\n\t"
      "s_mov_b32 s44, %[kboff]\n\t"
      "s_mov_b32 s45, %[ldx]\n\t"
      "s_mov_b32 s46, %[plo]\n\t"
      "s_mov_b32 s47, %[phi]\n\t"
      "s_mov_b32 s48, 0\n\t"
      "s_getpc_b64 s[74:75]\n\t"
      ".Lpc_%=:\n\t"
      "s_add_u32 s50, s74, .Lbs_b0_%= - .Lpc_%=\n\t"
      "s_addc_u32 s51, s75, 0\n\t"
      KODR_BS_PROLOGUE
      "s_mov_b32 s72, %[ngrp]\n\t"
      "s_cmp_eq_u32 s72, 0\n\t"
      "s_cbranch_scc1 .Ltail_%=\n\t"
      ".Lloop_%=:\n\t"
      KODR_BS_LOOP
      "s_sub_u32 s72, s72, 1\n\t"
      "s_cmp_lg_u32 s72, 0\n\t"
      "s_cbranch_scc1 .Lloop_%=\n\t"
      ".Ltail_%=:\n\t"
      KODR_BS_TAIL
      // XOR this wave's 64 accumulator planes into the workgroup's LDS sums
      KODR_BS_REDUCE
      "s_waitcnt lgkmcnt(0)\n\t"
      "s_branch .Lend_%=\n\t"
      KODR_BS_BODIES
      ".Lend_%=:\n\t"
      :
      : [xlo] "s"(xlo), [xhi] "s"(xhi), [nrec] "s"(nrec), [kboff] "s"(kboff), [ldx] "s"(sldx),
        [plo] "s"(plo), [phi] "s"(phi), [ngrp] "s"(ngrp), [col] "v"(col),
        [lds] "v"((uint32_t)lane * 4u)
      : KODR_BS_CLOBBERS);
  __syncthreads();

  // rows m0..m0+7 of this column chunk: planes -> bytes, store
  for (int it = tid; it < kBsRows * 64; it += 64 * KW) {
    const int m = it >> 6, l = it & 63;
    const int row = m0 + m;
    const int cc = (cx * 64 + l) * kBsBlock;
    if (row >= M || cc >= ncols) continue;
    uint32_t d[8];
#pragma unroll
    for (int p = 0; p < 8; p++) d[p] = red[(m * 8 + p) * 64 + l];
    bitslice32(d);
    uint8_t* dst = Y + (size_t)row * ldy + cc;
    if (cc + kBsBlock <= ncols) {
      reinterpret_cast<uint4*>(dst)[0] = make_uint4(d[0], d[1], d[2], d[3]);
      reinterpret_cast<uint4*>(dst)[1] = make_uint4(d[4], d[5], d[6], d[7]);
    } else {
      for (int i = 0; cc + i < ncols; i++) dst[i] = (uint8_t)(d[i >> 2] >> (8 * (i & 3)));
    }
  }
}

struct BsDevice {
  uint32_t* offs = nullptr;
  bool ready = false;
};
std::mutex g_bs_mu;
BsDevice g_bs[64];

hipError_t bs_offsets(int dev, const uint32_t** out) {
  std::lock_guard<std::mutex> lk(g_bs_mu);
  if (dev < 0 || dev >= 64) return hipErrorInvalidDevice;
  BsDevice& d = g_bs[dev];
  if (!d.ready) {
    hipError_t e = hipMalloc((void**)&d.offs, 256 * sizeof(uint32_t));
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(gf_bs_export_kernel, dim3(1), dim3(64), 0, 0, d.offs);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    if ((e = hipDeviceSynchronize()) != hipSuccess) return e;
    d.ready = true;
  }
  *out = d.offs;
  return hipSuccess;
}

template <int KW>
hipError_t bs_launch(const uint8_t* A, int lda, int M, int K, const uint8_t* X, int ldx, uint8_t* Y,
                     size_t ldy, int ncols, int rpw, int ncx, int nrg, uint32_t* prog,
                     const uint32_t* offs, hipStream_t st) {
  const int nb = (ncx + 7) / 8 * 8 * nrg;
  hipLaunchKernelGGL(gf_bs_kernel<KW>, dim3(nb), dim3(64 * KW), 64 * 64 * 4, st, A, lda, M, K, X, ldx, Y,
                     ldy, ncols, rpw, ncx, nrg, prog, offs);
  return hipGetLastError();
}

}  // namespace

hipError_t bs_body_offsets(int device, uint32_t* host_out) {
  const uint32_t* offs = nullptr;
  hipError_t e = bs_offsets(device, &offs);
  if (e != hipSuccess) return e;
  return hipMemcpy(host_out, offs, 256 * sizeof(uint32_t), hipMemcpyDeviceToHost);
}

hipError_t bitslice_rows(uint8_t* dX, size_t ldx, size_t rows, size_t ncols, hipStream_t stream) {
  if (!rows || !ncols) return hipSuccess;
  if (ldx % kBsBlock || ldx < (ncols + kBsBlock - 1) / kBsBlock * kBsBlock) return hipErrorInvalidValue;
  const size_t nblk = (ncols + kBsBlock - 1) / kBsBlock;
  const size_t total = rows * nblk;
  if (rows > 0x7fffffff || nblk > 0x7fffffff) return hipErrorInvalidValue;
  hipLaunchKernelGGL(bitslice_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, dX, ldx,
                     (int)rows, (int)nblk);
  return hipGetLastError();
}

BsPlan plan_gemm_bs(size_t M, size_t K, size_t ncols) {
  BsPlan p;
  p.ncx = (int)((ncols + kBsWaveCols - 1) / kBsWaveCols);
  p.nrg = (int)((M + kBsRows - 1) / kBsRows);
  const long tasks = (long)p.ncx * p.nrg;
  int kw = 1;
  while (kw < 16 && tasks * kw < 4096 && (long)kw * 8 * 2 <= (long)K) kw *= 2;
  p.kw = kw;
  const long per = ((long)K + kw - 1) / kw;
  p.rpw = (int)std::max<long>(8, (per + 7) / 8 * 8);
  p.blocks = (p.ncx + 7) / 8 * 8 * p.nrg;
  p.prog_bytes = (size_t)p.blocks * kw * p.rpw * kBsRows * sizeof(uint32_t);
  return p;
}

hipError_t gf_gemm_bs(const uint8_t* dA, size_t lda, size_t M, size_t K, const uint8_t* dXbs, size_t ldx,
                      uint8_t* dY, size_t ldy, size_t ncols, uint32_t* d_prog, size_t prog_bytes,
                      int device, hipStream_t stream) {
  if (M == 0 || ncols == 0) return hipSuccess;
  if (ldx % kBsBlock || ldy % 16 || (size_t)K * ldx >= ((size_t)1 << 32) || ldx > 0x7fffffff ||
      lda > 0x7fffffff || M > 0x7fffffff)
    return hipErrorInvalidValue;
  const BsPlan p = plan_gemm_bs(M, K, ncols);
  if (prog_bytes < p.prog_bytes) return hipErrorInvalidValue;
  const uint32_t* offs = nullptr;
  hipError_t e = bs_offsets(device, &offs);
  if (e != hipSuccess) return e;
  const int iM = (int)M, iK = (int)K, ild = (int)lda, ilx = (int)ldx, inc = (int)ncols;
  switch (p.kw) {
    case 1: return bs_launch<1>(dA, ild, iM, iK, dXbs, ilx, dY, ldy, inc, p.rpw, p.ncx, p.nrg, d_prog, offs, stream);
    case 2: return bs_launch<2>(dA, ild, iM, iK, dXbs, ilx, dY, ldy, inc, p.rpw, p.ncx, p.nrg, d_prog, offs, stream);
    case 4: return bs_launch<4>(dA, ild, iM, iK, dXbs, ilx, dY, ldy, inc, p.rpw, p.ncx, p.nrg, d_prog, offs, stream);
    case 8: return bs_launch<8>(dA, ild, iM, iK, dXbs, ilx, dY, ldy, inc, p.rpw, p.ncx, p.nrg, d_prog, offs, stream);
    default: return bs_launch<16>(dA, ild, iM, iK, dXbs, ilx, dY, ldy, inc, p.rpw, p.ncx, p.nrg, d_prog, offs, stream);
  }
}

}  // namespace kodr_amd
