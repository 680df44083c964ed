// gf_elim.hip -- kodr's decoder elimination on the GPU, one workgroup per
// generation (decoder), for batched AddPiece on fresh decoders.
//
// What kodr computes, and what the kernel may therefore compute instead.
// kodr's DecoderState (decoder_state.go:15-182) pivots on the diagonal only;
// its state keeps a zero strict lower triangle (decoder_core.cpp) and drops a
// row only when it becomes zero, which a linearly independent row never does.
// Two cases have a state that does not depend on the route:
//  * FULL: a batch of n >= k rows whose first k coding vectors C are linearly
//    independent.  kodr accepts all k (none can vanish, and rank counts kept
//    rows, so it reaches k exactly at row k - 1) and then holds an upper
//    triangular, invertible -- so diagonal -- coefficient half, which its
//    backward pass normalizes: the state is [I | C^-1], T's columns in arrival
//    order.  The kernel inverts C by Gauss-Jordan with a pivot search (the
//    lowest unused row with a non-zero entry in the column, so the clean case
//    pivots on the diagonal as kodr does); a column with no candidate means C
//    is singular and the whole batch goes back to the host (c = 0).
//  * CLEAN: fewer than k rows, all landing on their diagonals (after reduction
//    against the earlier pivots, row r has a non-zero entry in column r).
//    Then the state after c rows is the reduced row echelon form of
//    [C_c | I_c] (decoder_core.cpp add_panel), unique.  The kernel pivots on
//    the diagonal only and stops at the first zero: c = r.
// The host loads the state into DecoderCore and runs kodr's literal
// algorithm on whatever is left (decoder_core.cpp), so its quirks (zero
// diagonals with rank over-count, dependent rows) never need the GPU.  c < 2
// is reported as 0: kodr keeps the first piece unreduced until a second one
// arrives (full/decoder.go:58-61).
//
// Layout.  Row j (bytes [0, k) coefficients, [k, k + n) the transform T) lives
// in registers: wave w owns rows 16w .. 16w+15, lane l owns dwords l and
// l + 64 of each (DPL = 1 dword per lane for k <= 128, 2 for k <= 256).
//
// Multiply.  x -> f*x is GF(2)-linear, so f*x = T0[x & 7] ^ T1[(x >> 3) & 7] ^
// T2[x >> 6] with 8-, 8- and 4-entry byte tables of f (gf256.go:15-44, poly
// 0x11D), one v_perm_b32 each for 4 bytes.  The pivot row's selectors are
// computed once per step and shared by the rows each wave updates; a row's
// tables come from a table of all 256 multipliers through the scalar cache
// (the multiplier is wave-uniform).  The multiplier of row j at
// step r is byte r of row j, read wavefront-wide with v_readlane (its owner
// lane is r / 4); the pivot search takes the LDS atomic minimum of the
// waves' candidates.
//
// Sync.  Two workgroup barriers per step: after the candidates, and after the
// owner wave of the pivot has normalized it (multiplier inv(d), gf256.go:77-86)
// and published it in LDS (two buffers, alternating).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gf_kernels.hpp"

namespace kodr_amd {

namespace {

constexpr int kElimWaves = 16;
constexpr int kElimRowsPerWave = 16;   // 16 x 16 = 256 rows
constexpr int kNone = 0x7fffffff;

// LDS: two pivot buffers [2][128] dwords, the pivot choice (three rotating
// slots, LDS atomic min of the waves' candidates), the pivot column of every
// row, the stop word.  The field tables ([256][8]
// dwords: T0 lo/hi, T1 lo/hi, T2, pad; then the 256 inverse bytes) are read
// with scalar loads: every index is wave-uniform.
struct ElimLds {
  uint32_t piv[2][128];
  int best[3];               // pivot of step r: min over the waves' candidates, slot r % 3
  int colof[256];
  int stop;
};

__device__ __forceinline__ uint32_t gmul4(const uint4& t01, uint32_t t2, uint32_t s0, uint32_t s1, uint32_t s2) {
  return __builtin_amdgcn_perm(t01.y, t01.x, s0) ^ __builtin_amdgcn_perm(t01.w, t01.z, s1) ^
         __builtin_amdgcn_perm(t2, t2, s2);
}

template <int DPL>
__global__ __launch_bounds__(64 * kElimWaves) void gf_elim_kernel(ElimArgs args) {
  __shared__ ElimLds lds;
  const int g = blockIdx.x;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave index: uniform, keep it scalar
  const int k = args.k;
  const bool full = args.n[g] >= k;
  const int n = min(args.n[g], k);
  const int j0 = w * kElimRowsPerWave;  // this wave's first row
  const uint8_t* vec = args.vecs[g];
  const size_t vp = args.vpitch;
  // [256][8] tables, then 64 dwords of inverses; constant address space, so
  // the wave-uniform reads become scalar loads through the scalar cache
  typedef const __attribute__((address_space(4))) uint32_t cu32;
  cu32* tb = (cu32*)args.tables;

  for (int i = tid; i < 256; i += 64 * kElimWaves) lds.colof[i] = -1;
  if (tid < 3) lds.best[tid] = kNone;
  if (tid == 0) lds.stop = -1;

  // rows in registers: S[i][h] = dword (h * 64 + lane) of row j0 + i
  uint32_t S[kElimRowsPerWave][DPL];
#pragma unroll
  for (int i = 0; i < kElimRowsPerWave; i++) {
    const int j = j0 + i;
#pragma unroll
    for (int h = 0; h < DPL; h++) {
      uint32_t v = 0;
      if (j < n) {
#pragma unroll
        for (int b = 0; b < 4; b++) {
          const int col = (h * 64 + lane) * 4 + b;
          uint32_t byte = 0;
          if (col < k) byte = vec[(size_t)j * vp + col];
          else if (col == k + j) byte = 1;  // T row = e_j
          v |= byte << (8 * b);
        }
      }
      S[i][h] = v;
    }
  }
  uint32_t used = 0;  // this wave's rows already chosen as pivots (bit i)
  const uint32_t live = j0 >= n ? 0u : (n - j0 >= 32 ? 0xffffffffu : (1u << (n - j0)) - 1u) & 0xffffu;
  __syncthreads();

#ifdef KODR_ELIM_TIMING
  uint64_t ts[8];  // s_memtime of step 10's phases (wave 0), written to out (tuning only)
#endif
  for (int r = 0; r < n; r++) {
#ifdef KODR_ELIM_TIMING
    if (r == 10) ts[0] = __builtin_amdgcn_s_memtime();
#endif
    const int rl = r >> 2, rb = 8 * (r & 3);  // column r: lane r / 4 of dword 0, byte r % 4
    // rows of this wave with a non-zero entry in column r (wavefront-wide
    // v_readlane of the owner lane); candidate: FULL, the lowest unused one;
    // CLEAN, row r itself
    uint32_t nz = 0;
#pragma unroll
    for (int i = 0; i < kElimRowsPerWave; i++)
      nz |= (((__builtin_amdgcn_readlane(S[i][0], rl) >> rb) & 0xffu) != 0u ? 1u : 0u) << i;
    nz &= live;
    uint32_t cm = full ? (nz & ~used) : ((r >= j0 && r < j0 + kElimRowsPerWave) ? nz & (1u << (r - j0)) : 0u);
    cm = __builtin_amdgcn_readfirstlane(cm);
    if (lane == 0 && cm) atomicMin(&lds.best[r % 3], j0 + __builtin_ctz(cm));
    if (tid == 0) lds.best[(r + 1) % 3] = kNone;  // read two steps ago, next written next step
#ifdef KODR_ELIM_TIMING
    if (r == 10) ts[1] = __builtin_amdgcn_s_memtime();
#endif
    __syncthreads();
#ifdef KODR_ELIM_TIMING
    if (r == 10) ts[2] = __builtin_amdgcn_s_memtime();
#endif
    const int p = __builtin_amdgcn_readfirstlane(lds.best[r % 3]);
    if (p == kNone) {  // FULL: C singular; CLEAN: a zero diagonal (uniform)
      if (tid == 0) lds.stop = r;
      break;
    }
    if (p >= j0 && p < j0 + kElimRowsPerWave) {  // the owner: normalize row p, publish it
      const int io = p - j0;
#pragma unroll
      for (int i = 0; i < kElimRowsPerWave; i++)
        if (i == io) {
          const uint32_t d = (__builtin_amdgcn_readlane(S[i][0], rl) >> rb) & 0xffu;
          const uint32_t inv = (tb[256 * 8 + (d >> 2)] >> (8 * (d & 3))) & 0xffu;  // gf256.go:77-86
          const uint4 t01 = {tb[inv * 8], tb[inv * 8 + 1], tb[inv * 8 + 2], tb[inv * 8 + 3]};
          const uint32_t t2 = tb[inv * 8 + 4];
#pragma unroll
          for (int h = 0; h < DPL; h++) {
            const uint32_t x = S[i][h];
            S[i][h] = gmul4(t01, t2, x & 0x07070707u, (x >> 3) & 0x07070707u, (x >> 6) & 0x03030303u);
            lds.piv[r & 1][h * 64 + lane] = S[i][h];
          }
        }
      used |= 1u << io;
      if (lane == 0) lds.colof[p] = r;
    }
#ifdef KODR_ELIM_TIMING
    if (r == 10) ts[3] = __builtin_amdgcn_s_memtime();
#endif
    __syncthreads();
#ifdef KODR_ELIM_TIMING
    if (r == 10) ts[4] = __builtin_amdgcn_s_memtime();
#endif
    uint32_t s0[DPL], s1[DPL], s2[DPL];
#pragma unroll
    for (int h = 0; h < DPL; h++) {
      const uint32_t x = lds.piv[r & 1][h * 64 + lane];
      s0[h] = x & 0x07070707u;
      s1[h] = (x >> 3) & 0x07070707u;
      s2[h] = (x >> 6) & 0x03030303u;
    }
    // eliminate column r from every other row with a non-zero entry there
    const uint32_t todo = nz & ~(p >= j0 && p < j0 + kElimRowsPerWave ? 1u << (p - j0) : 0u);
    // in groups of 8 rows: all multipliers, then all their tables (scalar
    // loads issued together, one wait), then the arithmetic; a row that must
    // not change (the pivot, a zero entry, past n) has multiplier 0, whose
    // table is all zero
    constexpr int kGroup = 8;
#pragma unroll
    for (int i0 = 0; i0 < kElimRowsPerWave; i0 += kGroup) {
      uint32_t f[kGroup];
#pragma unroll
      for (int q = 0; q < kGroup; q++) {
        const uint32_t v = (__builtin_amdgcn_readlane(S[i0 + q][0], rl) >> rb) & 0xffu;
        f[q] = ((todo >> (i0 + q)) & 1u) ? v : 0u;
      }
      uint4 a[kGroup];
      uint32_t b[kGroup];
#pragma unroll
      for (int q = 0; q < kGroup; q++) {
        a[q] = {tb[f[q] * 8], tb[f[q] * 8 + 1], tb[f[q] * 8 + 2], tb[f[q] * 8 + 3]};
        b[q] = tb[f[q] * 8 + 4];
      }
#pragma unroll
      for (int q = 0; q < kGroup; q++)
#pragma unroll
        for (int h = 0; h < DPL; h++) S[i0 + q][h] ^= gmul4(a[q], b[q], s0[h], s1[h], s2[h]);
    }
#ifdef KODR_ELIM_TIMING
    if (r == 10) ts[5] = __builtin_amdgcn_s_memtime();
    if (r == 11) ts[6] = __builtin_amdgcn_s_memtime();
#endif
  }
#ifdef KODR_ELIM_TIMING
  ts[7] = __builtin_amdgcn_s_memtime();
  if (lane == 0) {
    uint64_t* o = reinterpret_cast<uint64_t*>(args.out + (size_t)g * args.out_gen_stride) + 8 * w;
    for (int q = 0; q < 8; q++) o[q] = ts[q];
  }
  return;
#endif
  __syncthreads();
  int c = lds.stop >= 0 ? lds.stop : n;
  if (full && c < k) c = 0;  // singular: kodr's own route (host) for the whole batch
  if (c < 2) c = 0;          // the first piece stays unreduced until a second one (full/decoder.go:58-61)
  // rows in pivot order: the row that pivoted column r is row r of the state
  uint8_t* out = args.out + (size_t)g * args.out_gen_stride;
#pragma unroll
  for (int i = 0; i < kElimRowsPerWave; i++) {
    const int j = j0 + i;
    const int at = j < 256 ? lds.colof[j] : -1;
    if (at < 0 || at >= c) continue;
#pragma unroll
    for (int h = 0; h < DPL; h++)
      reinterpret_cast<uint32_t*>(out + (size_t)at * args.out_pitch)[h * 64 + lane] = S[i][h];
  }
  if (tid == 0) args.counts[g] = c;
}

}  // namespace

void elim_tables(uint32_t* host_out) {
  // [256][8] dwords: T0 = f*{0..7}, T1 = f*({0..7} << 3), T2 = f*({0..3} << 6)
  // as little-endian byte tables for v_perm (lo dword = entries 0..3); then
  // the 256 inverse bytes (gf256.go:77-86; inv(0) unused)
  auto mul = [](unsigned a, unsigned b) {
    unsigned r = 0;
    while (b) {
      if (b & 1) r ^= a;
      a <<= 1;
      if (a & 0x100) a ^= 0x11D;
      b >>= 1;
    }
    return r;
  };
  for (unsigned f = 0; f < 256; f++) {
    uint8_t t[20] = {};
    for (unsigned i = 0; i < 8; i++) {
      t[i] = (uint8_t)mul(f, i);
      t[8 + i] = (uint8_t)mul(f, i << 3);
    }
    for (unsigned i = 0; i < 4; i++) t[16 + i] = (uint8_t)mul(f, i << 6);
    for (int q = 0; q < 8; q++) {
      uint32_t v = 0;
      if (q < 5)
        for (int b = 0; b < 4; b++) v |= (uint32_t)t[q * 4 + b] << (8 * b);
      host_out[f * 8 + q] = v;
    }
  }
  uint8_t inv[256] = {};
  for (unsigned a = 1; a < 256; a++)
    for (unsigned b = 1; b < 256; b++)
      if (mul(a, b) == 1) {
        inv[a] = (uint8_t)b;
        break;
      }
  for (int i = 0; i < 64; i++)
    host_out[256 * 8 + i] = (uint32_t)inv[4 * i] | ((uint32_t)inv[4 * i + 1] << 8) |
                            ((uint32_t)inv[4 * i + 2] << 16) | ((uint32_t)inv[4 * i + 3] << 24);
}

hipError_t gf_elim(const ElimArgs& args, int G, hipStream_t stream) {
  if (G <= 0) return hipSuccess;
  if (G > kElimMaxGens || args.k < 2 || args.k > 256 || args.out_pitch % 4 ||
      args.out_pitch < (size_t)(args.k <= 128 ? 256 : 512))
    return hipErrorInvalidValue;
  if (args.k <= 128)
    hipLaunchKernelGGL(gf_elim_kernel<1>, dim3(G), dim3(64 * kElimWaves), 0, stream, args);
  else
    hipLaunchKernelGGL(gf_elim_kernel<2>, dim3(G), dim3(64 * kElimWaves), 0, stream, args);
  return hipGetLastError();
}

}  // namespace kodr_amd
