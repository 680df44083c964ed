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

// What the last product launch of this thread ran (diagnostics behind
// rlnc_last_launch_plan: tests pin the exact instance the bench times).
// kernel 1 = gf_gemm_kernel, 2 = gf_bs_kernel.
struct LaunchPlan {
  int kernel = 0, tile_rows = 0, waves = 0, lane_groups = 0, ring = 0, rows_per_wave = 0, generations = 0,
      workgroups = 0;
};
LaunchPlan& last_launch_plan();

// A group of independent products of one shape (M, K, ncols, pitches) in one
// launch: product i reads X = x[i], A + i * a_stride and writes Y + i * y_stride.
constexpr int kGemmGroupMax = 32;
struct GemmGroup {
  const uint8_t* x[kGemmGroupMax];
};
struct GemmGroupArgs {
  int n;
  const uint8_t* const* x;
  size_t a_stride, y_stride;
};
// cache policy of a grouped launch's row loads (2 = nt: each generation is
// read once per launch)
constexpr int kGroupAux = 2;

// Y[m][j] = XOR_k A[m][k] * X[k][j], m < M, j < ncols.  All pointers device.
// accumulate: Y[m][j] ^= that product instead (one row chunk of a K-split).
// ldx/ldy multiples of 16 and >= ncols; X rows readable up to round_up(ncols,16).
hipError_t gf_gemm(const uint8_t* dA, size_t lda, size_t M, size_t K, const uint8_t* dX,
                   size_t ldx, uint8_t* dY, size_t ldy, size_t ncols, hipStream_t stream,
                   const GemmConfig* force = nullptr, bool accumulate = false,
                   const GemmGroupArgs* group = nullptr);

// dst (pitch dpitch) = width x rows contiguous bytes of host-mapped pinned
// memory (a device pointer of a hipHostMalloc buffer), copied by a kernel
// rather than a DMA engine.  width x rows <= kUploadSmallMax.
constexpr size_t kUploadSmallMax = 64 * 1024;
// download_small: up to this many bytes (the coding vectors of a batched
// AddPiece: 258 x 256 B at 32 MiB/256)
constexpr size_t kDownloadSmallMax = 256 * 1024;
hipError_t upload_small(const uint8_t* src_mapped, uint8_t* dst, size_t dpitch, size_t width, size_t rows,
                        hipStream_t stream);
// the reverse: width x rows bytes of device memory (pitch spitch) into
// host-mapped pinned memory, contiguous rows
hipError_t download_small(const uint8_t* src, size_t spitch, uint8_t* dst_mapped, size_t width, size_t rows,
                          hipStream_t stream);

// dY row r = the first ncols bytes of device row d_src[r] (d_src: device array
// of rows pointers, 16-byte aligned).  rows <= 65535.
// dst row r = the first ncols bytes of src row r, device to device, as a
// kernel: a few rows cost a launch (~2 us of host time) instead of a
// hipMemcpy2DAsync call.  rows <= 65535.
hipError_t copy_rows(const uint8_t* src, size_t spitch, uint8_t* dst, size_t dpitch, size_t rows, size_t ncols,
                     hipStream_t stream);

// dst row r = device row d_src[r] (16-byte aligned); written at d_dst[r] when
// d_dst (a device table) is given, else at dY + r * ldy.  rows <= 65535.  A
// source pointer with bit 0 set is a row of a bit-sliced twin (ncols a
// multiple of 32): its plain bytes are gathered (un-sliced on the way).
hipError_t gather_rows(const uint8_t* const* d_src, uint8_t* dY, size_t ldy, size_t rows, size_t ncols,
                       hipStream_t stream, uint8_t* const* d_dst = nullptr);

// rows x k coding vectors at row pitch ldv: rows [0, n_sys) = e_(sys_first+r),
// the rest counter-based pseudo-random bytes of (seed, row0 + r).  rows <= 65535.
hipError_t fill_vectors(uint8_t* dV, size_t ldv, size_t rows, size_t k, uint64_t seed, uint64_t row0,
                        size_t n_sys, size_t sys_first, hipStream_t stream);
// the same for n <= kGemmGroupMax encoders in one launch: encoder i writes
// rows x k bytes at v[i] (pitch ldv) from its own (seed, row0, n_sys, sys_first)
struct VectorGroup {
  uint8_t* v[kGemmGroupMax];
  uint64_t seed[kGemmGroupMax], row0[kGemmGroupMax];
  int n_sys[kGemmGroupMax], sys_first[kGemmGroupMax];
};
hipError_t fill_vectors_grouped(const VectorGroup& g, int n, size_t ldv, size_t rows, size_t k, hipStream_t stream);

// ---- decoder elimination on the GPU (gf_elim.hip) ----
// One workgroup per decoder: Gauss-Jordan of the first n coding vectors of
// generation g in arrival order while every pivot lands on its diagonal; the
// state after c clean rows (c x (k + c) bytes: coefficients [I | X], T) is
// written at out + g * out_gen_stride with row pitch out_pitch, and c (0 when
// fewer than 2 rows were clean) at counts[g].  2 <= k <= 256.
constexpr int kElimMaxGens = 64;
struct ElimArgs {
  const uint8_t* vecs[kElimMaxGens];  // generation g's first coding vector (device)
  int n[kElimMaxGens];                // its rows
  uint64_t vpitch;                    // bytes between consecutive vectors
  const uint32_t* tables;             // elim_tables(), on the device
  uint8_t* out;
  uint64_t out_gen_stride, out_pitch; // out_pitch >= 256 (k <= 128) or 512
  int* counts;
  int k;
  // gf_elim_mc only: the hand-off buffer (gf_elim_mc_pub_bytes, zeroed once
  // when allocated) and this launch's first tag: the launch uses tags epoch ..
  // epoch + gf_elim_mc_attempts() - 1 (one per attempt), all above every tag
  // an earlier launch on the buffer used, below 2^31
  uint64_t* pub;
  uint32_t epoch;
  // mc2 / mc4 ("direct"): T rows at out + row * out_pitch (no [I] part), and
  // the status words counts[g * groups + q] = epoch + a (done in attempt a)
  // or that | 0x80000000 (failed), stored with system-scope release after the
  // workgroup's T rows, so a host polling pinned memory can read them early
  int direct;
  // mc2 / mc4 only (optional): the T rows of a finished decoder also to
  // device memory, out_dev + g * k * k + row * k (GetPieces reads them there)
  uint8_t* out_dev;
};
// [256][8] tables of f, 64 dwords of inverse bytes, [256][8] tables of inv(f)
constexpr size_t kElimInvTables = 256 * 8 + 64;
constexpr size_t kElimTableWords = kElimInvTables + 256 * 8;
void elim_tables(uint32_t* host_out);  // kElimTableWords dwords
// true when gf_elim takes the blocked kernel for this launch: every count is
// then k (the state is [I | C^-1]: only T = C^-1 needs reading back) or 0
bool gf_elim_blocked(const ElimArgs& args, int G);
hipError_t gf_elim(const ElimArgs& args, int G, hipStream_t stream);
// Full batches on several workgroups per decoder (gf_elim_mc_kernel): the
// rows of a decoder are split into groups of 32, one workgroup each, which
// hand their pivot rows to each other through `pub`.  Taken by gf_elim for
// full batches when args.pub is set and G * groups <= kElimMcMaxBlocks.
// Instead of counts[g] it writes one status word per workgroup,
// counts[g * groups + q] = 1 (done) or 0 (a singular block or a timeout: the
// host then takes kodr's route); the decoder's T is valid when all are 1.
#ifndef KODR_ELIM_MC_MAX_BLOCKS  // (tuning builds only: more decoders per mc4 launch, the round-5 fault check)
#define KODR_ELIM_MC_MAX_BLOCKS 256
#endif
constexpr int kElimMcMaxBlocks = KODR_ELIM_MC_MAX_BLOCKS;
// workgroups per decoder of the multi-workgroup kernel a launch of G
// decoders takes: ceil(k / 32) (gf_elim_mc / mc2), or one per 8 rows plus the
// chain workgroup (mc4); and the most decoders one such launch takes
int gf_elim_mc_groups(int k, int G);
int gf_elim_mc_max_gens(int k);
size_t gf_elim_mc_pub_bytes(int k, int G);
// tags per launch: attempts with the rows in another order after a singular
// panel block (gf_elim.hip, kMcAttempts)
int gf_elim_mc_attempts();
bool gf_elim_mc_taken(const ElimArgs& args, int G);
// true when gf_elim_mc_taken and the launch honours args.direct (mc2)
bool gf_elim_mc_direct(const ElimArgs& args, int G);
bool gf_elim_mc_enabled();  // KODR_ELIM_MC != 0

// ---- bit-sliced path (gf_bs.hip) ----
// dst = src with every 32-byte block of rows [0, rows) x [0, round_up(ncols,
// 32)) turned into 8 bit planes (self-inverse); src == dst works in place.
// Both use pitch ldx, a multiple of 32; dst's bytes past those blocks are not
// written.
hipError_t bitslice_rows(const uint8_t* src, uint8_t* dst, size_t ldx, size_t rows, size_t ncols,
                         hipStream_t stream);
// the same from src (pitch spitch, 16-byte aligned rows; each row readable up
// to round_up(ncols, 32) bytes) into dst at pitch dpitch (multiple of 32)
hipError_t bitslice_rows_pitched(const uint8_t* src, size_t spitch, uint8_t* dst, size_t dpitch, size_t rows,
                                 size_t ncols, hipStream_t stream);

// dst rows = the first ncols bytes of src rows, and dst_bs rows = the same
// rows bit-sliced (as bitslice_rows), from one read of src.  ncols and dpitch
// multiples of 32; src, spitch, dst, dst_bs 16-byte aligned (else
// hipErrorInvalidValue: the caller copies and bit-slices in two passes).
// (dst == nullptr: the twin only)
hipError_t copy_bitslice_rows(const uint8_t* src, size_t spitch, uint8_t* dst, uint8_t* dst_bs, size_t dpitch,
                              size_t rows, size_t ncols, hipStream_t stream);
// copy_bitslice_rows for up to kCopyGroupMax row sets of one shape (ncols,
// pitches) in one launch: set i = rows[i] rows from src[i] to dst[i], dbs[i].
// The same alignment rules; copy_bitslice_ok checks one set.
constexpr int kCopyGroupMax = 64;
struct CopyGroup {
  const uint8_t* src[kCopyGroupMax];
  uint8_t* dst[kCopyGroupMax];
  uint8_t* dbs[kCopyGroupMax];
  int rows[kCopyGroupMax];
};
bool copy_bitslice_ok(const uint8_t* src, size_t spitch, const uint8_t* dst, const uint8_t* dst_bs, size_t dpitch,
                      size_t ncols);
// beside: the copies share the GPU with the elimination kernel (capped
// residency, so its workgroups find room); else they run alone
hipError_t copy_bitslice_rows_grouped(const CopyGroup& g, int n, size_t spitch, size_t dpitch, size_t ncols,
                                      hipStream_t stream, bool beside = false);

// byte offsets of the 256 coefficient bodies (copy 0) from body 0 (diagnostics)
hipError_t bs_body_offsets(int device, uint32_t* host_out);

// true once the bodies' addresses were exported and checked on this device
// (the bit-sliced path is usable); false sends callers to gf_gemm
bool bs_ready(int device);

struct BsPlan {
  int ncx = 0, nrg = 0, kw = 1, rpw = 8, blocks = 0;
  size_t lds_bytes = 0;  // per workgroup: row sums, offset table, programs
  bool ok = false;       // false when K is too large for the LDS program
};
// groups: independent products of this shape in one launch (grid rows)
// grouped: the launch is a grouped one (gf_gemm_bs with group), where one
// wave per workgroup takes the direct variant (no LDS fold)
BsPlan plan_gemm_bs(size_t M, size_t K, size_t ncols, int groups = 1, bool grouped = false);

// Side product of a single bit-sliced launch: y = A (x) x over plain rows of
// ncols bytes (the recoded coding vectors beside the recoded pieces); 16-byte
// aligned rows and pitches, ldx >= ncols rounded up to 16, K * ldx < 2^31.
struct BsSide {
  const uint8_t* x = nullptr;
  size_t ldx = 0;
  uint8_t* y = nullptr;
  size_t ldy = 0;
  size_t ncols = 0;
};
bool side_ok(const BsSide& side, size_t K);

// Y = A (x) X with X bit-sliced (bitslice_rows), Y in plain bytes.  group:
// up to kGemmGroupMax products of this shape in one launch (X = group->x[i],
// A + i * a_stride, Y + i * y_stride; dXbs unused).  side (single launches,
// not accumulating): also y = A (x) x in the same launch.
hipError_t gf_gemm_bs(const uint8_t* dA, size_t lda, size_t M, size_t K, const uint8_t* dXbs, size_t ldx,
                      uint8_t* dY, size_t ldy, size_t ncols, int device, hipStream_t stream,
                      bool accumulate = false, const GemmGroupArgs* group = nullptr,
                      const BsSide* side = nullptr);

}  // namespace kodr_amd
