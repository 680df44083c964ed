// capi_internal.hpp -- what the translation units of the C ABI share
// (capi.cpp: context, encoder, recoder; capi_decoder.cpp: decoder): the
// handle structs behind include/kodr_rlnc.h, the device-buffer wrapper, the
// error plumbing and the product helpers.  Internal: not installed.
#pragma once
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <stdio.h>
#include <string.h>
#include <sys/random.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <functional>
#include <future>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kodr_rlnc.h"
#include "decoder_core.hpp"
#include "host_gf.hpp"
#include "host_pool.hpp"
#include "gf_kernels.hpp"
#include "pool.hpp"
#include "staging.hpp"
#include "tune.hpp"

using kodr_amd::DecoderCore;
using kodr_amd::HostPool;

namespace kodr_capi {

inline thread_local std::string g_last_error;

inline int hip_fail(hipError_t e, const char* what) {
  g_last_error = std::string(what) + ": " + hipGetErrorString(e);
  return (e == hipErrorNoDevice || e == hipErrorInvalidDevice) ? RLNC_ERR_NO_DEVICE : RLNC_ERR_HIP;
}

#define HIPC(expr)                                 \
  do {                                             \
    hipError_t _e = (expr);                        \
    if (_e != hipSuccess) return hip_fail(_e, #expr); \
  } while (0)

constexpr size_t kPitchAlign = 256;
inline size_t round_up(size_t x, size_t a) { return (x + a - 1) / a * a; }
constexpr size_t kMaxDescBytes = (size_t)1 << 31;  // gf_gemm's signed 32-bit buffer offsets: X rows per launch

// Device buffer that only grows, from the device's caching pool (pool.hpp),
// ordered on the owner's stream (bind before the first reserve).
struct DevBuf {
  uint8_t* p = nullptr;
  size_t cap = 0;
  int dev = 0;
  hipStream_t st = nullptr;
  void bind(int device, hipStream_t stream) {
    dev = device;
    st = stream;
  }
  int reserve(size_t bytes) {
    if (bytes <= cap) return RLNC_OK;
    release();
    HIPC(kodr_amd::DevicePool::get(dev).alloc(bytes, st, &p, &cap));
    return RLNC_OK;
  }
  void release(bool idle = false) {  // idle: nothing pending uses p (DevicePool::free)
    if (p) kodr_amd::DevicePool::get(dev).free(p, cap, st, idle);
    p = nullptr;
    cap = 0;
  }
  // hand the block to the caller (who frees it with DevicePool::defer_free)
  void take(uint8_t** pp, size_t* pc) {
    *pp = p;
    *pc = cap;
    p = nullptr;
    cap = 0;
  }
};


}  // namespace kodr_capi

// the helpers of this header, unqualified in the C ABI's translation units
using namespace kodr_capi;

struct rlnc_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  kodr_amd::Staging stage;   // pinned chunks for host-pointer copies
  DevBuf elim_tab;           // gf_elim's field tables (once per context)
  bool elim_tab_ok = false;
  DevBuf elim_out;           // gf_elim's per-generation states and counts
  DevBuf elim_in;            // gf_elim's input for continued decoders: [coefficient rows ; vectors]
  DevBuf gtab;               // grouped flush: source and destination tables of the gathered pieces
  std::vector<uint8_t> elim_host;  // its read-back (grown once, never zero-filled)
  std::vector<uint8_t> elim_hin;   // host side of elim_in (grown once)
  DevBuf gtmat[2];           // grouped GetPieces: transforms of one chunk, alternating per chunk
  uint8_t* elim_pin = nullptr;      // gf_elim_mc2's direct output: status words + T rows (pinned, coherent)
  uint8_t* elim_pin_dev = nullptr;  // ... as the device sees it
  size_t elim_pin_cap = 0;
  DevBuf elim_pub;           // gf_elim_mc's hand-off granules (zeroed when allocated)
  uint32_t elim_epoch = 0;   // gf_elim_mc's last tag used: a launch takes the next gf_elim_mc_attempts()
  size_t route_min_k = 224;  // single decoders take the GPU elimination from this k (rlnc_ctx_set_route_min_k)
  // rlnc_decoder_elim_stats summed over the context's decoders (rlnc_ctx_elim_stats)
  std::atomic<size_t> n_elim_gpu{0}, n_elim_gpu_retried{0}, n_elim_host_after_gpu{0}, n_elim_host{0};
  DevBuf elim_tdev;          // fresh decoders' T rows (k x k each) as the last batched GPU AddPiece left them
  uint64_t tdev_seq = 0;     // ... one number per such call
  hipStream_t side = nullptr;      // batched GPU AddPiece: row copies beside the elimination
  hipEvent_t side_done = nullptr;  // ... and the context stream's wait for them
  hipEvent_t rows_ready = nullptr; // ... the rows' producer work: the side copies and the aux reads wait on it
  hipEvent_t elim_ready = nullptr; // recorded right before a direct elimination launch (its give-up clock)
  hipStream_t aux = nullptr;       // small downloads that must not queue behind the side copies
  // batched GPU AddPiece: the batch's coding vectors, downloaded beside every
  // elimination launch for the decoders it leaves to the host route
  uint8_t* vec_pin = nullptr;
  size_t vec_pin_cap = 0;
  hipEvent_t vec_ready = nullptr;
};

struct rlnc_encoder {
  rlnc_ctx* ctx = nullptr;
  int kind = RLNC_FULL;
  size_t k = 0, L = 0, pitch = 0, padding = 0;
  size_t sys_next = 0;       // systematic/encoder.go:8 currentPieceId
  uint64_t seed = 0, drawn = 0;  // device vector RNG: seed, rows drawn so far
  DevBuf pieces;             // k x pitch, zero padded
  DevBuf pieces_bs;          // bit-sliced twin of pieces, built on first large batch
  bool bs_valid = false;
  bool compact = false;      // rlnc_encoder_compact: only the twin is resident
  DevBuf vecs, out;          // staging for host-pointer calls
};

struct rlnc_recoder {
  rlnc_ctx* ctx = nullptr;
  size_t n = 0, k = 0, clen = 0, pitch = 0;
  size_t L = 0, ppitch = 0;  // piece length (clen - k) and the piece twin's pitch
  DevBuf flat;               // n x pitch wire rows (released when compact)
  DevBuf flat_bs;            // bit-sliced twin of the wire rows (shapes the split layout cannot take)
  bool bs_valid = false;
  DevBuf piece_bs;           // split layout: bit-sliced twin of the piece columns only (pitch ppitch)
  bool piece_bs_valid = false;
  DevBuf vecs;               // compact split recoder: the n coding vectors (pitch vpitch)
  size_t vpitch = 0;
  bool compact = false;      // rlnc_recoder_compact: only the twin (and, split, the vectors) resident
  DevBuf r, out, scratch;
};

struct rlnc_decoder {
  rlnc_ctx* ctx = nullptr;   // may be null: coefficient side only
  DecoderCore core;
  // this decoder's T (k x k, pitch k) in ctx->elim_tdev, valid while
  // ctx->tdev_seq == tdev_seq (the GPU elimination of a fresh full batch)
  const uint8_t* tdev = nullptr;
  uint64_t tdev_seq = 0;
  size_t L = 0, pitch = 0;
  bool have_len = false;
  DevBuf recv;               // received pieces, row i = piece i, pitch
  size_t recv_rows = 0;
  DevBuf recv_bs;            // bit-sliced twin of recv rows [0, bs_rows)
  size_t bs_rows = 0;
  // compact rows: received rows [cmp_lo, cmp_hi) exist only in the twin (the
  // batched device-row copies write the twin alone: T x R reads nothing else);
  // a plain-row reader un-slices them first (dec_uncompact), a gather of
  // systematic rows un-slices on the fly (gather_rows' twin rows)
  size_t cmp_lo = 0, cmp_hi = 0;
  DevBuf tmat;               // transform upload
  DevBuf decoded;            // useful x pitch, valid when decoded_ready
  DevBuf rowbuf;             // one row for partial GetPiece
  bool decoded_ready = false;
  std::vector<uint8_t> hT;
  std::vector<uint8_t> hvecs;  // coding vectors of a device batch
  std::vector<uint8_t> hTc;    // transform rows that need GF work
  std::vector<const uint8_t*> hsrc;  // per output row: source row of the gather
  DevBuf scratch;              // GF rows before the gather
  size_t last_gf_rows = 0, last_copy_rows = 0;
  bool last_bs = false;         // the last GF product ran on the bit-sliced kernel
  // progressive decode: original pieces materialized before
  // GetPieces, in slots of `prog` in the order they were made, or at row j of
  // the caller's bound output (rlnc_decoder_bind_output)
  int policy = RLNC_DECODE_LAZY;
  DevBuf prog;
  std::vector<int32_t> slot_of;  // per original piece: its slot, or -1
  size_t nslots = 0;
  uint8_t* out_ext = nullptr;    // bound output: piece j at out_ext + j * out_pitch
  size_t out_pitch = 0;
  std::vector<uint8_t*> hdst;    // per materialized row: its destination
  std::vector<int32_t> drow;     // DecoderCore::decoded() scratch
  std::vector<uint8_t> dscale;
  // Lazy AddPiece: coding vectors accepted while they cannot complete the
  // rank are queued and eliminated as one batch (DecoderCore::add_many, the
  // same state as row-by-row adds) when the state is next observed or could
  // be complete; device pieces are referenced until the next data flush and
  // then copied by one gather launch.  Every accessor flushes first, so what a
  // caller can observe is kodr's state after each AddPiece.
  bool lazy = true;
  std::vector<uint8_t> pend_v;           // queued coding vectors, k bytes each
  size_t npend = 0;
  std::vector<const uint8_t*> pend_src;  // queued device pieces (borrowed), arrival order
  size_t pend_row0 = 0;                  // received index of pend_src[0]
  DevBuf ptab;                           // the gather's source-row table
  // which route eliminated this decoder's batches (rlnc_decoder_elim_stats)
  size_t elim_gpu = 0, elim_gpu_retried = 0, elim_host_after_gpu = 0, elim_host = 0;
  bool gpu_rejected = false;  // the GPU elimination failed on the queue as it is: the host takes it
  int sticky = RLNC_OK;       // a HIP failure inside a state accessor, reported by the next call that can
  explicit rlnc_decoder(size_t k) : core(k) {}
};

namespace kodr_capi {

inline int set_dev(const rlnc_ctx* ctx) {
  if (!ctx) return RLNC_ERR_NO_DEVICE;
  HIPC(hipSetDevice(ctx->device));
  return RLNC_OK;
}

#define TRY(expr)              \
  do {                         \
    int _s = (expr);           \
    if (_s != RLNC_OK) return _s; \
  } while (0)

// split rules of data.go:103-166
inline int split_count(size_t len, size_t count, size_t* size, size_t* pad) {
  if (count < 2) return RLNC_ERR_BAD_PIECE_COUNT;
  if (count > len) return RLNC_ERR_PIECE_COUNT_MORE_THAN_TOTAL_BYTES;
  const size_t ps = (len + count - 1) / count;
  if (ps >= ps * count) return RLNC_ERR_BAD_PIECE_COUNT;
  *size = ps;
  *pad = count * ps - len;
  return RLNC_OK;
}

inline int split_size(size_t len, size_t size, size_t* count, size_t* pad) {
  if (size == 0) return RLNC_ERR_ZERO_PIECE_SIZE;
  if (size >= len) return RLNC_ERR_BAD_PIECE_COUNT;
  const size_t pc = (len + size - 1) / size;
  *count = pc;
  *pad = pc * size - len;
  return RLNC_OK;
}

// The kernels address X through 32-bit buffer offsets (signed in gf_gemm,
// unsigned in gf_bs) and gf_bs keeps each wave's program of (row, coefficient)
// targets in LDS, so one launch takes at most kc rows of X.  A taller X (a
// generation past 2 GiB, sized for 288 GB of HBM) is split into row chunks:
// the first chunk's launch writes Y, each later one XORs its product into Y in
// its store (byte j of Y needs only byte j of every row, data.go:20-28).
template <class F>
inline int gemm_k_chunked(size_t K, size_t kc, F launch) {
  if (K <= kc) return launch(0, K, false);
  // equal chunks (whole 8-row program chunks where kc allows): 256 rows of
  // 16 MiB split 128 + 128, not 248 + 8
  const size_t nch = (K + kc - 1) / kc;
  kc = std::min(kc, ((K + nch - 1) / nch + 7) / 8 * 8);
  int s = RLNC_OK;
  for (size_t k0 = 0; s == RLNC_OK && k0 < K; k0 += kc) s = launch(k0, std::min(kc, K - k0), k0 > 0);
  return s;
}

// rows of X per gf_gemm launch
inline size_t gemm_chunk_rows(size_t ldx) { return ldx ? (kMaxDescBytes - 1) / ldx : 0; }

// rows of X per gf_bs launch for M output rows (0: the bit-sliced path cannot run)
inline size_t bs_chunk_rows(size_t M, size_t K, size_t ldx, size_t ncols) {
  if (!ldx || ldx > 0x7fffffff) return 0;
  size_t kc = std::min<size_t>(K, (((size_t)1 << 32) - 1) / ldx);
  // K in one launch when it fits (the kernel reads rows >= K as zero); split
  // launches take whole 8-row program chunks
  if (kc < K && kc > 8) kc = kc / 8 * 8;
  while (kc && !kodr_amd::plan_gemm_bs(M, kc, ncols).ok) kc = kc > 8 ? kc / 2 / 8 * 8 : 0;
  return kc;
}

inline int gemm(rlnc_ctx* ctx, const uint8_t* dA, size_t lda, size_t M, size_t K, const uint8_t* dX,
         size_t ldx, uint8_t* dY, size_t ldy, size_t ncols) {
  const size_t kc = gemm_chunk_rows(ldx);
  if (kc == 0 || (ldx % 16) || (ldy % 16) || ldx < ncols || ldy < ncols || ldx > 0x7fffffff) {
    g_last_error = "gf_gemm: unsupported layout (pitch a multiple of 16 and below 2^31)";
    return RLNC_ERR_INVALID_ARGUMENT;
  }
  return gemm_k_chunked(K, kc, [&](size_t k0, size_t kn, bool acc) {
    HIPC(kodr_amd::gf_gemm(dA + k0, lda, M, kn, dX + k0 * ldx, ldx, dY, ldy, ncols, ctx->stream, nullptr, acc));
    return (int)RLNC_OK;
  });
}

// Y = A (x) X over a bit-sliced X (kodr_amd::bitslice_rows), plain Y; side:
// the same launch also writes side->y = A (x) side->x (one K chunk only)
inline int gemm_bs(rlnc_ctx* ctx, const uint8_t* dA, size_t lda, size_t M, size_t K, const uint8_t* dX,
            size_t ldx, uint8_t* dY, size_t ldy, size_t ncols, const kodr_amd::BsSide* side = nullptr) {
  if ((ldx % 32) || (ldy % 16) || ldx < ncols || ldy < ncols) {
    g_last_error = "gf_gemm_bs: unsupported layout (pitch a multiple of 32)";
    return RLNC_ERR_INVALID_ARGUMENT;
  }
  if (M == 0 || ncols == 0) return RLNC_OK;
  const size_t kc = bs_chunk_rows(M, std::max<size_t>(K, 1), ldx, ncols);
  if (kc == 0) {
    g_last_error = "gf_gemm_bs: no launch plan for this shape";
    return RLNC_ERR_INVALID_ARGUMENT;
  }
  if (side && kc < K) {
    g_last_error = "gf_gemm_bs: a side product needs one K chunk";
    return RLNC_ERR_INVALID_ARGUMENT;
  }
  return gemm_k_chunked(K, kc, [&](size_t k0, size_t kn, bool acc) {
    HIPC(kodr_amd::gf_gemm_bs(dA + k0, lda, M, kn, dX + k0 * ldx, ldx, dY, ldy, ncols, ctx->device, ctx->stream,
                              acc, nullptr, side));
    return (int)RLNC_OK;
  });
}

// Below this many output rows the perm-table kernel (gf_gemm) wins: the
// bit-sliced kernel runs one 8-row group however few rows are real, and with
// 1-2 waves per SIMD its short load ring leaves it latency-bound (~13 us for
// B = 1 at 32 MiB/256 against 9 us; B = 8: 17-19 against 16 us; B = 10: 20
// against 28 us; profiles/r01/bs_min_rows.log).
constexpr size_t kBsMinRows = 9;
// The decoder builds its twin per materialization (one pass over the rows
// received since the last one).  From 16 rows the bit-sliced kernel always
// wins; from 9 rows it wins when that pass is short: 12 GF rows at 16 MiB/128
// take 28 us on gf_gemm, 10 us + 9 us of twin on the bit-sliced path, while at
// 32 MiB/256 a fresh twin costs 15 us and gf_gemm keeps the edge
// (profiles/r01/dec_get.log).
constexpr size_t kBsMinRowsDecode = 16;
constexpr size_t kBsTwinBudget = 16u << 20;  // bytes of new twin rows worth building for 9..15 rows

// Few rows of narrow pieces: gf_gemm's one-wave tiles beat the bit-sliced
// launch's fixed cost (K = 16, 128 KiB rows, 9-32 output rows: 4.8-7.2 us
// against 8.7-9.0; K = 32: up to 16 rows; profiles/r01/bs_vs_gemm_small_k.log).
// Capped at the measured range: M <= 32.
inline bool few_narrow_rows(size_t M, size_t K, size_t ncols) {
  return K <= 32 && ncols <= ((size_t)256 << 10) && M <= 32 && (K <= 16 || M <= 16);
}

// The bit-sliced twin of a resident, immutable X (K rows at pitch ldx), built
// once: on the first product that needs it, or at construction time through
// rlnc_encoder_prepare / rlnc_recoder_prepare.
inline int build_twin(rlnc_ctx* ctx, const uint8_t* plain, DevBuf& twin, bool& twin_valid, size_t K, size_t ldx,
               size_t ncols) {
  if (twin_valid) return RLNC_OK;
  TRY(twin.reserve(std::max<size_t>(K * ldx, 1)));
  HIPC(kodr_amd::bitslice_rows(plain, twin.p, ldx, K, ncols, ctx->stream));
  twin_valid = true;
  return RLNC_OK;
}

// true when a product of M rows over this resident X takes the bit-sliced kernel
inline bool resident_uses_bs(rlnc_ctx* ctx, size_t M, size_t K, size_t ldx, size_t ncols) {
  return !(M < kBsMinRows || few_narrow_rows(M, K, ncols) || (ldx % 32) ||
           !bs_chunk_rows(M, std::max<size_t>(K, 1), ldx, ncols) || !kodr_amd::bs_ready(ctx->device));
}

// Y = A (x) X for a resident, immutable X: small M through gf_gemm on the
// plain rows, larger M through gf_gemm_bs on a bit-sliced twin built once.
// A compact X (plain == nullptr: only the twin is resident) takes gf_gemm_bs
// for every M.
inline int gemm_resident(rlnc_ctx* ctx, const uint8_t* dA, size_t lda, size_t M, size_t K, const uint8_t* plain,
                  DevBuf& twin, bool& twin_valid, size_t ldx, uint8_t* dY, size_t ldy, size_t ncols) {
  if (!plain) return gemm_bs(ctx, dA, lda, M, K, twin.p, ldx, dY, ldy, ncols);
  if (!resident_uses_bs(ctx, M, K, ldx, ncols)) return gemm(ctx, dA, lda, M, K, plain, ldx, dY, ldy, ncols);
  TRY(build_twin(ctx, plain, twin, twin_valid, K, ldx, ncols));
  return gemm_bs(ctx, dA, lda, M, K, twin.p, ldx, dY, ldy, ncols);
}

// Keep only the bit-sliced twin of a resident X (K rows at pitch ldx): half
// the HBM per generation.  Needs the bit-sliced path on this device.
inline int compact_resident(rlnc_ctx* ctx, DevBuf& plain, DevBuf& twin, bool& twin_valid, bool& compact, size_t K,
                     size_t ldx, size_t ncols) {
  if (compact) return RLNC_OK;
  if ((ldx % 32) || !kodr_amd::bs_ready(ctx->device) || !bs_chunk_rows(1, std::max<size_t>(K, 1), ldx, ncols)) {
    g_last_error = "compact residency needs the bit-sliced kernel for this shape";
    return RLNC_ERR_INVALID_ARGUMENT;
  }
  TRY(build_twin(ctx, plain.p, twin, twin_valid, K, ldx, ncols));
  HIPC(hipStreamSynchronize(ctx->stream));
  plain.release();
  compact = true;
  return RLNC_OK;
}

// plain rows [r0, r0 + n) of a compact X into dst (pitch dpitch, device):
// the bit-sliced layout is its own inverse
inline int uncompact_rows(rlnc_ctx* ctx, const DevBuf& twin, size_t ldx, size_t r0, size_t n, size_t ncols, DevBuf& scratch,
                   uint8_t* dst, size_t dpitch) {
  TRY(scratch.reserve(n * ldx));
  HIPC(kodr_amd::bitslice_rows(twin.p + r0 * ldx, scratch.p, ldx, n, ncols, ctx->stream));
  HIPC(hipMemcpy2DAsync(dst, dpitch, scratch.p, ldx, ncols, n, hipMemcpyDeviceToDevice, ctx->stream));
  return RLNC_OK;
}

inline int encoder_alloc(rlnc_ctx* ctx, int kind, size_t k, size_t L, rlnc_encoder** out) {
  if (!ctx || !out || (kind != RLNC_FULL && kind != RLNC_SYSTEMATIC) || k == 0 || L == 0)
    return RLNC_ERR_INVALID_ARGUMENT;
  TRY(set_dev(ctx));
  rlnc_encoder* e = new (std::nothrow) rlnc_encoder;
  if (!e) return RLNC_ERR_OUT_OF_MEMORY;
  e->ctx = ctx;
  for (DevBuf* b : {&e->pieces, &e->pieces_bs, &e->vecs, &e->out}) b->bind(ctx->device, ctx->stream);
  e->kind = kind;
  (void)rlnc_random_bytes(reinterpret_cast<uint8_t*>(&e->seed), sizeof(e->seed));
  e->k = k;
  e->L = L;
  e->pitch = round_up(L, kPitchAlign);
  if (e->pitch >= kMaxDescBytes) {
    delete e;
    g_last_error = "piece size of 2 GiB or more";
    return RLNC_ERR_INVALID_ARGUMENT;
  }
  int s = e->pieces.reserve(k * e->pitch);
  if (s == RLNC_OK) {
    hipError_t he = hipMemsetAsync(e->pieces.p, 0, k * e->pitch, ctx->stream);
    if (he != hipSuccess) s = hip_fail(he, "hipMemsetAsync");
  }
  if (s != RLNC_OK) {
    e->pieces.release();
    delete e;
    return s;
  }
  *out = e;
  return RLNC_OK;
}

// upload `len` bytes of data as k rows of L bytes (last row zero padded)
inline int upload_generation(rlnc_encoder* e, const uint8_t* data, size_t len) {
  const size_t full_rows = len / e->L, tail = len - full_rows * e->L;
  HIPC(e->ctx->stage.h2d(e->pieces.p, e->pitch, data, e->L, e->L, full_rows, e->ctx->stream));
  if (tail)
    HIPC(e->ctx->stage.h2d(e->pieces.p + full_rows * e->pitch, e->pitch, data + full_rows * e->L, tail, tail, 1,
                           e->ctx->stream));
  return RLNC_OK;
}

}  // namespace kodr_capi

// runs f on every exit from a scope (error returns included)
template <class F>
struct ScopeExit {
  F f;
  ~ScopeExit() { f(); }
};
template <class F>
inline ScopeExit<F> on_scope_exit(F f) {
  return ScopeExit<F>{f};
}
