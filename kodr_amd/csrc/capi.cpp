// capi.cpp -- implementation of include/kodr_rlnc.h: version, errors,
// context, splitting, encoder, recoder and the raw kernel entry point (the
// decoder is in capi_decoder.cpp; shared definitions in capi_internal.hpp).
//
// Host-side mirror of kodr's codec API (full/, systematic/, kodr_internals/)
// over device-resident generations.  Every data-plane byte is produced by the
// HIP kernel in gf_kernels.hip; the host only validates arguments, mirrors
// kodr's counters / pivot decisions (decoder_core.cpp) and moves bytes.  There
// is no CPU compute fallback: without a usable HIP device every data call
// fails with RLNC_ERR_NO_DEVICE / RLNC_ERR_HIP.
#include "capi_internal.hpp"

namespace {
const char* kErrText[] = {
    "",
    "additive identity of Gf(2^8) i.e. 0, doesn't have a multiplicative inverse",
    "can't perform matrix multiplication",
    "no more pieces required for decoding",
    "not enough pieces received yet to decode",
    "failed to copy whole data before splitting into pieces",
    "requested piece count > total bytes of original data",
    "pieces can't be sized as zero byte",
    "minimum 2 pieces required for RLNC",
    "coded data length != coded piece count x coded piece length",
    "coding vector length > coded piece length ( in total )",
    "piece not decoded yet, more pieces required",
    "requested piece index >= pieceCount ( pieces coded together )",
};
}  // namespace

extern "C" {

const char* rlnc_version(void) { return "kodr_amd 0.1.0 (gfx950)"; }

const char* rlnc_status_string(int s) {
  if (s >= 0 && s <= 12) return s == 0 ? "ok" : kErrText[s];
  switch (s) {
    case RLNC_ERR_INVALID_ARGUMENT: return "invalid argument";
    case RLNC_ERR_OUT_OF_MEMORY: return "out of memory";
    case RLNC_ERR_HIP: return "HIP runtime error";
    case RLNC_ERR_NO_DEVICE: return "no usable HIP device";
    default: return "unknown status";
  }
}

const char* rlnc_last_hip_error(void) { return g_last_error.c_str(); }

int rlnc_device_count(int* count) {
  if (!count) return RLNC_ERR_INVALID_ARGUMENT;
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    *count = 0;
    return hip_fail(e, "hipGetDeviceCount");
  }
  *count = n;
  return RLNC_OK;
}

int rlnc_ctx_create(int device, void* stream, rlnc_ctx** out) {
  if (!out) return RLNC_ERR_INVALID_ARGUMENT;
  int n = 0;
  TRY(rlnc_device_count(&n));
  if (device < 0 || device >= n) {
    g_last_error = "device index out of range";
    return RLNC_ERR_NO_DEVICE;
  }
  HIPC(hipSetDevice(device));
  rlnc_ctx* c = new (std::nothrow) rlnc_ctx;
  if (!c) return RLNC_ERR_OUT_OF_MEMORY;
  c->device = device;
  if (stream) {
    c->stream = (hipStream_t)stream;
  } else {
    hipError_t e = hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
      delete c;
      return hip_fail(e, "hipStreamCreate");
    }
    c->own_stream = true;
  }
  *out = c;
  return RLNC_OK;
}

int rlnc_ctx_destroy(rlnc_ctx* ctx) {
  if (!ctx) return RLNC_OK;
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->stream);
  kodr_amd::DevicePool::get(ctx->device).drop_stream(ctx->stream);  // destroyed decoders' blocks, now idle
  ctx->stage.release();
  ctx->elim_tab.release();
  ctx->elim_out.release();
  ctx->elim_in.release();
  ctx->elim_pub.release();
  ctx->elim_tdev.release();
  ctx->gtab.release();
  if (ctx->elim_pin) (void)hipHostFree(ctx->elim_pin);
  ctx->elim_pin = nullptr;
  ctx->gtmat[0].release();
  ctx->gtmat[1].release();
  if (ctx->aux) {
    (void)hipStreamSynchronize(ctx->aux);
    (void)hipStreamDestroy(ctx->aux);
  }
  if (ctx->vec_pin) (void)hipHostFree(ctx->vec_pin);  // (after the aux stream's downloads into it)
  ctx->vec_pin = nullptr;
  if (ctx->vec_ready) (void)hipEventDestroy(ctx->vec_ready);
  if (ctx->side) {
    (void)hipStreamSynchronize(ctx->side);
    (void)hipStreamDestroy(ctx->side);
    (void)hipEventDestroy(ctx->side_done);
    (void)hipEventDestroy(ctx->rows_ready);
    if (ctx->elim_ready) (void)hipEventDestroy(ctx->elim_ready);
  }
  if (ctx->own_stream) (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return RLNC_OK;
}

int rlnc_ctx_synchronize(rlnc_ctx* ctx) {
  TRY(set_dev(ctx));
  HIPC(hipStreamSynchronize(ctx->stream));
  // the aux stream's downloads of a batched AddPiece's coding vectors read the
  // caller's rows and are never joined into ctx->stream: covered here, so a
  // caller may reuse its rows once this returns (kodr_rlnc.h)
  if (ctx->aux) HIPC(hipStreamSynchronize(ctx->aux));
  return RLNC_OK;
}

void* rlnc_ctx_stream(rlnc_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int rlnc_ctx_elim_stats(const rlnc_ctx* ctx, size_t* gpu, size_t* gpu_retried, size_t* host_after_gpu,
                        size_t* host) {
  if (!ctx) return RLNC_ERR_INVALID_ARGUMENT;
  if (gpu) *gpu = ctx->n_elim_gpu;
  if (gpu_retried) *gpu_retried = ctx->n_elim_gpu_retried;
  if (host_after_gpu) *host_after_gpu = ctx->n_elim_host_after_gpu;
  if (host) *host = ctx->n_elim_host;
  return RLNC_OK;
}

int rlnc_ctx_set_route_min_k(rlnc_ctx* ctx, size_t min_k) {
  if (!ctx) return RLNC_ERR_INVALID_ARGUMENT;
  ctx->route_min_k = min_k;
  return RLNC_OK;
}

int rlnc_random_bytes(uint8_t* out, size_t n) {
  size_t got = 0;
  while (got < n) {
    ssize_t r = getrandom(out + got, n - got, 0);
    if (r < 0) return RLNC_ERR_INVALID_ARGUMENT;
    got += (size_t)r;
  }
  return RLNC_OK;
}

int rlnc_device_pool_trim(int device, size_t keep_bytes) {
  int n = 0;
  TRY(rlnc_device_count(&n));
  if (device < 0 || device >= n) return RLNC_ERR_NO_DEVICE;
  HIPC(hipSetDevice(device));
  kodr_amd::DevicePool::get(device).trim(keep_bytes);
  return RLNC_OK;
}

size_t rlnc_device_pool_cached(int device) {
  return device < 0 ? 0 : kodr_amd::DevicePool::get(device).cached();
}

int rlnc_dev_alloc(rlnc_ctx* ctx, size_t bytes, void** dptr) {
  if (!dptr) return RLNC_ERR_INVALID_ARGUMENT;
  TRY(set_dev(ctx));
  HIPC(hipMalloc(dptr, bytes ? bytes : 1));
  return RLNC_OK;
}
int rlnc_dev_free(rlnc_ctx* ctx, void* dptr) {
  TRY(set_dev(ctx));
  HIPC(hipFree(dptr));
  return RLNC_OK;
}
int rlnc_memcpy_h2d(rlnc_ctx* ctx, void* dst, const void* src, size_t bytes) {
  TRY(set_dev(ctx));
  HIPC(ctx->stage.h2d((uint8_t*)dst, bytes, (const uint8_t*)src, bytes, bytes, 1, ctx->stream));
  HIPC(hipStreamSynchronize(ctx->stream));
  return RLNC_OK;
}
int rlnc_memcpy_d2h(rlnc_ctx* ctx, void* dst, const void* src, size_t bytes) {
  TRY(set_dev(ctx));
  HIPC(ctx->stage.d2h((uint8_t*)dst, bytes, (const uint8_t*)src, bytes, bytes, 1, ctx->stream));
  return RLNC_OK;
}
int rlnc_host_register(rlnc_ctx* ctx, void* ptr, size_t bytes) {
  if (!ptr || !bytes) return RLNC_ERR_INVALID_ARGUMENT;
  TRY(set_dev(ctx));
  HIPC(hipHostRegister(ptr, bytes, hipHostRegisterDefault));
  return RLNC_OK;
}
int rlnc_host_unregister(rlnc_ctx* ctx, void* ptr) {
  if (!ptr) return RLNC_ERR_INVALID_ARGUMENT;
  TRY(set_dev(ctx));
  HIPC(hipHostUnregister(ptr));
  return RLNC_OK;
}
int rlnc_memcpy_d2d_async(rlnc_ctx* ctx, void* dst, const void* src, size_t bytes) {
  TRY(set_dev(ctx));
  HIPC(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, ctx->stream));
  return RLNC_OK;
}
int rlnc_event_create(rlnc_ctx* ctx, void** ev) {
  if (!ev) return RLNC_ERR_INVALID_ARGUMENT;
  TRY(set_dev(ctx));
  HIPC(hipEventCreate((hipEvent_t*)ev));
  return RLNC_OK;
}
int rlnc_event_record(rlnc_ctx* ctx, void* ev) {
  TRY(set_dev(ctx));
  HIPC(hipEventRecord((hipEvent_t)ev, ctx->stream));
  return RLNC_OK;
}
int rlnc_ctx_wait_event(rlnc_ctx* ctx, void* ev) {
  if (!ev) return RLNC_ERR_INVALID_ARGUMENT;
  TRY(set_dev(ctx));
  HIPC(hipStreamWaitEvent(ctx->stream, (hipEvent_t)ev, 0));
  return RLNC_OK;
}
int rlnc_event_elapsed_ms(void* a, void* b, float* ms) {
  if (!ms) return RLNC_ERR_INVALID_ARGUMENT;
  HIPC(hipEventSynchronize((hipEvent_t)b));
  HIPC(hipEventElapsedTime(ms, (hipEvent_t)a, (hipEvent_t)b));
  return RLNC_OK;
}
int rlnc_event_destroy(void* ev) {
  HIPC(hipEventDestroy((hipEvent_t)ev));
  return RLNC_OK;
}

/* ---- splitting ---------------------------------------------------------- */
int rlnc_split_by_piece_count(size_t len, size_t count, size_t* size, size_t* pad) {
  if (!size || !pad) return RLNC_ERR_INVALID_ARGUMENT;
  return split_count(len, count, size, pad);
}
int rlnc_split_by_piece_size(size_t len, size_t size, size_t* count, size_t* pad) {
  if (!count || !pad) return RLNC_ERR_INVALID_ARGUMENT;
  return split_size(len, size, count, pad);
}
int rlnc_coded_pieces_for_recoding(size_t len, size_t count, size_t together, size_t* cpl) {
  if (!cpl) return RLNC_ERR_INVALID_ARGUMENT;
  if (count == 0) return RLNC_ERR_CODED_DATA_LENGTH_MISMATCH;
  const size_t l = len / count;                                   // data.go:174
  if (l * count != len) return RLNC_ERR_CODED_DATA_LENGTH_MISMATCH;  // :175-177
  if (!(together < l)) return RLNC_ERR_CODING_VECTOR_LENGTH_MISMATCH;  // :179-181
  *cpl = l;
  return RLNC_OK;
}
int rlnc_is_systematic(const uint8_t* v, size_t n) {              // data.go:64-84
  long pos = -1;
  for (size_t i = 0; i < n; i++) {
    if (v[i] == 0) continue;
    if (v[i] != 1 || pos != -1) return 0;
    pos = (long)i;
  }
  return pos >= 0;
}

/* ---- encoder ------------------------------------------------------------ */
int rlnc_encoder_create_with_piece_count(rlnc_ctx* ctx, int kind, const uint8_t* data, size_t len,
                                         size_t count, rlnc_encoder** out) {
  size_t size = 0, pad = 0;
  TRY(split_count(len, count, &size, &pad));
  if (!data) return RLNC_ERR_INVALID_ARGUMENT;
  rlnc_encoder* e = nullptr;
  TRY(encoder_alloc(ctx, kind, count, size, &e));
  e->padding = pad;
  int s = upload_generation(e, data, len);
  if (s != RLNC_OK) {
    rlnc_encoder_destroy(e);
    return s;
  }
  *out = e;
  return RLNC_OK;
}

int rlnc_encoder_create_with_piece_size(rlnc_ctx* ctx, int kind, const uint8_t* data, size_t len,
                                        size_t size, rlnc_encoder** out) {
  size_t count = 0, pad = 0;
  TRY(split_size(len, size, &count, &pad));
  if (!data) return RLNC_ERR_INVALID_ARGUMENT;
  rlnc_encoder* e = nullptr;
  TRY(encoder_alloc(ctx, kind, count, size, &e));
  e->padding = pad;
  int s = upload_generation(e, data, len);
  if (s != RLNC_OK) {
    rlnc_encoder_destroy(e);
    return s;
  }
  *out = e;
  return RLNC_OK;
}

int rlnc_encoder_create(rlnc_ctx* ctx, int kind, const uint8_t* pieces, size_t k, size_t L,
                        rlnc_encoder** out) {
  if (!pieces) return RLNC_ERR_INVALID_ARGUMENT;
  rlnc_encoder* e = nullptr;
  TRY(encoder_alloc(ctx, kind, k, L, &e));
  int s = upload_generation(e, pieces, k * L);
  if (s != RLNC_OK) {
    rlnc_encoder_destroy(e);
    return s;
  }
  *out = e;
  return RLNC_OK;
}

int rlnc_encoder_create_device(rlnc_ctx* ctx, int kind, const uint8_t* d_pieces, size_t k, size_t L,
                               size_t pitch, rlnc_encoder** out) {
  if (!d_pieces || pitch < L) return RLNC_ERR_INVALID_ARGUMENT;
  rlnc_encoder* e = nullptr;
  TRY(encoder_alloc(ctx, kind, k, L, &e));
  hipError_t he = hipMemcpy2DAsync(e->pieces.p, e->pitch, d_pieces, pitch, L, k,
                                   hipMemcpyDeviceToDevice, ctx->stream);
  if (he == hipSuccess) he = hipStreamSynchronize(ctx->stream);
  if (he != hipSuccess) {
    rlnc_encoder_destroy(e);
    return hip_fail(he, "hipMemcpy2DAsync");
  }
  *out = e;
  return RLNC_OK;
}

int rlnc_encoder_destroy(rlnc_encoder* e) {
  if (!e) return RLNC_OK;
  (void)hipSetDevice(e->ctx->device);
  (void)hipStreamSynchronize(e->ctx->stream);
  e->pieces.release();
  e->pieces_bs.release();
  e->vecs.release();
  e->out.release();
  delete e;
  return RLNC_OK;
}

size_t rlnc_encoder_piece_count(const rlnc_encoder* e) { return e ? e->k : 0; }
size_t rlnc_encoder_piece_size(const rlnc_encoder* e) { return e ? e->L : 0; }
size_t rlnc_encoder_decodable_len(const rlnc_encoder* e) { return e ? e->k * (e->k + e->L) : 0; }
size_t rlnc_encoder_coded_piece_len(const rlnc_encoder* e) { return e ? e->k + e->L : 0; }
size_t rlnc_encoder_padding(const rlnc_encoder* e) { return e ? e->padding : 0; }
const uint8_t* rlnc_encoder_device_pieces(const rlnc_encoder* e, size_t* pitch) {
  if (!e || e->compact) return nullptr;
  if (pitch) *pitch = e->pitch;
  return e->pieces.p;
}
size_t rlnc_encoder_systematic_remaining(const rlnc_encoder* e) {
  if (!e || e->kind != RLNC_SYSTEMATIC) return 0;
  return e->k - std::min(e->sys_next, e->k);
}

int rlnc_encoder_coded_pieces(rlnc_encoder* e, uint8_t* vectors, size_t count, uint8_t* out) {
  if (!e || (count && (!vectors || !out))) return RLNC_ERR_INVALID_ARGUMENT;
  TRY(set_dev(e->ctx));
  const size_t k = e->k, L = e->L, clen = k + L;
  hipStream_t st = e->ctx->stream;
  size_t i = 0;
  // systematic/encoder.go:83-96: the first k calls return e_id ++ copy(P_id)
  if (e->kind == RLNC_SYSTEMATIC && e->sys_next < k && count) {
    const size_t n = std::min(count, k - e->sys_next), id0 = e->sys_next;
    for (size_t r = 0; r < n; r++) {
      memset(vectors + r * k, 0, k);
      vectors[r * k + id0 + r] = 1;
      memcpy(out + r * clen, vectors + r * k, k);
    }
    // consecutive piece ids: one strided copy of rows id0 .. id0+n-1
    const uint8_t* src = e->pieces.p + id0 * e->pitch;
    if (e->compact) {
      TRY(e->out.reserve(n * e->pitch));
      TRY(e->vecs.reserve(n * e->pitch));
      TRY(uncompact_rows(e->ctx, e->pieces_bs, e->pitch, id0, n, L, e->vecs, e->out.p, e->pitch));
      src = e->out.p;
    }
    HIPC(e->ctx->stage.d2h(out + k, clen, src, e->pitch, L, n, st));
    e->sys_next += n;
    i = n;
  }
  // full/encoder.go:61-71 (and systematic/encoder.go:98-108) in batches
  const size_t kBatch = 256;
  while (i < count) {
    const size_t B = std::min(kBatch, count - i);
    TRY(e->vecs.reserve(B * k));
    TRY(e->out.reserve(B * e->pitch));
    HIPC(e->ctx->stage.h2d(e->vecs.p, k, vectors + i * k, k, k, B, st));
    TRY(gemm_resident(e->ctx, e->vecs.p, k, B, k, e->pieces.p, e->pieces_bs, e->bs_valid, e->pitch, e->out.p,
                      e->pitch, L));
    for (size_t b = 0; b < B; b++) memcpy(out + (i + b) * clen, vectors + (i + b) * k, k);
    HIPC(e->ctx->stage.d2h(out + i * clen + k, clen, e->out.p, e->pitch, L, B, st));
    i += B;
  }
  HIPC(hipStreamSynchronize(st));
  return RLNC_OK;
}

int rlnc_encoder_coded_pieces_device(rlnc_encoder* e, const uint8_t* d_vectors, size_t count,
                                     uint8_t* d_out, size_t out_pitch) {
  if (!e || (count && (!d_vectors || !d_out)) || out_pitch < e->L) return RLNC_ERR_INVALID_ARGUMENT;
  TRY(set_dev(e->ctx));
  return gemm_resident(e->ctx, d_vectors, e->k, count, e->k, e->pieces.p, e->pieces_bs, e->bs_valid, e->pitch,
                       d_out, out_pitch, e->L);
}

int rlnc_encoder_prepare(rlnc_encoder* e) {
  if (!e) return RLNC_ERR_INVALID_ARGUMENT;
  TRY(set_dev(e->ctx));
  // any batch of >= kBsMinRows pieces that takes the bit-sliced kernel reads the twin
  if (e->compact || !resident_uses_bs(e->ctx, std::max<size_t>(e->k, 64), e->k, e->pitch, e->L)) return RLNC_OK;
  return build_twin(e->ctx, e->pieces.p, e->pieces_bs, e->bs_valid, e->k, e->pitch, e->L);
}

int rlnc_encoder_compact(rlnc_encoder* e) {
  if (!e) return RLNC_ERR_INVALID_ARGUMENT;
  TRY(set_dev(e->ctx));
  return compact_resident(e->ctx, e->pieces, e->pieces_bs, e->bs_valid, e->compact, e->k, e->pitch, e->L);
}

// grouped launches over resident twins: the bit-sliced kernel from this many
// pieces per generation (see rlnc_encoder_group_coded_pieces_device)
constexpr size_t kGroupBsMinRows = 5;
static size_t group_bs_min() {
  static const size_t v = kodr_amd::tune_env("KODR_GROUP_BS_MIN") ? (size_t)atol(kodr_amd::tune_env("KODR_GROUP_BS_MIN")) : kGroupBsMinRows;
  return v;
}


namespace {

// count coded pieces of each of n_enc resident generations (one ctx, one
// k and L): generation i's coefficient rows at dA + i * a_stride (pitch lda),
// its pieces at dY + i * y_stride (pitch ldy).  One launch streams up to
// kGemmGroupMax generations where the product runs in one row chunk (small
// batches on gf_gemm over the plain rows, larger ones on gf_bs_kernel over
// the twins); otherwise one product per generation.
int group_encode(rlnc_encoder* const* encs, size_t n_enc, const uint8_t* dA, size_t lda, size_t a_stride,
                 size_t count, uint8_t* dY, size_t ldy, size_t y_stride) {
  rlnc_encoder* e0 = encs[0];
  rlnc_ctx* ctx = e0->ctx;
  const size_t k = e0->k, L = e0->L;
  const bool yal = (ldy % 16) == 0 && ((uintptr_t)dY % 16) == 0 && (y_stride % 16) == 0;
  bool grouped = !resident_uses_bs(ctx, count, k, e0->pitch, L) && k * e0->pitch < kMaxDescBytes &&
                 (e0->pitch % 16) == 0 && yal;
  for (size_t i = 0; i < n_enc && grouped; i++) grouped = !encs[i]->compact;  // the grouped launch reads plain rows
  // larger batches: one bit-sliced launch per kGemmGroupMax generations over
  // their twins, when the product is a single row chunk.  Smaller batches
  // from kGroupBsMinRows take it too when every twin is already resident
  // (prepared or compact encoders): one 8-row group per column chunk costs
  // 6.6-6.9 us per 32 MiB/256 generation at 6-8 pieces against 10-11 us on
  // gf_gemm, equal at 3-4, gf_gemm ahead at 2 (profiles/r02/group_bs_small/).
  // KODR_GROUP_BS_MIN overrides it (measurements).
  bool twins = count >= group_bs_min() && count < kBsMinRows && !few_narrow_rows(count, k, L) &&
               (e0->pitch % 32) == 0 && kodr_amd::bs_ready(ctx->device);
  for (size_t i = 0; i < n_enc && twins; i++) twins = encs[i]->compact || encs[i]->bs_valid;
  if (twins) grouped = false;
  const bool grouped_bs = !grouped && (twins || resident_uses_bs(ctx, count, k, e0->pitch, L)) &&
                          bs_chunk_rows(count, k, e0->pitch, L) >= k && yal;
  if (grouped_bs) {
    for (size_t i = 0; i < n_enc; i++)
      if (!encs[i]->compact)
        TRY(build_twin(ctx, encs[i]->pieces.p, encs[i]->pieces_bs, encs[i]->bs_valid, k, e0->pitch, L));
    // (a batch of 8m + 1 or 8m + 2 pieces -- the round trip's k + 2 -- pays a
    // whole last 8-row group for its one or two tail rows: 16 x 258 pieces
    // 103-108 us per generation against 93-98 for 256.  Handing the tail to a
    // launch of its own -- the grouped v_perm kernel over the plain rows, or a
    // second bit-sliced launch that splits K over a workgroup's waves -- and
    // every plan's KW were measured no faster: the tail's launch must stream
    // the whole generation from HBM again (profiles/r06/split_tail/, r06/kw/).)
    const uint8_t* xs[kodr_amd::kGemmGroupMax];
    for (size_t g0 = 0; g0 < n_enc; g0 += kodr_amd::kGemmGroupMax) {
      const size_t n = std::min<size_t>(kodr_amd::kGemmGroupMax, n_enc - g0);
      for (size_t i = 0; i < n; i++) xs[i] = encs[g0 + i]->pieces_bs.p;
      const kodr_amd::GemmGroupArgs grp{(int)n, xs, a_stride, y_stride};
      HIPC(kodr_amd::gf_gemm_bs(dA + g0 * a_stride, lda, count, k, xs[0], e0->pitch, dY + g0 * y_stride, ldy, L,
                                ctx->device, ctx->stream, false, &grp));
    }
    return RLNC_OK;
  }
  if (!grouped) {
    for (size_t i = 0; i < n_enc; i++) {
      rlnc_encoder* e = encs[i];
      TRY(gemm_resident(ctx, dA + i * a_stride, lda, count, k, e->compact ? nullptr : e->pieces.p, e->pieces_bs,
                        e->bs_valid, e->pitch, dY + i * y_stride, ldy, L));
    }
    return RLNC_OK;
  }
  const uint8_t* xs[kodr_amd::kGemmGroupMax];
  for (size_t g0 = 0; g0 < n_enc; g0 += kodr_amd::kGemmGroupMax) {
    const size_t n = std::min<size_t>(kodr_amd::kGemmGroupMax, n_enc - g0);
    for (size_t i = 0; i < n; i++) xs[i] = encs[g0 + i]->pieces.p;
    const kodr_amd::GemmGroupArgs grp{(int)n, xs, a_stride, y_stride};
    HIPC(kodr_amd::gf_gemm(dA + g0 * a_stride, lda, count, k, xs[0], e0->pitch, dY + g0 * y_stride, ldy, L,
                           ctx->stream, nullptr, false, &grp));
  }
  return RLNC_OK;
}

// encoders of one ctx with equal k and L
int check_group(rlnc_encoder* const* encs, size_t n_enc) {
  rlnc_encoder* e0 = encs[0];
  for (size_t i = 1; i < n_enc; i++)
    if (!encs[i] || encs[i]->ctx != e0->ctx || encs[i]->k != e0->k || encs[i]->L != e0->L)
      return RLNC_ERR_INVALID_ARGUMENT;
  return RLNC_OK;
}

}  // namespace

int rlnc_encoder_group_coded_pieces_device(rlnc_encoder* const* encs, size_t n_enc, const uint8_t* d_vectors,
                                           size_t count, uint8_t* d_out, size_t out_pitch) {
  if (!encs || (n_enc && (!encs[0] || (count && (!d_vectors || !d_out))))) return RLNC_ERR_INVALID_ARGUMENT;
  if (!n_enc || !count) return RLNC_OK;
  rlnc_encoder* e0 = encs[0];
  if (out_pitch < e0->L) return RLNC_ERR_INVALID_ARGUMENT;
  TRY(check_group(encs, n_enc));
  TRY(set_dev(e0->ctx));
  return group_encode(encs, n_enc, d_vectors, e0->k, count * e0->k, count, d_out, out_pitch, count * out_pitch);
}

int rlnc_encoder_seed(rlnc_encoder* e, uint64_t seed) {
  if (!e) return RLNC_ERR_INVALID_ARGUMENT;
  e->seed = seed;
  e->drawn = 0;
  return RLNC_OK;
}

int rlnc_encoder_coded_wire_device(rlnc_encoder* e, size_t count, uint8_t* d_wire, size_t wire_pitch) {
  if (!e || (count && !d_wire)) return RLNC_ERR_INVALID_ARGUMENT;
  const size_t k = e->k, L = e->L;
  if (wire_pitch < k + L || count > 65535) return RLNC_ERR_INVALID_ARGUMENT;
  if (!count) return RLNC_OK;
  TRY(set_dev(e->ctx));
  hipStream_t st = e->ctx->stream;
  // systematic/encoder.go:83-96: the first k pieces are e_id ++ P_id
  size_t n_sys = 0;
  if (e->kind == RLNC_SYSTEMATIC && e->sys_next < k) n_sys = std::min(count, k - e->sys_next);
  HIPC(kodr_amd::fill_vectors(d_wire, wire_pitch, count, k, e->seed, e->drawn, n_sys, e->sys_next, st));
  // the systematic pieces are the pieces themselves (e_id x P = P_id): one
  // strided copy of rows sys_next.., no GF product
  if (n_sys && e->compact)
    TRY(uncompact_rows(e->ctx, e->pieces_bs, e->pitch, e->sys_next, n_sys, L, e->out, d_wire + k, wire_pitch));
  else if (n_sys)
    HIPC(hipMemcpy2DAsync(d_wire + k, wire_pitch, e->pieces.p + e->sys_next * e->pitch, e->pitch, L, n_sys,
                          hipMemcpyDeviceToDevice, st));
  // the coded rows' vectors are read in place as the coefficient matrix
  // (lda = wire_pitch)
  const size_t nc = count - n_sys;
  uint8_t* w0 = d_wire + n_sys * wire_pitch;
  const bool aligned = (k % 16) == 0 && (wire_pitch % 16) == 0 && ((uintptr_t)d_wire % 16) == 0;
  if (nc && aligned) {
    TRY(gemm_resident(e->ctx, w0, wire_pitch, nc, k, e->pieces.p, e->pieces_bs, e->bs_valid, e->pitch, w0 + k,
                      wire_pitch, L));
  } else if (nc) {  // piece columns not 16-byte aligned: compute aside, then one strided copy
    TRY(e->out.reserve(nc * e->pitch));
    TRY(gemm_resident(e->ctx, w0, wire_pitch, nc, k, e->pieces.p, e->pieces_bs, e->bs_valid, e->pitch, e->out.p,
                      e->pitch, L));
    HIPC(hipMemcpy2DAsync(w0 + k, wire_pitch, e->out.p, e->pitch, L, nc, hipMemcpyDeviceToDevice, st));
  }
  e->sys_next += n_sys;
  e->drawn += count;
  return RLNC_OK;
}

int rlnc_encoder_group_coded_wire_device(rlnc_encoder* const* encs, size_t n_enc, size_t count, uint8_t* d_wire,
                                         size_t wire_pitch) {
  if (!encs || (n_enc && (!encs[0] || (count && !d_wire)))) return RLNC_ERR_INVALID_ARGUMENT;
  if (!n_enc || !count) return RLNC_OK;
  rlnc_encoder* e0 = encs[0];
  const size_t k = e0->k, L = e0->L, wp = wire_pitch, gstride = count * wire_pitch;
  if (wp < k + L || count > 65535) return RLNC_ERR_INVALID_ARGUMENT;
  TRY(check_group(encs, n_enc));
  TRY(set_dev(e0->ctx));
  rlnc_ctx* ctx = e0->ctx;
  hipStream_t st = ctx->stream;
  // every encoder at the same point of its systematic phase (all full
  // encoders, or systematic ones created together) and 16-byte aligned piece
  // columns: one vector launch and grouped products; otherwise encoder by
  // encoder (same bytes, same stream state)
  auto n_sys_of = [&](const rlnc_encoder* e) -> size_t {
    return (e->kind == RLNC_SYSTEMATIC && e->sys_next < k) ? std::min(count, k - e->sys_next) : 0;
  };
  const size_t n_sys = n_sys_of(e0);
  bool grouped = (k % 16) == 0 && (wp % 16) == 0 && ((uintptr_t)d_wire % 16) == 0;
  for (size_t i = 1; i < n_enc && grouped; i++) grouped = n_sys_of(encs[i]) == n_sys;
  if (!grouped) {
    for (size_t i = 0; i < n_enc; i++) TRY(rlnc_encoder_coded_wire_device(encs[i], count, d_wire + i * gstride, wp));
    return RLNC_OK;
  }
  // the vectors of every row of every encoder from its own stream
  // (data.go:90-95 per coded piece; e_id for systematic rows,
  // systematic/encoder.go:60-68)
  for (size_t g0 = 0; g0 < n_enc; g0 += kodr_amd::kGemmGroupMax) {
    const size_t n = std::min<size_t>(kodr_amd::kGemmGroupMax, n_enc - g0);
    kodr_amd::VectorGroup vg = {};
    for (size_t i = 0; i < n; i++) {
      const rlnc_encoder* e = encs[g0 + i];
      vg.v[i] = d_wire + (g0 + i) * gstride;
      vg.seed[i] = e->seed;
      vg.row0[i] = e->drawn;
      vg.n_sys[i] = (int)n_sys;
      vg.sys_first[i] = (int)e->sys_next;
    }
    HIPC(kodr_amd::fill_vectors_grouped(vg, (int)n, wp, count, k, st));
  }
  // systematic rows: e_id x P = P_id, strided copies (systematic/encoder.go:83-96)
  for (size_t i = 0; i < n_enc && n_sys; i++) {
    rlnc_encoder* e = encs[i];
    uint8_t* dst = d_wire + i * gstride + k;
    if (e->compact)
      TRY(uncompact_rows(ctx, e->pieces_bs, e->pitch, e->sys_next, n_sys, L, e->out, dst, wp));
    else
      HIPC(hipMemcpy2DAsync(dst, wp, e->pieces.p + e->sys_next * e->pitch, e->pitch, L, n_sys,
                            hipMemcpyDeviceToDevice, st));
  }
  // coded rows: their vectors are read in place as the coefficient rows
  // (full/encoder.go:61-71, wire layout data.go:52-57)
  const size_t nc = count - n_sys;
  if (nc) {
    uint8_t* w0 = d_wire + n_sys * wp;
    TRY(group_encode(encs, n_enc, w0, wp, gstride, nc, w0 + k, wp, gstride));
  }
  for (size_t i = 0; i < n_enc; i++) {
    encs[i]->sys_next += n_sys;
    encs[i]->drawn += count;
  }
  return RLNC_OK;
}

/* ---- recoder ------------------------------------------------------------ */
namespace {

// Split layout.  A product of >= kBsMinRows recoded pieces reads a
// bit-sliced twin of the held pieces' columns only (pitch round_up(L, 256):
// at 32 MiB/256 exactly the encoder's 64 column chunks of 2 KiB), and the
// recoded coding vectors r x C (matrix.go:45-69) come from a narrow gf_gemm
// over the k vector columns.  A twin of the whole wire rows (k + L columns)
// has a 65th, 256-byte column chunk, which took the bit-sliced launch from
// one round of workgroups to two (B = 32: 30 us against 19.5 for the same
// MACs in an encode).  Wire-row twins remain for k not a multiple of 16.
bool rec_split(const rlnc_recoder* r) {
  return r->k % 16 == 0 && r->pitch % 16 == 0 && (r->ppitch % 32) == 0 && kodr_amd::bs_ready(r->ctx->device) &&
         bs_chunk_rows(64, r->n, r->ppitch, r->L) >= r->n;
}

// the n coding vectors (k columns): the plain wire rows, or a compact recoder's copy
const uint8_t* rec_vectors(const rlnc_recoder* r, size_t* ld) {
  *ld = r->compact ? r->vpitch : r->pitch;
  return r->compact ? r->vecs.p : r->flat.p;
}

int rec_build_piece_twin(rlnc_recoder* r) {
  if (r->piece_bs_valid) return RLNC_OK;
  TRY(r->piece_bs.reserve(std::max<size_t>(r->n * r->ppitch, 1)));
  HIPC(kodr_amd::bitslice_rows_pitched(r->flat.p + r->k, r->pitch, r->piece_bs.p, r->ppitch, r->n, r->L,
                                       r->ctx->stream));
  r->piece_bs_valid = true;
  return RLNC_OK;
}

bool rec_side_enabled() {
  static const bool v = kodr_amd::tune_env("KODR_REC_SIDE") ? atoi(kodr_amd::tune_env("KODR_REC_SIDE")) != 0 : true;
  return v;
}

// this product takes the split layout
bool rec_uses_split(const rlnc_recoder* r, size_t count) {
  return rec_split(r) && (r->compact || resident_uses_bs(r->ctx, count, r->n, r->ppitch, r->L));
}

// count recoded wire rows [r x C | sum r_i P_i] (full/recoder.go:32-40) into
// device rows dY (pitch ldy); dR: count x n recoding vectors
int rec_product(rlnc_recoder* r, const uint8_t* dR, size_t count, uint8_t* dY, size_t ldy) {
  rlnc_ctx* ctx = r->ctx;
  const size_t n = r->n, k = r->k, L = r->L;
  if (ldy % 16 || (uintptr_t)dY % 16) {  // any pitch: 16-byte aligned rows aside, then one strided copy
    const size_t sp = round_up(r->clen, 16);
    TRY(r->scratch.reserve(count * sp));
    TRY(rec_product(r, dR, count, r->scratch.p, sp));
    HIPC(hipMemcpy2DAsync(dY, ldy, r->scratch.p, sp, r->clen, count, hipMemcpyDeviceToDevice, ctx->stream));
    return RLNC_OK;
  }
  if (!rec_uses_split(r, count))  // one product over the wire rows
    return gemm_resident(ctx, dR, n, count, n, r->compact ? nullptr : r->flat.p, r->flat_bs, r->bs_valid, r->pitch,
                         dY, ldy, r->clen);
  size_t ldv = 0;
  const uint8_t* C = rec_vectors(r, &ldv);
  if (!r->compact) TRY(rec_build_piece_twin(r));
  uint8_t* yp = dY + k;
  // the vector columns as the bit-sliced launch's side product (one launch;
  // KODR_REC_SIDE=0: a gf_gemm launch of their own, for A/B)
  const kodr_amd::BsSide sd{C, ldv, dY, ldy, k};
  if (rec_side_enabled() && kodr_amd::side_ok(sd, n) && bs_chunk_rows(count, n, r->ppitch, L) >= n)
    return gemm_bs(ctx, dR, n, count, n, r->piece_bs.p, r->ppitch, yp, ldy, L, &sd);
  TRY(gemm(ctx, dR, n, count, n, C, ldv, dY, ldy, k));
  return gemm_bs(ctx, dR, n, count, n, r->piece_bs.p, r->ppitch, yp, ldy, L);  // k % 16 == 0: yp aligned
}

int recoder_alloc(rlnc_ctx* ctx, size_t n, size_t clen, size_t k, rlnc_recoder** out) {
  if (!ctx || !out || n == 0) return RLNC_ERR_INVALID_ARGUMENT;
  TRY(set_dev(ctx));
  rlnc_recoder* r = new (std::nothrow) rlnc_recoder;
  if (!r) return RLNC_ERR_OUT_OF_MEMORY;
  r->ctx = ctx;
  for (DevBuf* b : {&r->flat, &r->flat_bs, &r->piece_bs, &r->vecs, &r->r, &r->out, &r->scratch})
    b->bind(ctx->device, ctx->stream);
  r->n = n;
  r->k = k;
  r->clen = clen;
  r->L = clen - k;
  r->pitch = round_up(clen, kPitchAlign);
  r->ppitch = round_up(std::max<size_t>(r->L, 1), kPitchAlign);
  if (r->pitch >= kMaxDescBytes) {
    delete r;
    return RLNC_ERR_INVALID_ARGUMENT;
  }
  // (32 bytes of slack: the piece twin reads each row's piece columns up to
  // the next 32-byte block)
  int s = r->flat.reserve(n * r->pitch + 32);
  if (s == RLNC_OK) {
    hipError_t he = hipMemsetAsync(r->flat.p, 0, n * r->pitch + 32, ctx->stream);
    if (he != hipSuccess) s = hip_fail(he, "hipMemsetAsync");
  }
  if (s != RLNC_OK) {
    r->flat.release();
    delete r;
    return s;
  }
  *out = r;
  return RLNC_OK;
}

}  // namespace

int rlnc_recoder_create(rlnc_ctx* ctx, const uint8_t* flat, size_t len, size_t n, size_t together,
                        rlnc_recoder** out) {
  size_t clen = 0;
  TRY(rlnc_coded_pieces_for_recoding(len, n, together, &clen));  // full/recoder.go:64-67
  if (!flat) return RLNC_ERR_INVALID_ARGUMENT;
  rlnc_recoder* r = nullptr;
  TRY(recoder_alloc(ctx, n, clen, together, &r));
  hipError_t he = ctx->stage.h2d(r->flat.p, r->pitch, flat, clen, clen, n, ctx->stream);
  if (he != hipSuccess) {
    rlnc_recoder_destroy(r);
    return hip_fail(he, "hipMemcpy2DAsync");
  }
  *out = r;
  return RLNC_OK;
}

int rlnc_recoder_create_device(rlnc_ctx* ctx, const uint8_t* d_flat, size_t n, size_t clen,
                               size_t pitch, size_t together, rlnc_recoder** out) {
  if (!d_flat || pitch < clen) return RLNC_ERR_INVALID_ARGUMENT;
  if (!(together < clen)) return RLNC_ERR_CODING_VECTOR_LENGTH_MISMATCH;
  rlnc_recoder* r = nullptr;
  TRY(recoder_alloc(ctx, n, clen, together, &r));
  hipError_t he = hipMemcpy2DAsync(r->flat.p, r->pitch, d_flat, pitch, clen, n,
                                   hipMemcpyDeviceToDevice, ctx->stream);
  if (he == hipSuccess) he = hipStreamSynchronize(ctx->stream);
  if (he != hipSuccess) {
    rlnc_recoder_destroy(r);
    return hip_fail(he, "hipMemcpy2DAsync");
  }
  *out = r;
  return RLNC_OK;
}

int rlnc_recoder_prepare(rlnc_recoder* r) {
  if (!r) return RLNC_ERR_INVALID_ARGUMENT;
  TRY(set_dev(r->ctx));
  if (r->compact) return RLNC_OK;
  if (rec_split(r))
    return resident_uses_bs(r->ctx, std::max<size_t>(r->n, 64), r->n, r->ppitch, r->L) ? rec_build_piece_twin(r)
                                                                                       : RLNC_OK;
  if (!resident_uses_bs(r->ctx, std::max<size_t>(r->n, 64), r->n, r->pitch, r->clen)) return RLNC_OK;
  return build_twin(r->ctx, r->flat.p, r->flat_bs, r->bs_valid, r->n, r->pitch, r->clen);
}

int rlnc_recoder_compact(rlnc_recoder* r) {
  if (!r) return RLNC_ERR_INVALID_ARGUMENT;
  TRY(set_dev(r->ctx));
  if (r->compact) return RLNC_OK;
  if (!rec_split(r))
    return compact_resident(r->ctx, r->flat, r->flat_bs, r->bs_valid, r->compact, r->n, r->pitch, r->clen);
  // split: the piece twin plus a copy of the n coding vectors
  TRY(rec_build_piece_twin(r));
  r->vpitch = round_up(r->k, 16);
  TRY(r->vecs.reserve(r->n * r->vpitch));
  HIPC(hipMemcpy2DAsync(r->vecs.p, r->vpitch, r->flat.p, r->pitch, r->k, r->n, hipMemcpyDeviceToDevice,
                        r->ctx->stream));
  HIPC(hipStreamSynchronize(r->ctx->stream));
  r->flat.release();
  r->flat_bs.release();
  r->bs_valid = false;
  r->compact = true;
  return RLNC_OK;
}

int rlnc_recoder_destroy(rlnc_recoder* r) {
  if (!r) return RLNC_OK;
  (void)hipSetDevice(r->ctx->device);
  (void)hipStreamSynchronize(r->ctx->stream);
  for (DevBuf* b : {&r->flat, &r->flat_bs, &r->piece_bs, &r->vecs, &r->r, &r->out, &r->scratch}) b->release();
  delete r;
  return RLNC_OK;
}

size_t rlnc_recoder_piece_count(const rlnc_recoder* r) { return r ? r->n : 0; }
size_t rlnc_recoder_coded_piece_len(const rlnc_recoder* r) { return r ? r->clen : 0; }

int rlnc_recoder_coded_pieces(rlnc_recoder* r, const uint8_t* rv, size_t count, uint8_t* out) {
  if (!r || (count && (!rv || !out))) return RLNC_ERR_INVALID_ARGUMENT;
  TRY(set_dev(r->ctx));
  hipStream_t st = r->ctx->stream;
  const size_t kBatch = 256;
  for (size_t i = 0; i < count;) {
    const size_t B = std::min(kBatch, count - i);
    TRY(r->r.reserve(B * r->n));
    TRY(r->out.reserve(B * r->pitch));
    HIPC(r->ctx->stage.h2d(r->r.p, r->n, rv + i * r->n, r->n, r->n, B, st));
    TRY(rec_product(r, r->r.p, B, r->out.p, r->pitch));
    HIPC(r->ctx->stage.d2h(out + i * r->clen, r->clen, r->out.p, r->pitch, r->clen, B, st));
    i += B;
  }
  return RLNC_OK;
}

int rlnc_recoder_coded_pieces_device(rlnc_recoder* r, const uint8_t* d_r, size_t count,
                                     uint8_t* d_out, size_t out_pitch) {
  if (!r || (count && (!d_r || !d_out)) || out_pitch < r->clen) return RLNC_ERR_INVALID_ARGUMENT;
  if (!count) return RLNC_OK;
  TRY(set_dev(r->ctx));
  return rec_product(r, d_r, count, d_out, out_pitch);
}

// Recoders of one context and shape (n, clen) at once: count recoded pieces
// of each (full/recoder.go:27-46 per generation).  Split layout (every
// recoder): one narrow gf_gemm launch for the vector columns and one
// bit-sliced launch over the piece twins per kGemmGroupMax recoders; else
// one launch over the wire rows (gf_gemm below kBsMinRows, gf_bs_kernel on
// the wire-row twins from there); else one call per recoder.  Same bytes.
int rlnc_recoder_group_coded_pieces_device(rlnc_recoder* const* recs, size_t n_rec, const uint8_t* d_r,
                                           size_t count, uint8_t* d_out, size_t out_pitch) {
  if (!recs || (n_rec && (!recs[0] || (count && (!d_r || !d_out))))) return RLNC_ERR_INVALID_ARGUMENT;
  if (!n_rec || !count) return RLNC_OK;
  rlnc_recoder* r0 = recs[0];
  const size_t n = r0->n, clen = r0->clen, pitch = r0->pitch, k = r0->k, L = r0->L;
  if (out_pitch < clen) return RLNC_ERR_INVALID_ARGUMENT;
  for (size_t i = 1; i < n_rec; i++)
    if (!recs[i] || recs[i]->ctx != r0->ctx || recs[i]->n != n || recs[i]->clen != clen) return RLNC_ERR_INVALID_ARGUMENT;
  TRY(set_dev(r0->ctx));
  rlnc_ctx* ctx = r0->ctx;
  const size_t rstride = count * n, ostride = count * out_pitch;
  const bool oal = (out_pitch % 16) == 0 && ((uintptr_t)d_out % 16) == 0 && n_rec > 1;
  // as for encoders: from kGroupBsMinRows pieces on resident twins (prepared
  // or compact recoders), else from kBsMinRows
  const bool small = count >= group_bs_min() && count < kBsMinRows && !few_narrow_rows(count, n, clen) &&
                     kodr_amd::bs_ready(ctx->device);
  // split layout for every recoder: vectors by one grouped gf_gemm, pieces by
  // one grouped bit-sliced launch (their columns start at k, a multiple of 16)
  bool split = oal && rec_split(r0);
  bool twins_split = small;
  for (size_t i = 0; i < n_rec && (split || twins_split); i++) {
    twins_split = twins_split && (recs[i]->compact || recs[i]->piece_bs_valid);
    split = split && (recs[i]->compact == r0->compact);
  }
  split = split && (twins_split || rec_uses_split(r0, count));
  if (split) {
    for (size_t i = 0; i < n_rec; i++)
      if (!recs[i]->compact) TRY(rec_build_piece_twin(recs[i]));
    const uint8_t* xs[kodr_amd::kGemmGroupMax];
    size_t ldv = 0;
    (void)rec_vectors(r0, &ldv);
    for (size_t g0 = 0; g0 < n_rec; g0 += kodr_amd::kGemmGroupMax) {
      const size_t m = std::min<size_t>(kodr_amd::kGemmGroupMax, n_rec - g0);
      size_t ld = 0;
      for (size_t i = 0; i < m; i++) xs[i] = rec_vectors(recs[g0 + i], &ld);
      const kodr_amd::GemmGroupArgs gv{(int)m, xs, rstride, ostride};
      HIPC(kodr_amd::gf_gemm(d_r + g0 * rstride, n, count, n, xs[0], ldv, d_out + g0 * ostride, out_pitch, k,
                             ctx->stream, nullptr, false, &gv));
      for (size_t i = 0; i < m; i++) xs[i] = recs[g0 + i]->piece_bs.p;
      const kodr_amd::GemmGroupArgs gp{(int)m, xs, rstride, ostride};
      HIPC(kodr_amd::gf_gemm_bs(d_r + g0 * rstride, n, count, n, xs[0], r0->ppitch, d_out + g0 * ostride + k,
                                out_pitch, L, ctx->device, ctx->stream, false, &gp));
    }
    return RLNC_OK;
  }
  // wire-row products
  bool twins = small && (pitch % 32) == 0;
  for (size_t i = 0; i < n_rec && twins; i++) twins = !rec_split(recs[i]) && (recs[i]->compact || recs[i]->bs_valid);
  const bool bs = twins || resident_uses_bs(ctx, count, n, pitch, clen);
  bool grouped = oal;
  for (size_t i = 0; i < n_rec && grouped; i++) grouped = !rec_uses_split(recs[i], count);
  if (bs) {
    grouped = grouped && bs_chunk_rows(count, n, pitch, clen) >= n;
  } else {
    grouped = grouped && n * pitch < kMaxDescBytes && (pitch % 16) == 0;
    for (size_t i = 0; i < n_rec && grouped; i++) grouped = !recs[i]->compact;  // gf_gemm reads plain rows
  }
  if (!grouped) {
    for (size_t i = 0; i < n_rec; i++)
      TRY(rlnc_recoder_coded_pieces_device(recs[i], d_r + i * rstride, count, d_out + i * ostride, out_pitch));
    return RLNC_OK;
  }
  if (bs)
    for (size_t i = 0; i < n_rec; i++)
      if (!recs[i]->compact) TRY(build_twin(ctx, recs[i]->flat.p, recs[i]->flat_bs, recs[i]->bs_valid, n, pitch, clen));
  const uint8_t* xs[kodr_amd::kGemmGroupMax];
  for (size_t g0 = 0; g0 < n_rec; g0 += kodr_amd::kGemmGroupMax) {
    const size_t m = std::min<size_t>(kodr_amd::kGemmGroupMax, n_rec - g0);
    for (size_t i = 0; i < m; i++) xs[i] = bs ? recs[g0 + i]->flat_bs.p : recs[g0 + i]->flat.p;
    const kodr_amd::GemmGroupArgs grp{(int)m, xs, rstride, ostride};
    if (bs)
      HIPC(kodr_amd::gf_gemm_bs(d_r + g0 * rstride, n, count, n, xs[0], pitch, d_out + g0 * ostride, out_pitch, clen,
                                ctx->device, ctx->stream, false, &grp));
    else
      HIPC(kodr_amd::gf_gemm(d_r + g0 * rstride, n, count, n, xs[0], pitch, d_out + g0 * ostride, out_pitch, clen,
                             ctx->stream, nullptr, false, &grp));
  }
  return RLNC_OK;
}

/* ---- raw kernel ----------------------------------------------------------- */
int rlnc_bitslice_device(rlnc_ctx* ctx, uint8_t* dX, size_t ldx, size_t rows, size_t ncols) {
  if (!ctx || (rows && ncols && !dX)) return RLNC_ERR_INVALID_ARGUMENT;
  TRY(set_dev(ctx));
  HIPC(kodr_amd::bitslice_rows(dX, dX, ldx, rows, ncols, ctx->stream));
  return RLNC_OK;
}

int rlnc_bs_body_offsets(rlnc_ctx* ctx, uint32_t* out) {
  if (!ctx || !out) return RLNC_ERR_INVALID_ARGUMENT;
  TRY(set_dev(ctx));
  HIPC(kodr_amd::bs_body_offsets(ctx->device, out));
  return RLNC_OK;
}

int rlnc_gf_matmul_bs_device(rlnc_ctx* ctx, const uint8_t* dA, size_t lda, size_t M, size_t K,
                             const uint8_t* dXbs, size_t ldx, uint8_t* dY, size_t ldy, size_t ncols) {
  if (!ctx || (M && (!dA || !dXbs || !dY)) || lda < K) return RLNC_ERR_INVALID_ARGUMENT;
  TRY(set_dev(ctx));
  return gemm_bs(ctx, dA, lda, M, K, dXbs, ldx, dY, ldy, ncols);
}

int rlnc_gf_matmul_device(rlnc_ctx* ctx, const uint8_t* dA, size_t lda, size_t M, size_t K,
                          const uint8_t* dX, size_t ldx, uint8_t* dY, size_t ldy, size_t ncols) {
  if (!ctx || (M && (!dA || !dX || !dY)) || lda < K) return RLNC_ERR_INVALID_ARGUMENT;
  TRY(set_dev(ctx));
  return gemm(ctx, dA, lda, M, K, dX, ldx, dY, ldy, ncols);
}

}  // extern "C"
