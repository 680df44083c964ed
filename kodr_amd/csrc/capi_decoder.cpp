// capi_decoder.cpp -- the decoder half of include/kodr_rlnc.h: AddPiece
// (single, batched, lazy, on the GPU elimination or kodr's route on the
// host), GetPiece(s), progressive decode, destroy.  Shared definitions in
// capi_internal.hpp.
#include "capi_internal.hpp"

extern "C" {

/* ---- decoder ------------------------------------------------------------ */
int rlnc_decoder_create(rlnc_ctx* ctx, size_t k, rlnc_decoder** out) {
  if (!out) return RLNC_ERR_INVALID_ARGUMENT;
  if (ctx) TRY(set_dev(ctx));
  rlnc_decoder* d = new (std::nothrow) rlnc_decoder(k);
  if (!d) return RLNC_ERR_OUT_OF_MEMORY;
  d->ctx = ctx;
  if (ctx)
    for (DevBuf* b : {&d->recv, &d->recv_bs, &d->tmat, &d->decoded, &d->rowbuf, &d->scratch, &d->ptab})
      b->bind(ctx->device, ctx->stream);
  static const bool lazy = !kodr_amd::tune_env("KODR_DEC_LAZY") || atoi(kodr_amd::tune_env("KODR_DEC_LAZY")) != 0;  // A/B knob
  d->lazy = lazy;
  *out = d;
  return RLNC_OK;
}

int rlnc_decoder_destroy(rlnc_decoder* d) {
  if (!d) return RLNC_OK;
  // The device buffers go back to the stream-ordered pool without a host
  // wait: with the context stream idle (a query) at once, else pending until
  // the pool's next allocation orders them behind one event on that stream
  // (every use of them -- copies, products, the side stream's copies joined
  // into it -- is ordered there; DevicePool::defer_free).  The
  // host state goes now; no pending device work reads host memory of the
  // decoder's own.  (Until round 5 a destroy behind pending work waited for
  // the stream: the GPU sat idle from each round trip's GetPieces to the
  // next step's encode while the host woke up and freed.)
  DevBuf* bufs[] = {&d->recv, &d->tmat, &d->decoded, &d->rowbuf, &d->scratch, &d->recv_bs, &d->prog, &d->ptab};
  if (d->ctx) {
    (void)hipSetDevice(d->ctx->device);
    if (hipStreamQuery(d->ctx->stream) == hipSuccess) {
      for (DevBuf* b : bufs) b->release(true);
    } else {
      (void)hipGetLastError();  // (hipErrorNotReady from the query)
      kodr_amd::DevicePool& pool = kodr_amd::DevicePool::get(d->ctx->device);
      for (DevBuf* b : bufs) {
        uint8_t* p;
        size_t c;
        b->take(&p, &c);
        pool.defer_free(p, c, d->ctx->stream);
      }
    }
  } else {
    for (DevBuf* b : bufs) b->release(false);
  }
  delete d;
  return RLNC_OK;
}

namespace {

// the compact rows' plain bytes from their twin (bit-slicing is an involution)
int dec_uncompact(rlnc_decoder* d) {
  if (d->cmp_hi <= d->cmp_lo) return RLNC_OK;
  const size_t lo = d->cmp_lo, n = d->cmp_hi - d->cmp_lo;
  d->cmp_lo = d->cmp_hi = 0;
  HIPC(kodr_amd::bitslice_rows(d->recv_bs.p + lo * d->pitch, d->recv.p + lo * d->pitch, d->pitch, n, d->L,
                               d->ctx->stream));
  return RLNC_OK;
}

// grow the received-piece buffer so rows [0, need) fit; keeps rows [0, have)
int dec_reserve_rows(rlnc_decoder* d, size_t need, size_t have) {
  if (need <= d->recv_rows) return RLNC_OK;
  TRY(dec_uncompact(d));  // the copy below and the twin's rebuild read plain rows
  size_t nrows = std::max<size_t>(d->recv_rows ? d->recv_rows * 2 : d->core.piece_count() + 8, need);
  DevBuf nb;
  nb.bind(d->ctx->device, d->ctx->stream);
  TRY(nb.reserve(nrows * d->pitch));
  // the kernels read only rows < received, each through its pitch; only a
  // pitch past the piece length has bytes (zero padding) no copy writes
  if (d->pitch != d->L) HIPC(hipMemsetAsync(nb.p, 0, nrows * d->pitch, d->ctx->stream));
  if (d->recv.p && have)
    HIPC(hipMemcpyAsync(nb.p, d->recv.p, have * d->pitch, hipMemcpyDeviceToDevice, d->ctx->stream));
  d->recv.release();  // back to the pool, reusable once the stream passes the copy
  d->recv = nb;
  d->recv_rows = nrows;
  return RLNC_OK;
}

// store n pieces (source pitch spitch) as received rows [row0, row0 + n)
int dec_store_pieces(rlnc_decoder* d, size_t row0, const uint8_t* src, size_t spitch, size_t n, bool dev) {
  if (!d->ctx || !n) return RLNC_OK;
  TRY(dec_reserve_rows(d, row0 + n, row0));
  uint8_t* dst = d->recv.p + row0 * d->pitch;
  if (dev)
    HIPC(kodr_amd::copy_rows(src, spitch, dst, d->pitch, n, d->L, d->ctx->stream));
  else  // staged: the host buffer is only borrowed for the duration of the call
    HIPC(d->ctx->stage.h2d(dst, d->pitch, src, spitch, d->L, n, d->ctx->stream));
  return RLNC_OK;
}

int dec_check(rlnc_decoder* d, size_t vlen, const uint8_t* piece, size_t plen) {
  if (d->core.is_decoded()) return RLNC_ERR_ALL_USEFUL_PIECES_RECEIVED;  // full/decoder.go:52-54
  if (vlen != d->core.piece_count() || (d->ctx && !piece)) return RLNC_ERR_INVALID_ARGUMENT;
  if (d->have_len && plen != d->L) return RLNC_ERR_INVALID_ARGUMENT;
  if (d->ctx) TRY(set_dev(d->ctx));
  if (!d->have_len) {
    d->L = plen;
    d->pitch = round_up(std::max<size_t>(plen, 1), kPitchAlign);
    d->have_len = true;
  }
  return RLNC_OK;
}

int dec_progress(rlnc_decoder* d, long only);

extern "C++" {
template <class F>
int dec_elim_queues_gpu(rlnc_decoder* const* ds, size_t G, F before_read);
}

// a batch's elimination route, on the decoder and its context
enum ElimRoute { kElimGpu, kElimGpuRetried, kElimHostAfterGpu, kElimHost };
void count_elim(rlnc_decoder* d, ElimRoute r) {
  rlnc_ctx* c = d->ctx;
  switch (r) {
    case kElimGpuRetried:
      d->elim_gpu_retried++;
      if (c) c->n_elim_gpu_retried++;
      [[fallthrough]];
    case kElimGpu:
      d->elim_gpu++;
      if (c) c->n_elim_gpu++;
      break;
    case kElimHostAfterGpu:
      d->elim_host_after_gpu++;
      if (c) c->n_elim_host_after_gpu++;
      break;
    case kElimHost:
      d->elim_host++;
      if (c) c->n_elim_host++;
      break;
  }
}

// One decoder's elimination goes to the GPU (gf_elim_mc4: a chain workgroup
// beside row workgroups) instead of the host when its n new rows complete the
// rank of a state of kept rows (fresh or continued: the full-batch case) and
// k is at least the context's route_min_k (default 224, from where the GPU
// route measured at least as fast as the host's: 87 against 86 us at k = 224,
// 92-96 against 104-107 us at k = 256, profiles/r04/elim_modes/;
// rlnc_ctx_set_route_min_k).
bool dec_route_gpu(const rlnc_decoder* d, size_t n) {
  const size_t k = d->core.piece_count(), r = d->core.received();
  return d->ctx && k >= d->ctx->route_min_k && k <= 256 && n >= 2 && d->core.rank() == r && r + n >= k &&
         kodr_amd::gf_elim_mc_enabled();
}

// the queued coding vectors through kodr's elimination as one batch.  They
// were queued only while useful + queued < k, and each row raises the row
// count by at most one, so the rank can complete only at the last of them and
// add_many accepts all (none is refused as "all useful pieces received").
// A queue that completes the rank of a large decoder is eliminated on the GPU
// (dec_route_gpu); a singular one stays queued for the host.
// a systematic-looking queue (one of its first rows a unit vector) stays on
// the host, whose solver copies such rows (DecoderCore::solve_systematic_batch);
// the GPU's block pivots would find its blocks singular
bool queue_looks_systematic(const rlnc_decoder* d) {
  const size_t k = d->core.piece_count();
  for (size_t i = 0; i < std::min<size_t>(d->npend, 4); i++) {
    const uint8_t* v = d->pend_v.data() + i * k;
    size_t nz = 0;
    for (size_t j = 0; j < k && nz < 2; j++) nz += v[j] != 0;
    if (nz == 1) return true;
  }
  return false;
}

// (a queue the GPU already failed on -- a singular C -- goes straight to the
// host; a HIP error on the way is kept for the decoder's next call that
// returns a status, since the accessors that flush return none)
void dec_flush_coef(rlnc_decoder* d) {
  if (!d->npend) return;
  if (!d->gpu_rejected && dec_route_gpu(d, d->npend) && !queue_looks_systematic(d)) {
    rlnc_decoder* one = d;
    if (const int e = dec_elim_queues_gpu(&one, 1, [] { return RLNC_OK; }))
      if (d->sticky == RLNC_OK) d->sticky = e;
    if (!d->npend) return;
  }
  size_t used = 0;
  (void)d->core.add_many(d->pend_v.data(), d->core.piece_count(), d->npend, &used);
  count_elim(d, kElimHost);
  d->npend = 0;
  d->gpu_rejected = false;
}

// the HIP failure an accessor's flush met, once
int dec_take_sticky(rlnc_decoder* d) {
  const int e = d->sticky;
  d->sticky = RLNC_OK;
  return e;
}

// the queued device pieces into their received rows: one gather launch
constexpr size_t kPendMax = 1024;
int dec_flush_data(rlnc_decoder* d) {
  if (d->pend_src.empty()) return RLNC_OK;
  const size_t m = d->pend_src.size(), r0 = d->pend_row0;
  TRY(dec_reserve_rows(d, r0 + m, r0));
  TRY(d->ptab.reserve(m * sizeof(uint8_t*)));
  HIPC(d->ctx->stage.h2d(d->ptab.p, m * sizeof(uint8_t*), reinterpret_cast<const uint8_t*>(d->pend_src.data()),
                         m * sizeof(uint8_t*), m * sizeof(uint8_t*), 1, d->ctx->stream));
  HIPC(kodr_amd::gather_rows(reinterpret_cast<const uint8_t* const*>(d->ptab.p), d->recv.p + r0 * d->pitch, d->pitch,
                             m, d->L, d->ctx->stream));
  d->pend_src.clear();
  return RLNC_OK;
}

// everything queued: the state and the received rows are kodr's
int dec_flush(rlnc_decoder* d) {
  dec_flush_coef(d);
  TRY(dec_take_sticky(d));
  if (d->ctx && !d->pend_src.empty()) {
    TRY(set_dev(d->ctx));
    TRY(dec_flush_data(d));
  }
  return RLNC_OK;
}

// borrow: the caller keeps a device piece's bytes unchanged until the next
// data flush (rlnc_decoder_add_piece_device_borrowed); otherwise the piece is
// copied in the call
int dec_add(rlnc_decoder* d, const uint8_t* vec, size_t vlen, const uint8_t* piece, size_t plen,
            bool dev, bool borrow) {
  if (!d) return RLNC_ERR_INVALID_ARGUMENT;
  const size_t k = d->core.piece_count();
  // the queue could complete the rank: observe the state (full/decoder.go:52-54)
  if (d->npend && d->core.useful() + d->npend >= k) dec_flush_coef(d);
  TRY(dec_take_sticky(d));
  if (d->core.is_decoded()) return RLNC_ERR_ALL_USEFUL_PIECES_RECEIVED;
  if (!vec) return RLNC_ERR_INVALID_ARGUMENT;
  TRY(dec_check(d, vlen, piece, plen));
  const size_t row = d->core.received() + d->npend;  // this piece's arrival index
  d->decoded_ready = false;
  if (d->lazy && d->policy == RLNC_DECODE_LAZY) {
    d->pend_v.resize((d->npend + 1) * k);
    memcpy(d->pend_v.data() + d->npend * k, vec, k);
    d->npend++;
    d->gpu_rejected = false;  // a new queue
    if (!d->ctx) return RLNC_OK;
    if (dev && borrow && (uintptr_t)piece % 16 == 0) {  // borrowed until the next data flush
      if (d->pend_src.empty()) d->pend_row0 = row;
      d->pend_src.push_back(piece);
      if (d->pend_src.size() >= kPendMax) TRY(dec_flush_data(d));
      return RLNC_OK;
    }
    TRY(dec_flush_data(d));
    return dec_store_pieces(d, row, piece, d->L, 1, dev);
  }
  TRY(dec_flush(d));
  TRY(d->core.add(vec));
  count_elim(d, kElimHost);
  TRY(dec_store_pieces(d, d->core.received() - 1, piece, d->L, 1, dev));
  if (d->policy == RLNC_DECODE_EAGER) TRY(dec_progress(d, -1));
  return RLNC_OK;
}

// bit-sliced twin of the received rows: rows [bs_rows, received) added
// (all of them again when the plain buffer has grown)
int dec_extend_twin(rlnc_decoder* d) {
  const size_t recv = d->core.received();
  if (d->recv_bs.cap < d->recv_rows * d->pitch) {
    TRY(dec_uncompact(d));
    TRY(d->recv_bs.reserve(d->recv_rows * d->pitch));
    d->bs_rows = 0;
  }
  if (d->bs_rows < recv) {
    HIPC(kodr_amd::bitslice_rows(d->recv.p + d->bs_rows * d->pitch, d->recv_bs.p + d->bs_rows * d->pitch,
                                 d->pitch, recv - d->bs_rows, d->L, d->ctx->stream));
    d->bs_rows = recv;
  }
  return RLNC_OK;
}

// X = the received rows for a T x R product of M output rows: the plain rows
// for small M, else the bit-sliced twin with rows [bs_rows, received) added.
int dec_gemm(rlnc_decoder* d, const uint8_t* dA, size_t M, uint8_t* dY, size_t ldy) {
  const size_t recv = d->core.received();
  rlnc_ctx* ctx = d->ctx;
  const size_t twin_ok = d->recv_bs.cap >= d->recv_rows * d->pitch ? std::min(d->bs_rows, recv) : 0;
  size_t min_rows = (recv - twin_ok) * d->pitch <= kBsTwinBudget ? kBsMinRows : kBsMinRowsDecode;
#ifdef KODR_TUNE_MODES
  if (const char* env = kodr_amd::tune_env("KODR_BS_MIN_ROWS_DEC")) min_rows = (size_t)atol(env);
#endif
  d->last_bs = false;
  if (M < min_rows || few_narrow_rows(M, recv, d->L) || (d->pitch % 32) ||
      !bs_chunk_rows(M, std::max<size_t>(recv, 1), d->pitch, d->L) ||
      !kodr_amd::bs_ready(ctx->device)) {
    TRY(dec_uncompact(d));
    return gemm(ctx, dA, recv, M, recv, d->recv.p, d->pitch, dY, ldy, d->L);
  }
  d->last_bs = true;
  TRY(dec_extend_twin(d));
  return gemm_bs(ctx, dA, recv, M, recv, d->recv_bs.p, d->pitch, dY, ldy, d->L);
}

// decoded rows [0, rows) = T x R into dst (device, pitch dpitch).
// A row of T that is a unit vector e_j selects received piece j unchanged: a
// systematic piece (systematic/encoder.go:83-96), which kodr's elimination
// never modifies since it has no entry off its pivot column.  Those rows are
// copied, and only the other m rows go through the GF kernel: m x recv x L
// MACs instead of rows x recv x L (systematic/decoder.go:96-104
// leaves this undone).  The bytes are identical either way.
// With hdst (host array of rows destinations), row i goes to hdst[i] instead.
int dec_apply(rlnc_decoder* d, size_t rows, const uint8_t* trows, uint8_t* dst, size_t dpitch,
              uint8_t* const* hdst = nullptr) {
  const size_t recv = d->core.received();
  hipStream_t st = d->ctx->stream;
  d->hsrc.assign(rows, nullptr);
  size_t m = 0;
  for (size_t i = 0; i < rows; i++) {
    const uint8_t* t = trows + i * recv;
    size_t j = 0;
    while (j < recv && !t[j]) j++;
    bool unit = j < recv && t[j] == 1;
    for (size_t q = j + 1; unit && q < recv; q++) unit = !t[q];
    if (unit && j >= d->cmp_lo && j < d->cmp_hi)  // a compact row: gathered from its twin, un-sliced
      d->hsrc[i] = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(d->recv_bs.p + j * d->pitch) | 1);
    else if (unit)
      d->hsrc[i] = d->recv.p + j * d->pitch;
    else
      m++;
  }
  d->last_gf_rows = m;
  d->last_copy_rows = rows - m;
  if (!hdst && (m == rows || rows > 65535 || dpitch % 16)) {  // no unit rows: straight into dst
    d->last_gf_rows = rows;
    d->last_copy_rows = 0;
    TRY(d->tmat.reserve(std::max<size_t>(rows * recv, 1)));
    HIPC(d->ctx->stage.h2d(d->tmat.p, recv, trows, recv, recv, rows, st));
    return dec_gemm(d, d->tmat.p, rows, dst, dpitch);
  }
  // one upload ahead of both kernels: [the m GF rows of T | the gather's
  // source-row table | its destination table, if any].  A small H2D costs
  // ~15-20 us of DMA latency, so a second one between the kernels would stall
  // the stream.
  const size_t tbytes = (m * recv + 15) / 16 * 16, pbytes = rows * sizeof(uint8_t*);
  const size_t dbytes = hdst ? pbytes : 0;
  if (m) TRY(d->scratch.reserve(m * d->pitch));
  d->hTc.resize(tbytes + pbytes + dbytes);
  for (size_t i = 0, t = 0; i < rows; i++)
    if (!d->hsrc[i]) {
      memcpy(d->hTc.data() + t * recv, trows + i * recv, recv);
      d->hsrc[i] = d->scratch.p + t * d->pitch;
      t++;
    }
  memcpy(d->hTc.data() + tbytes, d->hsrc.data(), pbytes);
  if (hdst) memcpy(d->hTc.data() + tbytes + pbytes, hdst, dbytes);
  const size_t up = tbytes + pbytes + dbytes;
  TRY(d->tmat.reserve(up));
  HIPC(d->ctx->stage.h2d(d->tmat.p, up, d->hTc.data(), up, up, 1, st));
  if (m) TRY(dec_gemm(d, d->tmat.p, m, d->scratch.p, d->pitch));
  HIPC(kodr_amd::gather_rows(reinterpret_cast<const uint8_t* const*>(d->tmat.p + tbytes), dst, dpitch, rows, d->L,
                             st, hdst ? reinterpret_cast<uint8_t* const*>(d->tmat.p + tbytes + pbytes) : nullptr));
  return RLNC_OK;
}

// Materialize decoded original pieces that have no slot yet (all of them
// when `only` < 0, else just piece `only`) into new slots of d->prog: row
// T_i * inv(a) of the state row a*e_j, one dec_apply for the lot (systematic
// pieces are unit rows of T: copies).  Asynchronous on the context stream.
int dec_progress(rlnc_decoder* d, long only) {
  const size_t k = d->core.piece_count();
  if (!d->ctx || !d->have_len) return RLNC_OK;
  d->core.decoded(&d->drow, &d->dscale);
  if (d->slot_of.size() != k) d->slot_of.assign(k, -1);
  const size_t recv = d->core.received();
  std::vector<size_t> todo;
  for (size_t j = 0; j < k; j++)
    if (d->drow[j] >= 0 && d->slot_of[j] < 0 && (only < 0 || (size_t)only == j)) todo.push_back(j);
  if (todo.empty()) return RLNC_OK;
  if (d->out_ext) {  // straight into the caller's generation buffer, row j
    const kodr_amd::hostgf::Tables& t = kodr_amd::hostgf::T();
    for (size_t q0 = 0; q0 < todo.size(); q0 += 32768) {
      const size_t nq = std::min<size_t>(todo.size() - q0, 32768);
      std::vector<uint8_t> hT(nq * recv);
      d->hdst.resize(nq);
      for (size_t q = 0; q < nq; q++) {
        const size_t j = todo[q0 + q];
        const uint8_t* tr = d->core.t_row((size_t)d->drow[j]);
        const uint8_t a = d->dscale[j];
        for (size_t c = 0; c < recv; c++) hT[q * recv + c] = a == 1 ? tr[c] : t.mul(tr[c], t.inv(a));
        d->hdst[q] = d->out_ext + j * d->out_pitch;
      }
      TRY(dec_apply(d, nq, hT.data(), nullptr, 0, d->hdst.data()));
      for (size_t q = 0; q < nq; q++) d->slot_of[todo[q0 + q]] = (int32_t)todo[q0 + q];
    }
    return RLNC_OK;
  }
  if (d->prog.cap < k * d->pitch) {
    if (d->nslots) {  // keep the slots made so far
      DevBuf nb;
      nb.bind(d->ctx->device, d->ctx->stream);
      TRY(nb.reserve(k * d->pitch));
      HIPC(hipMemcpyAsync(nb.p, d->prog.p, d->nslots * d->pitch, hipMemcpyDeviceToDevice, d->ctx->stream));
      d->prog.release();
      d->prog = nb;
    } else {
      TRY(d->prog.reserve(k * d->pitch));
    }
  }
  const kodr_amd::hostgf::Tables& t = kodr_amd::hostgf::T();
  std::vector<uint8_t> hT(todo.size() * recv);
  for (size_t q = 0; q < todo.size(); q++) {
    const size_t j = todo[q];
    const uint8_t* tr = d->core.t_row((size_t)d->drow[j]);
    const uint8_t a = d->dscale[j];
    for (size_t c = 0; c < recv; c++) hT[q * recv + c] = a == 1 ? tr[c] : t.mul(tr[c], t.inv(a));
  }
  TRY(dec_apply(d, todo.size(), hT.data(), d->prog.p + d->nslots * d->pitch, d->pitch));
  for (size_t q = 0; q < todo.size(); q++) d->slot_of[todo[q]] = (int32_t)(d->nslots + q);
  d->nslots += todo.size();
  return RLNC_OK;
}

int dec_materialize(rlnc_decoder* d) {
  if (d->decoded_ready) return RLNC_OK;
  const size_t rows = d->core.rank(), recv = d->core.received();
  d->hT.resize(std::max<size_t>(rows * recv, 1));
  d->core.copy_transform(d->hT.data(), recv);
  TRY(d->decoded.reserve(std::max<size_t>(rows * d->pitch, 1)));
  TRY(dec_apply(d, rows, d->hT.data(), d->decoded.p, d->pitch));
  HIPC(hipStreamSynchronize(d->ctx->stream));
  d->decoded_ready = true;
  return RLNC_OK;
}

}  // namespace

int rlnc_decoder_add_piece(rlnc_decoder* d, const uint8_t* vec, size_t vlen, const uint8_t* piece,
                           size_t plen) {
  return dec_add(d, vec, vlen, piece, plen, false, false);
}

int rlnc_decoder_add_piece_device(rlnc_decoder* d, const uint8_t* vec, size_t vlen,
                                  const uint8_t* d_piece, size_t plen) {
  return dec_add(d, vec, vlen, d_piece, plen, true, false);
}

int rlnc_decoder_add_piece_device_borrowed(rlnc_decoder* d, const uint8_t* vec, size_t vlen,
                                           const uint8_t* d_piece, size_t plen) {
  return dec_add(d, vec, vlen, d_piece, plen, true, true);
}

namespace {

// Data side of a batched AddPiece, before the elimination: device rows and
// rows from pinned host memory are copied (and, for a large batch,
// bit-sliced into the decoder's twin) first, so the GPU work overlaps the
// elimination; rows past the ones accepted land beyond the received range
// and are never read.  The rows that can still be accepted before full rank
// (plus some slack for dependent ones) are copied first; the rest, if any are
// accepted, after (dec_batch_post).
struct BatchCopy {
  size_t row0 = 0, pre = 0, twin_end = 0;
  bool early = false;
};

// With `defer`, a fused copy of device rows is appended there instead of
// launched (rlnc_decoders_add_pieces_gpu launches all of them at once).
struct DeferredCopy {
  const uint8_t* src;
  uint8_t* dst;
  uint8_t* dbs;
  size_t rows, dpitch;
};
int dec_batch_pre(rlnc_decoder* d, const uint8_t* rows, size_t count, size_t pitch, bool dev, BatchCopy* bc,
                  std::vector<DeferredCopy>* defer = nullptr) {
  const size_t k = d->core.piece_count();
  bc->row0 = d->core.received();
  bc->early = d->ctx && (dev || kodr_amd::Staging::is_pinned(rows));
  bc->pre = bc->early ? std::min(count, d->core.required() + 16) : 0;
  bc->twin_end = 0;
  const size_t row0 = bc->row0, pre = bc->pre;
  if (!pre) return RLNC_OK;
  TRY(dec_reserve_rows(d, row0 + pre, row0));
  uint8_t* dst = d->recv.p + row0 * d->pitch;
  const bool twin = pre >= kBsMinRowsDecode && d->pitch % 32 == 0 &&
                    !few_narrow_rows(d->core.piece_count(), row0 + pre, d->L);  // else dec_gemm takes gf_gemm
  if (twin) {
    d->bs_rows = std::min(d->bs_rows, row0);  // rows [row0, ..) are new
    if (d->recv_bs.cap < d->recv_rows * d->pitch) {  // as dec_extend_twin, through row0 + pre
      TRY(dec_uncompact(d));
      TRY(d->recv_bs.reserve(d->recv_rows * d->pitch));
      d->bs_rows = 0;
    }
  }
  // device rows whose twin starts here: bit-sliced in one pass, into the twin
  // only (compact rows [row0, row0 + pre), appended to a compact range that
  // ends at row0) -- the plain copy's 1/3 of the pass's traffic is skipped
  uint8_t* dbs = twin ? d->recv_bs.p + row0 * d->pitch : nullptr;
  bool fused = false;
  if (twin && dev && d->bs_rows == row0 && d->L % 32 == 0) {
    if (d->cmp_hi > d->cmp_lo && d->cmp_hi != row0) TRY(dec_uncompact(d));
    if (defer && kodr_amd::copy_bitslice_ok(rows + k, pitch, nullptr, dbs, d->pitch, d->L) && pre <= 0x7fffffff) {
      defer->push_back({rows + k, nullptr, dbs, pre, d->pitch});
      fused = true;
    } else {
      fused = kodr_amd::copy_bitslice_rows(rows + k, pitch, nullptr, dbs, d->pitch, pre, d->L, d->ctx->stream) ==
              hipSuccess;
    }
    if (fused) {
      if (d->cmp_hi <= d->cmp_lo) d->cmp_lo = row0;
      d->cmp_hi = row0 + pre;
    }
  }
  if (!fused) {
    if (dev)
      HIPC(kodr_amd::copy_rows(rows + k, pitch, dst, d->pitch, pre, d->L, d->ctx->stream));
    else
      HIPC(hipMemcpy2DAsync(dst, d->pitch, rows + k, pitch, d->L, pre, hipMemcpyHostToDevice, d->ctx->stream));
    if (twin)
      HIPC(kodr_amd::bitslice_rows(d->recv.p + d->bs_rows * d->pitch, d->recv_bs.p + d->bs_rows * d->pitch,
                                   d->pitch, row0 + pre - d->bs_rows, d->L, d->ctx->stream));
  }
  if (twin) bc->twin_end = row0 + pre;
  return RLNC_OK;
}

// after the elimination accepted n rows of the batch
int dec_batch_post(rlnc_decoder* d, const uint8_t* rows, size_t pitch, bool dev, const BatchCopy& bc, size_t n) {
  const size_t k = d->core.piece_count();
  if (n) d->decoded_ready = false;
  if (bc.twin_end) d->bs_rows = bc.row0 + std::min(n, bc.pre);  // only accepted rows' twin counts
  if (d->cmp_hi > bc.row0 + n) d->cmp_hi = std::max(d->cmp_lo, bc.row0 + n);  // nor compact rows past them
  // accepted rows not copied yet (dependent rows past the slack, or the
  // staged path) -> one 2D copy
  if (n > bc.pre) TRY(dec_store_pieces(d, bc.row0 + bc.pre, rows + bc.pre * pitch + k, pitch, n - bc.pre, dev));
  if (bc.early && !dev) HIPC(hipStreamSynchronize(d->ctx->stream));  // the caller may reuse rows on return
  return RLNC_OK;
}

}  // namespace

}  // extern "C"
namespace {
// rlnc_decoder_add_pieces with kodr's elimination on the host
int dec_add_pieces_host(rlnc_decoder* d, const uint8_t* rows, size_t count, size_t pitch, size_t piece_len,
                        int is_device, size_t* consumed) {
  if (!d || !rows || !consumed) return RLNC_ERR_INVALID_ARGUMENT;
  *consumed = 0;
  if (!count) return RLNC_OK;
  const size_t k = d->core.piece_count();
  if (pitch < k + piece_len) return RLNC_ERR_INVALID_ARGUMENT;
  const bool dev = is_device != 0;
  if (dev && !d->ctx) return RLNC_ERR_NO_DEVICE;
  TRY(dec_flush(d));
  TRY(dec_check(d, k, rows + k, piece_len));
  const uint8_t* vecs = rows;
  size_t vpitch = pitch;
  // device rows: one strided copy of all coding vectors to the host (the
  // pieces never leave the device).  A small one is only started here and
  // awaited after the piece copies are enqueued behind it.
  int vticket = -1;
  if (dev) {
    d->hvecs.resize(count * k);
    if (count * k <= kodr_amd::kDownloadSmallMax)
      HIPC(d->ctx->stage.d2h_small_begin(rows, pitch, k, count, d->ctx->stream, &vticket));
    else
      HIPC(d->ctx->stage.d2h(d->hvecs.data(), k, rows, pitch, k, count, d->ctx->stream));
    vecs = d->hvecs.data();
    vpitch = k;
  }
  BatchCopy bc;
  if (const int e = dec_batch_pre(d, rows, count, pitch, dev, &bc)) {
    if (vticket >= 0) d->ctx->stage.d2h_small_cancel(vticket);  // else every later small download fails
    return e;
  }
  if (vticket >= 0) HIPC(d->ctx->stage.d2h_small_end(vticket, d->hvecs.data(), k, k, count));
  // coefficient side, exactly as repeated AddPiece calls
  size_t n = 0;
  const int st = d->core.add_many(vecs, vpitch, count, &n);
  count_elim(d, kElimHost);
  TRY(dec_batch_post(d, rows, pitch, dev, bc, n));
  if (n && d->policy == RLNC_DECODE_EAGER) TRY(dec_progress(d, -1));
  *consumed = n;
  return st;
}
}  // namespace
extern "C" {

// Batched AddPiece: device rows that complete the rank of a large decoder go
// through the GPU elimination (rlnc_decoder_add_pieces_gpu), the rest through
// kodr's algorithm on the host.  Same state either way.
int rlnc_decoder_add_pieces(rlnc_decoder* d, const uint8_t* rows, size_t count, size_t pitch,
                            size_t piece_len, int is_device, size_t* consumed) {
  if (d && rows && consumed && count && is_device && d->ctx && pitch >= d->core.piece_count() + piece_len) {
    TRY(dec_flush(d));
    if (dec_route_gpu(d, count)) return rlnc_decoder_add_pieces_gpu(d, rows, count, pitch, piece_len, consumed);
  }
  return dec_add_pieces_host(d, rows, count, pitch, piece_len, is_device, consumed);
}

namespace {

// KODR_ADD_SIDE=0 keeps the batched AddPiece's row copies on the context
// stream ahead of the elimination (A/B)
// The batched AddPiece's row copies: 2 (default) on the context stream after
// the elimination launch, 1 on the side stream beside it, 0 on the context
// stream ahead of it (A/B; profiles/r05/copy_order/).  Beside the elimination
// the two slow each other down (copy 336 against 186 us alone, elimination
// 228-258 against 150 for 16 C2 generations) and GetPieces waits on a
// cross-stream event; after it, the round trip's GetPieces follows the copy
// 6 us later (35 us earlier per step) and a single decoder's elimination runs
// alone.
int add_copy_mode() {
  static const int v = kodr_amd::tune_env("KODR_ADD_SIDE") ? atoi(kodr_amd::tune_env("KODR_ADD_SIDE")) : 2;
  return v;
}
bool add_side_stream() { return add_copy_mode() == 1; }

int ctx_side(rlnc_ctx* ctx) {
  if (ctx->side) return RLNC_OK;
  HIPC(hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking));
  HIPC(hipEventCreateWithFlags(&ctx->side_done, hipEventDisableTiming));
  HIPC(hipEventCreateWithFlags(&ctx->rows_ready, hipEventDisableTiming));
  HIPC(hipEventCreateWithFlags(&ctx->elim_ready, hipEventDisableTiming));
  return RLNC_OK;
}

// pinned host memory for `bytes` of a batch's coding vectors (grown as
// needed: the aux stream's downloads into the old buffer are waited for)
int ctx_vec_pin(rlnc_ctx* ctx, size_t bytes) {
  if (!ctx->vec_ready) HIPC(hipEventCreateWithFlags(&ctx->vec_ready, hipEventDisableTiming));
  if (bytes <= ctx->vec_pin_cap) return RLNC_OK;
  if (ctx->aux) HIPC(hipStreamSynchronize(ctx->aux));
  if (ctx->vec_pin) (void)hipHostFree(ctx->vec_pin);
  ctx->vec_pin = nullptr;
  ctx->vec_pin_cap = 0;
  HIPC(hipHostMalloc((void**)&ctx->vec_pin, std::max<size_t>(bytes, 64 << 10), hipHostMallocDefault));
  ctx->vec_pin_cap = std::max<size_t>(bytes, 64 << 10);
  return RLNC_OK;
}

// a stream for small reads of rows whose producers are ordered before
// ctx->rows_ready, and that must not wait for the copies queued after it
// (at the device's highest stream priority: a high-priority stream takes a
// hardware queue of its own pool, so the download -- a blit kernel for a
// strided D2H copy -- never queues behind a kernel of an application stream
// that shares a normal-priority hardware queue with it; beyond
// GPU_MAX_HW_QUEUES streams share those)
int ctx_aux_after_rows(rlnc_ctx* ctx, hipStream_t* st) {
  if (!ctx->aux) {
    int least = 0, greatest = 0;
    HIPC(hipDeviceGetStreamPriorityRange(&least, &greatest));
    HIPC(hipStreamCreateWithPriority(&ctx->aux, hipStreamNonBlocking, greatest));
  }
  HIPC(hipStreamWaitEvent(ctx->aux, ctx->rows_ready, 0));
  *st = ctx->aux;
  return RLNC_OK;
}

// the field tables gf_elim reads (uploaded once per context)
int ctx_elim_tables(rlnc_ctx* ctx) {
  if (ctx->elim_tab_ok) return RLNC_OK;
  ctx->elim_tab.bind(ctx->device, ctx->stream);
  TRY(ctx->elim_tab.reserve(kodr_amd::kElimTableWords * 4));
  std::vector<uint32_t> t(kodr_amd::kElimTableWords);
  kodr_amd::elim_tables(t.data());
  HIPC(ctx->stage.h2d(ctx->elim_tab.p, t.size() * 4, reinterpret_cast<const uint8_t*>(t.data()), t.size() * 4,
                      t.size() * 4, 1, ctx->stream));
  ctx->elim_tab_ok = true;
  return RLNC_OK;
}

constexpr size_t kElimHdr = 4 * kodr_amd::kElimMcMaxBlocks;  // counts / status words ahead of the states

// the multi-workgroup elimination's hand-off buffer for nc decoders and this
// launch's tags: gf_elim_mc_attempts() consecutive ones, after every tag any
// earlier launch of the context used.  Tags only grow, so neither the hand-off
// granules nor the status words in pinned memory (elim_pin) can hold a tag of
// this launch before it runs, whichever buffer was reallocated since; a new
// hand-off buffer is zeroed (tag 0: never a launch's).  When the tags would
// wrap, the stream is drained and both are zeroed before counting from 1.
int ctx_elim_mc(rlnc_ctx* ctx, size_t k, size_t nc, kodr_amd::ElimArgs* a) {
  const size_t bytes = kodr_amd::gf_elim_mc_pub_bytes((int)k, (int)nc);
  const uint32_t na = (uint32_t)kodr_amd::gf_elim_mc_attempts();
  ctx->elim_pub.bind(ctx->device, ctx->stream);
  const uint8_t* before = ctx->elim_pub.p;
  TRY(ctx->elim_pub.reserve(bytes));
  if (ctx->elim_epoch + na >= 0x7ffffff0u) {
    HIPC(hipStreamSynchronize(ctx->stream));
    if (ctx->elim_pin) memset(ctx->elim_pin, 0, std::min(ctx->elim_pin_cap, kElimHdr));
    HIPC(hipMemsetAsync(ctx->elim_pub.p, 0, ctx->elim_pub.cap, ctx->stream));
    ctx->elim_epoch = 0;
  } else if (ctx->elim_pub.p != before) {
    HIPC(hipMemsetAsync(ctx->elim_pub.p, 0, ctx->elim_pub.cap, ctx->stream));
  }
  a->pub = reinterpret_cast<uint64_t*>(ctx->elim_pub.p);
  a->epoch = ctx->elim_epoch + 1;
  ctx->elim_epoch += na;
  return RLNC_OK;
}

// decoders per elimination launch: the multi-workgroup kernel needs all of a
// launch's workgroups resident at once
size_t elim_chunk(size_t k, size_t n) {
  size_t c = std::min<size_t>(n, kodr_amd::kElimMaxGens);
  if (k >= 2 && k <= 256) c = std::min<size_t>(c, (size_t)kodr_amd::gf_elim_mc_max_gens((int)k));
  return std::max<size_t>(c, 1);
}

// per decoder of a launch: the number of state rows the kernel left (counts
// of the one-workgroup kernels; k when every workgroup of the multi-workgroup
// kernel reports done, else 0)
void elim_counts(const kodr_amd::ElimArgs& a, size_t nc, bool mc, const uint8_t* hdr, int* cnt) {
  const int* c = reinterpret_cast<const int*>(hdr);
  const int P = kodr_amd::gf_elim_mc_groups(a.k, (int)nc);
  for (size_t i = 0; i < nc; i++) {
    if (!mc) {
      cnt[i] = c[i];
      continue;
    }
    bool ok = true;
    for (int q = 0; q < P; q++) ok = ok && c[i * P + q] == 1;
    cnt[i] = ok ? a.k : 0;
  }
}

// the pinned, device-mapped buffer gf_elim_mc2 writes its status words and T
// rows into ("direct"), grown as needed and zeroed when allocated
int ctx_elim_pin(rlnc_ctx* ctx, size_t bytes) {
  if (bytes <= ctx->elim_pin_cap) return RLNC_OK;
  HIPC(hipStreamSynchronize(ctx->stream));
  if (ctx->elim_pin) (void)hipHostFree(ctx->elim_pin);
  ctx->elim_pin = nullptr;
  ctx->elim_pin_cap = 0;
  HIPC(hipHostMalloc((void**)&ctx->elim_pin, bytes, hipHostMallocCoherent));
  memset(ctx->elim_pin, 0, bytes);
  HIPC(hipHostGetDevicePointer((void**)&ctx->elim_pin_dev, ctx->elim_pin, 0));
  ctx->elim_pin_cap = bytes;
  return RLNC_OK;
}

// A direct launch's results: the host polls the status words in pinned
// memory (each workgroup stores its word after its T rows, system-scope
// release) instead of synchronising the stream and copying.  A word is
// reported when it carries one of the launch's tags (tag0 + attempt, bit 31
// set on failure).  Decoder i is resolved when every one of its workgroups
// reported success (cnt[i] = k, att[i] = the attempt that succeeded) or any
// reported failure (cnt[i] = 0: kodr's route on the host).  on_fail(i) runs
// as soon as decoder i fails, while the launch may still run.
// A decoder still unresolved kElimGiveUp after the launch became eligible to
// run -- its workgroups not resident, e.g. behind another kernel on the same
// GPU -- is given up the same way: the launch finishes in the background on
// the context stream, which every later use of its buffers and of the
// caller's rows is ordered behind (device rows are read asynchronously on
// that stream), and its late results are never read.  "Eligible": `ready`,
// recorded on the context stream right before the launch, has completed (the
// work queued ahead of the launch on the same stream -- a large encode, the
// previous step's GetPieces -- does not count against the launch).
constexpr auto kElimGiveUp = std::chrono::milliseconds(5);
int elim_direct_wait(rlnc_ctx* ctx, const kodr_amd::ElimArgs& a, size_t nc, int* cnt, int* att,
                     const std::function<int(size_t)>& on_fail, hipEvent_t ready) {
  const int P = kodr_amd::gf_elim_mc_groups(a.k, (int)nc);
  const uint32_t na = (uint32_t)kodr_amd::gf_elim_mc_attempts();
  const volatile uint32_t* st = reinterpret_cast<const volatile uint32_t*>(ctx->elim_pin);
  auto t0 = std::chrono::steady_clock::now();
  bool started = ready == nullptr;  // the give-up clock runs from t0 once the launch is eligible
  std::vector<int8_t> res(nc, 0);  // 0 open, 1 done, -1 failed or given up
  std::vector<int> satt(nc, 0);
  size_t open = nc;
  for (unsigned spins = 0; open;) {
    bool late = false;
    if (++spins < 4096) {
      _mm_pause();
    } else {
      std::this_thread::yield();
      if (!started) {
        const hipError_t q = hipEventQuery(ready);
        if (q == hipSuccess) {
          started = true;
          t0 = std::chrono::steady_clock::now();
        } else if (q != hipErrorNotReady) {
          HIPC(q);
        }
      }
      late = started && std::chrono::steady_clock::now() - t0 > kElimGiveUp;
    }
    for (size_t g = 0; g < nc; g++) {
      if (res[g]) continue;
      int done = 0;
      bool fail = false;
      uint32_t first = 0;
      for (int q = 0; q < P && !fail; q++) {
        const uint32_t v = st[g * P + q];
        const uint32_t t = (v & 0x7fffffffu) - a.epoch;
        if (t >= na) continue;  // not reported yet
        if (v & 0x80000000u) {
          fail = true;
        } else {
          done++;
          first = t;
        }
      }
      if (!fail && done < P && !late) continue;
      std::atomic_thread_fence(std::memory_order_acquire);
      res[g] = fail || done < P ? -1 : 1;
      satt[g] = (int)first;
      open--;
      if (res[g] < 0 && on_fail) TRY(on_fail(g));
    }
  }
  for (size_t i = 0; i < nc; i++) {
    cnt[i] = res[i] == 1 ? a.k : 0;
    att[i] = res[i] == 1 ? satt[i] : 0;
  }
  return RLNC_OK;
}

}  // namespace

int rlnc_decoders_add_pieces_gpu(rlnc_decoder* const* ds, size_t G, const uint8_t* const* rows,
                                 const size_t* counts, size_t pitch, size_t piece_len, size_t* consumed,
                                 int* status) {
  return rlnc_decoders_add_pieces_gpu_hook(ds, G, rows, counts, pitch, piece_len, consumed, status, nullptr,
                                           nullptr);
}

int rlnc_decoders_add_pieces_gpu_hook(rlnc_decoder* const* ds, size_t G, const uint8_t* const* rows,
                                      const size_t* counts, size_t pitch, size_t piece_len, size_t* consumed,
                                      int* status, rlnc_hook_fn after_launch, void* user) {
  if (!ds || !rows || !counts || !consumed || !status || !G) return RLNC_ERR_INVALID_ARGUMENT;
  // the caller's hook, once: after the first elimination launch, once the
  // work queued ahead of it on the context stream has completed (`ready`), so
  // that the launch's workgroups are dispatched before anything the hook
  // queues on other streams can take their CUs; else on the way out
  bool hooked = after_launch == nullptr;
  hipEvent_t hook_ev = nullptr;  // what the hook asked this call's later work to wait for
  auto run_hook = [&](hipEvent_t ready) -> int {
    if (hooked) return RLNC_OK;
    hooked = true;
    hipError_t q = hipSuccess;
    for (unsigned spins = 0; ready && (q = hipEventQuery(ready)) == hipErrorNotReady;)
      if (++spins < 4096)
        _mm_pause();
      else
        std::this_thread::yield();
    hook_ev = static_cast<hipEvent_t>(after_launch(user));
    HIPC(q == hipErrorNotReady ? hipSuccess : q);
    return RLNC_OK;
  };
  auto hook_guard = on_scope_exit([&] { (void)run_hook(nullptr); });
  rlnc_ctx* ctx = ds[0] ? ds[0]->ctx : nullptr;
  if (!ctx) return RLNC_ERR_NO_DEVICE;
  const size_t k = ds[0]->core.piece_count();
  for (size_t g = 0; g < G; g++) {
    if (!ds[g] || !rows[g]) return RLNC_ERR_INVALID_ARGUMENT;
    if (ds[g]->ctx != ctx || ds[g]->core.piece_count() != k) return RLNC_ERR_INVALID_ARGUMENT;
    consumed[g] = 0;
    status[g] = RLNC_OK;
  }
  {  // each decoder once: their host mirrors are loaded concurrently below
    std::vector<const rlnc_decoder*> u(ds, ds + G);
    std::sort(u.begin(), u.end());
    if (std::adjacent_find(u.begin(), u.end()) != u.end()) return RLNC_ERR_INVALID_ARGUMENT;
  }
  for (size_t g = 0; g < G; g++) TRY(dec_flush(ds[g]));
  if (pitch < k + piece_len) return RLNC_ERR_INVALID_ARGUMENT;
  TRY(set_dev(ctx));
  static const int timing = getenv("KODR_ADD_TIMING") ? atoi(getenv("KODR_ADD_TIMING")) : 0;
  const auto tnow = [] { return std::chrono::duration<double, std::micro>(
                             std::chrono::steady_clock::now().time_since_epoch()).count(); };
  const double tt0 = timing ? tnow() : 0;
  double tt1 = 0, tt2 = 0, tt3 = 0;
  // GPU elimination (kElimMaxGens per launch) for batches of >= 2 rows on
  //  * fresh decoders, from the rows' coding vectors;
  //  * decoders whose r received rows were all kept ("continued") and whose
  //    batch can complete the rank, from M = [their r coefficient rows ; the
  //    batch's first k - r vectors] (load_continued);
  // every other decoder takes rlnc_decoder_add_pieces.  (Continued batches
  // that cannot complete the rank would take the per-step kernel over all
  // r + n rows of M: measured slower than the host's add_panel, 1.7 against
  // 1.3 ms for 32 decoders at k = 256 adding 65 rows to 64, profiles/r03/elim_cont/.)
  std::vector<size_t> gpu;
  std::vector<BatchCopy> bcs(G);
  std::vector<DeferredCopy> defer;
  for (size_t g = 0; g < G; g++) {
    rlnc_decoder* d = ds[g];
    const size_t r = d->core.received();
    const bool cont = r >= 1 && r < k && d->core.rank() == r && r + counts[g] >= k;
    const bool ok = k >= 2 && k <= 256 && counts[g] >= 2 && (r == 0 || cont);
    if (!ok) {
      status[g] = dec_add_pieces_host(d, rows[g], counts[g], pitch, piece_len, 1, &consumed[g]);
      continue;
    }
    if ((status[g] = dec_check(d, k, rows[g] + k, piece_len)) != RLNC_OK) continue;
    gpu.push_back(g);
  }
  // the rows' reservations and deferred copies (dec_batch_pre), run after the
  // first elimination launch so that its kernel starts ahead of them; a
  // decoder whose preparation fails keeps its state (its launch result is
  // not loaded) and reports the error
  std::vector<uint8_t> pre_fail(G, 0);
  bool prepped = false;
  auto prep_rows = [&]() {
    if (prepped) return;
    prepped = true;
    for (size_t g : gpu)
      if ((status[g] = dec_batch_pre(ds[g], rows[g], counts[g], pitch, true, &bcs[g], &defer)) != RLNC_OK)
        pre_fail[g] = 1;
  };
  // the deferred row copies: one launch per kCopyGroupMax decoders (one piece
  // length, so one pitch).  With a side stream they run beside the
  // elimination, launched after it so that its workgroups get their CUs
  // first; the context stream waits for them before anything later.
  const bool side = !gpu.empty() && add_side_stream();
  const bool after = !gpu.empty() && add_copy_mode() == 2;
  // (the side stream's events also order the host route's vector reads of a
  // decoder whose launch failed or was given up: behind the rows' producers,
  // not behind the elimination)
  if (!gpu.empty()) TRY(ctx_side(ctx));
  auto launch_copies = [&]() -> int {
  for (size_t c0 = 0; c0 < defer.size(); c0 += kodr_amd::kCopyGroupMax) {
    const size_t nc = std::min<size_t>(kodr_amd::kCopyGroupMax, defer.size() - c0);
    kodr_amd::CopyGroup cg = {};
    for (size_t i = 0; i < nc; i++) {
      if (defer[c0 + i].dpitch != defer[c0].dpitch) return RLNC_ERR_INVALID_ARGUMENT;  // cannot happen
      cg.src[i] = defer[c0 + i].src;
      cg.dst[i] = defer[c0 + i].dst;
      cg.dbs[i] = defer[c0 + i].dbs;
      cg.rows[i] = (int)defer[c0 + i].rows;
    }
    HIPC(kodr_amd::copy_bitslice_rows_grouped(cg, (int)nc, pitch, defer[c0].dpitch, piece_len,
                                              side ? ctx->side : ctx->stream, side));
  }
  return RLNC_OK;
  };
  if (!gpu.empty()) HIPC(hipEventRecord(ctx->rows_ready, ctx->stream));  // the rows' producer work
  if (side) {
    HIPC(hipStreamWaitEvent(ctx->side, ctx->rows_ready, 0));  // ... ordered before the copies
  } else if (!after) {
    prep_rows();
    TRY(launch_copies());
  }
  bool copies_out = !side && !after;
  // an error return before the copies went out still launches them (the
  // decoders' row bookkeeping assumes them) and joins the side stream
  auto copies_guard = on_scope_exit([&] {
    if (copies_out) return;
    prep_rows();
    (void)launch_copies();
    if (!side) return;
    (void)hipEventRecord(ctx->side_done, ctx->side);
    (void)hipStreamWaitEvent(ctx->stream, ctx->side_done, 0);
  });
  if (timing) tt1 = tnow();
  if (gpu.empty()) return RLNC_OK;
  // fresh decoders first (their launches read the rows' vectors in place),
  // full batches first among them: launches of full batches only take the
  // blocked kernel
  std::vector<size_t> base(G, 0);  // rows a continued decoder held before
  for (size_t g : gpu) base[g] = ds[g]->core.received();
  std::stable_partition(gpu.begin(), gpu.end(), [&](size_t g) { return base[g] + counts[g] >= k; });
  std::stable_partition(gpu.begin(), gpu.end(), [&](size_t g) { return base[g] == 0; });
  const size_t nfresh = (size_t)std::count_if(gpu.begin(), gpu.end(), [&](size_t g) { return base[g] == 0; });
  TRY(ctx_elim_tables(ctx));
  const size_t opitch = k <= 128 ? 256 : 512, ostride = k * opitch, hdr = kElimHdr;
  const size_t chunk = elim_chunk(k, gpu.size());
  ctx->elim_out.bind(ctx->device, ctx->stream);
  TRY(ctx->elim_out.reserve(hdr + chunk * ostride));
  if (nfresh < gpu.size()) {  // continued decoders: their M, k x k each
    ctx->elim_in.bind(ctx->device, ctx->stream);
    TRY(ctx->elim_in.reserve(chunk * k * k));
  }
  // only what the kernel wrote is read back: no zero-fill, grown once per context
  if (ctx->elim_host.size() < hdr + chunk * ostride) ctx->elim_host.resize(hdr + chunk * ostride);
  uint8_t* const hostp = ctx->elim_host.data();
  std::vector<uint8_t>& hm = ctx->elim_hin;
  // chunks never mix fresh and continued decoders (one vector pitch per launch)
  for (size_t c0 = 0; c0 < gpu.size();) {
    const bool cont = c0 >= nfresh;
    const size_t nc = std::min(chunk, (cont ? gpu.size() : nfresh) - c0);
    kodr_amd::ElimArgs a = {};
    for (size_t i = 0; i < nc; i++) {
      const size_t g = gpu[c0 + i];
      a.n[i] = (int)std::min(base[g] + counts[g], k);
      a.vecs[i] = cont ? ctx->elim_in.p + i * k * k : rows[g];
    }
    if (cont) {
      // M of each decoder (k x k at pitch k): its coefficient rows, in row
      // order, in one upload for the chunk, then the batch's first k - r
      // vectors (device to device) below them
      if (hm.size() < nc * k * k) hm.resize(nc * k * k);  // rows past r: overwritten on the device below
      HostPool::get().run(nc, [&](size_t i) {
        const rlnc_decoder* d = ds[gpu[c0 + i]];
        for (size_t j = 0; j < base[gpu[c0 + i]]; j++) memcpy(hm.data() + (i * k + j) * k, d->core.coeff_row(j), k);
      });
      HIPC(ctx->stage.h2d(ctx->elim_in.p, k, hm.data(), k, k, nc * k, ctx->stream));
      // the vectors: one gather launch over all decoders of the chunk from
      // uploaded row tables when every row is 16-byte aligned, else a copy
      // per decoder
      bool aligned = k % 16 == 0 && pitch % 16 == 0;
      for (size_t i = 0; i < nc && aligned; i++) aligned = (uintptr_t)rows[gpu[c0 + i]] % 16 == 0;
      if (aligned) {
        std::vector<const void*> tab;
        for (int half = 0; half < 2; half++)
          for (size_t i = 0; i < nc; i++) {
            const size_t g = gpu[c0 + i], r = base[g];
            for (size_t j = 0; j < k - r; j++)
              tab.push_back(half ? (const void*)(ctx->elim_in.p + (i * k + r + j) * k)
                                 : (const void*)(rows[g] + j * pitch));
          }
        const size_t nr = tab.size() / 2, tb = tab.size() * sizeof(void*);
        ctx->gtab.bind(ctx->device, ctx->stream);
        TRY(ctx->gtab.reserve(tb));
        HIPC(ctx->stage.h2d(ctx->gtab.p, tb, reinterpret_cast<const uint8_t*>(tab.data()), tb, tb, 1, ctx->stream));
        const auto* src = reinterpret_cast<const uint8_t* const*>(ctx->gtab.p);
        const auto* dst = reinterpret_cast<uint8_t* const*>(ctx->gtab.p + nr * sizeof(void*));
        for (size_t r0 = 0; r0 < nr; r0 += 65535)
          HIPC(kodr_amd::gather_rows(src + r0, nullptr, 0, std::min<size_t>(65535, nr - r0), k, ctx->stream, dst + r0));
      } else {
        for (size_t i = 0; i < nc; i++) {
          const size_t g = gpu[c0 + i], r = base[g];
          HIPC(kodr_amd::copy_rows(rows[g], pitch, ctx->elim_in.p + (i * k + r) * k, k, k - r, k, ctx->stream));
        }
      }
    }
    a.vpitch = cont ? k : pitch;
    a.tables = reinterpret_cast<const uint32_t*>(ctx->elim_tab.p);
    a.out = ctx->elim_out.p + hdr;
    a.out_gen_stride = ostride;
    a.out_pitch = opitch;
    a.counts = reinterpret_cast<int*>(ctx->elim_out.p);
    a.k = (int)k;
    TRY(ctx_elim_mc(ctx, k, nc, &a));
    const bool mc = kodr_amd::gf_elim_mc_taken(a, (int)nc);
    const bool direct = kodr_amd::gf_elim_mc_direct(a, (int)nc);
    if (direct) {  // T and status straight into pinned host memory
      TRY(ctx_elim_pin(ctx, hdr + nc * k * k));
      a.direct = 1;
      a.out = ctx->elim_pin_dev + hdr;
      a.out_pitch = k;
      a.out_gen_stride = k * k;
      a.counts = reinterpret_cast<int*>(ctx->elim_pin_dev);
      if (!cont && c0 == 0) {  // fresh decoders: T on the device too, for a grouped GetPieces
        ctx->elim_tdev.bind(ctx->device, ctx->stream);
        TRY(ctx->elim_tdev.reserve(gpu.size() * k * k));
        ctx->tdev_seq++;
      }
      if (!cont) a.out_dev = ctx->elim_tdev.p + c0 * k * k;
    }
    // (the first launch starts right behind rows_ready; a later one behind the launch before it)
    if (direct && c0 > 0) HIPC(hipEventRecord(ctx->elim_ready, ctx->stream));
    HIPC(kodr_amd::gf_elim(a, (int)nc, ctx->stream));
    TRY(run_hook(c0 == 0 ? ctx->rows_ready : direct ? ctx->elim_ready : nullptr));
    if (hook_ev) {
      HIPC(hipStreamWaitEvent(ctx->stream, hook_ev, 0));  // the copies (context stream) after the caller's work
      hook_ev = nullptr;
    }
    if (!copies_out) {
      prep_rows();
      TRY(launch_copies());
      if (side) {
        HIPC(hipEventRecord(ctx->side_done, ctx->side));
        HIPC(hipStreamWaitEvent(ctx->stream, ctx->side_done, 0));  // everything after the read-back waits for them
      }
      copies_out = true;
    }
    // the chunk's coding vectors to pinned host memory by DMA on the aux
    // stream, ordered after the rows' producers only: a decoder this launch
    // leaves to the host route (a failed or given-up launch) reads them there.
    // Requested beside every launch: the copy may run as a blit kernel,
    // which needs a CU that a stalled launch, or whatever keeps it from being
    // resident, holds for the whole stall once its workgroups are waiting
    // (requested after a failure or after 1 ms of waiting, the 16-decoder
    // call took 18 ms beside the co-residency test's kernel, 57 ms with the
    // staged small copy; requested with the launch, 5.8-7 ms).
    std::vector<size_t> voff(nc + 1, 0);
    for (size_t i = 0; i < nc; i++) voff[i + 1] = voff[i] + counts[gpu[c0 + i]] * k;
    // (the pinned buffer is sized on every call: an allocation may wait for
    // the device, so it must not happen first in a stalled call)
    TRY(ctx_vec_pin(ctx, voff[nc]));
    bool vecs_out = false;
    auto fetch_vecs = [&]() -> int {
      if (vecs_out) return RLNC_OK;
      vecs_out = true;
      hipStream_t vs = ctx->stream;
      TRY(ctx_aux_after_rows(ctx, &vs));
      // decoders whose rows follow each other at the pitch inside one
      // allocation (the round trip's wire rows) share one 2D copy: a copy
      // may not span allocations, and each is a launch of its own
      for (size_t i = 0; i < nc;) {
        const uint8_t* r0 = rows[gpu[c0 + i]];
        size_t j = i + 1, nrow = counts[gpu[c0 + i]];
        hipDeviceptr_t base = nullptr;
        size_t size = 0;
        if (j < nc && hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)r0) == hipSuccess) {
          const uint8_t* end = reinterpret_cast<const uint8_t*>(base) + size;
          while (j < nc && rows[gpu[c0 + j]] == r0 + nrow * pitch &&
                 r0 + (nrow + counts[gpu[c0 + j]] - 1) * pitch + k <= end)
            nrow += counts[gpu[c0 + j++]];
        }
        (void)hipGetLastError();  // (a pointer the runtime does not know: no merge, no sticky error)
        HIPC(hipMemcpy2DAsync(ctx->vec_pin + voff[i], k, r0, pitch, k, nrow, hipMemcpyDeviceToHost, vs));
        i = j;
      }
      HIPC(hipEventRecord(ctx->vec_ready, vs));
      return RLNC_OK;
    };
    TRY(fetch_vecs());
    if (timing) tt2 = tnow();
    // the blocked kernel leaves [I | C^-1] or nothing: only the T halves come
    // back (one 2D copy: the generations' rows are evenly strided), else the
    // whole states
#ifdef KODR_ELIM_TIMING
    const bool tonly = false;  // the kernel's stamps sit in the state rows
#else
    const bool tonly = kodr_amd::gf_elim_blocked(a, (int)nc);
#endif
    std::vector<int> cntv(nc), attv(nc, 0);
    const uint8_t* tstates = hostp + hdr;  // T rows (tonly: k x k per decoder) or whole states
    // a decoder whose launch failed (a singular panel block, or a singular C)
    // takes kodr's route on the host from its state before the batch: started
    // on its own thread as soon as it reports, beside the rest of the launch
    std::vector<std::future<std::pair<int, size_t>>> early(nc);
    auto early_host = [&](size_t i) -> int {
      rlnc_decoder* d = ds[gpu[c0 + i]];
      const size_t g = gpu[c0 + i];
      if (d->core.is_decoded() || pre_fail[g]) return RLNC_OK;
      const size_t n = counts[g];
      TRY(fetch_vecs());
      const uint8_t* v = ctx->vec_pin + voff[i];
      hipEvent_t ev = ctx->vec_ready;
      early[i] = std::async(std::launch::async, [d, k, n, v, ev] {
        if (hipEventSynchronize(ev) != hipSuccess) return std::make_pair((int)RLNC_ERR_HIP, (size_t)0);
        size_t m = 0;
        const int st = d->core.add_many(v, k, n, &m);
        return std::make_pair(st, m);
      });
      return RLNC_OK;
    };
    // (a launch error below leaves the futures to their destructors, which wait)
    if (direct) {
      TRY(elim_direct_wait(ctx, a, nc, cntv.data(), attv.data(), std::function<int(size_t)>(early_host),
                           c0 == 0 ? ctx->rows_ready : ctx->elim_ready));
      tstates = ctx->elim_pin + hdr;
    } else if (tonly) {
      HIPC(ctx->stage.d2h(hostp, hdr, ctx->elim_out.p, hdr, hdr, 1, ctx->stream));
      HIPC(ctx->stage.d2h(hostp + hdr, k, ctx->elim_out.p + hdr + k, opitch, k, nc * k, ctx->stream));
    } else {
      HIPC(ctx->stage.d2h(hostp, hdr + nc * ostride, ctx->elim_out.p, hdr + nc * ostride,
                          hdr + nc * ostride, 1, ctx->stream));
    }
#ifdef KODR_ELIM_TIMING
    if (const char* dump = kodr_amd::tune_env("KODR_ELIM_DUMP")) {  // tuning build: the kernel's stamps
      if (FILE* fp = fopen(dump, "wb")) {
        if (direct)
          fwrite(ctx->elim_pin, 1, hdr + nc * k * k, fp);
        else
          fwrite(hostp, 1, hdr + nc * ostride, fp);
        fclose(fp);
      }
      for (size_t i = 0; i < nc; i++) memset(hostp + i * sizeof(int), 0, sizeof(int));
      for (size_t i = 0; i < nc; i++) cntv[i] = 0;  // the stamps overwrote T: kodr's route on the host
    }
#endif
    if (timing) tt3 = tnow();
    if (!direct) elim_counts(a, nc, mc, hostp, cntv.data());
    const int* cnt = cntv.data();
    // the states into the decoders' host mirrors: independent per decoder,
    // memory-bound (a 256 x 520-byte arena each), so spread over host threads.
    // got[i] = rows of the batch accepted
    std::vector<size_t> got(nc);
    const double tl0 = timing ? tnow() : 0;
    HostPool::get().run(nc, [&](size_t i) {
      rlnc_decoder* d = ds[gpu[c0 + i]];
      const size_t r = base[gpu[c0 + i]];
      if (pre_fail[gpu[c0 + i]]) {  // its rows were not prepared: the state stays as it was
        got[i] = 0;
        return;
      }
      size_t c = (size_t)std::max(cnt[i], 0);
      bool ok = false;
      if (c == k && cont)
        ok = tonly ? d->core.load_continued(tstates + i * k * k, k, true)
                   : d->core.load_continued(tstates + i * ostride, opitch, false);
      else if (c && !cont)
        ok = tonly ? c == k && d->core.load_inverse(tstates + i * k * k, k)
                   : d->core.load_rref(tstates + i * ostride, opitch, c);
      got[i] = ok ? c - r : 0;
      if (ok && c == k)
        count_elim(d, attv[i] ? kElimGpuRetried : kElimGpu);
      else
        count_elim(d, kElimHostAfterGpu);
      const bool on_dev = ok && c == k && !cont && a.out_dev;
      d->tdev = on_dev ? a.out_dev + i * k * k : nullptr;
      d->tdev_seq = on_dev ? ctx->tdev_seq : 0;
    });
    if (timing) fprintf(stderr, "add_pieces_gpu: states loaded %.1f us (%zu decoders)\n", tnow() - tl0, nc);
    for (size_t i = 0; i < nc; i++) {
      const size_t g = gpu[c0 + i];
      rlnc_decoder* d = ds[g];
      const size_t c = got[i];
      if (pre_fail[g]) continue;  // status[g] holds its error, consumed[g] = 0
      // the rest of the batch (past a row off its diagonal, or past k) through
      // kodr's algorithm on the host, from the state the GPU left
      int st = RLNC_OK;
      size_t n = c;
      const double tp0 = timing ? tnow() : 0;
      if (early[i].valid()) {  // started on the host while the launch ran (got[i] = 0)
        const auto res = early[i].get();
        st = res.first;
        n = res.second;
      } else if (c < counts[g]) {
        if (d->core.is_decoded()) {
          st = RLNC_ERR_ALL_USEFUL_PIECES_RECEIVED;  // full/decoder.go:52-54
        } else {
          const size_t rest = counts[g] - c;
          // the vectors of a batch the GPU left (downloaded beside the launch)
          const double tf0 = timing ? tnow() : 0;
          TRY(fetch_vecs());
          HIPC(hipEventSynchronize(ctx->vec_ready));
          const double tf1 = timing ? tnow() : 0;
          size_t m = 0;
          st = d->core.add_many(ctx->vec_pin + voff[i] + c * k, k, rest, &m);
          n += m;
          if (timing)
            fprintf(stderr, "add_pieces_gpu: decoder %zu on the host from row %zu: vectors %.1f us, solve %.1f\n", g,
                    c, tf1 - tf0, tnow() - tf1);
        }
      }
      const double tp1 = timing ? tnow() : 0;
      int pst = dec_batch_post(d, rows[g], pitch, true, bcs[g], n);
      if (timing && tnow() - tp0 > 1000)
        fprintf(stderr, "add_pieces_gpu: decoder %zu post: host route %.1f us, batch post %.1f\n", g, tp1 - tp0,
                tnow() - tp1);
      if (pst == RLNC_OK && n && d->policy == RLNC_DECODE_EAGER) pst = dec_progress(d, -1);
      consumed[g] = n;
      status[g] = pst != RLNC_OK ? pst : st;
    }
    c0 += nc;
  }
  if (timing)
    fprintf(stderr, "add_pieces_gpu G=%zu side=%d: pre+copies %.1f us, elim launch %.1f, wait+read-back %.1f, "
            "host post %.1f\n", G, (int)side, tt1 - tt0, tt2 - tt1, tt3 - tt2, tnow() - tt3);
  return RLNC_OK;
}

int rlnc_decoder_add_pieces_gpu(rlnc_decoder* d, const uint8_t* rows, size_t count, size_t pitch,
                                size_t piece_len, size_t* consumed) {
  if (!d || !rows || !consumed) return RLNC_ERR_INVALID_ARGUMENT;
  *consumed = 0;
  if (!count) return RLNC_OK;
  int st = RLNC_OK;
  TRY(rlnc_decoders_add_pieces_gpu(&d, 1, &rows, &count, pitch, piece_len, consumed, &st));
  return st;
}

}  // extern "C"
namespace {
// The lazy AddPiece queues of G decoders (one context, one piece_count)
// through the GPU elimination: every decoder whose queued vectors complete
// its rank from a state of kept rows (fresh or continued) in one launch per
// elim_chunk decoders, from M = [its r coefficient rows ; the queued vectors]
// (one upload); a singular M, and the decoders that do not qualify, keep
// their queues (the host flush takes them).  before_read runs after the
// launch and before the results are read (the grouped flush joins its gather
// there).
template <class F>
int dec_elim_queues_gpu(rlnc_decoder* const* ds, size_t G, F before_read) {
  rlnc_ctx* ctx = ds[0]->ctx;
  const size_t k = ds[0]->core.piece_count();
  TRY(set_dev(ctx));
  auto join = before_read;
  std::vector<size_t> el;
  for (size_t g = 0; g < G; g++) {
    const rlnc_decoder* d = ds[g];
    const size_t r = d->core.received();
    if (k >= 2 && k <= 256 && d->npend >= 2 && d->core.rank() == r && r + d->npend >= k) el.push_back(g);
  }
  if (!el.empty()) {
    TRY(ctx_elim_tables(ctx));
    const size_t opitch = k <= 128 ? 256 : 512, ostride = k * opitch, hdr = kElimHdr;
    const size_t chunk = elim_chunk(k, el.size());
    ctx->elim_out.bind(ctx->device, ctx->stream);
    TRY(ctx->elim_out.reserve(hdr + chunk * ostride));
    ctx->elim_in.bind(ctx->device, ctx->stream);
    TRY(ctx->elim_in.reserve(chunk * k * k));
    if (ctx->elim_host.size() < hdr + chunk * ostride) ctx->elim_host.resize(hdr + chunk * ostride);
    uint8_t* const hostp = ctx->elim_host.data();
    std::vector<uint8_t>& hm = ctx->elim_hin;  // grown once per context, never zero-filled again
    if (hm.size() < chunk * k * k) hm.resize(chunk * k * k);
    for (size_t c0 = 0; c0 < el.size(); c0 += chunk) {
      const size_t nc = std::min(chunk, el.size() - c0);
      kodr_amd::ElimArgs a = {};
      HostPool::get().run(nc, [&](size_t i) {  // M: coefficient rows in row order, then the queue
        const rlnc_decoder* d = ds[el[c0 + i]];
        const size_t r = d->core.received();
        uint8_t* m = hm.data() + i * k * k;
        for (size_t j = 0; j < r; j++) memcpy(m + j * k, d->core.coeff_row(j), k);
        memcpy(m + r * k, d->pend_v.data(), (k - r) * k);
      });
      for (size_t i = 0; i < nc; i++) {
        a.vecs[i] = ctx->elim_in.p + i * k * k;
        a.n[i] = (int)k;
      }
      HIPC(ctx->stage.h2d(ctx->elim_in.p, k, hm.data(), k, k, nc * k, ctx->stream));
      a.vpitch = k;
      a.tables = reinterpret_cast<const uint32_t*>(ctx->elim_tab.p);
      a.out = ctx->elim_out.p + hdr;
      a.out_gen_stride = ostride;
      a.out_pitch = opitch;
      a.counts = reinterpret_cast<int*>(ctx->elim_out.p);
      a.k = (int)k;
      TRY(ctx_elim_mc(ctx, k, nc, &a));
      const bool mc = kodr_amd::gf_elim_mc_taken(a, (int)nc);
      const bool direct = kodr_amd::gf_elim_mc_direct(a, (int)nc);
      if (direct) {
        TRY(ctx_elim_pin(ctx, hdr + nc * k * k));
        a.direct = 1;
        a.out = ctx->elim_pin_dev + hdr;
        a.out_pitch = k;
        a.out_gen_stride = k * k;
        a.counts = reinterpret_cast<int*>(ctx->elim_pin_dev);
      }
      if (direct) {
        TRY(ctx_side(ctx));
        HIPC(hipEventRecord(ctx->elim_ready, ctx->stream));
      }
      HIPC(kodr_amd::gf_elim(a, (int)nc, ctx->stream));
      TRY(join());
      const bool tonly = kodr_amd::gf_elim_blocked(a, (int)nc);
      std::vector<int> cntv(nc), attv(nc, 0);
      const uint8_t* tstates = hostp + hdr;
      if (direct) {
        TRY(elim_direct_wait(ctx, a, nc, cntv.data(), attv.data(), nullptr, ctx->elim_ready));
        tstates = ctx->elim_pin + hdr;
      } else {
        HIPC(ctx->stage.d2h(hostp, hdr, ctx->elim_out.p, hdr, hdr, 1, ctx->stream));
        if (tonly)
          HIPC(ctx->stage.d2h(hostp + hdr, k, ctx->elim_out.p + hdr + k, opitch, k, nc * k, ctx->stream));
        else
          HIPC(ctx->stage.d2h(hostp + hdr, nc * ostride, ctx->elim_out.p + hdr, nc * ostride, nc * ostride, 1,
                              ctx->stream));
        elim_counts(a, nc, mc, hostp, cntv.data());
      }
      const int* cnt = cntv.data();
      HostPool::get().run(nc, [&](size_t i) {
        rlnc_decoder* d = ds[el[c0 + i]];
        bool ok = false;
        if (cnt[i] == (int)k) {
          const uint8_t* st = tonly ? tstates + i * k * k : tstates + i * ostride;
          const size_t sp = tonly ? k : opitch;
          ok = d->core.received() == 0 ? (tonly ? d->core.load_inverse(st, sp) : d->core.load_rref(st, sp, k))
                                       : d->core.load_continued(st, sp, tonly);
        }
        if (ok) {
          d->npend = 0;
          count_elim(d, attv[i] ? kElimGpuRetried : kElimGpu);
        } else {  // M singular: the host flush takes the queue, without a second launch
          d->gpu_rejected = true;
          count_elim(d, kElimHostAfterGpu);
        }
      });
    }
  }
  return RLNC_OK;
}

}  // namespace
extern "C" {

// The lazy queues of G decoders (one AddPiece call per piece) eliminated
// together: every decoder whose queued vectors complete its rank from a
// state of kept rows -- fresh (r = 0) or continued -- in one GPU launch per
// kElimMaxGens, from M = [its r coefficient rows ; the queued vectors], all on
// the host already (one upload); the others, and any singular M, through
// the host flush their next state read would run.  Every decoder's borrowed
// device pieces are gathered by one launch beside the elimination.  Same
// state as G host flushes.
int rlnc_decoders_flush_gpu(rlnc_decoder* const* ds, size_t G) {
  if (!ds || !G || !ds[0]) return RLNC_ERR_INVALID_ARGUMENT;
  rlnc_ctx* ctx = ds[0]->ctx;
  if (!ctx) return RLNC_ERR_NO_DEVICE;
  const size_t k = ds[0]->core.piece_count();
  for (size_t g = 0; g < G; g++)
    if (!ds[g] || ds[g]->ctx != ctx || ds[g]->core.piece_count() != k) return RLNC_ERR_INVALID_ARGUMENT;
  {  // each decoder once: their host mirrors are loaded concurrently below
    std::vector<const rlnc_decoder*> u(ds, ds + G);
    std::sort(u.begin(), u.end());
    if (std::adjacent_find(u.begin(), u.end()) != u.end()) return RLNC_ERR_INVALID_ARGUMENT;
  }
  TRY(set_dev(ctx));
  // the borrowed device pieces of every decoder (of the first one's piece
  // length) in ONE gather launch from uploaded source / destination tables,
  // on the side stream beside the elimination
  std::vector<const void*> gsrc, gdst;
  std::vector<rlnc_decoder*> gdec;
  size_t gL = 0;
  for (size_t g = 0; g < G; g++) {
    rlnc_decoder* d = ds[g];
    if (d->pend_src.empty()) continue;
    if (!gL) gL = d->L;
    if (d->L != gL) continue;  // dec_flush below
    TRY(dec_reserve_rows(d, d->pend_row0 + d->pend_src.size(), d->pend_row0));
    gdec.push_back(d);
  }
  // every receive buffer is in place: the queues move into the tables
  for (rlnc_decoder* d : gdec) {
    for (size_t j = 0; j < d->pend_src.size(); j++) {
      gsrc.push_back(d->pend_src[j]);
      gdst.push_back(d->recv.p + (d->pend_row0 + j) * d->pitch);
    }
    d->pend_src.clear();
  }
  bool gjoined = true;
  // an error return joins too: the context stream must not run past a gather
  // that still reads gtab and writes receive rows
  auto join_guard = on_scope_exit([&] {
    if (!gjoined) (void)hipStreamWaitEvent(ctx->stream, ctx->side_done, 0);
  });
  if (!gsrc.empty()) {
    const size_t nr = gsrc.size();
    std::vector<const void*> tab(gsrc);
    tab.insert(tab.end(), gdst.begin(), gdst.end());
    ctx->gtab.bind(ctx->device, ctx->stream);
    TRY(ctx->gtab.reserve(tab.size() * sizeof(void*)));
    const size_t tb = tab.size() * sizeof(void*);
    HIPC(ctx->stage.h2d(ctx->gtab.p, tb, reinterpret_cast<const uint8_t*>(tab.data()), tb, tb, 1, ctx->stream));
    hipStream_t gs = ctx->stream;
    if (add_copy_mode() != 0) {  // (the flush's gathers stay beside its elimination)
      TRY(ctx_side(ctx));
      HIPC(hipEventRecord(ctx->side_done, ctx->stream));  // the tables and any grown receive buffers first
      HIPC(hipStreamWaitEvent(ctx->side, ctx->side_done, 0));
      gs = ctx->side;
      gjoined = false;
    }
    const auto* src = reinterpret_cast<const uint8_t* const*>(ctx->gtab.p);
    const auto* dst = reinterpret_cast<uint8_t* const*>(ctx->gtab.p + nr * sizeof(void*));
    for (size_t r0 = 0; r0 < nr; r0 += 65535)
      HIPC(kodr_amd::gather_rows(src + r0, nullptr, 0, std::min<size_t>(65535, nr - r0), gL, gs, dst + r0));
    if (!gjoined) HIPC(hipEventRecord(ctx->side_done, ctx->side));
  }
  auto join = [&]() -> int {  // everything after this point on the context stream sees the gathered rows
    if (!gjoined) HIPC(hipStreamWaitEvent(ctx->stream, ctx->side_done, 0));
    gjoined = true;
    return RLNC_OK;
  };
  TRY(dec_elim_queues_gpu(ds, G, join));
  TRY(join());
  for (size_t g = 0; g < G; g++) TRY(dec_flush(ds[g]));
  return RLNC_OK;
}

// The accessors observe kodr's state: queued AddPiece calls are eliminated
// first (a host-only batch; the handle's observable state does not change).
}  // extern "C"
namespace {
const DecoderCore& dec_state(const rlnc_decoder* d) {
  dec_flush_coef(const_cast<rlnc_decoder*>(d));
  return d->core;
}
}  // namespace
extern "C" {
int rlnc_decoder_is_decoded(const rlnc_decoder* d) { return d && dec_state(d).is_decoded(); }
size_t rlnc_decoder_required(const rlnc_decoder* d) { return d ? dec_state(d).required() : 0; }
size_t rlnc_decoder_useful(const rlnc_decoder* d) { return d ? dec_state(d).useful() : 0; }
size_t rlnc_decoder_received(const rlnc_decoder* d) { return d ? d->core.received() + d->npend : 0; }
size_t rlnc_decoder_piece_length(const rlnc_decoder* d) {
  return (d && d->core.received() + d->npend > 0) ? d->L : 0;  // full/decoder.go:18-25
}
size_t rlnc_decoder_piece_count(const rlnc_decoder* d) { return d ? d->core.piece_count() : 0; }

int rlnc_decoder_get_piece(rlnc_decoder* d, size_t idx, uint8_t* out) {
  if (!d) return RLNC_ERR_INVALID_ARGUMENT;
  TRY(dec_flush(d));
  TRY(d->core.piece_available(idx));  // decoder_state.go:222-256
  if (!out) return RLNC_ERR_INVALID_ARGUMENT;
  if (!d->ctx) return RLNC_ERR_NO_DEVICE;
  TRY(set_dev(d->ctx));
  if (d->core.rank() >= d->core.piece_count()) {
    TRY(dec_materialize(d));
    HIPC(d->ctx->stage.d2h(out, d->L, d->decoded.p + idx * d->pitch, d->pitch, d->L, 1, d->ctx->stream));
  } else {
    // partial decode (:233-260): materialise the single row idx
    const size_t recv = d->core.received();
    d->hT.assign(d->core.t_row(idx), d->core.t_row(idx) + recv);
    TRY(d->rowbuf.reserve(d->pitch));
    TRY(dec_apply(d, 1, d->hT.data(), d->rowbuf.p, d->pitch));
    HIPC(d->ctx->stage.d2h(out, d->L, d->rowbuf.p, d->pitch, d->L, 1, d->ctx->stream));
  }
  HIPC(hipStreamSynchronize(d->ctx->stream));
  return RLNC_OK;
}

int rlnc_decoder_get_pieces(rlnc_decoder* d, uint8_t* out) {
  if (!d || !out) return RLNC_ERR_INVALID_ARGUMENT;
  TRY(dec_flush(d));
  if (!d->core.is_decoded()) return RLNC_ERR_MORE_USEFUL_PIECES_REQUIRED;  // full/decoder.go:84-86
  if (!d->ctx) return RLNC_ERR_NO_DEVICE;
  TRY(set_dev(d->ctx));
  const size_t useful = d->core.useful();
  for (size_t i = 0; i < useful; i++) TRY(d->core.piece_available(i));  // :89-96
  TRY(dec_materialize(d));
  HIPC(d->ctx->stage.d2h(out, d->L, d->decoded.p, d->pitch, d->L, useful, d->ctx->stream));
  HIPC(hipStreamSynchronize(d->ctx->stream));
  return RLNC_OK;
}

int rlnc_decoder_get_pieces_device(rlnc_decoder* d, uint8_t* d_out, size_t out_pitch) {
  if (!d || !d_out) return RLNC_ERR_INVALID_ARGUMENT;
  TRY(dec_flush(d));
  if (!d->core.is_decoded()) return RLNC_ERR_MORE_USEFUL_PIECES_REQUIRED;
  if (!d->ctx) return RLNC_ERR_NO_DEVICE;
  if (out_pitch < d->L || out_pitch % 16) return RLNC_ERR_INVALID_ARGUMENT;
  TRY(set_dev(d->ctx));
  const size_t rows = d->core.rank(), recv = d->core.received();
  d->hT.resize(std::max<size_t>(rows * recv, 1));
  d->core.copy_transform(d->hT.data(), recv);
  // T where the GPU elimination left it (k x k on the device, this decoder's
  // batch the last one through the context's buffer): no upload, whose DMA
  // latency (15-20 us) sits in the stream ahead of the product.  Only without
  // unit rows, which the host route copies instead of multiplying.
  if (d->tdev && d->tdev_seq == d->ctx->tdev_seq && rows == recv && recv == d->core.piece_count()) {
    bool unit = false;
    for (size_t r = 0; r < rows && !unit; r++) {
      const uint8_t* t = d->hT.data() + r * recv;
      size_t nz = 0, last = 0;
      for (size_t j = 0; j < recv && nz < 2; j++)
        if (t[j]) nz++, last = j;
      unit = nz == 1 && t[last] == 1;
    }
    if (!unit) {
      d->last_gf_rows = rows;
      d->last_copy_rows = 0;
      return dec_gemm(d, d->tdev, rows, d_out, out_pitch);
    }
  }
  return dec_apply(d, rows, d->hT.data(), d_out, out_pitch);  // T is staged; no host buffer outlives the call
}

// GetPieces of G decoded generations, kGroupGetChunk decoders per launch:
// when a chunk's transforms are all coded-only (no unit row), the received
// counts agree and the product takes the bit-sliced kernel, the chunk's T
// are staged in one upload and applied by ONE gf_bs_kernel launch (grid row =
// decoder); otherwise that chunk goes decoder by decoder.  Launches are
// asynchronous, so the host's T preparation for chunk c + 1 overlaps chunk
// c's kernel; the T upload itself sits in the stream between launches
// (~25 us per chunk, profiles/r02/group_get/), hence chunks of 16.
constexpr size_t kGroupGetChunk = 16;

int rlnc_decoders_get_pieces_device(rlnc_decoder* const* ds, size_t G, uint8_t* d_out, size_t out_pitch) {
  if (!ds || !G || !d_out || !ds[0]) return RLNC_ERR_INVALID_ARGUMENT;
  static const int timing = getenv("KODR_ADD_TIMING") ? atoi(getenv("KODR_ADD_TIMING")) : 0;
  const auto tnow = [] { return std::chrono::duration<double, std::micro>(
                             std::chrono::steady_clock::now().time_since_epoch()).count(); };
  double tg[6] = {timing ? tnow() : 0, 0, 0, 0, 0, 0};
  rlnc_decoder* d0 = ds[0];
  for (size_t g = 0; g < G; g++)
    if (!ds[g]) return RLNC_ERR_INVALID_ARGUMENT;
  for (size_t g = 0; g < G; g++) TRY(dec_flush(ds[g]));
  if (timing) tg[1] = tnow();
  for (size_t g = 0; g < G; g++)  // full/decoder.go:84-86 for any of them before anything else
    if (!ds[g]->core.is_decoded()) return RLNC_ERR_MORE_USEFUL_PIECES_REQUIRED;
  for (size_t g = 0; g < G; g++) {
    rlnc_decoder* d = ds[g];
    if (!d->ctx) return RLNC_ERR_NO_DEVICE;
    if (d->ctx != d0->ctx || d->L != d0->L || d->core.piece_count() != d0->core.piece_count())
      return RLNC_ERR_INVALID_ARGUMENT;
  }
  const size_t L = d0->L, rows = d0->core.rank(), pitch = d0->pitch;
  // decoders that received different numbers of rows (a dependent piece
  // counts) share one launch over the largest: T padded with zero columns,
  // whose twin rows are never read arithmetically (coefficient 0)
  size_t recv = 0;
  for (size_t g = 0; g < G; g++) recv = std::max(recv, ds[g]->core.received());
  if (out_pitch < L || out_pitch % 16) return RLNC_ERR_INVALID_ARGUMENT;
  TRY(set_dev(d0->ctx));
  rlnc_ctx* ctx = d0->ctx;
  const size_t ostride = rows * out_pitch, tsz = rows * recv;
  const bool bs = G > 1 && rows >= kBsMinRows && !few_narrow_rows(rows, recv, L) && (pitch % 32) == 0 &&
                  bs_chunk_rows(rows, std::max<size_t>(recv, 1), pitch, L) >= recv && kodr_amd::bs_ready(ctx->device);
  if (!bs) {
    if (timing)
      fprintf(stderr, "get_pieces grouped G=%zu: per decoder (rows %zu, recv %zu, pitch %zu, chunk rows %zu)\n", G,
              rows, recv, pitch, bs_chunk_rows(rows, std::max<size_t>(recv, 1), pitch, L));
    for (size_t g = 0; g < G; g++) TRY(rlnc_decoder_get_pieces_device(ds[g], d_out + g * ostride, out_pitch));
    return RLNC_OK;
  }
  // transforms staged per chunk into two context buffers used in turn
  // (stream-ordered: chunk c's upload follows chunk c - 2's launch)
  for (DevBuf& b : ctx->gtmat) {
    b.bind(ctx->device, ctx->stream);
    TRY(b.reserve(std::min(G, kGroupGetChunk) * tsz));
  }
  std::vector<uint8_t> hT(kGroupGetChunk * tsz);
  const uint8_t* xs[kGroupGetChunk];
  for (size_t g0 = 0; g0 < G; g0 += kGroupGetChunk) {
    const size_t n = std::min(kGroupGetChunk, G - g0);
    bool grouped = n > 1;
    for (size_t i = 0; i < n && grouped; i++) {
      const rlnc_decoder* d = ds[g0 + i];
      grouped = d->core.rank() == rows && d->pitch == pitch && d->recv_rows >= recv;
    }
    // every T of the chunk where the GPU elimination left it, consecutive
    // (the decoders of one batched GPU AddPiece, in its order): no host
    // transform and no upload
    bool dev_t = grouped && recv == d0->core.piece_count();
    for (size_t i = 0; i < n && dev_t; i++) {
      const rlnc_decoder* d = ds[g0 + i];
      dev_t = d->tdev && d->tdev_seq == ctx->tdev_seq && d->core.received() == recv &&
              d->tdev == ds[g0]->tdev + i * tsz;
    }
    if (dev_t) {
      for (size_t i = 0; i < n; i++) {
        rlnc_decoder* d = ds[g0 + i];
        TRY(dec_extend_twin(d));
        d->last_gf_rows = rows;
        d->last_copy_rows = 0;
        d->last_bs = true;
        xs[i] = d->recv_bs.p;
      }
      const kodr_amd::GemmGroupArgs grp{(int)n, xs, tsz, ostride};
      HIPC(kodr_amd::gf_gemm_bs(ds[g0]->tdev, recv, rows, recv, xs[0], pitch, d_out + g0 * ostride, out_pitch, L,
                                ctx->device, ctx->stream, false, &grp));
      if (timing) fprintf(stderr, "get_pieces grouped: chunk %zu (%zu) T on the device %.1f us\n", g0, n, tnow() - tg[1]);
      continue;
    }
    // the transforms, one decoder per host task (disjoint slices of hT)
    std::vector<uint8_t> unit(n, 0);
    if (grouped)
      HostPool::get().run(n, [&](size_t i) {
        uint8_t* t = hT.data() + i * tsz;
        const size_t ri = ds[g0 + i]->core.received();
        ds[g0 + i]->core.copy_transform(t, recv);
        if (ri < recv)
          for (size_t r = 0; r < rows; r++) memset(t + r * recv + ri, 0, recv - ri);
        for (size_t r = 0; r < rows && !unit[i]; r++, t += recv) {  // a unit row is a copy: per-decoder route
          size_t nz = 0, last = 0;
          for (size_t j = 0; j < recv && nz < 2; j++)
            if (t[j]) nz++, last = j;
          unit[i] = nz == 1 && t[last] == 1;
        }
      });
    if (timing) tg[2] = tnow();
    for (size_t i = 0; i < n && grouped; i++) grouped = !unit[i];
    if (!grouped) {
      for (size_t i = 0; i < n; i++)
        TRY(rlnc_decoder_get_pieces_device(ds[g0 + i], d_out + (g0 + i) * ostride, out_pitch));
      continue;
    }
    for (size_t i = 0; i < n; i++) {
      rlnc_decoder* d = ds[g0 + i];
      TRY(dec_extend_twin(d));
      d->last_gf_rows = rows;
      d->last_copy_rows = 0;
      d->last_bs = true;
      xs[i] = d->recv_bs.p;
    }
    uint8_t* dT = ctx->gtmat[(g0 / kGroupGetChunk) & 1].p;
    if (timing) tg[3] = tnow();
    HIPC(ctx->stage.h2d(dT, n * tsz, hT.data(), n * tsz, n * tsz, 1, ctx->stream));
    if (timing) tg[4] = tnow();
    const kodr_amd::GemmGroupArgs grp{(int)n, xs, tsz, ostride};
    HIPC(kodr_amd::gf_gemm_bs(dT, recv, rows, recv, xs[0], pitch, d_out + g0 * ostride, out_pitch, L, ctx->device,
                              ctx->stream, false, &grp));
  }
  if (timing)
    fprintf(stderr, "get_pieces grouped G=%zu: flush %.1f us, checks+transforms %.1f, twins %.1f, T upload %.1f, "
            "launch %.1f\n", G, tg[1] - tg[0], tg[2] - tg[1], tg[3] - tg[2], tg[4] - tg[3], tnow() - tg[4]);
  return RLNC_OK;
}

int rlnc_decoder_apply_stats(const rlnc_decoder* d, size_t* gf_rows, size_t* copy_rows) {
  if (!d || !gf_rows || !copy_rows) return RLNC_ERR_INVALID_ARGUMENT;
  *gf_rows = d->last_gf_rows;
  *copy_rows = d->last_copy_rows;
  return RLNC_OK;
}

int rlnc_decoder_last_apply_bitsliced(const rlnc_decoder* d) { return d && d->last_bs ? 1 : 0; }

int rlnc_decoder_elim_stats(const rlnc_decoder* d, size_t* gpu, size_t* gpu_retried, size_t* host_after_gpu,
                            size_t* host) {
  if (!d) return RLNC_ERR_INVALID_ARGUMENT;
  if (gpu) *gpu = d->elim_gpu;
  if (gpu_retried) *gpu_retried = d->elim_gpu_retried;
  if (host_after_gpu) *host_after_gpu = d->elim_host_after_gpu;
  if (host) *host = d->elim_host;
  return RLNC_OK;
}

int rlnc_decoder_coefficients(const rlnc_decoder* d, uint8_t* out) {
  if (!d || !out) return RLNC_ERR_INVALID_ARGUMENT;
  dec_state(d).copy_coefficients(out);
  return RLNC_OK;
}

int rlnc_decoder_transform(const rlnc_decoder* d, uint8_t* out) {
  if (!d || !out) return RLNC_ERR_INVALID_ARGUMENT;
  dec_state(d).copy_transform(out, d->core.received());
  return RLNC_OK;
}

int rlnc_decoder_bind_output(rlnc_decoder* d, uint8_t* d_out, size_t pitch) {
  if (!d) return RLNC_ERR_INVALID_ARGUMENT;
  TRY(dec_flush(d));
  if (d_out && (!d->ctx || !d->have_len || pitch < d->L || pitch % 16 || (uintptr_t)d_out % 16))
    return RLNC_ERR_INVALID_ARGUMENT;
  d->out_ext = d_out;
  d->out_pitch = d_out ? pitch : 0;
  d->slot_of.assign(d->core.piece_count(), -1);  // slots made so far are dropped
  d->nslots = 0;
  if (d_out && d->policy == RLNC_DECODE_EAGER) {
    TRY(set_dev(d->ctx));
    TRY(dec_progress(d, -1));  // what is decoded already
  }
  return RLNC_OK;
}

int rlnc_decoder_set_policy(rlnc_decoder* d, int policy) {
  if (!d || (policy != RLNC_DECODE_LAZY && policy != RLNC_DECODE_EAGER)) return RLNC_ERR_INVALID_ARGUMENT;
  TRY(dec_flush(d));
  d->policy = policy;
  if (policy == RLNC_DECODE_EAGER && d->ctx && d->have_len) {
    TRY(set_dev(d->ctx));
    TRY(dec_progress(d, -1));  // what is decoded already
  }
  return RLNC_OK;
}

size_t rlnc_decoder_decoded_mask(const rlnc_decoder* d, uint8_t* mask) {
  if (!d) return 0;
  std::vector<int32_t> row;
  std::vector<uint8_t> sc;
  const size_t n = dec_state(d).decoded(&row, &sc);
  if (mask)
    for (size_t j = 0; j < row.size(); j++) mask[j] = row[j] >= 0 ? 1 : 0;
  return n;
}

int rlnc_decoder_get_decoded(rlnc_decoder* d, size_t j, uint8_t* out, int is_device) {
  if (!d || !out) return RLNC_ERR_INVALID_ARGUMENT;
  TRY(dec_flush(d));
  if (j >= d->core.piece_count()) return RLNC_ERR_PIECE_OUT_OF_BOUND;
  std::vector<int32_t> row;
  std::vector<uint8_t> sc;
  d->core.decoded(&row, &sc);
  if (row[j] < 0) return RLNC_ERR_PIECE_NOT_DECODED_YET;
  if (!d->ctx) return RLNC_ERR_NO_DEVICE;
  TRY(set_dev(d->ctx));
  hipStream_t st = d->ctx->stream;
  const uint8_t* src = nullptr;
  auto slot = [d](size_t j) -> const uint8_t* {
    return d->out_ext ? d->out_ext + j * d->out_pitch : d->prog.p + (size_t)d->slot_of[j] * d->pitch;
  };
  if (d->slot_of.size() == d->core.piece_count() && d->slot_of[j] >= 0) {
    src = slot(j);
  } else if (d->decoded_ready && sc[j] == 1 && !d->out_ext) {  // GetPieces' rows: row i of the state is piece j
    src = d->decoded.p + (size_t)row[j] * d->pitch;
  } else {
    TRY(dec_progress(d, (long)j));
    src = slot(j);
  }
  if (is_device) {
    if (out != src) HIPC(hipMemcpyAsync(out, src, d->L, hipMemcpyDeviceToDevice, st));
    return RLNC_OK;
  }
  HIPC(d->ctx->stage.d2h(out, d->L, src, d->pitch, d->L, 1, st));
  HIPC(hipStreamSynchronize(st));
  return RLNC_OK;
}

int rlnc_last_launch_plan(rlnc_launch_plan* out) {
  if (!out) return RLNC_ERR_INVALID_ARGUMENT;
  const kodr_amd::LaunchPlan& p = kodr_amd::last_launch_plan();
  *out = rlnc_launch_plan{p.kernel, p.tile_rows, p.waves, p.lane_groups, p.ring, p.rows_per_wave, p.generations,
                          p.workgroups};
  return RLNC_OK;
}

}  // extern "C"
