/*
 * kodr_rlnc.h -- C ABI of the MI355X-native RLNC engine (libkodr_rlnc.so).
 *
 * This is the drop-in boundary for kodr's full/ and systematic/ packages
 * (reference: itzmeanjan/kodr, paths relative to its checkout).  kodr is pure
 * Go with no FFI layer of its own; each entry point below is what a cgo
 * binding of that package would call in place of the Go method body named
 * next to it (INTEGRATION.md shows the Go side).  All arithmetic is GF(2^8)
 * with kodr's field (poly 0x11D, generator 2; gf256.go:15-44) and every result
 * is bit-identical to kodr's on the same input bytes and coding vectors.
 *
 * Conventions
 *  - Return value: 0 = OK; 1..12 = kodr's sentinel errors in the order of
 *    errors.go:6-17 (RLNC_ERR_*); negative = engine/HIP failures.
 *  - Host pointers are borrowed for the duration of the call only; the engine
 *    copies what it keeps (cgo pointer rule).  Nothing is aliased, unlike
 *    kodr's encoder (data.go:121-128) and decoder (decoder_state.go:205-208).
 *  - "*_device" entry points take device pointers, enqueue on the context's
 *    stream and return without synchronising.  All others are synchronous.
 *  - A handle is not thread-safe (kodr's types are not goroutine-safe either):
 *    one handle per thread.
 *  - Coding vectors are supplied by the caller (kodr draws them from
 *    crypto/rand, data.go:90-95); rlnc_random_bytes() is provided for callers
 *    without an RNG.  The wire layout of a coded piece is vector ++ piece
 *    (CodedPiece.Flatten, data.go:52-57).
 */
#ifndef KODR_RLNC_H
#define KODR_RLNC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes: errors.go:6-17, same order ------------------------- */
#define RLNC_OK                                   0
#define RLNC_ERR_CANNOT_INVERT_GF256_ADD_IDENTITY 1  /* errors.go:6  */
#define RLNC_ERR_MATRIX_DIMENSION_MISMATCH        2  /* errors.go:7  */
#define RLNC_ERR_ALL_USEFUL_PIECES_RECEIVED       3  /* errors.go:8  */
#define RLNC_ERR_MORE_USEFUL_PIECES_REQUIRED      4  /* errors.go:9  */
#define RLNC_ERR_COPY_FAILED_DURING_PIECE_CONSTRUCTION 5 /* errors.go:10 */
#define RLNC_ERR_PIECE_COUNT_MORE_THAN_TOTAL_BYTES 6 /* errors.go:11 */
#define RLNC_ERR_ZERO_PIECE_SIZE                  7  /* errors.go:12 */
#define RLNC_ERR_BAD_PIECE_COUNT                  8  /* errors.go:13 */
#define RLNC_ERR_CODED_DATA_LENGTH_MISMATCH       9  /* errors.go:14 */
#define RLNC_ERR_CODING_VECTOR_LENGTH_MISMATCH    10 /* errors.go:15 */
#define RLNC_ERR_PIECE_NOT_DECODED_YET            11 /* errors.go:16 */
#define RLNC_ERR_PIECE_OUT_OF_BOUND               12 /* errors.go:17 */
/* engine errors (no kodr counterpart) */
#define RLNC_ERR_INVALID_ARGUMENT                 -1
#define RLNC_ERR_OUT_OF_MEMORY                    -2
#define RLNC_ERR_HIP                              -3
#define RLNC_ERR_NO_DEVICE                        -4

typedef struct rlnc_ctx rlnc_ctx;
typedef struct rlnc_encoder rlnc_encoder;
typedef struct rlnc_recoder rlnc_recoder;
typedef struct rlnc_decoder rlnc_decoder;

/* ---- library / context ------------------------------------------------ */
const char* rlnc_version(void);
const char* rlnc_status_string(int status);      /* kodr's error text for 1..12 */
const char* rlnc_last_hip_error(void);           /* detail for RLNC_ERR_HIP (thread-local) */
int rlnc_device_count(int* count);
/* stream: a hipStream_t to enqueue on, or NULL for a stream owned by the ctx */
int rlnc_ctx_create(int device, void* stream, rlnc_ctx** out);
int rlnc_ctx_destroy(rlnc_ctx* ctx);
int rlnc_ctx_synchronize(rlnc_ctx* ctx);
void* rlnc_ctx_stream(rlnc_ctx* ctx);            /* the hipStream_t in use */
/* A single decoder's full batch (rlnc_decoder_add_pieces, the lazy AddPiece
 * flush) takes the GPU elimination from piece count min_k on (default 224,
 * where it measured at least as fast as the host's); a larger value keeps
 * every such batch on the host (kodr's algorithm, the same state). */
int rlnc_ctx_set_route_min_k(rlnc_ctx* ctx, size_t min_k);
/* rlnc_decoder_elim_stats summed over every decoder of the context so far */
int rlnc_ctx_elim_stats(const rlnc_ctx* ctx, size_t* gpu, size_t* gpu_retried, size_t* host_after_gpu,
                        size_t* host);
int rlnc_random_bytes(uint8_t* out, size_t n);   /* getrandom(2): crypto/rand stand-in */

/* The engine's own device buffers (generations, received rows, twins) come
 * from a per-device caching pool: a destroyed encoder/decoder returns them
 * for the next one instead of paying hipFree (~175 us per 32 MiB buffer).
 * Reuse is ordered on the owning streams.  At most KODR_POOL_BYTES (default
 * 8 GiB) stays cached per device; trim releases down to keep_bytes. */
int rlnc_device_pool_trim(int device, size_t keep_bytes);
size_t rlnc_device_pool_cached(int device);

/* device memory helpers (plumbing for device-resident callers and benches) */
int rlnc_dev_alloc(rlnc_ctx* ctx, size_t bytes, void** dptr);
int rlnc_dev_free(rlnc_ctx* ctx, void* dptr);
int rlnc_memcpy_h2d(rlnc_ctx* ctx, void* dst, const void* src, size_t bytes);  /* sync */
int rlnc_memcpy_d2h(rlnc_ctx* ctx, void* dst, const void* src, size_t bytes);  /* sync */
int rlnc_memcpy_d2d_async(rlnc_ctx* ctx, void* dst, const void* src, size_t bytes);
/* page-lock a caller buffer (e.g. a socket/file staging slab):
 * host-pointer entry points then DMA straight from / into it instead of
 * bouncing through the context's pinned chunks.  Unregister before freeing. */
int rlnc_host_register(rlnc_ctx* ctx, void* ptr, size_t bytes);
int rlnc_host_unregister(rlnc_ctx* ctx, void* ptr);
/* stream-ordered timing: record a named mark, read elapsed ms between two */
int rlnc_event_create(rlnc_ctx* ctx, void** ev);
int rlnc_event_record(rlnc_ctx* ctx, void* ev);
int rlnc_event_elapsed_ms(void* ev_start, void* ev_end, float* ms);   /* syncs ev_end */
/* the context's stream waits (on the device, no host wait) for ev, recorded
 * on any context's stream of the same device: e.g. decoders on one context
 * fed the wire rows an encoder on another context produced */
int rlnc_ctx_wait_event(rlnc_ctx* ctx, void* ev);
int rlnc_event_destroy(void* ev);

/* ---- piece splitting: data.go:103-166 (host only) ---------------------- */
/* OriginalPiecesFromDataAndPieceCount (data.go:137-166) */
int rlnc_split_by_piece_count(size_t data_len, size_t piece_count,
                              size_t* piece_size, size_t* padding);
/* OriginalPiecesFromDataAndPieceSize (data.go:103-132) */
int rlnc_split_by_piece_size(size_t data_len, size_t piece_size,
                             size_t* piece_count, size_t* padding);
/* CodedPiecesForRecoding validation (data.go:173-193) */
int rlnc_coded_pieces_for_recoding(size_t data_len, size_t piece_count,
                                   size_t pieces_coded_together, size_t* coded_piece_len);
/* CodedPiece.IsSystematic (data.go:64-84) */
int rlnc_is_systematic(const uint8_t* vector, size_t n);

/* ---- encoders: full/encoder.go, systematic/encoder.go ------------------ */
#define RLNC_FULL        0
#define RLNC_SYSTEMATIC  1
/* NewFullRLNCEncoderWithPieceCount (full/encoder.go:84-93) /
 * NewSystematicRLNCEncoderWithPieceCount (systematic/encoder.go:123-132) */
int rlnc_encoder_create_with_piece_count(rlnc_ctx* ctx, int kind, const uint8_t* data,
                                         size_t data_len, size_t piece_count, rlnc_encoder** out);
/* NewFullRLNCEncoderWithPieceSize (full/encoder.go:98-107) /
 * NewSystematicRLNCEncoderWithPieceSize (systematic/encoder.go:137-146) */
int rlnc_encoder_create_with_piece_size(rlnc_ctx* ctx, int kind, const uint8_t* data,
                                        size_t data_len, size_t piece_size, rlnc_encoder** out);
/* NewFullRLNCEncoder(pieces) (full/encoder.go:76-78) / NewSystematicRLNCEncoder
 * (systematic/encoder.go:115-117): k pieces of L bytes, row-major contiguous.
 * Size: a generation may exceed 4 GiB (products run in row chunks); a single
 * piece (its 256-byte row pitch) must stay below 2 GiB, else
 * RLNC_ERR_INVALID_ARGUMENT.  The same holds for recoders and decoders. */
int rlnc_encoder_create(rlnc_ctx* ctx, int kind, const uint8_t* pieces, size_t piece_count,
                        size_t piece_size, rlnc_encoder** out);
/* the same from a device buffer (k rows, row pitch `pitch` bytes), copied D2D */
int rlnc_encoder_create_device(rlnc_ctx* ctx, int kind, const uint8_t* d_pieces, size_t piece_count,
                               size_t piece_size, size_t pitch, rlnc_encoder** out);
int rlnc_encoder_destroy(rlnc_encoder* enc);
/* accessors: PieceCount/PieceSize/DecodableLen/CodedPieceLen/Padding (full/encoder.go:15-55) */
size_t rlnc_encoder_piece_count(const rlnc_encoder* enc);
size_t rlnc_encoder_piece_size(const rlnc_encoder* enc);
size_t rlnc_encoder_decodable_len(const rlnc_encoder* enc);
size_t rlnc_encoder_coded_piece_len(const rlnc_encoder* enc);
size_t rlnc_encoder_padding(const rlnc_encoder* enc);
/* device pointer of the resident generation (k rows of `pitch` bytes) */
const uint8_t* rlnc_encoder_device_pieces(const rlnc_encoder* enc, size_t* pitch);
/* count calls after which a systematic encoder emits coded pieces (0 for full) */
size_t rlnc_encoder_systematic_remaining(const rlnc_encoder* enc);
/* `count` consecutive CodedPiece() calls (full/encoder.go:61-71,
 * systematic/encoder.go:82-109).  vectors: count x k caller-drawn bytes; a
 * systematic encoder ignores (and overwrites with e_i) the rows it emits
 * systematically.  out: count x (k+L) bytes in wire layout (vector ++ piece). */
int rlnc_encoder_coded_pieces(rlnc_encoder* enc, uint8_t* vectors, size_t count, uint8_t* out);
/* device-resident batch: d_vectors count x k (device), d_out count rows of L
 * bytes at row pitch out_pitch (pieces only; the vectors are the caller's).
 * Full-RLNC semantics (no systematic phase).  Async on the ctx stream. */
int rlnc_encoder_coded_pieces_device(rlnc_encoder* enc, const uint8_t* d_vectors, size_t count,
                                     uint8_t* d_out, size_t out_pitch);
/* device-resident coded pieces in wire layout with the coding vectors drawn
 * on the device (replaces GenerateCodingVector's crypto/rand, data.go:90-95,
 * for large batches): d_wire gets `count` rows of k+L bytes
 * (vector ++ piece, as CodedPiece.Flatten) at pitch wire_pitch >= k+L.
 * Vector bytes are a counter-based pseudo-random stream of the encoder's seed
 * (drawn from getrandom at create; rlnc_encoder_seed resets it), uniform,
 * zeros allowed, not cryptographic.  A systematic encoder still emits e_id ++
 * P_id for its first k pieces (systematic/encoder.go:83-96).  count <= 65535.
 * Async on the ctx stream. */
int rlnc_encoder_coded_wire_device(rlnc_encoder* enc, size_t count, uint8_t* d_wire, size_t wire_pitch);
/* reseed the device vector stream (reproducible batches for tests/benches) */
int rlnc_encoder_seed(rlnc_encoder* enc, uint64_t seed);
/* construction-time preparation (the Go constructors' NewFullRLNCEncoder*,
 * full/encoder.go:76-107, end here): builds the bit-sliced twin that batches
 * of >= 9 coded pieces read, so that cost is paid once up front instead of by
 * the first large batch.  Optional; idempotent.  Async on the ctx stream. */
int rlnc_encoder_prepare(rlnc_encoder* enc);
/* Compact residency (no kodr counterpart): keep only the bit-sliced copy of
 * the generation and release the plain rows -- half the HBM per resident
 * generation.  Every product then runs on the bit-sliced kernel (a batch of
 * fewer than 9 pieces of one generation is slower than on the plain rows:
 * DESIGN.md), systematic pieces are converted back per call,
 * rlnc_encoder_device_pieces returns NULL, and grouped launches take compact
 * generations from 5 pieces per generation (one launch per generation below).
 * Idempotent; synchronizes the ctx stream.  RLNC_ERR_INVALID_ARGUMENT when
 * the bit-sliced path is unavailable for this shape or device. */
int rlnc_encoder_compact(rlnc_encoder* enc);
/* Many generations in one launch: coded pieces for each of n_enc resident
 * generations (full/encoder.go:61-71 once per generation), all encoders on one
 * ctx with equal piece count k and piece size L.  d_vectors: n_enc blocks of
 * count x k bytes (generation i at i*count*k); d_out: n_enc blocks of count
 * rows at out_pitch (generation i's first row at i*count*out_pitch).  Every
 * 32 generations take ONE kernel launch: small batches (the streaming regime,
 * count < 9) on the plain rows, larger ones on the bit-sliced twins (built
 * here if rlnc_encoder_prepare was not called; from 5 pieces when every twin
 * is already resident); shapes neither kernel takes in one row chunk fall
 * back to one launch per generation.
 * Full-RLNC semantics.  Async on the ctx stream. */
int rlnc_encoder_group_coded_pieces_device(rlnc_encoder* const* encs, size_t n_enc, const uint8_t* d_vectors,
                                           size_t count, uint8_t* d_out, size_t out_pitch);

/* Many generations' wire rows in one call: `count` coded pieces of each of
 * n_enc resident generations (one ctx, equal k and L) as rlnc_encoder_coded_wire_device
 * would write them -- generation i's rows at d_wire + i*count*wire_pitch, each
 * `vector ++ piece` (CodedPiece.Flatten, data.go:52-57) with the vector drawn
 * from that encoder's own device stream (data.go:90-95 replaced as in
 * rlnc_encoder_coded_wire_device), and a systematic encoder's first k pieces
 * e_id ++ P_id (systematic/encoder.go:82-109).  When every encoder is at the
 * same point of its systematic phase and k, wire_pitch and d_wire are
 * multiples of 16, ONE vector launch and one product launch per 32
 * generations; otherwise encoder by encoder.  Same bytes and the same
 * per-encoder stream state either way.  count <= 65535.  Async on the ctx
 * stream. */
int rlnc_encoder_group_coded_wire_device(rlnc_encoder* const* encs, size_t n_enc, size_t count, uint8_t* d_wire,
                                         size_t wire_pitch);

/* ---- recoder: full/recoder.go ------------------------------------------ */
/* NewFullRLNCRecoderWithFlattenData (full/recoder.go:63-70): flat holds
 * piece_count coded pieces (wire layout), each pieces_coded_together + L bytes */
int rlnc_recoder_create(rlnc_ctx* ctx, const uint8_t* flat, size_t flat_len, size_t piece_count,
                        size_t pieces_coded_together, rlnc_recoder** out);
/* the same from a device buffer of n wire rows at row pitch `pitch` */
int rlnc_recoder_create_device(rlnc_ctx* ctx, const uint8_t* d_flat, size_t piece_count,
                               size_t coded_piece_len, size_t pitch, size_t pieces_coded_together,
                               rlnc_recoder** out);
int rlnc_recoder_destroy(rlnc_recoder* rec);
/* Many recoders in one launch (no kodr counterpart; full/recoder.go:27-46 once
 * per generation): count recoded pieces of each of n_rec recoders of one ctx
 * with equal piece_count and coded piece length.  d_r: n_rec blocks of
 * count x piece_count recoding vectors (recoder i at i*count*piece_count);
 * d_out: n_rec blocks of count wire rows at out_pitch (recoder i's first row
 * at i*count*out_pitch).  One launch per 32 recoders (gf_gemm on the plain
 * rows below 9 pieces, the bit-sliced kernel on the twins from 9), else one
 * call per recoder; same bytes either way.  Async on the ctx stream. */
int rlnc_recoder_group_coded_pieces_device(rlnc_recoder* const* recs, size_t n_rec, const uint8_t* d_r,
                                           size_t count, uint8_t* d_out, size_t out_pitch);

/* as rlnc_encoder_prepare: build the held rows' bit-sliced twin up front
 * (NewFullRLNCRecoder*, full/recoder.go:52-70).  Optional; async. */
int rlnc_recoder_prepare(rlnc_recoder* rec);
/* as rlnc_encoder_compact, for the held coded pieces */
int rlnc_recoder_compact(rlnc_recoder* rec);
size_t rlnc_recoder_piece_count(const rlnc_recoder* rec);        /* n held coded pieces */
size_t rlnc_recoder_coded_piece_len(const rlnc_recoder* rec);    /* k + L */
/* `count` CodedPiece() calls (full/recoder.go:27-46): r = count x n caller
 * bytes; out = count x (k+L) wire rows [r x C | sum r_i P_i] */
int rlnc_recoder_coded_pieces(rlnc_recoder* rec, const uint8_t* r, size_t count, uint8_t* out);
/* device-resident: d_r count x n (device), d_out count wire rows at out_pitch
 * (any pitch >= k + L; rows that are not 16-byte aligned are computed aside and
 * copied).  From 9 pieces and k a multiple of 16, one bit-sliced launch writes
 * whole wire rows (the coding-vector columns are that launch's side product). */
int rlnc_recoder_coded_pieces_device(rlnc_recoder* rec, const uint8_t* d_r, size_t count,
                                     uint8_t* d_out, size_t out_pitch);

/* ---- decoder: full/decoder.go, systematic/decoder.go, decoder_state.go -- */
/* NewFullRLNCDecoder (full/decoder.go:109-112) == NewSystematicRLNCDecoder
 * (systematic/decoder.go:105-108).  ctx may be NULL: coefficient-side only
 * (counters, rank, transform; no piece data), used by host-logic tests. */
int rlnc_decoder_create(rlnc_ctx* ctx, size_t piece_count, rlnc_decoder** out);
/* Does not wait for the context stream: the decoder's device buffers go back
 * to the context's pool ordered behind its pending work there (device rows a
 * caller passed in are still read in stream order: keep them until the
 * stream passes, e.g. rlnc_ctx_synchronize). */
int rlnc_decoder_destroy(rlnc_decoder* dec);
/* AddPiece (full/decoder.go:50-66): returns RLNC_ERR_ALL_USEFUL_PIECES_RECEIVED
 * once decoded.  vector: piece_count bytes; piece: L bytes (L fixed by the
 * first piece; a different length is RLNC_ERR_INVALID_ARGUMENT). */
int rlnc_decoder_add_piece(rlnc_decoder* dec, const uint8_t* vector, size_t vector_len,
                           const uint8_t* piece, size_t piece_len);
/* same, with the piece bytes already on the device: the piece is copied D2D
 * on the context stream in the call (async), so the caller may reuse d_piece
 * for work queued on that stream after this call.
 * Lazy elimination (every AddPiece entry point): while the queued rows cannot
 * complete the rank (useful + queued < piece_count) AddPiece only queues the
 * coding vector; the queue goes through kodr's elimination as one batch when
 * any accessor (is_decoded, required, useful, coefficients, GetPiece...) or a
 * later AddPiece needs the state.  Every return code and every value an
 * accessor returns is exactly kodr's after the same calls. */
int rlnc_decoder_add_piece_device(rlnc_decoder* dec, const uint8_t* vector, size_t vector_len,
                                  const uint8_t* d_piece, size_t piece_len);
/* same, BORROWING the piece (opt-in; no kodr counterpart beyond kodr keeping
 * the caller's CodedPiece for good, decoder_state.go:205-208): under the LAZY
 * policy a 16-byte aligned d_piece is not copied in the call; the decoder
 * reads it on the context stream at its next data flush -- the next GetPiece/
 * GetPieces/get_decoded/bind_output/set_policy/batched AddPiece/
 * rlnc_decoders_flush_gpu call, or once 1024 pieces are queued -- so the
 * caller keeps those bytes unchanged until then.  Many pieces then cost one
 * gather launch instead of a copy each.  Unaligned pieces, and every piece
 * under EAGER, are copied in the call as above. */
int rlnc_decoder_add_piece_device_borrowed(rlnc_decoder* dec, const uint8_t* vector, size_t vector_len,
                                           const uint8_t* d_piece, size_t piece_len);
/* batch AddPiece over `count` wire rows (vector ++ piece, as CodedPiece.Flatten,
 * kodr_internals/coded.go) at row pitch `pitch` >= piece_count + piece_len,
 * on the host or the device (is_device).  piece_len follows AddPiece's rule
 * (fixed by the first piece).  Same result as calling AddPiece row by row:
 * stops at the first error (RLNC_ERR_ALL_USEFUL_PIECES_RECEIVED once decoded)
 * with *consumed = pieces accepted.  The accepted pieces are stored with ONE
 * strided copy (host rows staged through pinned memory; device rows D2D,
 * async, only the coding vectors are read back). */
int rlnc_decoder_add_pieces(rlnc_decoder* dec, const uint8_t* rows, size_t count, size_t pitch,
                            size_t piece_len, int is_device, size_t* consumed);
/* The same batch AddPiece over DEVICE wire rows, with the elimination
 * (decoder_state.go:15-182) on the GPU: one workgroup runs kodr's pivots for
 * the rows that land on their diagonals (gf_elim.hip); the rest of the batch,
 * if any, continues on the host from the state it left.  Same state, return
 * code and *consumed as rlnc_decoder_add_pieces (is_device = 1).  Used for
 * batches of >= 2 rows with 2 <= piece_count <= 256 on a fresh decoder, or
 * on one whose received pieces were all kept (none dependent) when the batch
 * can complete the rank or the held rows are diagonal pivots (the GPU then
 * eliminates [held coefficient rows ; batch vectors] and the host maps the
 * transform back to arrival order); otherwise it IS rlnc_decoder_add_pieces. */
int rlnc_decoder_add_pieces_gpu(rlnc_decoder* dec, const uint8_t* d_rows, size_t count, size_t pitch,
                                size_t piece_len, size_t* consumed);
/* G decoders of one context and one piece_count at once: one GPU launch
 * eliminates every eligible decoder's batch (a workgroup each), so G
 * generations cost about one.  d_rows[g], counts[g]: decoder g's batch;
 * per-decoder results in consumed[g] and status[g] (what
 * rlnc_decoder_add_pieces_gpu would return).  The call itself fails only on
 * bad arguments (including a decoder listed twice) or device errors. */
int rlnc_decoders_add_pieces_gpu(rlnc_decoder* const* decs, size_t G, const uint8_t* const* d_rows,
                                 const size_t* counts, size_t pitch, size_t piece_len, size_t* consumed,
                                 int* status);
/* The same, calling after_launch(user) once from inside the call after the
 * first elimination launch is queued and the work queued ahead of it on the
 * context's stream has completed (the launch is being dispatched; or, when
 * no batch goes to the GPU, before returning), while the call still waits for
 * the result: a caller queues its own independent work on another context's
 * stream there (e.g. the next batch's encode), so that it runs beside the
 * elimination on the CUs the elimination's workgroups leave free -- queued
 * earlier, it could hold the CUs those workgroups need to be resident
 * together.  The caller therefore need not wait for its earlier work on this
 * context (e.g. the previous batch's GetPieces) before the call.  The hook may
 * return a hipEvent_t (or NULL): the rest of the call's work on this
 * context's stream (the received rows' copies) is then ordered behind it.
 * The hook must not call into this context. */
typedef void* (*rlnc_hook_fn)(void* user);
int rlnc_decoders_add_pieces_gpu_hook(rlnc_decoder* const* decs, size_t G, const uint8_t* const* d_rows,
                                      const size_t* counts, size_t pitch, size_t piece_len, size_t* consumed,
                                      int* status, rlnc_hook_fn after_launch, void* user);
/* The pending AddPiece calls of G decoders (one context, one piece_count),
 * eliminated together: one AddPiece call per piece only queues the coding
 * vector while the queue cannot complete the rank (lazy AddPiece), and a
 * decoder's next state read eliminates its queue on the host.  This call
 * takes every decoder whose queue completes its rank from a state of kept
 * pieces (none dependent) through ONE GPU elimination launch (gf_elim.hip, a
 * workgroup each; no kodr counterpart: a server feeding many generations
 * piece by piece calls it once per tick); the rest, and singular batches,
 * take the host flush.  Queued device pieces are gathered as well.  The
 * state afterwards is the one the individual state reads would leave. */
int rlnc_decoders_flush_gpu(rlnc_decoder* const* decs, size_t G);
/* State reads.  is_decoded, required, useful, coefficients, transform and
 * decoded_mask first run the decoder's queued (lazy) AddPiece calls through
 * the elimination, so although they take a const handle they modify its
 * internal state: like every other call on one decoder (kodr's objects are not
 * goroutine-safe either), they must not run concurrently on the same handle. */
int rlnc_decoder_is_decoded(const rlnc_decoder* dec);        /* IsDecoded :32-34 */
size_t rlnc_decoder_required(const rlnc_decoder* dec);       /* Required  :38-40 */
size_t rlnc_decoder_useful(const rlnc_decoder* dec);         /* rank */
size_t rlnc_decoder_received(const rlnc_decoder* dec);
size_t rlnc_decoder_piece_length(const rlnc_decoder* dec);   /* PieceLength :18-25 */
size_t rlnc_decoder_piece_count(const rlnc_decoder* dec);
/* GetPiece (full/decoder.go:77-79 -> decoder_state.go:221-261) into out (L bytes) */
int rlnc_decoder_get_piece(rlnc_decoder* dec, size_t index, uint8_t* out);
/* GetPieces (full/decoder.go:83-99): out = useful x L bytes */
int rlnc_decoder_get_pieces(rlnc_decoder* dec, uint8_t* out);
/* GetPieces into device memory: useful rows of L bytes at out_pitch (async) */
int rlnc_decoder_get_pieces_device(rlnc_decoder* dec, uint8_t* d_out, size_t out_pitch);
/* GetPieces of G decoded generations (one context, one piece_count and
 * piece_len) into device memory: d_out holds G blocks of piece_count rows at
 * out_pitch (decoder g's first row at g*piece_count*out_pitch).  When every
 * decoder received the same number of pieces and none holds a systematic
 * (unit) row, ONE bit-sliced launch per 16 decoders applies their T x R
 * products (the host stages the next 16 transforms while it runs); other
 * decoders take rlnc_decoder_get_pieces_device one by one.  Same bytes
 * either way.  RLNC_ERR_MORE_USEFUL_PIECES_REQUIRED if any decoder is
 * not decoded (nothing is written).  Async on the ctx stream. */
int rlnc_decoders_get_pieces_device(rlnc_decoder* const* decs, size_t G, uint8_t* d_out, size_t out_pitch);
/* introspection of the mirrored decoder state (decoder_state.go:192-200):
 * coefficient matrix (useful x piece_count) and the transform T
 * (useful x received) with coded rows == T x received pieces */
int rlnc_decoder_coefficients(const rlnc_decoder* dec, uint8_t* out);
/* rows of the last data-side materialization (GetPiece/GetPieces) that went
 * through the GF kernel vs were plain copies of received systematic pieces */
int rlnc_decoder_apply_stats(const rlnc_decoder* dec, size_t* gf_rows, size_t* copy_rows);
/* 1 if the last materialization's GF product ran on the bit-sliced kernel
 * (gf_bs_kernel), 0 for the v_perm kernel or no GF rows (diagnostics) */
int rlnc_decoder_last_apply_bitsliced(const rlnc_decoder* dec);
/* which route eliminated the decoder's batches so far: gpu = states the GPU
 * elimination produced (gpu_retried of them after a permuted re-attempt:
 * a singular panel block, gf_elim.hip), host_after_gpu = GPU launches that
 * failed (a singular C, a structured batch) and left the batch to kodr's
 * algorithm on the host, host = host eliminations without a GPU launch.
 * Any pointer may be NULL. */
int rlnc_decoder_elim_stats(const rlnc_decoder* dec, size_t* gpu, size_t* gpu_retried, size_t* host_after_gpu,
                            size_t* host);
int rlnc_decoder_transform(const rlnc_decoder* dec, uint8_t* out);

/* ---- progressive decode (an extension) ---------------------- */
/* kodr's GetPiece before full rank follows decoder_state.go:233-256, whose
 * test ("every other coefficient non-zero") almost never holds, so a consumer
 * cannot read pieces early through it.  These read every original piece that
 * IS decoded: some row of the state is a*e_j on the coefficient side (a
 * systematic piece on arrival, every piece at full rank).
 * Data-side policy: LAZY (default) materializes on request; EAGER also
 * materializes, in every AddPiece call, the pieces that call decoded (on the
 * context stream, asynchronously), so a later read is a copy.  The state and
 * kodr's API results are the same under both. */
#define RLNC_DECODE_LAZY  0
#define RLNC_DECODE_EAGER 1
int rlnc_decoder_set_policy(rlnc_decoder* dec, int policy);
/* mask[j] = 1 for each decoded original piece j (mask: piece_count bytes or
 * NULL); returns how many are decoded */
size_t rlnc_decoder_decoded_mask(const rlnc_decoder* dec, uint8_t* mask);
/* original piece j (L bytes) into out (host, or device when is_device), or
 * RLNC_ERR_PIECE_NOT_DECODED_YET / RLNC_ERR_PIECE_OUT_OF_BOUND */
int rlnc_decoder_get_decoded(rlnc_decoder* dec, size_t j, uint8_t* out, int is_device);
/* Bind a device buffer (piece_count rows at `pitch`, both 16-byte aligned,
 * pitch >= piece length; AddPiece must have fixed the length) as the home of
 * the decoded generation: original piece j is materialized straight to
 * d_out + j * pitch (under EAGER, by the AddPiece call that decoded it, on the
 * context stream), so a consumer reads it in place once rlnc_decoder_decoded_mask
 * shows it and the context stream has passed that call.  NULL unbinds.
 * Binding drops the pieces materialized before it; GetPiece/GetPieces are
 * unchanged. */
int rlnc_decoder_bind_output(rlnc_decoder* dec, uint8_t* d_out, size_t pitch);

/* diagnostics: the plan of the last GF product launch made by the calling
 * thread (any entry point above that multiplies), so tests can pin the exact
 * kernel instance a benchmark times.  No kodr counterpart. */
typedef struct rlnc_launch_plan {
  int kernel;         /* 1 = gf_gemm_kernel (v_perm tables), 2 = gf_bs_kernel (bit-sliced),
                         3 = gf_gemv_kernel (one coded piece, register tables), 0 = none yet */
  int tile_rows;      /* output rows per workgroup tile (gf_bs_kernel: 8) */
  int waves;          /* waves per workgroup splitting K (KW) */
  int lane_groups;    /* gf_gemm_kernel: input rows per wave-step (S); gf_bs_kernel: 1 */
  int ring;           /* rows (gf_bs) or row-steps (gf_gemm) in flight per wave */
  int rows_per_wave;  /* input rows per wave (gf_gemm: per K-chunk) */
  int generations;    /* grid rows: products in one grouped launch, else 1 */
  int workgroups;     /* workgroups per generation (gridDim.x) */
} rlnc_launch_plan;
int rlnc_last_launch_plan(rlnc_launch_plan* out);

/* ---- raw kernel entry: Y = A (x) X over GF(2^8) ------------------------ */
/* Y[m][j] = XOR_k mul(A[m][k], X[k][j]) for m<M, j<ncols.  A is M x K host
 * bytes (row stride lda); X and Y are device rows at pitches ldx/ldy (multiples
 * of 16, >= ncols).  Async on the ctx stream. */
int rlnc_gf_matmul_device(rlnc_ctx* ctx, const uint8_t* d_A, size_t lda, size_t M, size_t K,
                          const uint8_t* d_X, size_t ldx, uint8_t* d_Y, size_t ldy, size_t ncols);
/* Bit-sliced layout: in place, every 32-byte block of rows
 * [0, rows) x [0, round_up(ncols, 32)) becomes 8 bit planes, plane i = bit i
 * of the block's 32 bytes.  Self-inverse.  ldx multiple of 32.  Async. */
int rlnc_bitslice_device(rlnc_ctx* ctx, uint8_t* d_X, size_t ldx, size_t rows, size_t ncols);
/* diagnostics: byte offsets of the bit-sliced kernel's 256 coefficient bodies
 * (first copy) from body 0; also runs the one-time check that enables the
 * bit-sliced path on this device */
int rlnc_bs_body_offsets(rlnc_ctx* ctx, uint32_t* out256);
/* Y = A (x) X like rlnc_gf_matmul_device, with X (K rows, pitch ldx, multiple
 * of 32, K*ldx < 2^32) in bit-sliced layout; Y in plain bytes.  Async.
 * Returns a HIP error ("operation not supported") if the bit-sliced path
 * failed its one-time check on this device (the engine's own callers then
 * use rlnc_gf_matmul_device's kernel instead). */
int rlnc_gf_matmul_bs_device(rlnc_ctx* ctx, const uint8_t* d_A, size_t lda, size_t M, size_t K,
                             const uint8_t* d_Xbs, size_t ldx, uint8_t* d_Y, size_t ldy, size_t ncols);

#ifdef __cplusplus
}
#endif
#endif /* KODR_RLNC_H */
