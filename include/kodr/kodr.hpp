// kodr.hpp -- C++ host API mirroring itzmeanjan/kodr's Go packages
// (full/, systematic/, kodr_internals/, errors.go) over the C ABI of
// libkodr_rlnc.so (include/kodr_rlnc.h).  Header-only.
//
// Go's (value, error) returns are mirrored as std::pair<value, Err> / Err, and
// the sentinel errors of errors.go:6-17 as kodr::Err values, so code written
// against kodr reads the same:
//
//   auto [enc, err] = kodr::full::NewFullRLNCEncoderWithPieceCount(data, 256);
//   auto dec = kodr::full::NewFullRLNCDecoder(256);
//   while (!dec->IsDecoded()) dec->AddPiece(enc->CodedPiece());
//   auto [pieces, err2] = dec->GetPieces();
//
// Every coded byte is computed on the GPU; coding vectors come from the OS
// CSPRNG (getrandom, like crypto/rand in data.go:90-95).  Encoders hand out
// pieces one CodedPiece() at a time but compute them `batch` at a time.
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <deque>
#include <memory>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

#include "../kodr_rlnc.h"

namespace kodr {

// errors.go:5-18 (values == C-ABI status codes)
enum class Err : int {
  None = RLNC_OK,
  CannotInvertGf256AdditiveIndentity = RLNC_ERR_CANNOT_INVERT_GF256_ADD_IDENTITY,
  MatrixDimensionMismatch = RLNC_ERR_MATRIX_DIMENSION_MISMATCH,
  AllUsefulPiecesReceived = RLNC_ERR_ALL_USEFUL_PIECES_RECEIVED,
  MoreUsefulPiecesRequired = RLNC_ERR_MORE_USEFUL_PIECES_REQUIRED,
  CopyFailedDuringPieceConstruction = RLNC_ERR_COPY_FAILED_DURING_PIECE_CONSTRUCTION,
  PieceCountMoreThanTotalBytes = RLNC_ERR_PIECE_COUNT_MORE_THAN_TOTAL_BYTES,
  ZeroPieceSize = RLNC_ERR_ZERO_PIECE_SIZE,
  BadPieceCount = RLNC_ERR_BAD_PIECE_COUNT,
  CodedDataLengthMismatch = RLNC_ERR_CODED_DATA_LENGTH_MISMATCH,
  CodingVectorLengthMismatch = RLNC_ERR_CODING_VECTOR_LENGTH_MISMATCH,
  PieceNotDecodedYet = RLNC_ERR_PIECE_NOT_DECODED_YET,
  PieceOutOfBound = RLNC_ERR_PIECE_OUT_OF_BOUND,
};
constexpr Err ErrCannotInvertGf256AdditiveIndentity = Err::CannotInvertGf256AdditiveIndentity;
constexpr Err ErrMatrixDimensionMismatch = Err::MatrixDimensionMismatch;
constexpr Err ErrAllUsefulPiecesReceived = Err::AllUsefulPiecesReceived;
constexpr Err ErrMoreUsefulPiecesRequired = Err::MoreUsefulPiecesRequired;
constexpr Err ErrCopyFailedDuringPieceConstruction = Err::CopyFailedDuringPieceConstruction;
constexpr Err ErrPieceCountMoreThanTotalBytes = Err::PieceCountMoreThanTotalBytes;
constexpr Err ErrZeroPieceSize = Err::ZeroPieceSize;
constexpr Err ErrBadPieceCount = Err::BadPieceCount;
constexpr Err ErrCodedDataLengthMismatch = Err::CodedDataLengthMismatch;
constexpr Err ErrCodingVectorLengthMismatch = Err::CodingVectorLengthMismatch;
constexpr Err ErrPieceNotDecodedYet = Err::PieceNotDecodedYet;
constexpr Err ErrPieceOutOfBound = Err::PieceOutOfBound;

inline std::string ErrorString(Err e) { return rlnc_status_string((int)e); }

// Engine failures (HIP errors, no device, invalid use) have no kodr sentinel
// and are thrown.
struct EngineError : std::runtime_error {
  int status;
  explicit EngineError(int s)
      : std::runtime_error(std::string("kodr_amd: ") + rlnc_status_string(s) + ": " + rlnc_last_hip_error()),
        status(s) {}
};

namespace detail {
// kodr errors -> Err, engine errors -> throw
inline Err check(int s) {
  if (s < 0) throw EngineError(s);
  return (Err)s;
}
}  // namespace detail

// One device + stream; every object below lives on one.
class Context {
 public:
  explicit Context(int device = 0, void* stream = nullptr) {
    detail::check(rlnc_ctx_create(device, stream, &h_));
  }
  ~Context() { rlnc_ctx_destroy(h_); }
  Context(const Context&) = delete;
  Context& operator=(const Context&) = delete;
  rlnc_ctx* get() const { return h_; }
  void Synchronize() { detail::check(rlnc_ctx_synchronize(h_)); }
  static Context& Default() {
    static Context c(0);
    return c;
  }

 private:
  rlnc_ctx* h_ = nullptr;
};

namespace kodr_internals {

using Piece = std::vector<uint8_t>;         // data.go:12
using CodingVector = std::vector<uint8_t>;  // data.go:34

struct CodedPiece {  // data.go:38-41
  CodingVector Vector;
  kodr_internals::Piece Piece;
  size_t Len() const { return Vector.size() + Piece.size(); }  // data.go:44-46
  std::vector<uint8_t> Flatten() const {                        // data.go:52-57
    std::vector<uint8_t> r(Vector);
    r.insert(r.end(), Piece.begin(), Piece.end());
    return r;
  }
  bool IsSystematic() const {  // data.go:64-84
    return rlnc_is_systematic(Vector.data(), Vector.size()) != 0;
  }
};

inline CodingVector GenerateCodingVector(size_t n) {  // data.go:90-95
  CodingVector v(n);
  detail::check(rlnc_random_bytes(v.data(), n));
  return v;
}

namespace detail_split {
inline std::vector<Piece> split(const std::vector<uint8_t>& data, size_t size, size_t count) {
  std::vector<Piece> out(count, Piece(size, 0));
  for (size_t i = 0; i < data.size(); i++) out[i / size][i % size] = data[i];
  return out;
}
}  // namespace detail_split

// data.go:103-132
inline std::pair<std::vector<Piece>, std::pair<size_t, Err>> OriginalPiecesFromDataAndPieceSize(
    const std::vector<uint8_t>& data, size_t pieceSize) {
  size_t count = 0, pad = 0;
  Err e = kodr::detail::check(rlnc_split_by_piece_size(data.size(), pieceSize, &count, &pad));
  if (e != Err::None) return {{}, {0, e}};
  return {detail_split::split(data, pieceSize, count), {pad, Err::None}};
}

// data.go:137-166
inline std::pair<std::vector<Piece>, std::pair<size_t, Err>> OriginalPiecesFromDataAndPieceCount(
    const std::vector<uint8_t>& data, size_t pieceCount) {
  size_t size = 0, pad = 0;
  Err e = kodr::detail::check(rlnc_split_by_piece_count(data.size(), pieceCount, &size, &pad));
  if (e != Err::None) return {{}, {0, e}};
  return {detail_split::split(data, size, pieceCount), {pad, Err::None}};
}

// data.go:173-193
inline std::pair<std::vector<CodedPiece>, Err> CodedPiecesForRecoding(const std::vector<uint8_t>& data,
                                                                      size_t pieceCount,
                                                                      size_t piecesCodedTogether) {
  size_t cpl = 0;
  Err e = kodr::detail::check(rlnc_coded_pieces_for_recoding(data.size(), pieceCount, piecesCodedTogether, &cpl));
  if (e != Err::None) return {{}, e};
  std::vector<CodedPiece> out(pieceCount);
  for (size_t i = 0; i < pieceCount; i++) {
    const uint8_t* row = data.data() + i * cpl;
    out[i].Vector.assign(row, row + piecesCodedTogether);
    out[i].Piece.assign(row + piecesCodedTogether, row + cpl);
  }
  return {out, Err::None};
}

}  // namespace kodr_internals

namespace detail {

class EncoderBase {
 public:
  EncoderBase(rlnc_encoder* h, size_t batch) : h_(h), batch_(batch ? batch : 1) {}
  ~EncoderBase() { rlnc_encoder_destroy(h_); }
  EncoderBase(const EncoderBase&) = delete;
  EncoderBase& operator=(const EncoderBase&) = delete;
  size_t PieceCount() const { return rlnc_encoder_piece_count(h_); }
  size_t PieceSize() const { return rlnc_encoder_piece_size(h_); }
  size_t DecodableLen() const { return rlnc_encoder_decodable_len(h_); }
  size_t CodedPieceLen() const { return rlnc_encoder_coded_piece_len(h_); }
  size_t Padding() const { return rlnc_encoder_padding(h_); }
  // extension (no kodr counterpart): keep only the bit-sliced copy of the
  // generation in HBM (rlnc_encoder_compact)
  Err Compact() { return check(rlnc_encoder_compact(h_)); }
  kodr_internals::CodedPiece CodedPiece() {
    if (queue_.empty()) refill();
    kodr_internals::CodedPiece p = std::move(queue_.front());
    queue_.pop_front();
    return p;
  }
  rlnc_encoder* handle() const { return h_; }

 private:
  void refill() {
    const size_t k = PieceCount(), clen = CodedPieceLen();
    std::vector<uint8_t> vec(batch_ * k), out(batch_ * clen);
    check(rlnc_random_bytes(vec.data(), vec.size()));
    check(rlnc_encoder_coded_pieces(h_, vec.data(), batch_, out.data()));
    for (size_t b = 0; b < batch_; b++) {
      kodr_internals::CodedPiece p;
      p.Vector.assign(out.begin() + b * clen, out.begin() + b * clen + k);
      p.Piece.assign(out.begin() + b * clen + k, out.begin() + (b + 1) * clen);
      queue_.push_back(std::move(p));
    }
  }
  rlnc_encoder* h_;
  size_t batch_;
  std::deque<kodr_internals::CodedPiece> queue_;
};

template <class E>
std::pair<std::unique_ptr<E>, Err> make_encoder(int kind, const std::vector<kodr_internals::Piece>& pieces,
                                                Context& ctx, size_t batch) {
  if (pieces.empty()) return {nullptr, Err::BadPieceCount};
  const size_t k = pieces.size(), L = pieces[0].size();
  std::vector<uint8_t> flat;
  flat.reserve(k * L);
  for (auto& p : pieces) flat.insert(flat.end(), p.begin(), p.end());
  rlnc_encoder* h = nullptr;
  Err e = check(rlnc_encoder_create(ctx.get(), kind, flat.data(), k, L, &h));
  if (e != Err::None) return {nullptr, e};
  return {std::unique_ptr<E>(new E(h, batch)), Err::None};
}

template <class E>
std::pair<std::unique_ptr<E>, Err> make_encoder_split(int kind, bool by_count, const std::vector<uint8_t>& data,
                                                      size_t n, Context& ctx, size_t batch) {
  rlnc_encoder* h = nullptr;
  Err e = check(by_count ? rlnc_encoder_create_with_piece_count(ctx.get(), kind, data.data(), data.size(), n, &h)
                         : rlnc_encoder_create_with_piece_size(ctx.get(), kind, data.data(), data.size(), n, &h));
  if (e != Err::None) return {nullptr, e};
  return {std::unique_ptr<E>(new E(h, batch)), Err::None};
}

class DecoderBase {  // full/decoder.go == systematic/decoder.go
 public:
  DecoderBase(size_t pieceCount, Context& ctx) { check(rlnc_decoder_create(ctx.get(), pieceCount, &h_)); }
  ~DecoderBase() { rlnc_decoder_destroy(h_); }
  DecoderBase(const DecoderBase&) = delete;
  DecoderBase& operator=(const DecoderBase&) = delete;
  size_t PieceLength() const { return rlnc_decoder_piece_length(h_); }  // :18-25
  bool IsDecoded() const { return rlnc_decoder_is_decoded(h_) != 0; }   // :32-34
  size_t Required() const { return rlnc_decoder_required(h_); }         // :38-40
  Err AddPiece(const kodr_internals::CodedPiece& p) {                  // :50-66
    return check(rlnc_decoder_add_piece(h_, p.Vector.data(), p.Vector.size(), p.Piece.data(), p.Piece.size()));
  }
  std::pair<kodr_internals::Piece, Err> GetPiece(size_t i) {            // :77-79
    kodr_internals::Piece out(PieceLength() ? PieceLength() : 1);
    Err e = check(rlnc_decoder_get_piece(h_, i, out.data()));
    out.resize(PieceLength());
    if (e != Err::None) return {{}, e};
    return {out, Err::None};
  }
  std::pair<std::vector<kodr_internals::Piece>, Err> GetPieces() {      // :83-99
    if (!IsDecoded()) return {{}, Err::MoreUsefulPiecesRequired};
    const size_t n = rlnc_decoder_useful(h_), L = PieceLength();
    std::vector<uint8_t> flat(n * L);
    Err e = check(rlnc_decoder_get_pieces(h_, flat.data()));
    if (e != Err::None) return {{}, e};
    std::vector<kodr_internals::Piece> out(n);
    for (size_t i = 0; i < n; i++) out[i].assign(flat.begin() + i * L, flat.begin() + (i + 1) * L);
    return {out, Err::None};
  }
  rlnc_decoder* handle() const { return h_; }

  // Extensions (no kodr counterpart): pieces decoded before full
  // rank.  SetEager(true): AddPiece materializes what it decoded.
  Err SetEager(bool eager) {
    return check(rlnc_decoder_set_policy(h_, eager ? RLNC_DECODE_EAGER : RLNC_DECODE_LAZY));
  }
  std::vector<bool> DecodedMask() const {
    const size_t k = PieceCount();
    std::vector<uint8_t> m(k ? k : 1);
    rlnc_decoder_decoded_mask(h_, m.data());
    return std::vector<bool>(m.begin(), m.begin() + k);
  }
  std::pair<kodr_internals::Piece, Err> GetDecodedPiece(size_t i) {
    kodr_internals::Piece out(PieceLength() ? PieceLength() : 1);
    Err e = check(rlnc_decoder_get_decoded(h_, i, out.data(), 0));
    out.resize(PieceLength());
    if (e != Err::None) return {{}, e};
    return {out, Err::None};
  }
  size_t PieceCount() const { return rlnc_decoder_required(h_) + rlnc_decoder_useful(h_); }

 private:
  rlnc_decoder* h_ = nullptr;
};

}  // namespace detail

namespace full {

class FullRLNCEncoder : public detail::EncoderBase {  // full/encoder.go:7-10
  using EncoderBase::EncoderBase;
};

// full/encoder.go:76-78
inline std::pair<std::unique_ptr<FullRLNCEncoder>, Err> NewFullRLNCEncoder(
    const std::vector<kodr_internals::Piece>& pieces, Context& ctx = Context::Default(), size_t batch = 16) {
  return detail::make_encoder<FullRLNCEncoder>(RLNC_FULL, pieces, ctx, batch);
}
// full/encoder.go:84-93
inline std::pair<std::unique_ptr<FullRLNCEncoder>, Err> NewFullRLNCEncoderWithPieceCount(
    const std::vector<uint8_t>& data, size_t pieceCount, Context& ctx = Context::Default(), size_t batch = 16) {
  return detail::make_encoder_split<FullRLNCEncoder>(RLNC_FULL, true, data, pieceCount, ctx, batch);
}
// full/encoder.go:98-107
inline std::pair<std::unique_ptr<FullRLNCEncoder>, Err> NewFullRLNCEncoderWithPieceSize(
    const std::vector<uint8_t>& data, size_t pieceSize, Context& ctx = Context::Default(), size_t batch = 16) {
  return detail::make_encoder_split<FullRLNCEncoder>(RLNC_FULL, false, data, pieceSize, ctx, batch);
}

class FullRLNCRecoder {  // full/recoder.go:8-11
 public:
  FullRLNCRecoder(rlnc_recoder* h, size_t k, size_t batch) : h_(h), k_(k), batch_(batch ? batch : 1) {}
  ~FullRLNCRecoder() { rlnc_recoder_destroy(h_); }
  FullRLNCRecoder(const FullRLNCRecoder&) = delete;
  FullRLNCRecoder& operator=(const FullRLNCRecoder&) = delete;
  // full/recoder.go:27-46 (error return kept for signature parity; never set)
  Err Compact() { return detail::check(rlnc_recoder_compact(h_)); }  // extension: rlnc_recoder_compact
  std::pair<kodr_internals::CodedPiece, Err> CodedPiece() {
    if (queue_.empty()) {
      const size_t n = rlnc_recoder_piece_count(h_), clen = rlnc_recoder_coded_piece_len(h_);
      std::vector<uint8_t> r(batch_ * n), out(batch_ * clen);
      detail::check(rlnc_random_bytes(r.data(), r.size()));
      Err e = detail::check(rlnc_recoder_coded_pieces(h_, r.data(), batch_, out.data()));
      if (e != Err::None) return {{}, e};
      for (size_t b = 0; b < batch_; b++) {
        kodr_internals::CodedPiece p;
        p.Vector.assign(out.begin() + b * clen, out.begin() + b * clen + k_);
        p.Piece.assign(out.begin() + b * clen + k_, out.begin() + (b + 1) * clen);
        queue_.push_back(std::move(p));
      }
    }
    kodr_internals::CodedPiece p = std::move(queue_.front());
    queue_.pop_front();
    return {p, Err::None};
  }

 private:
  rlnc_recoder* h_;
  size_t k_, batch_;
  std::deque<kodr_internals::CodedPiece> queue_;
};

// full/recoder.go:63-70
inline std::pair<std::unique_ptr<FullRLNCRecoder>, Err> NewFullRLNCRecoderWithFlattenData(
    const std::vector<uint8_t>& data, size_t pieceCount, size_t piecesCodedTogether,
    Context& ctx = Context::Default(), size_t batch = 16) {
  rlnc_recoder* h = nullptr;
  Err e = detail::check(rlnc_recoder_create(ctx.get(), data.data(), data.size(), pieceCount, piecesCodedTogether, &h));
  if (e != Err::None) return {nullptr, e};
  return {std::unique_ptr<FullRLNCRecoder>(new FullRLNCRecoder(h, piecesCodedTogether, batch)), Err::None};
}
// full/recoder.go:52-57
inline std::unique_ptr<FullRLNCRecoder> NewFullRLNCRecoder(const std::vector<kodr_internals::CodedPiece>& pieces,
                                                           Context& ctx = Context::Default(), size_t batch = 16) {
  std::vector<uint8_t> flat;
  for (auto& p : pieces) {
    auto f = p.Flatten();
    flat.insert(flat.end(), f.begin(), f.end());
  }
  const size_t k = pieces.empty() ? 0 : pieces[0].Vector.size();
  auto r = NewFullRLNCRecoderWithFlattenData(flat, pieces.size(), k, ctx, batch);
  if (r.second != Err::None) throw EngineError(RLNC_ERR_INVALID_ARGUMENT);
  return std::move(r.first);
}

class FullRLNCDecoder : public detail::DecoderBase {  // full/decoder.go:9-12
  using DecoderBase::DecoderBase;
};
// full/decoder.go:109-112
inline std::unique_ptr<FullRLNCDecoder> NewFullRLNCDecoder(size_t pieceCount, Context& ctx = Context::Default()) {
  return std::unique_ptr<FullRLNCDecoder>(new FullRLNCDecoder(pieceCount, ctx));
}

}  // namespace full

namespace systematic {

class SystematicRLNCEncoder : public detail::EncoderBase {  // systematic/encoder.go:7-11
  using EncoderBase::EncoderBase;
};
// systematic/encoder.go:115-117
inline std::pair<std::unique_ptr<SystematicRLNCEncoder>, Err> NewSystematicRLNCEncoder(
    const std::vector<kodr_internals::Piece>& pieces, Context& ctx = Context::Default(), size_t batch = 16) {
  return detail::make_encoder<SystematicRLNCEncoder>(RLNC_SYSTEMATIC, pieces, ctx, batch);
}
// systematic/encoder.go:123-132
inline std::pair<std::unique_ptr<SystematicRLNCEncoder>, Err> NewSystematicRLNCEncoderWithPieceCount(
    const std::vector<uint8_t>& data, size_t pieceCount, Context& ctx = Context::Default(), size_t batch = 16) {
  return detail::make_encoder_split<SystematicRLNCEncoder>(RLNC_SYSTEMATIC, true, data, pieceCount, ctx, batch);
}
// systematic/encoder.go:137-146
inline std::pair<std::unique_ptr<SystematicRLNCEncoder>, Err> NewSystematicRLNCEncoderWithPieceSize(
    const std::vector<uint8_t>& data, size_t pieceSize, Context& ctx = Context::Default(), size_t batch = 16) {
  return detail::make_encoder_split<SystematicRLNCEncoder>(RLNC_SYSTEMATIC, false, data, pieceSize, ctx, batch);
}

class SystematicRLNCDecoder : public detail::DecoderBase {  // systematic/decoder.go:9-12
  using DecoderBase::DecoderBase;
};
// systematic/decoder.go:105-108
inline std::unique_ptr<SystematicRLNCDecoder> NewSystematicRLNCDecoder(size_t pieceCount,
                                                                       Context& ctx = Context::Default()) {
  return std::unique_ptr<SystematicRLNCDecoder>(new SystematicRLNCDecoder(pieceCount, ctx));
}

}  // namespace systematic
}  // namespace kodr
