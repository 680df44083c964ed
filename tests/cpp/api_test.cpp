// kodr's Go tests restated against the C++ mirror (include/kodr/kodr.hpp).
// Built by tests/test_cpp_api.py; run on the GPU box (-m gpu).
#include <kodr/kodr.hpp>

#include <cstdio>
#include <random>

using namespace kodr;
using kodr_internals::CodedPiece;
using kodr_internals::Piece;

static int failures = 0;
#define EXPECT(c)                                                  \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
      failures++;                                                  \
    }                                                              \
  } while (0)

static std::mt19937_64 rng(7);
static std::vector<uint8_t> gen(size_t n) {
  std::vector<uint8_t> v(n);
  for (auto& x : v) x = (uint8_t)rng();
  return v;
}

// full/encoder_test.go:34-77
template <class Enc>
static void encoder_flow(Enc& enc, size_t pieceCount, size_t codedCount, const std::vector<Piece>& pieces) {
  std::vector<CodedPiece> coded;
  for (size_t i = 0; i < codedCount; i++) coded.push_back(enc.CodedPiece());
  auto dec = full::NewFullRLNCDecoder(pieceCount);
  for (size_t i = 0; i < codedCount; i++) {
    if (i < pieceCount) EXPECT(dec->GetPieces().second == ErrMoreUsefulPiecesRequired);
    if (dec->AddPiece(coded[i]) == ErrAllUsefulPiecesReceived) break;
  }
  EXPECT(dec->IsDecoded());
  for (size_t i = 0; i < codedCount - pieceCount; i++)
    EXPECT(dec->AddPiece(coded[pieceCount + i]) == ErrAllUsefulPiecesReceived);
  auto [d, err] = dec->GetPieces();
  EXPECT(err == Err::None);
  EXPECT(d == pieces);
}

int main() {
  {  // full/encoder_test.go:79-87
    std::vector<Piece> pieces;
    for (int i = 0; i < 128; i++) pieces.push_back(gen(8192));
    auto [enc, err] = full::NewFullRLNCEncoder(pieces);
    EXPECT(err == Err::None);
    encoder_flow(*enc, 128, 130, pieces);
  }
  {  // full/encoder_test.go:89-107 with padding
    auto data = gen(3001);
    auto [pieces, pe] = kodr_internals::OriginalPiecesFromDataAndPieceCount(data, 37);
    EXPECT(pe.second == Err::None);
    auto [enc, err] = full::NewFullRLNCEncoderWithPieceCount(data, 37);
    EXPECT(err == Err::None && enc->Padding() == pe.first);
    encoder_flow(*enc, 37, 39, pieces);
  }
  {  // error paths: data.go:103-166
    auto data = gen(100);
    EXPECT(full::NewFullRLNCEncoderWithPieceCount(data, 1).second == ErrBadPieceCount);
    EXPECT(full::NewFullRLNCEncoderWithPieceCount(data, 101).second == ErrPieceCountMoreThanTotalBytes);
    EXPECT(full::NewFullRLNCEncoderWithPieceSize(data, 0).second == ErrZeroPieceSize);
    EXPECT(full::NewFullRLNCEncoderWithPieceSize(data, 100).second == ErrBadPieceCount);
  }
  {  // full/recoder_test.go:57-80
    std::vector<Piece> pieces;
    for (int i = 0; i < 64; i++) pieces.push_back(gen(4096));
    auto [enc, err] = full::NewFullRLNCEncoder(pieces);
    std::vector<uint8_t> flat;
    for (int i = 0; i < 66; i++) {
      auto f = enc->CodedPiece().Flatten();
      flat.insert(flat.end(), f.begin(), f.end());
    }
    EXPECT(full::NewFullRLNCRecoderWithFlattenData(flat, 67, 64).second == ErrCodedDataLengthMismatch);
    auto [rec, rerr] = full::NewFullRLNCRecoderWithFlattenData(flat, 66, 64);
    EXPECT(rerr == Err::None);
    auto dec = full::NewFullRLNCDecoder(64);
    while (true) {
      auto [p, e] = rec->CodedPiece();
      EXPECT(e == Err::None);
      if (dec->AddPiece(p) == ErrAllUsefulPiecesReceived) break;
    }
    EXPECT(dec->GetPieces().first == pieces);
  }
  {  // systematic/encoder_test.go:35-56 and :58-139
    std::vector<Piece> pieces;
    for (int i = 0; i < 100; i++) pieces.push_back(gen(1000));
    auto [enc, err] = systematic::NewSystematicRLNCEncoder(pieces);
    auto dec = systematic::NewSystematicRLNCDecoder(100);
    size_t sent = 0;
    while (true) {
      auto p = enc->CodedPiece();
      EXPECT(p.IsSystematic() == (sent < 100));
      sent++;
      if (rng() & 1) continue;
      if (dec->AddPiece(p) == ErrAllUsefulPiecesReceived) {
        EXPECT(dec->Required() == 0);
        break;
      }
    }
    EXPECT(dec->GetPieces().first == pieces);
  }
  {  // decoder_state.go:221-227
    auto dec = full::NewFullRLNCDecoder(4);
    EXPECT(dec->GetPiece(4).second == ErrPieceOutOfBound);
    EXPECT(dec->GetPiece(0).second == ErrPieceNotDecodedYet);
  }
  {  // extensions: compact residency, progressive decode of a systematic stream
    std::vector<Piece> pieces;
    for (int i = 0; i < 48; i++) pieces.push_back(gen(2048));
    auto [enc, err] = systematic::NewSystematicRLNCEncoder(pieces);
    EXPECT(err == Err::None && enc->Compact() == Err::None);
    auto dec = systematic::NewSystematicRLNCDecoder(48);
    EXPECT(dec->SetEager(true) == Err::None);
    size_t sent = 0;
    while (true) {
      auto p = enc->CodedPiece();
      const bool sys = sent++ < 48;
      if (sys && sent % 5 == 0) continue;  // lose every fifth systematic piece
      if (dec->AddPiece(p) == ErrAllUsefulPiecesReceived) break;
      if (sys) {  // a systematic piece is readable on arrival
        auto m = dec->DecodedMask();
        EXPECT(m[sent - 1]);
        auto [d, e] = dec->GetDecodedPiece(sent - 1);
        EXPECT(e == Err::None && d == pieces[sent - 1]);
        if (sent % 5 == 4) EXPECT(dec->GetDecodedPiece(sent).second == ErrPieceNotDecodedYet);
      }
    }
    EXPECT(dec->GetPieces().first == pieces);
    EXPECT(dec->GetDecodedPiece(48).second == ErrPieceOutOfBound);
  }
  std::printf("%s (%d failures)\n", failures ? "FAILED" : "ok", failures);
  return failures ? 1 : 0;
}
