// decoder_core.hpp -- the coefficient side of kodr's decoder, mirrored exactly.
//
// kodr's DecoderState (kodr_internals/matrix/decoder_state.go) keeps the
// augmented matrix [coeffs | coded] and, on every AddPiece, re-runs
// clean_forward / clean_backward / remove_zero_rows over both halves.  Every
// pivot decision it makes depends only on the coefficient half, and every row
// operation is linear, so the coded half always equals T x R, where R are the
// received pieces (in arrival order) and T is obtained by applying the same row
// operations to an identity block.  DecoderCore therefore runs the elimination
// on rows [coeffs (k) | T (received)] -- a few hundred bytes each -- and the
// data plane computes T x R on the GPU once (gf_gemm), bit-identical to kodr's
// in-place result, quirks included (diagonal-only pivots and rank over-count,
// decoder_state.go:23-35,86-88; zero-row removal :136-165; first piece skips
// RREF, full/decoder.go:58-61).
#pragma once
#include <stddef.h>
#include <stdint.h>

#include <vector>

namespace kodr_amd {

class DecoderCore {
 public:
  explicit DecoderCore(size_t piece_count);

  // full/decoder.go:50-66 minus the data: append row `vec` (k bytes) as
  // received piece number received(); returns 0 or kodr's
  // ErrAllUsefulPiecesReceived (3).
  int add(const uint8_t* vec);
  // the same as n calls of add() on rows vecs + i * pitch, stopping at the
  // first call that does not return 0; *used = rows accepted.  Runs of rows
  // that stay diagonal pivots are eliminated 4 at a time (one pass over the
  // existing rows per 4 new ones); the result is the same state.
  int add_many(const uint8_t* vecs, size_t pitch, size_t n, size_t* used);

  // A fresh decoder (nothing received) takes the state kodr reaches after c
  // >= 2 pieces that all landed on their diagonals: the reduced row echelon
  // form of [first c vectors | I_c], given as c rows of k + c bytes
  // (coefficients, then T) at `pitch` -- computed elsewhere (gf_elim.hip).
  // Later add() / add_many() calls continue exactly as if those c pieces had
  // been added one by one.  Returns false (and changes nothing) otherwise.
  bool load_rref(const uint8_t* state, size_t pitch, size_t c);
  // A fresh decoder takes the state kodr reaches after k pieces whose vectors
  // C are independent: [I | C^-1], given as C^-1 (k rows of k bytes at `pitch`,
  // columns in arrival order).  Returns false (and changes nothing) otherwise.
  // The state is kept as that one k x k block until a row is read (coeff_row,
  // t_row): the counters, rank, decoded(), piece_available() and the copies
  // answer from the block, so a batched AddPiece followed by GetPieces never
  // spreads it into k rows (a quarter of a C2 AddPiece call's host time).
  bool load_inverse(const uint8_t* tinv, size_t pitch);
  // A decoder holding r = received() >= 1 rows, all kept (rank() == r),
  // whose next k - r arrivals make its first k coding vectors C independent:
  // kodr ends in [I | C^-1] from any such state (an independent row never
  // becomes zero, rank counts kept rows).  The state comes from elsewhere
  // (gf_elim.hip) over M = [its r coefficient rows, in row order ; those
  // k - r vectors] = diag(T_r, I) x C, T_r its transform: k rows of k
  // coefficient bytes (I) then F = M^-1 at `pitch`, or with `inverse` only
  // F; C^-1 = F x diag(T_r, I).  Returns false (and changes nothing) otherwise.
  bool load_continued(const uint8_t* state, size_t pitch, bool inverse);

  bool is_decoded() const { return useful_ >= k_; }   // full/decoder.go:32-34
  size_t required() const { return k_ - useful_; }    // full/decoder.go:38-40
  size_t useful() const { return useful_; }
  size_t received() const { return received_; }
  size_t piece_count() const { return k_; }
  size_t rank() const { return pinv_on_ ? k_ : rows_.size(); }  // decoder_state.go:187-189

  // decoder_state.go:221-261 availability rule for GetPiece(idx): 0 when row
  // idx of the coded matrix may be returned, else kodr's error code.
  int piece_available(size_t idx) const;

  // original pieces decoded now: for each row whose coefficient half is a*e_j,
  // row_of[j] = that row and scale[j] = a (row_of[j] = -1 otherwise);
  // returns the count
  size_t decoded(std::vector<int32_t>* row_of, std::vector<uint8_t>* scale) const;

  const uint8_t* coeff_row(size_t i) const {
    expand();
    return rows_[i];
  }
  const uint8_t* t_row(size_t i) const {
    expand();
    return rows_[i] + k_;
  }
  // copy T (rank x received) densely into out (row stride = received)
  void copy_transform(uint8_t* out, size_t ld) const;
  void copy_coefficients(uint8_t* out) const;

 private:
  // the block load_inverse kept -> k rows (before anything reads or changes them)
  void expand() const {
    if (pinv_on_) const_cast<DecoderCore*>(this)->expand_inverse();
  }
  void expand_inverse();
  void rref();
  void rref_clean();
  size_t add_panel(const uint8_t* vecs, size_t pitch, size_t np);
  bool append_unit(const uint8_t* vec);
  bool solve_systematic_batch(const uint8_t* vecs, size_t pitch);
  bool solve_full_batch(const uint8_t* vecs, size_t pitch);
  void update_clean();
  void ensure_tcap(size_t need);
  void axpy_row(size_t dst, size_t src, uint8_t q, size_t from);
  void scale_row(size_t i, size_t from, uint8_t q);
  // row bookkeeping; up_/ut_ move with rows_
  void push_row(uint8_t* row, int32_t p, int32_t t);
  void pop_row();
  void swap_rows(size_t a, size_t b);
  void make_dense(size_t pos);
  void forget_row(size_t pos);

  size_t k_;
  size_t useful_ = 0, received_ = 0;
  size_t tcap_ = 0;                    // T columns allocated per row
  std::vector<uint8_t> arena_;         // k_ slots of (k_ + tcap_) bytes
  std::vector<uint8_t*> rows_;         // current rows, in kodr's row order
  std::vector<uint8_t*> free_;         // unused slots
  std::vector<uint8_t> clean_;         // per row index: diagonal pivot with a clean column above
  std::vector<uint8_t> dirty_;         // per row index: row moved/changed in this forward pass
  std::vector<uint8_t> touched_;       // per row index: target of a row operation in this pass
  bool all_clean_ = false;             // every row is a diagonal pivot with a clean column
  std::vector<uint8_t> qbuf_;          // quotients of the blocked passes
  std::vector<uint8_t*> ptrs_;
  // Sparse rows.  A row is "unit" when its coefficient half is a*e_p and its
  // T half is b*e_t (a systematic piece that no row operation has touched
  // yet); up_[i] = p and ut_[i] = t for such a row, up_[i] = -1 otherwise
  // ("dense": any content).  Only the bookkeeping is sparse -- the bytes of
  // every row stay complete -- and it is used only to skip work that is
  // provably zero: a row operation with a unit source touches two bytes, and
  // a unit row is non-zero in exactly one coefficient column.
  std::vector<int32_t> up_, ut_;       // parallel to rows_
  std::vector<uint32_t> ucnt_;         // per coefficient column: unit rows with that pivot
  size_t ndense_ = 0;                  // dense rows in rows_
  std::vector<size_t> dense_pos_;      // positions of dense rows (rebuilt per literal pass)
  std::vector<uint8_t> pinv_;          // load_inverse's C^-1 (k x k) while pinv_on_
  bool pinv_on_ = false;
};

}  // namespace kodr_amd
