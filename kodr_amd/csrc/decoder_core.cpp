// decoder_core.cpp -- see decoder_core.hpp.  Line references are to
// kodr_internals/matrix/decoder_state.go unless stated otherwise.
#include "decoder_core.hpp"

#include <string.h>

#include <algorithm>

#include "host_gf.hpp"

namespace kodr_amd {

using hostgf::T;

DecoderCore::DecoderCore(size_t piece_count) : k_(piece_count) {
  ensure_tcap(std::max<size_t>(k_ + 8, 16));
}

void DecoderCore::ensure_tcap(size_t need) {
  if (need <= tcap_) return;
  size_t ncap = std::max(need, tcap_ * 2);
  const size_t slots = std::max<size_t>(k_, 1);
  const size_t w_old = k_ + tcap_, w_new = k_ + ncap;
  std::vector<uint8_t> arena(slots * w_new, 0);
  std::vector<uint8_t*> rows(rows_.size());
  for (size_t i = 0; i < rows_.size(); i++) {
    rows[i] = arena.data() + i * w_new;
    memcpy(rows[i], rows_[i], w_old);
  }
  free_.clear();
  for (size_t s = rows_.size(); s < slots; s++) free_.push_back(arena.data() + s * w_new);
  arena_.swap(arena);
  rows_.swap(rows);
  tcap_ = ncap;
  clean_.resize(slots + 1, 0);
  dirty_.resize(slots + 1, 0);
  touched_.resize(slots + 1, 0);
}

// rows_[dst] ^= q * rows_[src] over coefficient columns [from, k) and all T
// columns (the coded half in kodr is updated over its whole width, :66-73).
void DecoderCore::axpy_row(size_t dst, size_t src, uint8_t q, size_t from) {
  hostgf::axpy(rows_[dst] + from, rows_[src] + from, k_ - from + received_, q);
  touched_[dst] = 1;
}

int DecoderCore::add(const uint8_t* vec) {
  if (is_decoded()) return 3;                       // full/decoder.go:52-54
  ensure_tcap(received_ + 1);
  uint8_t* row = free_.back();                      // :205-208 (append)
  free_.pop_back();
  memcpy(row, vec, k_);
  memset(row + k_, 0, tcap_);
  row[k_ + received_] = 1;                          // T row = e_received
  rows_.push_back(row);
  received_++;                                      // full/decoder.go:57
  if (!(received_ > 1)) {                           // full/decoder.go:58-61
    useful_++;
    clean_[0] = 0;
    all_clean_ = false;
    touched_[0] = 1;  // never reduced: may be all-zero, test it in the next pass
    return 0;
  }
  rref();                                           // full/decoder.go:63
  useful_ = rows_.size();                           // full/decoder.go:64
  return 0;
}

int DecoderCore::add_many(const uint8_t* vecs, size_t pitch, size_t n, size_t* used) {
  size_t i = 0;
  int st = 0;
  while (i < n) {
    if (is_decoded()) {
      st = 3;  // full/decoder.go:52-54
      break;
    }
    const size_t np = std::min(std::min<size_t>(4, n - i), k_ - rows_.size());
    if (all_clean_ && received_ >= 1 && np >= 2) {
      const size_t c = add_panel(vecs + i * pitch, pitch, np);
      i += c;
      if (c == np) continue;
      // row i is not a diagonal pivot: it takes the literal path below
    }
    if ((st = add(vecs + i * pitch)) != 0) break;
    i++;
  }
  *used = i;
  return st;
}

// np new rows on a state of r diagonal pivots [I_r | X] (all_clean_), as np
// successive rref_clean() calls would add them.  While every new row keeps a
// non-zero diagonal the end state is the reduced row echelon form of
// [coefficients | identity over received rows] with pivots in columns
// 0..r+np-1, which is unique, so the order of the row operations is free:
//  1. each new row drops its columns < r against the old pivots (one pass
//     over the old rows for all new rows);
//  2. the new rows are eliminated among themselves in arrival order; the
//     first whose diagonal is then 0 ends the panel (it and those after it go
//     through add() as usual, from their original vectors);
//  3. the old rows drop the c accepted pivot columns (one rank-c pass).
// Returns c, the rows accepted.
size_t DecoderCore::add_panel(const uint8_t* vecs, size_t pitch, size_t np) {
  const hostgf::Tables& t = T();
  const size_t r = rows_.size(), m0 = received_;
  ensure_tcap(m0 + np);
  const size_t width = k_ + m0 + np;
  uint8_t* pr[4];
  for (size_t p = 0; p < np; p++) {
    pr[p] = free_.back();
    free_.pop_back();
    memcpy(pr[p], vecs + p * pitch, k_);
    memset(pr[p] + k_, 0, tcap_);
    pr[p][k_ + m0 + p] = 1;  // T row = e_(received index)
  }
  uint8_t* vp[4];
  if (r) {
    qbuf_.resize(np * r);
    ptrs_.resize(r);
    for (size_t p = 0; p < np; p++) {
      memcpy(qbuf_.data() + p * r, pr[p], r);
      vp[p] = pr[p] + r;
    }
    for (size_t i = 0; i < r; i++) ptrs_[i] = rows_[i] + r;
    hostgf::accumulate_multi(vp, np, ptrs_.data(), qbuf_.data(), r, r, width - r);
    for (size_t p = 0; p < np; p++) memset(pr[p], 0, r);
  }
  size_t c = np;
  for (size_t p = 0; p < np; p++) {
    for (size_t q = 0; q < p; q++) {
      const uint8_t f = pr[p][r + q];
      if (f) hostgf::axpy(pr[p] + r + q, pr[q] + r + q, width - r - q, f);
    }
    const uint8_t d = pr[p][r + p];
    if (!d) {
      c = p;
      break;
    }
    if (d != 1) hostgf::scale(pr[p] + r + p, width - r - p, t.inv(d));
    for (size_t q = 0; q < p; q++) {
      const uint8_t f = pr[q][r + p];
      if (f) hostgf::axpy(pr[q] + r + p, pr[p] + r + p, width - r - p, f);
    }
  }
  if (c && r) {
    qbuf_.resize(r * c);
    for (size_t j = 0; j < r; j++)
      for (size_t p = 0; p < c; p++) qbuf_[j * c + p] = rows_[j][r + p];
    for (size_t p = 0; p < c; p++) vp[p] = pr[p] + r;
    hostgf::rank_multi(ptrs_.data(), qbuf_.data(), r, vp, c, width - r);
  }
  for (size_t p = np; p-- > c;) free_.push_back(pr[p]);
  for (size_t p = 0; p < c; p++) {
    rows_.push_back(pr[p]);
    clean_[r + p] = 1;
  }
  received_ += c;
  useful_ = rows_.size();
  return c;
}

// Rref (:178-182) on a state whose rows 0..R-2 are the output of the previous
// Rref and row R-1 is the new piece.
void DecoderCore::rref() {
  const size_t R = rows_.size();
  if (all_clean_ && R - 1 < k_) return rref_clean();
  const hostgf::Tables& t = T();
  const size_t last = R - 1;
  const size_t boundary = std::min(R, k_);
  // indices whose row changed identity or content in this forward pass
  size_t dirty_list[4096];
  size_t ndirty = 0;
  std::vector<size_t> dirty_big;
  auto mark = [&](size_t i) {
    if (dirty_[i]) return;
    dirty_[i] = 1;
    if (ndirty < 4096) dirty_list[ndirty++] = i;
    else dirty_big.push_back(i);
  };

  // ---- clean_forward (:15-76).  Every earlier row r satisfies
  // coeffs[j][i] == 0 for j > i (the previous pass left the strict lower
  // triangle zero and zero-row removal only shifts rows up), so in the literal
  // pivot search (:23-35) and elimination (:51-74) the only row below i that
  // can be non-zero in column i is the last one.
  mark(last);
  touched_[last] = 1;  // the new row
  for (size_t i = 0; i < boundary; i++) {
    if (rows_[i][i] == 0) {
      if (i < last && rows_[last][i] != 0) {
        std::swap(rows_[i], rows_[last]);           // :37-48
        std::swap(touched_[i], touched_[last]);
        mark(i);
      } else {
        continue;                                   // :33-35
      }
    }
    if (i < last) {
      const uint8_t c = rows_[last][i];
      if (c != 0) axpy_row(last, i, t.div(c, rows_[i][i]), i);  // :51-74
    }
  }

  // ---- clean_backward (:78-134).  A column i whose pivot row survived the
  // previous pass unchanged with a non-zero diagonal was zeroed above the
  // diagonal then, so only the rows changed by this forward pass can be
  // non-zero there; every other column is scanned in full, as kodr does.
  std::sort(dirty_list, dirty_list + ndirty);
  std::sort(dirty_big.begin(), dirty_big.end());
  for (size_t ii = boundary; ii-- > 0;) {
    const size_t i = ii;
    const uint8_t d = rows_[i][i];
    if (d == 0) continue;                           // :86-88
    const bool full = dirty_[i] || !clean_[i];
    if (full) {
      for (size_t j = 0; j < i; j++) {              // :90-114
        const uint8_t c = rows_[j][i];
        if (c != 0) axpy_row(j, i, t.div(c, d), i);
      }
    } else {
      for (size_t n = 0; n < ndirty; n++) {
        const size_t j = dirty_list[n];
        if (j >= i) break;
        const uint8_t c = rows_[j][i];
        if (c != 0) axpy_row(j, i, t.div(c, d), i);
      }
      for (size_t j : dirty_big) {
        if (j >= i) break;
        const uint8_t c = rows_[j][i];
        if (c != 0) axpy_row(j, i, t.div(c, d), i);
      }
    }
    if (d == 1) continue;                           // :116-118
    // :120-132: coeffs[i][i] = 1, coeffs[i][j>i] *= inv, coded[i] *= inv.
    // Columns < i of row i are zero here, so scaling from column i is exact.
    hostgf::scale(rows_[i] + i, k_ - i + received_, t.inv(d));
  }
  for (size_t n = 0; n < ndirty; n++) dirty_[dirty_list[n]] = 0;
  for (size_t j : dirty_big) dirty_[j] = 0;

  // ---- remove_zero_rows (:136-165): stable removal of all-zero coefficient
  // rows.  Rows no operation touched in this pass were non-zero before it
  // (the previous pass removed every zero row), so only touched rows and the
  // new row need the test; the others keep their order.
  size_t out = 0;
  for (size_t i = 0; i < rows_.size(); i++) {
    const bool t = touched_[i];
    touched_[i] = 0;
    if (t && hostgf::all_zero(rows_[i], k_)) {
      free_.push_back(rows_[i]);
    } else {
      rows_[out++] = rows_[i];
    }
  }
  rows_.resize(out);
  // a row with a non-zero diagonal after this pass has a clean column above
  update_clean();
}

void DecoderCore::update_clean() {
  all_clean_ = true;
  for (size_t i = 0; i < rows_.size(); i++) {
    clean_[i] = (i < k_ && rows_[i][i] != 0) ? 1 : 0;
    all_clean_ = all_clean_ && clean_[i];
  }
}

// Rref when rows 0..r-1 are all diagonal pivots (= 1) with clean columns, i.e.
// the coefficient half is [I_r | X], and row r is the new piece.  Then kodr's
// literal passes reduce to, exactly:
//  clean_forward  (:22-75): no swap; the quotient for pivot i is the new row's
//                 own entry at column i (no other pivot row touches column i),
//                 so the new row becomes  v ^ XOR_i v[i] * row_i  -- one
//                 blocked accumulation;
//  clean_backward (:85-133): column r is eliminated from every row above with
//                 quotient c[j][r] / d (a rank-1 update), row r is scaled by
//                 1/d; every other column is already clean;
//  remove_zero_rows: only the new row can be zero.
void DecoderCore::rref_clean() {
  const hostgf::Tables& t = T();
  const size_t r = rows_.size() - 1, width = k_ + received_;
  uint8_t* v = rows_[r];
  qbuf_.assign(v, v + r);
  // columns < r of the result are exactly zero (pivot i cancels v[i], every
  // other pivot row is 0 there); accumulate only columns [r, k + received)
  ptrs_.resize(r);
  for (size_t i = 0; i < r; i++) ptrs_[i] = rows_[i] + r;
  hostgf::accumulate(v + r, ptrs_.data(), qbuf_.data(), r, width - r);
  memset(v, 0, r);
  const uint8_t d = v[r];
  if (d != 0) {
    // row_j[r..] ^= (c_j / d) * v[r..]  for every j < r, as one pass
    const uint8_t dinv = t.inv(d);
    ptrs_.resize(r);
    for (size_t j = 0; j < r; j++) {
      qbuf_[j] = t.mul(rows_[j][r], dinv);  // == Div(c_j, d) (gf256.go:121-127)
      ptrs_[j] = rows_[j] + r;
    }
    hostgf::rank1(ptrs_.data(), qbuf_.data(), r, v + r, width - r);
    if (d != 1) hostgf::scale(v + r, width - r, t.inv(d));
    clean_[r] = 1;  // all_clean_ stays true
    return;
  }
  // the new row has no pivot on the diagonal: it is either all-zero (dropped)
  // or kept as an off-diagonal row (kodr's rank over-count quirk)
  if (hostgf::all_zero(v, k_)) {
    free_.push_back(v);
    rows_.pop_back();
    return;
  }
  clean_[r] = 0;
  all_clean_ = false;
}

int DecoderCore::piece_available(size_t idx) const {
  if (idx >= k_) return 12;                         // :222-224 ErrPieceOutOfBound
  if (idx >= rows_.size()) return 11;               // :225-227 ErrPieceNotDecodedYet
  if (rows_.size() >= k_) return 0;                 // :229-231
  const uint8_t* c = rows_[idx];                    // :233-252
  for (size_t i = 0; i < k_; i++) {
    if (i == idx) {
      if (c[i] != 1) return 11;
    } else if (c[i] == 0) {
      return 11;
    }
  }
  return 0;
}

void DecoderCore::copy_transform(uint8_t* out, size_t ld) const {
  for (size_t i = 0; i < rows_.size(); i++) memcpy(out + i * ld, rows_[i] + k_, received_);
}

void DecoderCore::copy_coefficients(uint8_t* out) const {
  for (size_t i = 0; i < rows_.size(); i++) memcpy(out + i * k_, rows_[i], k_);
}

}  // namespace kodr_amd
