// decoder_core.cpp -- see decoder_core.hpp.  Line references are to
// kodr_internals/matrix/decoder_state.go unless stated otherwise.
#include "decoder_core.hpp"

#include <stdio.h>
#include <stdlib.h>
#include <time.h>
#include <string.h>

#include <algorithm>

#include "host_gf.hpp"
#include "tune.hpp"

namespace kodr_amd {

using hostgf::T;

DecoderCore::DecoderCore(size_t piece_count) : k_(piece_count), ucnt_(piece_count, 0) {
  ensure_tcap(std::max<size_t>(k_ + 8, 16));
}

// column of the only non-zero byte of v[0..n), or -1 (none, or several)
static int32_t unit_col(const uint8_t* v, size_t n) {
  int32_t c = -1;
  size_t i = 0;
  for (; i + 8 <= n; i += 8) {  // 8 bytes per step; a coded row exits at once
    uint64_t w;
    memcpy(&w, v + i, 8);
    if (!w) continue;
    const unsigned b = (unsigned)__builtin_ctzll(w) >> 3;
    if (c >= 0 || (w >> (8 * b) >> 8)) return -1;  // a second non-zero byte
    c = (int32_t)(i + b);
  }
  for (; i < n; i++) {
    if (!v[i]) continue;
    if (c >= 0) return -1;
    c = (int32_t)i;
  }
  return c;
}

void DecoderCore::push_row(uint8_t* row, int32_t p, int32_t t) {
  rows_.push_back(row);
  up_.push_back(p);
  ut_.push_back(t);
  if (p >= 0) ucnt_[p]++;
  else ndense_++;
}

void DecoderCore::forget_row(size_t pos) {
  if (up_[pos] >= 0) ucnt_[up_[pos]]--;
  else ndense_--;
}

void DecoderCore::pop_row() {
  forget_row(rows_.size() - 1);
  rows_.pop_back();
  up_.pop_back();
  ut_.pop_back();
}

void DecoderCore::swap_rows(size_t a, size_t b) {
  std::swap(rows_[a], rows_[b]);
  std::swap(up_[a], up_[b]);
  std::swap(ut_[a], ut_[b]);
  std::swap(touched_[a], touched_[b]);
}

// row `pos` is about to change: it is no longer known to be a unit row
void DecoderCore::make_dense(size_t pos) {
  if (up_[pos] < 0) return;
  ucnt_[up_[pos]]--;
  up_[pos] = -1;
  ndense_++;
  dense_pos_.push_back(pos);
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
// A unit source row has two non-zero bytes: the same result in two byte ops.
void DecoderCore::axpy_row(size_t dst, size_t src, uint8_t q, size_t from) {
  const int32_t p = up_[src];
  if (p >= 0) {
    const hostgf::Tables& t = T();
    uint8_t* d = rows_[dst];
    const uint8_t* s = rows_[src];
    if ((size_t)p >= from) d[p] ^= t.mul(q, s[p]);
    d[k_ + ut_[src]] ^= t.mul(q, s[k_ + ut_[src]]);
  } else {
    hostgf::axpy(rows_[dst] + from, rows_[src] + from, k_ - from + received_, q);
  }
  make_dense(dst);
  touched_[dst] = 1;
}

// rows_[i][from..) *= q (a unit row stays a unit row)
void DecoderCore::scale_row(size_t i, size_t from, uint8_t q) {
  const int32_t p = up_[i];
  if (p >= 0) {
    const hostgf::Tables& t = T();
    uint8_t* r = rows_[i];
    if ((size_t)p >= from) r[p] = t.mul(r[p], q);
    r[k_ + ut_[i]] = t.mul(r[k_ + ut_[i]], q);
    return;
  }
  hostgf::scale(rows_[i] + from, k_ - from + received_, q);
}

int DecoderCore::add(const uint8_t* vec) {
  if (is_decoded()) return 3;                       // full/decoder.go:52-54
  if (received_ >= 2 && append_unit(vec)) return 0;
  ensure_tcap(received_ + 1);
  uint8_t* row = free_.back();                      // :205-208 (append)
  free_.pop_back();
  memcpy(row, vec, k_);
  memset(row + k_, 0, tcap_);
  row[k_ + received_] = 1;                          // T row = e_received
  push_row(row, unit_col(vec, k_), (int32_t)received_);
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
  if (received_ == 0 && n >= k_ && (solve_systematic_batch(vecs, pitch) || solve_full_batch(vecs, pitch))) {
    *used = k_;
    return n > k_ ? 3 : 0;  // full/decoder.go:52-54 for the rows past k
  }
  size_t i = 0;
  int st = 0;
  while (i < n) {
    if (is_decoded()) {
      st = 3;  // full/decoder.go:52-54
      break;
    }
    if (received_ >= 2 && ndense_ == 0 && append_unit(vecs + i * pitch)) {
      i++;
      continue;
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

// A systematic piece a*e_q on a state that an Rref produced (received >= 2)
// whose rows are all unit rows, none with pivot q, with q >= R (the new row's
// index).  kodr's passes then leave every existing row as it is:
// clean_forward (:15-76) finds the new row zero in every column i < q, so it
// neither swaps nor eliminates; clean_backward (:78-134) finds column q zero
// above the new row and every other column as the previous pass left it;
// remove_zero_rows finds nothing.  What remains is the append and, when q is
// the diagonal (q == R), the normalization of the new row (:116-132).
bool DecoderCore::append_unit(const uint8_t* vec) {
  if (ndense_ != 0) return false;
  const size_t R = rows_.size();
  const int32_t q = unit_col(vec, k_);
  if (q < 0 || (size_t)q < R || ucnt_[q] != 0) return false;
  ensure_tcap(received_ + 1);
  uint8_t* row = free_.back();
  free_.pop_back();
  memset(row, 0, k_ + tcap_);
  const uint8_t a = vec[q];
  const bool diag = (size_t)q == R;
  row[q] = diag ? 1 : a;
  row[k_ + received_] = diag ? T().inv(a) : 1;
  push_row(row, q, (int32_t)received_);
  received_++;
  clean_[R] = diag ? 1 : 0;  // a diagonal pivot with a zero column above
  all_clean_ = all_clean_ && diag;
  touched_[R] = 0;
  useful_ = rows_.size();
  return true;
}

// A fresh decoder handed k or more rows whose first k coding vectors C are
// linearly independent ends, whatever route kodr's passes take, in the state
// [I | C^-1] with all k rows accepted: an independent row never becomes zero,
// rank counts kept rows, and the kept k x k coefficient half has a zero strict
// lower triangle, so it is upper triangular, invertible, hence diagonal, and
// the backward pass normalizes it (gf_elim.hip, full batches).  For a
// systematic batch -- unit rows a*e_p with distinct pivots and m dense rows
// among the first k, m small -- C^-1 follows from the m x m block X of the
// dense rows on the m columns no unit row covers ("lost"):
//  * column p of a unit row (arrival i, scale a): T[p] = inv(a) * e_i;
//  * lost column j (index j' among the lost ones): with x = row j' of X^-1,
//    w = sum_d x_d * dense row d is e_j plus entries w[p] on unit columns, so
//    T[j] = sum_d x_d * e_arrival(d) + sum_p w[p] * inv(a_p) * e_arrival(p).
// Returns false (nothing changed) when the batch is not of that form or C is
// singular; add_many then takes kodr's route row by row.
bool DecoderCore::solve_systematic_batch(const uint8_t* vecs, size_t pitch) {
  const size_t k = k_;
  if (received_ != 0 || k < 2) return false;
  const size_t mmax = std::max<size_t>(8, k / 8);
  std::vector<int32_t> unit_at(k, -1);  // arrival index of the unit row with pivot p
  std::vector<size_t> dense;
  for (size_t i = 0; i < k; i++) {
    const int32_t p = unit_col(vecs + i * pitch, k);
    if (p < 0) {
      if (dense.size() == mmax) return false;
      dense.push_back(i);
    } else {
      if (unit_at[p] >= 0) return false;  // two rows on one pivot: C singular
      unit_at[p] = (int32_t)i;
    }
  }
  const size_t m = dense.size();
  if (m == 0 || m == k) return false;  // no dense rows: the unit appends are as cheap; none: panels
  std::vector<size_t> lost;
  for (size_t c = 0; c < k; c++)
    if (unit_at[c] < 0) lost.push_back(c);
  // [X | I_m] -> [I_m | X^-1] by Gauss-Jordan with a pivot search
  const hostgf::Tables& t = T();
  const size_t w2 = 2 * m;
  std::vector<uint8_t> M(m * w2, 0);
  for (size_t r = 0; r < m; r++) {
    const uint8_t* v = vecs + dense[r] * pitch;
    for (size_t c = 0; c < m; c++) M[r * w2 + c] = v[lost[c]];
    M[r * w2 + m + r] = 1;
  }
  for (size_t c = 0; c < m; c++) {
    size_t pr = c;
    while (pr < m && !M[pr * w2 + c]) pr++;
    if (pr == m) return false;  // X singular, so is C
    if (pr != c)
      for (size_t q = 0; q < w2; q++) std::swap(M[pr * w2 + q], M[c * w2 + q]);
    hostgf::scale(&M[c * w2], w2, t.inv(M[c * w2 + c]));
    for (size_t r = 0; r < m; r++)
      if (r != c && M[r * w2 + c]) hostgf::axpy(&M[r * w2], &M[c * w2], w2, M[r * w2 + c]);
  }
  // state rows [e_j | T[j]], T over the k accepted rows in arrival order
  const size_t w = 2 * k;
  std::vector<uint8_t> S(k * w, 0), wrow(k);
  for (size_t p = 0; p < k; p++) {
    S[p * w + p] = 1;
    if (unit_at[p] >= 0) S[p * w + k + unit_at[p]] = t.inv(vecs[(size_t)unit_at[p] * pitch + p]);
  }
  for (size_t jj = 0; jj < m; jj++) {
    const uint8_t* x = &M[jj * w2 + m];
    uint8_t* row = &S[lost[jj] * w];
    std::fill(wrow.begin(), wrow.end(), 0);
    for (size_t d = 0; d < m; d++) {
      if (!x[d]) continue;
      row[k + dense[d]] = x[d];
      hostgf::axpy(wrow.data(), vecs + dense[d] * pitch, k, x[d]);
    }
    for (size_t p = 0; p < k; p++)
      if (unit_at[p] >= 0 && wrow[p])
        row[k + unit_at[p]] = t.mul(wrow[p], t.inv(vecs[(size_t)unit_at[p] * pitch + p]));
  }
  return load_rref(S.data(), w, k);
}

// ---- full batches: [C | I] -> [I | C^-1] by blocked Gauss-Jordan ----------
// Same premise as solve_systematic_batch: a fresh decoder handed k or more
// rows whose first k vectors C are independent ends in [I | C^-1], whatever
// route kodr's passes take, so any exact inversion gives kodr's state byte for
// byte.  The inversion runs on [C | I] in the decoder's own row slots, in
// panels of kFullNB columns:
//  A: pick kFullNB rows whose panel block is invertible -- rows that are no
//     pivot yet, in index order, each reduced against the rows picked so far
//     (Gauss-Jordan on [panel | tracking] vectors, so the tracking half ends
//     as S, the inverse of the picked rows' panel block);
//  B: per 64-byte column chunk: the new pivot rows S x (picked rows), and
//     every other row ^= Q[row] x (new pivot rows), Q = the row's panel bytes.
// Columns left of the panel never change (zero in every picked row), the
// panel's own columns end as 0 in every other row and as the identity in the
// picked ones (not stored: nothing reads them again, and the final rows'
// coefficient halves are written as I at the end), and T column t stays zero
// in every row until row t is picked (each unpicked row's own identity entry
// aside), so a row's bytes in play are [jb + nb, k + tmax): k bytes when the
// picked rows are the lowest unpicked ones, 4 full chunks at k = 256.  A
// panel with too few independent rows means C is singular: nothing is kept
// and add_many takes kodr's route.  One thread: the matrix is ~160 KB, and a
// spin-barrier thread pool splitting its 64-byte column chunks over cores
// (measured on the box: 2 threads 365 us, 8 threads 456 us, against 88 us on
// one) moved more cache lines between cores per panel than it saved.  Round
// 3 re-tried it with every cache line of every row owned by one thread for
// the whole solve (64-byte-aligned slots, the panel bytes passed through a
// 4 KB buffer): 199-255 us on 2-8 threads against 88 us on one
// (tools/probe/solve_threads.cpp, profiles/r03/solve_threads/).
namespace {

double now_us() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

constexpr int kFullNB = 16;
// Below this the 4-row panels of add_panel are as fast or faster on the box's
// EPYC (tools/full_solve_mink.sh, profiles/r02/elim/full_solve_min_k.log: equal
// within 1-3 us at k = 64-192, k = 224 route 55 us vs 68 blocked; k = 256 105
// vs 79-81, 14 us of it the panels' pivot picking, 63 us the row updates).
// KODR_FULL_MIN_K overrides it (measurements).
constexpr size_t kFullMinK = 240;

struct FullSolve {
  size_t k = 0;
  std::vector<uint8_t*> rows;           // physical rows, [C | I] at start
  std::vector<int16_t> cur;             // per row: panel column it pivots in this block, or -1
  std::vector<uint8_t> used;            // per row: a pivot already (this or an earlier block)
  std::vector<int32_t> pivrow;          // per column: its pivot row
  uint8_t S[kFullNB][kFullNB];          // S[q][t]: new pivot row q = sum_t S[q][t] * picked row t
  int32_t brow[kFullNB];                // picked rows
  int bpiv[kFullNB];                    // panel column of picked row q
  int nb = 0;
  size_t tmax = 0;                      // T columns [0, tmax) can be non-zero in a row not picked yet

  bool phase_a(size_t jb) {
    const hostgf::Tables& t = T();
    for (int q = 0; q < nb; q++) cur[brow[q]] = -1;  // the previous block's pivots
    nb = (int)std::min<size_t>(kFullNB, k - jb);
    alignas(64) uint8_t bas[kFullNB][2 * kFullNB];
    int nbas = 0;
    for (size_t i = 0; i < k && nbas < nb; i++) {
      if (used[i]) continue;
      alignas(64) uint8_t v[2 * kFullNB] = {0};
      memcpy(v, rows[i] + jb, nb);
      v[kFullNB + nbas] = 1;
      for (int q = 0; q < nbas; q++)
        if (const uint8_t c = v[bpiv[q]]) hostgf::axpy32(v, bas[q], c);
      int pc = -1;
      for (int c = 0; c < nb && pc < 0; c++)
        if (v[c]) pc = c;
      if (pc < 0) continue;  // dependent on the rows picked so far in this panel
      if (v[pc] != 1) hostgf::scale32(v, t.inv(v[pc]));
      for (int q = 0; q < nbas; q++)
        if (const uint8_t c = bas[q][pc]) hostgf::axpy32(bas[q], v, c);
      memcpy(bas[nbas], v, sizeof(v));
      bpiv[nbas] = pc;
      brow[nbas] = (int32_t)i;
      nbas++;
    }
    if (nbas < nb) return false;
    for (int q = 0; q < nb; q++) {
      memcpy(S[q], bas[q] + kFullNB, kFullNB);
      cur[brow[q]] = (int16_t)bpiv[q];
      used[brow[q]] = 1;
      tmax = std::max<size_t>(tmax, (size_t)brow[q] + 1);
      pivrow[jb + bpiv[q]] = brow[q];
    }
    return true;
  }

  void phase_b(size_t jb) {
    const size_t beg = jb + nb, end = k + tmax;
    for (size_t o = beg; o < end; o += 64)
      hostgf::panel_update<kFullNB>(rows.data(), k, o, std::min<size_t>(64, end - o), jb, brow, bpiv, S, nb,
                                    cur.data());
  }
};

}  // namespace

bool DecoderCore::solve_full_batch(const uint8_t* vecs, size_t pitch) {
  const size_t k = k_;
  static const bool enabled = !kodr_amd::tune_env("KODR_FULL_SOLVE") || atoi(kodr_amd::tune_env("KODR_FULL_SOLVE")) != 0;
  static const size_t min_k = kodr_amd::tune_env("KODR_FULL_MIN_K") ? (size_t)atol(kodr_amd::tune_env("KODR_FULL_MIN_K")) : kFullMinK;
  if (!enabled || received_ != 0 || k < min_k || !hostgf::have_gfni512()) return false;
  ensure_tcap(k);
  FullSolve F;
  F.k = k;
  F.rows.resize(k);
  for (size_t i = 0; i < k; i++) {
    uint8_t* r = free_[free_.size() - 1 - i];
    memcpy(r, vecs + i * pitch, k);
    memset(r + k, 0, tcap_);
    r[k + i] = 1;
    F.rows[i] = r;
  }
  F.cur.assign(k, -1);
  F.used.assign(k, 0);
  F.pivrow.assign(k, -1);
  static const bool timing = kodr_amd::tune_env("KODR_FULL_SOLVE") && atoi(kodr_amd::tune_env("KODR_FULL_SOLVE")) == 2;
  double ta = 0, tb = 0;
  for (size_t jb = 0; jb < k; jb += kFullNB) {
    const double t0 = timing ? now_us() : 0;
    if (!F.phase_a(jb)) return false;  // C singular; the slots are still free: nothing changed
    const double t1 = timing ? now_us() : 0;
    F.phase_b(jb);
    if (timing) {
      ta += t1 - t0;
      tb += now_us() - t1;
    }
  }
  if (timing) fprintf(stderr, "solve_full_batch k=%zu: panels %.1f us, updates %.1f us\n", k, ta, tb);
  free_.resize(free_.size() - k);
  for (size_t c = 0; c < k; c++) {
    uint8_t* row = F.rows[F.pivrow[c]];
    memset(row, 0, k);  // [I | C^-1]: the panels' columns were not stored
    row[c] = 1;
    push_row(row, -1, 0);
    clean_[c] = 1;
    touched_[c] = 0;
  }
  received_ = k;
  useful_ = k;
  all_clean_ = true;
  return true;
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
  if (c && r && ndense_ >= r) {  // every old row dense: one pass over all of them
    qbuf_.resize(r * c);
    for (size_t j = 0; j < r; j++)
      for (size_t p = 0; p < c; p++) qbuf_[j * c + p] = rows_[j][r + p];
    for (size_t p = 0; p < c; p++) vp[p] = pr[p] + r;
    hostgf::rank_multi(ptrs_.data(), qbuf_.data(), r, vp, c, width - r);
  } else if (c && r && ndense_) {  // unit rows j < r are e_j: zero in the new pivot columns
    // only rows with a non-zero entry in the c new pivot columns change
    qbuf_.resize(r * c);
    size_t nr = 0;
    for (size_t j = 0; j < r; j++) {
      bool any = false;
      for (size_t p = 0; p < c; p++) {
        qbuf_[nr * c + p] = rows_[j][r + p];
        any = any || rows_[j][r + p];
      }
      if (!any) continue;
      ptrs_[nr++] = rows_[j] + r;
      make_dense(j);
    }
    for (size_t p = 0; p < c; p++) vp[p] = pr[p] + r;
    if (nr) hostgf::rank_multi(ptrs_.data(), qbuf_.data(), nr, vp, c, width - r);
  }
  for (size_t p = np; p-- > c;) free_.push_back(pr[p]);
  for (size_t p = 0; p < c; p++) {
    push_row(pr[p], -1, 0);
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
    if (up_[i] >= 0 ? up_[i] != (int32_t)i : rows_[i][i] == 0) {
      if (i < last && rows_[last][i] != 0) {
        swap_rows(i, last);                         // :37-48
        mark(i);
      } else {
        continue;                                   // :33-35
      }
    }
    if (i < last) {
      const uint8_t c = rows_[last][i];
      if (c == 0) continue;
      if (up_[i] == (int32_t)i) {
        // unit pivot a*e_i | b*e_t: the new row's column i cancels and its T
        // column t takes (c / a) * b -- axpy_row's two bytes, inline
        uint8_t* v = rows_[last];
        const uint8_t* s = rows_[i];
        v[i] = 0;
        v[k_ + ut_[i]] ^= t.mul(t.div(c, s[i]), s[k_ + ut_[i]]);
        make_dense(last);
        touched_[last] = 1;
      } else {
        axpy_row(last, i, t.div(c, rows_[i][i]), i);  // :51-74
      }
    }
  }

  // ---- clean_backward (:78-134).  A column i whose pivot row survived the
  // previous pass unchanged with a non-zero diagonal was zeroed above the
  // diagonal then, so only the rows changed by this forward pass can be
  // non-zero there; every other column is scanned in full, as kodr does.
  //
  // Within column i only rows that can be non-zero there are visited: dense
  // rows, and unit rows whose pivot is i (a unit row is zero everywhere else).
  // Each elimination changes only its target row, so the order of the rows
  // within a column does not matter.
  std::sort(dirty_list, dirty_list + ndirty);
  std::sort(dirty_big.begin(), dirty_big.end());
  dense_pos_.clear();
  for (size_t j = 0; j < rows_.size(); j++)
    if (up_[j] < 0) dense_pos_.push_back(j);
  // that set is also exact for a clean column; take it there too when it is
  // smaller than the rows this forward pass changed (a systematic state after
  // a coded piece filled a gap: every unit row after the gap moved)
  const bool sparse = dense_pos_.size() < ndirty + dirty_big.size();
  for (size_t ii = boundary; ii-- > 0;) {
    const size_t i = ii;
    if (up_[i] >= 0 && up_[i] != (int32_t)i) continue;  // a unit row off its diagonal
    const uint8_t d = rows_[i][i];
    if (d == 0) continue;                           // :86-88
    const int32_t ci = (int32_t)i;
    const bool full = dirty_[i] || !clean_[i];
    if (full || sparse) {                           // :90-114
      const bool unit_i = up_[i] == ci;
      const uint8_t tq = unit_i ? rows_[i][k_ + ut_[i]] : 0;
      for (size_t n = 0; n < dense_pos_.size(); n++) {
        const size_t j = dense_pos_[n];
        if (j >= i) continue;
        uint8_t* rj = rows_[j];
        const uint8_t c = rj[i];
        if (c == 0) continue;
        if (unit_i) {  // axpy_row from a unit pivot, inline (row j is dense already)
          rj[i] = 0;
          rj[k_ + ut_[i]] ^= t.mul(t.div(c, d), tq);
          touched_[j] = 1;
        } else {
          axpy_row(j, i, t.div(c, d), i);
        }
      }
      // rows below i are zero in column i, so every unit row with pivot i
      // other than row i itself lies above it
      if (ucnt_[i] > (up_[i] == ci ? 1u : 0u)) {
        for (size_t j = 0; j < i; j++)
          if (up_[j] == ci) axpy_row(j, i, t.div(rows_[j][i], d), i);
      }
    } else {
      for (size_t n = 0; n < ndirty; n++) {
        const size_t j = dirty_list[n];
        if (j >= i) break;
        if (up_[j] >= 0 && up_[j] != ci) continue;
        const uint8_t c = rows_[j][i];
        if (c != 0) axpy_row(j, i, t.div(c, d), i);
      }
      for (size_t j : dirty_big) {
        if (j >= i) break;
        if (up_[j] >= 0 && up_[j] != ci) continue;
        const uint8_t c = rows_[j][i];
        if (c != 0) axpy_row(j, i, t.div(c, d), i);
      }
    }
    if (d == 1) continue;                           // :116-118
    // :120-132: coeffs[i][i] = 1, coeffs[i][j>i] *= inv, coded[i] *= inv.
    // Columns < i of row i are zero here, so scaling from column i is exact.
    scale_row(i, i, t.inv(d));
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
      forget_row(i);
      free_.push_back(rows_[i]);
    } else {
      rows_[out] = rows_[i];
      up_[out] = up_[i];
      ut_[out] = ut_[i];
      out++;
    }
  }
  rows_.resize(out);
  up_.resize(out);
  ut_.resize(out);
  // a row with a non-zero diagonal after this pass has a clean column above
  update_clean();
}

void DecoderCore::update_clean() {
  all_clean_ = true;
  for (size_t i = 0; i < rows_.size(); i++) {
    clean_[i] = (i < k_ && (up_[i] >= 0 ? up_[i] == (int32_t)i : rows_[i][i] != 0)) ? 1 : 0;
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
  // columns < r of the result are exactly zero (pivot i cancels v[i], every
  // other pivot row is 0 there); accumulate only columns [r, k + received).
  // A new row already zero there (a systematic piece e_q, q >= r) is unchanged.
  if (!hostgf::all_zero(v, r)) {
    qbuf_.assign(v, v + r);
    ptrs_.resize(r);
    for (size_t i = 0; i < r; i++) ptrs_[i] = rows_[i] + r;
    hostgf::accumulate(v + r, ptrs_.data(), qbuf_.data(), r, width - r);
    memset(v, 0, r);
    make_dense(r);
  }
  const uint8_t d = v[r];
  if (d != 0) {
    // row_j[r..] ^= (c_j / d) * v[r..]  for every j < r with c_j != 0, as
    // one pass; unit rows j < r are e_j, zero in column r
    const uint8_t dinv = t.inv(d);
    size_t nr = 0;
    if (ndense_ > r) {  // every row dense (the new one included): one pass
      qbuf_.resize(r);
      ptrs_.resize(r);
      for (size_t j = 0; j < r; j++) {
        qbuf_[j] = t.mul(rows_[j][r], dinv);  // == Div(c_j, d) (gf256.go:121-127)
        ptrs_[j] = rows_[j] + r;
      }
      nr = r;
    } else if (ndense_) {
      qbuf_.resize(r);
      ptrs_.resize(r);
      for (size_t j = 0; j < r; j++) {
        const uint8_t c = rows_[j][r];
        if (!c) continue;
        qbuf_[nr] = t.mul(c, dinv);  // == Div(c_j, d) (gf256.go:121-127)
        ptrs_[nr++] = rows_[j] + r;
        make_dense(j);
      }
    }
    if (nr) hostgf::rank1(ptrs_.data(), qbuf_.data(), nr, v + r, width - r);
    if (d != 1) scale_row(r, r, t.inv(d));
    clean_[r] = 1;  // all_clean_ stays true
    return;
  }
  // the new row has no pivot on the diagonal: it is either all-zero (dropped)
  // or kept as an off-diagonal row (kodr's rank over-count quirk)
  if (hostgf::all_zero(v, k_)) {
    free_.push_back(v);
    pop_row();
    return;
  }
  clean_[r] = 0;
  all_clean_ = false;
}

bool DecoderCore::load_rref(const uint8_t* state, size_t pitch, size_t c) {
  if (received_ != 0 || c < 2 || c > k_) return false;
  ensure_tcap(c);
  for (size_t i = 0; i < c; i++) {
    const uint8_t* src = state + i * pitch;
    if (src[i] != 1) return false;  // not the RREF with diagonal pivots: refuse (state untouched so far)
  }
  for (size_t i = 0; i < c; i++) {
    uint8_t* row = free_.back();
    free_.pop_back();
    memcpy(row, state + i * pitch, k_ + c);
    memset(row + k_ + c, 0, tcap_ - c);
    push_row(row, -1, 0);
    clean_[i] = 1;
    touched_[i] = 0;
  }
  received_ = c;
  useful_ = c;
  all_clean_ = true;
  return true;
}

bool DecoderCore::load_inverse(const uint8_t* tinv, size_t pitch) {
  const size_t k = k_;
  if (received_ != 0 || k < 2) return false;
  if (pitch == k) {
    pinv_.assign(tinv, tinv + k * k);  // (one pass: no zero fill before the copy)
  } else {
    pinv_.resize(k * k);
    for (size_t i = 0; i < k; i++) memcpy(pinv_.data() + i * k, tinv + i * pitch, k);
  }
  pinv_on_ = true;
  received_ = k;
  useful_ = k;
  all_clean_ = true;
  return true;
}

void DecoderCore::expand_inverse() {
  const size_t k = k_;
  pinv_on_ = false;
  ensure_tcap(k);
  for (size_t i = 0; i < k; i++) {
    uint8_t* row = free_.back();
    free_.pop_back();
    memset(row, 0, k);
    row[i] = 1;
    memcpy(row + k, pinv_.data() + i * k, k);
    memset(row + 2 * k, 0, tcap_ - k);
    push_row(row, -1, 0);
    clean_[i] = 1;
    touched_[i] = 0;
  }
  std::vector<uint8_t>().swap(pinv_);
}

bool DecoderCore::load_continued(const uint8_t* state, size_t pitch, bool inverse) {
  const size_t k = k_, r = received_, c = k;
  if (r == 0 || r >= k || rows_.size() != r) return false;
  if (!inverse)
    for (size_t i = 0; i < c; i++)
      if (state[i * pitch + i] != 1) return false;
  ensure_tcap(c);  // may move the rows: their pointers are read after it
  std::vector<const uint8_t*> tr(r);
  for (size_t m = 0; m < r; m++) tr[m] = rows_[m] + k;  // T_r, row m of M
  const size_t w = k + c;
  std::vector<uint8_t> buf(c * w, 0);
  const size_t f0 = inverse ? 0 : k;  // F's offset in a state row
  for (size_t i = 0; i < c; i++) {
    uint8_t* o = buf.data() + i * w;
    const uint8_t* f = state + i * pitch + f0;
    if (inverse) o[i] = 1;
    else memcpy(o, state + i * pitch, k);
    memcpy(o + k + r, f + r, c - r);  // the batch's columns
  }
  for (size_t i = 0; i < c; i += 4) {  // F[:, :r] x T_r, four output rows per pass over T_r
    const size_t np = std::min<size_t>(4, c - i);
    uint8_t* v[4];
    for (size_t p = 0; p < np; p++) v[p] = buf.data() + (i + p) * w + k;
    hostgf::accumulate_multi(v, np, tr.data(), state + i * pitch + f0, pitch, r, r);
  }
  for (uint8_t* row : rows_) free_.push_back(row);
  rows_.clear();
  up_.clear();
  ut_.clear();
  std::fill(ucnt_.begin(), ucnt_.end(), 0u);
  ndense_ = 0;
  dense_pos_.clear();
  for (size_t i = 0; i < c; i++) {
    uint8_t* row = free_.back();
    free_.pop_back();
    memcpy(row, buf.data() + i * w, w);
    memset(row + w, 0, tcap_ - c);
    push_row(row, -1, 0);
    clean_[i] = 1;
    touched_[i] = 0;
  }
  received_ = c;
  useful_ = c;
  all_clean_ = true;
  return true;
}

size_t DecoderCore::decoded(std::vector<int32_t>* row_of, std::vector<uint8_t>* scale) const {
  row_of->assign(k_, -1);
  scale->assign(k_, 0);
  if (pinv_on_) {  // [I | C^-1]: row j is e_j
    for (size_t j = 0; j < k_; j++) (*row_of)[j] = (int32_t)j, (*scale)[j] = 1;
    return k_;
  }
  size_t n = 0;
  for (size_t i = 0; i < rows_.size(); i++) {
    const int32_t p = up_[i] >= 0 ? up_[i] : unit_col(rows_[i], k_);
    if (p < 0 || (*row_of)[p] >= 0) continue;
    (*row_of)[p] = (int32_t)i;
    (*scale)[p] = rows_[i][p];
    n++;
  }
  return n;
}

int DecoderCore::piece_available(size_t idx) const {
  if (idx >= k_) return 12;                         // :222-224 ErrPieceOutOfBound
  if (idx >= rank()) return 11;                     // :225-227 ErrPieceNotDecodedYet
  if (rank() >= k_) return 0;                       // :229-231
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
  if (pinv_on_) {
    for (size_t i = 0; i < k_; i++) memcpy(out + i * ld, pinv_.data() + i * k_, k_);
    return;
  }
  for (size_t i = 0; i < rows_.size(); i++) memcpy(out + i * ld, rows_[i] + k_, received_);
}

void DecoderCore::copy_coefficients(uint8_t* out) const {
  if (pinv_on_) {
    memset(out, 0, k_ * k_);
    for (size_t i = 0; i < k_; i++) out[i * k_ + i] = 1;
    return;
  }
  for (size_t i = 0; i < rows_.size(); i++) memcpy(out + i * k_, rows_[i], k_);
}

}  // namespace kodr_amd
