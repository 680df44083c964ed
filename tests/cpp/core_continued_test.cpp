// DecoderCore::load_continued (and load_inverse's lazy block) on the CPU (kodr_amd/csrc/decoder_core.cpp):
// a decoder holding r rows takes the state of M = [its r coefficient rows ;
// the next k - r vectors] inverted elsewhere, and must end exactly where
// kodr's own route (decoder_state.go:15-182, here DecoderCore::add row by
// row, itself tied to the oracle by tests/test_capi_host.py) ends: [I | C^-1]
// with the same transform over the arrivals.  M^-1 comes from a second
// DecoderCore fed M's rows (its state is [I | M^-1]).  Prints "ok (0
// failures)".
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <random>
#include <vector>

#include "../../kodr_amd/csrc/decoder_core.hpp"

using kodr_amd::DecoderCore;

static int failures = 0;
#define CHECK(c, ...)                                  \
  do {                                                 \
    if (!(c)) {                                        \
      failures++;                                      \
      fprintf(stderr, "FAIL %s:%d ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                    \
      fprintf(stderr, "\n");                           \
    }                                                  \
  } while (0)

static std::vector<uint8_t> transform(const DecoderCore& d) {
  std::vector<uint8_t> t(d.rank() * d.received());
  d.copy_transform(t.data(), d.received());
  return t;
}

static std::vector<uint8_t> coefficients(const DecoderCore& d) {
  std::vector<uint8_t> c(d.rank() * d.piece_count());
  d.copy_coefficients(c.data());
  return c;
}

// kind 0: dense vectors; 1: the first r arrivals are scaled unit vectors
// (a systematic prefix, unit-row bookkeeping); 2: arrival 1 repeats arrival 0
// (a dependent row: load_continued must refuse)
static void run_case(size_t k, size_t r, int kind, bool inverse, std::mt19937& rng) {
  std::vector<uint8_t> C(k * k);
  for (;;) {
    for (auto& b : C) b = (uint8_t)(rng() & 0xff);
    if (kind == 1)
      for (size_t i = 0; i < r; i++) {
        memset(&C[i * k], 0, k);
        C[i * k + i] = (uint8_t)(1 + rng() % 255);
      }
    if (kind == 2 && r >= 2) memcpy(&C[k], &C[0], k);
    DecoderCore probe(k);
    for (size_t i = 0; i < k; i++) probe.add(&C[i * k]);
    if (kind == 2 || probe.is_decoded()) break;  // an invertible C (kind 2 is singular by design)
  }
  // kodr's route: every arrival through add()
  DecoderCore ref(k);
  for (size_t i = 0; i < k; i++) ref.add(&C[i * k]);
  // the continued decoder: r arrivals, then the state of M from elsewhere
  DecoderCore d(k);
  for (size_t i = 0; i < r; i++) d.add(&C[i * k]);
  const size_t rank0 = d.rank(), recv0 = d.received();
  const std::vector<uint8_t> coef0 = coefficients(d), t0 = transform(d);
  std::vector<uint8_t> M(k * k);
  for (size_t j = 0; j < r && j < d.rank(); j++) memcpy(&M[j * k], d.coeff_row(j), k);
  for (size_t j = d.rank(); j < k; j++) memcpy(&M[j * k], &C[(j - d.rank() + r) * k], k);
  DecoderCore inv(k);
  for (size_t j = 0; j < k; j++) inv.add(&M[j * k]);
  if (!inv.is_decoded()) {  // M singular: the engine leaves the host route to kodr
    CHECK(kind == 2, "k=%zu r=%zu kind=%d: M singular for an invertible C", k, r, kind);
    return;
  }
  const std::vector<uint8_t> minv = transform(inv);  // k x k, columns in M's row order
  std::vector<uint8_t> state;
  size_t pitch;
  if (inverse) {
    state = minv;
    pitch = k;
  } else {  // whole state rows [I | M^-1] at a padded pitch
    pitch = 2 * k + 8;
    state.assign(k * pitch, 0xEE);
    for (size_t i = 0; i < k; i++) {
      memset(&state[i * pitch], 0, k);
      state[i * pitch + i] = 1;
      memcpy(&state[i * pitch + k], &minv[i * k], k);
    }
  }
  const bool ok = d.load_continued(state.data(), pitch, inverse);
  if (kind == 2) {
    CHECK(!ok, "k=%zu r=%zu: a decoder with a dependent row took the continued state", k, r);
    CHECK(d.rank() == rank0 && d.received() == recv0 && coefficients(d) == coef0 && transform(d) == t0,
          "k=%zu r=%zu: a refused load changed the state", k, r);
    return;
  }
  CHECK(ok, "k=%zu r=%zu kind=%d inverse=%d: load refused", k, r, kind, (int)inverse);
  if (!ok) return;
  CHECK(d.is_decoded() && d.useful() == ref.useful() && d.received() == ref.received() && d.rank() == ref.rank(),
        "k=%zu r=%zu kind=%d: counters", k, r, kind);
  CHECK(coefficients(d) == coefficients(ref), "k=%zu r=%zu kind=%d: coefficients", k, r, kind);
  CHECK(transform(d) == transform(ref), "k=%zu r=%zu kind=%d inverse=%d: transform", k, r, kind, (int)inverse);
  // later calls behave as kodr's: the next AddPiece is refused once decoded
  std::vector<uint8_t> extra(k, 7);
  CHECK(d.add(extra.data()) == 3, "k=%zu r=%zu: AddPiece after the load not refused", k, r);
}

// DecoderCore::load_inverse keeps [I | C^-1] as one block until a row is
// read: every accessor before and after the rows are spread must answer as a
// decoder that took the k arrivals through add() (kodr's route)
static void run_inverse_case(size_t k, std::mt19937& rng) {
  std::vector<uint8_t> C(k * k);
  DecoderCore ref(k);
  for (;;) {
    for (auto& b : C) b = (uint8_t)(rng() & 0xff);
    DecoderCore probe(k);
    for (size_t i = 0; i < k; i++) probe.add(&C[i * k]);
    if (probe.is_decoded()) break;
  }
  for (size_t i = 0; i < k; i++) ref.add(&C[i * k]);
  const std::vector<uint8_t> tref = transform(ref), cref = coefficients(ref);
  // C^-1 at a padded pitch
  const size_t pitch = k + 5;
  std::vector<uint8_t> tinv(k * pitch, 0xEE);
  for (size_t i = 0; i < k; i++) memcpy(&tinv[i * pitch], &tref[i * k], k);
  for (int read_rows_first = 0; read_rows_first < 2; read_rows_first++) {
    DecoderCore d(k);
    CHECK(d.load_inverse(tinv.data(), pitch), "k=%zu: load_inverse refused", k);
    CHECK(!d.load_inverse(tinv.data(), pitch), "k=%zu: a second load_inverse taken", k);
    if (read_rows_first) {  // spread the rows now: every accessor below reads them
      for (size_t i = 0; i < k; i++)
        CHECK(memcmp(d.t_row(i), &tref[i * k], k) == 0 && memcmp(d.coeff_row(i), &cref[i * k], k) == 0,
              "k=%zu: row %zu", k, i);
    }
    CHECK(d.is_decoded() && d.useful() == ref.useful() && d.received() == ref.received() &&
              d.rank() == ref.rank() && d.required() == 0,
          "k=%zu rows=%d: counters", k, read_rows_first);
    CHECK(transform(d) == tref && coefficients(d) == cref, "k=%zu rows=%d: copies", k, read_rows_first);
    std::vector<int32_t> ro, ro_ref;
    std::vector<uint8_t> sc, sc_ref;
    CHECK(d.decoded(&ro, &sc) == ref.decoded(&ro_ref, &sc_ref) && ro == ro_ref && sc == sc_ref,
          "k=%zu rows=%d: decoded()", k, read_rows_first);
    for (size_t idx : {(size_t)0, k / 2, k - 1, k, k + 3})
      CHECK(d.piece_available(idx) == ref.piece_available(idx), "k=%zu rows=%d: piece_available(%zu)", k,
            read_rows_first, idx);
    std::vector<uint8_t> extra(k, 9);
    size_t used = 99;
    CHECK(d.add(extra.data()) == 3 && d.add_many(extra.data(), k, 1, &used) == 3 && used == 0,
          "k=%zu rows=%d: AddPiece after the load not refused", k, read_rows_first);
    // and the rows spread after the block answered
    for (size_t i = 0; i < k; i++)
      CHECK(memcmp(d.t_row(i), &tref[i * k], k) == 0 && memcmp(d.coeff_row(i), &cref[i * k], k) == 0,
            "k=%zu rows=%d: row %zu after", k, read_rows_first, i);
    CHECK(transform(d) == tref && coefficients(d) == cref, "k=%zu rows=%d: copies after", k, read_rows_first);
  }
  DecoderCore one(k);
  one.add(&C[0]);
  CHECK(!one.load_inverse(tinv.data(), pitch), "k=%zu: a decoder holding a row took an inverse", k);
}

int main() {
  {
    std::mt19937 rng(777);
    for (size_t k : {2, 3, 16, 64, 129, 256}) run_inverse_case(k, rng);
  }
  std::mt19937 rng(12345);
  const size_t ks[] = {2, 3, 16, 64, 129, 256};
  for (size_t k : ks) {
    const size_t rs[] = {1, 2, k / 3, k / 2, k - 1};
    for (size_t r : rs) {
      if (r < 1 || r >= k) continue;
      for (int kind = 0; kind < 3; kind++)
        if (kind != 2 || r >= 2)
          for (int inv = 0; inv < 2; inv++) run_case(k, r, kind, inv != 0, rng);
    }
  }
  // a fresh decoder is not continued
  DecoderCore fresh(8);
  std::vector<uint8_t> eye(64, 0);
  for (int i = 0; i < 8; i++) eye[i * 8 + i] = 1;
  CHECK(!fresh.load_continued(eye.data(), 8, true), "a fresh decoder took a continued state");
  printf("ok (%d failures)\n", failures);
  return failures ? 1 : 0;
}
