// Host full-batch solve (DecoderCore::solve_full_batch, k = 256): median and best over 25
// solves, back to back or with an idle gap (us) between them.  Round 3 ran it against a
// threaded solve (KODR_SOLVE_THREADS, a spinning thread team over cache-line slabs; slower
// on 2-8 threads, profiles/r03/solve_threads/, removed).  Measurement only.  Build: g++ -O3 -std=c++17 -pthread
// -I kodr_amd/csrc tools/probe/solve_threads.cpp kodr_amd/csrc/decoder_core.cpp
#include "decoder_core.hpp"
#include <chrono>
#include <cstdio>
#include <random>
#include <vector>
#include <memory>
#include <thread>
#include <algorithm>
using namespace kodr_amd;
int main(int argc, char** argv) {
  const size_t k = 256;
  const int gap_us = argc > 1 ? atoi(argv[1]) : 0;
  std::mt19937 rng(5);
  std::vector<std::vector<uint8_t>> vs(30, std::vector<uint8_t>(k * k));
  for (auto& v : vs) for (auto& x : v) x = rng() & 0xff;
  std::vector<double> ts;
  for (int rep = 0; rep < 30; rep++) {
    DecoderCore c(k);
    size_t used = 0;
    if (gap_us) std::this_thread::sleep_for(std::chrono::microseconds(gap_us));
    auto t0 = std::chrono::steady_clock::now();
    c.add_many(vs[rep].data(), k, k, &used);
    auto t1 = std::chrono::steady_clock::now();
    if (rep >= 5) ts.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
  }
  std::sort(ts.begin(), ts.end());
  printf("gap %d us: solve median %.1f us, best %.1f\n", gap_us, ts[ts.size() / 2], ts[0]);
}
