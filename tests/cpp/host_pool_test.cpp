// host_pool.hpp on the CPU: every task index runs exactly once per call,
// run() returns only after all of them, back-to-back calls and calls from
// two threads at once do not mix tasks, and a one-thread pool still works.
#include <atomic>
#include <cstdio>
#include <thread>
#include <vector>

#include "../../kodr_amd/csrc/host_pool.hpp"

int main() {
  using kodr_amd::HostPool;
  int failures = 0;
  for (int call = 0; call < 2000; call++) {
    const size_t n = 1 + call % 37;
    std::vector<std::atomic<int>> hits(n);
    for (auto& h : hits) h = 0;
    HostPool::get().run(n, [&](size_t i) { hits[i].fetch_add(1); });
    for (size_t i = 0; i < n; i++)
      if (hits[i].load() != 1) failures++;
  }
  // two callers at once: each sees its own tasks only
  auto caller = [&](int salt, std::atomic<int>* bad) {
    for (int call = 0; call < 500; call++) {
      std::vector<int> out(16, -1);
      HostPool::get().run(16, [&](size_t i) { out[i] = salt * 100 + (int)i; });
      for (int i = 0; i < 16; i++)
        if (out[i] != salt * 100 + i) bad->fetch_add(1);
    }
  };
  std::atomic<int> bad{0};
  std::thread a(caller, 1, &bad), b(caller, 2, &bad);
  a.join();
  b.join();
  failures += bad.load();
  printf("host_pool ok (%d failures)\n", failures);
  return failures ? 1 : 0;
}
