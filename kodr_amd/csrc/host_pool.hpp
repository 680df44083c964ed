// host_pool.hpp -- a few persistent host threads for per-decoder work of the
// grouped entry points (one task = one decoder's host state, ~5-25 us of
// memory-bound copying at k = 256).  The tasks of one call are independent
// (disjoint decoders, disjoint output slices), so the calling thread and the
// workers take task indices from one atomic counter; run() returns when all
// are done.  Not for fine-grained work inside one decoder (DecoderCore's own
// solve stays on one thread: cache lines would move between cores per panel).
#pragma once

#include <stdlib.h>

#include <algorithm>

#include <atomic>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

namespace kodr_amd {

class HostPool {
 public:
  // KODR_HOST_THREADS (default min(8, hardware threads)); 1 runs every task
  // on the calling thread
  static HostPool& get() {
    static HostPool p(threads_wanted());
    return p;
  }

  void run(size_t n, const std::function<void(size_t)>& fn) {
    if (n == 0) return;
    if (workers_.empty() || n == 1) {
      for (size_t i = 0; i < n; i++) fn(i);
      return;
    }
    // one batch object per call: a worker that wakes late holds the batch it
    // saw, whose counter is exhausted, and never runs another call's tasks
    auto b = std::make_shared<Batch>();
    b->fn = &fn;
    b->n = n;
    {
      std::lock_guard<std::mutex> lk(mu_);
      cur_ = b;
      gen_++;
    }
    cv_.notify_all();
    work(*b);
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [&] { return b->done.load() == n; });
    cur_.reset();
  }

  ~HostPool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
      gen_++;
    }
    cv_.notify_all();
    for (auto& t : workers_) t.join();
  }

 private:
  struct Batch {
    const std::function<void(size_t)>* fn = nullptr;
    size_t n = 0;
    std::atomic<size_t> next{0}, done{0};
  };

  static size_t threads_wanted() {
    if (const char* e = getenv("KODR_HOST_THREADS")) return (size_t)std::max(1, atoi(e));
    const unsigned hw = std::thread::hardware_concurrency();
    return std::min<size_t>(8, hw ? hw : 1);
  }

  explicit HostPool(size_t threads) {
    for (size_t i = 1; i < threads; i++) workers_.emplace_back([this] { loop(); });
  }

  // take tasks until none is left; the last finisher wakes run()
  void work(Batch& b) {
    for (size_t i; (i = b.next.fetch_add(1)) < b.n;) {
      (*b.fn)(i);
      if (b.done.fetch_add(1) + 1 == b.n) {
        std::lock_guard<std::mutex> lk(mu_);
        done_cv_.notify_all();
      }
    }
  }

  void loop() {
    uint64_t seen = 0;
    for (;;) {
      std::shared_ptr<Batch> b;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
        b = cur_;
      }
      if (b) work(*b);
    }
  }

  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::shared_ptr<Batch> cur_;
  uint64_t gen_ = 0;
  bool stop_ = false;
};

}  // namespace kodr_amd
