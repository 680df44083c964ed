// pool.hpp -- per-device caching allocator for the engine's own buffers.
//
// hipFree of a 32 MiB buffer costs ~175 us on MI355X (profiles/r01/alloc.log)
// and a decoder for 32 MiB/256 owns five such buffers, so a service that
// decodes one generation after another would spend more time freeing than
// decoding.  Freed blocks are kept instead, keyed by size, and handed to the
// next request that fits (at most 2x oversized).  Reuse is stream-ordered: a
// freed block carries an event recorded on the stream that last used it, and
// a request from another stream makes its stream wait on that event (no host
// synchronisation).  Blocks beyond the cache cap (KODR_POOL_BYTES, default
// 8 GiB per device) are really freed, oldest first.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include <algorithm>
#include <list>
#include <memory>
#include <mutex>

namespace kodr_amd {

class DevicePool {
 public:
  static DevicePool& get(int device) {
    static DevicePool pools[64];
    return pools[device & 63];
  }

  // size rounded up to the block granularity; *cap receives the block size
  hipError_t alloc(size_t bytes, hipStream_t stream, uint8_t** out, size_t* cap) {
    const size_t need = round(bytes);
    {
      std::lock_guard<std::mutex> lk(mu_);
      if (!pending_.empty()) flush_pending();
      auto best = free_.end();
      for (auto it = free_.begin(); it != free_.end(); ++it)
        if (it->size >= need && it->size <= 2 * need && (best == free_.end() || it->size < best->size)) best = it;
      if (best != free_.end()) {
        Block b = *best;
        free_.erase(best);
        cached_ -= b.size;
        hipError_t e = hipSuccess;
        if (b.ev && b.stream != stream) e = hipStreamWaitEvent(stream, b.ev, 0);
        if (b.ev && !b.shared) events_.push_back(b.ev);
        if (e != hipSuccess) return e;
        *out = b.p;
        *cap = b.size;
        return hipSuccess;
      }
    }
    hipError_t e = hipMalloc((void**)out, need);
    if (e != hipSuccess) {  // give the cache back to the driver and retry once
      trim(0);
      (void)hipGetLastError();
      e = hipMalloc((void**)out, need);
    }
    if (e == hipSuccess) *cap = need;
    return e;
  }

  // p (cap bytes, from alloc) is no longer needed once `stream` reaches here;
  // idle: no work that uses p is pending on any stream (reusable at once, no
  // event: a decoder's destroy frees several blocks after one stream query)
  void free(uint8_t* p, size_t cap, hipStream_t stream, bool idle = false) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(mu_);
    if (idle) {
      free_.push_front(Block{p, cap, stream, nullptr, nullptr});
      cached_ += cap;
      while (cached_ > limit() && !free_.empty()) release_oldest();
      return;
    }
    hipEvent_t ev = nullptr;
    if (!events_.empty()) {
      ev = events_.back();
      events_.pop_back();
    } else if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
      ev = nullptr;
    }
    if (!ev || hipEventRecord(ev, stream) != hipSuccess) {  // cannot order reuse: free for real
      if (ev) events_.push_back(ev);
      (void)hipStreamSynchronize(stream);
      (void)hipFree(p);
      return;
    }
    free_.push_front(Block{p, cap, stream, ev, nullptr});
    cached_ += cap;
    while (cached_ > limit() && !free_.empty()) release_oldest();
  }

  // free cached blocks until at most `keep` bytes remain
  void trim(size_t keep) {
    std::lock_guard<std::mutex> lk(mu_);
    if (!pending_.empty()) flush_pending();
    while (cached_ > keep && !free_.empty()) release_oldest();
  }

  // p is no longer needed once `stream` reaches its current end, but the
  // caller records nothing: the block waits in a pending list, and the next
  // alloc() orders all pending blocks of a stream behind ONE event recorded
  // there (a decoder's destroy while its stream still runs: no GPU packet
  // per buffer, no host wait; an event per buffer, or per decoder, sat as
  // marker packets between a round trip's GetPieces and the next encode)
  // (pending bytes count against the cache cap: past it they are ordered and
  // the oldest cached blocks released at once)
  void defer_free(uint8_t* p, size_t cap, hipStream_t stream) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(mu_);
    pending_.push_back(Block{p, cap, stream, nullptr, nullptr});
    pending_bytes_ += cap;
    if (cached_ + pending_bytes_ > limit()) flush_pending();
  }
  // the stream is idle (the caller synchronised it) and about to go away:
  // its pending blocks are reusable at once
  void drop_stream(hipStream_t stream) {
    std::lock_guard<std::mutex> lk(mu_);
    for (auto it = pending_.begin(); it != pending_.end();) {
      if (it->stream == stream) {
        free_.push_front(Block{it->p, it->size, nullptr, nullptr, nullptr});
        cached_ += it->size;
        pending_bytes_ -= it->size;
        it = pending_.erase(it);
      } else {
        ++it;
      }
    }
    while (cached_ > limit() && !free_.empty()) release_oldest();
  }

  // idle cached blocks plus those still pending (defer_free)
  size_t cached() {
    std::lock_guard<std::mutex> lk(mu_);
    return cached_ + pending_bytes_;
  }

 private:
  // an event shared by the pending blocks of one stream (flush_pending): back to events_ when
  // the last of them leaves the cache (its destructor runs with mu_ held)
  struct SharedEvent {
    hipEvent_t ev;
    DevicePool* pool;
    SharedEvent(hipEvent_t e, DevicePool* p) : ev(e), pool(p) {}
    SharedEvent(const SharedEvent&) = delete;
    ~SharedEvent() { pool->events_.push_back(ev); }
  };
  struct Block {
    uint8_t* p;
    size_t size;
    hipStream_t stream;
    hipEvent_t ev;
    std::shared_ptr<SharedEvent> shared;  // set: ev belongs to it (not returned per block)
  };

  static size_t round(size_t b) {
    const size_t g = b >= ((size_t)1 << 20) ? ((size_t)2 << 20) : ((size_t)64 << 10);
    return (std::max<size_t>(b, 1) + g - 1) / g * g;
  }
  static size_t limit() {
    static const size_t lim = [] {
      const char* s = getenv("KODR_POOL_BYTES");
      return s ? (size_t)strtoull(s, nullptr, 10) : ((size_t)8 << 30);
    }();
    return lim;
  }
  // the pending blocks into the cache, one event per stream (mu_ held)
  void flush_pending() {
    while (!pending_.empty()) {
      const hipStream_t st = pending_.front().stream;
      hipEvent_t ev = nullptr;
      if (!events_.empty()) {
        ev = events_.back();
        events_.pop_back();
      } else if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess) {
        ev = nullptr;
      }
      const bool ok = ev && hipEventRecord(ev, st) == hipSuccess;
      if (!ok) {  // cannot order reuse: wait for the stream
        if (ev) events_.push_back(ev);
        (void)hipGetLastError();
        (void)hipStreamSynchronize(st);
      }
      auto ref = ok ? std::make_shared<SharedEvent>(ev, this) : nullptr;
      for (auto it = pending_.begin(); it != pending_.end();) {
        if (it->stream == st) {
          free_.push_front(Block{it->p, it->size, st, ok ? ev : nullptr, ref});
          cached_ += it->size;
          pending_bytes_ -= it->size;
          it = pending_.erase(it);
        } else {
          ++it;
        }
      }
    }
    while (cached_ > limit() && !free_.empty()) release_oldest();
  }
  void release_oldest() {  // mu_ held
    Block b = free_.back();
    free_.pop_back();
    cached_ -= b.size;
    if (b.ev) (void)hipEventSynchronize(b.ev);
    (void)hipFree(b.p);
    if (b.ev && !b.shared) events_.push_back(b.ev);
  }

  std::mutex mu_;
  // (declared before the block lists: a block's SharedEvent returns its event
  // here when the lists are destroyed at exit)
  std::list<hipEvent_t> events_;
  std::list<Block> free_;  // most recently freed first
  std::list<Block> pending_;  // defer_free'd, not yet ordered by an event
  size_t cached_ = 0;
  size_t pending_bytes_ = 0;  // bytes in pending_
};

}  // namespace kodr_amd
