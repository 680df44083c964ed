// staging.hpp -- pinned double-buffered host<->device copies for the
// host-pointer entry points.  Host buffers handed to the C ABI are pageable
// (Go slices, numpy arrays); copying through two pinned chunks lets the DMA of
// one chunk overlap the CPU copy of the next, instead of the driver's slow
// pageable path.  Host pointers are never retained: h2d returns once the
// bytes are in pinned memory, d2h once they are in the caller's buffer.
// Transfers of at most kUploadSmallMax bytes (coefficients, transforms, row
// tables) are moved by a kernel that reads or writes the pinned chunk through
// its device mapping: a DMA copy that small is all latency, and the next
// kernel waits ~11 us more for the copy engine (profiles/r01/dec_get.log).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>

#include "gf_kernels.hpp"

namespace kodr_amd {

class Staging {
 public:
  static constexpr size_t kChunk = 8u << 20;

  ~Staging() { release(); }

  hipError_t h2d(uint8_t* dst, size_t dpitch, const uint8_t* src, size_t spitch, size_t width,
                 size_t height, hipStream_t s) {
    if (!width || !height) return hipSuccess;
    if (is_pinned(src)) {  // registered / pinned caller memory: DMA straight from it
      hipError_t e = hipMemcpy2DAsync(dst, dpitch, src, spitch, width, height, hipMemcpyHostToDevice, s);
      return e == hipSuccess ? hipStreamSynchronize(s) : e;  // the caller may reuse src on return
    }
    hipError_t e = ensure();
    if (e != hipSuccess) return e;
    if (width * height <= kUploadSmallMax) {  // coefficients, row tables: a kernel reads the pinned chunk
      const int b = take();
      if (pending_[b] && (e = hipEventSynchronize(ev_[b])) != hipSuccess) return e;
      pack(buf_[b], width, src, spitch, width, height);
      if ((e = upload_small(dev_[b], dst, dpitch, width, height, s)) != hipSuccess) return e;
      if ((e = hipEventRecord(ev_[b], s)) != hipSuccess) return e;
      pending_[b] = true;
      return hipSuccess;
    }
    if (width > kChunk) {  // rows wider than a chunk: each row as chunk-wide segments
      for (size_t r = 0; r < height; r++) {
        const size_t full = width / kChunk, tail = width - full * kChunk;
        if ((e = h2d(dst + r * dpitch, kChunk, src + r * spitch, kChunk, kChunk, full, s)) != hipSuccess) return e;
        if ((e = h2d(dst + r * dpitch + full * kChunk, tail, src + r * spitch + full * kChunk, tail, tail, 1, s)) !=
            hipSuccess)
          return e;
      }
      return hipSuccess;
    }
    const size_t per = kChunk / width;
    for (size_t r0 = 0; r0 < height; r0 += per) {
      const size_t n = std::min(per, height - r0);
      const int b = take();
      if (pending_[b] && (e = hipEventSynchronize(ev_[b])) != hipSuccess) return e;
      pack(buf_[b], width, src + r0 * spitch, spitch, width, n);
      e = hipMemcpy2DAsync(dst + r0 * dpitch, dpitch, buf_[b], width, width, n, hipMemcpyHostToDevice, s);
      if (e != hipSuccess) return e;
      if ((e = hipEventRecord(ev_[b], s)) != hipSuccess) return e;
      pending_[b] = true;
    }
    return hipSuccess;
  }

  // Split small download: begin enqueues the copy into a pinned chunk and
  // records its event (work enqueued after it does not delay end); end waits
  // for that event and unpacks into dst.  width * height <= kDownloadSmallMax.
  // The chunk stays reserved between the two: other staging calls in that
  // window use the other chunk only.  One ticket at a time.
  hipError_t d2h_small_begin(const uint8_t* src, size_t spitch, size_t width, size_t height, hipStream_t s,
                             int* ticket) {
    if (reserved_[0] || reserved_[1]) return hipErrorInvalidValue;
    hipError_t e = ensure();
    if (e != hipSuccess) return e;
    const int b = take();
    if (pending_[b] && (e = hipEventSynchronize(ev_[b])) != hipSuccess) return e;
    pending_[b] = false;
    if ((e = download_small(src, spitch, dev_[b], width, height, s)) != hipSuccess) return e;
    if ((e = hipEventRecord(ev_[b], s)) != hipSuccess) return e;
    pending_[b] = true;  // any other use of chunk b waits for the download
    reserved_[b] = true;
    *ticket = b;
    return hipSuccess;
  }
  hipError_t d2h_small_end(int b, uint8_t* dst, size_t dpitch, size_t width, size_t height) {
    reserved_[b] = false;  // released on every path (the event still orders the chunk's next use)
    hipError_t e = hipEventSynchronize(ev_[b]);
    if (e != hipSuccess) return e;
    pending_[b] = false;
    pack(dst, dpitch, buf_[b], width, width, height);
    return hipSuccess;
  }

  // drop a ticket whose download will not be unpacked (an error between
  // begin and end): the chunk is free again once its event has passed
  void d2h_small_cancel(int b) {
    if (b >= 0 && b < 2) reserved_[b] = false;
  }

  hipError_t d2h(uint8_t* dst, size_t dpitch, const uint8_t* src, size_t spitch, size_t width,
                 size_t height, hipStream_t s) {
    if (!width || !height) return hipSuccess;
    if (is_pinned(dst)) {
      hipError_t e = hipMemcpy2DAsync(dst, dpitch, src, spitch, width, height, hipMemcpyDeviceToHost, s);
      return e == hipSuccess ? hipStreamSynchronize(s) : e;
    }
    hipError_t e = ensure();
    if (e != hipSuccess) return e;
    if (width * height <= kDownloadSmallMax) {  // coding vectors of a batch: a kernel writes the pinned chunk
      int b;
      if ((e = d2h_small_begin(src, spitch, width, height, s, &b)) != hipSuccess) return e;
      return d2h_small_end(b, dst, dpitch, width, height);
    }
    if (width > kChunk) {
      for (size_t r = 0; r < height; r++) {
        const size_t full = width / kChunk, tail = width - full * kChunk;
        if ((e = d2h(dst + r * dpitch, kChunk, src + r * spitch, kChunk, kChunk, full, s)) != hipSuccess) return e;
        if ((e = d2h(dst + r * dpitch + full * kChunk, tail, src + r * spitch + full * kChunk, tail, tail, 1, s)) !=
            hipSuccess)
          return e;
      }
      return hipSuccess;
    }
    const size_t per = kChunk / width;
    size_t prev_r0 = 0, prev_n = 0;
    int prev_b = -1;
    for (size_t r0 = 0; r0 < height; r0 += per) {
      const size_t n = std::min(per, height - r0);
      const int b = take();
      if (b == prev_b) {  // one chunk free (the other reserved): unpack before reuse
        if ((e = hipEventSynchronize(ev_[b])) != hipSuccess) return e;
        pending_[b] = false;
        pack(dst + prev_r0 * dpitch, dpitch, buf_[b], width, width, prev_n);
        prev_b = -1;
      }
      if (pending_[b] && (e = hipEventSynchronize(ev_[b])) != hipSuccess) return e;
      e = hipMemcpy2DAsync(buf_[b], width, src + r0 * spitch, spitch, width, n, hipMemcpyDeviceToHost, s);
      if (e != hipSuccess) return e;
      if ((e = hipEventRecord(ev_[b], s)) != hipSuccess) return e;
      pending_[b] = true;
      if (prev_b >= 0) {  // unpack the previous chunk while this one is in flight
        if ((e = hipEventSynchronize(ev_[prev_b])) != hipSuccess) return e;
        pending_[prev_b] = false;
        pack(dst + prev_r0 * dpitch, dpitch, buf_[prev_b], width, width, prev_n);
      }
      prev_b = b;
      prev_r0 = r0;
      prev_n = n;
    }
    if (prev_b < 0) return hipSuccess;
    if ((e = hipEventSynchronize(ev_[prev_b])) != hipSuccess) return e;
    pending_[prev_b] = false;
    pack(dst + prev_r0 * dpitch, dpitch, buf_[prev_b], width, width, prev_n);
    return hipSuccess;
  }

  // page-locked host memory (hipHostMalloc or hipHostRegister, e.g. through
  // rlnc_host_register) needs no bounce buffer.  An unknown pointer makes
  // hipPointerGetAttributes fail; clear that error so it is not reported by
  // the next launch's hipGetLastError.
  static bool is_pinned(const void* p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    return a.type == hipMemoryTypeHost;
  }

  void release() {
    for (int b = 0; b < 2; b++) {
      if (pending_[b]) (void)hipEventSynchronize(ev_[b]);
      if (ev_[b]) (void)hipEventDestroy(ev_[b]);
      if (buf_[b]) (void)hipHostFree(buf_[b]);
      ev_[b] = nullptr;
      buf_[b] = nullptr;
      dev_[b] = nullptr;
      pending_[b] = false;
      reserved_[b] = false;
    }
  }

 private:
  hipError_t ensure() {
    if (buf_[0]) return hipSuccess;
    for (int b = 0; b < 2; b++) {
      hipError_t e = hipHostMalloc((void**)&buf_[b], kChunk, hipHostMallocDefault);
      if (e != hipSuccess) return e;
      if ((e = hipHostGetDevicePointer((void**)&dev_[b], buf_[b], 0)) != hipSuccess) return e;
      if ((e = hipEventCreateWithFlags(&ev_[b], hipEventDisableTiming)) != hipSuccess) return e;
    }
    return hipSuccess;
  }
  // the next chunk in turn, skipping one reserved by d2h_small_begin
  int take() {
    int b = next_;
    if (reserved_[b]) b ^= 1;
    next_ = b ^ 1;
    return b;
  }
  static void pack(uint8_t* dst, size_t dpitch, const uint8_t* src, size_t spitch, size_t width, size_t n) {
    if (dpitch == width && spitch == width) {
      memcpy(dst, src, width * n);
      return;
    }
    for (size_t i = 0; i < n; i++) memcpy(dst + i * dpitch, src + i * spitch, width);
  }

  uint8_t* buf_[2] = {nullptr, nullptr};
  uint8_t* dev_[2] = {nullptr, nullptr};  // the same chunks as the device sees them
  hipEvent_t ev_[2] = {nullptr, nullptr};
  bool pending_[2] = {false, false};
  bool reserved_[2] = {false, false};
  int next_ = 0;
};

}  // namespace kodr_amd
