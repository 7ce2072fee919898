// Pinned, pipelined host -> device ingest (see h2d.hpp).
#include "cylon/knobs.hpp"
#include "h2d.hpp"

#include <hip/hip_runtime.h>

#include <ATen/hip/HIPContext.h>
#include <c10/hip/HIPGuard.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../common.hpp"

#define H2D_CHECK(expr)                                                                              \
  do {                                                                                               \
    hipError_t _e = (expr);                                                                          \
    CYLON_CHECK(_e == hipSuccess, Code::ExecutionError, #expr << ": " << hipGetErrorString(_e));     \
  } while (0)

namespace cylon {
namespace io {

namespace {

constexpr int kSlots = 4;  // ring depth: chunks staged / in flight at once

// Persistent worker pool for the staging memcpys (one task = one slice of a chunk).
class CopyPool {
 public:
  explicit CopyPool(int n) {
    for (int i = 0; i < n; ++i) threads_.emplace_back([this] { run(); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> g(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto &t : threads_) t.join();
  }
  int size() const { return (int)threads_.size(); }

  // dst[0, len) = src[0, len) split over `parts` workers (the caller copies one part itself)
  void copy(void *dst, const void *src, size_t len, int parts) {
    parts = std::max(1, std::min(parts, size() + 1));
    const size_t piece = ((len + parts - 1) / parts + 4095) & ~size_t(4095);
    std::atomic<int> left{0};
    std::mutex dmu;
    std::condition_variable dcv;
    int queued = 0;
    for (int p = 1; p < parts; ++p) {
      const size_t off = piece * p;
      if (off >= len) break;
      const size_t l = std::min(piece, len - off);
      ++queued;
      left.fetch_add(1);
      push([=, &left, &dmu, &dcv] {
        std::memcpy(static_cast<char *>(dst) + off, static_cast<const char *>(src) + off, l);
        if (left.fetch_sub(1) == 1) {
          std::lock_guard<std::mutex> g(dmu);
          dcv.notify_one();
        }
      });
    }
    std::memcpy(dst, src, std::min(piece, len));
    if (queued) {
      std::unique_lock<std::mutex> g(dmu);
      dcv.wait(g, [&] { return left.load() == 0; });
    }
  }

 private:
  void push(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> g(mu_);
      q_.push_back(std::move(f));
    }
    cv_.notify_one();
  }
  void run() {
    for (;;) {
      std::function<void()> f;
      {
        std::unique_lock<std::mutex> g(mu_);
        cv_.wait(g, [this] { return stop_ || !q_.empty(); });
        if (stop_ && q_.empty()) return;
        f = std::move(q_.front());
        q_.pop_front();
      }
      f();
    }
  }
  std::vector<std::thread> threads_;
  std::deque<std::function<void()>> q_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_ = false;
};

int default_threads() {
  if (const int64_t t = knobs::Int("H2D_THREADS", 0)) return (int)std::max<int64_t>(1, t);
  const unsigned hc = std::thread::hardware_concurrency();
  return (int)std::max(1u, std::min(8u, hc ? hc / 2 : 1u));
}

CopyPool &pool() {
  static CopyPool p(default_threads() - 1);  // the calling thread copies one slice too
  return p;
}

// Per-device staging ring: pinned slots, the event of each slot's last DMA, a copy stream.
struct Ring {
  std::mutex mu;
  bool ready = false;
  void *slot[kSlots] = {nullptr};
  hipEvent_t ev[kSlots] = {nullptr};
  bool used[kSlots] = {false};
  hipEvent_t done = nullptr, start = nullptr;
  hipStream_t stream = nullptr;
};

Ring &ring(int device) {
  static Ring rings[64];
  return rings[device & 63];
}

}  // namespace

size_t StagedH2DChunkBytes() {
  static const size_t b = [] {
    const long mb = (long)std::max<int64_t>(1, knobs::Int("H2D_CHUNK_MB", 32));
    return (size_t)mb << 20;
  }();
  return b;
}

void StagedH2D(const void *src, void *dst, size_t bytes, int device, int threads, H2DStats *stats) {
  const auto t0 = std::chrono::steady_clock::now();
  if (bytes == 0) return;
  c10::hip::HIPGuard guard(device);
  Ring &r = ring(device);
  std::lock_guard<std::mutex> g(r.mu);
  const size_t chunk = StagedH2DChunkBytes();
  if (!r.ready) {
    for (int s = 0; s < kSlots; ++s) {
      H2D_CHECK(hipHostMalloc(&r.slot[s], chunk, hipHostMallocDefault));
      H2D_CHECK(hipEventCreateWithFlags(&r.ev[s], hipEventDisableTiming));
    }
    H2D_CHECK(hipEventCreateWithFlags(&r.done, hipEventDisableTiming));
    H2D_CHECK(hipEventCreateWithFlags(&r.start, hipEventDisableTiming));
    H2D_CHECK(hipStreamCreateWithFlags(&r.stream, hipStreamNonBlocking));
    r.ready = true;
  }
  const int parts = threads > 0 ? threads : pool().size() + 1;
  // the DMAs are ordered after the work already queued on the consumer stream: a destination
  // it is still filling or reading (a zero fill, memory the caching allocator just recycled)
  const hipStream_t consumer = c10::hip::getCurrentHIPStream(device).stream();
  H2D_CHECK(hipEventRecord(r.start, consumer));
  H2D_CHECK(hipStreamWaitEvent(r.stream, r.start, 0));
  int64_t nchunks = 0;
  for (size_t off = 0; off < bytes; off += chunk, ++nchunks) {
    const int s = (int)(nchunks % kSlots);
    const size_t len = std::min(chunk, bytes - off);
    if (r.used[s]) H2D_CHECK(hipEventSynchronize(r.ev[s]));  // the slot's previous DMA has drained
    pool().copy(r.slot[s], static_cast<const char *>(src) + off, len, parts);
    H2D_CHECK(hipMemcpyAsync(static_cast<char *>(dst) + off, r.slot[s], len, hipMemcpyHostToDevice, r.stream));
    H2D_CHECK(hipEventRecord(r.ev[s], r.stream));
    r.used[s] = true;
  }
  // the consumer (the device's current stream) is ordered after the last DMA; the host is not
  H2D_CHECK(hipEventRecord(r.done, r.stream));
  H2D_CHECK(hipStreamWaitEvent(consumer, r.done, 0));
  if (stats) {
    stats->bytes += (int64_t)bytes;
    stats->chunks += nchunks;
    stats->seconds += std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
}

}  // namespace io
}  // namespace cylon
