// Tracing / counters / logging implementation (see trace.hpp).
#include "cylon/knobs.hpp"
#include "trace.hpp"

#include <hip/hip_runtime_api.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <atomic>
#include <chrono>
#include <cstdlib>
#include <iostream>
#include <mutex>
#include <vector>

#include <c10/hip/HIPStream.h>

namespace cylon {
namespace trace {

namespace {
std::atomic<int> g_enabled{-1};
std::mutex g_mu;
struct Pending {
  std::string name;
  hipEvent_t start, stop;
};
std::vector<Pending> &pending() {
  static std::vector<Pending> p;
  return p;
}
std::map<std::string, PhaseStat> &stats() {
  static std::map<std::string, PhaseStat> s;
  return s;
}
std::map<std::string, int64_t> &ctrs() {
  static std::map<std::string, int64_t> c;
  return c;
}
int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
      .count();
}
}  // namespace

bool enabled() {
  int e = g_enabled.load();
  if (e < 0) {
    const char *v = knobs::Get("TRACE");
    e = (v && v[0] && v[0] != '0') ? 1 : 0;
    g_enabled.store(e);
  }
  return e == 1;
}

void set_enabled(bool on) { g_enabled.store(on ? 1 : 0); }

int log_level() {
  static int lvl = (int)knobs::Int("LOG_LEVEL", 1);
  return lvl;
}

void log(int level, const std::string &msg) {
  if (level <= log_level()) {
    static const char *tags[] = {"", "WARN", "INFO", "DEBUG"};
    std::cerr << "[cylon " << tags[level < 4 ? level : 3] << "] " << msg << std::endl;
  }
}

Phase::Phase(const char *name, const at::Device &dev) : name_(name) {
  if (!enabled()) return;
  active_ = true;
  roctxRangePushA(name);
  gpu_ = dev.is_cuda();
  if (gpu_) {
    dev_ = dev.index();
    hipStream_t s = c10::hip::getCurrentHIPStream(dev.index()).stream();
    hipEvent_t a, b;
    if (hipEventCreate(&a) == hipSuccess && hipEventCreate(&b) == hipSuccess && hipEventRecord(a, s) == hipSuccess) {
      start_ = a;
      stop_ = b;
    } else {
      gpu_ = false;  // timing falls back to the host clock
    }
  }
  if (!gpu_) t0_ns_ = now_ns();
}

Phase::~Phase() {
  if (!active_) return;
  roctxRangePop();
  std::lock_guard<std::mutex> lk(g_mu);
  hipStream_t s = gpu_ ? c10::hip::getCurrentHIPStream(dev_).stream() : nullptr;
  if (gpu_ && hipEventRecord(static_cast<hipEvent_t>(stop_), s) == hipSuccess) {
    pending().push_back({name_, static_cast<hipEvent_t>(start_), static_cast<hipEvent_t>(stop_)});
  } else if (gpu_) {
    (void)hipEventDestroy(static_cast<hipEvent_t>(start_));
    (void)hipEventDestroy(static_cast<hipEvent_t>(stop_));
    stats()[name_].calls++;  // counted, not timed
  } else {
    auto &st = stats()[name_];
    st.total_ms += (now_ns() - t0_ns_) / 1e6;
    st.calls++;
  }
}

void add_counter(const std::string &name, int64_t value) {
  if (!enabled()) return;
  std::lock_guard<std::mutex> lk(g_mu);
  ctrs()[name] += value;
}

std::map<std::string, PhaseStat> phases() {
  std::lock_guard<std::mutex> lk(g_mu);
  for (auto &p : pending()) {
    float ms = 0;
    if (hipEventSynchronize(p.stop) != hipSuccess || hipEventElapsedTime(&ms, p.start, p.stop) != hipSuccess)
      ms = 0;  // a failed query leaves the phase counted but untimed
    auto &st = stats()[p.name];
    st.total_ms += ms;
    st.calls++;
    (void)hipEventDestroy(p.start);
    (void)hipEventDestroy(p.stop);
  }
  pending().clear();
  return stats();
}

std::map<std::string, int64_t> counters() {
  std::lock_guard<std::mutex> lk(g_mu);
  return ctrs();
}

void reset() {
  phases();
  std::lock_guard<std::mutex> lk(g_mu);
  stats().clear();
  ctrs().clear();
}

}  // namespace trace
}  // namespace cylon
