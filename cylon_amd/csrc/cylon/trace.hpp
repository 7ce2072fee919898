// Tracing, phase timers, counters and leveled logging (aux subsystem).
//
// Reference: ad-hoc std::chrono + LOG(INFO) per phase (table.cpp:166-176,
// partition.cpp:58-60, hash_join.cpp:301-304, ...).  Here:
//   * Phase: an RAII scope that (when tracing is on) pushes a ROCTx range
//     (visible in `rocprofv3 --marker-trace`) and records a pair of HIP events on
//     the current stream (GPU) or a steady-clock interval (CPU); report()
//     resolves the events and returns per-phase totals;
//   * counters: rows in/out, bytes exchanged, ... per operator;
//   * CYLON_LOG_LEVEL (0 silent .. 3 debug) for host-side logging.
// Tracing is off by default (CYLON_TRACE=1 or set_enabled(true)): no events, no syncs.
#pragma once
#include <ATen/ATen.h>

#include <cstdint>
#include <map>
#include <string>

namespace cylon {
namespace trace {

bool enabled();
void set_enabled(bool on);
int log_level();
void log(int level, const std::string &msg);

class Phase {
 public:
  Phase(const char *name, const at::Device &dev);
  ~Phase();
  Phase(const Phase &) = delete;
  Phase &operator=(const Phase &) = delete;

 private:
  const char *name_;
  bool active_ = false;
  bool gpu_ = false;
  void *start_ = nullptr;
  void *stop_ = nullptr;
  int64_t t0_ns_ = 0;
  int dev_ = 0;
};

void add_counter(const std::string &name, int64_t value);

struct PhaseStat {
  double total_ms = 0;
  int64_t calls = 0;
};

// resolves pending GPU events (synchronising them) and returns totals
std::map<std::string, PhaseStat> phases();
std::map<std::string, int64_t> counters();
void reset();

}  // namespace trace
}  // namespace cylon

#define CYLON_CONCAT_INNER(a, b) a##b
#define CYLON_CONCAT(a, b) CYLON_CONCAT_INNER(a, b)
#define CYLON_PHASE(name, dev) ::cylon::trace::Phase CYLON_CONCAT(_cylon_phase_, __LINE__)(name, dev)
