#include "cylon/knobs.hpp"

#include <cstdlib>
#include <cstring>

#include "cylon/common.hpp"

namespace cylon {
namespace knobs {

const std::vector<KnobInfo> &Registry() {
  static const std::vector<KnobInfo> r = {
      // runtime / I/O
      {"LOG_LEVEL", "runtime", "native log level"},
      {"TRACE", "runtime", "phase timings and counters (C.trace_*) on from the start"},
      {"TCP_HOST", "runtime", "host address of the native TCP mesh"},
      {"H2D_CHUNK_MB", "runtime", "pinned staged host-to-device ingest: chunk size"},
      {"H2D_THREADS", "runtime", "pinned staged host-to-device ingest: copy threads"},
      // path thresholds (tests force the fast paths on small tables)
      {"RADIX_JOIN_MIN_ROWS", "threshold", "smallest side from which joins take the LDS radix path"},
      {"RADIX_GROUPBY_MIN_ROWS", "threshold", "rows from which group-bys take the LDS radix path"},
      {"RADIX_SETOP_MIN_ROWS", "threshold", "rows from which union / intersect / subtract / unique take the radix path"},
      {"RADIX_SORT_MIN_ROWS", "threshold", "rows from which sorts take the row-moving radix passes"},
      {"RANGE_JOIN", "threshold", "0: sort-algorithm inner joins skip the range-partitioned LDS join"},
      // distributed execution (each shadowed by a config key of the same name in lower case)
      {"FORCE_SHUFFLE", "distributed", "run the exchange path even at world 1 (config force_shuffle)"},
      {"SHUFFLE_CHUNKS", "distributed", "hash chunks per destination of the planned shuffle (config shuffle_chunks)"},
      {"SHUFFLE_NARROW", "distributed", "0: int64 columns never travel as uint32 offsets (config shuffle_narrow)"},
      {"SHUFFLE_SELF_RCCL", "distributed", "1: a rank's own rows go through RCCL too (config shuffle_self_rccl)"},
      {"VERIFY_SORT", "distributed", "1: check every sort's output order (config verify_sort)"},
      // test forcing of fallback paths that the defaults rarely take
      {"RJ_SLOT", "test", "0: join partitions by the exact LSD passes instead of slot mode"},
      {"RJ_FIRST_PASS_CHUNKS", "test", "0: bounded-memory joins of released int64-key inputs take the chunk-major pass instead of chunking the join's first radix pass"},
      {"RJ_EXACT_COUNT", "test", "1: the join counts every partition (no sampled output estimate)"},
      {"RJ_FUSED_MIN_PARTS", "test", "partitions from which the sampled output estimate is used (4096)"},
      {"RJ_ESTIMATE_SCALE", "test", "scales the sampled output estimate (< 1 forces the exact rerun)"},
      {"RJ_SHARE_KEY", "test", "0: an inner join writes the build side's key column instead of sharing the probe side's"},
      {"RJ_VAR_WORDS", "test", "0: variable-length string keys / payloads travel as a row number + byte gather, not padded words"},
      {"RJ_EXTRA_BITS", "test", "extra join partition bits (finer partitions)"},
      {"RJ_SPLIT_ROWS", "test", "build rows per chunk of a split (skewed) join partition (default: LDS capacity)"},
      {"SORT_LOOKBACK", "test", "0: sorts use the exact per-tile histogram passes"},
      {"PARTITION_LOOKBACK", "test", "0: stable two-pass hash partitions use exact tile histograms"},
      {"RP_DEBUG_UNSTABLE", "test", "1: every partition pass ranks unstably, so the ranking guard must fire"},
  };
  return r;
}

static bool registered(const char *name) {
  for (const auto &k : Registry())
    if (std::strcmp(k.name, name) == 0) return true;
  return false;
}

const char *Get(const char *name) {
  CYLON_CHECK(registered(name), Code::Invalid, "unregistered knob CYLON_" << name);
  const std::string var = std::string("CYLON_") + name;
  return std::getenv(var.c_str());
}

int64_t Int(const char *name, int64_t def) {
  const char *v = Get(name);
  return v && *v ? std::atoll(v) : def;
}

bool Flag(const char *name, bool def) {
  const char *v = Get(name);
  if (v && v[0] == '1') return true;
  if (v && v[0] == '0') return false;
  return def;
}

std::string ConfigOr(const std::string &config_value, const char *name) {
  if (!config_value.empty()) return config_value;
  const char *v = Get(name);
  return v ? std::string(v) : std::string();
}

}  // namespace knobs
}  // namespace cylon
