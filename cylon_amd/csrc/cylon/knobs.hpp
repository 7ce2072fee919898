#pragma once
// The native engine's environment knobs: ONE registry of every CYLON_* variable the C++ / HIP code
// reads (name, kind, effect).  Code reads a knob only through these accessors, which refuse an
// unregistered name, so the table below -- mirrored by docs/knobs.md and checked by
// tests/test_utils_aux.py::test_knob_registry_matches_docs -- is the complete list.  Knobs are read
// per call (tests flip them between operations).
#include <cstdint>
#include <string>
#include <vector>

namespace cylon {
namespace knobs {

struct KnobInfo {
  const char *name;    // without the CYLON_ prefix
  const char *group;   // runtime | threshold | distributed | test
  const char *effect;
};

const std::vector<KnobInfo> &Registry();

// getenv("CYLON_" + name) of a registered knob (nullptr when unset)
const char *Get(const char *name);
// integer value, or def when unset / empty
int64_t Int(const char *name, int64_t def);
// "1" -> true, "0" -> false, else def
bool Flag(const char *name, bool def);
// a config value (ctx.add_config) if set, else the knob's value, else ""
std::string ConfigOr(const std::string &config_value, const char *name);

}  // namespace knobs
}  // namespace cylon
