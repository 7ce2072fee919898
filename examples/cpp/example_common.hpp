// Shared helpers of the C++ examples: context from the command line, status checks and
// "name value" result lines (tests/test_cpp_examples.py parses them).
#pragma once
#include <cstdio>
#include <string>

#include "cylon/api.hpp"

#define CHECK_OK(expr)                                                       \
  do {                                                                       \
    cylon::Status _s = (expr);                                               \
    if (!_s.is_ok()) {                                                       \
      std::fprintf(stderr, "%s failed: %s\n", #expr, _s.get_msg().c_str()); \
      return 1;                                                              \
    }                                                                        \
  } while (0)

namespace example {

// "cpu" / "cuda:0": local context; "tcp" / "rccl": distributed from the torchrun environment
inline std::shared_ptr<cylon::CylonContext> make_context(const std::string &dev) {
  if (dev == "tcp" || dev == "rccl") {
    cylon::net::CommConfig cfg;
    cfg.type = dev == "tcp" ? cylon::net::CommType::TCP : cylon::net::CommType::RCCL;
    return cylon::CylonContext::InitDistributed(cfg);
  }
  return cylon::CylonContext::Init(at::Device(dev));
}

inline void report(const char *what, int64_t v) { std::printf("%s %lld\n", what, static_cast<long long>(v)); }
inline void report(const char *what, const cylon::TablePtr &t) { report(what, t->Rows()); }

// column c of t on the host as int64 / double (any numeric type)
inline at::Tensor host_i64(const cylon::TablePtr &t, int c) {
  return t->column(c).data.slice(0, 0, t->Rows()).to(at::kCPU).to(at::kLong);
}
inline at::Tensor host_f64(const cylon::TablePtr &t, int c) {
  return t->column(c).data.slice(0, 0, t->Rows()).to(at::kCPU).to(at::kDouble);
}

}  // namespace example
