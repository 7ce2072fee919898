// Common definitions shared by host code, CPU kernels and HIP kernels.
//
// The engine is written for MI355X (gfx950).  Kernel translation units are
// compiled by hipcc; orchestration units by the host C++ compiler.  Small
// element functions (hashing, comparisons) are shared between the HIP kernels
// and their CPU twins through CYLON_HD.
#pragma once

#include <cstdint>
#include <cstddef>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define CYLON_HD __host__ __device__ __forceinline__
#define CYLON_DEVICE __device__ __forceinline__
#else
#define CYLON_HD inline
#endif

#include <stdexcept>
#include <string>
#include <sstream>

namespace cylon {

// Error codes, numerically identical to the reference (cylon/code.cpp:19-39),
// which themselves follow Arrow's status codes.
enum Code : int {
  OK = 0,
  OutOfMemory = 1,
  KeyError = 2,
  TypeError = 3,
  Invalid = 4,
  IOError = 5,
  CapacityError = 6,
  IndexError = 7,
  UnknownError = 9,
  NotImplemented = 10,
  SerializationError = 11,
  GpuMemoryError = 12,
  RError = 13,
  CodeGenError = 40,
  ExpressionValidationError = 41,
  ExecutionError = 42,
  AlreadyExists = 45
};

// Exception used internally; the Status-returning C++ API (api.hpp) catches it
// and converts to Status, the Python binding maps it to CylonError.
class CylonError : public std::runtime_error {
 public:
  CylonError(int code, const std::string &msg) : std::runtime_error(msg), code_(code) {}
  int code() const { return code_; }

 private:
  int code_;
};

}  // namespace cylon

#define CYLON_THROW(code, msg_expr)                                   \
  do {                                                                \
    std::ostringstream _cy_oss;                                       \
    _cy_oss << msg_expr;                                              \
    throw ::cylon::CylonError((code), _cy_oss.str());                 \
  } while (0)

#define CYLON_CHECK(cond, code, msg_expr) \
  do {                                    \
    if (!(cond)) CYLON_THROW(code, msg_expr); \
  } while (0)
