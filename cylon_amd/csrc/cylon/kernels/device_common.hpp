// Device-side helpers shared by the HIP kernel translation units (gfx950).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include "../common.hpp"
#include "../hash.hpp"
#include "../types.hpp"
#include "kernels.hpp"

namespace cylon {
namespace hip {

constexpr int kWave = 64;        // CDNA wavefront width
constexpr int kBlock = 256;      // 4 waves: one per SIMD of a CU
constexpr int kNumCUs = 256;     // MI355X: 8 XCDs x 32 CUs
constexpr int kMaxGrid = kNumCUs * 8;

#define HIP_CHECK(expr)                                                                  \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess)                                                                \
      CYLON_THROW(::cylon::Code::ExecutionError,                                         \
                  "HIP error " << hipGetErrorString(_e) << " at " << __FILE__ << ":" << __LINE__); \
  } while (0)

#define HIP_LAUNCH_CHECK() HIP_CHECK(hipGetLastError())

inline int grid_for(int64_t n, int64_t per_block = kBlock, int64_t cap = kMaxGrid) {
  int64_t g = (n + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return static_cast<int>(g);
}

inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

// load the code object holding fn now (HIP loads a code object lazily, on its first launch)
inline void preload_code(const void *fn) {
  hipFuncAttributes a;
  (void)hipFuncGetAttributes(&a, fn);
}

__device__ __forceinline__ int lane_id() { return __lane_id(); }

__device__ __forceinline__ uint64_t lanemask_lt() {
  return (lane_id() == 0) ? 0ull : ((~0ull) >> (64 - lane_id()));
}

// Load a fixed-width element as raw little-endian bits.
__device__ __forceinline__ uint64_t load_bits(const uint8_t *base, int64_t i, int w) {
  switch (w) {
    case 1: return base[i];
    case 2: return reinterpret_cast<const uint16_t *>(base)[i];
    case 4: return reinterpret_cast<const uint32_t *>(base)[i];
    case 8: return reinterpret_cast<const uint64_t *>(base)[i];
    default: return 0;
  }
}

// Sign- or zero-extend raw bits of width w to 64 bits according to kind.
__device__ __forceinline__ int64_t extend_bits(uint64_t b, int w, int kind) {
  if (kind == static_cast<int>(ValueKind::SIGNED_INT)) {
    switch (w) {
      case 1: return (int64_t)(int8_t)b;
      case 2: return (int64_t)(int16_t)b;
      case 4: return (int64_t)(int32_t)b;
      default: return (int64_t)b;
    }
  }
  if (kind == static_cast<int>(ValueKind::FLOAT)) {
    // normalise -0.0 to +0.0 so that equal values have equal bits
    if (w == 8 && b == 0x8000000000000000ull) return 0;
    if (w == 4 && b == 0x80000000ull) return 0;
    if (w == 2 && b == 0x8000ull) return 0;
  }
  return (int64_t)b;
}

}  // namespace hip
}  // namespace cylon
