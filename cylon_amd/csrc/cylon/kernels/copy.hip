// Batched device-to-device copies (Merge / concatenation).  One launch moves every
// (column, part) buffer: blockIdx.y selects the copy, blockIdx.x strides over its
// 16-byte vectors (8-byte or byte fallback when misaligned).  The runtime's blit
// copy ran the 1B-row union's concatenation at ~2.4 TB/s
// (profiles/suite_cfg6_r02_kernels.txt); a plain streaming kernel reaches 4.7-5.7 TB/s
// (profiles/membench.txt).
#include "device_common.hpp"

namespace cylon {
namespace hip {

constexpr int kMaxCopies = 64;

struct CopyBatch {
  const uint8_t *src[kMaxCopies];
  uint8_t *dst[kMaxCopies];
  int64_t bytes[kMaxCopies];
};

__global__ __launch_bounds__(kBlock) void k_batched_copy(CopyBatch b) {
  const int c = blockIdx.y;
  const uint8_t *s = b.src[c];
  uint8_t *d = b.dst[c];
  const int64_t nb = b.bytes[c];
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uintptr_t al = reinterpret_cast<uintptr_t>(s) | reinterpret_cast<uintptr_t>(d) | (uintptr_t)nb;
  if ((al & 15) == 0) {
    const uint4 *s4 = reinterpret_cast<const uint4 *>(s);
    uint4 *d4 = reinterpret_cast<uint4 *>(d);
    const int64_t n4 = nb >> 4;
    for (int64_t i = t0; i < n4; i += 2 * step) {  // two vectors in flight per thread
      const int64_t j = i + step;
      const uint4 a = s4[i];
      uint4 x;
      if (j < n4) x = s4[j];
      d4[i] = a;
      if (j < n4) d4[j] = x;
    }
  } else if ((al & 7) == 0) {
    const uint64_t *s8 = reinterpret_cast<const uint64_t *>(s);
    uint64_t *d8 = reinterpret_cast<uint64_t *>(d);
    for (int64_t i = t0; i < (nb >> 3); i += step) d8[i] = s8[i];
  } else {
    for (int64_t i = t0; i < nb; i += step) d[i] = s[i];
  }
}

void batched_copy(const void *const *src, void *const *dst, const int64_t *bytes, int n, void *stream) {
  for (int base = 0; base < n; base += kMaxCopies) {
    CopyBatch b{};
    int m = 0;
    int64_t biggest = 0;
    for (int i = base; i < n && m < kMaxCopies; ++i) {
      if (bytes[i] <= 0) continue;
      b.src[m] = static_cast<const uint8_t *>(src[i]);
      b.dst[m] = static_cast<uint8_t *>(dst[i]);
      b.bytes[m] = bytes[i];
      biggest = std::max(biggest, bytes[i]);
      ++m;
    }
    if (m == 0) continue;
    // enough blocks for the largest copy (<= 2048 per copy), at least a wave of the chip overall
    const int64_t want = (biggest / 16 + 2LL * kBlock - 1) / (2LL * kBlock);
    const unsigned gx = (unsigned)std::max<int64_t>(1, std::min<int64_t>(want, 2048));
    hipLaunchKernelGGL(k_batched_copy, dim3(gx, (unsigned)m), dim3(kBlock), 0, as_stream(stream), b);
    HIP_LAUNCH_CHECK();
  }
}

// this file's code object is loaded at context creation (preload_device_code), not on first use
void preload_copy() { preload_code(reinterpret_cast<const void *>(&k_batched_copy)); }

}  // namespace hip
}  // namespace cylon
