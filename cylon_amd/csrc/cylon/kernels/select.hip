// K15 elementwise select over variable-width columns (string / binary where, fill_null) on
// gfx950.  Row i of the output takes a[i] where cond[i] != 0, else b[bi] with bi = i, or 0 when
// b is a one-row broadcast value (fill_null, where with a scalar); a b without offsets selects a
// null row (where(cond) with no `other`).  Two launches around a device scan, like gather_var:
// lengths (one thread per row), then bytes (one wave per row, 16-byte vector copies when the
// source and destination runs share their alignment, byte copies for the ragged ends).
// Reference: pycylon compute where / fillna (python/pycylon/pycylon/data/compute.pyx), which
// run Arrow's host if_else / fill_null kernels.
#include "device_common.hpp"

namespace cylon {
namespace hip {

__device__ __forceinline__ bool sel_src(const uint8_t *cond, int64_t i) { return cond == nullptr || cond[i] != 0; }

__global__ void k_select_var_lengths(ColView a, ColView b, int b_bcast, const uint8_t *__restrict__ cond, int64_t n,
                                     int64_t *__restrict__ out_lens) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    if (sel_src(cond, i)) {
      out_lens[i] = a.offsets[i + 1] - a.offsets[i];
    } else if (b.offsets) {
      const int64_t j = b_bcast ? 0 : i;
      out_lens[i] = b.offsets[j + 1] - b.offsets[j];
    } else {
      out_lens[i] = 0;
    }
  }
}

__device__ __forceinline__ void wave_copy_bytes(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                int64_t len, int lane) {
  // 16-byte vector body when src and dst agree modulo 16; a row shorter than 64 B is byte-copied
  const uintptr_t sa = reinterpret_cast<uintptr_t>(src), da = reinterpret_cast<uintptr_t>(dst);
  if (len >= 64 && ((sa ^ da) & 15u) == 0) {
    const int64_t head = (int64_t)((16u - (sa & 15u)) & 15u);
    for (int64_t k = lane; k < head; k += kWave) dst[k] = src[k];
    const int64_t nv = (len - head) >> 4;
    const uint4 *s4 = reinterpret_cast<const uint4 *>(src + head);
    uint4 *d4 = reinterpret_cast<uint4 *>(dst + head);
    for (int64_t k = lane; k < nv; k += kWave) d4[k] = s4[k];
    for (int64_t k = head + (nv << 4) + lane; k < len; k += kWave) dst[k] = src[k];
  } else {
    for (int64_t k = lane; k < len; k += kWave) dst[k] = src[k];
  }
}

__global__ void k_select_var_bytes(ColView a, ColView b, int b_bcast, const uint8_t *__restrict__ cond, int64_t n,
                                   const int64_t *__restrict__ out_off, uint8_t *__restrict__ out_bytes,
                                   uint8_t *__restrict__ out_valid) {
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x / kWave);
  const int lane = lane_id();
  for (int64_t i = (int64_t)blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave; i < n; i += waves) {
    const bool from_a = sel_src(cond, i);
    const int64_t j = from_a ? i : (b_bcast ? 0 : i);
    const ColView &s = from_a ? a : b;
    uint8_t valid = 0;
    if (s.offsets) {
      const int64_t sb = s.offsets[j], len = s.offsets[j + 1] - sb;
      wave_copy_bytes(s.data + sb, out_bytes + out_off[i], len, lane);
      valid = s.valid ? s.valid[j] : (uint8_t)1;
    }
    if (lane == 0 && out_valid) out_valid[i] = valid;
  }
}

void select_var_lengths(const ColView &a, const ColView &b, int b_bcast, const uint8_t *cond, int64_t n,
                        int64_t *out_lens, void *stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_select_var_lengths, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), a, b, b_bcast, cond,
                     n, out_lens);
  HIP_LAUNCH_CHECK();
}

void select_var_bytes(const ColView &a, const ColView &b, int b_bcast, const uint8_t *cond, int64_t n,
                      const int64_t *out_offsets, uint8_t *out_bytes, uint8_t *out_valid, void *stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_select_var_bytes, dim3(grid_for(n, kBlock / kWave)), dim3(kBlock), 0, as_stream(stream), a, b,
                     b_bcast, cond, n, out_offsets, out_bytes, out_valid);
  HIP_LAUNCH_CHECK();
}

// this file's code object is loaded at context creation (preload_device_code), not on first use
void preload_select() { preload_code(reinterpret_cast<const void *>(&k_select_var_lengths)); }

}  // namespace hip
}  // namespace cylon
