// Arrow validity bitmaps <-> the engine's byte masks (the Arrow boundary: import,
// export, C Device Data interface).  Reference: util/copy_arrray.cpp:24-110 builds
// bitmaps row by row on the host.  Here a wave64 ballot IS one LSB-first bitmap
// word: pack is one coalesced byte load and one 8-byte store per 64 rows; unpack is
// one byte store per row.
#include "device_common.hpp"

namespace cylon {
namespace hip {

__global__ void k_pack_validity(const uint8_t *__restrict__ bytes, int64_t n, uint64_t *__restrict__ bitmap,
                                unsigned long long *__restrict__ nulls) {
  const int64_t words = (n + 63) / 64;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kWave;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) / kWave;
  const int lane = lane_id();
  unsigned long long z = 0;
  for (int64_t w = wave; w < words; w += nwaves) {
    const int64_t i = w * 64 + lane;
    const bool v = i < n && bytes[i] != 0;
    const uint64_t word = __ballot(v);
    if (lane == 0) {
      bitmap[w] = word;
      const int64_t valid_bits = (n - w * 64) < 64 ? (n - w * 64) : 64;
      z += (unsigned long long)(valid_bits - __popcll(word));
    }
  }
  if (lane == 0 && z) atomicAdd(nulls, z);
}

void pack_validity(const uint8_t *bytes, int64_t n, uint64_t *bitmap, int64_t *nulls, void *stream) {
  if (n == 0) return;
  const int64_t words = (n + 63) / 64;
  hipLaunchKernelGGL(k_pack_validity, dim3(grid_for(words * kWave)), dim3(kBlock), 0, as_stream(stream), bytes, n,
                     bitmap, reinterpret_cast<unsigned long long *>(nulls));
  HIP_LAUNCH_CHECK();
}

__global__ void k_unpack_validity(const uint8_t *__restrict__ bits, int64_t bit_offset, int64_t n,
                                  uint8_t *__restrict__ bytes) {
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += step) {
    const int64_t b = bit_offset + i;
    bytes[i] = (bits[b >> 3] >> (b & 7)) & 1;
  }
}

void unpack_validity(const uint8_t *bits, int64_t bit_offset, int64_t n, uint8_t *bytes, void *stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_unpack_validity, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), bits, bit_offset, n,
                     bytes);
  HIP_LAUNCH_CHECK();
}


// ---------------------------------------------------------------------------
// byte columns <-> 8-byte words (radix passes: validity bytes ride in 8-byte rows)
// ---------------------------------------------------------------------------
constexpr int kMaxByteCols = 64;

struct ByteCols {
  const uint8_t *in[kMaxByteCols];
  uint8_t *out[kMaxByteCols];
  const uint64_t *win[kMaxByteCols / 8];
  uint64_t *wout[kMaxByteCols / 8];
};

__global__ void k_pack_byte_columns(ByteCols c, int k, int64_t n) {
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  const int nw = (k + 7) / 8;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += step) {
#pragma unroll 1
    for (int w = 0; w < nw; ++w) {
      uint64_t word = 0;
      for (int j = 0; j < 8 && 8 * w + j < k; ++j) word |= (uint64_t)c.in[8 * w + j][i] << (8 * j);
      c.wout[w][i] = word;
    }
  }
}

__global__ void k_unpack_byte_columns(ByteCols c, int k, int64_t n) {
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  const int nw = (k + 7) / 8;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += step) {
#pragma unroll 1
    for (int w = 0; w < nw; ++w) {
      const uint64_t word = c.win[w][i];
      for (int j = 0; j < 8 && 8 * w + j < k; ++j) c.out[8 * w + j][i] = (uint8_t)(word >> (8 * j));
    }
  }
}

void pack_byte_columns(const uint8_t *const *cols, int k, int64_t n, uint64_t *const *words, void *stream) {
  CYLON_CHECK(k >= 1 && k <= kMaxByteCols, Code::Invalid, "byte column count " << k);
  if (n == 0) return;
  ByteCols c{};
  for (int j = 0; j < k; ++j) c.in[j] = cols[j];
  for (int w = 0; w < (k + 7) / 8; ++w) c.wout[w] = words[w];
  hipLaunchKernelGGL(k_pack_byte_columns, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), c, k, n);
  HIP_LAUNCH_CHECK();
}

void unpack_byte_columns(const uint64_t *const *words, int k, int64_t n, uint8_t *const *cols, void *stream) {
  CYLON_CHECK(k >= 1 && k <= kMaxByteCols, Code::Invalid, "byte column count " << k);
  if (n == 0) return;
  ByteCols c{};
  for (int j = 0; j < k; ++j) c.out[j] = cols[j];
  for (int w = 0; w < (k + 7) / 8; ++w) c.win[w] = words[w];
  hipLaunchKernelGGL(k_unpack_byte_columns, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), c, k, n);
  HIP_LAUNCH_CHECK();
}

// this file's code object is loaded at context creation (preload_device_code), not on first use
void preload_bitmap() { preload_code(reinterpret_cast<const void *>(&k_pack_validity)); }

}  // namespace hip
}  // namespace cylon
