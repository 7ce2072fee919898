#pragma once
// Shared device helpers and constants of the radix pass / LDS join kernels (radix_join.hip,
// lds_join.hip, range_join.hip).
#include "cylon/knobs.hpp"
#include <atomic>
#include <climits>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <type_traits>
#include <vector>

#include "stable_rank.hpp"

namespace cylon {
namespace hip {

constexpr int kRPThreads = 1024;                 // partition pass block (16 waves)
constexpr int kRPWaves = kRPThreads / kWave;
constexpr int kRPItems = 8;                      // rows per thread per tile
constexpr int kRPTile = kRPThreads * kRPItems;   // 8192 rows
constexpr int kRPMaxBuckets = 1024;
constexpr int kRJMaxDigitBits = 10;
constexpr int kRJRowArea = 154496;               // LDS bytes for the staged build rows (1 block per CU; 1 KB left for the emit owner map)
constexpr int kRJMaxRows = 5120;                 // build rows per partition (5 per thread)
constexpr int kRJThreads = 1024;
constexpr int kRankBallot = 0, kRankBlockAtomic = 1, kRankWaveAtomic = 2;
constexpr int kRJWaves = kRJThreads / kWave;

struct ColSet {
  const uint8_t *in[kMaxFusedCols];
  uint8_t *out[kMaxFusedCols];
  int width[kMaxFusedCols];
  int n;
  uint64_t key_xor;  // XORed into column 0 as it is stored (a sort's last pass rebuilds int64 keys from images)
  // Ranking guard (passes that must be stable): inside every bucket run of the sorted tile the
  // input rows must ascend; a violation -- the wave-atomic ranking relies on gfx950 returning one
  // instruction's same-address LDS atomics in lane order -- sets *order_bad.
  int check_order;
  int *order_bad;
  // Next-digit side output (LSD sort): as column 0 is stored at row r, nd_out[r] = (stored >>
  // nd_shift) & nd_mask -- the NEXT pass's digit, so that pass's per-tile histogram reads 2 bytes
  // per row instead of the 8-byte key (nullptr: off)
  uint16_t *nd_out;
  int nd_shift;
  uint32_t nd_mask;
  uint64_t nd_sub;  // the sort's ImageDigit::sub
};

// Digit read from a next-digit array written by the previous pass (histogram kernels only)
struct NdDigit {
  const uint16_t *d;
  __device__ __forceinline__ void init() {}
  __device__ __forceinline__ uint32_t operator()(int64_t i) const { return d[i]; }
};

// Digits of the pass kernels share: kNarrow (column 0 is stored as a uint32 offset, see
// PartDigitN), init() (per-block setup of device-resident fields) and key_at(i) (column 0's value).
#define CYLON_DIGIT_COMMON                                                                   \
  static constexpr bool kNarrow = false;                                                     \
  __device__ __forceinline__ void init() {}                                                  \
  __device__ __forceinline__ uint64_t key_at(int64_t i) const { return (uint64_t)keys[i]; } \
  __device__ __forceinline__ uint64_t narrow(uint64_t kv) const { return kv; }              \
  __device__ __forceinline__ bool too_wide(uint64_t) const { return false; }              \
  __device__ __forceinline__ void report_bad() const {}

__device__ __forceinline__ uint32_t part_of(int64_t key, int bits) {
  return bits == 0 ? 0u : (uint32_t)(hashing::fmix64((uint64_t)key) >> (64 - bits));
}

__device__ __forceinline__ long long rj_shfl_xor64(long long x, int mask) {
  const uint32_t lo = __shfl_xor((uint32_t)(uint64_t)x, mask, kWave);
  const uint32_t hi = __shfl_xor((uint32_t)((uint64_t)x >> 32), mask, kWave);
  return (long long)(((uint64_t)hi << 32) | lo);
}

__device__ __forceinline__ uint64_t ld_elem(const uint8_t *src, int64_t i, int w) {
  switch (w) {
    case 1: return src[i];
    case 2: return reinterpret_cast<const uint16_t *>(src)[i];
    case 4: return reinterpret_cast<const uint32_t *>(src)[i];
    default: return reinterpret_cast<const uint64_t *>(src)[i];
  }
}

__device__ __forceinline__ void st_elem(uint8_t *dst, int64_t i, int w, uint64_t v) {
  switch (w) {
    case 1: dst[i] = (uint8_t)v; break;
    case 2: reinterpret_cast<uint16_t *>(dst)[i] = (uint16_t)v; break;
    case 4: reinterpret_cast<uint32_t *>(dst)[i] = (uint32_t)v; break;
    default: reinterpret_cast<uint64_t *>(dst)[i] = v;
  }
}

// Column loops below are unrolled to compile-time bounds with `q < n` guards, so
// every ColSet field is a statically indexed kernel argument (SGPRs, loaded
// once); a runtime-indexed field would be re-fetched with a dependent scalar
// load per element.  W8 = every column 8 bytes wide (no width dispatch).
template <bool W8>
__device__ __forceinline__ uint64_t ldw(const uint8_t *p, int64_t i, int w) {
  return W8 ? reinterpret_cast<const uint64_t *>(p)[i] : ld_elem(p, i, w);
}
template <bool W8>
__device__ __forceinline__ void stw(uint8_t *p, int64_t i, int w, uint64_t v) {
  if (W8) reinterpret_cast<uint64_t *>(p)[i] = v; else st_elem(p, i, w, v);
}


constexpr int kXcds = 8;
__device__ __forceinline__ int xcc_id() {
  int x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & (kXcds - 1);
}

// LDS-DMA of `bytes` (a multiple of 4) contiguous global bytes into LDS at dst (16-byte aligned)
// by the block's WAVES waves: 1 KB pieces with global_load_lds_dwordx4 (a wave-instruction lands
// at its uniform base + lane * 16; the source may be only 8-byte aligned), the last < 16 bytes as
// dwords.  No VGPRs hold the data.
template <int WAVES>
__device__ __forceinline__ void rj_dma_block(const uint8_t *src, int bytes, uint8_t *dst, int wave, int lane) {
  const int nq = bytes >> 4;
  for (int c0 = wave * kWave; c0 < nq; c0 += WAVES * kWave)
    if (c0 + lane < nq)
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(src + (int64_t)(c0 + lane) * 16),
                                       (__attribute__((address_space(3))) void *)(dst + c0 * 16), 16, 0, 0);
  const int t0 = nq << 2, nd = bytes >> 2;  // tail dwords (at most 3)
  if (wave == WAVES - 1 && t0 + lane < nd)
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void *)(src + (int64_t)(t0 + lane) * 4),
                                     (__attribute__((address_space(3))) void *)(dst + t0 * 4), 4, 0, 0);
}

// block-wide exclusive scan of one uint32 per thread (WAVES waves)
template <int WAVES = kRPWaves>
__device__ __forceinline__ uint32_t rp_block_exscan(uint32_t c, uint32_t *wsum) {
  const int lane = lane_id(), wave = threadIdx.x / kWave;
  uint32_t inc = c;
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const uint32_t t = __shfl_up(inc, d, kWave);
    if (lane >= d) inc += t;
  }
  if (lane == kWave - 1) wsum[wave] = inc;
  __syncthreads();
  uint32_t off = 0;
#pragma unroll
  for (int w = 0; w < WAVES; ++w) off += (w < wave) ? wsum[w] : 0u;
  return off + inc - c;
}

}  // namespace hip
}  // namespace cylon
