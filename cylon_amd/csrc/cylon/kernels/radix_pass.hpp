// One LSD radix pass (8-bit digit) with an LDS-staged local shuffle (K6).
//
// Per block: a contiguous row range processed in 2048-row sub-tiles
// (256 threads x 8 rounds).  Rows are ranked per digit with the wave64 ballot
// match (stable_rank.hpp), then written into an LDS staging buffer in
// digit-sorted order and streamed out so that consecutive threads store
// consecutive destinations: each digit's run of the sub-tile (~8 rows on
// uniform keys, 64 B of keys) leaves as one contiguous segment instead of 8-byte
// stores to 64 different lines per wave instruction.
//
// The digit is a functor of the key so the same pass sorts plain keys
// (PlainDigit) or keys by their hash-table slot (SlotDigit, used by the
// atomic-free hash-join build).  A null value input means "value = row id".
#pragma once
#include "stable_rank.hpp"

namespace cylon {
namespace hip {

constexpr int kRadixBits = 8;
constexpr int kRadixBuckets = 1 << kRadixBits;

struct PlainDigit {
  int shift;
  __device__ __forceinline__ uint32_t operator()(uint64_t key) const {
    return (uint32_t)(key >> shift) & (kRadixBuckets - 1);
  }
};

// digit of the table slot of a key: slot = fmix64(key) >> slot_shift
struct SlotDigit {
  int slot_shift;
  int shift;
  __device__ __forceinline__ uint32_t operator()(uint64_t key) const {
    return (uint32_t)(hashing::slot_of(key, slot_shift) >> shift) & (kRadixBuckets - 1);
  }
};

template <class D>
struct KeyArrayDigit {
  const uint64_t *keys;
  D d;
  __device__ __forceinline__ uint32_t operator()(int64_t i) const { return d(keys[i]); }
};

__device__ __forceinline__ uint32_t block_excl_scan_u32(uint32_t v, uint32_t *lds_waves, uint32_t *total) {
  const int lane = lane_id();
  const int wave = threadIdx.x / kWave;
  uint32_t inc = v;
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const uint32_t t = __shfl_up(inc, d, kWave);
    if (lane >= d) inc += t;
  }
  if (lane == kWave - 1) lds_waves[wave] = inc;
  __syncthreads();
  uint32_t off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kBlock / kWave; ++w) {
    const uint32_t x = lds_waves[w];
    if (w < wave) off += x;
    tot += x;
  }
  __syncthreads();
  *total = tot;
  return off + inc - v;
}

// keys: uint64; vals: int64 (one 8-byte payload word per row; vin == nullptr -> row id)
template <class D>
__global__ __launch_bounds__(kBlock) void k_radix_pass_staged(D digit, const uint64_t *__restrict__ kin,
                                                              const int64_t *__restrict__ vin,
                                                              uint64_t *__restrict__ kout, int64_t *__restrict__ vout,
                                                              int64_t n, int64_t rows_per_block, int64_t nblocks,
                                                              const int64_t *__restrict__ bh_scan) {
  __shared__ __attribute__((aligned(16))) uint64_t skey[kRankSubTile];
  __shared__ __attribute__((aligned(16))) int64_t sval[kRankSubTile];
  __shared__ int64_t running[kRadixBuckets];
  __shared__ unsigned int wcnt[kBlock / kWave][kRadixBuckets];
  __shared__ uint32_t toff[kRadixBuckets];
  __shared__ uint32_t spk[kRankSubTile];
  __shared__ uint32_t scan_tmp[kBlock / kWave];

  const int64_t b = blockIdx.x;
  for (int p = threadIdx.x; p < kRadixBuckets; p += blockDim.x) {
    running[p] = bh_scan[(int64_t)p * nblocks + b];
#pragma unroll
    for (int w = 0; w < kBlock / kWave; ++w) wcnt[w][p] = 0;
  }
  __syncthreads();
  const int wave = threadIdx.x / kWave;
  const int lane = lane_id();
  const uint64_t lt = lanemask_lt();
  const int64_t begin = b * rows_per_block;
  const int64_t end = (begin + rows_per_block < n) ? begin + rows_per_block : n;
  unsigned int *mycnt = wcnt[wave];

  for (int64_t tile = begin; tile < end; tile += kRankSubTile) {
    uint64_t kk[kRankItems];
    int64_t vv[kRankItems];
    uint32_t pk[kRankItems];
    uint32_t lk[kRankItems];
    const int64_t wbase = tile + (int64_t)wave * kWave * kRankItems;
#pragma unroll
    for (int k = 0; k < kRankItems; ++k) {
      const int64_t i = wbase + (int64_t)k * kWave + lane;
      const bool active = i < end;
      kk[k] = active ? kin[i] : 0ull;
      vv[k] = active ? (vin ? vin[i] : i) : 0;
    }
#pragma unroll
    for (int k = 0; k < kRankItems; ++k) {
      const int64_t i = wbase + (int64_t)k * kWave + lane;
      const bool active = i < end;
      const uint32_t p = digit(kk[k]);
      uint64_t m = __ballot(active);
#pragma unroll
      for (int bit = 0; bit < kRadixBits; ++bit) {
        const uint32_t x = (p >> bit) & 1u;
        const uint64_t bb = __ballot(x);
        m &= x ? bb : ~bb;
      }
      const uint32_t rank = (uint32_t)__popcll(m & lt);
      uint32_t base = 0;
      if (active) base = mycnt[p];
      __builtin_amdgcn_wave_barrier();
      if (active && (m & lt) == 0) mycnt[p] = base + (uint32_t)__popcll(m);
      __builtin_amdgcn_wave_barrier();
      pk[k] = active ? p : 0xffffffffu;
      lk[k] = base + rank;
    }
    __syncthreads();
    {  // per-digit sub-tile counts -> local exclusive offsets (kBlock == kRadixBuckets)
      const int p = threadIdx.x;
      uint32_t c = 0;
#pragma unroll
      for (int w = 0; w < kBlock / kWave; ++w) c += wcnt[w][p];
      uint32_t tot;
      toff[p] = block_excl_scan_u32(c, scan_tmp, &tot);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kRankItems; ++k) {  // stage in digit order
      const uint32_t p = pk[k];
      if (p == 0xffffffffu) continue;
      uint32_t pos = toff[p] + lk[k];
      for (int w = 0; w < wave; ++w) pos += wcnt[w][p];
      skey[pos] = kk[k];
      sval[pos] = vv[k];
      spk[pos] = p;
    }
    __syncthreads();
    const int64_t cnt = (end - tile) < kRankSubTile ? (end - tile) : kRankSubTile;
    for (int j = threadIdx.x; j < cnt; j += kBlock) {  // consecutive threads -> consecutive destinations
      const uint32_t p = spk[j];
      const int64_t d = running[p] + (j - (int64_t)toff[p]);
      kout[d] = skey[j];
      vout[d] = sval[j];
    }
    __syncthreads();
    {
      const int p = threadIdx.x;
      int64_t tot = 0;
#pragma unroll
      for (int w = 0; w < kBlock / kWave; ++w) {
        tot += wcnt[w][p];
        wcnt[w][p] = 0;
      }
      running[p] += tot;
    }
    __syncthreads();
  }
}

// histogram -> scan -> staged scatter; ws holds stable_rank_workspace(n, 256)
template <class D>
inline void radix_pass(D digit, const uint64_t *kin, const int64_t *vin, uint64_t *kout, int64_t *vout, int64_t n,
                       int64_t *ws, hipStream_t s) {
  RankGeometry g = rank_geometry(n);
  const int64_t m = g.nblocks * (int64_t)kRadixBuckets;
  int64_t *bh = ws;
  int64_t *bh_scan = ws + m;
  int64_t *scan_ws = bh_scan + m + 1;
  hipLaunchKernelGGL(k_bucket_hist<KeyArrayDigit<D>>, dim3((unsigned)g.nblocks), dim3(kBlock),
                     kRadixBuckets * sizeof(unsigned int), s, KeyArrayDigit<D>{kin, digit}, n,
                     (uint32_t)kRadixBuckets, g.rows_per_block, g.nblocks, bh);
  HIP_LAUNCH_CHECK();
  exclusive_scan(bh, m, bh_scan, scan_ws, reinterpret_cast<void *>(s));
  hipLaunchKernelGGL(k_radix_pass_staged<D>, dim3((unsigned)g.nblocks), dim3(kBlock), 0, s, digit, kin, vin, kout,
                     vout, n, g.rows_per_block, g.nblocks, (const int64_t *)bh_scan);
  HIP_LAUNCH_CHECK();
}

}  // namespace hip
}  // namespace cylon
