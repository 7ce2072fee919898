// Stable bucket-ranking core shared by the partition scatter (K3) and the LSD
// radix sort passes (K6).
//
// A block owns a contiguous row range (rows_per_block, a multiple of the
// 2048-row sub-tile).  For every row the kernel finds the row's destination
//   dest = bh_scan[bucket * nblocks + block] + (#earlier rows of the block in bucket)
// which is a stable counting-sort position.  Inside a wave the rows that share
// a bucket are found by a wave64 "match": nbits 64-bit ballots, one per bucket
// bit; the in-wave rank is a single popcount.  Each wave keeps running bucket
// counters in LDS across its 8 rounds; the cross-wave prefix is formed once
// per sub-tile.  LDS: 8 B * buckets (running) + 16 B * buckets (4 waves).
#pragma once
#include "device_common.hpp"

namespace cylon {
namespace hip {

constexpr int kRankItems = 8;                     // rounds of 64 rows per wave per sub-tile
constexpr int kRankSubTile = kBlock * kRankItems;  // 2048 rows

struct RankGeometry {
  int64_t nblocks;
  int64_t rows_per_block;
};

inline RankGeometry rank_geometry(int64_t n, int64_t max_blocks = 4096) {
  RankGeometry g;
  int64_t tiles = (n + kRankSubTile - 1) / kRankSubTile;
  if (tiles < 1) tiles = 1;
  const int64_t nb = tiles < max_blocks ? tiles : max_blocks;
  const int64_t tiles_per_block = (tiles + nb - 1) / nb;
  g.rows_per_block = tiles_per_block * kRankSubTile;
  g.nblocks = (n + g.rows_per_block - 1) / g.rows_per_block;
  if (g.nblocks < 1) g.nblocks = 1;
  return g;
}

inline size_t rank_lds_bytes(uint32_t nbuckets) {
  return sizeof(int64_t) * nbuckets + sizeof(unsigned int) * (kBlock / kWave) * nbuckets;
}

// Block histogram: bh[bucket * nblocks + block] = #rows of the block in bucket.
template <class DigitFn>
__global__ __launch_bounds__(kBlock) void k_bucket_hist(DigitFn digit, int64_t n, uint32_t nbuckets,
                                                        int64_t rows_per_block, int64_t nblocks,
                                                        int64_t *__restrict__ bh) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned int *hist = reinterpret_cast<unsigned int *>(smem);
  for (uint32_t p = threadIdx.x; p < nbuckets; p += blockDim.x) hist[p] = 0;
  __syncthreads();
  const int64_t b = blockIdx.x;
  const int64_t begin = b * rows_per_block;
  const int64_t end = (begin + rows_per_block < n) ? begin + rows_per_block : n;
  for (int64_t i = begin + threadIdx.x; i < end; i += blockDim.x) atomicAdd(&hist[digit(i)], 1u);
  __syncthreads();
  for (uint32_t p = threadIdx.x; p < nbuckets; p += blockDim.x) bh[(int64_t)p * nblocks + b] = hist[p];
}

// WAVE_ATOMIC: the wave's own LDS counters hand out ranks by atomicAdd (stable because gfx950
// returns one instruction's same-address LDS atomics in lane order; radix_join.hip
// lds_lane_order_ok checks that on the device), instead of nbits ballots per row.
template <class DigitFn, class SinkFn, bool WAVE_ATOMIC>
__global__ __launch_bounds__(kBlock) void k_stable_rank(DigitFn digit, SinkFn sink, int64_t n, uint32_t nbuckets,
                                                        int nbits, int64_t rows_per_block, int64_t nblocks,
                                                        const int64_t *__restrict__ bh_scan) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  int64_t *running = reinterpret_cast<int64_t *>(smem);
  unsigned int *wcnt = reinterpret_cast<unsigned int *>(smem + sizeof(int64_t) * nbuckets);
  const int64_t b = blockIdx.x;
  for (uint32_t p = threadIdx.x; p < nbuckets; p += blockDim.x) {
    running[p] = bh_scan[(int64_t)p * nblocks + b];
#pragma unroll
    for (int w = 0; w < kBlock / kWave; ++w) wcnt[w * nbuckets + p] = 0;
  }
  __syncthreads();
  const int wave = threadIdx.x / kWave;
  const int lane = lane_id();
  const uint64_t lt = lanemask_lt();
  const int64_t begin = b * rows_per_block;
  const int64_t end = (begin + rows_per_block < n) ? begin + rows_per_block : n;
  unsigned int *mycnt = wcnt + wave * nbuckets;

  for (int64_t tile = begin; tile < end; tile += kRankSubTile) {
    uint32_t pk[kRankItems];
    uint32_t lk[kRankItems];
    const int64_t wbase = tile + (int64_t)wave * kWave * kRankItems;
#pragma unroll
    for (int k = 0; k < kRankItems; ++k) {
      const int64_t i = wbase + (int64_t)k * kWave + lane;
      const bool active = i < end;
      const uint32_t p = active ? digit(i) : 0u;
      if (WAVE_ATOMIC) {
        pk[k] = active ? p : 0xffffffffu;
        lk[k] = active ? atomicAdd(&mycnt[p], 1u) : 0u;
        continue;
      }
      uint64_t m = __ballot(active);
      for (int bit = 0; bit < nbits; ++bit) {
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
#pragma unroll
    for (int k = 0; k < kRankItems; ++k) {
      const uint32_t p = pk[k];
      if (p == 0xffffffffu) continue;
      int64_t off = running[p];
      for (int w = 0; w < wave; ++w) off += wcnt[w * nbuckets + p];
      sink(wbase + (int64_t)k * kWave + lane, off + lk[k]);
    }
    __syncthreads();
    for (uint32_t p = threadIdx.x; p < nbuckets; p += blockDim.x) {
      int64_t tot = 0;
#pragma unroll
      for (int w = 0; w < kBlock / kWave; ++w) {
        tot += wcnt[w * nbuckets + p];
        wcnt[w * nbuckets + p] = 0;
      }
      running[p] += tot;
    }
    __syncthreads();
  }
}

// Host driver: histogram -> scan -> stable rank.  ws must hold
// stable_rank_workspace(n, nbuckets) int64 values.
inline int64_t stable_rank_workspace(int64_t n, uint32_t nbuckets) {
  RankGeometry g = rank_geometry(n);
  const int64_t m = g.nblocks * (int64_t)nbuckets;
  return m + (m + 1) + scan_workspace(m);
}

template <class DigitFn, class SinkFn>
void stable_rank_launch(DigitFn digit, SinkFn sink, int64_t n, uint32_t nbuckets, int64_t *ws, hipStream_t s,
                        int64_t **bh_scan_out = nullptr, int64_t *nblocks_out = nullptr) {
  RankGeometry g = rank_geometry(n);
  const int64_t m = g.nblocks * (int64_t)nbuckets;
  int64_t *bh = ws;
  int64_t *bh_scan = ws + m;
  int64_t *scan_ws = bh_scan + m + 1;
  hipLaunchKernelGGL(k_bucket_hist<DigitFn>, dim3((unsigned)g.nblocks), dim3(kBlock),
                     nbuckets * sizeof(unsigned int), s, digit, n, nbuckets, g.rows_per_block, g.nblocks, bh);
  HIP_LAUNCH_CHECK();
  exclusive_scan(bh, m, bh_scan, scan_ws, reinterpret_cast<void *>(s));
  int nbits = 0;
  while ((1u << nbits) < nbuckets) ++nbits;
  if (lds_lane_order_ok(reinterpret_cast<void *>(s)))
    hipLaunchKernelGGL((k_stable_rank<DigitFn, SinkFn, true>), dim3((unsigned)g.nblocks), dim3(kBlock),
                       rank_lds_bytes(nbuckets), s, digit, sink, n, nbuckets, nbits, g.rows_per_block, g.nblocks,
                       bh_scan);
  else
    hipLaunchKernelGGL((k_stable_rank<DigitFn, SinkFn, false>), dim3((unsigned)g.nblocks), dim3(kBlock),
                       rank_lds_bytes(nbuckets), s, digit, sink, n, nbuckets, nbits, g.rows_per_block, g.nblocks,
                       bh_scan);
  HIP_LAUNCH_CHECK();
  if (bh_scan_out) *bh_scan_out = bh_scan;
  if (nblocks_out) *nblocks_out = g.nblocks;
}

}  // namespace hip
}  // namespace cylon
