// LDS radix hash join for large inner joins on a single exact int key (K3 + K5, gfx950).
//
// Measured on MI355X (tools/membench.hip, profiles/membench.txt): streaming
// copies run at 5.7 TB/s, but 8-byte accesses scattered over anything larger
// than an XCD's L2 (4 MB) run at ~50 G accesses/s whatever the window (1 MB
// ... 64 GB), i.e. < 0.5 TB/s of useful data.  A join built on random probes
// or gathers over the inputs is therefore bound by that rate (the global-table
// path: probe 200 ms + gathers 110 ms for 1B x 1B).  This path touches HBM
// only with coalesced streams:
//   1. radix-partition BOTH relations, all fixed-width columns (validity bytes
//      included), by the top `bits` bits of fmix64(key), with LSD passes of
//      <= 10 bits.  A pass ranks an 8192-row tile per digit (wave64 ballot
//      match, 16 waves), then moves each column through a 64 KB LDS stage:
//      coalesced loads are written to LDS at their sorted slot, and the
//      sorted tile is stored so that each digit's run (8192/512 = 16 rows =
//      128 B per 8-byte column on average) is one contiguous segment.
//   2. join bucket p of both sides in one workgroup: the build side's rows
//      (key + payload) are copied into LDS with coalesced loads and indexed by
//      an LDS open-addressing table (4096 slots, CAS insert).  A count kernel
//      gives per-partition output sizes, a device scan the offsets, and the
//      write kernel streams the probe rows, emitting every output column
//      directly (probe payload from HBM, build payload from LDS).  Each wave
//      owns a contiguous slice of the probe rows (wave-level scans only).
// Partitions whose build side exceeds the LDS capacity are reported; the
// caller then falls back to the global-table join.
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
};

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

// --------------------------------------------------------------------------
// partition pass
// --------------------------------------------------------------------------
// NARROW (narrow-key join, join.cpp radix_join): the two relations' keys span < 2^32 values, so
// a key's low 32 bits identify it; the partition hash is taken over those bits and column 0
// (the key) leaves the pass as uint32 -- 4 B/row less in every later pass and in the join
// kernels.  K = int64_t: the first pass reads the original keys; K = uint32_t: later passes.
template <class K, bool NARROW>
struct PartDigitT {
  static constexpr bool kNarrow = NARROW;  // column 0 is stored as uint32
  const K *keys;
  int bits;   // total partition bits
  int shift;  // digit = (part >> shift) & mask
  uint32_t mask;
  __device__ __forceinline__ uint32_t of_key(int64_t k) const {
    return (part_of(NARROW ? (int64_t)(uint32_t)(uint64_t)k : k, bits) >> shift) & mask;
  }
  __device__ __forceinline__ uint32_t operator()(int64_t i) const { return of_key((int64_t)keys[i]); }
};
using PartDigit = PartDigitT<int64_t, false>;
using PartDigitN64 = PartDigitT<int64_t, true>;   // first narrow pass: int64 keys in, uint32 out
using PartDigitN32 = PartDigitT<uint32_t, true>;  // later narrow passes


// Shuffle digit: the reference's partition of a single 8-byte integer key
// (ModuloPartitionKernel: h = (uint32)key, pid = h % P, or h & (P-1) for powers
// of two; partition.hip partition_f + hashing::partitioner), so one LDS-staged
// pass produces the partition-major order of the whole table.
struct ModDigit {
  static constexpr bool kNarrow = false;
  const int64_t *keys;
  uint32_t nparts;
  __device__ __forceinline__ uint32_t of_key(int64_t k) const {
    return hashing::partitioner((uint32_t)(uint64_t)k, nparts);
  }
  __device__ __forceinline__ uint32_t operator()(int64_t i) const { return of_key(keys[i]); }
};

// Sort digit: bits [shift, shift + log2(mask+1)) of an order-preserving uint64 image (K6).
struct ImageDigit {
  static constexpr bool kNarrow = false;
  const int64_t *keys;
  int shift;
  uint32_t mask;
  uint64_t flip;  // image = key ^ flip (0 once column 0 holds images)
  __device__ __forceinline__ uint32_t of_key(int64_t k) const {
    return (uint32_t)(((uint64_t)k ^ flip) >> shift) & mask;
  }
  __device__ __forceinline__ uint32_t operator()(int64_t i) const { return of_key(keys[i]); }
};

// Order-preserving range digit (K7 range join): the partition of key k is
// ((k ^ flip) - mn) >> rshift -- key ranges in key order -- and a pass's digit is
// bits [shift, shift + log2(mask + 1)) of that partition id.
struct RangeDigit {
  static constexpr bool kNarrow = false;
  const int64_t *keys;
  uint64_t flip, mn;
  int rshift, shift;
  uint32_t mask;
  __device__ __forceinline__ uint32_t of_key(int64_t k) const {
    return (uint32_t)((((uint64_t)k ^ flip) - mn) >> (rshift + shift)) & mask;
  }
  __device__ __forceinline__ uint32_t operator()(int64_t i) const { return of_key(keys[i]); }
};

template <class Digit>
__global__ __launch_bounds__(kRPThreads) void k_rp_hist(Digit digit, int64_t n, uint32_t nbuckets,
                                                        int64_t rows_per_block, int64_t nblocks,
                                                        int64_t *__restrict__ bh) {
  __shared__ unsigned int hist[kRPMaxBuckets];
  for (uint32_t p = threadIdx.x; p < nbuckets; p += blockDim.x) hist[p] = 0;
  __syncthreads();
  const int64_t begin = (int64_t)blockIdx.x * rows_per_block;
  const int64_t end = (begin + rows_per_block < n) ? begin + rows_per_block : n;
  for (int64_t i0 = begin; i0 < end; i0 += 4 * kRPThreads) {
    uint32_t d[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t i = i0 + u * kRPThreads + threadIdx.x;
      d[u] = i < end ? digit(i) : 0xffffffffu;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (d[u] != 0xffffffffu) atomicAdd(&hist[d[u]], 1u);
  }
  __syncthreads();
  for (uint32_t p = threadIdx.x; p < nbuckets; p += blockDim.x) bh[(int64_t)p * nblocks + blockIdx.x] = hist[p];
}

// k_rp_hist of a narrow-key join's first pass (low-32-bit digit) that also reduces the int64
// keys' min and max into mm[0] / mm[1] (atomics, initialised by the caller): the join decides
// from both relations' ranges whether the narrow passes apply, before the first pass runs.
__global__ __launch_bounds__(kRPThreads) void k_rp_hist_minmax(PartDigitN64 digit, int64_t n, uint32_t nbuckets,
                                                               int64_t rows_per_block, int64_t nblocks,
                                                               int64_t *__restrict__ bh, long long *__restrict__ mm) {
  __shared__ unsigned int hist[kRPMaxBuckets];
  for (uint32_t p = threadIdx.x; p < nbuckets; p += blockDim.x) hist[p] = 0;
  __syncthreads();
  const int64_t begin = (int64_t)blockIdx.x * rows_per_block;
  const int64_t end = (begin + rows_per_block < n) ? begin + rows_per_block : n;
  long long lo = LLONG_MAX, hi = LLONG_MIN;
  for (int64_t i0 = begin; i0 < end; i0 += 4 * kRPThreads) {
    int64_t k[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t i = i0 + u * kRPThreads + threadIdx.x;
      k[u] = i < end ? digit.keys[i] : 0;
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i0 + u * kRPThreads + threadIdx.x < end) {
        atomicAdd(&hist[digit.of_key(k[u])], 1u);
        lo = k[u] < lo ? k[u] : lo;
        hi = k[u] > hi ? k[u] : hi;
      }
  }
  for (int d = kWave / 2; d > 0; d >>= 1) {
    const long long a = rj_shfl_xor64(lo, d), b = rj_shfl_xor64(hi, d);
    lo = a < lo ? a : lo;
    hi = b > hi ? b : hi;
  }
  if (lane_id() == 0 && lo <= hi) {
    atomicMin(&mm[0], lo);
    atomicMax(&mm[1], hi);
  }
  __syncthreads();
  for (uint32_t p = threadIdx.x; p < nbuckets; p += blockDim.x) bh[(int64_t)p * nblocks + blockIdx.x] = hist[p];
}

// Chained-scan passes (decoupled lookback).  Histogram mode runs k_rp_hist before every pass:
// it re-reads the keys (8 B/row, 15 % of a key-only sort) to give each block's contiguous chunk
// its bucket offsets.  Lookback mode counts every pass's digits ONCE (k_lb_hist: the counts of a
// digit do not depend on the row order) and lets the pass kernel find a tile's offsets itself:
// tiles are claimed in row order from a ticket counter; a tile publishes its per-bucket count,
// then sums its predecessors' published counts back to the nearest tile that already published
// an inclusive prefix, and publishes its own.  Status words are 64-bit (flag | pass epoch | rows)
// relaxed agent-scope atomics: the value travels with its flag, so no fence is needed, and a
// word left by an earlier pass of the same session (other epoch) reads as "not ready".
constexpr int kLbMaxPasses = 8;
constexpr unsigned long long kLbAgg = 1ull << 62, kLbPrefix = 2ull << 62, kLbValue = (1ull << 56) - 1;

struct Lookback {
  const int64_t *gstart;         // exclusive global start of every bucket of this pass
  unsigned long long *status;    // [tile][nbuckets]
  unsigned int *ticket;          // next tile to claim
  unsigned long long epoch;      // 1..63
  // XCD-tile mode (XT): per-tile bucket offsets and one ticket per XCD (see k_rp_hist_tiles)
  const uint32_t *xt_off;        // [tile][nbuckets] output row of the tile's first row of each bucket
  unsigned int *xt_ticket;       // [8] next tile of each XCD's contiguous chunk
  int64_t xt_tiles;              // tiles of the pass
};

// XCD-tile mode.  Histogram mode gives each block a contiguous chunk of rows, so the tiles of
// one block write a bucket's consecutive runs ~34 us apart and the partial 128-B line at every
// run boundary has left the XCD's 4 MB L2 before the next tile completes it (~20 % extra HBM
// bytes, profiles/r03/pmc_join_1B_dma_vs_regstage.txt).  Here the tiles are split into 8
// contiguous chunks, one per XCD, and the XCD's CUs claim its tiles IN ORDER from a per-XCD
// ticket: at any moment an XCD's 32 CUs hold ~32 consecutive tiles, whose runs of each bucket
// are adjacent in the output and are written within a few us of each other into the same L2.
// Offsets are exact per tile (k_rp_hist_tiles + k_ts_*), so which CU takes a tile changes only
// speed; a block whose own chunk is exhausted takes tiles from the other chunks.
constexpr int kXcds = 8;
__device__ __forceinline__ int xcc_id() {
  int x;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(x));
  return x & (kXcds - 1);
}
// first row of the next tile this block processes, or n_rows when every chunk is exhausted
__device__ __forceinline__ int64_t xt_claim(const Lookback &lb, int home, int64_t tile_rows, int64_t n_rows) {
  for (int k = 0; k < kXcds; ++k) {
    const int x = (home + k) & (kXcds - 1);
    const int64_t lo = lb.xt_tiles * x / kXcds, hi = lb.xt_tiles * (x + 1) / kXcds;
    if (lo >= hi) continue;
    const int64_t j = (int64_t)atomicAdd(&lb.xt_ticket[x], 1u);
    if (lo + j < hi) return (lo + j) * tile_rows;
  }
  return n_rows;
}

// Windowed lookback in two steps: lb_publish stores tile t's count of bucket p right after the
// scan (successors can sum it while this tile ranks its slots); lb_exclusive then reads its
// predecessors' words kLbWin at a time (independent loads, one round trip per window),
// consumes them in order (waiting for any tile not ranked yet) until it meets an inclusive
// prefix, publishes t's own prefix and returns the rows of bucket p in tiles < t plus the
// bucket's global start.  One dependent load per predecessor cost the key-only sort ~50 % per
// pass: hundreds of tiles are in flight, and the walk back to the nearest prefix is long.  The
// window is not held across the slot phase (the loads' registers spill there).
constexpr int kLbWin = 8;

__device__ __forceinline__ unsigned long long lb_load(const unsigned long long *w) {
  return __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void lb_store(unsigned long long *w, unsigned long long v) {
  __hip_atomic_store(w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void lb_publish(const Lookback &lb, uint32_t nb, int64_t t, uint32_t p, uint32_t cnt) {
  const unsigned long long tag = lb.epoch << 56;
  if (t == 0) lb_store(lb.status + p, kLbPrefix | tag | (unsigned long long)(lb.gstart[p] + cnt));
  else lb_store(lb.status + t * nb + p, kLbAgg | tag | cnt);
}

__device__ __forceinline__ int64_t lb_exclusive(const Lookback &lb, uint32_t nb, int64_t t, uint32_t p, uint32_t cnt) {
  if (t == 0) return lb.gstart[p];
  int64_t excl = 0;
  for (int64_t j = t - 1;; j -= kLbWin) {
    unsigned long long v[kLbWin];
#pragma unroll
    for (int w = 0; w < kLbWin; ++w) v[w] = j - w >= 0 ? lb_load(lb.status + (j - w) * nb + p) : 0ull;
    bool found = false;
#pragma unroll
    for (int w = 0; w < kLbWin; ++w) {
      if (found || j - w < 0) continue;  // tile 0 always holds a prefix: the walk ends there at the latest
      unsigned long long x = v[w];
      while (((x >> 56) & 63ull) != lb.epoch) {  // tile j - w not ranked yet (its block is running)
        __builtin_amdgcn_s_sleep(1);
        x = lb_load(lb.status + (j - w) * nb + p);
      }
      excl += (int64_t)(x & kLbValue);
      found = (x & kLbPrefix) != 0;
    }
    if (found) break;
  }
  lb_store(lb.status + t * nb + p, kLbPrefix | (lb.epoch << 56) | (unsigned long long)(excl + cnt));
  return excl;
}

template <class Digit>
struct DigitSet {
  Digit d[kLbMaxPasses];
  int n;
};

// every pass's digit histogram in one read of the keys: hist[s][p] (u64, accumulated)
template <class Digit>
__global__ __launch_bounds__(kRPThreads) void k_lb_hist(DigitSet<Digit> ds, int64_t n, uint32_t nb,
                                                        unsigned long long *__restrict__ gh) {
  __shared__ unsigned int hist[kLbMaxPasses * kRPMaxBuckets];
  for (uint32_t q = threadIdx.x; q < (uint32_t)ds.n * nb; q += blockDim.x) hist[q] = 0;
  __syncthreads();
  const int64_t *keys = ds.d[0].keys;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t k = keys[i];
#pragma unroll
    for (int s = 0; s < kLbMaxPasses; ++s)
      if (s < ds.n) atomicAdd(&hist[s * nb + ds.d[s].of_key(k)], 1u);
  }
  __syncthreads();
  for (uint32_t q = threadIdx.x; q < (uint32_t)ds.n * nb; q += blockDim.x)
    if (hist[q]) atomicAdd(&gh[q], (unsigned long long)hist[q]);
}

// gstart[s][p] = exclusive scan of hist[s][.] (one block per pass)
__global__ __launch_bounds__(kRPThreads) void k_lb_scan(const unsigned long long *__restrict__ gh, uint32_t nb,
                                                        int64_t *__restrict__ gstart) {
  __shared__ int64_t wsum[kRPWaves];
  const int s = blockIdx.x, lane = lane_id(), wave = threadIdx.x / kWave;
  const uint32_t p = threadIdx.x;
  const int64_t c = p < nb ? (int64_t)gh[s * nb + p] : 0;
  int64_t inc = c;
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const int64_t t = __shfl_up(inc, d, kWave);
    if (lane >= d) inc += t;
  }
  if (lane == kWave - 1) wsum[wave] = inc;
  __syncthreads();
  int64_t off = 0;
  for (int w = 0; w < wave; ++w) off += wsum[w];
  if (p < nb) gstart[s * nb + p] = off + inc - c;
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

// The same DMA issued from inline asm (the recipe of cdna_hip_programming.md §4): hipcc then keeps
// no bookkeeping for it, so it does not drain it with vmcnt(0) before every later LDS access (it
// cannot tell the DMA's destination from the ranking counters) -- the caller waits for it with an
// explicit s_waitcnt before the buffer is read.  lds_base: the buffer's LDS byte address.
template <int WAVES>
__device__ __forceinline__ void rp_dma_asm(const uint8_t *src, int bytes, uint32_t lds_base, int wave, int lane) {
  const int nq = bytes >> 4;
  for (int c0 = wave * kWave; c0 < nq; c0 += WAVES * kWave) {
    const uint32_t dst = (uint32_t)__builtin_amdgcn_readfirstlane((int)(lds_base + (uint32_t)c0 * 16u));
    if (c0 + lane < nq) {
      const uint8_t *g = src + (int64_t)(c0 + lane) * 16;
      unsigned keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(g), "s"(dst) : "memory");
    }
  }
  const int t0 = nq << 2, nd = bytes >> 2;  // tail dwords (at most 3)
  if (wave == WAVES - 1 && t0 + lane < nd) {
    const uint32_t dst = (uint32_t)__builtin_amdgcn_readfirstlane((int)(lds_base + (uint32_t)t0 * 4u));
    const uint8_t *g = src + (int64_t)(t0 + lane) * 4;
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dword %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(dst) : "memory");
  }
}

// Block barrier.  RAW: LDS-only (lgkmcnt(0) + s_barrier) -- an LDS-DMA in flight stays in
// flight (__syncthreads() waits vmcnt(0) while one is outstanding: cdna_hip_programming.md §5).
template <bool RAW>
__device__ __forceinline__ void rp_sync() {
  if (RAW) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  } else {
    __syncthreads();
  }
}

// block-wide exclusive scan of one uint32 per thread (WAVES waves)
template <int WAVES = kRPWaves, bool RAW = false>
__device__ __forceinline__ uint32_t rp_block_exscan(uint32_t c, uint32_t *wsum) {
  const int lane = lane_id(), wave = threadIdx.x / kWave;
  uint32_t inc = c;
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const uint32_t t = __shfl_up(inc, d, kWave);
    if (lane >= d) inc += t;
  }
  if (lane == kWave - 1) wsum[wave] = inc;
  rp_sync<RAW>();
  uint32_t off = 0;
#pragma unroll
  for (int w = 0; w < WAVES; ++w) off += (w < wave) ? wsum[w] : 0u;
  return off + inc - c;
}

// ---- XCD-tile mode (XT) offsets: per-tile bucket counts, then exact output rows per (tile, bucket)
// th[t][p]: rows of bucket p in kRPTile-row tile t (uint16: a tile has <= 8192 rows).  512-thread
// blocks (up to four per CU), 16 rows per thread; the next tile's digits are loaded while this
// tile's LDS atomics and counter writes run, so the key stream never waits on the histogram.
constexpr int kHTThreads = 512, kHTItems = kRPTile / kHTThreads;
template <class Digit>
__device__ __forceinline__ void ht_load(const Digit &digit, int64_t n, int64_t t, int64_t ntiles,
                                        uint32_t (&d)[kHTItems]) {
  const int64_t r0 = t * kRPTile;
#pragma unroll
  for (int u = 0; u < kHTItems; ++u) {
    const int64_t i = r0 + u * kHTThreads + threadIdx.x;
    d[u] = t < ntiles && i < n ? digit(i) : 0xffffffffu;
  }
}
template <class Digit>
__global__ __launch_bounds__(kHTThreads) void k_rp_hist_tiles(Digit digit, int64_t n, uint32_t nb, int64_t ntiles,
                                                              uint16_t *__restrict__ th) {
  __shared__ unsigned int hist[kRPMaxBuckets];
  uint32_t d[kHTItems];
  ht_load(digit, n, blockIdx.x, ntiles, d);
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    for (uint32_t p = threadIdx.x; p < nb; p += blockDim.x) hist[p] = 0;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kHTItems; ++u)
      if (d[u] != 0xffffffffu) atomicAdd(&hist[d[u]], 1u);
    ht_load(digit, n, t + gridDim.x, ntiles, d);  // next tile in flight during the flush
    __syncthreads();
    for (uint32_t p = threadIdx.x; p < nb; p += blockDim.x) th[t * nb + p] = (uint16_t)hist[p];
    __syncthreads();
  }
}

constexpr int64_t kTsChunk = 512;  // tiles per chunk of the tile-offset scan

// csum[c][p] = rows of bucket p in chunk c's tiles (one thread per bucket)
__global__ void k_ts_chunk_sums(const uint16_t *__restrict__ th, uint32_t nb, int64_t ntiles,
                                uint32_t *__restrict__ csum) {
  const int64_t c = blockIdx.x, t0 = c * kTsChunk, t1 = t0 + kTsChunk < ntiles ? t0 + kTsChunk : ntiles;
  const uint32_t p = threadIdx.x;
  if (p >= nb) return;
  uint32_t acc = 0;
#pragma unroll 8
  for (int64_t t = t0; t < t1; ++t) acc += th[t * nb + p];
  csum[c * nb + p] = acc;
}

// cpre[c][p] = rows of bucket p in the chunks before c; bbase[p] = output row of bucket p's first
// row (bucket-major order).  One block; each thread batches its chunk loads (independent addresses).
__global__ __launch_bounds__(kRPThreads) void k_ts_chunk_prefix(const uint32_t *__restrict__ csum, uint32_t nb,
                                                                int64_t nchunks, uint32_t *__restrict__ cpre,
                                                                uint32_t *__restrict__ bbase) {
  __shared__ uint32_t wsum[kRPWaves];
  constexpr int B = 16;
  const uint32_t p = threadIdx.x;
  uint32_t acc = 0;
  if (p < nb)
    for (int64_t c0 = 0; c0 < nchunks; c0 += B) {
      uint32_t x[B];
#pragma unroll
      for (int u = 0; u < B; ++u) x[u] = c0 + u < nchunks ? csum[(c0 + u) * nb + p] : 0u;
#pragma unroll
      for (int u = 0; u < B; ++u)
        if (c0 + u < nchunks) {
          cpre[(c0 + u) * nb + p] = acc;
          acc += x[u];
        }
    }
  const uint32_t base = rp_block_exscan<kRPWaves>(p < nb ? acc : 0u, wsum);
  if (p < nb) bbase[p] = base;
}

// off[t][p] = output row of tile t's first row of bucket p
__global__ void k_ts_offsets(const uint16_t *__restrict__ th, const uint32_t *__restrict__ cpre,
                             const uint32_t *__restrict__ bbase, uint32_t nb, int64_t ntiles,
                             uint32_t *__restrict__ off) {
  const int64_t c = blockIdx.x, t0 = c * kTsChunk, t1 = t0 + kTsChunk < ntiles ? t0 + kTsChunk : ntiles;
  const uint32_t p = threadIdx.x;
  if (p >= nb) return;
  uint32_t acc = cpre[c * nb + p] + bbase[p];
#pragma unroll 8
  for (int64_t t = t0; t < t1; ++t) {
    off[t * nb + p] = acc;
    acc += th[t * nb + p];
  }
}


// LDS: running (8 KB) + toff (4 KB) + one 64 KB union that holds the per-wave
// digit counters and the sorted-slot digits while ranking, then the column
// stage (76 KB).  One 1024-thread block per CU (the ranking needs ~120 VGPRs);
// global latency is hidden by software pipelining in registers instead: the
// loads of column c+1 (and, during the last column, the next tile's keys) are
// in flight while column c streams out of the stage.  Column 0 is the key.
//
// THREADS = 512 runs two 4096-row blocks per CU instead of one 8192-row block, so
// one block's ranking overlaps the other's memory traffic (every stage write waits
// with vmcnt(0) for all outstanding loads AND stores: gfx9 counts both on one
// counter).  Issuing several columns' loads per wait instead (more VGPRs, fewer
// waves) measured slower -- profiles/rows_pass_experiments_r02.txt.
// Debug phase stamps (CYLON_RP_STAMPS=1, rows_pass_launch): wave 0 of block 0 records the
// shader clock at each phase boundary of its first kRPStampTiles tiles; nullptr otherwise.
constexpr int kRPStampTiles = 64, kRPStampSlots = 16;
#define RP_STAMP(slot)                                                                               \
  do {                                                                                               \
    if (stamps != nullptr && blockIdx.x == 0 && tix >= 0 && tix < kRPStampTiles && (slot) < kRPStampSlots) { \
      unsigned long long t_;                                                                         \
      __builtin_amdgcn_sched_barrier(0);                                                             \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                    \
      __builtin_amdgcn_sched_barrier(0);                                                             \
      if (threadIdx.x == 0) stamps[tix * kRPStampSlots + (slot)] = t_;                               \
    }                                                                                                \
  } while (0)

// RANK: kRankBallot (stable wave64 ballot match), kRankBlockAtomic (one LDS atomic per row
// on block-wide counters: unstable), kRankWaveAtomic (LDS atomics on the wave's own packed
// 16-bit counters: stable exactly when one instruction's same-address atomics return in lane
// order -- tools/lds_atomic_order.hip measures that on the device).
// LB: lookback mode (tiles claimed from lb.ticket, offsets by decoupled lookback; bh_scan unused).
// DMA1 (W8, >= 2 columns, column 1 read from memory): column 1 of the tile is fetched by LDS-DMA
// into a second 64 KB buffer as soon as the tile's digits are known, so the load streams during the
// ranking / scan / slot / destination phases (which move no bytes of their own) instead of behind
// column 0's scatter; those phases then synchronise with LDS-only barriers.
template <class Digit, bool W8, int THREADS, int RANK, bool LB, bool DMA1 = false, bool XT = false>
__global__ __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(4))) void k_rows_pass(
    Digit digit, int nbits, uint32_t nbuckets, ColSet cols, int64_t n, int64_t rows_per_block, int64_t nblocks,
    const int64_t *__restrict__ bh_scan, Lookback lb, unsigned long long *__restrict__ stamps) {
  constexpr int WAVES = THREADS / kWave;
  constexpr int TILE = THREADS * kRPItems;
  constexpr int BPT = (kRPMaxBuckets + THREADS - 1) / THREADS;  // buckets per thread in the offset scan
  constexpr bool K4 = Digit::kNarrow;  // column 0 (the key) is stored as uint32
  static_assert(WAVES * kRPMaxBuckets * 2 + TILE * 4 <= TILE * 8, "ranking scratch must fit the stage");
  static_assert(!LB || (THREADS >= kRPMaxBuckets && TILE == kRPTile), "lookback: one bucket a thread, 8192-row tiles");
  static_assert(!DMA1 || (W8 && !LB), "column-1 DMA: 8-byte columns, histogram mode");
  static_assert(!(LB && XT), "one tile schedule");
  constexpr bool TICKET = LB || XT;  // tiles claimed one by one (not a contiguous chunk per block)
  const int xhome = XT ? xcc_id() : 0;
  __shared__ int64_t running[kRPMaxBuckets];
  __shared__ __attribute__((aligned(16))) uint64_t land[DMA1 ? TILE : 1];  // column 1 of the tile (DMA1)
  __shared__ uint32_t toff[kRPMaxBuckets + 1];
  __shared__ uint64_t ustage[TILE];  // column stage | {wcnt[WAVES][nb] u16, sdig[TILE] u32}
  __shared__ uint32_t wsum[WAVES];
  uint16_t *wcnt = reinterpret_cast<uint16_t *>(ustage);
  constexpr bool STABLE = RANK != kRankBlockAtomic;
  uint32_t *bcnt = reinterpret_cast<uint32_t *>(ustage);  // block-atomic ranking: block-wide counters
  static_assert(WAVES * kRPMaxBuckets * 2 >= kRPMaxBuckets * 4, "block counters must fit the wave counters");
  // sorted slot j -> digit << 16 | input row in the tile (the row feeds the ranking guard)
  uint32_t *sdig = reinterpret_cast<uint32_t *>(wcnt + WAVES * kRPMaxBuckets);
  uint8_t *st = reinterpret_cast<uint8_t *>(ustage);
  __shared__ int64_t s_next;  // LB: first row of the next claimed tile
  bool order_bad = false;

  const int64_t b = blockIdx.x;
  int64_t begin, end;
  if (TICKET) {
    if (threadIdx.x == 0) s_next = XT ? xt_claim(lb, xhome, TILE, n) : (int64_t)atomicAdd(lb.ticket, 1u) * TILE;
    __syncthreads();
    begin = s_next;
    end = n;
  } else {
    for (uint32_t p = threadIdx.x; p < nbuckets; p += blockDim.x) running[p] = bh_scan[(int64_t)p * nblocks + b];
    begin = b * rows_per_block;
    end = (begin + rows_per_block < n) ? begin + rows_per_block : n;
  }
  const int wave = threadIdx.x / kWave;
  const int lane = lane_id();
  const uint64_t lt = lanemask_lt();
  uint16_t *mycnt = wcnt + wave * nbuckets;
  const int wrow = wave * kWave * kRPItems;

  uint64_t kv[kRPItems];  // keys of the current tile (column 0)
#pragma unroll
  for (int k = 0; k < kRPItems; ++k) {
    const int64_t i = begin + wrow + k * kWave + lane;
    if (i < end) kv[k] = (uint64_t)digit.keys[i];
  }
  for (int64_t tile = begin, next = 0; tile < end; tile = next) {
    next = tile + TILE;
    const int tix = (int)((tile - begin) / TILE);
    RP_STAMP(0);
    const int cnt = (int)((end - tile) < TILE ? (end - tile) : TILE);
    // XT: this tile's bucket offsets (consumed after the slot phase; the load overlaps the ranking)
    const uint32_t xoff = XT && threadIdx.x < nbuckets ? lb.xt_off[(tile / TILE) * nbuckets + threadIdx.x] : 0u;
    uint32_t pl[kRPItems];  // digit, then (in-wave rank << 16) | digit, then sorted slot; ~0 = inactive
#pragma unroll
    for (int k = 0; k < kRPItems; ++k)
      pl[k] = (wrow + k * kWave + lane < cnt) ? digit.of_key((int64_t)kv[k]) : 0xffffffffu;
    // the digits consumed the prefetched keys (their loads are retired), so this DMA is the only
    // vector-memory work in flight through the LDS-only barriers below
    if (DMA1)
      rp_dma_asm<WAVES>(cols.in[1] + tile * 8, cnt * 8,
                        (uint32_t)(uintptr_t)(__attribute__((address_space(3))) uint64_t *)(land),
                        wave, lane);
    RP_STAMP(1);
    if (STABLE) {
      for (uint32_t q = threadIdx.x; q < WAVES * nbuckets; q += blockDim.x) wcnt[q] = 0;
    } else {
      for (uint32_t q = threadIdx.x; q < nbuckets; q += blockDim.x) bcnt[q] = 0;
    }
    rp_sync<DMA1>();  // also orders the previous tile's stage reads before the counters reuse it
    if (!STABLE) {
      // order inside a bucket's run is free (join partitions): one LDS atomic per row
      // replaces the nbits ballots of the stable match
#pragma unroll
      for (int k = 0; k < kRPItems; ++k)
        if (pl[k] != 0xffffffffu) pl[k] |= atomicAdd(&bcnt[pl[k]], 1u) << 16;
    } else if (RANK == kRankWaveAtomic) {
      uint32_t *myw = reinterpret_cast<uint32_t *>(mycnt);  // nbuckets is even: word-aligned rows
#pragma unroll
      for (int k = 0; k < kRPItems; ++k)
        if (pl[k] != 0xffffffffu) {
          const uint32_t p = pl[k], sh = (p & 1u) * 16u;
          pl[k] |= ((atomicAdd(&myw[p >> 1], 1u << sh) >> sh) & 0xffffu) << 16;
        }
    } else
#pragma unroll
    for (int k = 0; k < kRPItems; ++k) {
      const bool active = pl[k] != 0xffffffffu;
      const uint32_t p = active ? pl[k] : 0u;
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
      if (active && (m & lt) == 0) mycnt[p] = (uint16_t)(base + (uint32_t)__popcll(m));
      __builtin_amdgcn_wave_barrier();
      pl[k] = active ? (((base + rank) << 16) | p) : 0xffffffffu;
    }
    rp_sync<DMA1>();
    RP_STAMP(2);
    {  // thread owns buckets [t*BPT, t*BPT+BPT): exclusive prefix over waves (in place), then a
       // block scan of the thread totals
      uint32_t loc[BPT];
      uint32_t total = 0;
#pragma unroll
      for (int i = 0; i < BPT; ++i) {
        const uint32_t p = threadIdx.x * BPT + i;
        loc[i] = total;
        uint32_t run = 0;
        if (p < nbuckets) {
          if (STABLE) {
#pragma unroll
            for (int w = 0; w < WAVES; ++w) {
              const uint32_t c = wcnt[w * nbuckets + p];
              wcnt[w * nbuckets + p] = (uint16_t)run;
              run += c;
            }
          } else {
            run = bcnt[p];
          }
        }
        total += run;
      }
      const uint32_t ex = rp_block_exscan<WAVES, DMA1>(total, wsum);
#pragma unroll
      for (int i = 0; i < BPT; ++i) {
        const uint32_t p = threadIdx.x * BPT + i;
        if (p < nbuckets) toff[p] = ex + loc[i];
      }
      if (threadIdx.x == THREADS - 1) toff[nbuckets] = ex + total;
    }
    rp_sync<DMA1>();
    RP_STAMP(3);
    // LB: this tile's bucket offsets from its predecessors (read by the dst phase): count published
    // before the slot phase, lookback after it.  nbuckets <= THREADS: one bucket a thread
    const uint32_t lbc = LB && threadIdx.x < nbuckets ? toff[threadIdx.x + 1] - toff[threadIdx.x] : 0u;
    if (LB && threadIdx.x < nbuckets) lb_publish(lb, nbuckets, tile / TILE, threadIdx.x, lbc);
#pragma unroll
    for (int k = 0; k < kRPItems; ++k) {
      if (pl[k] == 0xffffffffu) continue;
      const uint32_t p = pl[k] & 0xffffu;
      const uint32_t pos = toff[p] + (STABLE ? (uint32_t)wcnt[wave * nbuckets + p] : 0u) + (pl[k] >> 16);
      sdig[pos] = (p << 16) | (uint32_t)(wrow + k * kWave + lane);
      pl[k] = pos;
    }
    if (LB && threadIdx.x < nbuckets) running[threadIdx.x] = lb_exclusive(lb, nbuckets, tile / TILE, threadIdx.x, lbc);
    if (XT && threadIdx.x < nbuckets) running[threadIdx.x] = xoff;
    rp_sync<DMA1>();
    RP_STAMP(4);
    int64_t dst[kRPItems];  // destination of sorted slot j = threadIdx.x + q * THREADS
#pragma unroll
    for (int q = 0; q < kRPItems; ++q) {
      const int j = threadIdx.x + q * THREADS;
      if (j < cnt) {
        const uint32_t e = sdig[j], p = e >> 16;
        dst[q] = running[p] + (j - (int64_t)toff[p]);
        if (cols.check_order && j > 0) {  // same bucket as the previous slot: input order kept?
          const uint32_t f = sdig[j - 1];
          order_bad |= (f >> 16) == p && f > e;
        }
      }
    }
    rp_sync<DMA1>();  // counters / digits dead: the union becomes the column stage
    RP_STAMP(5);
    // load column c+1 while column c streams out of the stage
    uint64_t v[kRPItems];
#pragma unroll
    for (int k = 0; k < kRPItems; ++k) v[k] = kv[k];
#pragma unroll 1
    for (int c = 0; c < cols.n; ++c) {  // column fields fetched once per column (scalar loads)
      const int w = cols.width[c];
      if (DMA1 && c == 1) {  // column 1 landed by DMA (waited for at the end of column 0)
#pragma unroll
        for (int k = 0; k < kRPItems; ++k) v[k] = land[wrow + k * kWave + lane];
      }
      uint8_t *out = cols.out[c];
      const uint64_t x = c == 0 ? cols.key_xor : 0ull;
      if (TICKET && c + 1 == cols.n && threadIdx.x == 0)
        s_next = XT ? xt_claim(lb, xhome, TILE, n) : (int64_t)atomicAdd(lb.ticket, 1u) * TILE;
      const bool k4 = K4 && c == 0;  // narrow key: column 0 leaves as its low 32 bits
      if (k4) {
#pragma unroll
        for (int k = 0; k < kRPItems; ++k)
          if (pl[k] != 0xffffffffu) reinterpret_cast<uint32_t *>(st)[pl[k]] = (uint32_t)v[k];
      } else {
#pragma unroll
        for (int k = 0; k < kRPItems; ++k)
          if (pl[k] != 0xffffffffu) stw<W8>(st, pl[k], w, v[k] ^ x);
      }
      __syncthreads();
      if (TICKET && c + 1 == cols.n) next = s_next;
      RP_STAMP(6 + 2 * c);
      if (DMA1 && c == 0) {
        // column 1 is in flight by DMA: nothing to prefetch behind column 0
      } else if (c + 1 < cols.n) {  // prefetch column c+1 of this tile
        const uint8_t *in = cols.in[c + 1];
        const int w1 = cols.width[c + 1];
        if (in == nullptr) {  // row-id column: the pass generates it (no 8 B/row array to read)
#pragma unroll
          for (int k = 0; k < kRPItems; ++k) v[k] = (uint64_t)(tile + wrow + k * kWave + lane);
        } else {
#pragma unroll
          for (int k = 0; k < kRPItems; ++k)
            if (pl[k] != 0xffffffffu) v[k] = ldw<W8>(in, tile + wrow + k * kWave + lane, w1);
        }
      } else {  // prefetch the next tile's keys
#pragma unroll
        for (int k = 0; k < kRPItems; ++k) {
          const int64_t i = next + wrow + k * kWave + lane;
          if (i < end) kv[k] = (uint64_t)digit.keys[i];
        }
      }
      if (k4) {
#pragma unroll
        for (int q = 0; q < kRPItems; ++q) {
          const int j = threadIdx.x + q * THREADS;
          if (j < cnt) reinterpret_cast<uint32_t *>(out)[dst[q]] = reinterpret_cast<const uint32_t *>(st)[j];
        }
      } else {
#pragma unroll
        for (int q = 0; q < kRPItems; ++q) {
          const int j = threadIdx.x + q * THREADS;
          if (j < cnt) stw<W8>(out, dst[q], w, ldw<W8>(st, j, w));
        }
      }
      if (DMA1 && c == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // column 1 has landed
      __syncthreads();
      RP_STAMP(7 + 2 * c);
    }
    if (!TICKET)
      for (uint32_t p = threadIdx.x; p < nbuckets; p += blockDim.x) running[p] += toff[p + 1] - toff[p];
  }
  if (order_bad) atomicOr(cols.order_bad, 1);
}

// Register-lean pass: the same tile algorithm (8192-row tiles, LDS-atomic ranking, one
// 64 KB column stage), restructured so that TWO 1024-thread blocks fit a CU (<= 64 VGPRs,
// 76 KB LDS each): one block's ranking / scans / barriers then run while the other block's
// columns stream, instead of leaving the CU's share of HBM idle for a third of every tile
// (profiles/rank_variants_r02.txt: 33 % of a join tile has no memory traffic).  What the
// classic kernel held in registers across phases is dropped or packed:
//   * no cross-column / cross-tile prefetch (the second block hides the load latency);
//   * the destination of sorted slot j is packed as (digit << 16 | j - toff[digit]) and
//     completed from running[] in LDS at store time (8 VGPRs instead of 16).
template <class Digit, bool W8, int RANK, bool LB, bool XT = false>
__global__ __launch_bounds__(kRPThreads) __attribute__((amdgpu_waves_per_eu(8))) void k_rows_pass_lean(
    Digit digit, int nbits, uint32_t nbuckets, ColSet cols, int64_t n, int64_t rows_per_block, int64_t nblocks,
    const int64_t *__restrict__ bh_scan, Lookback lb) {
  constexpr int THREADS = kRPThreads, WAVES = THREADS / kWave, TILE = THREADS * kRPItems;
  constexpr int BPT = (kRPMaxBuckets + THREADS - 1) / THREADS;
  static_assert(WAVES * kRPMaxBuckets * 2 + TILE * 4 <= TILE * 8, "ranking scratch must fit the stage");
  __shared__ int64_t running[kRPMaxBuckets];
  __shared__ uint32_t toff[kRPMaxBuckets + 1];
  __shared__ uint64_t ustage[TILE];  // column stage | {wcnt[WAVES][nb] u16 or bcnt[nb] u32, sdig[TILE] u16}
  __shared__ uint32_t wsum[WAVES];
  constexpr bool STABLE = RANK != kRankBlockAtomic;
  uint16_t *wcnt = reinterpret_cast<uint16_t *>(ustage);
  uint32_t *bcnt = reinterpret_cast<uint32_t *>(ustage);
  uint32_t *sdig = reinterpret_cast<uint32_t *>(wcnt + WAVES * kRPMaxBuckets);  // digit << 16 | input row
  uint8_t *st = reinterpret_cast<uint8_t *>(ustage);
  __shared__ int64_t s_next;  // LB / XT: first row of the next claimed tile
  bool order_bad = false;
  (void)nbits;
  static_assert(!(LB && XT), "one tile schedule");
  constexpr bool TICKET = LB || XT;
  const int xhome = XT ? xcc_id() : 0;

  const int64_t b = blockIdx.x;
  int64_t begin, end;
  if (TICKET) {
    if (threadIdx.x == 0) s_next = XT ? xt_claim(lb, xhome, TILE, n) : (int64_t)atomicAdd(lb.ticket, 1u) * TILE;
    __syncthreads();
    begin = s_next;
    end = n;
  } else {
    for (uint32_t p = threadIdx.x; p < nbuckets; p += THREADS) running[p] = bh_scan[(int64_t)p * nblocks + b];
    begin = b * rows_per_block;
    end = (begin + rows_per_block < n) ? begin + rows_per_block : n;
  }
  // wave index made provably uniform: per-wave base pointers then live in SGPRs and every
  // load / store addresses its row with a 32-bit lane offset plus an immediate
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  uint16_t *mycnt = wcnt + wave * nbuckets;
  const int wrow = wave * kWave * kRPItems;

  for (int64_t tile = begin, next = 0; tile < end; tile = next) {
    next = tile + TILE;
    const int cnt = (int)((end - tile) < TILE ? (end - tile) : TILE);
    // per-thread constants are recomputed every tile from an opaque copy of the thread id:
    // hoisted out of the tile loop they outlive the 64-VGPR budget and spill
    int tx = (int)threadIdx.x;
    asm volatile("" : "+v"(tx));
    const int lane = tx & (kWave - 1);
    // XT: this tile's bucket offsets (stored to running[] after the slot phase)
    const uint32_t xoff = XT && (uint32_t)tx < nbuckets ? lb.xt_off[(tile / TILE) * nbuckets + tx] : 0u;
    uint32_t pl[kRPItems];  // digit | in-tile rank << 16, then the sorted slot; ~0 = inactive
    const int64_t *kbase = digit.keys + tile + wrow;  // wave-uniform
    const int lim = cnt - wrow;                       // rows of this wave's slice that exist
    {  // the keys are not held across the ranking: column 0 re-reads them (L2 hits) like any column
      uint64_t kk[kRPItems];
#pragma unroll
      for (int k = 0; k < kRPItems; ++k) kk[k] = (k * kWave + lane < lim) ? (uint64_t)kbase[k * kWave + lane] : 0ull;
#pragma unroll
      for (int k = 0; k < kRPItems; ++k) pl[k] = (k * kWave + lane < lim) ? digit.of_key((int64_t)kk[k]) : 0xffffffffu;
    }
    if (STABLE) {
      for (uint32_t q = tx; q < WAVES * nbuckets; q += THREADS) wcnt[q] = 0;
    } else {
      for (uint32_t q = tx; q < nbuckets; q += THREADS) bcnt[q] = 0;
    }
    __syncthreads();  // also: the previous tile's stage reads are done
    if (!STABLE) {
#pragma unroll
      for (int k = 0; k < kRPItems; ++k)
        if (pl[k] != 0xffffffffu) pl[k] |= atomicAdd(&bcnt[pl[k]], 1u) << 16;
    } else {
      uint32_t *myw = reinterpret_cast<uint32_t *>(mycnt);
#pragma unroll
      for (int k = 0; k < kRPItems; ++k)
        if (pl[k] != 0xffffffffu) {
          const uint32_t p = pl[k], sh = (p & 1u) * 16u;
          pl[k] |= ((atomicAdd(&myw[p >> 1], 1u << sh) >> sh) & 0xffffu) << 16;
        }
    }
    __syncthreads();
    {
      uint32_t loc[BPT];
      uint32_t total = 0;
#pragma unroll
      for (int i = 0; i < BPT; ++i) {
        const uint32_t p = tx * BPT + i;
        loc[i] = total;
        uint32_t run = 0;
        if (p < nbuckets) {
          if (STABLE) {
#pragma unroll
            for (int w = 0; w < WAVES; ++w) {
              const uint32_t c = wcnt[w * nbuckets + p];
              wcnt[w * nbuckets + p] = (uint16_t)run;
              run += c;
            }
          } else {
            run = bcnt[p];
          }
        }
        total += run;
      }
      const uint32_t ex = rp_block_exscan<WAVES>(total, wsum);
#pragma unroll
      for (int i = 0; i < BPT; ++i) {
        const uint32_t p = tx * BPT + i;
        if (p < nbuckets) toff[p] = ex + loc[i];
      }
      if (tx == THREADS - 1) toff[nbuckets] = ex + total;
    }
    __syncthreads();
    // LB: this tile's bucket offsets (read by the column stores): count published before the slot
    // phase, lookback after it.  nbuckets <= THREADS: one bucket a thread
    const uint32_t lbc = LB && (uint32_t)tx < nbuckets ? toff[tx + 1] - toff[tx] : 0u;
    if (LB && (uint32_t)tx < nbuckets) lb_publish(lb, nbuckets, tile / TILE, tx, lbc);
#pragma unroll
    for (int k = 0; k < kRPItems; ++k) {
      if (pl[k] == 0xffffffffu) continue;
      const uint32_t p = pl[k] & 0xffffu;
      const uint32_t pos = toff[p] + (STABLE ? (uint32_t)wcnt[wave * nbuckets + p] : 0u) + (pl[k] >> 16);
      sdig[pos] = (p << 16) | (uint32_t)(wrow + k * kWave + lane);
      pl[k] = pos;
    }
    if (LB && (uint32_t)tx < nbuckets) running[tx] = lb_exclusive(lb, nbuckets, tile / TILE, tx, lbc);
    if (XT && (uint32_t)tx < nbuckets) running[tx] = xoff;
    __syncthreads();
    uint32_t dp[kRPItems];  // sorted slot j = tx + q * THREADS -> digit << 16 | offset in its run
#pragma unroll
    for (int q = 0; q < kRPItems; ++q) {
      const int j = tx + q * THREADS;
      const uint32_t e = j < cnt ? sdig[j] : 0u, p = e >> 16;
      dp[q] = (p << 16) | (uint32_t)(j - (int)toff[p]);
      if (cols.check_order && j > 0 && j < cnt) {  // same bucket as the previous slot: input order kept?
        const uint32_t f = sdig[j - 1];
        order_bad |= (f >> 16) == p && f > e;
      }
    }
    __syncthreads();  // counters / digits dead: the union becomes the column stage
#pragma unroll 1
    for (int c = 0; c < cols.n; ++c) {
      const int w = cols.width[c];
      uint8_t *out = cols.out[c];
      uint64_t v[kRPItems];
      const uint8_t *in = cols.in[c];
      if (in == nullptr) {  // generated row-id column (computed here, not hoisted: 16 VGPRs)
        int64_t rbase = tile + wrow;
        asm volatile("" : "+s"(rbase));
#pragma unroll
        for (int k = 0; k < kRPItems; ++k) v[k] = (uint64_t)(rbase + k * kWave + lane);
      } else {
        const uint8_t *ibase = in + (tile + wrow) * (int64_t)w;  // wave-uniform
#pragma unroll
        for (int k = 0; k < kRPItems; ++k) v[k] = (k * kWave + lane < lim) ? ldw<W8>(ibase, k * kWave + lane, w) : 0ull;
      }
      const uint64_t x = c == 0 ? cols.key_xor : 0ull;
      if (TICKET && c + 1 == cols.n && tx == 0)
        s_next = XT ? xt_claim(lb, xhome, TILE, n) : (int64_t)atomicAdd(lb.ticket, 1u) * TILE;
#pragma unroll
      for (int k = 0; k < kRPItems; ++k)
        if (pl[k] != 0xffffffffu) stw<W8>(st, pl[k], w, v[k] ^ x);
      __syncthreads();
      if (TICKET && c + 1 == cols.n) next = s_next;
#pragma unroll
      for (int q = 0; q < kRPItems; ++q) {
        const int j = tx + q * THREADS;
        if (j < cnt) stw<W8>(out, running[dp[q] >> 16] + (int64_t)(dp[q] & 0xffffu), w, ldw<W8>(st, j, w));
      }
      __syncthreads();
    }
    if (!TICKET)
      for (uint32_t p = tx; p < nbuckets; p += THREADS) running[p] += toff[p + 1] - toff[p];
  }
  if (order_bad) atomicOr(cols.order_bad, 1);
}

struct RPGeometry {
  int64_t nblocks, rows_per_block;
};

// Pass block size.  With LDS-atomic ranking (cheap_rank) one 1024-thread block per CU
// (8192-row tiles, 16-row write runs per bucket) wins for every width: 1B-row union
// 130 -> 118 ms, 250M sort 16.4 -> 14.4 ms, group-by 27.9 -> 27.0 ms
// (profiles/rank_variants_r02.txt).  With the ballot ranking, two 512-thread blocks per CU
// (4096-row tiles) interleave one block's ranking with the other's memory traffic, which
// pays for 1-2 column passes (2B sort 137 -> 120 ms) but not for wide rows
// (profiles/rows_pass_experiments_r02.txt).  CYLON_RP_THREADS=512|1024 forces one.
static int rp_threads(int ncols, bool cheap_rank) {
  static const int forced = [] {
    const char *e = std::getenv("CYLON_RP_THREADS");
    const int t = e ? std::atoi(e) : 0;
    return t == 512 || t == 1024 ? t : 0;
  }();
  return forced ? forced : (ncols <= 2 && !cheap_rank ? 512 : 1024);
}

// Self-check of kRankWaveAtomic's precondition: every lane of a wave adds 1 to a
// pseudo-random packed 16-bit counter of the wave's own row (bucket ranges of 2 ... 1024,
// so many lanes share an address or a word) and compares the returned count with the
// stable rank from ballots (count before + #lower lanes in the same bucket).  gfx950
// returns same-address LDS atomics of one instruction in lane order: 0 violations in
// 4.3e10 lane-ops (tools/lds_atomic_order.hip, profiles/rank_variants_r02.txt).
// The probe runs the shapes the ranking code launches: 1024-thread blocks with packed 16-bit
// counters (k_rows_pass, k_rows_pass_lean) and 256-thread blocks with 32-bit counters
// (stable_rank.hpp k_stable_rank).
template <int THREADS, bool PACKED16>
__global__ __launch_bounds__(THREADS) void k_lane_order_check(int rounds, unsigned long long *bad) {
  constexpr int WORDS = PACKED16 ? kRPMaxBuckets / 2 : kRPMaxBuckets;
  __shared__ uint32_t cnt[(THREADS / kWave) * WORDS];
  const int wave = threadIdx.x / kWave, lane = lane_id();
  const uint64_t lt = lanemask_lt();
  uint32_t *mine = cnt + wave * WORDS;
  unsigned long long nbad = 0;
  constexpr int RESTART = PACKED16 ? 256 : 1 << 20;  // 16-bit halves: restart every 256 rounds
  for (int r0 = 0; r0 < rounds; r0 += RESTART) {
    for (int q = lane; q < WORDS; q += kWave) mine[q] = 0;
    __builtin_amdgcn_wave_barrier();
    for (int r = r0; r < r0 + RESTART && r < rounds; ++r) {
      const int nbits = 1 + (r % 10);
      const uint32_t b = (uint32_t)hashing::fmix64(((uint64_t)blockIdx.x << 40) ^ ((uint64_t)r << 12) ^ threadIdx.x) &
                         ((1u << nbits) - 1u);
      uint64_t m = ~0ull;
      for (int bit = 0; bit < nbits; ++bit) {
        const uint32_t x = (b >> bit) & 1u;
        const uint64_t bb = __ballot(x);
        m &= x ? bb : ~bb;
      }
      uint32_t before, got;
      if (PACKED16) {
        const uint32_t sh = (b & 1u) * 16u;
        before = (mine[b >> 1] >> sh) & 0xffffu;
        __builtin_amdgcn_wave_barrier();
        got = (atomicAdd(&mine[b >> 1], 1u << sh) >> sh) & 0xffffu;
      } else {
        before = mine[b];
        __builtin_amdgcn_wave_barrier();
        got = atomicAdd(&mine[b], 1u);
      }
      __builtin_amdgcn_wave_barrier();
      nbad += got != before + (uint32_t)__popcll(m & lt);
    }
  }
  for (int d = kWave / 2; d > 0; d >>= 1) nbad += __shfl_xor(nbad, d, kWave);
  if (lane == 0 && nbad) atomicAdd(bad, nbad);
}

int64_t lds_lane_order_violations(int blocks, int rounds, void *stream) {
  hipStream_t s = as_stream(stream);
  unsigned long long *d = nullptr, h = 0;
  HIP_CHECK(hipMalloc(reinterpret_cast<void **>(&d), sizeof(h)));
  HIP_CHECK(hipMemsetAsync(d, 0, sizeof(h), s));
  hipLaunchKernelGGL((k_lane_order_check<256, true>), dim3((unsigned)blocks), dim3(256), 0, s, rounds, d);
  HIP_LAUNCH_CHECK();
  hipLaunchKernelGGL((k_lane_order_check<1024, true>), dim3((unsigned)blocks), dim3(1024), 0, s, rounds / 4, d);
  HIP_LAUNCH_CHECK();
  hipLaunchKernelGGL((k_lane_order_check<256, false>), dim3((unsigned)blocks), dim3(256), 0, s, rounds, d);
  HIP_LAUNCH_CHECK();
  HIP_CHECK(hipMemcpyAsync(&h, d, sizeof(h), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  HIP_CHECK(hipFree(d));
  return (int64_t)h;
}

// Stable ranking method per device: wave-atomic when the device passed the lane-order
// self-check (run once per device, at context creation -- CylonContext::Init calls
// lds_lane_order_ok -- not inside a pass), else ballots.  A stability violation seen by a
// pass's ranking guard (rp_take_order_violation) switches the device to ballots for the rest
// of the process.  CYLON_RP_RANK=wave|ballot forces one.
static std::atomic<int> g_lane_ok[64];  // 0 unknown, 1 ok, 2 not ok

static int current_device() {
  int d = 0;
  HIP_CHECK(hipGetDevice(&d));
  return d & 63;
}

bool lds_lane_order_ok(void *stream) {
  static const int forced = [] {
    const char *e = std::getenv("CYLON_RP_RANK");
    if (!e) return -1;
    return std::string(e) == "wave" ? 1 : (std::string(e) == "ballot" ? 0 : -1);
  }();
  if (forced >= 0) return forced == 1;
  std::atomic<int> &st = g_lane_ok[current_device()];
  int v = st.load();
  if (v == 0) {
    v = lds_lane_order_violations(64, 1024, stream) == 0 ? 1 : 2;
    int expect = 0;
    st.compare_exchange_strong(expect, v);
    v = st.load();
  }
  return v == 1;
}

// per-device flag the passes' ranking guard raises (allocated once per device)
static int *order_flag() {
  static std::atomic<int *> flags[64];
  const int d = current_device();
  int *f = flags[d].load();
  if (!f) {
    HIP_CHECK(hipMalloc(reinterpret_cast<void **>(&f), sizeof(int)));
    HIP_CHECK(hipMemset(f, 0, sizeof(int)));
    int *expect = nullptr;
    if (!flags[d].compare_exchange_strong(expect, f)) {
      HIP_CHECK(hipFree(f));
      f = expect;
    }
  }
  return f;
}

void rp_reset_lane_order() {  // forget every device's ranking verdict (tests): re-probe on next use
  for (auto &v : g_lane_ok) v.store(0);
}

bool rp_take_order_violation(void *stream) {
  hipStream_t s = as_stream(stream);
  int h = 0;
  int *f = order_flag();
  HIP_CHECK(hipMemcpyAsync(&h, f, sizeof(int), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  if (h) {
    HIP_CHECK(hipMemsetAsync(f, 0, sizeof(int), s));
    g_lane_ok[current_device()].store(2);  // stable passes rank with ballots from now on
  }
  return h != 0;
}
static bool rp_wave_atomic(hipStream_t s) { return lds_lane_order_ok(reinterpret_cast<void *>(s)); }

// Pass kernel: "lean" (two register-lean blocks per CU) or "classic" (one block per CU with
// register software pipelining).  Measured on one box, same tree (profiles/r03/lean_pass_ab.txt):
// lean wins for passes that move 1-2 columns (2B-row sort 107.5 -> 99.2 ms, 1B group-by 27.6 ->
// 25.0 ms; its two blocks overlap each other's ranking and barriers) and loses for the 4-column
// join passes (17.9 -> 20.0 ms per pass: without the classic kernel's next-column prefetch each
// column's load latency is exposed).  CYLON_RP_KERNEL=lean|classic forces one (read per launch).
static bool rp_lean(int ncols) {
  const char *e = std::getenv("CYLON_RP_KERNEL");
  if (e && std::string(e) == "lean") return true;
  if (e && std::string(e) == "classic") return false;
  return ncols <= 2;
}

// resident: blocks per CU that run at once (lean pass: 2 x 1024 threads)
static RPGeometry rp_geometry(int64_t n, int threads, int resident = 1) {
  const int64_t tile = (int64_t)threads * kRPItems;
  const int64_t tiles = std::max<int64_t>(1, (n + tile - 1) / tile);
  const int64_t want = 2 * kNumCUs * (1024 / threads) * resident;  // two rounds of resident blocks
  const int64_t nb = tiles < want ? tiles : want;
  RPGeometry g;
  g.rows_per_block = ((tiles + nb - 1) / nb) * tile;
  g.nblocks = std::max<int64_t>(1, (n + g.rows_per_block - 1) / g.rows_per_block);
  return g;
}

// XCD-tile mode (k_rows_pass / k_rows_pass_lean XT), default on: 1B x 1B join 116-121 -> 102-103 ms,
// passes 21 -> 15.5 ms, pass HBM traffic back to the column bytes (profiles/r03/xcd_tiles_ab.txt).
// CYLON_RP_XT=0 returns to per-block contiguous chunks (read per call).
static bool rp_xt() {
  const char *e = std::getenv("CYLON_RP_XT");
  return !(e && e[0] == '0');
}

struct XtLayout {  // int64-word offsets of the XT buffers in a pass workspace
  int64_t ntiles, nchunks, th, off, csum, cpre, bbase, tickets, words;
};
static XtLayout xt_layout(int64_t n, uint32_t nb) {
  XtLayout l;
  l.ntiles = std::max<int64_t>(1, (n + kRPTile - 1) / kRPTile);
  l.nchunks = (l.ntiles + kTsChunk - 1) / kTsChunk;
  const int64_t cells = l.ntiles * nb, ccells = l.nchunks * nb;
  l.th = 0;                                   // uint16 [ntiles][nb]
  l.off = l.th + (cells * 2 + 7) / 8;         // uint32 [ntiles][nb]
  l.csum = l.off + (cells * 4 + 7) / 8;       // uint32 [nchunks][nb]
  l.cpre = l.csum + (ccells * 4 + 7) / 8;     // uint32 [nchunks][nb]
  l.bbase = l.cpre + (ccells * 4 + 7) / 8;    // uint32 [nb]
  l.tickets = l.bbase + (nb * 4 + 7) / 8;     // uint32 [kXcds]
  l.words = l.tickets + kXcds;
  return l;
}

int64_t radix_rows_pass_workspace(int64_t n, int digit_bits) {  // covers both block sizes and the lean pass
  int64_t ws = rp_xt() ? xt_layout(n, 1u << digit_bits).words : 0;
  for (int threads : {512, 1024, 2048}) {
    const int64_t m = (threads == 2048 ? rp_geometry(n, 1024, 2) : rp_geometry(n, threads)).nblocks *
                      (int64_t(1) << digit_bits);
    ws = std::max(ws, m + (m + 1) + scan_workspace(m));
  }
  return ws;
}

// Column-1 LDS-DMA of the one-block-per-CU pass (k_rows_pass DMA1): 8-byte columns, >= 2 of them,
// column 1 read from memory.  Opt-in (CYLON_RP_DMA=1, read per launch): measured SLOWER on the
// 1B x 1B join (profiles/r03/lds_dma_ab.txt: tile 82-86K -> 88-103K cycles).  hipcc's own
// s_waitcnt vmcnt(0) before the kernel's register-spill reloads in the slot phase (it cannot count
// the asm DMA) and the DMA issue behind the previous tile's outstanding scatter stores put the
// transfer back on the critical path: the keys phase grows 1.4K -> 10K cycles, the slot phase
// 2K -> 7K, while column 0's scatter shrinks only 16K -> 8-9K.
static bool rp_dma1(bool w8, const ColSet &cs) {
  const char *e = std::getenv("CYLON_RP_DMA");
  return w8 && cs.n >= 2 && cs.in[1] != nullptr && e && e[0] == '1';
}

template <class Digit, int THREADS, int RANK, bool LB = false>
static void rows_pass_kernel(bool w8, const RPGeometry &g, hipStream_t s, const Digit &dg, int digit_bits, uint32_t nb,
                             const ColSet &cs, int64_t n, const int64_t *bh_scan, const Lookback &lb = Lookback{},
                             bool xt = false) {
  static const bool stamp = std::getenv("CYLON_RP_STAMPS") != nullptr;  // debug: phase stamps to stderr
  unsigned long long *st = nullptr;
  if (stamp && !LB) {
    HIP_CHECK(hipStreamSynchronize(s));
    HIP_CHECK(hipMalloc(&st, sizeof(unsigned long long) * kRPStampTiles * kRPStampSlots));
    HIP_CHECK(hipMemset(st, 0, sizeof(unsigned long long) * kRPStampTiles * kRPStampSlots));
  }
  bool launched = false;
  if constexpr (THREADS == 1024 && !LB) {
    if (xt) {
      if (w8)
        hipLaunchKernelGGL((k_rows_pass<Digit, true, THREADS, RANK, false, false, true>), dim3((unsigned)g.nblocks),
                           dim3(THREADS), 0, s, dg, digit_bits, nb, cs, n, g.rows_per_block, g.nblocks, bh_scan, lb, st);
      else
        hipLaunchKernelGGL((k_rows_pass<Digit, false, THREADS, RANK, false, false, true>), dim3((unsigned)g.nblocks),
                           dim3(THREADS), 0, s, dg, digit_bits, nb, cs, n, g.rows_per_block, g.nblocks, bh_scan, lb, st);
      launched = true;
    } else if (rp_dma1(w8, cs)) {
      hipLaunchKernelGGL((k_rows_pass<Digit, true, THREADS, RANK, LB, true>), dim3((unsigned)g.nblocks), dim3(THREADS),
                         0, s, dg, digit_bits, nb, cs, n, g.rows_per_block, g.nblocks, bh_scan, lb, st);
      launched = true;
    }
  }
  if (launched) {
  } else if (w8)
    hipLaunchKernelGGL((k_rows_pass<Digit, true, THREADS, RANK, LB>), dim3((unsigned)g.nblocks), dim3(THREADS), 0, s,
                       dg, digit_bits, nb, cs, n, g.rows_per_block, g.nblocks, bh_scan, lb, st);
  else
    hipLaunchKernelGGL((k_rows_pass<Digit, false, THREADS, RANK, LB>), dim3((unsigned)g.nblocks), dim3(THREADS), 0,
                       s, dg, digit_bits, nb, cs, n, g.rows_per_block, g.nblocks, bh_scan, lb, st);
  if (st) {
    HIP_CHECK(hipStreamSynchronize(s));
    std::vector<unsigned long long> h(kRPStampTiles * kRPStampSlots);
    HIP_CHECK(hipMemcpy(h.data(), st, h.size() * sizeof(h[0]), hipMemcpyDeviceToHost));
    HIP_CHECK(hipFree(st));
    // mean cycles of each phase over the full tiles after the first (tile i: slot j - slot j-1,
    // slot 0 of tile i+1 closes the last column)
    const int last = 7 + 2 * (cs.n - 1);
    double sum[kRPStampSlots] = {0};
    int tiles = 0;
    for (int t = 1; t + 1 < kRPStampTiles; ++t) {
      if (h[(t + 1) * kRPStampSlots] == 0) break;
      for (int j = 1; j <= last && j < kRPStampSlots; ++j)
        sum[j] += (double)(h[t * kRPStampSlots + j] - h[t * kRPStampSlots + j - 1]);
      sum[0] += (double)(h[(t + 1) * kRPStampSlots] - h[t * kRPStampSlots]);
      ++tiles;
    }
    if (tiles > 0) {
      std::fprintf(stderr, "rp_stamps threads=%d stable=%d ncols=%d bits=%d tiles=%d tile_total=%.0f |", THREADS,
                   RANK, cs.n, digit_bits, tiles, sum[0] / tiles);
      static const char *names[] = {"", "keys", "rank", "scan", "slot", "dst"};
      for (int j = 1; j <= last && j < kRPStampSlots; ++j) {
        if (j <= 5) std::fprintf(stderr, " %s=%.0f", names[j], sum[j] / tiles);
        else std::fprintf(stderr, " c%d_%s=%.0f", (j - 6) / 2, (j % 2 == 0) ? "stage" : "scatter", sum[j] / tiles);
      }
      std::fprintf(stderr, "\n");
    }
  }
}

template <class Digit, int RANK, bool LB>
static void lean_kernel(bool w8, const RPGeometry &g, hipStream_t s, const Digit &dg, int digit_bits, uint32_t nb,
                        const ColSet &cs, int64_t n, const int64_t *bh_scan, const Lookback &lb, bool xt = false) {
  if constexpr (!LB) {
    if (xt) {
      if (w8)
        hipLaunchKernelGGL((k_rows_pass_lean<Digit, true, RANK, false, true>), dim3((unsigned)g.nblocks),
                           dim3(kRPThreads), 0, s, dg, digit_bits, nb, cs, n, g.rows_per_block, g.nblocks, bh_scan, lb);
      else
        hipLaunchKernelGGL((k_rows_pass_lean<Digit, false, RANK, false, true>), dim3((unsigned)g.nblocks),
                           dim3(kRPThreads), 0, s, dg, digit_bits, nb, cs, n, g.rows_per_block, g.nblocks, bh_scan, lb);
      return;
    }
  }
  if (w8)
    hipLaunchKernelGGL((k_rows_pass_lean<Digit, true, RANK, LB>), dim3((unsigned)g.nblocks), dim3(kRPThreads), 0, s,
                       dg, digit_bits, nb, cs, n, g.rows_per_block, g.nblocks, bh_scan, lb);
  else
    hipLaunchKernelGGL((k_rows_pass_lean<Digit, false, RANK, LB>), dim3((unsigned)g.nblocks), dim3(kRPThreads), 0, s,
                       dg, digit_bits, nb, cs, n, g.rows_per_block, g.nblocks, bh_scan, lb);
}

// ---- lookback session workspace (int64 words):
//   [hist u64: kLbMaxPasses x kRPMaxBuckets][gstart: same][tickets: kLbMaxPasses u32 (4 words)][status: tiles x 2^maxbits]
constexpr int64_t kLbHistWords = (int64_t)kLbMaxPasses * kRPMaxBuckets;
static int64_t lb_tiles(int64_t n) { return std::max<int64_t>(1, (n + kRPTile - 1) / kRPTile); }

// Off by default: measured slower on MI355X (profiles/r03/lookback_ab.txt: 2B sort 99.3 -> 110.1 ms,
// headline join 110.8 -> 118.6 ms).  Tiles claimed by ticket land in row order on whichever XCD
// is free, so consecutive tiles' partial 128-B runs of one bucket are written from different
// L2s instead of merging in one (the per-block chunks of histogram mode keep a bucket's
// consecutive runs in one block, one L2), and every tile waits on agent-scope status words.
// CYLON_RP_LOOKBACK=1 enables it.
bool radix_lookback_enabled() {
  const char *e = std::getenv("CYLON_RP_LOOKBACK");
  return e && e[0] == '1';
}

int64_t radix_lb_workspace(int64_t n, int max_digit_bits) {
  return 2 * kLbHistWords + kLbMaxPasses / 2 + lb_tiles(n) * (int64_t(1) << max_digit_bits);
}

template <class Digit>
static void lb_prepare(const DigitSet<Digit> &ds, int64_t n, int max_digit_bits, int64_t *lbws, hipStream_t s) {
  CYLON_CHECK(ds.n >= 1 && ds.n <= kLbMaxPasses, Code::Invalid, "lookback passes " << ds.n);
  CYLON_CHECK(max_digit_bits >= 1 && max_digit_bits <= kRJMaxDigitBits, Code::Invalid, "digit bits " << max_digit_bits);
  const uint32_t nb = 1u << max_digit_bits;
  // histograms, tickets and status words start at zero (epoch 0 is never a pass's tag)
  HIP_CHECK(hipMemsetAsync(lbws, 0, sizeof(int64_t) * radix_lb_workspace(n, max_digit_bits), s));
  if (n > 0) {
    hipLaunchKernelGGL(k_lb_hist<Digit>, dim3(grid_for(n, kRPThreads * 8, kNumCUs * 2)), dim3(kRPThreads), 0, s, ds, n,
                       nb, reinterpret_cast<unsigned long long *>(lbws));
    HIP_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(k_lb_scan, dim3(ds.n), dim3(kRPThreads), 0, s, reinterpret_cast<unsigned long long *>(lbws), nb,
                     lbws + kLbHistWords);
  HIP_LAUNCH_CHECK();
}

// Every pass of one session uses the same bucket count (2^max_digit_bits histogram rows; a pass
// with fewer digit bits leaves the upper rows empty).
void radix_lb_prepare_part(const int64_t *keys, int64_t n, int total_bits, const int *shifts, const int *dbits,
                           int npass, int max_digit_bits, int64_t *lbws, void *stream) {
  DigitSet<PartDigit> ds{};
  ds.n = npass;
  for (int s = 0; s < npass; ++s) ds.d[s] = PartDigit{keys, total_bits, shifts[s], (1u << dbits[s]) - 1};
  lb_prepare(ds, n, max_digit_bits, lbws, as_stream(stream));
}

void radix_lb_prepare_sort(const int64_t *keys, int64_t n, uint64_t flip, const int *shifts, const int *dbits,
                           int npass, int max_digit_bits, int64_t *lbws, void *stream) {
  DigitSet<ImageDigit> ds{};
  ds.n = npass;
  for (int s = 0; s < npass; ++s) ds.d[s] = ImageDigit{keys, shifts[s], (1u << dbits[s]) - 1, flip};
  lb_prepare(ds, n, max_digit_bits, lbws, as_stream(stream));
}

void radix_lb_prepare_range(const int64_t *keys, int64_t n, uint64_t flip, uint64_t mn, int rshift, const int *shifts,
                            const int *dbits, int npass, int max_digit_bits, int64_t *lbws, void *stream) {
  DigitSet<RangeDigit> ds{};
  ds.n = npass;
  for (int s = 0; s < npass; ++s) ds.d[s] = RangeDigit{keys, flip, mn, rshift, shifts[s], (1u << dbits[s]) - 1};
  lb_prepare(ds, n, max_digit_bits, lbws, as_stream(stream));
}

// pass `pass` of a lookback session: its gstart row, ticket and epoch
static Lookback lb_args(int64_t *lbws, int pass, int max_digit_bits) {
  Lookback lb;
  lb.gstart = lbws + kLbHistWords + (int64_t)pass * (int64_t(1) << max_digit_bits);
  lb.ticket = reinterpret_cast<unsigned int *>(lbws + 2 * kLbHistWords) + pass;
  lb.status = reinterpret_cast<unsigned long long *>(lbws + 2 * kLbHistWords + kLbMaxPasses / 2);
  lb.epoch = (unsigned long long)(pass + 1);
  return lb;
}

// stable = false (join partitions only) ranks rows with LDS atomics: rows of one
// bucket keep no particular order inside a tile's run.  Instantiated for PartDigit
// only; every other digit (sort, shuffle, range join) needs the stable order.
// lbws != nullptr: lookback mode, pass `lb_pass` of the session radix_lb_prepare_* set up with
// `lb_bits` histogram bits (digit_bits <= lb_bits); ws is not used.
template <class Digit, bool CAN_UNSTABLE = std::is_same<Digit, PartDigit>::value>
static void rows_pass_launch(const Digit &dg, int64_t n, int digit_bits, const uint8_t *const *in, uint8_t *const *out,
                             const int *widths, int ncols, int64_t *ws, void *stream, uint64_t key_xor = 0,
                             bool stable = true, int64_t *lbws = nullptr, int lb_pass = 0, int lb_bits = 0,
                             bool tiles_prescanned = false) {
  if (n == 0) return;
  CYLON_CHECK(digit_bits >= 1 && digit_bits <= kRJMaxDigitBits, Code::Invalid, "digit bits " << digit_bits);
  CYLON_CHECK(ncols >= 1 && ncols <= kMaxFusedCols, Code::Invalid, "bad column count " << ncols);
  CYLON_CHECK(in[0] == reinterpret_cast<const uint8_t *>(dg.keys) && widths[0] == 8, Code::Invalid,
              "radix pass: column 0 must be the key");
  static_assert(!Digit::kNarrow, "narrow-key passes launch through narrow_pass_launch");
  // key_xor rebuilds int64 keys from order images: only a sort's image digit may set it
  // (partition / mod / range digits store column 0 as read)
  CYLON_CHECK((key_xor == 0 || std::is_same<Digit, ImageDigit>::value), Code::Invalid,
              "radix pass: key_xor is only valid for order-image digits");
  const bool lbm = lbws != nullptr;
  CYLON_CHECK(!lbm || (lb_pass >= 0 && lb_pass < kLbMaxPasses && digit_bits <= lb_bits), Code::Invalid,
              "radix pass: bad lookback pass " << lb_pass);
  hipStream_t s = as_stream(stream);
  const uint32_t nb = 1u << digit_bits;
  CYLON_CHECK(stable || CAN_UNSTABLE, Code::Invalid, "radix pass: only partition digits may rank unstably");
  // test knob: every partition pass ranks unstably, so LSD passes after the first scramble the
  // order they received -- rows end in wrong partitions and the join's ranking guard must fire
  const bool want_stable = stable;  // the ranking guard checks what the caller asked for
  const char *dbg = std::getenv("CYLON_RP_DEBUG_UNSTABLE");
  if (CAN_UNSTABLE && dbg && dbg[0] == '1') stable = false;
  const bool unstable = CAN_UNSTABLE && !stable;
  const bool wave_atomic = !unstable && rp_wave_atomic(s);
  // lookback tiles are 8192 rows: 1024-thread kernels only
  const int threads = lbm ? 1024 : rp_threads(ncols, unstable || wave_atomic);
  const bool lean = rp_lean(ncols) && (unstable || wave_atomic) && threads == 1024;
  RPGeometry g;
  const int64_t *bh_scan = nullptr;
  Lookback lb{};
  const bool xt = !lbm && threads == 1024 && n < (int64_t(1) << 32) && rp_xt();
  if (!xt) tiles_prescanned = false;  // histogram mode counts its own blocks (the prescan is unused)
  if (xt) {  // exact per-tile offsets, tiles claimed in order per XCD (see xt_claim)
    const XtLayout L = xt_layout(n, nb);
    uint16_t *th = reinterpret_cast<uint16_t *>(ws + L.th);
    uint32_t *off = reinterpret_cast<uint32_t *>(ws + L.off);
    uint32_t *csum = reinterpret_cast<uint32_t *>(ws + L.csum), *cpre = reinterpret_cast<uint32_t *>(ws + L.cpre);
    unsigned *tk = reinterpret_cast<unsigned *>(ws + L.tickets);
    HIP_CHECK(hipMemsetAsync(tk, 0, kXcds * sizeof(unsigned), s));
    if (!tiles_prescanned) {  // else the caller already wrote th (radix_sort_prehist + fold)
      hipLaunchKernelGGL(k_rp_hist_tiles<Digit>, dim3((unsigned)std::min<int64_t>(L.ntiles, kNumCUs * 16)),
                         dim3(kHTThreads), 0, s, dg, n, nb, L.ntiles, th);
      HIP_LAUNCH_CHECK();
    }
    const unsigned bt = (unsigned)std::max<uint32_t>(kWave, (nb + kWave - 1) / kWave * kWave);
    hipLaunchKernelGGL(k_ts_chunk_sums, dim3((unsigned)L.nchunks), dim3(bt), 0, s, th, nb, L.ntiles, csum);
    HIP_LAUNCH_CHECK();
    uint32_t *bbase = reinterpret_cast<uint32_t *>(ws + L.bbase);
    hipLaunchKernelGGL(k_ts_chunk_prefix, dim3(1), dim3(kRPThreads), 0, s, csum, nb, L.nchunks, cpre, bbase);
    HIP_LAUNCH_CHECK();
    hipLaunchKernelGGL(k_ts_offsets, dim3((unsigned)L.nchunks), dim3(bt), 0, s, th, cpre, bbase, nb, L.ntiles, off);
    HIP_LAUNCH_CHECK();
    lb.xt_off = off;
    lb.xt_ticket = tk;
    lb.xt_tiles = L.ntiles;
    g.rows_per_block = kRPTile;
    g.nblocks = std::min<int64_t>(L.ntiles, (int64_t)kNumCUs * (lean ? 2 : 1));  // persistent: all resident
  } else if (lbm) {
    // status rows are 2^lb_bits wide; a pass with fewer bits indexes them with its own nb
    lb = lb_args(lbws, lb_pass, lb_bits);
    g.rows_per_block = kRPTile;
    g.nblocks = std::min<int64_t>(lb_tiles(n), (int64_t)kNumCUs * (lean ? 2 : 1));  // persistent, tiles by ticket
  } else {
    g = rp_geometry(n, threads, lean ? 2 : 1);
    const int64_t m = g.nblocks * (int64_t)nb;
    int64_t *bh = ws;
    int64_t *scan_out = ws + m, *scan_ws = scan_out + m + 1;
    hipLaunchKernelGGL(k_rp_hist<Digit>, dim3((unsigned)g.nblocks), dim3(kRPThreads), 0, s, dg, n, nb,
                       g.rows_per_block, g.nblocks, bh);
    HIP_LAUNCH_CHECK();
    exclusive_scan(bh, m, scan_out, scan_ws, stream);
    bh_scan = scan_out;
  }
  ColSet cs;
  cs.n = ncols;
  cs.key_xor = key_xor;
  const char *gd = std::getenv("CYLON_RP_GUARD");  // A/B knob: 0 disables the ranking guard
  cs.check_order = want_stable && !(gd && gd[0] == '0') ? 1 : 0;
  cs.order_bad = order_flag();
  for (int c = 0; c < kMaxFusedCols; ++c) {
    cs.in[c] = c < ncols ? in[c] : nullptr;
    cs.out[c] = c < ncols ? out[c] : nullptr;
    cs.width[c] = c < ncols ? widths[c] : 8;
  }
  bool w8 = true;
  for (int c = 0; c < ncols; ++c) {
    w8 &= widths[c] == 8;
    CYLON_CHECK(in[c] != nullptr || (c > 0 && widths[c] == 8), Code::Invalid,
                "radix pass: a generated row-id column must be an 8-byte payload column");
  }
  const bool big = threads == 1024;
  if (lean) {
    constexpr int R = CAN_UNSTABLE ? kRankBlockAtomic : kRankWaveAtomic;
    if (lbm) {
      if (unstable) lean_kernel<Digit, R, true>(w8, g, s, dg, digit_bits, nb, cs, n, bh_scan, lb);
      else lean_kernel<Digit, kRankWaveAtomic, true>(w8, g, s, dg, digit_bits, nb, cs, n, bh_scan, lb);
    } else {
      if (unstable) lean_kernel<Digit, R, false>(w8, g, s, dg, digit_bits, nb, cs, n, bh_scan, lb, xt);
      else lean_kernel<Digit, kRankWaveAtomic, false>(w8, g, s, dg, digit_bits, nb, cs, n, bh_scan, lb, xt);
    }
    HIP_LAUNCH_CHECK();
    return;
  }
  if (lbm) {
    constexpr int R = CAN_UNSTABLE ? kRankBlockAtomic : kRankBallot;
    if (unstable) rows_pass_kernel<Digit, 1024, R, true>(w8, g, s, dg, digit_bits, nb, cs, n, bh_scan, lb);
    else if (wave_atomic) rows_pass_kernel<Digit, 1024, kRankWaveAtomic, true>(w8, g, s, dg, digit_bits, nb, cs, n, bh_scan, lb);
    else rows_pass_kernel<Digit, 1024, kRankBallot, true>(w8, g, s, dg, digit_bits, nb, cs, n, bh_scan, lb);
  } else if (unstable) {
    constexpr int R = CAN_UNSTABLE ? kRankBlockAtomic : kRankBallot;
    if (big) rows_pass_kernel<Digit, 1024, R>(w8, g, s, dg, digit_bits, nb, cs, n, bh_scan, lb, xt);
    else rows_pass_kernel<Digit, 512, R>(w8, g, s, dg, digit_bits, nb, cs, n, bh_scan);
  } else if (wave_atomic) {
    if (big) rows_pass_kernel<Digit, 1024, kRankWaveAtomic>(w8, g, s, dg, digit_bits, nb, cs, n, bh_scan, lb, xt);
    else rows_pass_kernel<Digit, 512, kRankWaveAtomic>(w8, g, s, dg, digit_bits, nb, cs, n, bh_scan);
  } else {
    if (big) rows_pass_kernel<Digit, 1024, kRankBallot>(w8, g, s, dg, digit_bits, nb, cs, n, bh_scan, lb, xt);
    else rows_pass_kernel<Digit, 512, kRankBallot>(w8, g, s, dg, digit_bits, nb, cs, n, bh_scan);
  }
  HIP_LAUNCH_CHECK();
}

void radix_rows_pass(const int64_t *keys, int64_t n, int total_bits, int shift, int digit_bits, const uint8_t *const *in,
                     uint8_t *const *out, const int *widths, int ncols, int64_t *ws, void *stream, bool stable,
                     int64_t *lbws, int lb_pass, int lb_bits) {
  const uint32_t nb = 1u << digit_bits;
  rows_pass_launch(PartDigit{keys, total_bits, shift, nb - 1}, n, digit_bits, in, out, widths, ncols, ws, stream, 0,
                   stable, lbws, lb_pass, lb_bits);
}

// ---- narrow-key join passes: the one-block-per-CU kernel (8192-row tiles, next-column prefetch)
// for every column count; the first pass (int64 keys in, block-atomic ranking) may take its
// scanned histogram from radix_narrow_prehist, later passes (uint32 keys) rank stably.
static RPGeometry narrow_geometry(int64_t n) { return rp_geometry(n, 1024, 1); }

void radix_narrow_prehist(const int64_t *keys, int64_t n, int total_bits, int digit_bits, int64_t *ws, int64_t *mm,
                          void *stream) {
  CYLON_CHECK(digit_bits >= 1 && digit_bits <= kRJMaxDigitBits, Code::Invalid, "digit bits " << digit_bits);
  hipStream_t s = as_stream(stream);
  if (n == 0) return;
  const RPGeometry g = narrow_geometry(n);
  const uint32_t nb = 1u << digit_bits;
  const int64_t m = g.nblocks * (int64_t)nb;
  hipLaunchKernelGGL(k_rp_hist_minmax, dim3((unsigned)g.nblocks), dim3(kRPThreads), 0, s,
                     PartDigitN64{keys, total_bits, 0, nb - 1}, n, nb, g.rows_per_block, g.nblocks, ws,
                     reinterpret_cast<long long *>(mm));
  HIP_LAUNCH_CHECK();
  exclusive_scan(ws, m, ws + m, ws + 2 * m + 1, stream);
}

template <class Digit>
static void narrow_pass_launch(const Digit &dg, int64_t n, int digit_bits, const uint8_t *const *in,
                               uint8_t *const *out, const int *widths, int ncols, int64_t *ws, hipStream_t s,
                               bool stable, bool prescanned) {
  static_assert(Digit::kNarrow, "narrow digits only");
  if (n == 0) return;
  CYLON_CHECK(digit_bits >= 1 && digit_bits <= kRJMaxDigitBits, Code::Invalid, "digit bits " << digit_bits);
  CYLON_CHECK(ncols >= 1 && ncols <= kMaxFusedCols, Code::Invalid, "bad column count " << ncols);
  CYLON_CHECK(in[0] == reinterpret_cast<const uint8_t *>(dg.keys) && widths[0] == 4, Code::Invalid,
              "narrow radix pass: column 0 must be the key, stored as uint32");
  const bool want_stable = stable;
  const char *dbg = std::getenv("CYLON_RP_DEBUG_UNSTABLE");  // ranking-guard test knob (rows_pass_launch)
  if (dbg && dbg[0] == '1') stable = false;
  const RPGeometry g = narrow_geometry(n);
  const uint32_t nb = 1u << digit_bits;
  const int64_t m = g.nblocks * (int64_t)nb;
  if (!prescanned) {
    hipLaunchKernelGGL(k_rp_hist<Digit>, dim3((unsigned)g.nblocks), dim3(kRPThreads), 0, s, dg, n, nb,
                       g.rows_per_block, g.nblocks, ws);
    HIP_LAUNCH_CHECK();
    exclusive_scan(ws, m, ws + m, ws + 2 * m + 1, reinterpret_cast<void *>(s));
  }
  ColSet cs;
  cs.n = ncols;
  cs.key_xor = 0;
  const char *gd = std::getenv("CYLON_RP_GUARD");
  cs.check_order = want_stable && !(gd && gd[0] == '0') ? 1 : 0;
  cs.order_bad = order_flag();
  bool w8 = true;
  for (int c = 0; c < kMaxFusedCols; ++c) {
    cs.in[c] = c < ncols ? in[c] : nullptr;
    cs.out[c] = c < ncols ? out[c] : nullptr;
    cs.width[c] = c < ncols ? widths[c] : 8;
    if (c > 0 && c < ncols) {
      w8 &= widths[c] == 8;
      CYLON_CHECK(in[c] != nullptr, Code::Invalid, "narrow radix pass: no generated columns");
    }
  }
  if (!stable) rows_pass_kernel<Digit, 1024, kRankBlockAtomic>(w8, g, s, dg, digit_bits, nb, cs, n, ws + m);
  else if (rp_wave_atomic(s)) rows_pass_kernel<Digit, 1024, kRankWaveAtomic>(w8, g, s, dg, digit_bits, nb, cs, n, ws + m);
  else rows_pass_kernel<Digit, 1024, kRankBallot>(w8, g, s, dg, digit_bits, nb, cs, n, ws + m);
  HIP_LAUNCH_CHECK();
}

void radix_narrow_rows_pass(const void *keys, int key_bytes, int64_t n, int total_bits, int shift, int digit_bits,
                            const uint8_t *const *in, uint8_t *const *out, const int *widths, int ncols, int64_t *ws,
                            void *stream, bool stable, bool prescanned) {
  CYLON_CHECK(key_bytes == 8 || key_bytes == 4, Code::Invalid, "narrow radix pass: key bytes " << key_bytes);
  const uint32_t nb = 1u << digit_bits;
  hipStream_t s = as_stream(stream);
  if (key_bytes == 8)
    narrow_pass_launch(PartDigitN64{reinterpret_cast<const int64_t *>(keys), total_bits, shift, nb - 1}, n, digit_bits,
                       in, out, widths, ncols, ws, s, stable, prescanned);
  else
    narrow_pass_launch(PartDigitN32{reinterpret_cast<const uint32_t *>(keys), total_bits, shift, nb - 1}, n,
                       digit_bits, in, out, widths, ncols, ws, s, stable, prescanned);
}

void radix_sort_rows_pass(const int64_t *keys, int64_t n, int shift, int digit_bits, const uint8_t *const *in,
                          uint8_t *const *out, const int *widths, int ncols, int64_t *ws, void *stream,
                          uint64_t key_xor, uint64_t digit_flip, int64_t *lbws, int lb_pass, int lb_bits,
                          bool tiles_prescanned) {
  const uint32_t nb = 1u << digit_bits;
  rows_pass_launch(ImageDigit{keys, shift, nb - 1, digit_flip}, n, digit_bits, in, out, widths, ncols, ws, stream,
                   key_xor, true, lbws, lb_pass, lb_bits, tiles_prescanned);
}

bool radix_xt_enabled() { return rp_xt(); }

// ---- sort prologue: the keys' varying bits (OR ^ AND) and the first pass's per-tile histogram of
// the order image's low 10 bits in ONE read of the keys (the separate reduction read them once more)
constexpr int kSPBits = 10;
__global__ __launch_bounds__(kHTThreads) void k_sort_prehist(const int64_t *__restrict__ keys, int64_t n,
                                                             uint64_t flip, int64_t ntiles, uint16_t *__restrict__ th,
                                                             unsigned long long *__restrict__ orand) {
  constexpr uint32_t nb = 1u << kSPBits;
  __shared__ unsigned int hist[nb];
  uint64_t o = 0, a = ~0ull;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    uint64_t k[kHTItems];
    const int64_t r0 = t * kRPTile;
#pragma unroll
    for (int u = 0; u < kHTItems; ++u) {
      const int64_t i = r0 + u * kHTThreads + threadIdx.x;
      k[u] = i < n ? (uint64_t)keys[i] : 0ull;
    }
    for (uint32_t p = threadIdx.x; p < nb; p += blockDim.x) hist[p] = 0;
    __syncthreads();
#pragma unroll
    for (int u = 0; u < kHTItems; ++u)
      if (r0 + u * kHTThreads + threadIdx.x < n) {
        o |= k[u];
        a &= k[u];
        atomicAdd(&hist[(uint32_t)((k[u] ^ flip) & (nb - 1))], 1u);
      }
    __syncthreads();
    for (uint32_t p = threadIdx.x; p < nb; p += blockDim.x) th[t * nb + p] = (uint16_t)hist[p];
    __syncthreads();
  }
#pragma unroll
  for (int d = kWave / 2; d > 0; d >>= 1) {
    o |= rj_shfl_xor64((long long)o, d);
    a &= rj_shfl_xor64((long long)a, d);
  }
  if (lane_id() == 0) {
    atomicOr(&orand[0], (unsigned long long)o);
    atomicAnd(&orand[1], (unsigned long long)a);
  }
}

// th[t][d] (2^db buckets) from the 10-bit histogram: digits that agree in their low db bits
__global__ void k_sort_prehist_fold(const uint16_t *__restrict__ th10, int64_t ntiles, int db,
                                    uint16_t *__restrict__ th) {
  const uint32_t nb = 1u << db, groups = 1u << (kSPBits - db);
  const int64_t cells = ntiles * nb, stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < cells; c += stride) {
    const int64_t t = c / nb;
    const uint32_t d = (uint32_t)(c % nb);
    uint32_t sum = 0;
    for (uint32_t g = 0; g < groups; ++g) sum += th10[t * (1 << kSPBits) + d + (g << db)];
    th[c] = (uint16_t)sum;
  }
}

int64_t radix_sort_prehist_workspace(int64_t n) { return xt_layout(n, 1u << kSPBits).words + 2; }

uint64_t radix_sort_prehist(const int64_t *keys, int64_t n, uint64_t flip, int64_t *pre_ws, void *stream) {
  hipStream_t s = as_stream(stream);
  const XtLayout L = xt_layout(n, 1u << kSPBits);
  unsigned long long *orand = reinterpret_cast<unsigned long long *>(pre_ws + L.words);
  const unsigned long long init[2] = {0ull, ~0ull};
  HIP_CHECK(hipMemcpyAsync(orand, init, sizeof(init), hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_sort_prehist, dim3((unsigned)std::min<int64_t>(L.ntiles, kNumCUs * 16)), dim3(kHTThreads), 0,
                     s, keys, n, flip, L.ntiles, reinterpret_cast<uint16_t *>(pre_ws + L.th), orand);
  HIP_LAUNCH_CHECK();
  unsigned long long h[2];
  HIP_CHECK(hipMemcpyAsync(h, orand, sizeof(h), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  return n <= 1 ? 0ull : (uint64_t)(h[0] ^ h[1]);
}

void radix_sort_prehist_fold(const int64_t *pre_ws, int64_t n, int db, int64_t *ws, void *stream) {
  CYLON_CHECK(db >= 1 && db <= kSPBits, Code::Invalid, "sort prehist fold: digit bits " << db);
  const XtLayout P = xt_layout(n, 1u << kSPBits), L = xt_layout(n, 1u << db);
  const uint16_t *th10 = reinterpret_cast<const uint16_t *>(pre_ws + P.th);
  uint16_t *th = reinterpret_cast<uint16_t *>(ws + L.th);
  const int64_t cells = L.ntiles * (int64_t(1) << db);
  hipLaunchKernelGGL(k_sort_prehist_fold, dim3(grid_for(cells)), dim3(kBlock), 0, as_stream(stream), th10, L.ntiles,
                     db, th);
  HIP_LAUNCH_CHECK();
}

void radix_range_rows_pass(const int64_t *keys, int64_t n, uint64_t flip, uint64_t mn, int rshift, int shift,
                           int digit_bits, const uint8_t *const *in, uint8_t *const *out, const int *widths, int ncols,
                           int64_t *ws, void *stream, int64_t *lbws, int lb_pass, int lb_bits) {
  const uint32_t nb = 1u << digit_bits;
  rows_pass_launch(RangeDigit{keys, flip, mn, rshift, shift, nb - 1}, n, digit_bits, in, out, widths, ncols, ws,
                   stream, 0, true, lbws, lb_pass, lb_bits);
}

static int bits_for(uint32_t nparts) {
  int b = 1;
  while ((1u << b) < nparts) ++b;
  return b;
}

int64_t radix_mod_rows_pass_workspace(int64_t n, uint32_t nparts) {
  return radix_rows_pass_workspace(n, bits_for(nparts));
}

void radix_mod_rows_pass(const int64_t *keys, int64_t n, uint32_t nparts, const uint8_t *const *in, uint8_t *const *out,
                         const int *widths, int ncols, int64_t *ws, void *stream) {
  CYLON_CHECK(nparts >= 1 && nparts <= (uint32_t)kRPMaxBuckets, Code::Invalid, "partition count " << nparts);
  rows_pass_launch(ModDigit{keys, nparts}, n, bits_for(nparts), in, out, widths, ncols, ws, stream);
}

__global__ __launch_bounds__(kRPThreads) void k_mod_counts(ModDigit digit, int64_t n,
                                                           unsigned long long *__restrict__ counts) {
  __shared__ unsigned int hist[kRPMaxBuckets];
  for (uint32_t p = threadIdx.x; p < digit.nparts; p += blockDim.x) hist[p] = 0;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) atomicAdd(&hist[digit(i)], 1u);
  __syncthreads();
  for (uint32_t p = threadIdx.x; p < digit.nparts; p += blockDim.x)
    if (hist[p]) atomicAdd(&counts[p], (unsigned long long)hist[p]);
}

void mod_partition_counts(const int64_t *keys, int64_t n, uint32_t nparts, int64_t *counts, void *stream) {
  CYLON_CHECK(nparts >= 1 && nparts <= (uint32_t)kRPMaxBuckets, Code::Invalid, "partition count " << nparts);
  hipStream_t s = as_stream(stream);
  HIP_CHECK(hipMemsetAsync(counts, 0, sizeof(int64_t) * nparts, s));
  if (n == 0) return;
  hipLaunchKernelGGL(k_mod_counts, dim3(grid_for(n, kRPThreads, kNumCUs * 2)), dim3(kRPThreads), 0, s,
                     ModDigit{keys, nparts}, n, reinterpret_cast<unsigned long long *>(counts));
  HIP_LAUNCH_CHECK();
}

// offsets[p] = first row of partition p in partition-sorted keys (binary search), offsets[P] = n
__global__ void k_part_offsets(const int64_t *__restrict__ keys, int64_t n, int bits, int64_t nparts,
                               int64_t *__restrict__ offs) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p <= nparts; p += stride) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if ((int64_t)part_of(keys[mid], bits) < p) lo = mid + 1; else hi = mid;
    }
    offs[p] = lo;
  }
}

void radix_part_offsets(const int64_t *keys, int64_t n, int bits, int64_t *offs, void *stream) {
  const int64_t np = int64_t(1) << bits;
  hipLaunchKernelGGL(k_part_offsets, dim3(grid_for(np + 1)), dim3(kBlock), 0, as_stream(stream), keys, n, bits, np,
                     offs);
  HIP_LAUNCH_CHECK();
}

// same over narrow-key partitions (uint32 keys, partition hash of the low 32 bits)
__global__ void k_part_offsets_u32(const uint32_t *__restrict__ keys, int64_t n, int bits, int64_t nparts,
                                   int64_t *__restrict__ offs) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p <= nparts; p += stride) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if ((int64_t)part_of((int64_t)keys[mid], bits) < p) lo = mid + 1; else hi = mid;
    }
    offs[p] = lo;
  }
}

void radix_narrow_part_offsets(const uint32_t *keys, int64_t n, int bits, int64_t *offs, void *stream) {
  const int64_t np = int64_t(1) << bits;
  hipLaunchKernelGGL(k_part_offsets_u32, dim3(grid_for(np + 1)), dim3(kBlock), 0, as_stream(stream), keys, n, bits,
                     np, offs);
  HIP_LAUNCH_CHECK();
}

__global__ void k_range_part_offsets(const int64_t *__restrict__ keys, int64_t n, uint64_t flip, uint64_t mn,
                                     int rshift, int64_t nparts, int64_t *__restrict__ offs) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p <= nparts; p += stride) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if ((int64_t)((((uint64_t)keys[mid] ^ flip) - mn) >> rshift) < p) lo = mid + 1; else hi = mid;
    }
    offs[p] = lo;
  }
}

void radix_range_part_offsets(const int64_t *keys, int64_t n, uint64_t flip, uint64_t mn, int rshift, int bits,
                              int64_t *offs, void *stream) {
  const int64_t np = int64_t(1) << bits;
  hipLaunchKernelGGL(k_range_part_offsets, dim3(grid_for(np + 1)), dim3(kBlock), 0, as_stream(stream), keys, n, flip,
                     mn, rshift, np, offs);
  HIP_LAUNCH_CHECK();
}

// --------------------------------------------------------------------------
// per-partition LDS join
// --------------------------------------------------------------------------
// The build rows of a partition are indexed by a bucketed (CSR) hash in LDS:
// 2048 buckets by the low bits of fmix64(key) (independent of the partition
// bits, which are the top bits), bucket starts as uint16, the keys stored in
// bucket order and a uint16 permutation back to the staged row.  A probe scans
// exactly its bucket (mean occupancy < 1): no clustering, no tombstones, and a
// lane's loop length is its bucket's size.  Built with one LDS atomic per row
// (16-bit counters packed in pairs), a block scan and one scatter.
constexpr int kRJBuckets = 4096;

// Build rows per partition that fit the LDS row area: key (8 B) + permutation
// (2 B) + the staged build columns (widths w[q]; in[q] == nullptr marks the key
// column itself, which is not staged twice).
int64_t radix_join_capacity(const int *widths, const uint8_t *const *in, int n, int key_bytes) {
  int64_t row = key_bytes + 2;
  for (int q = 0; q < n; ++q)
    if (in[q]) row += widths[q];
  int64_t cap = kRJRowArea / row;
  cap = std::min<int64_t>(cap, kRJMaxRows);
  return cap & ~int64_t(7);  // multiple of 8: every column region stays 8-byte aligned
}

__device__ __forceinline__ uint32_t rj_bucket(int64_t k) {
  return (uint32_t)hashing::fmix64((uint64_t)k) & (kRJBuckets - 1);
}
// narrow keys (low 32 bits): bucket from fmix32, independent of the partition's fmix64 bits
__device__ __forceinline__ uint32_t rj_bucket(uint32_t k) { return hashing::fmix32(k) & (kRJBuckets - 1); }

// output value of a join key: int64 keys as they are; narrow keys rebuilt from their low 32 bits
// and the relations' minimum (every key lies in [kmin, kmin + 2^32))
__device__ __forceinline__ int64_t rj_widen(int64_t k, int64_t) { return k; }
__device__ __forceinline__ int64_t rj_widen(uint32_t k, int64_t kmin) {
  return kmin + (int64_t)(uint32_t)(k - (uint32_t)(uint64_t)kmin);
}
__device__ __forceinline__ int64_t rj_shfl_key(int64_t x, int src);
__device__ __forceinline__ uint32_t rj_shfl_key(uint32_t x, int src) { return __shfl(x, src, kWave); }

// Build rows of one partition: thread t owns rows t + i * kRJThreads (cap <= kRJMaxRows).
constexpr int kRJRowsPerThread = kRJMaxRows / kRJThreads;
static_assert(kRJRowsPerThread * kRJThreads == kRJMaxRows, "build rows per thread");
constexpr int kRJProbeRounds = 1;  // probe rounds of 64 rows per wave prefetched into VGPRs

// bst[0..kRJBuckets) holds per-bucket counts on entry (exclusive starts on exit), bst[kRJBuckets] = total
template <int THREADS = kRJThreads>
__device__ __forceinline__ void rj_scan_buckets(uint16_t *bst, uint32_t *wsum) {
  constexpr int BPT = kRJBuckets / THREADS;
  const int lane = lane_id(), wave = threadIdx.x / kWave;
  uint32_t c[BPT], t = 0;
#pragma unroll
  for (int j = 0; j < BPT; ++j) {
    c[j] = bst[threadIdx.x * BPT + j];
    t += c[j];
  }
  uint32_t inc = t;
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const uint32_t x = __shfl_up(inc, d, kWave);
    if (lane >= d) inc += x;
  }
  if (lane == kWave - 1) wsum[wave] = inc;
  __syncthreads();
  uint32_t off = inc - t;
  for (int w = 0; w < wave; ++w) off += wsum[w];
#pragma unroll
  for (int j = 0; j < BPT; ++j) {
    bst[threadIdx.x * BPT + j] = (uint16_t)off;
    off += c[j];
  }
  if (threadIdx.x == THREADS - 1) bst[kRJBuckets] = (uint16_t)off;
}

// count one bucket's rank for a new row: 16-bit counters packed in pairs
__device__ __forceinline__ uint32_t rj_claim(uint16_t *bst, uint32_t b) {
  const uint32_t sh = (b & 1u) * 16u;
  const uint32_t old = atomicAdd(reinterpret_cast<uint32_t *>(bst) + (b >> 1), 1u << sh);
  return (old >> sh) & 0xffffu;
}

template <class KT>
__device__ __forceinline__ uint32_t rj_count(const uint16_t *bst, const KT *skeys, KT k) {
  const uint32_t b = rj_bucket(k);
  uint32_t c = 0;
  for (uint32_t i = bst[b], e = bst[b + 1]; i < e; ++i) c += (skeys[i] == k);
  return c;
}

// Count kernel block: 512 threads (10 build + 10 probe keys per thread) so two or three
// blocks share a CU (48 KB LDS each) and one block's key loads overlap another's probing;
// the 1024-thread version ran one latency-bound block per CU (128 VGPRs).
constexpr int kRCThreads = 512;
constexpr int kRCWaves = kRCThreads / kWave;
constexpr int kRCRowsPerThread = kRJMaxRows / kRCThreads;
static_assert(kRCRowsPerThread * kRCThreads == kRJMaxRows, "count rows per thread");

template <class KT>
__global__ __launch_bounds__(kRCThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_rj_count(const KT *__restrict__ pkeys,
                                                      const int64_t *__restrict__ poffs,
                                                      const KT *__restrict__ bkeys,
                                                      const int64_t *__restrict__ boffs, int64_t nparts, int cap,
                                                      int64_t pstride, int64_t *__restrict__ counts, int *overflow) {
  // pstride > 1: only partitions 0, pstride, 2 pstride, ... are counted, into counts[p / pstride]
  // (the sampled output-size estimate of the fused write path)
  __shared__ __attribute__((aligned(16))) uint16_t bst[kRJBuckets + 8];
  __shared__ KT skeys[kRJMaxRows];
  __shared__ uint32_t wsum[kRCWaves];
  __shared__ unsigned long long csum[kRCWaves];
  const int64_t nsample = (nparts + pstride - 1) / pstride;
  for (int64_t ci = blockIdx.x; ci < nsample; ci += gridDim.x) {
    const int64_t p = ci * pstride;
    const int64_t rb = boffs[p], nr = boffs[p + 1] - rb;
    const int64_t lb = poffs[p], nl = poffs[p + 1] - lb;
    if (nr > cap) {  // uniform branch: whole block
      if (threadIdx.x == 0) {
        atomicOr(overflow, 1);
        counts[ci] = 0;
      }
      continue;
    }
    if (nr == 0 || nl == 0) {
      if (threadIdx.x == 0) counts[ci] = 0;
      continue;
    }
    // build keys are read twice (claim, then place): the second read hits L2 and the block
    // keeps only 16-bit ranks in registers (two 512-thread blocks per CU without spills)
    __syncthreads();  // previous partition done with bst / skeys / csum
    for (int s = threadIdx.x; s < kRJBuckets / 2; s += blockDim.x) reinterpret_cast<uint32_t *>(bst)[s] = 0;
    __syncthreads();
    uint32_t rk[kRCRowsPerThread];
#pragma unroll
    for (int i = 0; i < kRCRowsPerThread; ++i) {
      const int r = threadIdx.x + i * kRCThreads;
      if (r < nr) rk[i] = rj_claim(bst, rj_bucket(bkeys[rb + r]));
    }
    __syncthreads();
    rj_scan_buckets<kRCThreads>(bst, wsum);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kRCRowsPerThread; ++i) {
      const int r = threadIdx.x + i * kRCThreads;
      if (r < nr) {
        const KT k = bkeys[rb + r];
        skeys[bst[rj_bucket(k)] + rk[i]] = k;
      }
    }
    __syncthreads();
    unsigned long long c = 0;
    for (int64_t l0 = threadIdx.x; l0 < nl; l0 += 4 * kRCThreads) {  // 4 probe loads in flight
      KT pk[4];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (l0 + u * kRCThreads < nl) pk[u] = pkeys[lb + l0 + u * kRCThreads];
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (l0 + u * kRCThreads < nl) c += rj_count(bst, skeys, pk[u]);
    }
    for (int d = kWave / 2; d > 0; d >>= 1) c += __shfl_xor(c, d, kWave);
    if (lane_id() == 0) csum[threadIdx.x / kWave] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long tot = 0;
      for (int w = 0; w < kRCWaves; ++w) tot += csum[w];
      counts[ci] = (int64_t)tot;
    }
  }
}

__device__ __forceinline__ int64_t rj_shfl64(int64_t x, int src) {
  const uint32_t lo = __shfl((uint32_t)(uint64_t)x, src, kWave);
  const uint32_t hi = __shfl((uint32_t)((uint64_t)x >> 32), src, kWave);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ int64_t rj_shfl_key(int64_t x, int src) { return rj_shfl64(x, src); }

struct BuildOut {               // build-side output columns
  uint8_t *out[kMaxFusedCols];
  int width[kMaxFusedCols];
  int lds_off[kMaxFusedCols];   // byte offset of the staged column in the LDS row area, -1 = key
  int n;
};

// OM: emit finds each output slot's probe lane through a per-wave LDS owner map (lanes write
// their lane id into the slots of their matches) instead of a 6-step binary search over the
// wave's match scan with cross-lane permutes (CYLON_RJ_OWNERMAP=1 selects it; A/B knob).
// KT: key type of the partitions (int64_t, or uint32_t low halves of a narrow-key join: kmin
// rebuilds the output keys).  pkey: index of the probe column that IS the key (its value comes
// from the probe key, not a second load; -1 none).
// the write kernel's build staging: rj_dma_block over its 16 waves
__device__ __forceinline__ void rj_dma(const uint8_t *src, int bytes, uint8_t *dst, int wave, int lane) {
  rj_dma_block<kRJWaves>(src, bytes, dst, wave, lane);
}

// DMA: stage the build columns by LDS-DMA (needs W8) instead of register round trips per column.
template <int MAXP, int MAXB, bool W8, bool OM, class KT, bool DMA>
__global__ __launch_bounds__(kRJThreads, 4) void k_rj_write(const KT *__restrict__ pkeys,
                                                            const int64_t *__restrict__ poffs,
                                                            const KT *__restrict__ bkeys,
                                                            const int64_t *__restrict__ boffs, int64_t nparts,
                                                            int cap, const int64_t *__restrict__ out_offs, ColSet pc,
                                                            ColSet bs, BuildOut bo,
                                                            unsigned long long *__restrict__ cursor, int64_t out_cap,
                                                            int *__restrict__ overflow,
                                                            unsigned long long *__restrict__ stamps, int64_t kmin,
                                                            int pkey) {
  // out_offs != nullptr: partition p's rows start at out_offs[p] (exact count kernel ran first).
  // out_offs == nullptr: fused count -- each partition claims its rows from *cursor with one
  // atomic after counting its matches (output partitions land in claim order); a claim past
  // out_cap sets overflow bit 2 and writes nothing (the cursor still totals the rows needed),
  // a build side beyond the LDS capacity sets bit 1.
  // pc: probe columns (in -> out); bs: staged build columns (in, width), LDS
  // region j at 10*cap + sum of cap*width of the earlier ones; bo: build outputs.
  // Row area: keys in bucket order [0, 8 cap), permutation to the staged row
  // [8 cap, 10 cap), payload columns in staged (original) row order.
  __shared__ __attribute__((aligned(16))) uint16_t bst[kRJBuckets + 8];
  __shared__ __attribute__((aligned(16))) uint8_t area[kRJRowArea];
  __shared__ uint32_t wtot[kRJWaves];
  __shared__ int64_t sclaim;
  __shared__ uint8_t ownmap[OM ? kRJWaves * kWave : 1];
  KT *skeys = reinterpret_cast<KT *>(area);
  uint16_t *perm = reinterpret_cast<uint16_t *>(area + sizeof(KT) * (int64_t)cap);
  const int lane = lane_id();
  const int wave = threadIdx.x / kWave;
  int tix = -1;  // debug stamps (CYLON_RJ_STAMPS): block 0's partition count, RP_STAMP slots 0..5
  for (int64_t p = blockIdx.x; p < nparts; p += gridDim.x) {
    const int64_t rb = boffs[p], nr = boffs[p + 1] - rb;
    const int64_t lb = poffs[p], nl = poffs[p + 1] - lb;
    if (nr > cap && out_offs == nullptr && threadIdx.x == 0) atomicOr(overflow, 1);
    if (nr == 0 || nl == 0 || nr > cap) continue;
    ++tix;
    RP_STAMP(0);
    const int64_t obase = out_offs ? out_offs[p] : 0;
    // ---- phase A: probe rows of this wave's slice into VGkRJProbeRoundss (in flight during the build)
    const int64_t per = (nl + kRJWaves - 1) / kRJWaves;  // each wave owns a contiguous probe slice
    const int64_t s0 = lb + std::min<int64_t>(nl, wave * per);
    const int64_t s1 = lb + std::min<int64_t>(nl, (wave + 1) * per);
    KT pk[kRJProbeRounds];
    uint64_t pv[kRJProbeRounds][MAXP];
#pragma unroll
    for (int u = 0; u < kRJProbeRounds; ++u) {
      const int64_t l = s0 + u * kWave + lane;
      if (l < s1) {
        pk[u] = pkeys[l];
#pragma unroll
        for (int q = 0; q < MAXP; ++q)
          if (q < pc.n && q != pkey) pv[u][q] = ldw<W8>(pc.in[q], l, pc.width[q]);
      }
    }
    KT bk[kRJRowsPerThread];
    if (!DMA) {
#pragma unroll
      for (int i = 0; i < kRJRowsPerThread; ++i) {
        const int r = threadIdx.x + i * kRJThreads;
        if (r < nr) bk[i] = bkeys[rb + r];
      }
    }
    // ---- phase B: stage + index the build rows
    __syncthreads();  // previous partition fully done with bst / area / wtot
    for (int s = threadIdx.x; s < kRJBuckets / 2; s += blockDim.x) reinterpret_cast<uint32_t *>(bst)[s] = 0;
    if (DMA) {  // every build column in ONE round trip: the keys (raw order) into the key region,
                // the payload columns into theirs; the loads hold no VGPRs
      rj_dma(reinterpret_cast<const uint8_t *>(bkeys + rb), nr * (int)sizeof(KT), area, wave, lane);
      int64_t off = (int64_t)(sizeof(KT) + 2) * cap;
#pragma unroll
      for (int j = 0; j < MAXB; ++j)
        if (j < bs.n) {
          rj_dma(bs.in[j] + rb * 8, nr * 8, area + off, wave, lane);
          off += (int64_t)cap * 8;
        }
      for (int j = MAXB; j < bs.n; ++j) {  // rare: wide build rows
        for (int r = threadIdx.x; r < nr; r += kRJThreads)
          stw<true>(area + off, r, 8, ldw<true>(bs.in[j], rb + r, 8));
        off += (int64_t)cap * 8;
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else {  // payload columns, column by column (5 loads in flight per column)
      int64_t off = (int64_t)(sizeof(KT) + 2) * cap;
#pragma unroll
      for (int j = 0; j < MAXB; ++j) {
        if (j < bs.n) {
          uint64_t x[kRJRowsPerThread];
#pragma unroll
          for (int i = 0; i < kRJRowsPerThread; ++i)
            if (threadIdx.x + i * kRJThreads < nr) x[i] = ldw<W8>(bs.in[j], rb + threadIdx.x + i * kRJThreads, bs.width[j]);
#pragma unroll
          for (int i = 0; i < kRJRowsPerThread; ++i)
            if (threadIdx.x + i * kRJThreads < nr) stw<W8>(area + off, threadIdx.x + i * kRJThreads, bs.width[j], x[i]);
          off += (int64_t)cap * bs.width[j];
          __builtin_amdgcn_sched_barrier(0);
        }
      }
      for (int j = MAXB; j < bs.n; ++j) {  // rare: wide build rows
        for (int r = threadIdx.x; r < nr; r += kRJThreads)
          stw<W8>(area + off, r, bs.width[j], ldw<W8>(bs.in[j], rb + r, bs.width[j]));
        off += (int64_t)cap * bs.width[j];
      }
    }
    __syncthreads();
    if (DMA) {  // raw keys back from the key region (bucket placement overwrites it after the scan)
#pragma unroll
      for (int i = 0; i < kRJRowsPerThread; ++i) {
        const int r = threadIdx.x + i * kRJThreads;
        if (r < nr) bk[i] = skeys[r];
      }
    }
    RP_STAMP(1);
    uint32_t rk[kRJRowsPerThread];
#pragma unroll
    for (int i = 0; i < kRJRowsPerThread; ++i)
      if (threadIdx.x + i * kRJThreads < nr) rk[i] = rj_claim(bst, rj_bucket(bk[i]));
    __syncthreads();
    rj_scan_buckets(bst, wtot);
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kRJRowsPerThread; ++i) {
      const int r = threadIdx.x + i * kRJThreads;
      if (r < nr) {
        const uint32_t pos = bst[rj_bucket(bk[i])] + rk[i];
        skeys[pos] = bk[i];
        perm[pos] = (uint16_t)r;
      }
    }
    __syncthreads();
    RP_STAMP(2);
    // ---- phase C: count this wave's matches, slice offsets
    uint32_t c = 0;
#pragma unroll
    for (int u = 0; u < kRJProbeRounds; ++u)
      if (s0 + u * kWave + lane < s1) c += rj_count(bst, skeys, pk[u]);
    {  // later rounds' probe keys two rounds at a time (both loads in flight before either count)
      int64_t l = s0 + kRJProbeRounds * kWave + lane;
      for (; l + kWave < s1; l += 2 * kWave) {
        const KT ka = pkeys[l], kb = pkeys[l + kWave];
        c += rj_count(bst, skeys, ka) + rj_count(bst, skeys, kb);
      }
      if (l < s1) c += rj_count(bst, skeys, pkeys[l]);
    }
    for (int d = kWave / 2; d > 0; d >>= 1) c += __shfl_xor(c, d, kWave);
    if (lane == 0) wtot[wave] = c;
    __syncthreads();
    int64_t base = obase;
    if (out_offs == nullptr) {
      if (threadIdx.x == 0) {
        unsigned long long tot = 0;
        for (int w = 0; w < kRJWaves; ++w) tot += wtot[w];
        const unsigned long long at = tot ? atomicAdd(cursor, tot) : 0ull;
        const bool fits = at + tot <= (unsigned long long)out_cap;
        if (!fits) atomicOr(overflow, 2);
        sclaim = fits ? (int64_t)at : -1;
      }
      __syncthreads();
      base = sclaim;
      if (base < 0) continue;  // uniform: the block's claim did not fit
    }
    for (int w = 0; w < wave; ++w) base += wtot[w];
    RP_STAMP(3);
    // ---- phase D: emit.  Round u + 1's probe row is loaded while round u expands (kn / vn), so
    // only the first round after the phase-A prefetch waits on memory.
    static_assert(kRJProbeRounds == 1, "emit prefetch assumes one phase-A round");
    KT kn = 0;
    uint64_t vn[MAXP] = {};
    for (int u = 0; s0 + (int64_t)u * kWave < s1; ++u) {
      const int64_t l = s0 + (int64_t)u * kWave + lane;
      const bool active = l < s1;
      KT k = 0;
      uint64_t v[MAXP] = {};
      if (u == 0) {
        k = pk[0];
#pragma unroll
        for (int q = 0; q < MAXP; ++q) v[q] = pv[0][q];
      } else {
        k = kn;
#pragma unroll
        for (int q = 0; q < MAXP; ++q) v[q] = vn[q];
      }
      if (l + kWave < s1) {  // prefetch round u + 1
        kn = pkeys[l + kWave];
#pragma unroll
        for (int q = 0; q < MAXP; ++q)
          if (q < pc.n && q != pkey) vn[q] = ldw<W8>(pc.in[q], l + kWave, pc.width[q]);
      }
      uint32_t i0 = 0, i1 = 0, mc = 0;
      if (active) {
        const uint32_t b = rj_bucket(k);
        i0 = bst[b];
        i1 = bst[b + 1];
        for (uint32_t i = i0; i < i1; ++i) mc += (skeys[i] == k);
      }
      uint32_t inc = mc;  // wave inclusive scan of match counts
#pragma unroll
      for (int d = 1; d < kWave; d <<= 1) {
        const uint32_t x = __shfl_up(inc, d, kWave);
        if (lane >= d) inc += x;
      }
      const uint32_t wsum = __shfl(inc, kWave - 1, kWave);
      const uint32_t excl = inc - mc;
      // Load-balanced expansion: lane t writes output rows base + t, base + 64 + t, ...
      // of this round, so every store covers a contiguous, fully active run of the
      // output column (a lane-per-probe-row loop over bucket entries would issue
      // sparse partial-line stores).  The producing probe lane ("owner") of row
      // s is found by a binary search over the wave's inclusive match counts and
      // its key / bucket / payload are read with cross-lane permutes.
      for (uint32_t t0 = 0; t0 < wsum; t0 += kWave) {
        const uint32_t so = t0 + lane;
        const bool act = so < wsum;
        int owner = 0;
        if (OM) {
          uint8_t *om = ownmap + wave * kWave;
          const uint32_t e0 = excl > t0 ? excl : t0, e1 = excl + mc < t0 + kWave ? excl + mc : t0 + kWave;
          __builtin_amdgcn_wave_barrier();  // the previous window's reads are done
          for (uint32_t x = e0; x < e1; ++x) om[x - t0] = (uint8_t)lane;
          __builtin_amdgcn_wave_barrier();
          owner = act ? om[lane] : 0;
        } else {
#pragma unroll
          for (int step = kWave / 2; step >= 1; step >>= 1) {
            const uint32_t ic = __shfl(inc, owner + step - 1, kWave);
            if (ic <= so) owner += step;
          }
        }
        const uint32_t j = so - __shfl(excl, owner, kWave);  // match rank inside the owner's bucket
        const KT ko = rj_shfl_key(k, owner);
        const uint64_t kw = (uint64_t)rj_widen(ko, kmin);
        const uint32_t b0 = __shfl(i0, owner, kWave), b1 = __shfl(i1, owner, kWave);
        uint64_t vo[MAXP];
#pragma unroll
        for (int q = 0; q < MAXP; ++q) vo[q] = q == pkey ? kw : (uint64_t)rj_shfl64((int64_t)v[q], owner);
        if (act) {
          int r = 0;
          for (uint32_t i = b0, c = 0; i < b1; ++i) {
            if (skeys[i] != ko) continue;
            if (c == j) {
              r = perm[i];
              break;
            }
            ++c;
          }
          const int64_t o = base + so;
#pragma unroll
          for (int q = 0; q < MAXP; ++q)
            if (q < pc.n) stw<W8>(pc.out[q], o, pc.width[q], vo[q]);
          if (pc.n > MAXP) {
            const int64_t lo = s0 + (int64_t)u * kWave + owner;
            for (int q = MAXP; q < pc.n; ++q)
              stw<W8>(pc.out[q], o, pc.width[q], q == pkey ? kw : ldw<W8>(pc.in[q], lo, pc.width[q]));
          }
#pragma unroll
          for (int q = 0; q < MAXB + 1; ++q)
            if (q < bo.n)
              stw<W8>(bo.out[q], o, bo.width[q],
                      bo.lds_off[q] < 0 ? kw : ldw<W8>(area + bo.lds_off[q], r, bo.width[q]));
          for (int q = MAXB + 1; q < bo.n; ++q)
            stw<W8>(bo.out[q], o, bo.width[q],
                    bo.lds_off[q] < 0 ? kw : ldw<W8>(area + bo.lds_off[q], r, bo.width[q]));
        }
      }
      base += wsum;
    }
    RP_STAMP(4);
  }
}

static int rj_grid(int64_t nparts) { return (int)std::min<int64_t>(nparts, kNumCUs * 8); }

void radix_join_count(const void *pkeys, const int64_t *poffs, const void *bkeys, const int64_t *boffs,
                      int64_t nparts, int64_t cap, int64_t *counts, int *overflow, void *stream, int64_t pstride,
                      int key_bytes) {
  CYLON_CHECK(cap > 0 && cap <= kRJMaxRows, Code::Invalid, "radix join capacity " << cap);
  CYLON_CHECK(pstride >= 1, Code::Invalid, "partition stride " << pstride);
  CYLON_CHECK(key_bytes == 8 || key_bytes == 4, Code::Invalid, "radix join key bytes " << key_bytes);
  hipStream_t s = as_stream(stream);
  HIP_CHECK(hipMemsetAsync(overflow, 0, sizeof(int), s));
  const int64_t nsample = (nparts + pstride - 1) / pstride;
  const dim3 grid((unsigned)std::max<int64_t>(1, std::min<int64_t>(nsample, kNumCUs * 12)));
  if (key_bytes == 8)
    hipLaunchKernelGGL(k_rj_count<int64_t>, grid, dim3(kRCThreads), 0, s, static_cast<const int64_t *>(pkeys), poffs,
                       static_cast<const int64_t *>(bkeys), boffs, nparts, (int)cap, pstride, counts, overflow);
  else
    hipLaunchKernelGGL(k_rj_count<uint32_t>, grid, dim3(kRCThreads), 0, s, static_cast<const uint32_t *>(pkeys), poffs,
                       static_cast<const uint32_t *>(bkeys), boffs, nparts, (int)cap, pstride, counts, overflow);
  HIP_LAUNCH_CHECK();
}

void radix_join_write(const void *pkeys, const int64_t *poffs, const void *bkeys, const int64_t *boffs,
                      int64_t nparts, int64_t cap, const int64_t *out_offs, const uint8_t *const *pin,
                      uint8_t *const *pout, const int *pw, int npc, const uint8_t *const *bin, uint8_t *const *bout,
                      const int *bw, int nbc, void *stream, int64_t *cursor, int64_t out_cap, int *overflow,
                      int key_bytes, int64_t kmin, int pkey) {
  CYLON_CHECK(key_bytes == 8 || key_bytes == 4, Code::Invalid, "radix join key bytes " << key_bytes);
  CYLON_CHECK(pkey >= -1 && pkey < npc, Code::Invalid, "radix join probe key column " << pkey);
  CYLON_CHECK(npc <= kMaxFusedCols && nbc <= kMaxFusedCols, Code::Invalid, "too many columns");
  CYLON_CHECK(out_offs != nullptr || (cursor != nullptr && overflow != nullptr), Code::Invalid,
              "radix join write: needs partition offsets or an output cursor");
  CYLON_CHECK(cap > 0 && cap <= radix_join_capacity(bw, bin, nbc, key_bytes), Code::Invalid,
              "radix join capacity " << cap);
  ColSet pc, bs;
  BuildOut bo;
  pc.n = npc;
  bs.n = 0;
  bo.n = nbc;
  bool w8 = true;
  for (int q = 0; q < kMaxFusedCols; ++q) {
    pc.in[q] = q < npc ? pin[q] : nullptr;
    pc.out[q] = q < npc ? pout[q] : nullptr;
    pc.width[q] = q < npc ? pw[q] : 8;
    bs.in[q] = nullptr;
    bs.out[q] = nullptr;
    bs.width[q] = 8;
    bo.out[q] = q < nbc ? bout[q] : nullptr;
    bo.width[q] = q < nbc ? bw[q] : 8;
    bo.lds_off[q] = -1;
    if (q < npc) w8 &= pw[q] == 8;
    if (q < nbc) w8 &= bw[q] == 8;
  }
  int64_t off = (key_bytes + 2) * cap;
  for (int q = 0; q < nbc; ++q)
    if (bin[q]) {
      bo.lds_off[q] = (int)off;
      off += cap * bw[q];
      bs.in[bs.n] = bin[q];
      bs.width[bs.n++] = bw[q];
    }
  CYLON_CHECK(off <= kRJRowArea, Code::Invalid, "radix join LDS rows " << off);
  hipStream_t s = as_stream(stream);
  // probe columns beyond 4 and staged build columns beyond 3 are loaded in place (slower, correct)
  unsigned long long *cur = reinterpret_cast<unsigned long long *>(cursor);
  static const bool stamp = std::getenv("CYLON_RJ_STAMPS") != nullptr;  // debug: phase stamps to stderr
  unsigned long long *st = nullptr;
  if (stamp) {
    HIP_CHECK(hipStreamSynchronize(s));
    HIP_CHECK(hipMalloc(&st, sizeof(unsigned long long) * kRPStampTiles * kRPStampSlots));
    HIP_CHECK(hipMemset(st, 0, sizeof(unsigned long long) * kRPStampTiles * kRPStampSlots));
  }
  const char *om = std::getenv("CYLON_RJ_OWNERMAP");
  const bool ownermap = om && om[0] == '1';
  const dim3 grid(rj_grid(nparts));
  const int64_t *pk8 = static_cast<const int64_t *>(pkeys), *bk8 = static_cast<const int64_t *>(bkeys);
  const uint32_t *pk4 = static_cast<const uint32_t *>(pkeys), *bk4 = static_cast<const uint32_t *>(bkeys);
  // LDS-DMA build staging: write kernel 33.9 -> 32.9 ms per 1B x 1B join (profiles/r03/lds_dma_ab.txt)
  const char *dm = std::getenv("CYLON_RJ_DMA");  // A/B knob: 0 = register staging
  const bool dma = w8 && !(dm && dm[0] == '0');
  if (key_bytes == 4 && dma)
    hipLaunchKernelGGL((k_rj_write<4, 3, true, false, uint32_t, true>), grid, dim3(kRJThreads), 0, s, pk4, poffs, bk4,
                       boffs, nparts, (int)cap, out_offs, pc, bs, bo, cur, out_cap, overflow, st, kmin, pkey);
  else if (dma && !ownermap)
    hipLaunchKernelGGL((k_rj_write<4, 3, true, false, int64_t, true>), grid, dim3(kRJThreads), 0, s, pk8, poffs, bk8,
                       boffs, nparts, (int)cap, out_offs, pc, bs, bo, cur, out_cap, overflow, st, kmin, pkey);
  else if (key_bytes == 4 && w8)
    hipLaunchKernelGGL((k_rj_write<4, 3, true, false, uint32_t, false>), grid, dim3(kRJThreads), 0, s, pk4, poffs, bk4, boffs,
                       nparts, (int)cap, out_offs, pc, bs, bo, cur, out_cap, overflow, st, kmin, pkey);
  else if (key_bytes == 4)
    hipLaunchKernelGGL((k_rj_write<4, 3, false, false, uint32_t, false>), grid, dim3(kRJThreads), 0, s, pk4, poffs, bk4,
                       boffs, nparts, (int)cap, out_offs, pc, bs, bo, cur, out_cap, overflow, st, kmin, pkey);
  else if (w8 && ownermap)
    hipLaunchKernelGGL((k_rj_write<4, 3, true, true, int64_t, false>), grid, dim3(kRJThreads), 0, s, pk8, poffs, bk8, boffs,
                       nparts, (int)cap, out_offs, pc, bs, bo, cur, out_cap, overflow, st, kmin, pkey);
  else if (w8)
    hipLaunchKernelGGL((k_rj_write<4, 3, true, false, int64_t, false>), grid, dim3(kRJThreads), 0, s, pk8, poffs, bk8, boffs,
                       nparts, (int)cap, out_offs, pc, bs, bo, cur, out_cap, overflow, st, kmin, pkey);
  else
    hipLaunchKernelGGL((k_rj_write<4, 3, false, false, int64_t, false>), grid, dim3(kRJThreads), 0, s, pk8, poffs, bk8,
                       boffs, nparts, (int)cap, out_offs, pc, bs, bo, cur, out_cap, overflow, st, kmin, pkey);
  HIP_LAUNCH_CHECK();
  if (st) {  // mean cycles per partition: load+stage, index build, count+claim, emit, then to the next
    HIP_CHECK(hipStreamSynchronize(s));
    std::vector<unsigned long long> h(kRPStampTiles * kRPStampSlots);
    HIP_CHECK(hipMemcpy(h.data(), st, h.size() * sizeof(h[0]), hipMemcpyDeviceToHost));
    HIP_CHECK(hipFree(st));
    double sum[5] = {0};
    int np = 0;
    for (int t = 1; t + 1 < kRPStampTiles; ++t) {
      const unsigned long long *a = &h[t * kRPStampSlots], *b = &h[(t + 1) * kRPStampSlots];
      if (b[0] == 0 || a[4] == 0) break;
      for (int j = 1; j <= 4; ++j) sum[j - 1] += (double)(a[j] - a[j - 1]);
      sum[4] += (double)(b[0] - a[0]);
      ++np;
    }
    if (np)
      std::fprintf(stderr, "rj_stamps partitions=%d total=%.0f | stage=%.0f index=%.0f count=%.0f emit=%.0f\n", np,
                   sum[4] / np, sum[0] / np, sum[1] / np, sum[2] / np, sum[3] / np);
  }
}


// --------------------------------------------------------------------------
// K7 range join: sort-algorithm inner join on range partitions
// --------------------------------------------------------------------------
// Both relations are partitioned by RangeDigit into key ranges of 2^rshift
// values (rshift <= 12), so inside a partition the low rshift bits of
// (key ^ flip) - mn are an exact key offset.  Per partition one workgroup
// counts both sides by key offset in LDS (4096 buckets), scans the counts into
// CSR starts and output offsets, scatters each side's row numbers into key
// order (uint16 permutations), and then emits output rows slot-major: output
// row t of the partition finds its key by a binary search over the output
// offsets and its (left, right) pair as (idx / |R_v|, idx % |R_v|).  The output
// is therefore ordered by key (partitions are key ranges in order), with no key
// comparisons at all and every output column written as contiguous runs.
constexpr int kRGThreads = 1024;
constexpr int kRGMaxRows = 8192;  // rows per side per partition (uint16 permutations)
constexpr int kRGBuckets = 4096;
constexpr int kRGBucketsPerThread = kRGBuckets / kRGThreads;

int64_t range_join_max_rows() { return kRGMaxRows; }
int range_join_max_shift() { return 12; }

constexpr int kRGRowsPerThread = kRGMaxRows / kRGThreads;

// Low 32 bits of a partition's keys (all the bucket needs: the offset is taken
// mod 2^rshift) held in registers, kRGRowsPerThread per thread; loaded for the
// next partition while the current one is processed.
struct RGKeys {
  int64_t b = 0, n = 0;
  uint32_t k[kRGRowsPerThread];
};

__device__ __forceinline__ void rg_load(const int64_t *__restrict__ keys, const int64_t *__restrict__ offs, int64_t p,
                                        RGKeys &s) {
  s.b = offs[p];
  s.n = offs[p + 1] - s.b;
  const uint32_t *k32 = reinterpret_cast<const uint32_t *>(keys);
#pragma unroll
  for (int i = 0; i < kRGRowsPerThread; ++i) {
    const int64_t r = threadIdx.x + i * kRGThreads;
    if (r < s.n && r < kRGMaxRows) s.k[i] = k32[2 * (s.b + r)];  // little endian: low half
  }
}

__device__ __forceinline__ uint32_t rg_bucket32(uint32_t k, uint32_t flip, uint32_t mn, uint32_t bmask) {
  return ((k ^ flip) - mn) & bmask;
}

__global__ __launch_bounds__(kRGThreads) void k_rg_count(const int64_t *__restrict__ lkeys,
                                                         const int64_t *__restrict__ loffs,
                                                         const int64_t *__restrict__ rkeys,
                                                         const int64_t *__restrict__ roffs, int64_t nparts,
                                                         uint64_t flip, uint64_t mn, uint32_t bmask,
                                                         int64_t *__restrict__ counts, int *overflow) {
  __shared__ uint32_t hl[kRGBuckets], hr[kRGBuckets];
  __shared__ unsigned long long wsum[kRGThreads / kWave];
  const uint32_t nb = bmask + 1, f32 = (uint32_t)flip, m32 = (uint32_t)mn;
  RGKeys nl_, nr_;
  if ((int64_t)blockIdx.x < nparts) {
    rg_load(lkeys, loffs, blockIdx.x, nl_);
    rg_load(rkeys, roffs, blockIdx.x, nr_);
  }
  for (int64_t p = blockIdx.x; p < nparts; p += gridDim.x) {
    const RGKeys L = nl_, R = nr_;
    if (p + gridDim.x < nparts) {  // next partition's keys in flight during this one
      rg_load(lkeys, loffs, p + gridDim.x, nl_);
      rg_load(rkeys, roffs, p + gridDim.x, nr_);
    }
    if (L.n > kRGMaxRows || R.n > kRGMaxRows) {  // uniform branch
      if (threadIdx.x == 0) {
        atomicOr(overflow, 1);
        counts[p] = 0;
      }
      continue;
    }
    if (L.n == 0 || R.n == 0) {
      if (threadIdx.x == 0) counts[p] = 0;
      continue;
    }
    __syncthreads();  // previous partition done with hl / hr / wsum
    for (uint32_t v = threadIdx.x; v < nb; v += kRGThreads) hl[v] = hr[v] = 0;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kRGRowsPerThread; ++i) {
      const int64_t r = threadIdx.x + i * kRGThreads;
      if (r < L.n) atomicAdd(&hl[rg_bucket32(L.k[i], f32, m32, bmask)], 1u);
      if (r < R.n) atomicAdd(&hr[rg_bucket32(R.k[i], f32, m32, bmask)], 1u);
    }
    __syncthreads();
    unsigned long long c = 0;
    for (uint32_t v = threadIdx.x; v < nb; v += kRGThreads) c += (unsigned long long)hl[v] * hr[v];
    for (int d = kWave / 2; d > 0; d >>= 1) c += __shfl_xor(c, d, kWave);
    if (lane_id() == 0) wsum[threadIdx.x / kWave] = c;
    __syncthreads();
    if (threadIdx.x == 0) {
      unsigned long long t = 0;
      for (int w = 0; w < kRGThreads / kWave; ++w) t += wsum[w];
      counts[p] = (int64_t)t;
    }
  }
}

// exclusive scan of a[0..nb) in place (a[nb] = total), kRGBucketsPerThread values per thread
template <class T>
__device__ __forceinline__ void rg_scan(T *a, uint32_t nb, T *wtot) {
  const int lane = lane_id(), wave = threadIdx.x / kWave;
  T c[kRGBucketsPerThread], t = 0;
#pragma unroll
  for (int j = 0; j < kRGBucketsPerThread; ++j) {
    const uint32_t v = threadIdx.x * kRGBucketsPerThread + j;
    c[j] = v < nb ? a[v] : T(0);
    t += c[j];
  }
  T inc = t;
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const T x = __shfl_up(inc, d, kWave);
    if (lane >= d) inc += x;
  }
  if (lane == kWave - 1) wtot[wave] = inc;
  __syncthreads();
  T off = inc - t;
  for (int w = 0; w < wave; ++w) off += wtot[w];
  T total = 0;
  for (int w = 0; w < kRGThreads / kWave; ++w) total += wtot[w];
#pragma unroll
  for (int j = 0; j < kRGBucketsPerThread; ++j) {
    const uint32_t v = threadIdx.x * kRGBucketsPerThread + j;
    if (v < nb) a[v] = off;
    off += c[j];
  }
  if (threadIdx.x == 0) a[nb] = total;
}

constexpr int kRGEmit = 4;  // output rows per thread per emit chunk (4096 per chunk)

// stream one column of a partition side into the LDS stage (coalesced), then write
// the chunk's output rows from it: an output row's payload is a random row of the
// partition, so gathering it straight from global memory would pull a whole cache
// line through L2 -> L1 per 8-byte value (the first version of this kernel was
// bound by exactly that).
template <bool W8>
__device__ __forceinline__ void rg_emit_column(uint8_t *stage, const uint8_t *in, int64_t base, int64_t rows,
                                               uint8_t *out, int w, int64_t obase, uint32_t c0, uint32_t total,
                                               const uint16_t *pos) {
  __syncthreads();  // stage free
  for (int64_t r0 = 0; r0 < rows; r0 += 4 * kRGThreads) {  // four loads in flight per thread
    uint64_t x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t r = r0 + u * kRGThreads + threadIdx.x;
      if (r < rows) x[u] = ldw<W8>(in, base + r, w);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t r = r0 + u * kRGThreads + threadIdx.x;
      if (r < rows) stw<W8>(stage, r, w, x[u]);
    }
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < kRGEmit; ++e) {
    const uint32_t t = c0 + e * kRGThreads + threadIdx.x;
    if (t < total) stw<W8>(out, obase + t, w, ldw<W8>(stage, pos[e], w));
  }
}

template <bool W8>
__global__ __launch_bounds__(kRGThreads) void k_rg_write(const int64_t *__restrict__ lkeys,
                                                         const int64_t *__restrict__ loffs,
                                                         const int64_t *__restrict__ rkeys,
                                                         const int64_t *__restrict__ roffs, int64_t nparts,
                                                         uint64_t flip, uint64_t mn, uint32_t bmask,
                                                         const int64_t *__restrict__ out_offs, ColSet lc, ColSet rc) {
  __shared__ uint32_t ls[kRGBuckets + 1], rs[kRGBuckets + 1], oo[kRGBuckets + 1];
  __shared__ uint16_t pl[kRGMaxRows], pr[kRGMaxRows];
  __shared__ uint64_t stage64[kRGMaxRows];  // scatter cursors, then one payload column at a time
  __shared__ uint32_t wtot[3][kRGThreads / kWave];
  uint8_t *stage = reinterpret_cast<uint8_t *>(stage64);
  uint32_t *lcur = reinterpret_cast<uint32_t *>(stage64), *rcur = lcur + kRGBuckets;
  static_assert(2 * kRGBuckets * sizeof(uint32_t) <= kRGMaxRows * sizeof(uint64_t), "cursors fit the stage");
  const uint32_t nb = bmask + 1, f32 = (uint32_t)flip, m32 = (uint32_t)mn;
  RGKeys nl_, nr_;
  if ((int64_t)blockIdx.x < nparts) {
    rg_load(lkeys, loffs, blockIdx.x, nl_);
    rg_load(rkeys, roffs, blockIdx.x, nr_);
  }
  for (int64_t p = blockIdx.x; p < nparts; p += gridDim.x) {
    const RGKeys L = nl_, R = nr_;
    if (p + gridDim.x < nparts) {  // next partition's keys in flight during this one
      rg_load(lkeys, loffs, p + gridDim.x, nl_);
      rg_load(rkeys, roffs, p + gridDim.x, nr_);
    }
    const int64_t lb = L.b, nl = L.n, rb = R.b, nr = R.n;
    if (nl == 0 || nr == 0 || nl > kRGMaxRows || nr > kRGMaxRows) continue;
    const int64_t obase = out_offs[p];
    __syncthreads();  // previous partition fully done with the LDS arrays
    for (uint32_t v = threadIdx.x; v < nb; v += kRGThreads) ls[v] = rs[v] = 0;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kRGRowsPerThread; ++i) {
      const int64_t r = threadIdx.x + i * kRGThreads;
      if (r < nl) atomicAdd(&ls[rg_bucket32(L.k[i], f32, m32, bmask)], 1u);
      if (r < nr) atomicAdd(&rs[rg_bucket32(R.k[i], f32, m32, bmask)], 1u);
    }
    __syncthreads();
    for (uint32_t v = threadIdx.x; v < nb; v += kRGThreads) oo[v] = ls[v] * rs[v];
    __syncthreads();
    rg_scan(ls, nb, wtot[0]);
    rg_scan(rs, nb, wtot[1]);
    rg_scan(oo, nb, wtot[2]);
    __syncthreads();
    for (uint32_t v = threadIdx.x; v < nb; v += kRGThreads) {
      lcur[v] = ls[v];
      rcur[v] = rs[v];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kRGRowsPerThread; ++i) {
      const int64_t r = threadIdx.x + i * kRGThreads;
      if (r < nl) pl[atomicAdd(&lcur[rg_bucket32(L.k[i], f32, m32, bmask)], 1u)] = (uint16_t)r;
      if (r < nr) pr[atomicAdd(&rcur[rg_bucket32(R.k[i], f32, m32, bmask)], 1u)] = (uint16_t)r;
    }
    __syncthreads();
    const uint32_t total = oo[nb];
    for (uint32_t c0 = 0; c0 < total; c0 += kRGEmit * kRGThreads) {
      uint16_t lp[kRGEmit], rp[kRGEmit];  // partition rows of this thread's output rows
#pragma unroll
      for (int e = 0; e < kRGEmit; ++e) {
        const uint32_t t = c0 + e * kRGThreads + threadIdx.x;
        lp[e] = rp[e] = 0;
        if (t < total) {
          uint32_t lo = 0, hi = nb;  // largest v with oo[v] <= t (always a non-empty key)
          while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (oo[mid] <= t) lo = mid; else hi = mid;
          }
          const uint32_t idx = t - oo[lo], cr = rs[lo + 1] - rs[lo];
          const uint32_t li = idx / cr, ri = idx - li * cr;
          lp[e] = pl[ls[lo] + li];
          rp[e] = pr[rs[lo] + ri];
        }
      }
#pragma unroll 1
      for (int q = 0; q < lc.n; ++q)
        rg_emit_column<W8>(stage, lc.in[q], lb, nl, lc.out[q], lc.width[q], obase, c0, total, lp);
#pragma unroll 1
      for (int q = 0; q < rc.n; ++q)
        rg_emit_column<W8>(stage, rc.in[q], rb, nr, rc.out[q], rc.width[q], obase, c0, total, rp);
    }
  }
}

static int rg_grid(int64_t nparts) { return (int)std::min<int64_t>(nparts, kNumCUs * 4); }

void range_join_count(const int64_t *lkeys, const int64_t *loffs, const int64_t *rkeys, const int64_t *roffs,
                      int64_t nparts, uint64_t flip, uint64_t mn, int rshift, int64_t *counts, int *overflow,
                      void *stream) {
  CYLON_CHECK(rshift >= 0 && rshift <= 12, Code::Invalid, "range join key bits per partition " << rshift);
  hipStream_t s = as_stream(stream);
  HIP_CHECK(hipMemsetAsync(overflow, 0, sizeof(int), s));
  if (nparts == 0) return;
  hipLaunchKernelGGL(k_rg_count, dim3(rg_grid(nparts)), dim3(kRGThreads), 0, s, lkeys, loffs, rkeys, roffs, nparts,
                     flip, mn, (uint32_t)((1u << rshift) - 1), counts, overflow);
  HIP_LAUNCH_CHECK();
}

void range_join_write(const int64_t *lkeys, const int64_t *loffs, const int64_t *rkeys, const int64_t *roffs,
                      int64_t nparts, uint64_t flip, uint64_t mn, int rshift, const int64_t *out_offs,
                      const uint8_t *const *lin, uint8_t *const *lout, const int *lw, int nlc,
                      const uint8_t *const *rin, uint8_t *const *rout, const int *rw, int nrc, void *stream) {
  CYLON_CHECK(rshift >= 0 && rshift <= 12, Code::Invalid, "range join key bits per partition " << rshift);
  CYLON_CHECK(nlc <= kMaxFusedCols && nrc <= kMaxFusedCols, Code::Invalid, "too many columns");
  if (nparts == 0) return;
  ColSet lc, rc;
  lc.n = nlc;
  rc.n = nrc;
  bool w8 = true;
  for (int q = 0; q < kMaxFusedCols; ++q) {
    lc.in[q] = q < nlc ? lin[q] : nullptr;
    lc.out[q] = q < nlc ? lout[q] : nullptr;
    lc.width[q] = q < nlc ? lw[q] : 8;
    rc.in[q] = q < nrc ? rin[q] : nullptr;
    rc.out[q] = q < nrc ? rout[q] : nullptr;
    rc.width[q] = q < nrc ? rw[q] : 8;
    if (q < nlc) w8 &= lw[q] == 8;
    if (q < nrc) w8 &= rw[q] == 8;
  }
  const uint32_t bmask = (uint32_t)((1u << rshift) - 1);
  hipStream_t s = as_stream(stream);
  if (w8)
    hipLaunchKernelGGL(k_rg_write<true>, dim3(rg_grid(nparts)), dim3(kRGThreads), 0, s, lkeys, loffs, rkeys, roffs,
                       nparts, flip, mn, bmask, out_offs, lc, rc);
  else
    hipLaunchKernelGGL(k_rg_write<false>, dim3(rg_grid(nparts)), dim3(kRGThreads), 0, s, lkeys, loffs, rkeys, roffs,
                       nparts, flip, mn, bmask, out_offs, lc, rc);
  HIP_LAUNCH_CHECK();
}

}  // namespace hip
}  // namespace cylon
