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
#include "radix_common.hpp"

namespace cylon {
namespace hip {

// --------------------------------------------------------------------------
// partition pass
// --------------------------------------------------------------------------
// Join digit: bits [shift, shift + log2(mask+1)) of the top `bits` bits of fmix64(key).
struct PartDigit {
  const int64_t *keys;
  int bits;   // total partition bits
  int shift;  // digit = (part >> shift) & mask
  uint32_t mask;
  CYLON_DIGIT_COMMON
  __device__ __forceinline__ uint32_t of_key(int64_t k) const { return (part_of(k, bits) >> shift) & mask; }
  __device__ __forceinline__ uint32_t operator()(int64_t i) const { return of_key(keys[i]); }
  // look-back counting: the next pass's digit of a stored key
  __device__ __forceinline__ uint32_t next_of(uint64_t stored, int nshift, uint32_t nmask, uint64_t) const {
    return (part_of((int64_t)stored, bits) >> nshift) & nmask;
  }
};


// Narrowed join digit (join partitions of int64 keys): every key of a join lies in [base, base + 2^32)
// with base = (left key 0) - 2^31 (checked on the fly; a key outside sets *bad and the join
// repartitions without narrowing), so column 0 travels as the uint32 offset key - base -- 4 B/row
// less in every pass write, in the second pass's reads and in the join kernel's reads -- and the
// partition is the top bits of fmix32(offset) (a bijection: equal offsets <=> equal keys).
struct PartDigitN {
  static constexpr bool kNarrow = true;
  const void *keys;          // int64 keys (first pass) or uint32 offsets (later passes)
  int kin4;                  // keys holds uint32 offsets
  const int64_t *base_src;   // base = base_src[0] - 2^31, read by init()
  unsigned int *bad;         // set when a key lies outside [base, base + 2^32)
  int bits;                  // total partition bits
  int shift;                 // digit = (part >> shift) & mask
  uint32_t mask;
  int64_t base;
  __device__ __forceinline__ void init() { base = (int64_t)((uint64_t)base_src[0] - (uint64_t(1) << 31)); }
  __device__ __forceinline__ uint64_t key_at(int64_t i) const {
    return kin4 ? (uint64_t)reinterpret_cast<const uint32_t *>(keys)[i]
                : (uint64_t)reinterpret_cast<const int64_t *>(keys)[i];
  }
  __device__ __forceinline__ uint64_t narrow(uint64_t kv) const {
    return kin4 ? (kv & 0xffffffffull) : ((kv - (uint64_t)base) & 0xffffffffull);
  }
  __device__ __forceinline__ bool too_wide(uint64_t kv) const { return !kin4 && (kv - (uint64_t)base) > 0xffffffffull; }
  __device__ __forceinline__ void report_bad() const { atomicOr(bad, 1u); }
  __device__ __forceinline__ uint32_t of_key(int64_t k) const { return of_offset((uint32_t)narrow((uint64_t)k)); }
  __device__ __forceinline__ uint32_t of_offset(uint32_t off) const {
    return bits == 0 ? 0u : ((hashing::fmix32(off) >> (32 - bits)) >> shift) & mask;
  }
  __device__ __forceinline__ uint32_t operator()(int64_t i) const { return of_key((int64_t)key_at(i)); }
};

// Shuffle digit: the reference's partition of a single 8-byte integer key
// (ModuloPartitionKernel: h = (uint32)key, pid = h % P, or h & (P-1) for powers
// of two; partition.hip partition_f + hashing::partitioner), so one LDS-staged
// pass produces the partition-major order of the whole table.
struct ModDigit {
  const int64_t *keys;
  uint32_t nparts;
  CYLON_DIGIT_COMMON
  __device__ __forceinline__ uint32_t of_key(int64_t k) const {
    return hashing::partitioner((uint32_t)(uint64_t)k, nparts);
  }
  __device__ __forceinline__ uint32_t operator()(int64_t i) const { return of_key(keys[i]); }
};

// Sort digit: bits [shift, shift + log2(mask+1)) of an order-preserving uint64 image (K6), less
// the smallest image (sub): keys spanning less than their varying bits need fewer digit bits
// (uniform keys in [-2^62, 2^62) vary in all 64 bits but span 63: 7 x 9-bit digits, not 10 + 6 x 9)
struct ImageDigit {
  const int64_t *keys;
  int shift;
  uint32_t mask;
  uint64_t flip;  // image = key ^ flip (0 once column 0 holds images)
  uint64_t sub;
  CYLON_DIGIT_COMMON
  __device__ __forceinline__ uint32_t of_key(int64_t k) const {
    return (uint32_t)((((uint64_t)k ^ flip) - sub) >> shift) & mask;
  }
  __device__ __forceinline__ uint32_t operator()(int64_t i) const { return of_key(keys[i]); }
  // look-back counting: the next pass's digit of a stored image
  __device__ __forceinline__ uint32_t next_of(uint64_t stored, int nshift, uint32_t nmask, uint64_t nsub) const {
    return (uint32_t)((stored - nsub) >> nshift) & nmask;
  }
};

// digits whose pass can write the next pass's digit of every stored key (ColSet::nd_out)
template <class Digit>
constexpr bool kNdDigit = std::is_same<Digit, ImageDigit>::value || std::is_same<Digit, PartDigit>::value;

// Order-preserving range digit (K7 range join): the partition of key k is
// ((k ^ flip) - mn) >> rshift -- key ranges in key order -- and a pass's digit is
// bits [shift, shift + log2(mask + 1)) of that partition id.
struct RangeDigit {
  const int64_t *keys;
  uint64_t flip, mn;
  int rshift, shift;
  uint32_t mask;
  CYLON_DIGIT_COMMON
  __device__ __forceinline__ uint32_t of_key(int64_t k) const {
    return (uint32_t)((((uint64_t)k ^ flip) - mn) >> (rshift + shift)) & mask;
  }
  __device__ __forceinline__ uint32_t operator()(int64_t i) const { return of_key(keys[i]); }
};

template <class Digit>
__global__ __launch_bounds__(kRPThreads) void k_rp_hist(Digit digit0, int64_t n, uint32_t nbuckets,
                                                        int64_t rows_per_block, int64_t nblocks,
                                                        int64_t *__restrict__ bh) {
  Digit digit = digit0;
  digit.init();
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

// Tile schedule of the XCD-tile passes: per-tile bucket offsets and one ticket per XCD.
struct TileSched {
  const uint32_t *xt_off;        // [tile][nbuckets] output row of the tile's first row of each bucket
  unsigned int *xt_ticket;       // [8] next tile of each XCD's contiguous chunk
  int64_t xt_tiles;              // tiles of the pass
  // slot mode (k_rows_pass<..., SLOT>, the histogram-free passes of a join partition): the input
  // is a list of row segments [ss[g], se[g]); a tile never straddles a segment, and digit d of
  // segment g goes to output slot (g >> sl_gshift) * nbuckets * sl_B + d * sl_B + (g & sl_gmask)
  // of sl_slot rows (claimed with one atomic per (tile, digit)); a run that does not fit goes to
  // the trash rows after the last slot and raises sl_overflow (the caller repartitions exactly).
  // XCD x (blockIdx % 8) owns segments [x S / 8, (x + 1) S / 8).
  //   first pass over a table: S = 8 chunks of n / 8 rows, slot = g * nb + d (one slot per
  //     (XCD, bucket): every slot is filled from ONE XCD's L2, and XCD-major cursors keep each
  //     XCD's claim atomics on cache lines of its own);
  //   second pass: S = 8 * nb1 slots of that pass (or nb1 exact buckets), slot = (g >> 3) * nb + d.
  const uint32_t *sl_tpre = nullptr;  // [S + 1] first tile of each segment (exclusive scan)
  const uint32_t *sl_ss = nullptr;    // [S] first row of each segment
  const uint32_t *sl_se = nullptr;    // [S] end row of each segment
  unsigned int *sl_cursor = nullptr;  // [nslots] rows claimed in each output slot
  unsigned int *sl_overflow = nullptr;
  int64_t sl_slot = 0;                // rows per output slot
  int64_t sl_nslots = 0;              // output slots (the trash rows start at sl_nslots * sl_slot)
  int sl_nseg = 0;                    // S <= kSlotMaxSeg
  int sl_gshift = 0, sl_gmask = 0, sl_B = 1;
  // look-back sort passes (k_rows_pass_lean<..., LBM>, see "look-back sort passes" below)
  const uint32_t *lb_plan = nullptr;  // in: chunk rows / tiles / bases of this pass (LBM & 2)
  uint32_t *lb_state = nullptr;       // in: [tile][nb] flag | value + 1 words, zeroed
  unsigned int *lb_err = nullptr;     // in: set when a look-back wait timed out
  uint32_t *lb_gcnt = nullptr;        // out: [block][8][nbn] (chunk, next digit) counts (LBM & 1)
  int lb_xshift = 0;                  // out: next pass's chunk = this pass's digit >> lb_xshift
};
constexpr int kSlotMaxSeg = 4096;

// ---- look-back sort passes (LSD sort of 1-2 all-8-byte columns; CYLON_SORT_LOOKBACK=0 disables)
// The exact XT pass needs every tile's digit counts before it starts (k_rp_hist_tiles over the
// previous pass's next-digit array + k_ts_* scans: ~1 ms, and writing that 2-byte array ~2 ms, of
// every 2B-row pass).  Here instead:
//   * the input is split into 8 chunks by the top 3 bits of the PREVIOUS pass's digit (contiguous:
//     that pass left the rows in that order), chunk x claimed tile by tile in order by XCD x;
//   * the previous pass counted, per (chunk, this pass's digit), the rows it stored (LDS counters,
//     flushed to per-block global rows) -> per-(chunk, digit) output bases (k_lb_plan);
//   * inside a chunk a tile's offset is the sum of its predecessors' digit counts, found by a
//     decoupled look-back: each tile publishes its counts (AGGREGATE) right after ranking, then walks
//     back over its predecessors' words until an INCLUSIVE prefix, and publishes its own.
// A word is 0 (not yet), value + 1 (aggregate) or 2^31 | value + 1 (inclusive prefix): flag and
// value travel in one 32-bit agent-scope atomic store / load, so no fence orders them.  Tiles are
// claimed in order per chunk, so a tile waits only on tiles already claimed by running blocks; a
// wait that exceeds kLbSpinLimit polls (never expected) sets lb_err and the sort falls back.
constexpr int kLbChunks = 8, kLbMaxBuckets = 512;
// plan[kLbLocal] = 1: chunk x runs only on XCD x and the look-back words are stored without
// write-through, so they stay in that XCD's L2 where its CUs' L1-bypassing loads find them (a
// round trip to L2 instead of HBM; 2B-row sort 92.8 -> 83.8 ms, profiles/r04/sort_lookback_ab.txt);
// 0: any XCD takes a chunk's tiles once its own are done and the words are written through.  The
// plan chooses local when no chunk exceeds 1.5x the mean.
constexpr int kLbCnt = 0, kLbC = kLbChunks * kLbMaxBuckets, kLbTP = kLbC + 16, kLbLocal = kLbTP + 12,
              kLbBase = kLbTP + 16,
              kLbTickets = kLbBase + kLbChunks * kLbMaxBuckets, kLbPlanWords = kLbTickets + 16;
constexpr int kLbSpinLimit = 1 << 20, kLbWindow = 4;

// XCD-tile mode.  Histogram mode gives each block a contiguous chunk of rows, so the tiles of
// one block write a bucket's consecutive runs ~34 us apart and the partial 128-B line at every
// run boundary has left the XCD's 4 MB L2 before the next tile completes it (~20 % extra HBM
// bytes, profiles/r03/pmc_join_1B_dma_vs_regstage.txt).  Here the tiles are split into 8
// contiguous chunks, one per XCD, and the XCD's CUs claim its tiles IN ORDER from a per-XCD
// ticket: at any moment an XCD's 32 CUs hold ~32 consecutive tiles, whose runs of each bucket
// are adjacent in the output and are written within a few us of each other into the same L2.
// Offsets are exact per tile (k_rp_hist_tiles + k_ts_*), so which CU takes a tile changes only
// speed; a block whose own chunk is exhausted takes tiles from the other chunks.
// slot mode: input bucket of tile t (tp: LDS copy of sl_tpre; the last bucket whose first tile <= t)
__device__ __forceinline__ int sl_segment(const uint32_t *tp, int nb1, int64_t t) {
  int lo = 0, hi = nb1 - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if ((int64_t)tp[mid] <= t) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// first row of the next tile this block processes, or n_rows when every chunk is exhausted
__device__ __forceinline__ int64_t xt_claim(const TileSched &lb, int home, int64_t tile_rows, int64_t n_rows) {
  for (int k = 0; k < kXcds; ++k) {
    const int x = (home + k) & (kXcds - 1);
    const int64_t lo = lb.xt_tiles * x / kXcds, hi = lb.xt_tiles * (x + 1) / kXcds;
    if (lo >= hi) continue;
    const int64_t j = (int64_t)atomicAdd(&lb.xt_ticket[x], 1u);
    if (lo + j < hi) return (lo + j) * tile_rows;
  }
  return n_rows;
}

// look-back passes: first row of the next tile of chunk home (else of another chunk), or n_rows
__device__ __forceinline__ int64_t lb_claim(const TileSched &lb, const uint32_t *sC, const uint32_t *sTP, int home,
                                            int64_t tile_rows, int64_t n_rows) {
  const bool local = sTP[kLbChunks + 1] != 0;  // s_TP[9]: the plan's local flag
  for (int k = 0; k < (local ? 1 : kXcds); ++k) {
    const int x = (home + k) & (kXcds - 1);
    const uint32_t T = sTP[x + 1] - sTP[x];
    if (T == 0) continue;
    const uint32_t j = atomicAdd(&lb.xt_ticket[x], 1u);
    if (j < T) return (int64_t)sC[x] + (int64_t)j * tile_rows;
  }
  return n_rows;
}

// look-back counting: add the packed 16-bit LDS counters to the block's global row g and clear them
// (every thread of the block calls it)
template <int THREADS>
__device__ __forceinline__ void lb_flush(uint32_t *lc, uint32_t *g, uint32_t lwords) {
  __syncthreads();
  for (uint32_t w = threadIdx.x; w < lwords; w += THREADS) {
    const uint32_t v = lc[w];
    if (v) {
      g[2 * w] += v & 0xffffu;
      g[2 * w + 1] += v >> 16;
    }
    lc[w] = 0;
  }
  __syncthreads();
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
__global__ __launch_bounds__(kHTThreads) void k_rp_hist_tiles(Digit digit0, int64_t n, uint32_t nb, int64_t ntiles,
                                                              uint16_t *__restrict__ th) {
  Digit digit = digit0;
  digit.init();
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

// off[t][p] = output row of tile t's first row of bucket p.  extra (optional, gapped layouts of the
// planned shuffle): rows of free space placed before bucket p, so a bucket can be followed by a
// receive region of the exchange (ops/shuffle.cpp planned_shuffle).
__global__ void k_ts_offsets(const uint16_t *__restrict__ th, const uint32_t *__restrict__ cpre,
                             const uint32_t *__restrict__ bbase, uint32_t nb, int64_t ntiles,
                             uint32_t *__restrict__ off, const uint32_t *__restrict__ extra) {
  const int64_t c = blockIdx.x, t0 = c * kTsChunk, t1 = t0 + kTsChunk < ntiles ? t0 + kTsChunk : ntiles;
  const uint32_t p = threadIdx.x;
  if (p >= nb) return;
  uint32_t acc = cpre[c * nb + p] + bbase[p] + (extra != nullptr ? extra[p] : 0u);
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

// RANK: kRankBallot (stable wave64 ballot match), kRankBlockAtomic (one LDS atomic per row
// on block-wide counters: unstable), kRankWaveAtomic (LDS atomics on the wave's own packed
// 16-bit counters: stable exactly when one instruction's same-address atomics return in lane
// order -- tools/lds_atomic_order.hip measures that on the device).
// XT: XCD-tile schedule (tiles claimed in order per XCD, exact per-tile bucket offsets in lb).
// SLOT: slot mode (TileSched): tiles of one input bucket each, per-(tile, digit) slot claims.
template <class Digit, bool W8, int THREADS, int RANK, bool XT = false, bool SLOT = false>
__global__ __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(4))) void k_rows_pass(
    Digit digit0, int nbits, uint32_t nbuckets, ColSet cols, int64_t n, int64_t rows_per_block, int64_t nblocks,
    const int64_t *__restrict__ bh_scan, TileSched lb) {
  constexpr int WAVES = THREADS / kWave;
  constexpr int TILE = THREADS * kRPItems;
  constexpr int BPT = (kRPMaxBuckets + THREADS - 1) / THREADS;  // buckets per thread in the offset scan
  Digit digit = digit0;
  digit.init();
  bool narrow_bad = false;  // PartDigitN: a key outside the uint32 offset range
  static_assert(WAVES * kRPMaxBuckets * 2 + TILE * 4 <= TILE * 8, "ranking scratch must fit the stage");
  constexpr bool TICKET = XT || SLOT;  // tiles claimed one by one (not a contiguous chunk per block)
  static_assert(!(XT && SLOT), "one tile schedule");
  static_assert(!SLOT || RANK == kRankBlockAtomic, "slot mode ranks with block atomics (counts in bcnt)");
  const int xhome = TICKET ? xcc_id() : 0;
  __shared__ int64_t running[kRPMaxBuckets];
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
  __shared__ int64_t s_next;  // XT: first row of the next claimed tile
  // SLOT: end row / input bucket of the current ([par]) and the next ([par ^ 1]) tile, in LDS
  // rather than registers (the classic pass already runs at the 128-VGPR budget)
  __shared__ int64_t s_tend[2], s_tr0[2];
  __shared__ int s_tb[2];
  int par = 0;
  bool order_bad = false;
  // SLOT: the segments' first tiles / first rows / end rows in LDS; tiles are dealt statically --
  // XCD x (= blockIdx % 8, the dispatcher's round robin) owns the tiles of its segments, its j-th
  // block takes every nblk-th of them -- so taking the next tile is a few LDS reads (no atomic, no
  // global load on the barrier path), and an XCD's CUs work on adjacent tiles of the same segment.
  __shared__ uint32_t tp[SLOT ? kSlotMaxSeg : 1], sss[SLOT ? kSlotMaxSeg : 1], sse[SLOT ? kSlotMaxSeg : 1];
  __shared__ int64_t s_tix, s_thi;  // SLOT (thread 0): this block's next tile index, its XCD's end
  auto sl_take = [&](int slot) {    // thread 0: take the next tile, resolve its rows and slot base
    const int64_t t = s_tix;
    if (t >= s_thi) {  // none left (slot-mode inputs may have rows beyond n: a sentinel, not n; row
                       // arithmetic on it must not overflow)
      s_tr0[slot] = INT64_MAX / 4;
      s_tend[slot] = 0;
      s_tb[slot] = 0;
      return;
    }
    s_tix = t + ((int64_t)gridDim.x - (blockIdx.x & (kXcds - 1)) + kXcds - 1) / kXcds;
    const int g = sl_segment(tp, lb.sl_nseg, t);
    const int64_t gend = (int64_t)sse[g];
    const int64_t r0 = (int64_t)sss[g] + (t - (int64_t)tp[g]) * TILE;
    s_tr0[slot] = r0;
    s_tend[slot] = r0 + TILE < gend ? r0 + TILE : gend;
    // digit d of this tile goes to slot s_tb + d * sl_B
    s_tb[slot] = (g >> lb.sl_gshift) * (int)nbuckets * lb.sl_B + (g & lb.sl_gmask);
  };

  const int64_t b = blockIdx.x;
  int64_t begin, end;
  if (SLOT) {
    for (int i = threadIdx.x; i < lb.sl_nseg; i += THREADS) {
      tp[i] = lb.sl_tpre[i];
      sss[i] = lb.sl_ss[i];
      sse[i] = lb.sl_se[i];
    }
    if (threadIdx.x == 0) {
      const int x = blockIdx.x & (kXcds - 1);
      const int g0 = lb.sl_nseg * x / kXcds, g1 = lb.sl_nseg * (x + 1) / kXcds;
      s_tix = (int64_t)lb.sl_tpre[g0] + blockIdx.x / kXcds;
      s_thi = lb.sl_tpre[g1];
    }
    __syncthreads();
    if (threadIdx.x == 0) {  // the first two tiles; later claims run at the end of a tile, two ahead
      sl_take(0);
      sl_take(1);
    }
    __syncthreads();
    begin = s_tr0[0];
    end = INT64_MAX / 4;  // the loop runs until sl_take reports no tile
  } else if (TICKET) {
    if (threadIdx.x == 0) s_next = xt_claim(lb, xhome, TILE, n);
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

  // keys of the current tile (column 0); narrowed digits hold the uint32 offset from the load on
  // (8 fewer VGPRs in a kernel that spills at the 128-VGPR limit)
  using KVT = typename std::conditional<Digit::kNarrow, uint32_t, uint64_t>::type;
  KVT kv[kRPItems];
  auto load_key = [&](int64_t i) -> KVT {
    const uint64_t raw = digit.key_at(i);
    if constexpr (Digit::kNarrow) {
      narrow_bad |= digit.too_wide(raw);
      return (KVT)digit.narrow(raw);
    } else {
      return (KVT)raw;
    }
  };
#pragma unroll
  for (int k = 0; k < kRPItems; ++k) {
    const int64_t i = begin + wrow + k * kWave + lane;
    if (i < (SLOT ? s_tend[0] : end)) kv[k] = load_key(i);
  }
  for (int64_t tile = begin, next = 0; tile < end; tile = next) {
    next = tile + TILE;
    const int cnt = SLOT ? (int)(s_tend[par] - tile) : (int)((end - tile) < TILE ? (end - tile) : TILE);
    // XT: this tile's bucket offsets (consumed after the slot phase; the load overlaps the ranking)
    const uint32_t xoff = XT && threadIdx.x < nbuckets ? lb.xt_off[(tile / TILE) * nbuckets + threadIdx.x] : 0u;
    uint32_t pl[kRPItems];  // digit, then (in-wave rank << 16) | digit, then sorted slot; ~0 = inactive
#pragma unroll
    for (int k = 0; k < kRPItems; ++k) {
      const bool act = wrow + k * kWave + lane < cnt;
      if constexpr (Digit::kNarrow) pl[k] = act ? digit.of_offset(kv[k]) : 0xffffffffu;
      else pl[k] = act ? digit.of_key((int64_t)kv[k]) : 0xffffffffu;
    }
    if (STABLE) {
      for (uint32_t q = threadIdx.x; q < WAVES * nbuckets; q += blockDim.x) wcnt[q] = 0;
    } else {
      for (uint32_t q = threadIdx.x; q < nbuckets; q += blockDim.x) bcnt[q] = 0;
    }
    __syncthreads();  // also orders the previous tile's stage reads before the counters reuse it
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
    __syncthreads();
    // SLOT: claim this tile's run in every output slot it feeds as soon as the counts exist (the
    // atomics' latency hides behind the scan and the slot phase)
    uint32_t sl_c = 0, sl_base = 0;
    if (SLOT && threadIdx.x < nbuckets) {
      sl_c = STABLE ? 0u : bcnt[threadIdx.x];
      if (sl_c) sl_base = atomicAdd(&lb.sl_cursor[(int64_t)s_tb[par] + (int64_t)threadIdx.x * lb.sl_B], sl_c);
    }
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
      const uint32_t ex = rp_block_exscan<WAVES>(total, wsum);
#pragma unroll
      for (int i = 0; i < BPT; ++i) {
        const uint32_t p = threadIdx.x * BPT + i;
        if (p < nbuckets) toff[p] = ex + loc[i];
      }
      if (threadIdx.x == THREADS - 1) toff[nbuckets] = ex + total;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kRPItems; ++k) {
      if (pl[k] == 0xffffffffu) continue;
      const uint32_t p = pl[k] & 0xffffu;
      const uint32_t pos = toff[p] + (STABLE ? (uint32_t)wcnt[wave * nbuckets + p] : 0u) + (pl[k] >> 16);
      sdig[pos] = (p << 16) | (uint32_t)(wrow + k * kWave + lane);
      pl[k] = pos;
    }
    if (XT && threadIdx.x < nbuckets) running[threadIdx.x] = xoff;
    if (SLOT && threadIdx.x < nbuckets) {
      const bool fits = (int64_t)sl_base + sl_c <= lb.sl_slot;
      if (sl_c && !fits) atomicOr(lb.sl_overflow, 1u);
      running[threadIdx.x] = fits ? ((int64_t)s_tb[par] + (int64_t)threadIdx.x * lb.sl_B) * lb.sl_slot + sl_base
                                  : lb.sl_nslots * lb.sl_slot;  // the trash rows
    }
    __syncthreads();
    // destination of sorted slot j = threadIdx.x + q * THREADS.  SLOT: packed as digit << 16 | offset
    // in its run and completed from running[] (LDS) at each store -- 8 VGPRs instead of 16 in the
    // instance that also carries the slot bookkeeping (the trick of the lean kernel)
    // (SLOT could pack them as digit << 16 | offset and complete them from running[] at each store --
    // 8 fewer VGPRs -- but the dependent LDS read per store measured slower: r04m, 17.3 vs 14.3 ms)
    // SLOT: destinations as uint32 rows (slot layouts stay below 2^32 rows, radix_slot_eligible):
    // 8 fewer VGPRs in a kernel that runs at the 128-VGPR limit
    constexpr bool PACKDST = false;
    using DstT = typename std::conditional<SLOT, uint32_t, int64_t>::type;
    DstT dst[kRPItems];
#define RP_DEST(q) \
  ((SLOT && PACKDST) ? running[(uint32_t)dst[q] >> 16] + (int64_t)((uint32_t)dst[q] & 0xffffu) : (int64_t)dst[q])
#pragma unroll
    for (int q = 0; q < kRPItems; ++q) {
      const int j = threadIdx.x + q * THREADS;
      if (j < cnt) {
        const uint32_t e = sdig[j], p = e >> 16;
        if constexpr (SLOT && PACKDST) dst[q] = (p << 16) | (uint32_t)(j - (int)toff[p]);
        else dst[q] = (DstT)(running[p] + (j - (int64_t)toff[p]));
        if (cols.check_order && j > 0) {  // same bucket as the previous slot: input order kept?
          const uint32_t f = sdig[j - 1];
          order_bad |= (f >> 16) == p && f > e;
        }
      }
    }
    __syncthreads();  // counters / digits dead: the union becomes the column stage
    // load column c+1 while column c streams out of the stage
    uint64_t v[kRPItems];
#pragma unroll
    for (int k = 0; k < kRPItems; ++k) v[k] = kv[k];
#pragma unroll 1
    for (int c = 0; c < cols.n; ++c) {  // column fields fetched once per column (scalar loads)
      const int w = cols.width[c];
      uint8_t *out = cols.out[c];
      const uint64_t x = c == 0 ? cols.key_xor : 0ull;
      if (TICKET && c + 1 == cols.n && threadIdx.x == 0) {
        if (!SLOT) s_next = xt_claim(lb, xhome, TILE, n);
      }
      const bool n4 = Digit::kNarrow && c == 0;  // column 0 as the uint32 offset
      if (n4) {  // (v holds the narrowed offsets already)
#pragma unroll
        for (int k = 0; k < kRPItems; ++k)
          if (pl[k] != 0xffffffffu) stw<false>(st, pl[k], 4, v[k] & 0xffffffffull);
      } else {
#pragma unroll
        for (int k = 0; k < kRPItems; ++k)
          if (pl[k] != 0xffffffffu) stw<W8>(st, pl[k], w, v[k] ^ x);
      }
      __syncthreads();
      if (TICKET && c + 1 == cols.n) next = SLOT ? s_tr0[par ^ 1] : s_next;
      if (c + 1 < cols.n) {  // prefetch column c+1 of this tile
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
          if (i < (SLOT ? s_tend[par ^ 1] : end)) kv[k] = load_key(i);
        }
      }
      if (kNdDigit<Digit> && c == 0 && cols.nd_out != nullptr) {  // sorts, stable hash partitions
#pragma unroll
        for (int q = 0; q < kRPItems; ++q) {
          const int j = threadIdx.x + q * THREADS;
          if (j < cnt) {
            const uint64_t kv0 = ldw<W8>(st, j, w);
            const int64_t o = RP_DEST(q);
            stw<W8>(out, o, w, kv0);
            if constexpr (kNdDigit<Digit>)
              cols.nd_out[o] = (uint16_t)digit.next_of(kv0, cols.nd_shift, cols.nd_mask, cols.nd_sub);
          }
        }
      } else if (n4) {
#pragma unroll
        for (int q = 0; q < kRPItems; ++q) {
          const int j = threadIdx.x + q * THREADS;
          if (j < cnt) stw<false>(out, RP_DEST(q), 4, ldw<false>(st, j, 4));
        }
      } else {
#pragma unroll
        for (int q = 0; q < kRPItems; ++q) {
          const int j = threadIdx.x + q * THREADS;
          if (j < cnt) stw<W8>(out, RP_DEST(q), w, ldw<W8>(st, j, w));
        }
      }
      __syncthreads();
    }
#undef RP_DEST
    if (!TICKET)
      for (uint32_t p = threadIdx.x; p < nbuckets; p += blockDim.x) running[p] += toff[p + 1] - toff[p];
    if (SLOT) {
      par ^= 1;
      // the tile after the next one, into the slot of the tile just finished: claimed here, where
      // only the next tile's keys are live (its rows are read two tiles' barriers later)
      if (threadIdx.x == 0) sl_take(par ^ 1);
    }
  }
  if (order_bad) atomicOr(cols.order_bad, 1);
  if (Digit::kNarrow && narrow_bad) digit.report_bad();
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
// LBM (sorts, XT only): bit 1 = offsets by look-back (lb_plan / lb_state), bit 0 = count the
// (chunk, next digit) pairs for the next look-back pass (lb_gcnt); both limit digits to 9 bits.
template <class Digit, bool W8, int RANK, bool XT = false, int LBM = 0>
__global__ __launch_bounds__(kRPThreads) __attribute__((amdgpu_waves_per_eu(8))) void k_rows_pass_lean(
    Digit digit, int nbits, uint32_t nbuckets, ColSet cols, int64_t n, int64_t rows_per_block, int64_t nblocks,
    const int64_t *__restrict__ bh_scan, TileSched lb) {
  constexpr int THREADS = kRPThreads, WAVES = THREADS / kWave, TILE = THREADS * kRPItems;
  constexpr bool LBIN = (LBM & 2) != 0, CNT = (LBM & 1) != 0;
  static_assert(LBM == 0 || (XT && (std::is_same<Digit, ImageDigit>::value || std::is_same<Digit, PartDigit>::value)),
                "look-back passes are XT sort / hash-partition passes");
  constexpr int MAXB = LBM ? kLbMaxBuckets : kRPMaxBuckets;
  constexpr int BPT = (MAXB + THREADS - 1) / THREADS;
  static_assert(WAVES * MAXB * 2 + TILE * 4 <= TILE * 8, "ranking scratch must fit the stage");
  __shared__ int64_t running[MAXB];
  __shared__ uint32_t toff[MAXB + 1];
  __shared__ uint64_t ustage[TILE];  // column stage | {wcnt[WAVES][nb] u16 or bcnt[nb] u32, sdig[TILE] u16}
  __shared__ uint32_t wsum[WAVES];
  // look-back: chunk first rows / first tiles; counting: packed 16-bit (chunk, next digit) counters
  __shared__ uint32_t s_C[LBIN ? kLbChunks + 1 : 1], s_TP[LBIN ? kLbChunks + 2 : 1];  // s_TP[9] = local flag
  __shared__ uint32_t lcnt[CNT ? kLbChunks * kLbMaxBuckets / 2 : 1];
  constexpr bool STABLE = RANK != kRankBlockAtomic;
  uint16_t *wcnt = reinterpret_cast<uint16_t *>(ustage);
  uint32_t *bcnt = reinterpret_cast<uint32_t *>(ustage);
  uint32_t *sdig = reinterpret_cast<uint32_t *>(wcnt + WAVES * MAXB);  // digit << 16 | input row
  uint8_t *st = reinterpret_cast<uint8_t *>(ustage);
  __shared__ int64_t s_next;  // XT: first row of the next claimed tile
  bool order_bad = false;
  (void)nbits;
  constexpr bool TICKET = XT;
  const int xhome = XT ? xcc_id() : 0;
  const uint32_t nbn = cols.nd_mask + 1u;               // counting: next pass's buckets
  const uint32_t lwords = CNT ? kLbChunks * nbn / 2 : 0;  // counting: LDS words in use
  int since_flush = 0;

  const int64_t b = blockIdx.x;
  int64_t begin, end;
  if (CNT)
    for (uint32_t w = threadIdx.x; w < lwords; w += THREADS) lcnt[w] = 0;
  if (LBIN && threadIdx.x <= kLbChunks) {
    s_C[threadIdx.x] = lb.lb_plan[kLbC + threadIdx.x];
    s_TP[threadIdx.x] = lb.lb_plan[kLbTP + threadIdx.x];
  }
  if (LBIN && threadIdx.x == kLbChunks + 1) s_TP[kLbChunks + 1] = lb.lb_plan[kLbLocal];
  if (TICKET) {
    if (LBIN) __syncthreads();
    if (threadIdx.x == 0) s_next = LBIN ? lb_claim(lb, s_C, s_TP, xhome, TILE, n) : xt_claim(lb, xhome, TILE, n);
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
    // look-back: the tile's chunk (uniform) and its index in the chunk
    int cx = 0;
    if (LBIN)
      while (cx + 1 < kLbChunks && (int64_t)s_C[cx + 1] <= tile) ++cx;
    const int64_t ck = LBIN ? (tile - (int64_t)s_C[cx]) / TILE : 0;
    const int64_t tend = LBIN ? (int64_t)s_C[cx + 1] : end;
    const int cnt = (int)((tend - tile) < TILE ? (tend - tile) : TILE);
    // per-thread constants are recomputed every tile from an opaque copy of the thread id:
    // hoisted out of the tile loop they outlive the 64-VGPR budget and spill
    int tx = (int)threadIdx.x;
    asm volatile("" : "+v"(tx));
    const int lane = tx & (kWave - 1);
    // XT: this tile's bucket offsets (stored to running[] after the slot phase)
    const uint32_t xoff = XT && !LBIN && (uint32_t)tx < nbuckets ? lb.xt_off[(tile / TILE) * nbuckets + tx] : 0u;
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
    const int64_t lgid = LBIN ? (int64_t)s_TP[cx] + ck : 0;  // look-back: the tile's state row
    if (LBIN && (uint32_t)tx < nbuckets) {  // publish this tile's counts (the chunk's first: its prefix)
      const uint32_t v = (ck == 0 ? 0x80000000u : 0u) | (toff[tx + 1] - toff[tx] + 1u);
      if (s_TP[kLbChunks + 1])
        __hip_atomic_store(&lb.lb_state[lgid * nbuckets + tx], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      else
        __hip_atomic_store(&lb.lb_state[lgid * nbuckets + tx], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
#pragma unroll
    for (int k = 0; k < kRPItems; ++k) {
      if (pl[k] == 0xffffffffu) continue;
      const uint32_t p = pl[k] & 0xffffu;
      const uint32_t pos = toff[p] + (STABLE ? (uint32_t)wcnt[wave * nbuckets + p] : 0u) + (pl[k] >> 16);
      sdig[pos] = (p << 16) | (uint32_t)(wrow + k * kWave + lane);
      pl[k] = pos;
    }
    if (XT && !LBIN && (uint32_t)tx < nbuckets) running[tx] = xoff;
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
      // look-back passes claim their next tile only once this one is written (below): a tile claimed
      // ahead would publish its counts a whole tile later and stall its successors' look-back
      if (TICKET && !LBIN && c + 1 == cols.n && tx == 0) s_next = xt_claim(lb, xhome, TILE, n);
#pragma unroll
      for (int k = 0; k < kRPItems; ++k)
        if (pl[k] != 0xffffffffu) stw<W8>(st, pl[k], w, v[k] ^ x);
      __syncthreads();
      if (TICKET && !LBIN && c + 1 == cols.n) next = s_next;
      // look back over the chunk's earlier tiles only now that the keys are staged: the predecessors
      // have had this tile's ranking AND staging time to publish their prefixes (fewer round trips)
      if (LBIN && c == 0 && (uint32_t)tx < nbuckets) {
        const uint32_t own = toff[tx + 1] - toff[tx];
        uint32_t excl = 0;
        if (ck > 0) {
          // windowed walk: the next kLbWindow predecessors' words are loaded together (one round trip
          // per window instead of per tile; a walk is a few tiles long: those claimed just before)
          const int64_t lo = (int64_t)s_TP[cx];  // the chunk's first tile (always an inclusive prefix)
          int64_t j = lgid - 1;
          for (int spin = 0;;) {
            uint32_t w[kLbWindow];
#pragma unroll
            for (int i = 0; i < kLbWindow; ++i)
              w[i] = j - i >= lo ? __hip_atomic_load(&lb.lb_state[(j - i) * nbuckets + tx], __ATOMIC_RELAXED,
                                                     __HIP_MEMORY_SCOPE_AGENT)
                                 : 0u;
            int used = 0;
            bool done = false;
#pragma unroll
            for (int i = 0; i < kLbWindow; ++i) {
              if (done || used < i || w[i] == 0u) continue;  // stop at the first word not yet published
              excl += (w[i] & 0x7fffffffu) - 1u;
              used = i + 1;
              done = (w[i] & 0x80000000u) != 0u;
            }
            if (done) break;
            j -= used;
            if (used == 0) {  // the nearest predecessor has not published yet
              __builtin_amdgcn_s_sleep(1);
              // give up after kLbSpinLimit polls, or at once after any other wait gave up (the result
              // is discarded then, so the grid only has to drain)
              if (++spin > kLbSpinLimit ||
                  ((spin & 255) == 0 && __hip_atomic_load(lb.lb_err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT))) {
                atomicOr(lb.lb_err, 1u);
                break;
              }
            }
          }
          if (s_TP[kLbChunks + 1])
            __hip_atomic_store(&lb.lb_state[lgid * nbuckets + tx], 0x80000000u | (excl + own + 1u), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_WORKGROUP);
          else
            __hip_atomic_store(&lb.lb_state[lgid * nbuckets + tx], 0x80000000u | (excl + own + 1u), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
        }
        running[tx] = (int64_t)lb.lb_plan[kLbBase + cx * nbuckets + tx] + excl;
      }
      if (LBIN && c == 0) __syncthreads();
      if (CNT && c == 0) {  // count (chunk of the next pass, next digit) as the keys are stored
        const int xsh = lb.lb_xshift;
#pragma unroll
        for (int q = 0; q < kRPItems; ++q) {
          const int j = tx + q * THREADS;
          if (j < cnt) {
            const uint32_t p = dp[q] >> 16;
            const int64_t o = running[p] + (int64_t)(dp[q] & 0xffffu);
            const uint64_t kv0 = ldw<W8>(st, j, w);
            stw<W8>(out, o, w, kv0);
            uint32_t nd = 0;
            if constexpr (LBM != 0) nd = digit.next_of(kv0, cols.nd_shift, cols.nd_mask, cols.nd_sub);
            const uint32_t cell = (p >> xsh) * nbn + nd;
            atomicAdd(&lcnt[cell >> 1], 1u << ((cell & 1u) << 4));
          }
        }
      } else if (kNdDigit<Digit> && c == 0 && cols.nd_out != nullptr) {  // sorts, stable hash partitions
#pragma unroll
        for (int q = 0; q < kRPItems; ++q) {
          const int j = tx + q * THREADS;
          if (j < cnt) {
            const int64_t o = running[dp[q] >> 16] + (int64_t)(dp[q] & 0xffffu);
            const uint64_t kv0 = ldw<W8>(st, j, w);
            stw<W8>(out, o, w, kv0);
            if constexpr (kNdDigit<Digit>)
              cols.nd_out[o] = (uint16_t)digit.next_of(kv0, cols.nd_shift, cols.nd_mask, cols.nd_sub);
          }
        }
      } else {
#pragma unroll
        for (int q = 0; q < kRPItems; ++q) {
          const int j = tx + q * THREADS;
          if (j < cnt) stw<W8>(out, running[dp[q] >> 16] + (int64_t)(dp[q] & 0xffffu), w, ldw<W8>(st, j, w));
        }
      }
      __syncthreads();
    }
    if (!TICKET)
      for (uint32_t p = tx; p < nbuckets; p += THREADS) running[p] += toff[p + 1] - toff[p];
    if (LBIN) {  // (the column loop ended with a barrier)
      if (tx == 0) s_next = lb_claim(lb, s_C, s_TP, xhome, TILE, n);
      __syncthreads();
      next = s_next;
    }
    if (CNT && ++since_flush == 7) {  // 7 tiles x 8192 rows fit a 16-bit counter
      lb_flush<THREADS>(lcnt, lb.lb_gcnt + (int64_t)blockIdx.x * (2 * lwords), lwords);
      since_flush = 0;
    }
  }
  if (CNT && since_flush > 0) lb_flush<THREADS>(lcnt, lb.lb_gcnt + (int64_t)blockIdx.x * (2 * lwords), lwords);
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
// (profiles/rows_pass_experiments_r02.txt).
static int rp_threads(int ncols, bool cheap_rank) { return ncols <= 2 && !cheap_rank ? 512 : 1024; }

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
// of the process.  rp_set_ranking (tests) forces one.
static std::atomic<int> g_lane_ok[64];  // 0 unknown, 1 ok, 2 not ok

static int current_device() {
  int d = 0;
  HIP_CHECK(hipGetDevice(&d));
  return d & 63;
}

bool lds_lane_order_ok(void *stream) {
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

// tests: 0 = forget every device's ranking verdict (re-probe on next use), 1 = wave-atomic, 2 = ballots
void rp_set_ranking(int mode) {
  for (auto &v : g_lane_ok) v.store(mode == 1 ? 1 : (mode == 2 ? 2 : 0));
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
int *rp_order_flag() { return order_flag(); }
void rp_note_order_violation(void *stream) {
  HIP_CHECK(hipMemsetAsync(order_flag(), 0, sizeof(int), as_stream(stream)));
  g_lane_ok[current_device()].store(2);
}
static bool rp_wave_atomic(hipStream_t s) { return lds_lane_order_ok(reinterpret_cast<void *>(s)); }

// Pass kernel: "lean" (two register-lean blocks per CU) or "classic" (one block per CU with
// register software pipelining).  Measured on one box, same tree (profiles/r03/lean_pass_ab.txt):
// lean wins for passes that move 1-2 columns (2B-row sort 107.5 -> 99.2 ms, 1B group-by 27.6 ->
// 25.0 ms; its two blocks overlap each other's ranking and barriers) and loses for the 4-column
// join passes (17.9 -> 20.0 ms per pass: without the classic kernel's next-column prefetch each
// column's load latency is exposed).
static bool rp_lean(int ncols) { return ncols <= 2; }

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
// The per-block-chunk schedule (histogram mode) remains for 512-thread ballot passes and n >= 2^32.
static bool rp_xt() { return true; }

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

template <class Digit, int THREADS, int RANK>
static void rows_pass_kernel(bool w8, const RPGeometry &g, hipStream_t s, const Digit &dg, int digit_bits, uint32_t nb,
                             const ColSet &cs, int64_t n, const int64_t *bh_scan, const TileSched &lb = TileSched{},
                             bool xt = false) {
  bool launched = false;
  if constexpr (THREADS == 1024) {
    if (xt) {
      if (w8)
        hipLaunchKernelGGL((k_rows_pass<Digit, true, THREADS, RANK, true>), dim3((unsigned)g.nblocks), dim3(THREADS), 0,
                           s, dg, digit_bits, nb, cs, n, g.rows_per_block, g.nblocks, bh_scan, lb);
      else
        hipLaunchKernelGGL((k_rows_pass<Digit, false, THREADS, RANK, true>), dim3((unsigned)g.nblocks), dim3(THREADS), 0,
                           s, dg, digit_bits, nb, cs, n, g.rows_per_block, g.nblocks, bh_scan, lb);
      launched = true;
    }
  }
  if (launched) {
  } else if (w8)
    hipLaunchKernelGGL((k_rows_pass<Digit, true, THREADS, RANK>), dim3((unsigned)g.nblocks), dim3(THREADS), 0, s, dg,
                       digit_bits, nb, cs, n, g.rows_per_block, g.nblocks, bh_scan, lb);
  else
    hipLaunchKernelGGL((k_rows_pass<Digit, false, THREADS, RANK>), dim3((unsigned)g.nblocks), dim3(THREADS), 0, s, dg,
                       digit_bits, nb, cs, n, g.rows_per_block, g.nblocks, bh_scan, lb);
}

template <class Digit, int RANK>
static void lean_kernel(bool w8, const RPGeometry &g, hipStream_t s, const Digit &dg, int digit_bits, uint32_t nb,
                        const ColSet &cs, int64_t n, const int64_t *bh_scan, const TileSched &lb, bool xt = false,
                        int lbm = 0) {
  if (lbm) {  // look-back sort passes: XT, all columns 8 bytes wide (checked by the caller)
    if constexpr ((std::is_same<Digit, ImageDigit>::value || std::is_same<Digit, PartDigit>::value) &&
                  RANK == kRankWaveAtomic) {
      const dim3 gr((unsigned)g.nblocks), bl(kRPThreads);
      if (lbm == 1)
        hipLaunchKernelGGL((k_rows_pass_lean<Digit, true, RANK, true, 1>), gr, bl, 0, s, dg, digit_bits, nb, cs, n,
                           g.rows_per_block, g.nblocks, bh_scan, lb);
      else if (lbm == 2)
        hipLaunchKernelGGL((k_rows_pass_lean<Digit, true, RANK, true, 2>), gr, bl, 0, s, dg, digit_bits, nb, cs, n,
                           g.rows_per_block, g.nblocks, bh_scan, lb);
      else
        hipLaunchKernelGGL((k_rows_pass_lean<Digit, true, RANK, true, 3>), gr, bl, 0, s, dg, digit_bits, nb, cs, n,
                           g.rows_per_block, g.nblocks, bh_scan, lb);
      return;
    }
    CYLON_THROW(Code::Invalid, "look-back pass: sort / partition digits with stable wave ranking only");
  }
  if (xt) {
    if (w8)
      hipLaunchKernelGGL((k_rows_pass_lean<Digit, true, RANK, true>), dim3((unsigned)g.nblocks), dim3(kRPThreads), 0, s,
                         dg, digit_bits, nb, cs, n, g.rows_per_block, g.nblocks, bh_scan, lb);
    else
      hipLaunchKernelGGL((k_rows_pass_lean<Digit, false, RANK, true>), dim3((unsigned)g.nblocks), dim3(kRPThreads), 0, s,
                         dg, digit_bits, nb, cs, n, g.rows_per_block, g.nblocks, bh_scan, lb);
    return;
  }
  if (w8)
    hipLaunchKernelGGL((k_rows_pass_lean<Digit, true, RANK>), dim3((unsigned)g.nblocks), dim3(kRPThreads), 0, s, dg,
                       digit_bits, nb, cs, n, g.rows_per_block, g.nblocks, bh_scan, lb);
  else
    hipLaunchKernelGGL((k_rows_pass_lean<Digit, false, RANK>), dim3((unsigned)g.nblocks), dim3(kRPThreads), 0, s, dg,
                       digit_bits, nb, cs, n, g.rows_per_block, g.nblocks, bh_scan, lb);
}

// ---- look-back sort passes, host side (see "look-back sort passes")
// cnt[c] += gcnt[b][c] over a slice of the blocks (grid: cells / 256 x kLbReduceSlices)
constexpr int kLbReduceSlices = 32;
__global__ __launch_bounds__(256) void k_lb_reduce(const uint32_t *__restrict__ gcnt, int64_t nblk, int cells,
                                                   uint32_t *__restrict__ cnt) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= cells) return;
  const int64_t b0 = nblk * blockIdx.y / kLbReduceSlices, b1 = nblk * (blockIdx.y + 1) / kLbReduceSlices;
  uint32_t acc = 0;
  for (int64_t b = b0; b < b1; ++b) acc += gcnt[b * cells + c];
  if (acc) atomicAdd(&cnt[c], acc);
}

// plan of a look-back pass from its (chunk, digit) counts: chunk first rows C, first tiles TP
// (tiles never straddle chunks) and bases[x][d] = rows of digits < d + rows of digit d in chunks < x
__global__ __launch_bounds__(kLbMaxBuckets) void k_lb_plan(uint32_t *__restrict__ plan, uint32_t nb) {
  __shared__ uint32_t wsum[kLbMaxBuckets / kWave];
  __shared__ uint32_t csz[kLbChunks];
  const uint32_t d = threadIdx.x;
  if (d < kLbChunks) csz[d] = 0;
  uint32_t c[kLbChunks], tot = 0;
#pragma unroll
  for (int x = 0; x < kLbChunks; ++x) {
    c[x] = d < nb ? plan[kLbCnt + x * nb + d] : 0u;
    tot += c[x];
  }
  __syncthreads();
  uint32_t run = rp_block_exscan<kLbMaxBuckets / kWave>(tot, wsum);
#pragma unroll
  for (int x = 0; x < kLbChunks; ++x) {
    if (d < nb) plan[kLbBase + x * nb + d] = run;
    run += c[x];
    if (c[x]) atomicAdd(&csz[x], c[x]);
  }
  __syncthreads();
  if (d == 0) {
    uint32_t r = 0, t = 0;
    for (int x = 0; x < kLbChunks; ++x) {
      plan[kLbC + x] = r;
      plan[kLbTP + x] = t;
      r += csz[x];
      t += (csz[x] + kRPTile - 1) / kRPTile;
    }
    plan[kLbC + kLbChunks] = r;
    plan[kLbTP + kLbChunks] = t;
    uint32_t mx = 0;
    for (int x = 0; x < kLbChunks; ++x) mx = csz[x] > mx ? csz[x] : mx;
    plan[kLbLocal] = (uint64_t)mx * kLbChunks * 2 <= (uint64_t)r * 3 ? 1u : 0u;
  }
}

// local look-back mode: every chunk's tiles were claimed (XCD x had blocks), else err |= 2
__global__ void k_lb_check(const uint32_t *__restrict__ plan, unsigned int *err) {
  const int x = threadIdx.x;
  if (x < kLbChunks && plan[kLbTickets + x] < plan[kLbTP + x + 1] - plan[kLbTP + x]) atomicOr(err, 2u);
}

static void lb_plan_next(const SortLbArgs *lba, int64_t nblk, uint32_t nbn, int64_t n, hipStream_t s) {
  const int cells = kLbChunks * (int)nbn;
  HIP_CHECK(hipMemsetAsync(lba->plan_out + kLbCnt, 0, sizeof(uint32_t) * cells, s));
  hipLaunchKernelGGL(k_lb_reduce, dim3((unsigned)((cells + 255) / 256), kLbReduceSlices), dim3(256), 0, s, lba->gcnt,
                     nblk, cells, lba->plan_out + kLbCnt);
  HIP_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_lb_plan, dim3(1), dim3(kLbMaxBuckets), 0, s, lba->plan_out, nbn);
  HIP_LAUNCH_CHECK();
  (void)n;
}

// stable = false (join partitions only) ranks rows with LDS atomics: rows of one
// bucket keep no particular order inside a tile's run.  Instantiated for PartDigit
// only; every other digit (sort, shuffle, range join) needs the stable order.
// column 0 of a pass input: the int64 key, or (narrowed join passes after the first) uint32 offsets
template <class Digit>
static bool key_column_ok(const Digit &dg, const uint8_t *const *in, const int *widths) {
  if constexpr (Digit::kNarrow)
    return in[0] == reinterpret_cast<const uint8_t *>(dg.keys) && widths[0] == (dg.kin4 ? 4 : 8);
  else
    return in[0] == reinterpret_cast<const uint8_t *>(dg.keys) && widths[0] == 8;
}

template <class Digit,
          bool CAN_UNSTABLE = std::is_same<Digit, PartDigit>::value || std::is_same<Digit, PartDigitN>::value>
static void rows_pass_launch(const Digit &dg, int64_t n, int digit_bits, const uint8_t *const *in, uint8_t *const *out,
                             const int *widths, int ncols, int64_t *ws, void *stream, uint64_t key_xor = 0,
                             bool stable = true, bool tiles_prescanned = false,
                             const uint32_t *bucket_extra = nullptr, const uint16_t *nd_in = nullptr,
                             uint16_t *nd_out = nullptr, int nd_shift = 0, uint32_t nd_mask = 0,
                             uint64_t nd_sub = 0, const SortLbArgs *lba = nullptr) {
  if (n == 0) return;
  CYLON_CHECK(digit_bits >= 1 && digit_bits <= kRJMaxDigitBits, Code::Invalid, "digit bits " << digit_bits);
  CYLON_CHECK(ncols >= 1 && ncols <= kMaxFusedCols, Code::Invalid, "bad column count " << ncols);
  CYLON_CHECK(key_column_ok(dg, in, widths), Code::Invalid, "radix pass: column 0 must be the key");
  // key_xor rebuilds int64 keys from order images: only a sort's image digit may set it
  // (partition / mod / range digits store column 0 as read)
  CYLON_CHECK((key_xor == 0 || std::is_same<Digit, ImageDigit>::value), Code::Invalid,
              "radix pass: key_xor is only valid for order-image digits");
  hipStream_t s = as_stream(stream);
  const uint32_t nb = 1u << digit_bits;
  CYLON_CHECK(stable || CAN_UNSTABLE, Code::Invalid, "radix pass: only partition digits may rank unstably");
  // test knob: every partition pass ranks unstably, so LSD passes after the first scramble the
  // order they received -- rows end in wrong partitions and the join's ranking guard must fire
  const bool want_stable = stable;  // the ranking guard checks what the caller asked for
  if (CAN_UNSTABLE && knobs::Flag("RP_DEBUG_UNSTABLE", false)) stable = false;
  const bool unstable = CAN_UNSTABLE && !stable;
  const bool wave_atomic = !unstable && rp_wave_atomic(s);
  const int threads = rp_threads(ncols, unstable || wave_atomic);
  const bool lean = !Digit::kNarrow && rp_lean(ncols) && (unstable || wave_atomic) && threads == 1024;
  RPGeometry g;
  const int64_t *bh_scan = nullptr;
  TileSched lb{};
  const bool xt = threads == 1024 && n < (int64_t(1) << 32) && rp_xt();
  CYLON_CHECK(xt || bucket_extra == nullptr, Code::Invalid, "radix pass: gapped layouts need the XCD-tile schedule");
  const bool lbin = lba && lba->plan_in, lbcnt = lba && lba->plan_out;
  if (lbin || lbcnt) {
    bool w8all = true;
    for (int c = 0; c < ncols; ++c) w8all &= widths[c] == 8;
    CYLON_CHECK(xt && lean && !unstable && wave_atomic && w8all && nb <= (uint32_t)kLbMaxBuckets &&
                    n < (int64_t(1) << 31) - 2 && (!lbcnt || (digit_bits >= 3 && nd_mask + 1 <= (uint32_t)kLbMaxBuckets)),
                Code::Invalid, "look-back sort pass not eligible");
  }
  if (!xt) tiles_prescanned = false;  // histogram mode counts its own blocks (the prescan is unused)
  if (!xt) nd_in = nullptr;            // ... and reads the keys (the previous pass's digits go unused)
  if (xt && lbin) {  // look-back offsets: the previous pass planned the chunks (see k_lb_plan)
    const int64_t ntiles = (n + kRPTile - 1) / kRPTile;
    HIP_CHECK(hipMemsetAsync(const_cast<uint32_t *>(lba->plan_in) + kLbTickets, 0, kXcds * sizeof(uint32_t), s));
    CYLON_CHECK((ntiles + kLbChunks) * nb <= lba->state_words, Code::Invalid, "look-back state too small");
    HIP_CHECK(hipMemsetAsync(lba->state, 0, sizeof(uint32_t) * (ntiles + kLbChunks) * nb, s));
    lb.lb_plan = lba->plan_in;
    lb.lb_state = lba->state;
    lb.lb_err = lba->err;
    lb.xt_ticket = const_cast<uint32_t *>(lba->plan_in) + kLbTickets;
    g.rows_per_block = kRPTile;
    g.nblocks = std::min<int64_t>(ntiles + kLbChunks, (int64_t)kNumCUs * 2);
  } else if (xt) {  // exact per-tile offsets, tiles claimed in order per XCD (see xt_claim)
    const XtLayout L = xt_layout(n, nb);
    uint16_t *th = reinterpret_cast<uint16_t *>(ws + L.th);
    uint32_t *off = reinterpret_cast<uint32_t *>(ws + L.off);
    uint32_t *csum = reinterpret_cast<uint32_t *>(ws + L.csum), *cpre = reinterpret_cast<uint32_t *>(ws + L.cpre);
    unsigned *tk = reinterpret_cast<unsigned *>(ws + L.tickets);
    HIP_CHECK(hipMemsetAsync(tk, 0, kXcds * sizeof(unsigned), s));
    if (!tiles_prescanned && nd_in != nullptr) {  // the previous pass wrote this pass's digits
      hipLaunchKernelGGL(k_rp_hist_tiles<NdDigit>, dim3((unsigned)std::min<int64_t>(L.ntiles, kNumCUs * 16)),
                         dim3(kHTThreads), 0, s, NdDigit{nd_in}, n, nb, L.ntiles, th);
      HIP_LAUNCH_CHECK();
    } else if (!tiles_prescanned) {  // else the caller already wrote th (radix_sort_prehist + fold)
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
    hipLaunchKernelGGL(k_ts_offsets, dim3((unsigned)L.nchunks), dim3(bt), 0, s, th, cpre, bbase, nb, L.ntiles, off,
                       bucket_extra);
    HIP_LAUNCH_CHECK();
    lb.xt_off = off;
    lb.xt_ticket = tk;
    lb.xt_tiles = L.ntiles;
    g.rows_per_block = kRPTile;
    g.nblocks = std::min<int64_t>(L.ntiles, (int64_t)kNumCUs * (lean ? 2 : 1));  // persistent: all resident
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
  cs.nd_out = nd_out;
  cs.nd_shift = nd_shift;
  cs.nd_mask = nd_mask;
  cs.nd_sub = nd_sub;
  cs.check_order = want_stable ? 1 : 0;
  cs.order_bad = order_flag();
  for (int c = 0; c < kMaxFusedCols; ++c) {
    cs.in[c] = c < ncols ? in[c] : nullptr;
    cs.out[c] = c < ncols ? out[c] : nullptr;
    cs.width[c] = c < ncols ? widths[c] : 8;
  }
  bool w8 = true;  // (a narrowed column 0 is stored as 4 bytes by its own path)
  for (int c = 0; c < ncols; ++c) {
    w8 &= widths[c] == 8 || (Digit::kNarrow && c == 0);
    CYLON_CHECK(in[c] != nullptr || (c > 0 && widths[c] == 8), Code::Invalid,
                "radix pass: a generated row-id column must be an 8-byte payload column");
  }
  const bool big = threads == 1024;
  if (lbcnt) {  // per-block (chunk, next digit) rows, summed into the next pass's plan below
    const int64_t words = g.nblocks * kLbChunks * (int64_t)(nd_mask + 1);
    CYLON_CHECK(words <= lba->gcnt_words, Code::Invalid, "look-back counters too small");
    HIP_CHECK(hipMemsetAsync(lba->gcnt, 0, sizeof(uint32_t) * words, s));
    lb.lb_gcnt = lba->gcnt;
    lb.lb_xshift = digit_bits - 3;
  }
  if (lean) {
    if constexpr (!Digit::kNarrow) {
      constexpr int R = CAN_UNSTABLE ? kRankBlockAtomic : kRankWaveAtomic;
      const int lbm = (lbin ? 2 : 0) | (lbcnt ? 1 : 0);
      if (unstable) lean_kernel<Digit, R>(w8, g, s, dg, digit_bits, nb, cs, n, bh_scan, lb, xt);
      else lean_kernel<Digit, kRankWaveAtomic>(w8, g, s, dg, digit_bits, nb, cs, n, bh_scan, lb, xt, lbm);
    }
    HIP_LAUNCH_CHECK();
    if (lbin) {  // local chunks: XCD x had blocks
      hipLaunchKernelGGL(k_lb_check, dim3(1), dim3(kWave), 0, s, lba->plan_in, lba->err);
      HIP_LAUNCH_CHECK();
    }
    if (lbcnt) lb_plan_next(lba, g.nblocks, nd_mask + 1, n, s);
    return;
  }
  if (unstable) {
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
                     const SortLbArgs *lb, int nd_bits, const NarrowKeys *nk, bool tiles_prescanned,
                     const uint16_t *nd_in, uint16_t *nd_out) {
  const uint32_t nb = 1u << digit_bits;
  if (nk && nk->base_src) {  // narrowed join partition pass (no look-back counting)
    CYLON_CHECK(!(lb && (lb->plan_in || lb->plan_out)), Code::Invalid, "narrowed pass: no look-back");
    rows_pass_launch(PartDigitN{keys, nk->kin4, nk->base_src, nk->bad, total_bits, shift, nb - 1, 0}, n, digit_bits, in,
                     out, widths, ncols, ws, stream, 0, stable);
    return;
  }
  CYLON_CHECK(!(lb && lb->plan_out) || (nd_bits >= 1 && nd_bits <= 9 && stable && !nd_out), Code::Invalid,
              "look-back counting partition pass: next digit of " << nd_bits << " bits");
  CYLON_CHECK(!nd_out || (nd_bits >= 1 && nd_bits <= 16), Code::Invalid, "partition pass: next-digit output");
  rows_pass_launch(PartDigit{keys, total_bits, shift, nb - 1}, n, digit_bits, in, out, widths, ncols, ws, stream, 0,
                   stable, tiles_prescanned, nullptr, lb && lb->plan_in ? nullptr : nd_in, nd_out, shift + digit_bits,
                   (lb && lb->plan_out) || nd_out ? (1u << nd_bits) - 1u : 0u, 0, lb);
}

int64_t radix_rows_pass_th_offset(int64_t n, int digit_bits) { return xt_layout(n, 1u << digit_bits).th; }

void radix_sort_rows_pass(const int64_t *keys, int64_t n, int shift, int digit_bits, const uint8_t *const *in,
                          uint8_t *const *out, const int *widths, int ncols, int64_t *ws, void *stream,
                          uint64_t key_xor, uint64_t digit_flip, bool tiles_prescanned, const uint16_t *nd_in,
                          uint16_t *nd_out, int nd_shift, int nd_bits, uint64_t sub, const SortLbArgs *lb) {
  const uint32_t nb = 1u << digit_bits;
  CYLON_CHECK(!(lb && lb->plan_out) || (nd_out == nullptr && nd_bits >= 1 && nd_bits <= 9), Code::Invalid,
              "look-back counting pass: next digit of " << nd_bits << " bits");
  // (the digits come from column 0 as stored: images on every pass but a last one that restores keys)
  CYLON_CHECK(nd_out == nullptr || (nd_bits >= 1 && nd_bits <= 16), Code::Invalid,
              "sort pass: next-digit output of " << nd_bits << " bits");
  rows_pass_launch(ImageDigit{keys, shift, nb - 1, digit_flip, sub}, n, digit_bits, in, out, widths, ncols, ws,
                   stream, key_xor, true, tiles_prescanned, nullptr, lb && lb->plan_in ? nullptr : nd_in, nd_out,
                   nd_shift, nd_out || (lb && lb->plan_out) ? (1u << nd_bits) - 1u : 0u, sub, lb);
}

bool radix_sort_lb_eligible(int64_t n, int ncols, const int *widths, const int *dbits, int npass, void *stream) {
  if (!knobs::Flag("SORT_LOOKBACK", true) || !rp_xt() || npass < 2 || n < 1 || n >= (int64_t(1) << 31) - 2) return false;
  if (rp_threads(ncols, true) != 1024 || !rp_lean(ncols) || !rp_wave_atomic(as_stream(stream))) return false;
  for (int c = 0; c < ncols; ++c)
    if (widths[c] != 8) return false;
  for (int p = 0; p < npass; ++p)
    if (dbits[p] < 3 || dbits[p] > 9) return false;
  return true;
}

static int64_t lb_state_words(int64_t n) { return ((n + kRPTile - 1) / kRPTile + kLbChunks) * kLbMaxBuckets; }
static int64_t lb_gcnt_words() { return int64_t(2) * kNumCUs * kLbChunks * kLbMaxBuckets; }

int64_t radix_sort_lb_workspace(int64_t n) {
  const int64_t u32 = 2 * (int64_t)kLbPlanWords + 16 + lb_state_words(n) + lb_gcnt_words();
  return (u32 + 1) / 2;
}

SortLbArgs radix_sort_lb_args(int64_t *ws, int64_t n, int pass, int npass, void *stream) {
  uint32_t *w = reinterpret_cast<uint32_t *>(ws);
  SortLbArgs a{};
  a.err = w + 2 * kLbPlanWords;
  a.state = a.err + 16;
  a.state_words = lb_state_words(n);
  a.gcnt = a.state + a.state_words;
  a.gcnt_words = lb_gcnt_words();
  if (pass == 0) HIP_CHECK(hipMemsetAsync(a.err, 0, sizeof(uint32_t), as_stream(stream)));
  a.plan_in = pass > 0 ? w + ((pass - 1) & 1) * kLbPlanWords : nullptr;
  a.plan_out = pass + 1 < npass ? w + (pass & 1) * kLbPlanWords : nullptr;
  return a;
}

bool radix_sort_lb_failed(const int64_t *ws, void *stream) {
  unsigned h = 0;
  const uint32_t *w = reinterpret_cast<const uint32_t *>(ws);
  HIP_CHECK(hipMemcpyAsync(&h, w + 2 * kLbPlanWords, sizeof(h), hipMemcpyDeviceToHost, as_stream(stream)));
  HIP_CHECK(hipStreamSynchronize(as_stream(stream)));
  return h != 0;
}


// ---- slot mode (the histogram-free passes of a join partition; TileSched)
// Segment list of a slot pass and the tile prefix over it (one block; S <= kSlotMaxSeg):
//   src 0: the table itself, 8 chunks [n g / 8, n (g + 1) / 8)
//   src 1: the exact buckets of an XT pass (bucket bases in its workspace: bbase)
//   src 2: the slots of a previous slot pass (slot g at g * pslot, pcnt[g] rows)
// (SRC is a template parameter: with a runtime source the compiler merged the bbase / pcnt branches
// and loaded through the null pointer of the unused one -- the fault of gpurun_out/r04j)
template <int SRC>
__global__ __launch_bounds__(kRPThreads) void k_sl_segments(int S, int64_t n, const uint32_t *__restrict__ bbase,
                                                            const int64_t *__restrict__ pcnt, int64_t pslot,
                                                            uint32_t *__restrict__ ss, uint32_t *__restrict__ se,
                                                            uint32_t *__restrict__ tpre) {
  __shared__ uint32_t wsum[kRPWaves];
  constexpr int PER = kSlotMaxSeg / kRPThreads;
  uint32_t tiles[PER];
  uint32_t tot = 0;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int g = threadIdx.x * PER + i;
    tiles[i] = 0;
    if (g < S) {
      int64_t a, e;
      if constexpr (SRC == 0) {
        a = n * g / S;
        e = n * (g + 1) / S;
      } else if constexpr (SRC == 1) {
        a = bbase[g];
        e = g + 1 < S ? (int64_t)bbase[g + 1] : n;
      } else {  // segment g = (bucket g >> 3, XCD g & 7) is first-pass slot (g & 7) * (S / 8) + (g >> 3)
        const int64_t sl = (int64_t)(g & (kXcds - 1)) * (S / kXcds) + (g >> 3);
        a = sl * pslot;
        e = a + (pcnt[sl] < pslot ? pcnt[sl] : pslot);
      }
      ss[g] = (uint32_t)a;
      se[g] = (uint32_t)e;
      tiles[i] = (uint32_t)((e - a + kRPTile - 1) / kRPTile);
    }
    tot += tiles[i];
  }
  uint32_t ex = rp_block_exscan<kRPWaves>(tot, wsum);
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int g = threadIdx.x * PER + i;
    if (g < S) tpre[g] = ex;
    ex += tiles[i];
  }
  if (threadIdx.x == kRPThreads - 1) tpre[S] = ex;
}

// rows in each slot (a slot that overflowed reports its capacity; the caller discards the result)
__global__ void k_sl_counts(const unsigned int *__restrict__ cursor, int64_t nslots, int64_t slot,
                            int64_t *__restrict__ counts) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nslots; i += stride)
    counts[i] = (int64_t)cursor[i] < slot ? (int64_t)cursor[i] : slot;
}

int64_t radix_slot_tile_rows() { return kRPTile; }

bool radix_slot_eligible(int64_t n, int ncols, int first_bits, int second_bits) {
  return rp_xt() && n > 0 && rp_threads(ncols, true) == 1024 && first_bits >= 1 && first_bits <= kRJMaxDigitBits &&
         second_bits >= 1 && second_bits <= kRJMaxDigitBits && (int64_t(kXcds) << first_bits) * 2 < (int64_t(1) << 32) &&
         n < (int64_t(1) << 31);
}

bool radix_slot_first_pass_ok(int first_bits) { return (kXcds << first_bits) <= kSlotMaxSeg; }

int64_t radix_slot_workspace(int first_bits, int second_bits) {  // int64 words: segments + cursors
  const int64_t segs = std::max<int64_t>(kXcds << first_bits, int64_t(1) << first_bits);
  const int64_t u32 = 3 * (segs + 1) + (int64_t(kXcds) << first_bits) + (int64_t(1) << (first_bits + second_bits));
  return (u32 + 1) / 2;
}

template <class Digit>
static void slot_pass(const Digit &dg, int64_t n, int digit_bits, const uint8_t *const *in, uint8_t *const *out,
                      const int *widths, int ncols, int src, int S, const uint32_t *bbase, const int64_t *pcnt,
                      int64_t pslot, int gshift, int gmask, int B, int64_t nslots, int64_t slot, int64_t *ws,
                      int64_t *counts, unsigned int *overflow, hipStream_t s, uint64_t key_xor = 0) {
  CYLON_CHECK(S >= 1 && S <= kSlotMaxSeg && ncols >= 1 && ncols <= kMaxFusedCols && slot > 0, Code::Invalid,
              "slot pass arguments");
  CYLON_CHECK(key_column_ok(dg, in, widths), Code::Invalid, "slot pass: column 0 must be the key");
  CYLON_CHECK(nslots * slot + kRPTile < (int64_t(1) << 32), Code::Invalid, "slot pass: output rows beyond 2^32");
  const uint32_t nb = 1u << digit_bits;
  uint32_t *w32 = reinterpret_cast<uint32_t *>(ws);
  uint32_t *ss = w32, *se = ss + S, *tpre = se + S;
  unsigned int *cursor = tpre + S + 1;
  HIP_CHECK(hipMemsetAsync(cursor, 0, sizeof(uint32_t) * nslots, s));
  CYLON_CHECK((src == 0) || (src == 1 && bbase) || (src == 2 && pcnt), Code::Invalid, "slot pass source " << src);
  if (src == 0)
    hipLaunchKernelGGL(k_sl_segments<0>, dim3(1), dim3(kRPThreads), 0, s, S, n, bbase, pcnt, pslot, ss, se, tpre);
  else if (src == 1)
    hipLaunchKernelGGL(k_sl_segments<1>, dim3(1), dim3(kRPThreads), 0, s, S, n, bbase, pcnt, pslot, ss, se, tpre);
  else
    hipLaunchKernelGGL(k_sl_segments<2>, dim3(1), dim3(kRPThreads), 0, s, S, n, bbase, pcnt, pslot, ss, se, tpre);
  HIP_LAUNCH_CHECK();
  TileSched lb{};
  lb.sl_tpre = tpre;
  lb.sl_ss = ss;
  lb.sl_se = se;
  lb.sl_cursor = cursor;
  lb.sl_overflow = overflow;
  lb.sl_slot = slot;
  lb.sl_nslots = nslots;
  lb.sl_nseg = S;
  lb.sl_gshift = gshift;
  lb.sl_gmask = gmask;
  lb.sl_B = B;
  ColSet cs;
  cs.n = ncols;
  cs.key_xor = key_xor;  // (a sort's first MSD pass stores order images)
  cs.check_order = 0;  // the order inside a slot is free
  cs.order_bad = order_flag();
  cs.nd_out = nullptr;
  cs.nd_shift = 0;
  cs.nd_mask = 0;
  cs.nd_sub = 0;
  bool w8 = true;
  for (int c = 0; c < kMaxFusedCols; ++c) {
    cs.in[c] = c < ncols ? in[c] : nullptr;
    cs.out[c] = c < ncols ? out[c] : nullptr;
    cs.width[c] = c < ncols ? widths[c] : 8;
    if (c < ncols) {
      w8 &= widths[c] == 8 || (Digit::kNarrow && c == 0);
      CYLON_CHECK(in[c] != nullptr, Code::Invalid, "slot pass: every column is read");
    }
  }
  // every XCD needs at least one block: its segments' tiles are dealt to its own blocks only
  const int64_t nblocks = std::max<int64_t>(kXcds, std::min<int64_t>((n + kRPTile - 1) / kRPTile + S, kNumCUs));
  // (a pipelined variant that ranked tile t+1 under tile t's column traffic measured no gain --
  // 85.25 / 85.55 vs 85.50 / 85.00 ms at 1B x 1B, profiles/r06/pipelined_pass_ab.txt -- and was removed:
  // the passes are bound by their partial-line write traffic, not by the ranking phases)
  if (w8)
    hipLaunchKernelGGL((k_rows_pass<Digit, true, 1024, kRankBlockAtomic, false, true>), dim3((unsigned)nblocks),
                       dim3(1024), 0, s, dg, digit_bits, nb, cs, n, (int64_t)kRPTile, nblocks, nullptr, lb);
  else
    hipLaunchKernelGGL((k_rows_pass<Digit, false, 1024, kRankBlockAtomic, false, true>), dim3((unsigned)nblocks),
                       dim3(1024), 0, s, dg, digit_bits, nb, cs, n, (int64_t)kRPTile, nblocks, nullptr, lb);
  HIP_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_sl_counts, dim3(grid_for(nslots)), dim3(kBlock), 0, s, cursor, nslots, slot, counts);
  HIP_LAUNCH_CHECK();
}

void radix_slot_first_pass(const int64_t *keys, int64_t n, int total_bits, int first_bits, int second_bits,
                           const uint8_t *const *in, uint8_t *const *out, const int *widths, int ncols, int64_t slot,
                           int64_t *ws, int64_t *counts, unsigned int *overflow, void *stream, const NarrowKeys *nk) {
  CYLON_CHECK(radix_slot_eligible(n, ncols, first_bits, second_bits) && radix_slot_first_pass_ok(first_bits),
              Code::Invalid, "slot first pass not eligible");
  const int nb1 = 1 << first_bits;
  // the high digit; slot x * 2^first_bits + d holds bucket d's rows from XCD x's chunk of the table
  // (XCD-major: the cursors one XCD claims from share cache lines only with each other -- the
  // bucket-major order d * 8 + x put 8 XCDs' atomics on every line)
  if (nk && nk->base_src)
    slot_pass(PartDigitN{keys, nk->kin4, nk->base_src, nk->bad, total_bits, second_bits, (uint32_t)nb1 - 1, 0}, n,
              first_bits, in, out, widths, ncols, 0, kXcds, nullptr, nullptr, 0, 0, 0, 1, int64_t(kXcds) * nb1, slot, ws,
              counts, overflow, as_stream(stream));
  else
    slot_pass(PartDigit{keys, total_bits, second_bits, (uint32_t)nb1 - 1}, n, first_bits, in, out, widths, ncols, 0,
              kXcds, nullptr, nullptr, 0, 0, 0, 1, int64_t(kXcds) * nb1, slot, ws, counts, overflow, as_stream(stream));
}

template <class Digit>
static void slot_rows_pass(const Digit &dg, int64_t n, int first_bits, int second_bits, const uint8_t *const *in,
                           uint8_t *const *out, const int *widths, int ncols, const int64_t *first_ws,
                           const int64_t *first_counts, int64_t first_slot, int64_t slot, int64_t *ws, int64_t *counts,
                           unsigned int *overflow, void *stream);

void radix_slot_rows_pass(const int64_t *keys, int64_t n, int total_bits, int first_bits, int second_bits,
                          const uint8_t *const *in, uint8_t *const *out, const int *widths, int ncols,
                          const int64_t *first_ws, const int64_t *first_counts, int64_t first_slot, int64_t slot,
                          int64_t *ws, int64_t *counts, unsigned int *overflow, void *stream, const NarrowKeys *nk) {
  if (nk && nk->base_src) {
    slot_rows_pass(PartDigitN{keys, nk->kin4, nk->base_src, nk->bad, total_bits, 0, (1u << second_bits) - 1, 0}, n,
                   first_bits, second_bits, in, out, widths, ncols, first_ws, first_counts, first_slot, slot, ws, counts,
                   overflow, stream);
  } else {
    slot_rows_pass(PartDigit{keys, total_bits, 0, (1u << second_bits) - 1}, n, first_bits, second_bits, in, out,
                   widths, ncols, first_ws, first_counts, first_slot, slot, ws, counts, overflow, stream);
  }
}

template <class Digit>
static void slot_rows_pass(const Digit &dg, int64_t n, int first_bits, int second_bits, const uint8_t *const *in,
                           uint8_t *const *out, const int *widths, int ncols, const int64_t *first_ws,
                           const int64_t *first_counts, int64_t first_slot, int64_t slot, int64_t *ws, int64_t *counts,
                           unsigned int *overflow, void *stream) {
  CYLON_CHECK(radix_slot_eligible(n, ncols, first_bits, second_bits), Code::Invalid, "slot pass not eligible");
  const int nb1 = 1 << first_bits;
  const int64_t nslots = int64_t(nb1) << second_bits;
  if (first_counts != nullptr) {  // after a slot first pass: segment g = (bucket g >> 3, XCD g & 7)
    slot_pass(dg, n, second_bits, in, out, widths, ncols, 2, kXcds * nb1, nullptr, first_counts, first_slot, 3, 0, 1,
              nslots, slot, ws, counts, overflow, as_stream(stream));
  } else {  // after an XT first pass: segment g = exact bucket g (bases in its workspace)
    CYLON_CHECK(nb1 <= kSlotMaxSeg, Code::Invalid, "slot pass: too many input buckets");
    const uint32_t *bbase = reinterpret_cast<const uint32_t *>(first_ws + xt_layout(n, (uint32_t)nb1).bbase);
    slot_pass(dg, n, second_bits, in, out, widths, ncols, 1, nb1, bbase, nullptr, 0, 0, 0, 1, nslots, slot, ws,
              counts, overflow, as_stream(stream));
  }
}

// Second pass of a bounded-memory join chunk (ops/join.cpp radix_join_chunked): the input is the
// chunk's rows of an exact narrowed first pass -- nseg consecutive first-pass buckets, bucket g
// starting at row bbase[g] (relative to the chunk) -- and digit d = the low second_bits bits of the
// total_bits partition id goes to slot g * 2^second_bits + d, so the chunk's partitions come out
// in partition order.
void radix_slot_segment_pass(const uint32_t *keys, int64_t n, int total_bits, int second_bits, const uint8_t *const *in,
                             uint8_t *const *out, const int *widths, int ncols, const uint32_t *bbase, int nseg,
                             int64_t slot, int64_t *ws, int64_t *counts, unsigned int *overflow, void *stream,
                             const NarrowKeys *nk) {
  CYLON_CHECK(nk && nk->base_src && nseg >= 1 && nseg <= kSlotMaxSeg && n > 0 && n < (int64_t(1) << 31),
              Code::Invalid, "segment slot pass arguments");
  const int64_t nslots = int64_t(nseg) << second_bits;
  slot_pass(PartDigitN{keys, 1, nk->base_src, nk->bad, total_bits, 0, (1u << second_bits) - 1, 0}, n, second_bits,
            in, out, widths, ncols, 1, nseg, bbase, nullptr, 0, 0, 0, 1, nslots, slot, ws, counts, overflow,
            as_stream(stream));
}

// ---- sampled partition histogram (join slot-mode decision): hist[part] += 1 for keys i = k * stride
template <class Digit>
__global__ void k_part_sample(Digit dg, int64_t n, int64_t stride, uint32_t *__restrict__ hist) {
  dg.init();
  const int64_t m = (n + stride - 1) / stride;
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < m; k += step)
    atomicAdd(&hist[dg(k * stride)], 1u);
}

void radix_part_sample(const int64_t *keys, int64_t n, int bits, int64_t stride, uint32_t *hist,
                       const NarrowKeys *nk, void *stream) {
  CYLON_CHECK(bits >= 1 && bits <= 24 && stride >= 1, Code::Invalid, "partition sample: " << bits << " bits");
  hipStream_t s = as_stream(stream);
  HIP_CHECK(hipMemsetAsync(hist, 0, sizeof(uint32_t) << bits, s));
  const int64_t m = (n + stride - 1) / stride;
  if (m == 0) return;
  const uint32_t mask = (uint32_t)((int64_t(1) << bits) - 1);
  if (nk && nk->base_src)
    hipLaunchKernelGGL(k_part_sample<PartDigitN>, dim3(grid_for(m)), dim3(kBlock), 0, s,
                       PartDigitN{keys, 0, nk->base_src, nk->bad, bits, 0, mask, 0}, n, stride, hist);
  else
    hipLaunchKernelGGL(k_part_sample<PartDigit>, dim3(grid_for(m)), dim3(kBlock), 0, s,
                       PartDigit{keys, bits, 0, mask}, n, stride, hist);
  HIP_LAUNCH_CHECK();
}

// MSD passes of a keys-only sort (seg_sort.hip sorts each final partition in LDS): the first takes
// bits [hr - db1, hr) of image - sub from the raw keys and stores the images (key ^ key_xor) -- into
// (XCD, bucket) slots when 8 x 2^db1 segments fit the second pass's table (slot > 0), else exactly
// (XCD-tile pass: bucket bases in ws) -- the second bits [hr - db1 - db2, hr - db1) into slots.
// Partitions come out in key order.
void radix_sort_msd_first_pass(const int64_t *keys, int64_t n, int hr, int db1, int db2, uint64_t key_xor,
                               uint64_t sub, int64_t *out, int64_t slot, int64_t *ws, int64_t *counts,
                               unsigned int *overflow, void *stream) {
  CYLON_CHECK(radix_slot_eligible(n, 1, db1, db2) && hr >= db1 + db2 && hr <= 64 &&
                  (slot == 0 || radix_slot_first_pass_ok(db1)),
              Code::Invalid, "MSD sort pass not eligible");
  const int nb1 = 1 << db1;
  const uint8_t *in[1] = {reinterpret_cast<const uint8_t *>(keys)};
  uint8_t *o[1] = {reinterpret_cast<uint8_t *>(out)};
  const int w[1] = {8};
  const ImageDigit dg{keys, hr - db1, (uint32_t)nb1 - 1, key_xor, sub};
  if (slot > 0)
    slot_pass(dg, n, db1, in, o, w, 1, 0, kXcds, nullptr, nullptr, 0, 0, 0, 1, int64_t(kXcds) * nb1, slot, ws, counts,
              overflow, as_stream(stream), key_xor);
  else {  // (the second pass reads the bucket bases of an XCD-tile pass: wave-atomic ranking, 1024 threads)
    CYLON_CHECK(rp_xt() && rp_wave_atomic(as_stream(stream)), Code::Invalid, "MSD sort: exact first pass needs XT");
    rows_pass_launch(dg, n, db1, in, o, w, 1, ws, stream, key_xor);
  }
}

void radix_sort_msd_second_pass(const int64_t *images, int64_t n, int hr, int db1, int db2, uint64_t sub,
                                const int64_t *first_ws, const int64_t *first_counts, int64_t first_slot, int64_t *out,
                                int64_t slot, int64_t *ws, int64_t *counts, unsigned int *overflow, void *stream) {
  CYLON_CHECK(hr >= db1 + db2 && hr <= 64 && (first_counts != nullptr || first_ws != nullptr), Code::Invalid,
              "MSD sort pass digits");
  const uint8_t *in[1] = {reinterpret_cast<const uint8_t *>(images)};
  uint8_t *o[1] = {reinterpret_cast<uint8_t *>(out)};
  const int w[1] = {8};
  slot_rows_pass(ImageDigit{images, hr - db1 - db2, (1u << db2) - 1, 0, sub}, n, db1, db2, in, o, w, 1, first_ws,
                 first_counts, first_slot, slot, ws, counts, overflow, stream);
}

// ---- sort prologue: the keys' varying bits (OR ^ AND), the images' min and max, and the first
// pass's per-tile histogram of the order image's low 10 bits in ONE read of the keys (the separate
// reduction read them once more)
constexpr int kSPBits = 10;
__global__ __launch_bounds__(kHTThreads) void k_sort_prehist(const int64_t *__restrict__ keys, int64_t n,
                                                             uint64_t flip, int64_t ntiles, uint16_t *__restrict__ th,
                                                             unsigned long long *__restrict__ orand) {
  constexpr uint32_t nb = 1u << kSPBits;
  __shared__ unsigned int hist[nb];
  uint64_t o = 0, a = ~0ull, mn = ~0ull, mx = 0;
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
        const uint64_t im = k[u] ^ flip;
        mn = im < mn ? im : mn;
        mx = im > mx ? im : mx;
        atomicAdd(&hist[(uint32_t)(im & (nb - 1))], 1u);
      }
    __syncthreads();
    for (uint32_t p = threadIdx.x; p < nb; p += blockDim.x) th[t * nb + p] = (uint16_t)hist[p];
    __syncthreads();
  }
#pragma unroll
  for (int d = kWave / 2; d > 0; d >>= 1) {
    o |= rj_shfl_xor64((long long)o, d);
    a &= rj_shfl_xor64((long long)a, d);
    const uint64_t m0 = (uint64_t)rj_shfl_xor64((long long)mn, d), m1 = (uint64_t)rj_shfl_xor64((long long)mx, d);
    mn = m0 < mn ? m0 : mn;
    mx = m1 > mx ? m1 : mx;
  }
  if (lane_id() == 0) {
    atomicOr(&orand[0], (unsigned long long)o);
    atomicAnd(&orand[1], (unsigned long long)a);
    atomicMin(&orand[2], (unsigned long long)mn);
    atomicMax(&orand[3], (unsigned long long)mx);
  }
}

// th[t][d] (2^db buckets) from the 10-bit histogram of the images: the low db bits of image - sub
// are d exactly when the image's are (d + sub) mod 2^db (rot = sub mod 2^db)
__global__ void k_sort_prehist_fold(const uint16_t *__restrict__ th10, int64_t ntiles, int db, uint32_t rot,
                                    uint16_t *__restrict__ th) {
  const uint32_t nb = 1u << db, groups = 1u << (kSPBits - db);
  const int64_t cells = ntiles * nb, stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; c < cells; c += stride) {
    const int64_t t = c / nb;
    const uint32_t d = (uint32_t)(c % nb);
    uint32_t sum = 0;
    const uint32_t v = (d + rot) & (nb - 1);
    for (uint32_t g = 0; g < groups; ++g) sum += th10[t * (1 << kSPBits) + v + (g << db)];
    th[c] = (uint16_t)sum;
  }
}

int64_t radix_sort_prehist_workspace(int64_t n) { return xt_layout(n, 1u << kSPBits).words + 4; }

uint64_t radix_sort_prehist(const int64_t *keys, int64_t n, uint64_t flip, int64_t *pre_ws, void *stream,
                            uint64_t *img_min, uint64_t *img_max) {
  hipStream_t s = as_stream(stream);
  const XtLayout L = xt_layout(n, 1u << kSPBits);
  unsigned long long *orand = reinterpret_cast<unsigned long long *>(pre_ws + L.words);
  const unsigned long long init[4] = {0ull, ~0ull, ~0ull, 0ull};
  HIP_CHECK(hipMemcpyAsync(orand, init, sizeof(init), hipMemcpyHostToDevice, s));
  hipLaunchKernelGGL(k_sort_prehist, dim3((unsigned)std::min<int64_t>(L.ntiles, kNumCUs * 16)), dim3(kHTThreads), 0,
                     s, keys, n, flip, L.ntiles, reinterpret_cast<uint16_t *>(pre_ws + L.th), orand);
  HIP_LAUNCH_CHECK();
  unsigned long long h[4];
  HIP_CHECK(hipMemcpyAsync(h, orand, sizeof(h), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  if (img_min) *img_min = h[2];
  if (img_max) *img_max = h[3];
  return n <= 1 ? 0ull : (uint64_t)(h[0] ^ h[1]);
}

void radix_sort_prehist_fold(const int64_t *pre_ws, int64_t n, int db, int64_t *ws, void *stream, uint64_t sub) {
  CYLON_CHECK(db >= 1 && db <= kSPBits, Code::Invalid, "sort prehist fold: digit bits " << db);
  const XtLayout P = xt_layout(n, 1u << kSPBits), L = xt_layout(n, 1u << db);
  const uint16_t *th10 = reinterpret_cast<const uint16_t *>(pre_ws + P.th);
  uint16_t *th = reinterpret_cast<uint16_t *>(ws + L.th);
  const int64_t cells = L.ntiles * (int64_t(1) << db);
  hipLaunchKernelGGL(k_sort_prehist_fold, dim3(grid_for(cells)), dim3(kBlock), 0, as_stream(stream), th10, L.ntiles,
                     db, (uint32_t)(sub & ((1u << db) - 1)), th);
  HIP_LAUNCH_CHECK();
}

void radix_range_rows_pass(const int64_t *keys, int64_t n, uint64_t flip, uint64_t mn, int rshift, int shift,
                           int digit_bits, const uint8_t *const *in, uint8_t *const *out, const int *widths, int ncols,
                           int64_t *ws, void *stream) {
  const uint32_t nb = 1u << digit_bits;
  rows_pass_launch(RangeDigit{keys, flip, mn, rshift, shift, nb - 1}, n, digit_bits, in, out, widths, ncols, ws,
                   stream, 0, true);
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

// The same pass into a gapped layout: bucket p's rows start extra[p] rows further on (device
// uint32[2^bits(nparts)], non-decreasing).  Only the XCD-tile schedule takes per-bucket bases: false
// (nothing launched) when it cannot run (CYLON_RP_XT=0, ballot ranking, >= 2^32 output rows).
bool radix_mod_rows_pass_gapped(const int64_t *keys, int64_t n, uint32_t nparts, const uint8_t *const *in,
                                uint8_t *const *out, const int *widths, int ncols, int64_t *ws, void *stream,
                                const uint32_t *extra, int64_t out_rows) {
  CYLON_CHECK(nparts >= 1 && nparts <= (uint32_t)kRPMaxBuckets, Code::Invalid, "partition count " << nparts);
  if (!rp_xt() || out_rows >= (int64_t(1) << 32) || n == 0) return false;
  if (!rp_wave_atomic(as_stream(stream)) && rp_threads(ncols, false) != 1024) return false;
  rows_pass_launch(ModDigit{keys, nparts}, n, bits_for(nparts), in, out, widths, ncols, ws, stream, 0, true, false,
                   extra);
  return true;
}

// Shuffle descriptor counts: rows per modulo partition, and (minmax != nullptr) the key column's
// min / max from the same read of the keys -- the wire narrowing's range (ops/shuffle.cpp
// planned_shuffle), which otherwise costs a second full read of the key column (aminmax).
__global__ __launch_bounds__(kRPThreads) void k_mod_counts(ModDigit digit, int64_t n,
                                                           unsigned long long *__restrict__ counts,
                                                           long long *__restrict__ minmax) {
  __shared__ unsigned int hist[kRPMaxBuckets];
  __shared__ long long wmin[kRPWaves], wmax[kRPWaves];
  for (uint32_t p = threadIdx.x; p < digit.nparts; p += blockDim.x) hist[p] = 0;
  __syncthreads();
  long long lo = LLONG_MAX, hi = LLONG_MIN;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t k = digit.keys[i];
    atomicAdd(&hist[digit.of_key(k)], 1u);
    lo = k < lo ? k : lo;
    hi = k > hi ? k : hi;
  }
  if (minmax != nullptr) {  // wave64 butterfly, then one global atomic pair per block
#pragma unroll
    for (int o = kWave / 2; o > 0; o >>= 1) {
      const long long a = __shfl_xor(lo, o), b = __shfl_xor(hi, o);
      lo = a < lo ? a : lo;
      hi = b > hi ? b : hi;
    }
    const int w = threadIdx.x / kWave;
    if (lane_id() == 0) {
      wmin[w] = lo;
      wmax[w] = hi;
    }
  }
  __syncthreads();
  for (uint32_t p = threadIdx.x; p < digit.nparts; p += blockDim.x)
    if (hist[p]) atomicAdd(&counts[p], (unsigned long long)hist[p]);
  if (minmax != nullptr && threadIdx.x == 0) {
    for (int w = 1; w < (int)(blockDim.x / kWave); ++w) {
      lo = wmin[w] < lo ? wmin[w] : lo;
      hi = wmax[w] > hi ? wmax[w] : hi;
    }
    lo = wmin[0] < lo ? wmin[0] : lo;
    hi = wmax[0] > hi ? wmax[0] : hi;
    atomicMin(&minmax[0], lo);
    atomicMax(&minmax[1], hi);
  }
}

__global__ void k_minmax_init(long long *minmax) {
  if (threadIdx.x == 0) {
    minmax[0] = LLONG_MAX;
    minmax[1] = LLONG_MIN;
  }
}

void mod_partition_counts(const int64_t *keys, int64_t n, uint32_t nparts, int64_t *counts, void *stream,
                          int64_t *minmax) {
  CYLON_CHECK(nparts >= 1 && nparts <= (uint32_t)kRPMaxBuckets, Code::Invalid, "partition count " << nparts);
  hipStream_t s = as_stream(stream);
  HIP_CHECK(hipMemsetAsync(counts, 0, sizeof(int64_t) * nparts, s));
  long long *mm = reinterpret_cast<long long *>(minmax);
  if (mm != nullptr) {
    hipLaunchKernelGGL(k_minmax_init, dim3(1), dim3(kWave), 0, s, mm);
    HIP_LAUNCH_CHECK();
  }
  if (n == 0) return;
  hipLaunchKernelGGL(k_mod_counts, dim3(grid_for(n, kRPThreads, kNumCUs * 2)), dim3(kRPThreads), 0, s,
                     ModDigit{keys, nparts}, n, reinterpret_cast<unsigned long long *>(counts), mm);
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

// narrowed join keys (PartDigitN): partition = top bits of fmix32(offset)
__global__ void k_part_offsets32(const uint32_t *__restrict__ keys, int64_t n, int bits, int64_t nparts,
                                 int64_t *__restrict__ offs) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p <= nparts; p += stride) {
    int64_t lo = 0, hi = n;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if ((int64_t)(hashing::fmix32(keys[mid]) >> (32 - bits)) < p) lo = mid + 1; else hi = mid;
    }
    offs[p] = lo;
  }
}

void radix_part_offsets32(const uint32_t *keys, int64_t n, int bits, int64_t *offs, void *stream) {
  CYLON_CHECK(bits >= 1 && bits <= 31, Code::Invalid, "narrowed partition bits " << bits);
  const int64_t np = int64_t(1) << bits;
  hipLaunchKernelGGL(k_part_offsets32, dim3(grid_for(np + 1)), dim3(kBlock), 0, as_stream(stream), keys, n, bits, np,
                     offs);
  HIP_LAUNCH_CHECK();
}

void radix_part_offsets(const int64_t *keys, int64_t n, int bits, int64_t *offs, void *stream) {
  const int64_t np = int64_t(1) << bits;
  hipLaunchKernelGGL(k_part_offsets, dim3(grid_for(np + 1)), dim3(kBlock), 0, as_stream(stream), keys, n, bits, np,
                     offs);
  HIP_LAUNCH_CHECK();
}

// ---- key-hash chunks of the bounded-memory join (ops/join.cpp radix_join_chunked): chunk = the LOW
// cbits bits of fmix64(key) -- independent of the join's partition, which takes the TOP bits -- so
// every chunk's own radix join still spreads over all of its partitions.  One exact (XT) pass moves
// every column into chunk-major order; chunk c is then rows [offs[c], offs[c + 1]).
__global__ void k_low_chunk_offsets(const int64_t *__restrict__ keys, int64_t n, uint32_t mask, int64_t nchunks,
                                    int64_t *__restrict__ offs) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c > nchunks) return;
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if ((int64_t)((uint32_t)hashing::fmix64((uint64_t)keys[mid]) & mask) < c) lo = mid + 1; else hi = mid;
  }
  offs[c] = lo;
}

void radix_chunk_pass(const int64_t *keys, int64_t n, int cbits, const uint8_t *const *in, uint8_t *const *out,
                      const int *widths, int ncols, int64_t *ws, int64_t *offs, void *stream, bool stable) {
  CYLON_CHECK(cbits >= 1 && cbits <= kRJMaxDigitBits, Code::Invalid, "chunk pass bits " << cbits);
  const uint32_t nb = 1u << cbits;
  // stable: exact per-tile offsets AND a stable in-tile rank, so every pass over the same keys moves
  // row i to the same place (column groups of one table, moved by separate passes)
  rows_pass_launch(PartDigit{keys, 64, 0, nb - 1}, n, cbits, in, out, widths, ncols, ws, stream, 0, stable);
  if (offs == nullptr) return;
  // (column 0 of the output: the keys in chunk-major order)
  hipLaunchKernelGGL(k_low_chunk_offsets, dim3(grid_for((int64_t)nb + 1)), dim3(kBlock), 0, as_stream(stream),
                     reinterpret_cast<const int64_t *>(out[0]), n, nb - 1, (int64_t)nb, offs);
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

// this file's code object is loaded at context creation (preload_device_code), not on first use
void preload_radix_join() { preload_code(reinterpret_cast<const void *>(&k_sl_counts)); }

}  // namespace hip
}  // namespace cylon
