// Per-partition LDS join kernels of the radix hash join (K5): count / write over partition pairs
// produced by the radix passes (radix_join.hip), with split work items for skewed partitions.
#include "radix_common.hpp"

namespace cylon {
namespace hip {

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
// column itself, which is not staged twice) + a matched flag (build-preserving outer joins).
int64_t radix_join_capacity(const int *widths, const uint8_t *const *in, int n, bool match_flags, int key_bytes) {
  int64_t row = key_bytes + 2 + (match_flags ? 1 : 0);
  for (int q = 0; q < n; ++q)
    if (in[q]) row += widths[q];
  int64_t cap = kRJRowArea / row;
  cap = std::min<int64_t>(cap, kRJMaxRows);
  return cap & ~int64_t(7);  // multiple of 8: every column region stays 8-byte aligned
}

__device__ __forceinline__ uint32_t rj_bucket(int64_t k) {
  return (uint32_t)hashing::fmix64((uint64_t)k) & (kRJBuckets - 1);
}
// narrowed keys (uint32 offsets, radix_join.hip PartDigitN): the partition is the TOP bits of
// fmix32(offset), the LDS bucket its low bits
__device__ __forceinline__ uint32_t rj_bucket(uint32_t k) { return hashing::fmix32(k) & (kRJBuckets - 1); }

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

// Outer joins (OJ bits): 1 = probe rows without a match are emitted once with a null build side,
// 2 = build rows without a match are emitted after the partition's matches with a null probe side.
constexpr int kOJProbe = 1, kOJBuild = 2;

// matches of k in its bucket; OJ & 2: the matched build slots are flagged (plain byte stores of 1)
template <int OJ, class KT>
__device__ __forceinline__ uint32_t rj_count_mark(const uint16_t *bst, const KT *skeys, KT k, uint8_t *flg) {
  const uint32_t b = rj_bucket(k);
  uint32_t c = 0;
  for (uint32_t i = bst[b], e = bst[b + 1]; i < e; ++i)
    if (skeys[i] == k) {
      ++c;
      if (OJ & kOJBuild) flg[i] = 1;
    }
  return c;
}

// Count kernel block: 512 threads (10 build + 10 probe keys per thread) so two or three
// blocks share a CU (48 KB LDS each) and one block's key loads overlap another's probing;
// the 1024-thread version ran one latency-bound block per CU (128 VGPRs).
constexpr int kRCThreads = 512;
constexpr int kRCWaves = kRCThreads / kWave;
constexpr int kRCRowsPerThread = kRJMaxRows / kRCThreads;
static_assert(kRCRowsPerThread * kRCThreads == kRJMaxRows, "count rows per thread");

// rows of partition p: offs[p] .. offs[p + 1] (exact passes), or slot-mode partitions (slot > 0:
// radix_slot_rows_pass) at p * slot holding offs[p] rows
__device__ __forceinline__ void part_span(const int64_t *offs, int64_t slot, int64_t p, int64_t &b, int64_t &n) {
  if (slot > 0) {
    b = p * slot;
    n = offs[p];
  } else {
    b = offs[p];
    n = offs[p + 1] - b;
  }
}

template <int OJ, bool NK>
__global__ __launch_bounds__(kRCThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_rj_count(
    const int64_t *__restrict__ pkeys0, const int64_t *__restrict__ poffs, const int64_t *__restrict__ bkeys0,
    const int64_t *__restrict__ boffs, int64_t nparts, int cap, int64_t pstride, int64_t *__restrict__ counts,
    int *overflow, int64_t pslot, int64_t bslot, const int64_t *__restrict__ items, int64_t nitems,
    const uint8_t *__restrict__ skip) {
  using KT = typename std::conditional<NK, uint32_t, int64_t>::type;  // NK: uint32 key offsets
  const KT *__restrict__ pkeys = reinterpret_cast<const KT *>(pkeys0);
  const KT *__restrict__ bkeys = reinterpret_cast<const KT *>(bkeys0);
  // pstride > 1: only partitions 0, pstride, 2 pstride, ... are counted, into counts[p / pstride]
  // (the sampled output-size estimate of the fused write path).  Output rows per partition:
  // matches, + unmatched probe rows (OJ & 1), + unmatched build rows (OJ & 2).  items != nullptr:
  // counts[i] = output rows of split item i (its deferred sides' unmatched rows excluded); skip[p]:
  // partition p is covered by items (counts 0, never an LDS overflow).
  __shared__ __attribute__((aligned(16))) uint16_t bst[kRJBuckets + 8];
  __shared__ KT skeys[kRJMaxRows];
  __shared__ uint8_t flg[(OJ & kOJBuild) ? kRJMaxRows : 1];
  __shared__ uint32_t wsum[kRCWaves];
  __shared__ unsigned long long csum[kRCWaves];
  const int64_t nsample = items ? nitems : (nparts + pstride - 1) / pstride;
  for (int64_t ci = blockIdx.x; ci < nsample; ci += gridDim.x) {
    int64_t rb, nr, lb, nl;
    int iflags = 0;
    if (items) {
      const int64_t *it = items + ci * kRJItemWords;
      lb = it[0];
      nl = it[1];
      rb = it[2];
      nr = it[3];
      iflags = (int)it[4];
    } else {
      const int64_t p = ci * pstride;
      if (skip && skip[p]) {
        if (threadIdx.x == 0) counts[ci] = 0;
        continue;
      }
      part_span(boffs, bslot, p, rb, nr);
      part_span(poffs, pslot, p, lb, nl);
    }
    // unmatched rows of a side count here unless the item defers them (emitted by emission items)
    const bool pun = (OJ & kOJProbe) && !(iflags & kRJItemPDefer);
    const bool bun = (OJ & kOJBuild) && !(iflags & kRJItemBDefer);
    if (nr > cap) {  // uniform branch: whole block
      if (threadIdx.x == 0) {
        atomicOr(overflow, 1);
        counts[ci] = 0;
      }
      continue;
    }
    if (nr == 0 || nl == 0) {
      if (threadIdx.x == 0)
        counts[ci] = (nr == 0 && pun ? nl : 0) + (nl == 0 && bun ? nr : 0);
      continue;
    }
    // build keys are read twice (claim, then place): the second read hits L2 and the block
    // keeps only 16-bit ranks in registers (two 512-thread blocks per CU without spills)
    __syncthreads();  // previous partition done with bst / skeys / csum / flg
    for (int s = threadIdx.x; s < kRJBuckets / 2; s += blockDim.x) reinterpret_cast<uint32_t *>(bst)[s] = 0;
    if (OJ & kOJBuild)
      for (int i = threadIdx.x; i < nr; i += blockDim.x) flg[i] = 0;
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
        if (l0 + u * kRCThreads < nl) {
          const uint32_t mc = rj_count_mark<OJ, KT>(bst, skeys, pk[u], flg);
          c += pun && mc == 0 ? 1u : mc;
        }
    }
    if ((OJ & kOJBuild) && bun) {  // uniform branch
      __syncthreads();  // every probe has flagged its matches
      for (int i = threadIdx.x; i < nr; i += blockDim.x) c += flg[i] ? 0u : 1u;
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
__device__ __forceinline__ uint32_t rj_shfl_key(uint32_t x, int src) { return __shfl(x, src, kWave); }

struct BuildOut {               // build-side output columns
  uint8_t *out[kMaxFusedCols];
  int width[kMaxFusedCols];
  int lds_off[kMaxFusedCols];   // byte offset of the staged column in the LDS row area, -1 = key
  int n;
  int match_off;                // OJ & 2: byte offset of the build rows' matched flags in the row area
};

// Outer joins (OJ bits, see rj_count_mark): presence bytes (ppres / bpres: 1 = that side holds a
// row) are written for the side(s) that can be null; the host turns them into the output
// columns' validity (join.cpp radix_join).

// the write kernel's build staging: rj_dma_block over its 16 waves
__device__ __forceinline__ void rj_dma(const uint8_t *src, int bytes, uint8_t *dst, int wave, int lane) {
  rj_dma_block<kRJWaves>(src, bytes, dst, wave, lane);
}

// pkey: index of the probe column that IS the key (its value comes from the probe key, not a
// second load; -1 none).  DMA: stage the build columns by LDS-DMA (needs W8) instead of register
// round trips per column.
template <int MAXP, int MAXB, bool W8, bool DMA, int OJ, bool NK>
__global__ __launch_bounds__(kRJThreads, 4) void k_rj_write(const int64_t *__restrict__ pkeys0,
                                                            const int64_t *__restrict__ poffs,
                                                            const int64_t *__restrict__ bkeys0,
                                                            const int64_t *__restrict__ boffs, int64_t nparts,
                                                            int cap, const int64_t *__restrict__ out_offs, ColSet pc,
                                                            ColSet bs, BuildOut bo,
                                                            unsigned long long *__restrict__ cursor, int64_t out_cap,
                                                            int *__restrict__ overflow,
                                                            int pkey,
                                                            uint8_t *__restrict__ ppres, uint8_t *__restrict__ bpres,
                                                            int64_t pslot, int64_t bslot,
                                                            const int64_t *__restrict__ items, int64_t nitems,
                                                            const uint8_t *__restrict__ skip,
                                                            uint8_t *__restrict__ gprobe,
                                                            uint8_t *__restrict__ gbuild,
                                                            const int64_t *__restrict__ narrow_base) {
  // NK: keys are uint32 offsets from base = narrow_base[0] - 2^31 (radix_join.hip PartDigitN); the
  // key output columns get base + offset
  using KT = typename std::conditional<NK, uint32_t, int64_t>::type;
  const KT *__restrict__ pkeys = reinterpret_cast<const KT *>(pkeys0);
  const KT *__restrict__ bkeys = reinterpret_cast<const KT *>(bkeys0);
  const uint64_t nbase = NK ? (uint64_t)narrow_base[0] - (uint64_t(1) << 31) : 0;
  auto key_value = [&](KT k) -> uint64_t { return NK ? (uint64_t)nbase + (uint64_t)k : (uint64_t)k; };
  // out_offs != nullptr: partition p's rows start at out_offs[p] (exact count kernel ran first).
  // out_offs == nullptr: fused count -- each partition claims its rows from *cursor with one
  // atomic after counting its matches (output partitions land in claim order); a claim past
  // out_cap sets overflow bit 2 and writes nothing (the cursor still totals the rows needed),
  // a build side beyond the LDS capacity sets bit 1.
  // pc: probe columns (in -> out); bs: staged build columns (in, width), LDS
  // region j at 10*cap + sum of cap*width of the earlier ones; bo: build outputs.
  // Row area: keys in bucket order [0, 8 cap), permutation to the staged row
  // [8 cap, 10 cap), payload columns in staged (original) row order, then (OJ & 2) one matched
  // flag per bucket slot.
  __shared__ __attribute__((aligned(16))) uint16_t bst[kRJBuckets + 8];
  __shared__ __attribute__((aligned(16))) uint8_t area[kRJRowArea];
  __shared__ uint32_t wtot[kRJWaves];
  __shared__ int64_t sclaim;
  KT *skeys = reinterpret_cast<KT *>(area);
  uint16_t *perm = reinterpret_cast<uint16_t *>(area + sizeof(KT) * (int64_t)cap);
  uint8_t *flg = area + ((OJ & kOJBuild) ? bo.match_off : 0);
  const int lane = lane_id();
  const int wave = threadIdx.x / kWave;
  // work w < nitems: split item w (heaviest first: they lead the grid-stride order); else partition
  // w - nitems unless skip marks it as covered by items.  Items run in cursor mode only.
  for (int64_t w = blockIdx.x; w < nitems + nparts; w += gridDim.x) {
    int64_t rb, nr, lb, nl, p = -1;
    int iflags = 0;
    if (w < nitems) {
      const int64_t *it = items + w * kRJItemWords;
      lb = it[0];
      nl = it[1];
      rb = it[2];
      nr = it[3];
      iflags = (int)it[4];
    } else {
      p = w - nitems;
      if (skip && skip[p]) continue;
      part_span(boffs, bslot, p, rb, nr);
      part_span(poffs, pslot, p, lb, nl);
    }
    const bool pdefer = (iflags & kRJItemPDefer) != 0, bdefer = (iflags & kRJItemBDefer) != 0;
    const bool pemit = (iflags & kRJItemPEmit) != 0, bemit = (iflags & kRJItemBEmit) != 0;
    if (nr > cap && out_offs == nullptr && threadIdx.x == 0) atomicOr(overflow, 1);
    // inner: both sides needed; outer: a preserved side alone still emits its rows
    const bool live = (nr > 0 && nl > 0) || ((OJ & kOJProbe) && nl > 0) || ((OJ & kOJBuild) && nr > 0);
    if (!live || nr > cap) continue;
    const int64_t obase = out_offs && p >= 0 ? out_offs[p] : 0;
    // ---- phase A: probe rows of this wave's slice into VGPRs (in flight during the build)
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
    if (OJ & kOJBuild)
      for (int i = threadIdx.x; i < nr; i += blockDim.x) flg[i] = 0;
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
        if ((OJ & kOJBuild) && bemit) flg[pos] = gbuild[rb + r];  // matched by an earlier item
      }
    }
    __syncthreads();
    // ---- phase C: count this wave's output rows (matches; a lone row for an unmatched probe row
    // of a probe-preserving join), flag matched build slots, slice offsets
    // (a deferring item emits no lone probe rows; an emission item skips rows an earlier item matched)
    auto emitted = [&](uint32_t mc) -> uint32_t { return (OJ & kOJProbe) && !pdefer ? (mc > 0u ? mc : 1u) : mc; };
    auto plive = [&](int64_t l) -> bool { return !pemit || gprobe[l] == 0; };
    // output rows of probe row l (key k); a deferring item records the row's match here, before the
    // output claim (a claim that does not fit must still leave the flags of an exact rerun's count)
    auto count_row = [&](int64_t l, KT k) -> uint32_t {
      const uint32_t mc = rj_count_mark<OJ, KT>(bst, skeys, k, flg);
      if ((OJ & kOJProbe) && pdefer && mc) gprobe[l] = 1;
      return plive(l) ? emitted(mc) : 0u;
    };
    uint32_t c = 0;
#pragma unroll
    for (int u = 0; u < kRJProbeRounds; ++u)
      if (s0 + u * kWave + lane < s1) c += count_row(s0 + u * kWave + lane, pk[u]);
    {  // later rounds' probe keys two rounds at a time (both loads in flight before either count)
      int64_t l = s0 + kRJProbeRounds * kWave + lane;
      for (; l + kWave < s1; l += 2 * kWave) {
        const KT ka = pkeys[l], kb = pkeys[l + kWave];
        c += count_row(l, ka) + count_row(l + kWave, kb);
      }
      if (l < s1) c += count_row(l, pkeys[l]);
    }
    for (int d = kWave / 2; d > 0; d >>= 1) c += __shfl_xor(c, d, kWave);
    if (lane == 0) wtot[wave] = c;
    __syncthreads();
    // unmatched build rows (flags final after the barrier above): emitted after every match, or
    // recorded for a later emission item (bdefer)
    uint32_t unm = 0;
    if ((OJ & kOJBuild) && bdefer) {
      for (int i = threadIdx.x; i < nr; i += blockDim.x)
        if (flg[i]) gbuild[rb + perm[i]] = 1;
    } else if (OJ & kOJBuild) {
      uint32_t u = 0;
      for (int i = threadIdx.x; i < nr; i += blockDim.x) u += flg[i] ? 0u : 1u;
      for (int d = kWave / 2; d > 0; d >>= 1) u += __shfl_xor(u, d, kWave);
      __shared__ uint32_t usum[kRJWaves];
      if (lane == 0) usum[wave] = u;
      __syncthreads();
#pragma unroll
      for (int w = 0; w < kRJWaves; ++w) unm += usum[w];
    }
    int64_t base = obase;
    if (out_offs == nullptr) {
      if (threadIdx.x == 0) {
        unsigned long long tot = unm;
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
    int64_t ubase = base;  // first output row of the unmatched build rows
#pragma unroll
    for (int w = 0; w < kRJWaves; ++w) ubase += wtot[w];
    for (int w = 0; w < wave; ++w) base += wtot[w];
    // ---- phase D: emit.  Round u + 1's probe row is loaded while round u expands (kn / vn), so
    // only the first round after the phase-A prefetch waits on memory.
    static_assert(kRJProbeRounds == 1, "emit prefetch assumes one phase-A round");
    KT kn = 0;
    uint64_t vn[MAXP] = {};
    for (int u = 0; s0 + (int64_t)u * kWave < s1; ++u) {
      const int64_t l = s0 + (int64_t)u * kWave + lane;
      const bool active = l < s1 && plive(l);
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
      // i0: the first match (scans for match rank j start there); pure: the matches are adjacent, so
      // match j is slot i0 + j (a hot key's chunk fills its bucket: no O(mc^2) rank scans)
      uint32_t i0 = 0, i1 = 0, mc = 0, pure = 0;
      if (active) {
        const uint32_t b = rj_bucket(k);
        i1 = bst[b + 1];
        uint32_t last = 0;
        for (uint32_t i = bst[b]; i < i1; ++i)
          if (skeys[i] == k) {
            if (mc == 0) i0 = i;
            last = i;
            ++mc;
          }
        pure = mc > 0 && last - i0 + 1 == mc;
      }
      const uint32_t ec = active ? emitted(mc) : 0u;  // output rows of this probe row
      uint32_t inc = ec;  // wave inclusive scan of output counts
#pragma unroll
      for (int d = 1; d < kWave; d <<= 1) {
        const uint32_t x = __shfl_up(inc, d, kWave);
        if (lane >= d) inc += x;
      }
      const uint32_t wsum = __shfl(inc, kWave - 1, kWave);
      const uint32_t excl = inc - ec;
      // Load-balanced expansion: lane t writes output rows base + t, base + 64 + t, ...
      // of this round, so every store covers a contiguous, fully active run of the
      // output column (a lane-per-probe-row loop over bucket entries would issue
      // sparse partial-line stores).  The producing probe lane ("owner") of row
      // s is found by a binary search over the wave's inclusive output counts and
      // its key / bucket / payload are read with cross-lane permutes.
      for (uint32_t t0 = 0; t0 < wsum; t0 += kWave) {
        const uint32_t so = t0 + lane;
        const bool act = so < wsum;
        int owner = 0;
#pragma unroll
        for (int step = kWave / 2; step >= 1; step >>= 1) {
          const uint32_t ic = __shfl(inc, owner + step - 1, kWave);
          if (ic <= so) owner += step;
        }
        const uint32_t j = so - __shfl(excl, owner, kWave);  // match rank inside the owner's bucket
        const KT ko = rj_shfl_key(k, owner);
        const uint64_t kw = key_value(ko);
        const uint32_t b0 = __shfl(i0, owner, kWave), b1 = __shfl(i1, owner, kWave);
        const bool opure = __shfl(pure, owner, kWave) != 0u;
        const bool omatched = !(OJ & kOJProbe) || __shfl(mc, owner, kWave) > 0u;
        uint64_t vo[MAXP];
#pragma unroll
        for (int q = 0; q < MAXP; ++q) vo[q] = q == pkey ? kw : (uint64_t)rj_shfl64((int64_t)v[q], owner);
        if (act) {
          int r = -1;
          if (omatched && opure)
            r = perm[b0 + j];
          else if (omatched)
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
          if ((OJ & kOJProbe) && r < 0) {  // unmatched probe row: build side null
#pragma unroll
            for (int q = 0; q < MAXB + 1; ++q)
              if (q < bo.n) stw<W8>(bo.out[q], o, bo.width[q], 0ull);
            for (int q = MAXB + 1; q < bo.n; ++q) stw<W8>(bo.out[q], o, bo.width[q], 0ull);
          } else {
#pragma unroll
            for (int q = 0; q < MAXB + 1; ++q)
              if (q < bo.n)
                stw<W8>(bo.out[q], o, bo.width[q],
                        bo.lds_off[q] < 0 ? kw : ldw<W8>(area + bo.lds_off[q], r, bo.width[q]));
            for (int q = MAXB + 1; q < bo.n; ++q)
              stw<W8>(bo.out[q], o, bo.width[q],
                      bo.lds_off[q] < 0 ? kw : ldw<W8>(area + bo.lds_off[q], r, bo.width[q]));
          }
          if (OJ & kOJProbe) bpres[o] = r >= 0 ? 1 : 0;
          if (OJ & kOJBuild) ppres[o] = 1;
        }
      }
      base += wsum;
    }
    if ((OJ & kOJBuild) && !bdefer) {  // ---- phase E: the unmatched build rows, in bucket-slot order
      __syncthreads();  // every wave is done with wtot
      int64_t at = ubase;
      for (int i0 = 0; i0 < nr; i0 += kRJThreads) {
        const int i = i0 + (int)threadIdx.x;
        const uint32_t um = (i < nr && !flg[i]) ? 1u : 0u;
        const uint32_t ex = rp_block_exscan<kRJWaves>(um, wtot);
        uint32_t tot = 0;
#pragma unroll
        for (int w = 0; w < kRJWaves; ++w) tot += wtot[w];
        if (um) {
          const int64_t o = at + ex;
          const int r = perm[i];
          const uint64_t kw = key_value(skeys[i]);
          for (int q = 0; q < pc.n; ++q) stw<W8>(pc.out[q], o, pc.width[q], q == pkey ? kw : 0ull);
          for (int q = 0; q < bo.n; ++q)
            stw<W8>(bo.out[q], o, bo.width[q], bo.lds_off[q] < 0 ? kw : ldw<W8>(area + bo.lds_off[q], r, bo.width[q]));
          ppres[o] = 0;
          if (OJ & kOJProbe) bpres[o] = 1;
        }
        at += tot;
        __syncthreads();  // wtot reused by the next round
      }
    }
  }
}

static int rj_grid(int64_t nparts) { return (int)std::min<int64_t>(nparts, kNumCUs * 8); }

void radix_join_count(const int64_t *pkeys, const int64_t *poffs, const int64_t *bkeys, const int64_t *boffs,
                      int64_t nparts, int64_t cap, int64_t *counts, int *overflow, void *stream, int64_t pstride,
                      int outer, int64_t pslot, int64_t bslot, const RJSplit *split, const int64_t *narrow_base) {
  CYLON_CHECK(cap > 0 && cap <= kRJMaxRows, Code::Invalid, "radix join capacity " << cap);
  CYLON_CHECK(pstride >= 1, Code::Invalid, "partition stride " << pstride);
  CYLON_CHECK(outer >= 0 && outer <= 3, Code::Invalid, "radix join outer mode " << outer);
  hipStream_t s = as_stream(stream);
  HIP_CHECK(hipMemsetAsync(overflow, 0, sizeof(int), s));
  const int64_t *items = split ? split->items : nullptr;
  const int64_t nitems = items ? split->nitems : 0;
  const uint8_t *skip = split ? split->skip : nullptr;
  const int64_t nsample = items ? nitems : (nparts + pstride - 1) / pstride;
  if (nsample == 0) return;
  const dim3 grid((unsigned)std::max<int64_t>(1, std::min<int64_t>(nsample, kNumCUs * 12)));
  switch (outer) {
    case 0:
      if (narrow_base)
        hipLaunchKernelGGL((k_rj_count<0, true>), grid, dim3(kRCThreads), 0, s, pkeys, poffs, bkeys, boffs, nparts,
                           (int)cap, pstride, counts, overflow, pslot, bslot, items, nitems, skip);
      else
        hipLaunchKernelGGL((k_rj_count<0, false>), grid, dim3(kRCThreads), 0, s, pkeys, poffs, bkeys, boffs, nparts,
                           (int)cap, pstride, counts, overflow, pslot, bslot, items, nitems, skip);
      break;
    case 1:
      if (narrow_base)
        hipLaunchKernelGGL((k_rj_count<1, true>), grid, dim3(kRCThreads), 0, s, pkeys, poffs, bkeys, boffs, nparts,
                           (int)cap, pstride, counts, overflow, pslot, bslot, items, nitems, skip);
      else
        hipLaunchKernelGGL((k_rj_count<1, false>), grid, dim3(kRCThreads), 0, s, pkeys, poffs, bkeys, boffs, nparts,
                           (int)cap, pstride, counts, overflow, pslot, bslot, items, nitems, skip);
      break;
    case 2:
      if (narrow_base)
        hipLaunchKernelGGL((k_rj_count<2, true>), grid, dim3(kRCThreads), 0, s, pkeys, poffs, bkeys, boffs, nparts,
                           (int)cap, pstride, counts, overflow, pslot, bslot, items, nitems, skip);
      else
        hipLaunchKernelGGL((k_rj_count<2, false>), grid, dim3(kRCThreads), 0, s, pkeys, poffs, bkeys, boffs, nparts,
                           (int)cap, pstride, counts, overflow, pslot, bslot, items, nitems, skip);
      break;
    default:
      if (narrow_base)
        hipLaunchKernelGGL((k_rj_count<3, true>), grid, dim3(kRCThreads), 0, s, pkeys, poffs, bkeys, boffs, nparts,
                           (int)cap, pstride, counts, overflow, pslot, bslot, items, nitems, skip);
      else
        hipLaunchKernelGGL((k_rj_count<3, false>), grid, dim3(kRCThreads), 0, s, pkeys, poffs, bkeys, boffs, nparts,
                           (int)cap, pstride, counts, overflow, pslot, bslot, items, nitems, skip);
  }
  HIP_LAUNCH_CHECK();
}

template <bool W8, bool DMA, int OJ>
static void rj_write_launch(dim3 grid, hipStream_t s, const int64_t *pk, const int64_t *poffs, const int64_t *bk,
                            const int64_t *boffs, int64_t nparts, int cap, const int64_t *out_offs, const ColSet &pc,
                            const ColSet &bs, const BuildOut &bo, unsigned long long *cur, int64_t out_cap,
                            int *overflow, int pkey, uint8_t *ppres, uint8_t *bpres,
                            int64_t pslot, int64_t bslot, const RJSplit &sp, const int64_t *nb) {
  if (nb)
    hipLaunchKernelGGL((k_rj_write<4, 3, W8, DMA, OJ, true>), grid, dim3(kRJThreads), 0, s, pk, poffs, bk, boffs, nparts,
                       cap, out_offs, pc, bs, bo, cur, out_cap, overflow, pkey, ppres, bpres, pslot, bslot, sp.items,
                       sp.nitems, sp.skip, sp.gprobe, sp.gbuild, nb);
  else
    hipLaunchKernelGGL((k_rj_write<4, 3, W8, DMA, OJ, false>), grid, dim3(kRJThreads), 0, s, pk, poffs, bk, boffs,
                       nparts, cap, out_offs, pc, bs, bo, cur, out_cap, overflow, pkey, ppres, bpres, pslot, bslot,
                       sp.items, sp.nitems, sp.skip, sp.gprobe, sp.gbuild, nb);
}

void radix_join_write(const int64_t *pkeys, const int64_t *poffs, const int64_t *bkeys, const int64_t *boffs,
                      int64_t nparts, int64_t cap, const int64_t *out_offs, const uint8_t *const *pin,
                      uint8_t *const *pout, const int *pw, int npc, const uint8_t *const *bin, uint8_t *const *bout,
                      const int *bw, int nbc, void *stream, int64_t *cursor, int64_t out_cap, int *overflow, int pkey,
                      int outer, uint8_t *ppres, uint8_t *bpres, int64_t pslot, int64_t bslot,
                      const RJSplit *split, const int64_t *narrow_base) {
  CYLON_CHECK(pkey >= -1 && pkey < npc, Code::Invalid, "radix join probe key column " << pkey);
  CYLON_CHECK(npc <= kMaxFusedCols && nbc <= kMaxFusedCols, Code::Invalid, "too many columns");
  CYLON_CHECK(out_offs != nullptr || (cursor != nullptr && overflow != nullptr), Code::Invalid,
              "radix join write: needs partition offsets or an output cursor");
  CYLON_CHECK(outer >= 0 && outer <= 3, Code::Invalid, "radix join outer mode " << outer);
  CYLON_CHECK(!(outer & kOJProbe) || bpres, Code::Invalid, "radix join: probe-preserving mode needs build presence");
  CYLON_CHECK(!(outer & kOJBuild) || ppres, Code::Invalid, "radix join: build-preserving mode needs probe presence");
  const RJSplit sp = split ? *split : RJSplit{};
  CYLON_CHECK(sp.nitems == 0 || (out_offs == nullptr && sp.items), Code::Invalid,
              "radix join write: split items need the cursor mode");
  if (sp.nitems + nparts == 0) return;
  const int kbytes = narrow_base ? 4 : 8;
  CYLON_CHECK(cap > 0 && cap <= radix_join_capacity(bw, bin, nbc, outer & kOJBuild, kbytes), Code::Invalid,
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
  int64_t off = (kbytes + 2) * cap;
  for (int q = 0; q < nbc; ++q)
    if (bin[q]) {
      bo.lds_off[q] = (int)off;
      off += cap * bw[q];
      bs.in[bs.n] = bin[q];
      bs.width[bs.n++] = bw[q];
    }
  bo.match_off = (int)off;
  if (outer & kOJBuild) off += cap;
  CYLON_CHECK(off <= kRJRowArea, Code::Invalid, "radix join LDS rows " << off);
  hipStream_t s = as_stream(stream);
  // probe columns beyond 4 and staged build columns beyond 3 are loaded in place (slower, correct)
  unsigned long long *cur = reinterpret_cast<unsigned long long *>(cursor);
  const dim3 grid(rj_grid(nparts + sp.nitems));
  // LDS-DMA build staging: write kernel 33.9 -> 32.9 ms per 1B x 1B join (profiles/r03/lds_dma_ab.txt)
  const bool dma = w8;
  const int ci = (int)cap;
#define RJW(W8_, DMA_, OJ_)                                                                                        \
  rj_write_launch<W8_, DMA_, OJ_>(grid, s, pkeys, poffs, bkeys, boffs, nparts, ci, out_offs, pc, bs, bo, cur, out_cap, \
                                  overflow, pkey, ppres, bpres, pslot, bslot, sp, narrow_base)
  if (outer == 0) {
    if (dma) RJW(true, true, 0);
    else if (w8) RJW(true, false, 0);
    else RJW(false, false, 0);
  } else if (outer == 1) {
    if (dma) RJW(true, true, 1);
    else RJW(false, false, 1);
  } else if (outer == 2) {
    if (dma) RJW(true, true, 2);
    else RJW(false, false, 2);
  } else {
    if (dma) RJW(true, true, 3);
    else RJW(false, false, 3);
  }
#undef RJW
  HIP_LAUNCH_CHECK();
}


// this file's code object is loaded at context creation (preload_device_code), not on first use
void preload_lds_join() { preload_code(reinterpret_cast<const void *>(&(k_rj_count<0, false>))); }

}  // namespace hip
}  // namespace cylon
