// LDS radix hash group-by for large single-integer-key aggregations (K8, gfx950).
//
// Reference behaviour: cpp/src/cylon/groupby/hash_groupby.cpp:30-190 (one
// pass over rows into a std::unordered_map of per-group aggregation states).
// On MI355X a group table far beyond the 4 MB per-XCD L2 turns every row into
// a random global atomic (~50 G accesses/s, tools/membench.hip), so this path
//   1. estimates the number of distinct keys with a HyperLogLog sketch
//      (2^14 registers, LDS-privatised per block, one pass over the keys);
//   2. radix-partitions key + value columns by the top bits of fmix64(key)
//      (radix_join.hip passes) so each partition holds ~0.6 x 4096 distinct
//      keys;
//   3. aggregates one partition per workgroup in an LDS open-addressing table
//      (64-bit LDS CAS on the key, LDS atomics for the states: f64 add, i64
//      add, u64 min/max on order-preserving images, counts), then compacts
//      the partition's groups with a block scan into a slab at the
//      partition's row offset (groups <= rows), with the group count per
//      partition;
//   4. a copy kernel packs the slabs after a device scan of the counts.
// A partition whose distinct keys overflow the table is reported and the
// caller falls back to the global path.
#include <cstdio>
#include <cstdlib>

#include "device_common.hpp"

namespace cylon {
namespace hip {

constexpr int kHllBits = 12;  // 4096 registers: 1.6% standard error, 16 KB of LDS per block
constexpr int kHllRegs = 1 << kHllBits;
constexpr int kRGThreads = 512;
constexpr int kRGWaves = kRGThreads / kWave;
constexpr int64_t kRGEmpty = INT64_MIN;  // empty-slot sentinel; the key INT64_MIN itself gets slot S

__device__ __forceinline__ void hll_add(uint32_t *r, int64_t key) {
  const uint64_t h = hashing::fmix64((uint64_t)key);
  const uint32_t idx = (uint32_t)(h >> (64 - kHllBits));
  const uint32_t rho = (uint32_t)__clzll((h << kHllBits) | (1ull << (kHllBits - 1))) + 1;
  atomicMax(&r[idx], rho);
}

// two keys per thread per step (16-byte loads); LDS-privatised registers
__global__ __launch_bounds__(kBlock) void k_hll(const int64_t *__restrict__ keys, int64_t n,
                                                uint32_t *__restrict__ regs) {
  __shared__ uint32_t r[kHllRegs];
  for (int i = threadIdx.x; i < kHllRegs; i += blockDim.x) r[i] = 0;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool vec = (reinterpret_cast<uintptr_t>(keys) & 15) == 0;
  if (vec) {
    for (int64_t i = t0; i < (n >> 1); i += stride) {
      const longlong2 k2 = reinterpret_cast<const longlong2 *>(keys)[i];
      hll_add(r, k2.x);
      hll_add(r, k2.y);
    }
    if ((n & 1) && t0 == 0) hll_add(r, keys[n - 1]);
  } else {
    for (int64_t i = t0; i < n; i += stride) hll_add(r, keys[i]);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < kHllRegs; i += blockDim.x)
    if (r[i]) atomicMax(&regs[i], r[i]);
}

double distinct_estimate(const int64_t *keys, int64_t n, uint32_t *regs, void *stream) {
  hipStream_t s = as_stream(stream);
  HIP_CHECK(hipMemsetAsync(regs, 0, sizeof(uint32_t) * kHllRegs, s));
  if (n > 0) {
    hipLaunchKernelGGL(k_hll, dim3(grid_for((n + 1) / 2, kBlock, kNumCUs * 8)), dim3(kBlock), 0, s, keys, n, regs);
    HIP_LAUNCH_CHECK();
  }
  std::vector<uint32_t> h(kHllRegs);
  HIP_CHECK(hipMemcpyAsync(h.data(), regs, sizeof(uint32_t) * kHllRegs, hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  double z = 0.0;
  int zeros = 0;
  for (uint32_t x : h) {
    z += std::ldexp(1.0, -(int)x);
    zeros += x == 0;
  }
  const double m = kHllRegs;
  double est = (0.7213 / (1.0 + 1.079 / m)) * m * m / z;
  if (est <= 2.5 * m && zeros > 0) est = m * std::log(m / zeros);  // linear counting
  return est;
}

// accumulator kinds
enum RGKind : int { RG_SUMF = 0, RG_SUMI = 1, RG_MIN = 2, RG_MAX = 3, RG_CNT = 4, RG_M2 = 5 };

constexpr int kRGMaxAcc = 8;
struct RGArgs {
  RGAccDesc acc[kRGMaxAcc];
  int nacc;
  int has_m2;  // some accumulator is RG_M2: a second pass over the partition's rows
};

__device__ __forceinline__ uint64_t rg_img(uint64_t bits, int w, int kind) {
  const int nb = 8 * w;
  const uint64_t mask = (nb == 64) ? ~0ull : ((1ull << nb) - 1);
  const uint64_t sign = 1ull << (nb - 1);
  bits &= mask;
  if (kind == static_cast<int>(ValueKind::SIGNED_INT)) return bits ^ sign;
  if (kind == static_cast<int>(ValueKind::FLOAT)) {
    if (bits == sign) bits = 0;
    return (bits & sign) ? (~bits & mask) : (bits | sign);
  }
  return bits;
}

__device__ __forceinline__ double rg_double(uint64_t b, int w, int kind) {
  if (kind == static_cast<int>(ValueKind::FLOAT)) {
    if (w == 8) return __longlong_as_double((long long)b);
    if (w == 4) return (double)__int_as_float((int)b);
    return (double)__half2float(__ushort_as_half((unsigned short)b));
  }
  if (kind == static_cast<int>(ValueKind::SIGNED_INT)) return (double)extend_bits(b, w, kind);
  return (double)b;
}

__device__ __forceinline__ uint64_t rg_init(int kind) { return kind == RG_MIN ? ~0ull : 0ull; }

template <int A, int S>
__global__ __launch_bounds__(kRGThreads) void k_rg_agg(const int64_t *__restrict__ keys,
                                                       const int64_t *__restrict__ offs, int64_t nparts, RGArgs a,
                                                       int64_t *__restrict__ okeys, uint64_t *__restrict__ oacc,
                                                       int64_t n, int64_t *__restrict__ gcount, int *overflow) {
  __shared__ int64_t tk[S + 1];
  __shared__ unsigned long long ta[A][S + 1];
  __shared__ uint32_t wsum[kRGWaves];
  __shared__ int bad;
  const int lane = lane_id(), wave = threadIdx.x / kWave;
  for (int64_t p = blockIdx.x; p < nparts; p += gridDim.x) {
    const int64_t rb = offs[p], re = offs[p + 1];
    if (rb == re) {
      if (threadIdx.x == 0) gcount[p] = 0;
      continue;
    }
    if (rb > re || re > n || rb < 0) {  // corrupt partition offsets: report, touch nothing
      if (threadIdx.x == 0) {
        atomicOr(overflow, 8);
        gcount[p] = 0;
      }
      continue;
    }
    __syncthreads();  // previous partition done with the table
    for (int s = threadIdx.x; s <= S; s += blockDim.x) {
      tk[s] = kRGEmpty;
#pragma unroll
      for (int j = 0; j < A; ++j) ta[j][s] = rg_init(a.acc[j].kind);
    }
    if (threadIdx.x == 0) bad = 0;
    __syncthreads();
    for (int64_t r = rb + threadIdx.x; r < re; r += blockDim.x) {
      const int64_t k = keys[r];
      uint64_t vb[A];
#pragma unroll
      for (int j = 0; j < A; ++j) vb[j] = load_bits(a.acc[j].src, r, a.acc[j].width);
      int slot = S;
      if (k != kRGEmpty) {
        uint32_t s = (uint32_t)hashing::fmix64((uint64_t)k) & (S - 1);
        int probes = 0;
        while (true) {
          const int64_t cur = tk[s];
          if (cur == k) break;
          if (cur == kRGEmpty) {
            const unsigned long long prev = atomicCAS(reinterpret_cast<unsigned long long *>(&tk[s]),
                                                      (unsigned long long)kRGEmpty, (unsigned long long)k);
            if (prev == (unsigned long long)kRGEmpty || prev == (unsigned long long)k) break;
            continue;  // lost the race to another key: re-read this slot
          }
          s = (s + 1) & (S - 1);
          if (++probes >= S) {
            s = S + 1;  // table full
            break;
          }
        }
        if (s > S) {
          atomicOr(&bad, 1);
          continue;
        }
        slot = (int)s;
      }  // else: the INT64_MIN key accumulates into slot S
#pragma unroll
      for (int j = 0; j < A; ++j) {
        const RGAccDesc &c = a.acc[j];
        if (c.valid && !c.valid[r]) continue;
        unsigned long long *t = &ta[j][slot];
        switch (c.kind) {
          case RG_SUMF: atomicAdd(reinterpret_cast<double *>(t), rg_double(vb[j], c.width, c.vkind)); break;
          case RG_SUMI: atomicAdd(t, (unsigned long long)extend_bits(vb[j], c.width, c.vkind)); break;
          case RG_MIN: atomicMin(t, (unsigned long long)rg_img(vb[j], c.width, c.vkind)); break;
          case RG_MAX: atomicMax(t, (unsigned long long)rg_img(vb[j], c.width, c.vkind)); break;
          case RG_M2: break;  // second pass
          default: atomicAdd(t, 1ull);
        }
      }
      if (slot == S) atomicOr(&bad, 2);  // INT64_MIN present
    }
    __syncthreads();
    if (bad & 1) {
      if (threadIdx.x == 0) {
        atomicOr(overflow, 1);
        gcount[p] = 0;
      }
      continue;
    }
    if (a.has_m2) {
      // VAR / STDDEV: squared deviations from the group mean, once every row's sum and count are
      // in (the two-pass form of the global path, groupby.cpp kM2; the partition's rows are L2 hits)
      for (int64_t r = rb + threadIdx.x; r < re; r += blockDim.x) {
        const int64_t k = keys[r];
        int slot = S;
        if (k != kRGEmpty) {
          uint32_t s = (uint32_t)hashing::fmix64((uint64_t)k) & (S - 1);
          while (tk[s] != k) s = (s + 1) & (S - 1);  // present: inserted by the first pass
          slot = (int)s;
        }
#pragma unroll
        for (int j = 0; j < A; ++j) {
          if (a.acc[j].kind != RG_M2) continue;
          const RGAccDesc &c = a.acc[j];
          if (c.valid && !c.valid[r]) continue;
          const double sum = __longlong_as_double((long long)ta[c.sum_acc][slot]);
          const double cnt = (double)(long long)ta[c.cnt_acc][slot];
          const double d = rg_double(load_bits(c.src, r, c.width), c.width, c.vkind) - sum / cnt;
          atomicAdd(reinterpret_cast<double *>(&ta[j][slot]), d * d);
        }
      }
      __syncthreads();
    }
    // compact occupied slots (+ slot S when the INT64_MIN key occurred) into the slab at rb
    constexpr int kPer = (S + kRGThreads - 1) / kRGThreads;
    uint32_t occ = 0;
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      const int s = threadIdx.x * kPer + q;
      if (s < S && tk[s] != kRGEmpty) occ |= 1u << q;
    }
    const uint32_t c = __popc(occ);
    uint32_t inc = c;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
      const uint32_t x = __shfl_up(inc, d, kWave);
      if (lane >= d) inc += x;
    }
    if (lane == kWave - 1) wsum[wave] = inc;
    __syncthreads();
    uint32_t pos = inc - c, tot = 0;
    for (int w = 0; w < kRGWaves; ++w) {
      pos += (w < wave) ? wsum[w] : 0u;
      tot += wsum[w];
    }
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      if (!(occ >> q & 1u)) continue;
      const int s = threadIdx.x * kPer + q;
      const int64_t o = rb + pos++;
      if (o >= re) {  // more groups than rows: report, write nothing
        atomicOr(overflow, 16);
        continue;
      }
      okeys[o] = tk[s];
#pragma unroll
      for (int j = 0; j < A; ++j) {
        oacc[(int64_t)j * n + o] = ta[j][s];
      }
    }
    if (threadIdx.x == 0) {
      const bool has_min = (bad & 2) != 0;
      if (has_min && rb + tot >= re) atomicOr(overflow, 16);
      if (has_min && rb + tot < re) {
        const int64_t o = rb + tot;
        okeys[o] = kRGEmpty;
        for (int j = 0; j < A; ++j) oacc[(int64_t)j * n + o] = ta[j][S];
      }
      gcount[p] = tot + (has_min ? 1 : 0);
    }
  }
}

// out[goff[p] + i] = slab[offs[p] + i] for i < count[p] (keys + nacc accumulator planes)
__global__ void k_rg_pack(const int64_t *__restrict__ offs, const int64_t *__restrict__ goff, int64_t nparts,
                          const int64_t *__restrict__ okeys, const uint64_t *__restrict__ oacc, int64_t n, int nacc,
                          int64_t *__restrict__ keys_out, uint64_t *__restrict__ acc_out, int64_t ngroups) {
  for (int64_t p = blockIdx.x; p < nparts; p += gridDim.x) {
    const int64_t src = offs[p], dst = goff[p], cnt = goff[p + 1] - dst;
    for (int64_t i = threadIdx.x; i < cnt; i += blockDim.x) {
      keys_out[dst + i] = okeys[src + i];
      for (int j = 0; j < nacc; ++j) acc_out[(int64_t)j * ngroups + dst + i] = oacc[(int64_t)j * n + src + i];
    }
  }
}

// ---- QUANTILE on the radix path.  The rows (group key, value) are partitioned
// by the group key's hash into partitions of <= kQCap rows (whole groups); one workgroup per
// partition then takes each group's order statistics:
//   1. the partition's rows are read once from HBM into LDS; a Fibonacci hash of the key picks one
//      of kQBuckets local buckets (LDS atomics count them, a block scan places them) and the rows
//      are moved to bucket order inside LDS -- a bucket holds one group (rarely a few: ~10 groups
//      per partition);
//   2. the non-empty buckets of <= kQWaveRows rows are dealt round-robin to the block's waves: a
//      one-key bucket takes the type-2 order statistics by a wave radix select over ballots
//      (q_wave_select), a mixed bucket is sorted by (key, value) in registers (q_wave_bitonic);
//      rows of larger buckets count their rank over the bucket;
//   3. the type-2 position (global path k_quantile: np = nv q, j = floor(np), pos = min(j, nv - 1),
//      the mean with the (pos - 1)-th when np is whole) is written per group at a slot from an LDS
//      counter (gcount per partition; radix_groupby_pack packs the slabs).
// Nulls rank after every value (excluded, as the global path does).  Values compare as
// order-preserving images of their doubles (NaN canonicalised).
constexpr int kQCap = 4096, kQThreads = 512, kQPer = kQCap / kQThreads, kQBBits = 11, kQBuckets = 1 << kQBBits;
constexpr int kQWaveRows = 128;  // buckets one wave sorts in registers (2 rows per lane)

// block-wide exclusive scan of one uint32 per thread
__device__ __forceinline__ uint32_t q_block_exscan(uint32_t c, uint32_t *wsum) {
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
  for (int w = 0; w < kQThreads / kWave; ++w) off += (w < wave) ? wsum[w] : 0u;
  return off + inc - c;
}

__device__ __forceinline__ uint64_t q_image(double d) {
  uint64_t b = (uint64_t)__double_as_longlong(d != d ? __longlong_as_double(0x7ff8000000000000ll) : d);
  return (b >> 63) ? ~b : (b | 0x8000000000000000ull);
}
__device__ __forceinline__ double q_unimage(uint64_t m) {
  return __longlong_as_double((long long)((m >> 63) ? (m & 0x7fffffffffffffffull) : ~m));
}

struct alignas(16) QKV {  // one row of a partition in LDS: group key, value image (~0: null)
  int64_t k;
  uint64_t v;
};

// lane ^ j exchange of a 64-bit value: DPP lane permutes (VALU source modifiers, no LDS round trip)
// where one exists -- quad_perm [1,0,3,2] / [2,3,0,1] for j = 1 / 2, row_ror:8 for j = 8 --, ds_swizzle
// (bit mode, xor mask j within 32-lane halves; no address VGPR) for j = 4, 16, ds_bpermute (__shfl_xor)
// across the halves for j = 32.  j is a constant after the bitonic loops unroll; every lane of the wave
// is active in the sorts (pads fill the bucket), so no DPP source lane is disabled.
template <int J>
__device__ __forceinline__ uint32_t q_swz(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_ds_swizzle((int)x, (J << 10) | 0x1F);
}
template <int CTRL>
__device__ __forceinline__ uint32_t q_dpp(uint32_t x) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, CTRL, 0xF, 0xF, false);
}
__device__ __forceinline__ uint64_t q_xor64(uint64_t v, int j) {
  const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  uint32_t a, b;
  switch (j) {
    case 1: a = q_dpp<0xB1>(lo); b = q_dpp<0xB1>(hi); break;    // quad_perm [1,0,3,2]
    case 2: a = q_dpp<0x4E>(lo); b = q_dpp<0x4E>(hi); break;    // quad_perm [2,3,0,1]
    case 4: a = q_swz<4>(lo); b = q_swz<4>(hi); break;
    case 8: a = q_dpp<0x128>(lo); b = q_dpp<0x128>(hi); break;  // row_ror:8 = lane ^ 8 in a row
    case 16: a = q_swz<16>(lo); b = q_swz<16>(hi); break;
    default: return (uint64_t)__shfl_xor((unsigned long long)v, j);
  }
  return (uint64_t)a | ((uint64_t)b << 32);
}

__device__ __forceinline__ bool q_less(int64_t ak, uint64_t av, int64_t bk, uint64_t bv) {
  return ak != bk ? ak < bk : av < bv;
}

// Bitonic sort of 64 * S (key, value) rows held by one wave, element e = s * 64 + lane in slot s of
// lane `lane`: distances < 64 exchange through cross-lane shuffles, distance >= 64 inside the lane.
// Fully unrolled (constant shuffle distances and direction masks): the rolled form measured 89 vs
// 77 ms per 1B-row call, although unrolled the compiler spills lane masks through v_readlane.
template <int S>
__device__ __forceinline__ void q_wave_bitonic(int64_t (&k)[S], uint64_t (&v)[S]) {
  const int lane = lane_id();
#pragma unroll
  for (int kk = 2; kk <= 64 * S; kk <<= 1) {
#pragma unroll
    for (int j = kk >> 1; j > 0; j >>= 1) {
      if (j >= 64) {
        const int js = j >> 6;
#pragma unroll
        for (int s = 0; s < S; ++s) {
          if (s & js) continue;  // the pair (s, s | js), handled from its lower slot
          const int t = s | js;
          const bool asc = ((s * 64 + lane) & kk) == 0;
          if (q_less(k[t], v[t], k[s], v[s]) == asc) {
            const int64_t tk = k[s];
            const uint64_t tv = v[s];
            k[s] = k[t];
            v[s] = v[t];
            k[t] = tk;
            v[t] = tv;
          }
        }
      } else {
#pragma unroll
        for (int s = 0; s < S; ++s) {
          const int64_t ok = (int64_t)q_xor64((uint64_t)k[s], j);
          const uint64_t ov = q_xor64(v[s], j);
          const bool asc = ((s * 64 + lane) & kk) == 0, lower = (lane & j) == 0;
          const bool take = lower == asc ? q_less(ok, ov, k[s], v[s]) : q_less(k[s], v[s], ok, ov);
          if (take) {
            k[s] = ok;
            v[s] = ov;
          }
        }
      }
    }
  }
}

// Output of one group (a writer row): its slot comes from the partition's LDS counter, so the
// groups of a partition come out in no fixed order (group-by order is unspecified).  FUSE: the
// valid values' sum, count, min and max go to the four fz planes at the same slot.
template <bool FUSE>
__device__ __forceinline__ void q_emit(unsigned int *nout, int64_t *okeys, uint64_t *oq, uint64_t *ovalid,
                                       uint64_t *fz, int64_t n, int64_t b, int64_t key, bool has, double qv,
                                       double sum, int64_t cnt, double mn, double mx) {
  const int64_t g = b + (int64_t)atomicAdd(nout, 1u);
  okeys[g] = key;
  oq[g] = has ? (uint64_t)__double_as_longlong(qv) : 0ull;
  ovalid[g] = has ? 1ull : 0ull;
  if constexpr (FUSE) {
    fz[g] = (uint64_t)__double_as_longlong(sum);
    fz[n + g] = (uint64_t)cnt;
    fz[2 * n + g] = has ? (uint64_t)__double_as_longlong(mn) : 0ull;
    fz[3 * n + g] = has ? (uint64_t)__double_as_longlong(mx) : 0ull;
  }
}

// Wave-uniform copy of a value every lane holds (readfirstlane of both halves): keeps the select's
// loop counters and branches scalar.
__device__ __forceinline__ uint64_t q_uniform64(uint64_t x) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32));
  return (uint64_t)lo | ((uint64_t)hi << 32);
}

// One word (W = 1: high 32 bits, 0: low) of the wave radix select below: per bit, the candidates
// with a 0 there (a ballot per slot) keep the order statistic if more than k of them remain, else
// the 1s do with k reduced; stops once one candidate is left.  Bits, counts and masks are scalar.
template <int S, int W>
__device__ __forceinline__ void q_select_word(const uint64_t (&v)[S], uint64_t (&A)[S], uint32_t &k, uint32_t &na,
                                              int top) {
  for (int bit = top; bit >= 0 && na > 1; --bit) {
    const uint32_t m = 1u << bit;
    uint64_t z[S];
    uint32_t c = 0;
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const uint32_t w = W ? (uint32_t)(v[s] >> 32) : (uint32_t)v[s];
      z[s] = __ballot((w & m) == 0u) & A[s];
      c += (uint32_t)__popcll(z[s]);
    }
    if (k < c) {
#pragma unroll
      for (int s = 0; s < S; ++s) A[s] = z[s];
      na = c;
    } else {
#pragma unroll
      for (int s = 0; s < S; ++s) A[s] &= ~z[s];
      k -= c;
      na -= c;
    }
  }
}

// The k-th smallest (0-based, k < nv) of the wave's valid values (v != the null image ~0; pads are
// ~0 too) by an MSB-first radix select over ballots, starting at hb, the highest bit in which the
// valid values' min and max differ (every valid value shares the bits above it).  Replaces the
// bitonic sort of a single-key bucket: ~10-20 scalar-heavy bit steps instead of 28 exchange stages.
template <int S>
__device__ __forceinline__ uint64_t q_wave_select(const uint64_t (&v)[S], uint32_t k, uint32_t nv, int hb) {
  uint64_t A[S];
#pragma unroll
  for (int s = 0; s < S; ++s) A[s] = __ballot(v[s] != ~0ull);
  uint32_t na = nv;
  if (hb >= 32) q_select_word<S, 1>(v, A, k, na, hb - 32);
  q_select_word<S, 0>(v, A, k, na, hb >= 32 ? 31 : hb);
  // one candidate left, or several equal ones (all bits from hb down decided): the first of them
  uint64_t r = 0;
  bool found = false;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    if (!found && A[s] != 0ull) {
      const int l = __builtin_ctzll(A[s]);
      const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v[s], l);
      const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(v[s] >> 32), l);
      r = (uint64_t)lo | ((uint64_t)hi << 32);
      found = true;
    }
  }
  return r;
}

// One wave ranks one bucket of sz <= 64 * S rows (slots [e0, e0 + sz) of skv).  A bucket of one key
// (nearly all) takes its order statistics by q_wave_select, min / max / sum by wave reductions, and
// lane 0 emits it.  Otherwise: sort by (key, value)
// -- pads (the bucket's largest key, the null image) sort after every real row and tie only with
// that key's null rows, whose content they share -- then each group's rows are contiguous with its
// valid values first in value order, so the type-2 position is index arithmetic.  The sorted rows go
// back to skv, and each group's LAST valid row (its first row when every value is null) emits the
// group: the quantile rows are read back from skv at start + pos (and pos - 1); FUSE: the sum from a
// segmented wave scan, min / max the first / last valid values.
template <int S, bool FUSE>
__device__ __forceinline__ void q_rank_bucket(QKV *skv, int e0, int sz, double q, unsigned int *nout, int64_t *okeys,
                                              uint64_t *oq, uint64_t *ovalid, uint64_t *fz, int64_t n, int64_t b) {
  const int lane = lane_id();
  int64_t k[S];
  uint64_t v[S];
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int e = s * 64 + lane;
    if (e < sz) {
      const QKV r = skv[e0 + e];
      k[s] = r.k;
      v[s] = r.v;
    }
  }
  // one key?  Row 0 always exists (sz >= 1): one compare per row and a ballot against its key
  const int64_t k0 = (int64_t)q_uniform64((uint64_t)k[0]);
  bool other = false;
#pragma unroll
  for (int s = 0; s < S; ++s)
    if (s * 64 + lane < sz) other |= k[s] != k0;
  if (__ballot(other) == 0ull) {  // one group (nearly every bucket): order statistics by a wave radix select
    const int64_t kmax = k0;
#pragma unroll
    for (int s = 0; s < S; ++s)
      if (s * 64 + lane >= sz) v[s] = ~0ull;
    uint32_t nv = 0;
    double sum = 0.0;
    uint64_t mn = ~0ull, mx = 0;  // smallest / largest valid image (every valid image is > 0)
#pragma unroll
    for (int s = 0; s < S; ++s) {
      const bool ok = v[s] != ~0ull;
      nv += (uint32_t)__popcll(__ballot(ok));
      if constexpr (FUSE) sum += ok ? q_unimage(v[s]) : 0.0;
      if (ok) {
        mn = v[s] < mn ? v[s] : mn;
        mx = v[s] > mx ? v[s] : mx;
      }
    }
#pragma unroll
    for (int j = 1; j < 64; j <<= 1) {
      const uint64_t a = q_xor64(mn, j), c = q_xor64(mx, j);
      mn = a < mn ? a : mn;
      mx = c > mx ? c : mx;
      if constexpr (FUSE) sum += __longlong_as_double((long long)q_xor64((uint64_t)__double_as_longlong(sum), j));
    }
    if (nv == 0) {
      if (lane == 0) q_emit<FUSE>(nout, okeys, oq, ovalid, fz, n, b, kmax, false, 0.0, 0.0, 0, 0.0, 0.0);
      return;
    }
    mn = q_uniform64(mn);
    mx = q_uniform64(mx);
    const double np = (double)nv * q, jf = floor(np);
    const bool whole = np == jf;
    int pos = (int)jf;
    if (pos >= (int)nv) pos = (int)nv - 1;
    pos = __builtin_amdgcn_readfirstlane(pos);
    uint64_t at = mn, below = mn;
    if (mn != mx) {
      at = q_wave_select<S>(v, (uint32_t)pos, nv, 63 - __builtin_clzll(mn ^ mx));
      below = at;
      if (whole && pos > 0) {  // the (pos - 1)-th: the largest value below `at`, unless `at` repeats
        uint32_t cl = 0;
        uint64_t bm = 0;
#pragma unroll
        for (int s = 0; s < S; ++s) {
          const bool lt = v[s] < at;  // (nulls and pads, ~0, never are)
          cl += (uint32_t)__popcll(__ballot(lt));
          if (lt) bm = v[s] > bm ? v[s] : bm;
        }
        if (cl >= (uint32_t)pos) {
#pragma unroll
          for (int j = 1; j < 64; j <<= 1) {
            const uint64_t a = q_xor64(bm, j);
            bm = a > bm ? a : bm;
          }
          below = q_uniform64(bm);
        }
      }
    }
    if (lane == 0) {  // the group's row
      const double qv = (whole && pos > 0) ? 0.5 * (q_unimage(below) + q_unimage(at)) : q_unimage(at);
      q_emit<FUSE>(nout, okeys, oq, ovalid, fz, n, b, kmax, true, qv, sum, (int64_t)nv, q_unimage(mn), q_unimage(mx));
    }
    return;
  }
  int64_t kmax = INT64_MIN;  // pads take the bucket's largest key
#pragma unroll
  for (int s = 0; s < S; ++s)
    if (s * 64 + lane < sz) kmax = k[s] > kmax ? k[s] : kmax;
#pragma unroll
  for (int j = 1; j < 64; j <<= 1) {
    const int64_t x = (int64_t)q_xor64((uint64_t)kmax, j);
    kmax = x > kmax ? x : kmax;
  }
#pragma unroll
  for (int s = 0; s < S; ++s)
    if (s * 64 + lane >= sz) {
      k[s] = kmax;
      v[s] = ~0ull;
    }
  q_wave_bitonic<S>(k, v);
  bool head[S], last_valid[S];
  int start[S];
  double sum[S];
  int carry = 0;
  double scarry = 0.0;
#pragma unroll
  for (int s = 0; s < S; ++s) {
    int64_t pk = __shfl_up((long long)k[s], 1), nk = __shfl_down((long long)k[s], 1);
    uint64_t nvv = (uint64_t)__shfl_down((unsigned long long)v[s], 1);
    if (s > 0) {
      const int64_t lk = __shfl((long long)k[s - 1], 63);
      if (lane == 0) pk = lk;
    }
    if (s + 1 < S) {
      const int64_t fk = __shfl((long long)k[s + 1], 0);
      const uint64_t fv = (uint64_t)__shfl((unsigned long long)v[s + 1], 0);
      if (lane == 63) {
        nk = fk;
        nvv = fv;
      }
    }
    const int e = s * 64 + lane;
    head[s] = e == 0 || k[s] != pk;
    last_valid[s] = v[s] != ~0ull && (e == 64 * S - 1 || nk != k[s] || nvv == ~0ull);
    int st = head[s] ? e : 0;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const int x = __shfl_up(st, d);
      if (lane >= d) st = x > st ? x : st;
    }
    st = st > carry ? st : carry;
    start[s] = st;
    carry = __shfl(st, 63);
    if constexpr (FUSE) {  // segmented inclusive sum of the valid values (nulls and pads add 0)
      double x = v[s] != ~0ull ? q_unimage(v[s]) : 0.0;
      bool f = head[s];
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const double y = __shfl_up(x, d);
        const int g = __shfl_up((int)f, d);
        if (lane >= d && !f) {
          x += y;
          f = g != 0;
        }
      }
      if (!f) x += scarry;
      sum[s] = x;
      scarry = __shfl(x, 63);
    }
  }
#pragma unroll
  for (int s = 0; s < S; ++s)
    if (s * 64 + lane < sz) skv[e0 + s * 64 + lane] = QKV{k[s], v[s]};
  __builtin_amdgcn_wave_barrier();  // (one wave's LDS writes complete in order before its reads)
#pragma unroll
  for (int s = 0; s < S; ++s) {
    const int e = s * 64 + lane;
    if (e >= sz) continue;
    if (head[s] && v[s] == ~0ull) {  // every value of the group is null (valid values sort first)
      q_emit<FUSE>(nout, okeys, oq, ovalid, fz, n, b, k[s], false, 0.0, 0.0, 0, 0.0, 0.0);
      continue;
    }
    if (!last_valid[s]) continue;
    const int nv = e - start[s] + 1;
    const double np = (double)nv * q, jf = floor(np);
    const bool whole = np == jf;
    int pos = (int)jf;
    if (pos >= nv) pos = nv - 1;
    const double at = q_unimage(skv[e0 + start[s] + pos].v);
    const double qv = (whole && pos > 0) ? 0.5 * (q_unimage(skv[e0 + start[s] + pos - 1].v) + at) : at;
    double mn = 0.0;
    if constexpr (FUSE) mn = q_unimage(skv[e0 + start[s]].v);
    q_emit<FUSE>(nout, okeys, oq, ovalid, fz, n, b, k[s], true, qv, FUSE ? sum[s] : 0.0, nv, mn, q_unimage(v[s]));
  }
}

// 72 KB of LDS (the partition's rows as 16-byte (key, value) pairs, bucket counters): two blocks per
// CU.  Per partition: the rows are read ONCE from HBM into LDS (input order, bucket counts by LDS
// atomics), moved to bucket order inside LDS, ranked (a wave per bucket of <= kQWaveRows rows; every
// row of a larger bucket counts its rank over the bucket), and each group is written by one row at
// a slot from an LDS counter -- one HBM round trip and six barriers per partition.
template <bool FUSE>
__global__ __launch_bounds__(kQThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_rg_quantile(
    const int64_t *__restrict__ keys, const uint8_t *__restrict__ vals, int vwidth, int vkind,
    const uint8_t *__restrict__ valid, const int64_t *__restrict__ offs, int64_t nparts, int bits, double q,
    int64_t *__restrict__ okeys, uint64_t *__restrict__ oq, uint64_t *__restrict__ ovalid,
    uint64_t *__restrict__ fz, int64_t n, int64_t *__restrict__ gcount, int *__restrict__ overflow) {
  __shared__ QKV skv[kQCap];            // rows (input order, then bucket order)
  __shared__ uint32_t bcnt[kQBuckets];  // rows per bucket, then the bucket's first slot
  __shared__ uint32_t wsum[kQThreads / kWave];
  __shared__ unsigned int s_nout;       // groups emitted by this partition
  __shared__ uint16_t sbl[kQBuckets];   // the partition's buckets of <= kQWaveRows rows, compacted
  __shared__ int s_big;                 // the partition has a bucket of > kQWaveRows rows
  // bucket of a key inside its partition: a Fibonacci hash of the key's folded halves (one 32-bit
  // multiply, not a second fmix64 per row; the partition itself came from the fmix64 bits, so the
  // two are independent).  Keys that share a bucket take the mixed (key, value) path, still exact.
  (void)bits;
  auto bucket_of = [](int64_t k) -> uint32_t {
    const uint32_t f = (uint32_t)(uint64_t)k ^ (uint32_t)((uint64_t)k >> 32);
    return (f * 0x9E3779B1u) >> (32 - kQBBits);
  };
  // the bucket counters and flags start zeroed; every partition zeroes them again for the next one
  // before its trailing barrier (no barrier of its own for the reset)
  for (int i = threadIdx.x; i < kQBuckets; i += kQThreads) bcnt[i] = 0;
  if (threadIdx.x == 0) {
    s_nout = 0;
    s_big = 0;
  }
  __syncthreads();
  for (int64_t p = blockIdx.x; p < nparts; p += gridDim.x) {
    const int64_t b = offs[p], cnt = offs[p + 1] - b;
    if (cnt > kQCap) {  // (block-uniform: the LDS state stays zeroed)
      if (threadIdx.x == 0) {
        atomicOr(overflow, 1);
        gcount[p] = 0;
      }
      continue;
    }
    uint32_t rbk[kQPer];  // bucket << 16 | slot in the bucket (~0: no row)
#pragma unroll
    for (int u = 0; u < kQPer; ++u) rbk[u] = 0xffffffffu;
    if (vwidth == 8) {
      // 8-byte values (float64 / int64): two rows per thread per batch, every key, value and
      // validity load of the batch issued before any is used (the value is loaded whether or not
      // the row is null), so a typical partition (<= 1024 rows) costs one HBM latency, not a
      // chain of dependent ones per row round
      const uint64_t *v8 = reinterpret_cast<const uint64_t *>(vals);
#pragma unroll
      for (int u0 = 0; u0 < kQPer; u0 += 2) {
        int64_t kk[2];
        uint64_t raw[2];
        bool ok[2];
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int i = (u0 + t) * kQThreads + threadIdx.x;
          if (i < cnt) {
            kk[t] = keys[b + i];
            raw[t] = v8[b + i];
            ok[t] = valid == nullptr || valid[b + i];
          }
        }
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int i = (u0 + t) * kQThreads + threadIdx.x;
          if (i < cnt) {
            skv[i] = QKV{kk[t], ok[t] ? q_image(rg_double(raw[t], 8, vkind)) : ~0ull};
            const uint32_t bk = bucket_of(kk[t]);
            rbk[u0 + t] = bk << 16 | atomicAdd(&bcnt[bk], 1u);
          }
        }
        if ((u0 + 2) * kQThreads >= cnt) break;
      }
    } else {
#pragma unroll
      for (int u = 0; u < kQPer; ++u) {
        const int i = u * kQThreads + threadIdx.x;
        if (i < cnt) {
          const int64_t kk = keys[b + i];
          const uint64_t vv = (valid == nullptr || valid[b + i])
                                  ? q_image(rg_double(load_bits(vals, b + i, vwidth), vwidth, vkind))
                                  : ~0ull;
          skv[i] = QKV{kk, vv};
          const uint32_t bk = bucket_of(kk);
          rbk[u] = bk << 16 | atomicAdd(&bcnt[bk], 1u);
        }
      }
    }
    __syncthreads();
    {  // bucket first slots (exclusive scan; kQBuckets / kQThreads buckets per thread)
      constexpr int BPT = kQBuckets / kQThreads;
      uint32_t c[BPT], tot = 0;
#pragma unroll
      for (int j = 0; j < BPT; ++j) {
        c[j] = bcnt[threadIdx.x * BPT + j];
        tot += c[j];
      }
      uint32_t ex = q_block_exscan(tot, wsum);
#pragma unroll
      for (int j = 0; j < BPT; ++j) {
        bcnt[threadIdx.x * BPT + j] = ex;
        ex += c[j];
      }
    }
    {  // input order -> bucket order, inside LDS
      QKV r[kQPer];
#pragma unroll
      for (int u = 0; u < kQPer; ++u)
        if (rbk[u] != 0xffffffffu) r[u] = skv[u * kQThreads + threadIdx.x];
      __syncthreads();  // (also orders the scan's bcnt writes before the reads below)
#pragma unroll
      for (int u = 0; u < kQPer; ++u)
        if (rbk[u] != 0xffffffffu) skv[bcnt[rbk[u] >> 16] + (rbk[u] & 0xffffu)] = r[u];
    }
    __syncthreads();
    // buckets of <= kQWaveRows rows (nearly all: a bucket holds one group, rarely a few): one wave
    // sorts each.  The non-empty ones are listed first (ballots + a block scan over the waves) and
    // dealt round-robin, so every wave sorts ~(buckets / 8) of them: a partition's ~10 groups per 8
    // waves, instead of whichever waves' bucket ranges they hash into (PMC: 75 % of wave cycles
    // waiting, mostly at the barrier behind the busiest wave)
    const int wave = threadIdx.x / kWave, lane = lane_id();
    {
      constexpr int PER = kQBuckets / (kQThreads / kWave);  // buckets a wave lists
      uint64_t mk[PER / kWave];
      uint32_t mine = 0;
      bool big = false;
#pragma unroll
      for (int c = 0; c < PER / kWave; ++c) {
        const int bk = wave * PER + c * kWave + lane;
        const int szl = (bk + 1 < kQBuckets ? (int)bcnt[bk + 1] : (int)cnt) - (int)bcnt[bk];
        mk[c] = __ballot(szl > 0 && szl <= kQWaveRows);
        mine += (uint32_t)__popcll(mk[c]);
        big |= szl > kQWaveRows;
      }
      if (lane == 0) wsum[wave] = mine;
      if (big) s_big = 1;
      __syncthreads();
      uint32_t at = 0, tot = 0;
#pragma unroll
      for (int w = 0; w < kQThreads / kWave; ++w) {
        at += w < wave ? wsum[w] : 0u;
        tot += wsum[w];
      }
#pragma unroll
      for (int c = 0; c < PER / kWave; ++c) {
        if ((mk[c] >> lane) & 1ull) sbl[at + (uint32_t)__popcll(mk[c] & lanemask_lt())] = (uint16_t)(wave * PER + c * kWave + lane);
        at += (uint32_t)__popcll(mk[c]);
      }
      __syncthreads();
      for (uint32_t j = wave; j < tot; j += kQThreads / kWave) {
        const int bk = sbl[j];
        const int e0 = (int)bcnt[bk], sz = (bk + 1 < kQBuckets ? (int)bcnt[bk + 1] : (int)cnt) - e0;
        if (sz <= 64) q_rank_bucket<1, FUSE>(skv, e0, sz, q, &s_nout, okeys, oq, ovalid, fz, n, b);
        else q_rank_bucket<2, FUSE>(skv, e0, sz, q, &s_nout, okeys, oq, ovalid, fz, n, b);
      }
    }
    // rows of larger buckets (never touched by the wave phase): every row counts its rank over its
    // bucket; the row at the type-2 position emits the group.  Skipped (block-uniform s_big, written
    // before the listing's barriers) when the partition has none -- nearly always.
#pragma unroll 1
    for (int u = 0; u < (s_big ? kQPer : 0); ++u) {
      const int i = u * kQThreads + threadIdx.x;  // slot in bucket order
      if (i >= cnt) break;
      const QKV me = skv[i];
      const int64_t k = me.k;
      const uint64_t v = me.v;
      const uint32_t bk = bucket_of(k);
      const int e0 = (int)bcnt[bk], e1 = bk + 1 < (uint32_t)kQBuckets ? (int)bcnt[bk + 1] : (int)cnt;
      if (e1 - e0 <= kQWaveRows) continue;
      int rank = 0, nv = 0, lead = 1;  // lead: no earlier row of this key
      uint64_t below = 0;              // the largest valid value ranked just below (0: none -- every
                                       // valid image is > 0, the null image ~0 the largest)
      double gsum = 0.0;               // FUSE: the group's valid sum / smallest / largest image
      uint64_t gmin = ~0ull, gmax = 0;
#pragma unroll 1
      for (int j = e0; j < e1; j += 4) {
        QKV r[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) r[t] = j + t < e1 ? skv[j + t] : QKV{k ^ 1, 0};
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          if (r[t].k != k) continue;
          const int jj = j + t;
          const uint64_t vj = r[t].v;
          lead &= jj >= i;
          nv += vj != ~0ull;
          if constexpr (FUSE) {
            if (vj != ~0ull) {
              gsum += q_unimage(vj);
              gmin = vj < gmin ? vj : gmin;
              gmax = vj > gmax ? vj : gmax;
            }
          }
          if (vj < v || (vj == v && jj < i)) {
            ++rank;
            if (vj != ~0ull && vj > below) below = vj;
          }
        }
      }
      if (nv == 0) {  // every value of the group is null: its first row emits a null quantile
        if (lead) q_emit<FUSE>(&s_nout, okeys, oq, ovalid, fz, n, b, k, false, 0.0, 0.0, 0, 0.0, 0.0);
        continue;
      }
      if (v == ~0ull) continue;
      const double np = (double)nv * q, jf = floor(np);
      const bool whole = np == jf;  // (a comparison: `np - j == 0` is contracted into an fma)
      int pos = (int)jf;
      if (pos >= nv) pos = nv - 1;
      if (rank != pos) continue;
      const double qv = (whole && pos > 0) ? 0.5 * (q_unimage(below) + q_unimage(v)) : q_unimage(v);
      q_emit<FUSE>(&s_nout, okeys, oq, ovalid, fz, n, b, k, true, qv, gsum, nv, q_unimage(gmin), q_unimage(gmax));
    }
    __syncthreads();  // every read of bcnt / skv / s_nout of this partition is done
    for (int i = threadIdx.x; i < kQBuckets; i += kQThreads) bcnt[i] = 0;
    if (threadIdx.x == 0) {
      gcount[p] = s_nout;
      s_nout = 0;
      s_big = 0;
    }
    __syncthreads();  // (zeroed state and skv reused by the next partition)
  }
}

int64_t radix_quantile_capacity() { return kQCap; }

void radix_groupby_quantile(const int64_t *keys, const uint8_t *vals, int vwidth, int vkind, const uint8_t *valid,
                            const int64_t *offs, int64_t nparts, int bits, double q, int64_t *okeys, uint64_t *oq,
                            uint64_t *ovalid, int64_t *gcount, int *overflow, void *stream, uint64_t *fused,
                            int64_t n) {
  hipStream_t s = as_stream(stream);
  HIP_CHECK(hipMemsetAsync(overflow, 0, sizeof(int), s));
  if (nparts == 0) return;
  const int grid = (int)std::min<int64_t>(nparts, 16 * 256);
  if (fused)
    hipLaunchKernelGGL(k_rg_quantile<true>, dim3(grid), dim3(kQThreads), 0, s, keys, vals, vwidth, vkind, valid, offs,
                       nparts, bits, q, okeys, oq, ovalid, fused, n, gcount, overflow);
  else
    hipLaunchKernelGGL(k_rg_quantile<false>, dim3(grid), dim3(kQThreads), 0, s, keys, vals, vwidth, vkind, valid, offs,
                       nparts, bits, q, okeys, oq, ovalid, fused, n, gcount, overflow);
  HIP_LAUNCH_CHECK();
}

int64_t distinct_estimate_workspace() { return kHllRegs; }

template <int A, int S>
static void rg_launch(int grid, hipStream_t s, const int64_t *keys, const int64_t *offs, int64_t nparts,
                      const RGArgs &a, int64_t *okeys, uint64_t *oacc, int64_t n, int64_t *gcount, int *overflow) {
  hipLaunchKernelGGL((k_rg_agg<A, S>), dim3(grid), dim3(kRGThreads), 0, s, keys, offs, nparts, a, okeys, oacc, n,
                     gcount, overflow);
}

// Accumulator planes (oacc holds planes * n words): 1-4 accumulators use their own table instance,
// 5-8 the 8-plane one (idle planes are real counts of their own)
int radix_groupby_planes(int nacc) { return nacc <= 4 ? nacc : kRGMaxAcc; }

// Every accumulator slot of a table instance is live: A == planes, and a padded slot is a real
// count (src = the keys) writing its own plane.  Round 3 ran two accumulators in the <3, 2048>
// table and guarded the idle slot with `j < nacc`; hipcc (ROCm 7.2, gfx950) materialised that
// uniform guard as a lane mask inside the table-init loop, whose last trip (slot S of S + 1)
// runs with one lane active, and reused the mask for the compaction stores under another EXEC:
// the idle slot's store to oacc[2n + o] then executed past the 2n-word allocation
// (profiles/r04/rg_agg_fault_isa.txt).  Without runtime slot guards nothing can mis-evaluate.
void radix_groupby_agg(const int64_t *keys, const int64_t *offs, int64_t nparts, const RGAccDesc *acc, int nacc,
                       int64_t *okeys, uint64_t *oacc, int64_t n, int64_t *gcount, int *overflow, void *stream) {
  CYLON_CHECK(nacc >= 1 && nacc <= kRGMaxAcc, Code::Invalid, "radix group-by: 1 to 8 accumulators");
  const int A = radix_groupby_planes(nacc);
  RGArgs a;
  a.nacc = A;
  a.has_m2 = 0;
  for (int j = 0; j < kRGMaxAcc; ++j) {
    const bool real = j < nacc;
    a.acc[j].src = real && acc[j].src ? acc[j].src : reinterpret_cast<const uint8_t *>(keys);
    a.acc[j].valid = real ? acc[j].valid : nullptr;
    a.acc[j].kind = real ? acc[j].kind : RG_CNT;
    a.acc[j].width = real && acc[j].src ? acc[j].width : 8;
    a.acc[j].vkind = real ? acc[j].vkind : 0;
    a.acc[j].sum_acc = real ? acc[j].sum_acc : 0;
    a.acc[j].cnt_acc = real ? acc[j].cnt_acc : 0;
    if (real && acc[j].kind == RG_M2) {
      CYLON_CHECK(acc[j].src && acc[j].sum_acc >= 0 && acc[j].sum_acc < nacc && acc[j].cnt_acc >= 0 &&
                      acc[j].cnt_acc < nacc && acc[acc[j].sum_acc].kind == RG_SUMF &&
                      acc[acc[j].cnt_acc].kind == RG_CNT,
                  Code::Invalid, "radix group-by: M2 accumulator needs its column's sum and count");
      a.has_m2 = 1;
    }
  }
  hipStream_t s = as_stream(stream);
  HIP_CHECK(hipMemsetAsync(overflow, 0, sizeof(int), s));
  const int grid = (int)std::min<int64_t>(nparts, kNumCUs * 4);
  switch (A) {
    case 1: rg_launch<1, 4096>(grid, s, keys, offs, nparts, a, okeys, oacc, n, gcount, overflow); break;
    case 2: rg_launch<2, 2048>(grid, s, keys, offs, nparts, a, okeys, oacc, n, gcount, overflow); break;
    case 3: rg_launch<3, 2048>(grid, s, keys, offs, nparts, a, okeys, oacc, n, gcount, overflow); break;
    case 4: rg_launch<4, 1024>(grid, s, keys, offs, nparts, a, okeys, oacc, n, gcount, overflow); break;
    default: rg_launch<kRGMaxAcc, 1024>(grid, s, keys, offs, nparts, a, okeys, oacc, n, gcount, overflow);
  }
  HIP_LAUNCH_CHECK();
}

int64_t radix_groupby_slots(int nacc) { return nacc <= 1 ? 4096 : (nacc <= 3 ? 2048 : 1024); }  // (5-8: 1024)

void radix_groupby_pack(const int64_t *offs, const int64_t *goff, int64_t nparts, const int64_t *okeys,
                        const uint64_t *oacc, int64_t n, int nacc, int64_t *keys_out, uint64_t *acc_out,
                        int64_t ngroups, void *stream) {
  const int grid = (int)std::min<int64_t>(nparts, kNumCUs * 8);
  hipLaunchKernelGGL(k_rg_pack, dim3(grid), dim3(kBlock), 0, as_stream(stream), offs, goff, nparts, okeys, oacc, n,
                     nacc, keys_out, acc_out, ngroups);
  HIP_LAUNCH_CHECK();
}

// this file's code object is loaded at context creation (preload_device_code), not on first use
void preload_radix_groupby() { preload_code(reinterpret_cast<const void *>(&k_hll)); }

}  // namespace hip
}  // namespace cylon
