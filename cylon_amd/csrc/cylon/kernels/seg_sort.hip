// LDS segment sort: the last stage of the MSD keys-only sort (ops/sort.cpp radix_sort_keys_msd).
//
// Two histogram-free MSD slot passes (radix_join.hip radix_sort_msd_*_pass) leave every 8-byte
// order image in one of 2^bits partitions of at most kSegCap rows (partition p at row p * slot,
// counts[p] rows), partitions in key order.  Here one 512-thread workgroup sorts a whole partition
// inside LDS by the image bits below the MSD digits -- stable LSD rounds of <= 9 bits, ranked with
// per-wave 16-bit LDS counters (gfx950 returns one instruction's same-address LDS atomics in lane
// order: radix_join.hip lds_lane_order_ok) -- and writes it once, coalesced, at its output offset.
// A 2B-key sort then moves its keys through HBM three times (two MSD passes + this kernel) instead
// of seven times (one per 9-bit LSD pass); the LSD rounds here touch only LDS.
// Reference: the reference sorts with arrow::compute::SortIndices (cpp/src/cylon/util/arrow_utils.cpp:30-108).
#include "radix_common.hpp"

namespace cylon {
namespace hip {

constexpr int kSegThreads = 512, kSegWaves = kSegThreads / kWave, kSegItems = 12;
constexpr int kSegCap = kSegThreads * kSegItems;  // 6144 keys per partition
constexpr int kSegBits = 9, kSegBuckets = 1 << kSegBits;

int64_t seg_sort_capacity() { return kSegCap; }

// Row r of a partition is held by wave r / (64 * kSegItems), round (r / 64) % kSegItems, lane r % 64;
// within a wave the rounds rank in order and the lanes of a round in lane order, so equal digits keep
// their row order (stable) and every round's LDS / global access is one contiguous 64-row run.
struct SegRank {
  uint32_t *wcnt;  // [kSegWaves][kSegBuckets] 16-bit counters, packed in pairs
  uint32_t *toff;  // [kSegBuckets + 1] digit offsets
  uint32_t *wsum;
};

// one counting round over the digit (key - sub) >> shift & dmask: keys scattered into buf in digit
// order (stable); toff[d] = first row of digit d, toff[kSegBuckets] = c
__device__ __forceinline__ void seg_round(const SegRank &R, uint64_t *buf, const uint64_t (&k)[kSegItems], int c,
                                          int rbase, int wave, uint64_t sub, int shift, uint32_t dmask) {
  uint16_t *wc16 = reinterpret_cast<uint16_t *>(R.wcnt);
  for (int w = threadIdx.x; w < kSegWaves * kSegBuckets / 2; w += kSegThreads) R.wcnt[w] = 0u;
  __syncthreads();  // (also: earlier reads of buf are done)
  uint32_t dr[kSegItems];  // digit << 16 | rank inside this wave's rows of the digit
#pragma unroll
  for (int i = 0; i < kSegItems; ++i) {
    if (rbase + i * kWave < c) {
      const uint32_t d = (uint32_t)((k[i] - sub) >> shift) & dmask;
      const uint32_t cell = (uint32_t)wave * kSegBuckets + d, sh = (cell & 1u) * 16u;
      const uint32_t old = atomicAdd(&R.wcnt[cell >> 1], 1u << sh);
      dr[i] = (d << 16) | ((old >> sh) & 0xffffu);
    }
  }
  __syncthreads();
  {  // thread t owns digit t: wave counts -> wave offsets, digit totals -> digit offsets
    const int d = threadIdx.x;  // kSegThreads == kSegBuckets
    uint32_t run = 0;
#pragma unroll
    for (int w = 0; w < kSegWaves; ++w) {
      const uint32_t x = wc16[w * kSegBuckets + d];
      wc16[w * kSegBuckets + d] = (uint16_t)run;
      run += x;
    }
    R.toff[d] = rp_block_exscan<kSegWaves>(run, R.wsum);
    if (d == kSegBuckets - 1) R.toff[kSegBuckets] = (uint32_t)c;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < kSegItems; ++i) {
    if (rbase + i * kWave < c) {
      const uint32_t d = dr[i] >> 16;
      buf[R.toff[d] + wc16[wave * kSegBuckets + d] + (dr[i] & 0xffffu)] = k[i];
    }
  }
  __syncthreads();
}

// A partition's keys are uniform over its local bits in the common case: two stable rounds on the
// top <= 18 local bits (lower digit first) leave buckets of a few keys (mean c / 512) already
// ordered by their next 9 bits, which thread d then insertion-sorts in place (buckets of <= kSegRun
// keys).  A partition with a larger bucket (clustered low bits) is sorted by full LSD rounds over
// all its local bits instead.
constexpr int kSegRun = 48;

__global__ __launch_bounds__(kSegThreads, 2) void k_seg_sort(const uint64_t *__restrict__ in,
                                                            const int64_t *__restrict__ counts, int64_t slot,
                                                            int64_t nparts, const int64_t *__restrict__ out_offs,
                                                            uint64_t sub, int local_bits, uint64_t out_xor,
                                                            uint64_t *__restrict__ out) {
  __shared__ uint64_t buf[kSegCap];
  __shared__ uint32_t wcnt[kSegWaves * kSegBuckets / 2];
  __shared__ uint32_t toff[kSegBuckets + 1];
  __shared__ uint32_t wsum[kSegWaves];
  __shared__ uint32_t smax;
  const SegRank R{wcnt, toff, wsum};
  const int lane = lane_id();
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
  const int rbase = wave * kWave * kSegItems + lane;
  const int topb = local_bits < kSegBits ? local_bits : kSegBits;  // bits of the MSD round
  const int npass = (local_bits + kSegBits - 1) / kSegBits;         // LSD fallback rounds
  const int dbits = npass ? (local_bits + npass - 1) / npass : 0;
  for (int64_t p = blockIdx.x; p < nparts; p += gridDim.x) {
    const int c = (int)counts[p];  // <= slot <= kSegCap (the host checked the slot size)
    const uint64_t *src = in + p * slot;
    uint64_t k[kSegItems];
#pragma unroll
    for (int i = 0; i < kSegItems; ++i) {
      const int r = rbase + i * kWave;
      k[i] = r < c ? src[r] : 0ull;
    }
    if (topb > 0) {
      if (local_bits > kSegBits) {  // the 9 bits below the top ones first (LSD), then the top ones:
        // buckets then hold keys already ordered by their next 9 bits, so the insertion sort below
        // mostly compares (a single round left ~7.5 unordered keys per bucket: the wave's largest
        // bucket, ~17 keys, cost ~150 LDS steps)
        const int lb = local_bits - kSegBits < kSegBits ? local_bits - kSegBits : kSegBits;
        seg_round(R, buf, k, c, rbase, wave, sub, local_bits - kSegBits - lb, (1u << lb) - 1u);
#pragma unroll
        for (int i = 0; i < kSegItems; ++i) {
          const int r = rbase + i * kWave;
          if (r < c) k[i] = buf[r];
        }
      }
      seg_round(R, buf, k, c, rbase, wave, sub, local_bits - topb, (1u << topb) - 1u);
      if (threadIdx.x == 0) smax = 0u;
      __syncthreads();
      const uint32_t run = toff[threadIdx.x + 1] - toff[threadIdx.x];
      uint32_t m = run;
      for (int d = kWave / 2; d > 0; d >>= 1) {
        const uint32_t o = __shfl_xor(m, d, kWave);
        m = o > m ? o : m;
      }
      if (lane == 0) atomicMax(&smax, m);
      __syncthreads();
      if (local_bits <= 2 * kSegBits) {
        // the rounds sorted every local bit
      } else if (smax <= (uint32_t)kSegRun) {
        const uint32_t b = toff[threadIdx.x], e = b + run;
        for (uint32_t i = b + 1; i < e; ++i) {  // images compare as unsigned integers
          const uint64_t v = buf[i];
          uint32_t j = i;
          while (j > b && buf[j - 1] > v) {
            buf[j] = buf[j - 1];
            --j;
          }
          buf[j] = v;
        }
        __syncthreads();
      } else {  // clustered local bits: full LSD rounds (the keys come back from the MSD round's order)
#pragma unroll
        for (int i = 0; i < kSegItems; ++i) {
          const int r = rbase + i * kWave;
          if (r < c) k[i] = buf[r];
        }
        for (int ps = 0; ps < npass; ++ps) {
          seg_round(R, buf, k, c, rbase, wave, sub, ps * dbits, (1u << dbits) - 1u);
#pragma unroll
          for (int i = 0; i < kSegItems; ++i) {
            const int r = rbase + i * kWave;
            if (r < c) k[i] = buf[r];
          }
        }
        __syncthreads();  // (every thread read its keys: buf is final)
      }
    } else {  // no local bits: the partition holds equal images
#pragma unroll
      for (int i = 0; i < kSegItems; ++i) {
        const int r = rbase + i * kWave;
        if (r < c) buf[r] = k[i];
      }
      __syncthreads();
    }
    uint64_t *dst = out + out_offs[p];
#pragma unroll
    for (int i = 0; i < kSegItems; ++i) {
      const int r = rbase + i * kWave;
      if (r < c) dst[r] = buf[r] ^ out_xor;
    }
    __syncthreads();  // buf / toff / wsum reuse by the next partition
  }
}

void seg_sort_local(const int64_t *in, const int64_t *counts, int64_t slot, int64_t nparts, const int64_t *out_offs,
                    uint64_t sub, int local_bits, uint64_t out_xor, int64_t *out, void *stream) {
  CYLON_CHECK(slot > 0 && slot <= kSegCap && local_bits >= 0 && local_bits <= 64 &&
                  (local_bits + kSegBits - 1) / kSegBits * kSegBits >= local_bits,
              Code::Invalid, "segment sort: slot " << slot << ", local bits " << local_bits);
  static_assert(kSegThreads == kSegBuckets, "one digit per thread in the offset scan");
  if (nparts == 0) return;
  const int grid = (int)std::min<int64_t>(nparts, (int64_t)kNumCUs * 2);
  hipLaunchKernelGGL(k_seg_sort, dim3(grid), dim3(kSegThreads), 0, as_stream(stream),
                     reinterpret_cast<const uint64_t *>(in), counts, slot, nparts, out_offs, sub, local_bits, out_xor,
                     reinterpret_cast<uint64_t *>(out));
  HIP_LAUNCH_CHECK();
}

// this file's code object is loaded at context creation (preload_device_code), not on first use
void preload_seg_sort() { preload_code(reinterpret_cast<const void *>(&k_seg_sort)); }

}  // namespace hip
}  // namespace cylon
