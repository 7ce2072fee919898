// K7 range join kernels (sort-algorithm inner join on range partitions).
#include "radix_common.hpp"

namespace cylon {
namespace hip {

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

// this file's code object is loaded at context creation (preload_device_code), not on first use
void preload_range_join() { preload_code(reinterpret_cast<const void *>(&k_rg_count)); }

}  // namespace hip
}  // namespace cylon
