// K13 range partitioning for the distributed sample sort (gfx950).
// Reference: cpp/src/cylon/arrow/arrow_partition_kernels.cpp:334-455
// (sample -> MinMax -> bin histogram (num_bins + 2) -> allreduce -> quantile
// walk -> per-row bin_to_partition[get_bin_pos(v)], descending = P-1-p).
// Bins are computed in double (the reference's integer (v-min)*bins can
// overflow for wide int64 ranges).  The per-row pass keeps the bin->partition
// table in LDS and builds the partition histogram with LDS atomics.
#include "device_common.hpp"

namespace cylon {
namespace hip {

__device__ __forceinline__ double value_as_double(const ColView &c, int64_t i) {
  const uint64_t b = load_bits(c.data, i, c.width);
  if (c.kind == static_cast<int>(ValueKind::FLOAT)) {
    if (c.width == 8) return __longlong_as_double((long long)b);
    if (c.width == 4) return (double)__int_as_float((int)b);
    return (double)__half2float(__ushort_as_half((unsigned short)b));
  }
  if (c.kind == static_cast<int>(ValueKind::SIGNED_INT)) return (double)extend_bits(b, c.width, c.kind);
  return (double)b;
}

__device__ __forceinline__ int64_t bin_pos(double v, double vmin, double vmax, int64_t nbins) {
  if (!(v >= vmin)) return 0;  // also NaN
  if (v >= vmax) return nbins + 1;
  int64_t b = 1 + (int64_t)floor((v - vmin) * (double)nbins / (vmax - vmin));
  return b > nbins ? nbins : b;
}

__global__ void k_range_minmax(ColView c, const int64_t *__restrict__ idx, int64_t m, double *out) {
  double lo = INFINITY, hi = -INFINITY;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride) {
    const int64_t i = idx ? idx[j] : j;
    if (c.valid && !c.valid[i]) continue;
    const double v = value_as_double(c, i);
    lo = fmin(lo, v);
    hi = fmax(hi, v);
  }
  for (int d = kWave / 2; d > 0; d >>= 1) {
    lo = fmin(lo, __shfl_xor(lo, d, kWave));
    hi = fmax(hi, __shfl_xor(hi, d, kWave));
  }
  if (lane_id() == 0) {
    // order-preserving integer images for atomic min/max of doubles
    unsigned long long l = __double_as_longlong(lo), h = __double_as_longlong(hi);
    l = (l >> 63) ? ~l : (l | 0x8000000000000000ull);
    h = (h >> 63) ? ~h : (h | 0x8000000000000000ull);
    atomicMin(reinterpret_cast<unsigned long long *>(out), l);
    atomicMax(reinterpret_cast<unsigned long long *>(out) + 1, h);
  }
}

__global__ void k_minmax_fix(double *out) {
  unsigned long long *u = reinterpret_cast<unsigned long long *>(out);
  for (int k = 0; k < 2; ++k) {
    unsigned long long x = u[k];
    x = (x >> 63) ? (x & 0x7fffffffffffffffull) : ~x;
    u[k] = x;
  }
}

void range_minmax(const ColView &c, const int64_t *idx, int64_t m, double *out, void *stream) {
  hipStream_t s = as_stream(stream);
  unsigned long long init[2] = {~0ull, 0ull};
  HIP_CHECK(hipMemcpyAsync(out, init, sizeof(init), hipMemcpyHostToDevice, s));
  if (m > 0) {
    hipLaunchKernelGGL(k_range_minmax, dim3(grid_for(m, kBlock, 1024)), dim3(kBlock), 0, s, c, idx, m, out);
    HIP_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(k_minmax_fix, dim3(1), dim3(1), 0, s, out);
  HIP_LAUNCH_CHECK();
  HIP_CHECK(hipStreamSynchronize(s));  // out is consumed on the host right after
}

__global__ void k_range_hist(ColView c, const int64_t *__restrict__ idx, int64_t m, double vmin, double vmax,
                             int64_t nbins, unsigned long long *hist) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride) {
    const int64_t i = idx ? idx[j] : j;
    atomicAdd(&hist[bin_pos(value_as_double(c, i), vmin, vmax, nbins)], 1ull);
  }
}

void range_histogram(const ColView &c, const int64_t *idx, int64_t m, double vmin, double vmax, int64_t nbins,
                     int64_t *hist, void *stream) {
  if (m == 0) return;
  hipLaunchKernelGGL(k_range_hist, dim3(grid_for(m)), dim3(kBlock), 0, as_stream(stream), c, idx, m, vmin, vmax,
                     nbins, reinterpret_cast<unsigned long long *>(hist));
  HIP_LAUNCH_CHECK();
}

__global__ void k_range_partition(ColView c, int64_t n, double vmin, double vmax, int64_t nbins,
                                  const uint32_t *__restrict__ b2p, uint32_t nparts, bool desc,
                                  uint32_t *__restrict__ pid, unsigned long long *counts) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  uint32_t *lb2p = reinterpret_cast<uint32_t *>(smem);
  unsigned int *lcnt = reinterpret_cast<unsigned int *>(smem + sizeof(uint32_t) * (nbins + 2));
  for (int64_t b = threadIdx.x; b < nbins + 2; b += blockDim.x) lb2p[b] = b2p[b];
  for (uint32_t p = threadIdx.x; p < nparts; p += blockDim.x) lcnt[p] = 0;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    uint32_t p = lb2p[bin_pos(value_as_double(c, i), vmin, vmax, nbins)];
    if (desc) p = nparts - 1 - p;
    pid[i] = p;
    atomicAdd(&lcnt[p], 1u);
  }
  __syncthreads();
  for (uint32_t p = threadIdx.x; p < nparts; p += blockDim.x)
    if (lcnt[p]) atomicAdd(&counts[p], (unsigned long long)lcnt[p]);
}

void range_partition(const ColView &c, int64_t n, double vmin, double vmax, int64_t nbins, const uint32_t *b2p,
                     uint32_t nparts, bool desc, uint32_t *pid, int64_t *counts, void *stream) {
  if (n == 0) return;
  const size_t lds = sizeof(uint32_t) * (nbins + 2) + sizeof(unsigned int) * nparts;
  CYLON_CHECK(lds <= 64 * 1024, Code::Invalid, "too many range bins " << nbins);
  hipLaunchKernelGGL(k_range_partition, dim3(grid_for(n)), dim3(kBlock), lds, as_stream(stream), c, n, vmin, vmax,
                     nbins, b2p, nparts, desc, pid, reinterpret_cast<unsigned long long *>(counts));
  HIP_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------
// Sample-sort partition by exact composite splitters (see kernel_decls.inc).
// The splitters (<= 1023 x (2 * kMaxSortKeys + 1) words) are staged in LDS;
// every row binary-searches them, and a block histogram in LDS feeds one
// atomic per partition per block.
// ---------------------------------------------------------------------------
constexpr int kMaxSortKeys = 4;
constexpr int kMaxSplitParts = 1024;

struct SplitKeys {
  const uint64_t *img[kMaxSortKeys];
  const uint8_t *nul[kMaxSortKeys];
};

__global__ __launch_bounds__(kBlock) void k_splitter_partition(SplitKeys keys, int nkeys, int64_t n, int64_t gid0,
                                                               const uint64_t *__restrict__ spl, uint32_t nparts,
                                                               uint32_t *__restrict__ pid,
                                                               unsigned long long *__restrict__ counts) {
  extern __shared__ uint64_t s_spl[];  // (nparts - 1) * stride words, then nparts u32 counters
  const int stride = 2 * nkeys + 1;
  const int nw = (int)(nparts - 1) * stride;
  for (int i = threadIdx.x; i < nw; i += blockDim.x) s_spl[i] = spl[i];
  unsigned int *hist = reinterpret_cast<unsigned int *>(s_spl + nw);
  for (uint32_t p = threadIdx.x; p < nparts; p += blockDim.x) hist[p] = 0;
  __syncthreads();
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += step) {
    uint64_t k[2 * kMaxSortKeys + 1];
#pragma unroll
    for (int c = 0; c < kMaxSortKeys; ++c)
      if (c < nkeys) {
        k[2 * c] = keys.nul[c] ? (uint64_t)(keys.nul[c][i] != 0) : 0ull;
        k[2 * c + 1] = keys.img[c][i];
      }
    k[2 * nkeys] = (uint64_t)(gid0 + i);
    // lower bound: first splitter >= key; pid = number of splitters < key
    uint32_t lo = 0, hi = nparts - 1;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      const uint64_t *s = s_spl + (int64_t)mid * stride;
      int cmp = 0;
      for (int w = 0; w < stride && cmp == 0; ++w) cmp = s[w] < k[w] ? -1 : (s[w] > k[w] ? 1 : 0);
      if (cmp < 0) lo = mid + 1; else hi = mid;
    }
    pid[i] = lo;
    atomicAdd(&hist[lo], 1u);
  }
  __syncthreads();
  for (uint32_t p = threadIdx.x; p < nparts; p += blockDim.x)
    if (hist[p]) atomicAdd(&counts[p], (unsigned long long)hist[p]);
}

void splitter_partition(const uint64_t *const *images, const uint8_t *const *nulls, int nkeys, int64_t n,
                        int64_t gid0, const uint64_t *splitters, uint32_t nparts, uint32_t *pid, int64_t *counts,
                        void *stream) {
  CYLON_CHECK(nkeys >= 1 && nkeys <= kMaxSortKeys, Code::Invalid, "splitter partition over " << nkeys << " keys");
  CYLON_CHECK(nparts >= 1 && nparts <= (uint32_t)kMaxSplitParts, Code::Invalid, "partition count " << nparts);
  if (n == 0) return;
  SplitKeys k{};
  for (int c = 0; c < nkeys; ++c) {
    k.img[c] = images[c];
    k.nul[c] = nulls[c];
  }
  const size_t lds = (size_t)(nparts - 1) * (2 * nkeys + 1) * sizeof(uint64_t) + nparts * sizeof(unsigned int);
  hipLaunchKernelGGL(k_splitter_partition, dim3(grid_for(n, kBlock, kNumCUs * 4)), dim3(kBlock), lds,
                     as_stream(stream), k, nkeys, n, gid0, splitters, nparts, pid,
                     reinterpret_cast<unsigned long long *>(counts));
  HIP_LAUNCH_CHECK();
}

// this file's code object is loaded at context creation (preload_device_code), not on first use
void preload_range() { preload_code(reinterpret_cast<const void *>(&k_range_minmax)); }

}  // namespace hip
}  // namespace cylon
