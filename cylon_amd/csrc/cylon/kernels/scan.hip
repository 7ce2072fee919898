// Device-wide scans and stream compaction (K11), gfx950.
//
// Reference: arrow::compute::Filter used for every mask -> table step
// (cpp/src/cylon/table.cpp:522-527,567,586,652,710,968), prefix sums implicit in
// Arrow builders.  Here: a three-phase reduce-then-scan with wave64 shuffles
// (6 __shfl_up steps per wave) and an LDS cross-wave step; compaction ranks
// rows with one 64-bit ballot + popcount per wave, so output order is the
// input order (stable).
#include "device_common.hpp"

namespace cylon {
namespace hip {

constexpr int kScanItems = 16;
constexpr int kScanTile = kBlock * kScanItems;  // 4096 elements per block

__device__ __forceinline__ int64_t wave_inclusive_scan(int64_t v) {
  const int lane = lane_id();
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const int64_t t = __shfl_up(v, d, kWave);
    if (lane >= d) v += t;
  }
  return v;
}

// Block-wide exclusive scan of one value per thread; returns the exclusive
// prefix and writes the block total to *total.
__device__ __forceinline__ int64_t block_exclusive_scan(int64_t v, int64_t *lds_waves, int64_t *total) {
  const int lane = lane_id();
  const int wave = threadIdx.x / kWave;
  const int64_t inc = wave_inclusive_scan(v);
  if (lane == kWave - 1) lds_waves[wave] = inc;
  __syncthreads();
  int64_t wave_off = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < kBlock / kWave; ++w) {
    const int64_t x = lds_waves[w];
    if (w < wave) wave_off += x;
    tot += x;
  }
  __syncthreads();
  *total = tot;
  return wave_off + inc - v;
}

// Tile loads are wave-coalesced: element base + k * kBlock + t (the sum does not care about order);
// the scan stages its tile through LDS (one pad element per 16, so the per-thread runs of 16 read
// back without bank conflicts) and scans 16 consecutive elements per thread.
__global__ __launch_bounds__(kBlock) void k_block_sums(const int64_t *__restrict__ in, int64_t n,
                                                       int64_t *__restrict__ sums) {
  __shared__ int64_t lds[kBlock / kWave];
  const int64_t base = (int64_t)blockIdx.x * kScanTile + threadIdx.x;
  int64_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    const int64_t i = base + (int64_t)k * kBlock;
    if (i < n) s += in[i];
  }
  int64_t tot;
  block_exclusive_scan(s, lds, &tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}

__device__ __forceinline__ int scan_pad(int i) { return i + (i >> 4); }

__global__ __launch_bounds__(kBlock) void k_block_scan(const int64_t *__restrict__ in, int64_t n,
                                                       const int64_t *__restrict__ offs,
                                                       int64_t *__restrict__ out) {
  __shared__ int64_t lds[kBlock / kWave];
  __shared__ int64_t tile[kScanTile + kScanTile / 16];
  const int64_t t0 = (int64_t)blockIdx.x * kScanTile;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    const int e = k * kBlock + threadIdx.x;
    tile[scan_pad(e)] = (t0 + e < n) ? in[t0 + e] : 0;
  }
  __syncthreads();
  int64_t v[kScanItems];
  int64_t s = 0;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    v[k] = tile[scan_pad(threadIdx.x * kScanItems + k)];
    s += v[k];
  }
  int64_t tot;
  int64_t run = block_exclusive_scan(s, lds, &tot) + (offs ? offs[blockIdx.x] : 0);
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    tile[scan_pad(threadIdx.x * kScanItems + k)] = run;
    run += v[k];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    const int e = k * kBlock + threadIdx.x;
    if (t0 + e < n) out[t0 + e] = tile[scan_pad(e)];
  }
  // out[n] = grand total, written by the thread owning element n-1
  const int64_t base = t0 + (int64_t)threadIdx.x * kScanItems;
  if (n > 0 && base <= n - 1 && n - 1 < base + kScanItems) out[n] = run;
}

int64_t scan_workspace(int64_t n) {
  const int64_t nb = (n + kScanTile - 1) / kScanTile;
  if (nb <= 1) return 1;
  return nb + (nb + 1) + scan_workspace(nb);
}

void exclusive_scan(const int64_t *in, int64_t n, int64_t *out, int64_t *ws, void *stream) {
  hipStream_t s = as_stream(stream);
  if (n == 0) {
    HIP_CHECK(hipMemsetAsync(out, 0, sizeof(int64_t), s));
    return;
  }
  const int64_t nb = (n + kScanTile - 1) / kScanTile;
  if (nb == 1) {
    hipLaunchKernelGGL(k_block_scan, dim3(1), dim3(kBlock), 0, s, in, n, (const int64_t *)nullptr, out);
    HIP_LAUNCH_CHECK();
    return;
  }
  int64_t *sums = ws;
  int64_t *sums_scan = ws + nb;
  int64_t *sub_ws = sums_scan + nb + 1;
  hipLaunchKernelGGL(k_block_sums, dim3((unsigned)nb), dim3(kBlock), 0, s, in, n, sums);
  HIP_LAUNCH_CHECK();
  exclusive_scan(sums, nb, sums_scan, sub_ws, stream);
  hipLaunchKernelGGL(k_block_scan, dim3((unsigned)nb), dim3(kBlock), 0, s, in, n, (const int64_t *)sums_scan,
                     out);
  HIP_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------
// inclusive max scan (hash-join placement: pos_i = i + max_{j<=i}(slot_j - j))
// ---------------------------------------------------------------------------
__device__ __forceinline__ int64_t wave_inclusive_max(int64_t v) {
  const int lane = lane_id();
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    const int64_t t = __shfl_up(v, d, kWave);
    if (lane >= d) v = t > v ? t : v;
  }
  return v;
}

// block-wide exclusive max (INT64_MIN identity) of one value per thread
__device__ __forceinline__ int64_t block_exclusive_max(int64_t v, int64_t *lds_waves, int64_t *total) {
  const int lane = lane_id();
  const int wave = threadIdx.x / kWave;
  const int64_t inc = wave_inclusive_max(v);
  if (lane == kWave - 1) lds_waves[wave] = inc;
  __syncthreads();
  int64_t wave_off = INT64_MIN, tot = INT64_MIN;
#pragma unroll
  for (int w = 0; w < kBlock / kWave; ++w) {
    const int64_t x = lds_waves[w];
    if (w < wave) wave_off = x > wave_off ? x : wave_off;
    tot = x > tot ? x : tot;
  }
  __syncthreads();
  *total = tot;
  int64_t prev = __shfl_up(inc, 1, kWave);
  if (lane == 0) prev = INT64_MIN;
  return prev > wave_off ? prev : wave_off;
}

__global__ __launch_bounds__(kBlock) void k_block_max(const int64_t *__restrict__ in, int64_t n,
                                                      int64_t *__restrict__ out) {
  __shared__ int64_t lds[kBlock / kWave];
  const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
  int64_t m = INT64_MIN;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    const int64_t i = base + k;
    if (i < n) m = in[i] > m ? in[i] : m;
  }
  int64_t tot;
  block_exclusive_max(m, lds, &tot);
  if (threadIdx.x == 0) out[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kBlock) void k_block_max_scan(const int64_t *__restrict__ in, int64_t n,
                                                           const int64_t *__restrict__ carry_incl,
                                                           int64_t *__restrict__ out) {
  __shared__ int64_t lds[kBlock / kWave];
  const int64_t base = (int64_t)blockIdx.x * kScanTile + (int64_t)threadIdx.x * kScanItems;
  int64_t v[kScanItems];
  int64_t m = INT64_MIN;
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    const int64_t i = base + k;
    v[k] = (i < n) ? in[i] : INT64_MIN;
    m = v[k] > m ? v[k] : m;
  }
  int64_t tot;
  int64_t run = block_exclusive_max(m, lds, &tot);
  if (carry_incl && blockIdx.x > 0) {
    const int64_t c = carry_incl[blockIdx.x - 1];
    run = c > run ? c : run;
  }
#pragma unroll
  for (int k = 0; k < kScanItems; ++k) {
    const int64_t i = base + k;
    run = v[k] > run ? v[k] : run;
    if (i < n) out[i] = run;
  }
}

int64_t max_scan_workspace(int64_t n) {
  const int64_t nb = (n + kScanTile - 1) / kScanTile;
  if (nb <= 1) return 1;
  return nb + nb + max_scan_workspace(nb);
}

void inclusive_max_scan(const int64_t *in, int64_t n, int64_t *out, int64_t *ws, void *stream) {
  hipStream_t s = as_stream(stream);
  if (n == 0) return;
  const int64_t nb = (n + kScanTile - 1) / kScanTile;
  if (nb == 1) {
    hipLaunchKernelGGL(k_block_max_scan, dim3(1), dim3(kBlock), 0, s, in, n, (const int64_t *)nullptr, out);
    HIP_LAUNCH_CHECK();
    return;
  }
  int64_t *bmax = ws;
  int64_t *bscan = ws + nb;
  int64_t *sub = bscan + nb;
  hipLaunchKernelGGL(k_block_max, dim3((unsigned)nb), dim3(kBlock), 0, s, in, n, bmax);
  HIP_LAUNCH_CHECK();
  inclusive_max_scan(bmax, nb, bscan, sub, stream);
  hipLaunchKernelGGL(k_block_max_scan, dim3((unsigned)nb), dim3(kBlock), 0, s, in, n, (const int64_t *)bscan, out);
  HIP_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------
// K11 compaction
// ---------------------------------------------------------------------------
constexpr int kCompactRounds = 16;                    // rounds of 256 rows per block
constexpr int kCompactTile = kBlock * kCompactRounds;  // 4096 rows

__global__ __launch_bounds__(kBlock) void k_mask_count(const uint8_t *__restrict__ mask, int64_t n, bool invert,
                                                       int64_t *__restrict__ counts) {
  __shared__ int64_t lds[kBlock / kWave];
  const int64_t base = (int64_t)blockIdx.x * kCompactTile;
  int64_t c = 0;
  for (int r = 0; r < kCompactRounds; ++r) {
    const int64_t i = base + (int64_t)r * kBlock + threadIdx.x;
    if (i < n) c += ((mask[i] != 0) != invert) ? 1 : 0;
  }
  int64_t tot;
  block_exclusive_scan(c, lds, &tot);
  if (threadIdx.x == 0) counts[blockIdx.x] = tot;
}

__global__ __launch_bounds__(kBlock) void k_mask_write(const uint8_t *__restrict__ mask, int64_t n, bool invert,
                                                       const int64_t *__restrict__ offs,
                                                       int64_t *__restrict__ out) {
  __shared__ int64_t lds[kBlock / kWave];
  const int64_t base = (int64_t)blockIdx.x * kCompactTile;
  int64_t running = offs[blockIdx.x];
  for (int r = 0; r < kCompactRounds; ++r) {
    const int64_t i = base + (int64_t)r * kBlock + threadIdx.x;
    const int64_t f = (i < n && ((mask[i] != 0) != invert)) ? 1 : 0;
    int64_t tot;
    const int64_t ex = block_exclusive_scan(f, lds, &tot);
    if (f) out[running + ex] = i;
    running += tot;
  }
}

int64_t mask_to_indices_workspace(int64_t n) {
  const int64_t nb = (n + kCompactTile - 1) / kCompactTile;
  return nb + (nb + 1) + scan_workspace(nb) + 1;
}

void mask_to_indices(const uint8_t *mask, int64_t n, bool invert, int64_t *ws, int64_t *out, int64_t *count,
                     void *stream) {
  hipStream_t s = as_stream(stream);
  if (n == 0) {
    HIP_CHECK(hipMemsetAsync(count, 0, sizeof(int64_t), s));
    return;
  }
  const int64_t nb = (n + kCompactTile - 1) / kCompactTile;
  int64_t *counts = ws;
  int64_t *offs = ws + nb;
  int64_t *sws = offs + nb + 1;
  hipLaunchKernelGGL(k_mask_count, dim3((unsigned)nb), dim3(kBlock), 0, s, mask, n, invert, counts);
  HIP_LAUNCH_CHECK();
  exclusive_scan(counts, nb, offs, sws, stream);
  hipLaunchKernelGGL(k_mask_write, dim3((unsigned)nb), dim3(kBlock), 0, s, mask, n, invert,
                     (const int64_t *)offs, out);
  HIP_LAUNCH_CHECK();
  HIP_CHECK(hipMemcpyAsync(count, offs + nb, sizeof(int64_t), hipMemcpyDeviceToDevice, s));
}

__global__ void k_iota(int64_t *out, int64_t n, int64_t start) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = start + i;
}

void iota(int64_t *out, int64_t n, int64_t start, void *stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_iota, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), out, n, start);
  HIP_LAUNCH_CHECK();
}

__global__ void k_mark_indices(const int64_t *__restrict__ idx, int64_t m, uint8_t *__restrict__ flags) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride) {
    const int64_t s = idx[j];
    if (s >= 0) flags[s] = 1;
  }
}

void mark_indices(const int64_t *idx, int64_t m, uint8_t *flags, void *stream) {
  if (m == 0) return;
  hipLaunchKernelGGL(k_mark_indices, dim3(grid_for(m)), dim3(kBlock), 0, as_stream(stream), idx, m, flags);
  HIP_LAUNCH_CHECK();
}

// this file's code object is loaded at context creation (preload_device_code), not on first use
void preload_scan() { preload_code(reinterpret_cast<const void *>(&k_block_sums)); }

void preload_bitmap();
void preload_copy();
void preload_delay();
void preload_groupby();
void preload_hash_join();
void preload_index();
void preload_lds_join();
void preload_merge();
void preload_partition();
void preload_radix_groupby();
void preload_radix_join();
void preload_radix_setops();
void preload_range();
void preload_range_join();
void preload_seg_sort();
void preload_select();
void preload_sort();
void preload_strcast();

// Every kernel file's code object, once per process and device (HIP loads a code object on the first
// launch from it: inside a pipelined join that stalled the host for up to 40 ms while the posted
// transfers ran with nothing to overlap, profiles/r05/first_step_overlap.txt)
void preload_device_code() {
  preload_bitmap();
  preload_copy();
  preload_delay();
  preload_groupby();
  preload_hash_join();
  preload_index();
  preload_lds_join();
  preload_merge();
  preload_partition();
  preload_radix_groupby();
  preload_radix_join();
  preload_radix_setops();
  preload_range();
  preload_range_join();
  preload_scan();
  preload_seg_sort();
  preload_select();
  preload_sort();
  preload_strcast();
}

}  // namespace hip
}  // namespace cylon
