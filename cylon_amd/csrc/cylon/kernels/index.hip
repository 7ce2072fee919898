// K16 persistent index kernels (reference cpp/src/cylon/indexing/index.hpp:81-700:
// HashIndex = unordered_multimap value -> positions, LinearIndex = scan).  An index is
// built once: the order images of the index column sorted with their row numbers
// (stable radix sort, so equal values keep row order), plus for the hash schema an
// open-addressing table over the distinct images pointing at their run in the sorted
// arrays.  A lookup is then one probe per label (hash) or a binary search (sorted
// schemas), a scan of the per-label counts and one gather of the positions: labels
// in label order, rows in row order (pandas `loc`).
#include "device_common.hpp"

namespace cylon {
namespace hip {

__device__ __forceinline__ int64_t lower_bound_img(const uint64_t *a, int64_t n, uint64_t v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ int64_t upper_bound_img(const uint64_t *a, int64_t n, uint64_t v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] <= v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__global__ void k_index_bounds(const uint64_t *__restrict__ sorted, int64_t n, const uint64_t *__restrict__ probe,
                               int64_t m, int64_t *__restrict__ lo, int64_t *__restrict__ cnt) {
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += step) {
    const uint64_t v = probe[i];
    const int64_t a = lower_bound_img(sorted, n, v);
    lo[i] = a;
    cnt[i] = upper_bound_img(sorted + a, n - a, v);
  }
}

void index_bounds(const uint64_t *sorted, int64_t n, const uint64_t *probe, int64_t m, int64_t *lo, int64_t *cnt,
                  void *stream) {
  if (m == 0) return;
  hipLaunchKernelGGL(k_index_bounds, dim3(grid_for(m)), dim3(kBlock), 0, as_stream(stream), sorted, n, probe, m, lo,
                     cnt);
  HIP_LAUNCH_CHECK();
}

__device__ __forceinline__ uint64_t idx_slot(uint64_t k, int64_t cap) {
  return hashing::fmix64(k) & (uint64_t)(cap - 1);
}

__global__ void k_hash_index_build(const uint64_t *__restrict__ sorted, int64_t n, uint64_t *__restrict__ tkeys,
                                   int32_t *__restrict__ used, int64_t *__restrict__ tlo, int64_t *__restrict__ tcnt,
                                   int64_t cap) {
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += step) {
    const uint64_t v = sorted[i];
    if (i > 0 && sorted[i - 1] == v) continue;  // one entry per run (its first slot)
    const int64_t len = upper_bound_img(sorted + i, n - i, v);
    uint64_t s = idx_slot(v, cap);
    for (int64_t probe = 0; probe < cap; ++probe) {
      if (atomicCAS(&used[s], 0, 1) == 0) {
        tkeys[s] = v;
        tlo[s] = i;
        tcnt[s] = len;
        break;
      }
      s = (s + 1) & (uint64_t)(cap - 1);
    }
  }
}

void hash_index_build(const uint64_t *sorted, int64_t n, uint64_t *tkeys, int32_t *used, int64_t *tlo, int64_t *tcnt,
                      int64_t cap, void *stream) {
  CYLON_CHECK(cap > 0 && (cap & (cap - 1)) == 0, Code::Invalid, "index table capacity " << cap);
  if (n == 0) return;
  hipLaunchKernelGGL(k_hash_index_build, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), sorted, n, tkeys,
                     used, tlo, tcnt, cap);
  HIP_LAUNCH_CHECK();
}

__global__ void k_hash_index_probe(const uint64_t *__restrict__ tkeys, const int32_t *__restrict__ used,
                                   const int64_t *__restrict__ tlo, const int64_t *__restrict__ tcnt, int64_t cap,
                                   const uint64_t *__restrict__ probe, int64_t m, int64_t *__restrict__ lo,
                                   int64_t *__restrict__ cnt) {
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < m; i += step) {
    const uint64_t v = probe[i];
    uint64_t s = idx_slot(v, cap);
    int64_t l = 0, c = 0;
    for (int64_t p = 0; p < cap && used[s]; ++p) {
      if (tkeys[s] == v) {
        l = tlo[s];
        c = tcnt[s];
        break;
      }
      s = (s + 1) & (uint64_t)(cap - 1);
    }
    lo[i] = l;
    cnt[i] = c;
  }
}

void hash_index_probe(const uint64_t *tkeys, const int32_t *used, const int64_t *tlo, const int64_t *tcnt, int64_t cap,
                      const uint64_t *probe, int64_t m, int64_t *lo, int64_t *cnt, void *stream) {
  if (m == 0) return;
  hipLaunchKernelGGL(k_hash_index_probe, dim3(grid_for(m)), dim3(kBlock), 0, as_stream(stream), tkeys, used, tlo, tcnt,
                     cap, probe, m, lo, cnt);
  HIP_LAUNCH_CHECK();
}

// one wave per label: lanes copy the label's run of positions (coalesced reads of sorted_pos)
__global__ void k_index_gather_positions(const int64_t *__restrict__ sorted_pos, const int64_t *__restrict__ lo,
                                         const int64_t *__restrict__ cnt, const int64_t *__restrict__ offs, int64_t m,
                                         int64_t *__restrict__ out) {
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x / kWave);
  const int lane = lane_id();
  for (int64_t i = (int64_t)blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave; i < m; i += waves) {
    const int64_t l = lo[i], c = cnt[i], o = offs[i];
    for (int64_t j = lane; j < c; j += kWave) out[o + j] = sorted_pos[l + j];
  }
}

void index_gather_positions(const int64_t *sorted_pos, const int64_t *lo, const int64_t *cnt, const int64_t *offs,
                            int64_t m, int64_t *out, void *stream) {
  if (m == 0) return;
  hipLaunchKernelGGL(k_index_gather_positions, dim3(grid_for(m * kWave)), dim3(kBlock), 0, as_stream(stream),
                     sorted_pos, lo, cnt, offs, m, out);
  HIP_LAUNCH_CHECK();
}

// the bytes of row r of a var-width (offsets) or fixed-width column
__device__ __forceinline__ void idx_bytes(const ColView &c, int64_t r, const uint8_t *&p, int64_t &len) {
  if (c.offsets) {
    p = c.data + c.offsets[r];
    len = c.offsets[r + 1] - c.offsets[r];
  } else {
    p = c.data + r * (int64_t)c.width;
    len = c.width;
  }
}

// one wave per label, one lane per candidate row of the label's hash run
__global__ void k_index_verify_bytes(ColView col, ColView labels, const int64_t *__restrict__ sorted_pos,
                                     const int64_t *__restrict__ lo, const int64_t *__restrict__ cnt,
                                     const int64_t *__restrict__ offs, int64_t m, uint8_t *__restrict__ keep) {
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x / kWave);
  const int lane = lane_id();
  for (int64_t i = (int64_t)blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave; i < m; i += waves) {
    const int64_t l = lo[i], c = cnt[i], o = offs[i];
    const uint8_t *lp;
    int64_t ll;
    idx_bytes(labels, i, lp, ll);
    for (int64_t j = lane; j < c; j += kWave) {
      const uint8_t *cp;
      int64_t cl;
      idx_bytes(col, sorted_pos[l + j], cp, cl);
      bool eq = cl == ll;
      for (int64_t b = 0; eq && b < ll; ++b) eq = cp[b] == lp[b];
      keep[o + j] = eq ? 1 : 0;
    }
  }
}

void index_verify_bytes(const ColView &col, const ColView &labels, const int64_t *sorted_pos, const int64_t *lo,
                        const int64_t *cnt, const int64_t *offs, int64_t m, uint8_t *keep, void *stream) {
  if (m == 0) return;
  hipLaunchKernelGGL(k_index_verify_bytes, dim3(grid_for(m * kWave)), dim3(kBlock), 0, as_stream(stream), col, labels,
                     sorted_pos, lo, cnt, offs, m, keep);
  HIP_LAUNCH_CHECK();
}

// this file's code object is loaded at context creation (preload_device_code), not on first use
void preload_index() { preload_code(reinterpret_cast<const void *>(&k_index_bounds)); }

}  // namespace hip
}  // namespace cylon
