// K8/K9/K10/K12: group ids, distinct, group-by aggregation and scalar
// reductions (gfx950).
//
// Reference: cpp/src/cylon/groupby/hash_groupby.cpp:92-320 (bytell_hash_map
// row -> group id in first-occurrence order, per-op state update/finalize),
// compute/aggregate_kernels.hpp:268-545 (SUM/MIN/MAX/COUNT/MEAN/VAR/STDDEV/
// NUNIQUE/QUANTILE), compute/aggregates.cpp:26-152 (scalar Sum/Count/Min/Max).
//
// MI355X design:
//   * group_insert: a concurrent open-addressing hash SET keyed by the 64-bit
//     key itself (slot claimed by atomicCAS on the key word, sentinel INT64_MIN;
//     rows whose key equals the sentinel share one extra slot).  First
//     occurrence per slot = atomicMin of the row id, so dense group ids come
//     out in first-occurrence order exactly like the reference's HashGroupBy.
//   * aggregation: every op is an atomic accumulate into a per-group array:
//     f64 sums use the hardware fp64 atomic add, integer sums u64 adds,
//     MIN/MAX use unsigned atomicMin/Max on order-preserving 64-bit images of
//     the value (one code path for every numeric type).  When the group count
//     is small the block first accumulates in LDS (ds atomics) and issues one
//     global atomic per (block, group) - no hot global address.
//   * scalar reductions (ngroups == 1): registers -> wave64 shuffle tree ->
//     LDS -> one atomic per block.
#include "device_common.hpp"

namespace cylon {
namespace hip {

constexpr int64_t kGroupSentinel = (int64_t)0x8000000000000000ull;
constexpr int kLdsGroups = 2048;

__global__ void k_group_insert(const int64_t *__restrict__ keys, int64_t n, int64_t *slot_keys, int64_t cap,
                               int64_t *__restrict__ slot_of_row, unsigned long long *slot_first) {
  const uint64_t mask = (uint64_t)cap - 1;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t k = keys[i];
    int64_t slot;
    if (k == kGroupSentinel) {
      slot = cap;
    } else {
      uint64_t h = hashing::fmix64((uint64_t)k) & mask;
      while (true) {
        const int64_t cur = slot_keys[h];
        if (cur == k) break;
        if (cur == kGroupSentinel) {
          const unsigned long long prev = atomicCAS(reinterpret_cast<unsigned long long *>(&slot_keys[h]),
                                                    (unsigned long long)kGroupSentinel, (unsigned long long)k);
          if (prev == (unsigned long long)kGroupSentinel || (int64_t)prev == k) break;
        }
        h = (h + 1) & mask;
      }
      slot = (int64_t)h;
    }
    slot_of_row[i] = slot;
    atomicMin(&slot_first[slot], (unsigned long long)i);
  }
}

void group_insert(const int64_t *keys, int64_t n, int64_t *slot_keys, int64_t cap, int64_t *slot_of_row,
                  int64_t *slot_first, void *stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_group_insert, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), keys, n, slot_keys, cap,
                     slot_of_row, reinterpret_cast<unsigned long long *>(slot_first));
  HIP_LAUNCH_CHECK();
}

__global__ void k_mark_firsts(const int64_t *__restrict__ v, int64_t m, uint8_t *__restrict__ flags) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride) {
    const int64_t x = v[j];
    if (x >= 0 && x != INT64_MAX) flags[x] = 1;
  }
}

void mark_firsts(const int64_t *slot_first, int64_t m, uint8_t *flags, void *stream) {
  if (m == 0) return;
  hipLaunchKernelGGL(k_mark_firsts, dim3(grid_for(m)), dim3(kBlock), 0, as_stream(stream), slot_first, m, flags);
  HIP_LAUNCH_CHECK();
}

__global__ void k_scatter_iota(const int64_t *__restrict__ idx, int64_t m, int64_t *__restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < m; g += stride) out[idx[g]] = g;
}

void scatter_iota(const int64_t *idx, int64_t m, int64_t *out, void *stream) {
  if (m == 0) return;
  hipLaunchKernelGGL(k_scatter_iota, dim3(grid_for(m)), dim3(kBlock), 0, as_stream(stream), idx, m, out);
  HIP_LAUNCH_CHECK();
}

__global__ void k_gather2(const int64_t *__restrict__ a, const int64_t *__restrict__ b,
                          const int64_t *__restrict__ c, int64_t n, int64_t *__restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = c[b[a[i]]];
}

void gather_chain2(const int64_t *a, const int64_t *b, const int64_t *c, int64_t n, int64_t *out, void *stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_gather2, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), a, b, c, n, out);
  HIP_LAUNCH_CHECK();
}

__global__ void k_permute_assign(const int64_t *__restrict__ dst, const int64_t *__restrict__ src,
                                 const int64_t *__restrict__ table, int64_t n, int64_t *__restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    out[dst[i]] = table[src ? src[i] : i];
}

void permute_assign(const int64_t *dst, const int64_t *src, const int64_t *table, int64_t n, int64_t *out,
                    void *stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_permute_assign, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), dst, src, table, n,
                     out);
  HIP_LAUNCH_CHECK();
}

// segment heads of a sorted permutation: flag[i] = 1 if row perm[i] differs from perm[i-1]
struct ColSet3 {
  ColView c[kMaxFusedCols];
};

__device__ __forceinline__ bool val_eq(const ColView &a, int64_t i, int64_t j) {
  const bool va = a.valid == nullptr || a.valid[i] != 0;
  const bool vb = a.valid == nullptr || a.valid[j] != 0;
  if (!va || !vb) return va == vb;
  if (a.kind == static_cast<int>(ValueKind::VAR_BYTES)) {
    const int64_t ab = a.offsets[i], al = a.offsets[i + 1] - ab;
    const int64_t bb = a.offsets[j], bl = a.offsets[j + 1] - bb;
    if (al != bl) return false;
    for (int64_t k = 0; k < al; ++k)
      if (a.data[ab + k] != a.data[bb + k]) return false;
    return true;
  }
  if (a.kind == static_cast<int>(ValueKind::FIXED_BYTES)) {
    for (int k = 0; k < a.width; ++k)
      if (a.data[i * a.width + k] != a.data[j * a.width + k]) return false;
    return true;
  }
  const int64_t x = extend_bits(load_bits(a.data, i, a.width), a.width, a.kind);
  const int64_t y = extend_bits(load_bits(a.data, j, a.width), a.width, a.kind);
  if (x == y) return true;
  if (a.kind == static_cast<int>(ValueKind::FLOAT)) {  // NaN == NaN for grouping
    if (a.width == 8) {
      const double dx = __longlong_as_double(x), dy = __longlong_as_double(y);
      return dx != dx && dy != dy;
    }
    if (a.width == 4) {
      const float fx = __int_as_float((int)x), fy = __int_as_float((int)y);
      return fx != fx && fy != fy;
    }
  }
  return false;
}

__global__ void k_segment_heads(ColSet3 cols, int ncols, const int64_t *__restrict__ perm, int64_t n,
                                uint8_t *__restrict__ heads) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    bool h = (i == 0);
    if (!h) {
      const int64_t a = perm[i], b = perm[i - 1];
      for (int c = 0; c < ncols && !h; ++c) h = !val_eq(cols.c[c], a, b);
    }
    heads[i] = h ? 1 : 0;
  }
}

void segment_heads(const ColView *cols, int ncols, const int64_t *perm, int64_t n, uint8_t *heads, void *stream) {
  if (n == 0) return;
  CYLON_CHECK(ncols <= kMaxFusedCols, Code::Invalid, "too many key columns " << ncols);
  ColSet3 s;
  for (int c = 0; c < ncols; ++c) s.c[c] = cols[c];
  hipLaunchKernelGGL(k_segment_heads, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), s, ncols, perm, n,
                     heads);
  HIP_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------
// aggregation
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t img(uint64_t bits, int w, int kind) {
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

__device__ __forceinline__ double as_double(const ColView &c, int64_t i) {
  const uint64_t b = load_bits(c.data, i, c.width);
  if (c.kind == static_cast<int>(ValueKind::FLOAT)) {
    if (c.width == 8) return __longlong_as_double((long long)b);
    if (c.width == 4) return (double)__int_as_float((int)b);
    return (double)__half2float(__ushort_as_half((unsigned short)b));
  }
  if (c.kind == static_cast<int>(ValueKind::SIGNED_INT)) return (double)extend_bits(b, c.width, c.kind);
  return (double)b;
}

__device__ __forceinline__ int64_t as_i64(const ColView &c, int64_t i) {
  return extend_bits(load_bits(c.data, i, c.width), c.width, c.kind);
}

// kinds: 0 SUM_F64, 1 SUM_I64, 2 MIN_IMG, 3 MAX_IMG, 4 COUNT, 5 M2 (needs mean)
template <int KIND>
__device__ __forceinline__ void acc_global(void *acc, int64_t g, const ColView &v, int64_t i, const double *mean) {
  if (KIND == 0) atomicAdd(reinterpret_cast<double *>(acc) + g, as_double(v, i));
  if (KIND == 1) atomicAdd(reinterpret_cast<unsigned long long *>(acc) + g, (unsigned long long)as_i64(v, i));
  if (KIND == 2)
    atomicMin(reinterpret_cast<unsigned long long *>(acc) + g, (unsigned long long)img(load_bits(v.data, i, v.width), v.width, v.kind));
  if (KIND == 3)
    atomicMax(reinterpret_cast<unsigned long long *>(acc) + g, (unsigned long long)img(load_bits(v.data, i, v.width), v.width, v.kind));
  if (KIND == 4) atomicAdd(reinterpret_cast<unsigned long long *>(acc) + g, 1ull);
  if (KIND == 5) {
    const double d = as_double(v, i) - mean[g];
    atomicAdd(reinterpret_cast<double *>(acc) + g, d * d);
  }
}

template <int KIND>
__global__ __launch_bounds__(kBlock) void k_agg_global(const int64_t *__restrict__ gid, int64_t n, ColView v,
                                                       void *acc, const double *__restrict__ mean) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    if (v.valid && !v.valid[i]) continue;
    acc_global<KIND>(acc, gid[i], v, i, mean);
  }
}

// LDS-privatised variant for ngroups <= kLdsGroups
template <int KIND>
__global__ __launch_bounds__(kBlock) void k_agg_lds(const int64_t *__restrict__ gid, int64_t n, int64_t ngroups,
                                                    ColView v, void *acc, const double *__restrict__ mean) {
  __shared__ __attribute__((aligned(16))) unsigned long long lacc[kLdsGroups];
  const unsigned long long init = (KIND == 2) ? ~0ull : 0ull;
  for (int64_t g = threadIdx.x; g < ngroups; g += blockDim.x) lacc[g] = init;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    if (v.valid && !v.valid[i]) continue;
    const int64_t g = gid ? gid[i] : 0;
    if (KIND == 0) atomicAdd(reinterpret_cast<double *>(&lacc[g]), as_double(v, i));
    if (KIND == 1) atomicAdd(&lacc[g], (unsigned long long)as_i64(v, i));
    if (KIND == 2) atomicMin(&lacc[g], (unsigned long long)img(load_bits(v.data, i, v.width), v.width, v.kind));
    if (KIND == 3) atomicMax(&lacc[g], (unsigned long long)img(load_bits(v.data, i, v.width), v.width, v.kind));
    if (KIND == 4) atomicAdd(&lacc[g], 1ull);
    if (KIND == 5) {
      const double d = as_double(v, i) - mean[g];
      atomicAdd(reinterpret_cast<double *>(&lacc[g]), d * d);
    }
  }
  __syncthreads();
  for (int64_t g = threadIdx.x; g < ngroups; g += blockDim.x) {
    const unsigned long long x = lacc[g];
    if (x == init && KIND != 0 && KIND != 5) continue;
    if (KIND == 0 || KIND == 5) {
      const double d = __longlong_as_double((long long)x);
      if (d != 0.0) atomicAdd(reinterpret_cast<double *>(acc) + g, d);
    } else if (KIND == 1 || KIND == 4) {
      atomicAdd(reinterpret_cast<unsigned long long *>(acc) + g, x);
    } else if (KIND == 2) {
      atomicMin(reinterpret_cast<unsigned long long *>(acc) + g, x);
    } else {
      atomicMax(reinterpret_cast<unsigned long long *>(acc) + g, x);
    }
  }
}

// single group: register accumulation + wave64 tree + one atomic per block
template <int KIND>
__global__ __launch_bounds__(kBlock) void k_agg_scalar(int64_t n, ColView v, void *acc, const double *__restrict__ mean) {
  __shared__ unsigned long long wred[kBlock / kWave];
  double fs = 0.0;
  unsigned long long us = (KIND == 2) ? ~0ull : 0ull;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    if (v.valid && !v.valid[i]) continue;
    if (KIND == 0) fs += as_double(v, i);
    if (KIND == 5) {
      const double d = as_double(v, i) - mean[0];
      fs += d * d;
    }
    if (KIND == 1) us += (unsigned long long)as_i64(v, i);
    if (KIND == 4) us += 1;
    if (KIND == 2) {
      const unsigned long long x = img(load_bits(v.data, i, v.width), v.width, v.kind);
      us = x < us ? x : us;
    }
    if (KIND == 3) {
      const unsigned long long x = img(load_bits(v.data, i, v.width), v.width, v.kind);
      us = x > us ? x : us;
    }
  }
  const bool fp = (KIND == 0 || KIND == 5);
#pragma unroll
  for (int d = kWave / 2; d > 0; d >>= 1) {
    if (fp) {
      fs += __shfl_xor(fs, d, kWave);
    } else {
      const unsigned long long o = __shfl_xor(us, d, kWave);
      if (KIND == 2) us = o < us ? o : us;
      else if (KIND == 3) us = o > us ? o : us;
      else us += o;
    }
  }
  const int wave = threadIdx.x / kWave;
  if (lane_id() == 0) wred[wave] = fp ? (unsigned long long)__double_as_longlong(fs) : us;
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kBlock / kWave; ++w) {
      const unsigned long long o = wred[w];
      if (fp) fs += __longlong_as_double((long long)o);
      else if (KIND == 2) us = o < us ? o : us;
      else if (KIND == 3) us = o > us ? o : us;
      else us += o;
    }
    if (fp) atomicAdd(reinterpret_cast<double *>(acc), fs);
    else if (KIND == 2) atomicMin(reinterpret_cast<unsigned long long *>(acc), us);
    else if (KIND == 3) atomicMax(reinterpret_cast<unsigned long long *>(acc), us);
    else atomicAdd(reinterpret_cast<unsigned long long *>(acc), us);
  }
}

template <int KIND>
static void launch_agg(const int64_t *gid, int64_t n, int64_t ngroups, const ColView &v, void *acc, const double *mean,
                       hipStream_t s) {
  if (ngroups == 1) {
    hipLaunchKernelGGL(k_agg_scalar<KIND>, dim3(grid_for(n, kBlock, 1024)), dim3(kBlock), 0, s, n, v, acc, mean);
  } else if (ngroups <= kLdsGroups) {
    // fewer blocks: each block's LDS flush costs ngroups global atomics
    hipLaunchKernelGGL(k_agg_lds<KIND>, dim3(grid_for(n, kBlock * 16, 1024)), dim3(kBlock), 0, s, gid, n, ngroups, v,
                       acc, mean);
  } else {
    hipLaunchKernelGGL(k_agg_global<KIND>, dim3(grid_for(n)), dim3(kBlock), 0, s, gid, n, v, acc, mean);
  }
  HIP_LAUNCH_CHECK();
}

void agg_accumulate(const int64_t *gid, int64_t n, int64_t ngroups, const ColView &v, int kind, void *acc,
                    const double *mean, void *stream) {
  if (n == 0 || ngroups == 0) return;
  hipStream_t s = as_stream(stream);
  switch (kind) {
    case 0: launch_agg<0>(gid, n, ngroups, v, acc, mean, s); break;
    case 1: launch_agg<1>(gid, n, ngroups, v, acc, mean, s); break;
    case 2: launch_agg<2>(gid, n, ngroups, v, acc, mean, s); break;
    case 3: launch_agg<3>(gid, n, ngroups, v, acc, mean, s); break;
    case 4: launch_agg<4>(gid, n, ngroups, v, acc, mean, s); break;
    case 5: launch_agg<5>(gid, n, ngroups, v, acc, mean, s); break;
    default: CYLON_THROW(Code::Invalid, "unknown accumulate kind " << kind);
  }
}

// images -> values of the original type (in place into out, width w)
__global__ void k_unimg(const uint64_t *__restrict__ in, int64_t m, int w, int kind, uint8_t *__restrict__ out) {
  const int nb = 8 * w;
  const uint64_t mask = (nb == 64) ? ~0ull : ((1ull << nb) - 1);
  const uint64_t sign = 1ull << (nb - 1);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < m; g += stride) {
    uint64_t b = in[g] & mask;
    if (kind == static_cast<int>(ValueKind::SIGNED_INT)) b ^= sign;
    else if (kind == static_cast<int>(ValueKind::FLOAT)) b = (b & sign) ? (b ^ sign) : (~b & mask);
    switch (w) {
      case 1: out[g] = (uint8_t)b; break;
      case 2: reinterpret_cast<uint16_t *>(out)[g] = (uint16_t)b; break;
      case 4: reinterpret_cast<uint32_t *>(out)[g] = (uint32_t)b; break;
      default: reinterpret_cast<uint64_t *>(out)[g] = b;
    }
  }
}

void agg_unimage(const uint64_t *in, int64_t m, int width, int kind, uint8_t *out, void *stream) {
  if (m == 0) return;
  hipLaunchKernelGGL(k_unimg, dim3(grid_for(m)), dim3(kBlock), 0, as_stream(stream), in, m, width, kind, out);
  HIP_LAUNCH_CHECK();
}

// type-2 quantile on values sorted by (group, value); offs = group offsets (ngroups + 1)
__global__ void k_quantile(const ColView v, const int64_t *__restrict__ perm, const int64_t *__restrict__ offs,
                           int64_t ngroups, double q, double *__restrict__ out, uint8_t *__restrict__ valid) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < ngroups; g += stride) {
    const int64_t b = offs[g], cnt = offs[g + 1] - b;
    if (cnt == 0) {
      out[g] = 0.0;
      valid[g] = 0;
      continue;
    }
    const double np = (double)cnt * q;
    const double j = floor(np);
    const bool whole = np == j;  // (a comparison: `np - j == 0` may be contracted into fma(cnt, q, -j))
    int64_t pos = (int64_t)j;
    if (pos >= cnt) pos = cnt - 1;
    double r;
    if (whole && pos > 0) r = 0.5 * (as_double(v, perm[b + pos - 1]) + as_double(v, perm[b + pos]));
    else r = as_double(v, perm[b + pos]);
    out[g] = r;
    valid[g] = 1;
  }
}

void group_quantile(const ColView &v, const int64_t *perm, const int64_t *offs, int64_t ngroups, double q,
                    double *out, uint8_t *valid, void *stream) {
  if (ngroups == 0) return;
  hipLaunchKernelGGL(k_quantile, dim3(grid_for(ngroups)), dim3(kBlock), 0, as_stream(stream), v, perm, offs, ngroups, q,
                     out, valid);
  HIP_LAUNCH_CHECK();
}

// this file's code object is loaded at context creation (preload_device_code), not on first use
void preload_groupby() { preload_code(reinterpret_cast<const void *>(&k_group_insert)); }

}  // namespace hip
}  // namespace cylon
