// K6 LSD radix sort of (uint64 key, int64 value) pairs and K7 sort-merge join
// expansion (gfx950).
//
// Reference: cpp/src/cylon/arrow/arrow_kernels.cpp:199-465 (IndexSortKernel,
// InplaceIndexSortKernel = introsort, multi-column comparator chains) and
// cpp/src/cylon/join/sort_join.cpp:110-370 (advance equal runs, cross product).
//
// MI355X design:
//   * keys are first mapped to order-preserving unsigned 64-bit images
//     (sign flip for ints, IEEE flip for floats, bitwise NOT for descending),
//     so every column type sorts with the same unsigned radix passes;
//   * one OR/AND reduction over the keys finds the byte positions that are
//     constant across all keys; those passes are skipped (an int64 key column
//     holding values < 2^32 needs 4 passes, not 8);
//   * each 8-bit pass = block histogram (LDS) -> scan -> stable rank kernel
//     (stable_rank.hpp: wave64 ballot-match ranking, 256 buckets) that
//     scatters key and value directly (no intermediate position array);
//   * merge join: per left key a lower/upper bound search in the sorted right
//     keys (count pass stores the lower bound), scan, and a write pass that
//     expands the equal range into (left row, right row) pairs.
#include "radix_pass.hpp"

namespace cylon {
namespace hip {

// ---------------------------------------------------------------------------
// key images
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t order_image(uint64_t bits, int w, int kind) {
  const int nb = 8 * w;
  const uint64_t mask = (nb == 64) ? ~0ull : ((1ull << nb) - 1);
  const uint64_t sign = 1ull << (nb - 1);
  bits &= mask;
  if (kind == static_cast<int>(ValueKind::SIGNED_INT)) return bits ^ sign;
  if (kind == static_cast<int>(ValueKind::FLOAT)) {
    // canonicalise -0.0 to +0.0 and every NaN to the positive quiet NaN (sorts last)
    if (bits == sign) bits = 0;
    const uint64_t exp_mask = (w == 8) ? 0x7ff0000000000000ull : (w == 4 ? 0x7f800000ull : 0x7c00ull);
    const uint64_t man_mask = (w == 8) ? 0x000fffffffffffffull : (w == 4 ? 0x007fffffull : 0x03ffull);
    if ((bits & exp_mask) == exp_mask && (bits & man_mask) != 0) bits = exp_mask | ((man_mask + 1) >> 1);
    return (bits & sign) ? (~bits & mask) : (bits | sign);
  }
  return bits;
}

__device__ __forceinline__ bool is_nan_bits(uint64_t bits, int w) {
  if (w == 8) return (bits & 0x7ff0000000000000ull) == 0x7ff0000000000000ull && (bits & 0x000fffffffffffffull);
  if (w == 4) return (bits & 0x7f800000ull) == 0x7f800000ull && (bits & 0x007fffffull);
  return (bits & 0x7c00ull) == 0x7c00ull && (bits & 0x03ffull);
}

// acc != nullptr: also OR / AND-reduce the images into acc[0] / acc[1] (the bits
// that vary, for the radix pass count) so the sort needs no second read of them
__global__ void k_sort_keys(ColView c, const int64_t *__restrict__ perm, int64_t n, bool desc,
                            uint64_t *__restrict__ out, unsigned long long *acc) {
  const int nb = 8 * c.width;
  uint64_t o = 0, a = ~0ull;
  const uint64_t mask = (nb == 64) ? ~0ull : ((1ull << nb) - 1);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t s = perm ? perm[i] : i;
    const uint64_t bits = load_bits(c.data, s, c.width);
    uint64_t k = order_image(bits, c.width, c.kind);
    if (desc) k = ~k & mask;
    if (c.kind == static_cast<int>(ValueKind::FLOAT) && is_nan_bits(bits, c.width)) k = mask;  // NaN last
    // a null's image is a constant: null rows keep their order from the previous (less
    // significant) sort columns, so equal rows stay adjacent in multi-column sorts
    if (c.valid != nullptr && c.valid[s] == 0) k = mask;
    if (out != nullptr) out[i] = k;  // null: reduction only (8-byte integer keys imaged by the first pass)
    o |= k;
    a &= k;
  }
  if (acc == nullptr) return;
#pragma unroll
  for (int d = kWave / 2; d > 0; d >>= 1) {
    o |= __shfl_xor(o, d, kWave);
    a &= __shfl_xor(a, d, kWave);
  }
  if (lane_id() == 0) {
    atomicOr(&acc[0], (unsigned long long)o);
    atomicAnd(&acc[1], (unsigned long long)a);
  }
}

void sort_keys_from_column(const ColView &col, const int64_t *perm, int64_t n, bool desc, uint64_t *out,
                           void *stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_sort_keys, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), col, perm, n, desc, out,
                     nullptr);
  HIP_LAUNCH_CHECK();
}


// OR / AND accumulators of a key scan (varying bits = OR ^ AND): acc[0] = 0, acc[1] = ~0
// are set on the stream (no host staging), the readback is the only synchronisation.
static unsigned long long *or_and_init(int64_t *ws2, hipStream_t s) {
  unsigned long long *acc = reinterpret_cast<unsigned long long *>(ws2);
  HIP_CHECK(hipMemsetAsync(acc, 0, sizeof(unsigned long long), s));
  HIP_CHECK(hipMemsetAsync(acc + 1, 0xff, sizeof(unsigned long long), s));
  return acc;
}

static uint64_t or_and_diff(const unsigned long long *acc, hipStream_t s) {
  unsigned long long oa[2];
  HIP_CHECK(hipMemcpyAsync(oa, acc, sizeof(oa), hipMemcpyDeviceToHost, s));
  HIP_CHECK(hipStreamSynchronize(s));
  return oa[0] ^ oa[1];
}

uint64_t sort_keys_varying_bits(const ColView &col, int64_t n, bool desc, uint64_t *out, int64_t *ws2,
                                void *stream) {
  if (n == 0) return 0;
  hipStream_t s = as_stream(stream);
  unsigned long long *acc = or_and_init(ws2, s);
  hipLaunchKernelGGL(k_sort_keys, dim3(grid_for(n)), dim3(kBlock), 0, s, col, nullptr, n, desc, out, acc);
  HIP_LAUNCH_CHECK();
  const uint64_t diff = or_and_diff(acc, s);
  return n <= 1 ? 0 : diff;
}

// ---------------------------------------------------------------------------
// radix sort
// ---------------------------------------------------------------------------
__global__ void k_or_and(const uint64_t *__restrict__ k, int64_t n, unsigned long long *acc) {
  uint64_t o = 0, a = ~0ull;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t v = k[i];
    o |= v;
    a &= v;
  }
#pragma unroll
  for (int d = kWave / 2; d > 0; d >>= 1) {
    o |= __shfl_xor(o, d, kWave);
    a &= __shfl_xor(a, d, kWave);
  }
  if (lane_id() == 0) {
    atomicOr(&acc[0], (unsigned long long)o);
    atomicAnd(&acc[1], (unsigned long long)a);
  }
}

struct RadixDigit {
  const uint64_t *keys;
  int shift;
  __device__ __forceinline__ uint32_t operator()(int64_t i) const { return (uint32_t)(keys[i] >> shift) & 0xffu; }
};

struct RadixSink {
  const uint64_t *kin;
  const int64_t *vin;
  uint64_t *kout;
  int64_t *vout;
  __device__ __forceinline__ void operator()(int64_t i, int64_t d) const {
    kout[d] = kin[i];
    vout[d] = vin[i];
  }
};

int64_t radix_sort_workspace(int64_t n) { return stable_rank_workspace(n, 256) + 2; }

uint64_t varying_bits(const uint64_t *keys, int64_t n, int64_t *ws2, void *stream) {
  if (n <= 1) return 0;
  hipStream_t s = as_stream(stream);
  unsigned long long *acc = or_and_init(ws2, s);
  hipLaunchKernelGGL(k_or_and, dim3(grid_for(n, kBlock, 1024)), dim3(kBlock), 0, s, keys, n, acc);
  HIP_LAUNCH_CHECK();
  return or_and_diff(acc, s);
}

int radix_sort_pairs(uint64_t *keys, int64_t *vals, int64_t n, uint64_t *keys_alt, int64_t *vals_alt, int begin_bit,
                     int end_bit, int64_t *ws, void *stream) {
  if (n <= 1) return 0;
  hipStream_t s = as_stream(stream);
  unsigned long long *acc = or_and_init(ws, s);
  hipLaunchKernelGGL(k_or_and, dim3(grid_for(n, kBlock, 1024)), dim3(kBlock), 0, s, keys, n, acc);
  HIP_LAUNCH_CHECK();
  const uint64_t diff = or_and_diff(acc, s);
  int cur = 0;
  uint64_t *kb[2] = {keys, keys_alt};
  int64_t *vb[2] = {vals, vals_alt};
  for (int shift = begin_bit; shift < end_bit; shift += 8) {
    if (((diff >> shift) & 0xffull) == 0) continue;  // constant digit: pass is the identity
    radix_pass(PlainDigit{shift}, kb[cur], vb[cur], kb[cur ^ 1], vb[cur ^ 1], n, ws + 2, s);
    cur ^= 1;
  }
  return cur;
}

// ---------------------------------------------------------------------------
// K7 merge join on sorted key arrays
// ---------------------------------------------------------------------------
__device__ __forceinline__ int64_t lower_bound_u64(const uint64_t *a, int64_t n, uint64_t v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] < v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__device__ __forceinline__ int64_t upper_bound_u64(const uint64_t *a, int64_t n, uint64_t v) {
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a[mid] <= v) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// Both key arrays are sorted, so a tile of 2048 consecutive left keys matches a
// contiguous right window [lb(first), ub(last)). k_merge_bounds finds each tile's
// window with two global binary searches (one thread per tile, all tiles in
// parallel); k_merge_count stages the tile and, when it fits, the window in LDS,
// and each thread walks its 8 consecutive left keys with a forward pointer
// (galloping to a binary search after a few steps, so sparse/dense mixes stay
// O(log) per key). This replaces one 30-step random-access global binary search
// per left row (72 ms at 1B x 1B) with two streaming reads.
constexpr int kMJThreads = 256;
constexpr int kMJPerThread = 8;
constexpr int kMJTile = kMJThreads * kMJPerThread;
constexpr int kMJWindow = 4096;

__device__ __forceinline__ int mj_pad(int i) { return i + i / kMJPerThread; }  // +1 slot per thread: no bank clash

// the window bounds of tile b are parked in lo_out[b*T] / counts[b*T]: only block b
// reads them, before it overwrites them
__global__ void k_merge_bounds(const uint64_t *__restrict__ lk, int64_t nl, const uint64_t *__restrict__ rk,
                               int64_t nr, int64_t *__restrict__ lo_out, int64_t *__restrict__ counts) {
  const int64_t tiles = (nl + kMJTile - 1) / kMJTile;
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= tiles) return;
  const int64_t base = b * kMJTile;
  const int64_t last = (base + kMJTile < nl ? base + kMJTile : nl) - 1;
  const uint64_t first_key = lk[base], last_key = lk[last];
  lo_out[base] = lower_bound_u64(rk, nr, first_key);
  counts[base] = upper_bound_u64(rk, nr, last_key);
}

template <typename RP>
__device__ __forceinline__ void mj_walk(const uint64_t *lt, RP rw, int64_t wn, int r0, int rows, int64_t *lo_v,
                                        int64_t *c_v) {
  if (r0 >= rows) return;
  int64_t p = 0;
  {
    int64_t hi = wn;
    const uint64_t v = lt[mj_pad(r0)];
    while (p < hi) {
      const int64_t mid = (p + hi) >> 1;
      if (rw[mid] < v) p = mid + 1; else hi = mid;
    }
  }
#pragma unroll
  for (int j = 0; j < kMJPerThread; ++j) {
    if (r0 + j < rows) {
      const uint64_t v = lt[mj_pad(r0 + j)];
      int step = 0;
      while (p < wn && rw[p] < v && step < 4) { ++p; ++step; }
      if (p < wn && rw[p] < v) {
        int64_t hi = wn;
        while (p < hi) {
          const int64_t mid = (p + hi) >> 1;
          if (rw[mid] < v) p = mid + 1; else hi = mid;
        }
      }
      int64_t q = p;
      step = 0;
      while (q < wn && rw[q] == v && step < 4) { ++q; ++step; }
      if (q < wn && rw[q] == v) {
        int64_t hi = wn;
        while (q < hi) {
          const int64_t mid = (q + hi) >> 1;
          if (rw[mid] <= v) q = mid + 1; else hi = mid;
        }
      }
      lo_v[j] = p;
      c_v[j] = q - p;
    }
  }
}

__global__ __launch_bounds__(kMJThreads) void k_merge_count(const uint64_t *__restrict__ lk, int64_t nl,
                                                            const uint64_t *__restrict__ rk, int64_t nr,
                                                            int64_t *__restrict__ lo_out,
                                                            int64_t *__restrict__ counts) {
  __shared__ uint64_t lt[kMJTile + kMJThreads];
  __shared__ uint64_t rw[kMJWindow];
  const int64_t base = (int64_t)blockIdx.x * kMJTile;
  const int rows = (int)(nl - base < kMJTile ? nl - base : kMJTile);
  const int64_t rs = lo_out[base], wn = counts[base] - rs;
  const int tid = threadIdx.x;
  for (int i = tid; i < rows; i += kMJThreads) lt[mj_pad(i)] = lk[base + i];
  const bool in_lds = wn <= kMJWindow;
  if (in_lds)
    for (int i = tid; i < wn; i += kMJThreads) rw[i] = rk[rs + i];
  __syncthreads();
  const int r0 = tid * kMJPerThread;
  int64_t lo_v[kMJPerThread], c_v[kMJPerThread];
  if (in_lds) mj_walk(lt, (const uint64_t *)rw, wn, r0, rows, lo_v, c_v);
  else mj_walk(lt, rk + rs, wn, r0, rows, lo_v, c_v);
  // stage both outputs through the tile buffer so the global stores coalesce
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kMJPerThread; ++j)
    if (r0 + j < rows) lt[mj_pad(r0 + j)] = (uint64_t)(rs + lo_v[j]);
  __syncthreads();
  for (int i = tid; i < rows; i += kMJThreads) lo_out[base + i] = (int64_t)lt[mj_pad(i)];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kMJPerThread; ++j)
    if (r0 + j < rows) lt[mj_pad(r0 + j)] = (uint64_t)c_v[j];
  __syncthreads();
  for (int i = tid; i < rows; i += kMJThreads) counts[base + i] = (int64_t)lt[mj_pad(i)];
}

__global__ void k_merge_write(const int64_t *__restrict__ lperm, int64_t nl, const int64_t *__restrict__ rperm,
                              const int64_t *__restrict__ lo, const int64_t *__restrict__ offs,
                              int64_t *__restrict__ out_l, int64_t *__restrict__ out_r) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < nl; i += stride) {
    const int64_t o = offs[i], c = offs[i + 1] - o;
    const int64_t l = lperm[i], b = lo[i];
    for (int64_t k = 0; k < c; ++k) {
      out_l[o + k] = l;
      out_r[o + k] = rperm[b + k];
    }
  }
}

void merge_join_count(const uint64_t *lk, int64_t nl, const uint64_t *rk, int64_t nr, int64_t *lo, int64_t *counts,
                      void *stream) {
  if (nl == 0) return;
  hipStream_t s = as_stream(stream);
  const int64_t tiles = (nl + kMJTile - 1) / kMJTile;
  hipLaunchKernelGGL(k_merge_bounds, dim3((unsigned)((tiles + kBlock - 1) / kBlock)), dim3(kBlock), 0, s, lk, nl, rk,
                     nr, lo, counts);
  HIP_LAUNCH_CHECK();
  hipLaunchKernelGGL(k_merge_count, dim3((unsigned)tiles), dim3(kMJThreads), 0, s, lk, nl, rk, nr, lo, counts);
  HIP_LAUNCH_CHECK();
}

void merge_join_write(const int64_t *lperm, int64_t nl, const int64_t *rperm, const int64_t *lo, const int64_t *offs,
                      int64_t *out_l, int64_t *out_r, void *stream) {
  if (nl == 0) return;
  hipLaunchKernelGGL(k_merge_write, dim3(grid_for(nl)), dim3(kBlock), 0, as_stream(stream), lperm, nl, rperm, lo,
                     offs, out_l, out_r);
  HIP_LAUNCH_CHECK();
}

}  // namespace hip
}  // namespace cylon

namespace cylon {
namespace hip {

__global__ void k_string_chunk_keys(ColView c, const int64_t *__restrict__ perm, int64_t n, int64_t chunk, bool desc,
                                    uint64_t *__restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t s = perm ? perm[i] : i;
    const int64_t b = c.offsets[s], len = c.offsets[s + 1] - b;
    uint64_t k = 0;
    if (chunk < 0) {
      k = (uint64_t)len;
    } else {
      const int64_t st = chunk * 8;
      for (int j = 0; j < 8; ++j) {
        const int64_t p = st + j;
        k = (k << 8) | (p < len ? (uint64_t)c.data[b + p] : 0ull);
      }
    }
    out[i] = (c.valid != nullptr && c.valid[s] == 0) ? ~0ull : (desc ? ~k : k);  // nulls: constant image
  }
}

void sort_string_chunk_keys(const ColView &col, const int64_t *perm, int64_t n, int64_t chunk, bool desc,
                            uint64_t *out, void *stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_string_chunk_keys, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), col, perm, n, chunk,
                     desc, out);
  HIP_LAUNCH_CHECK();
}

// this file's code object is loaded at context creation (preload_device_code), not on first use
void preload_sort() { preload_code(reinterpret_cast<const void *>(&k_sort_keys)); }

}  // namespace hip
}  // namespace cylon
