// K5 hash join build/probe, generic row hashing and row equality (gfx950).
//
// Reference: cpp/src/cylon/join/hash_join.cpp:21-346 (std::unordered_multimap of
// key -> row on the build side; probe emits (probe, build) index pairs),
// multi-key variant via TwoTableRowIndexHash (arrow_comparator.cpp:449-528).
//
// MI355X design: the build side goes into an open-addressing multimap of
// 16-byte {key, row} slots (load factor <= 0.5, linear probing, fmix64 slot
// hash) living in HBM.  A probe step is a single global_load_dwordx4; linear
// probing keeps the collision chain inside one 128-B line most of the time.
// Output cardinality is unknown, so the probe runs twice: a count pass, a
// device-wide scan (scan.hip) and a write pass that emits pairs in probe-row
// order (deterministic output).  Multi-column, nullable and var-width keys are
// reduced to a 64-bit row hash first; candidate pairs are then confirmed by
// rows_equal (null == null, pandas semantics).
#include "device_common.hpp"

namespace cylon {
namespace hip {

struct ColSet2 {
  ColView c[kMaxFusedCols];
};

__global__ void k_table_init(HashSlot *table, int64_t cap) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < cap; i += stride) {
    HashSlot s;
    s.key = 0;
    s.row = -1;
    table[i] = s;
  }
}

void hash_table_init(HashSlot *table, int64_t cap, void *stream) {
  hipLaunchKernelGGL(k_table_init, dim3(grid_for(cap)), dim3(kBlock), 0, as_stream(stream), table, cap);
  HIP_LAUNCH_CHECK();
}

__global__ void k_hash_build(const int64_t *__restrict__ keys, int64_t n, HashSlot *table, int64_t cap) {
  const uint64_t mask = (uint64_t)cap - 1;
  const int shift = 64 - __builtin_ctzll((unsigned long long)cap);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t k = keys[i];
    uint64_t slot = hashing::slot_of((uint64_t)k, shift);
    while (true) {
      unsigned long long *rowp = reinterpret_cast<unsigned long long *>(&table[slot].row);
      const unsigned long long prev = atomicCAS(rowp, ~0ull, (unsigned long long)i);
      if (prev == ~0ull) {
        table[slot].key = k;
        break;
      }
      slot = (slot + 1) & mask;
    }
  }
}

void hash_build(const int64_t *keys, int64_t n, HashSlot *table, int64_t cap, void *stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_hash_build, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), keys, n, table, cap);
  HIP_LAUNCH_CHECK();
}

__global__ void k_hash_probe_count(const int64_t *__restrict__ keys, int64_t n, const HashSlot *__restrict__ table,
                                   int64_t cap, int64_t *__restrict__ counts) {
  const uint64_t mask = (uint64_t)cap - 1;
  const int shift = 64 - __builtin_ctzll((unsigned long long)cap);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t k = keys[i];
    uint64_t slot = hashing::slot_of((uint64_t)k, shift);
    int64_t c = 0;
    while (true) {
      const HashSlot s = table[slot];
      if (s.row < 0) break;
      c += (s.key == k);
      slot = (slot + 1) & mask;
    }
    counts[i] = c;
  }
}

void hash_probe_count(const int64_t *keys, int64_t n, const HashSlot *table, int64_t cap, int64_t *counts,
                      void *stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_hash_probe_count, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), keys, n, table,
                     cap, counts);
  HIP_LAUNCH_CHECK();
}

__global__ void k_hash_probe_write(const int64_t *__restrict__ keys, int64_t n, const HashSlot *__restrict__ table,
                                   int64_t cap, const int64_t *__restrict__ offsets, int64_t *__restrict__ out_p,
                                   int64_t *__restrict__ out_b) {
  const uint64_t mask = (uint64_t)cap - 1;
  const int shift = 64 - __builtin_ctzll((unsigned long long)cap);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    int64_t o = offsets[i];
    const int64_t end = offsets[i + 1];
    if (o == end) continue;
    const int64_t k = keys[i];
    uint64_t slot = hashing::slot_of((uint64_t)k, shift);
    while (o < end) {
      const HashSlot s = table[slot];
      if (s.row < 0) break;
      if (s.key == k) {
        out_p[o] = i;
        out_b[o] = s.row;
        ++o;
      }
      slot = (slot + 1) & mask;
    }
  }
}

void hash_probe_write(const int64_t *keys, int64_t n, const HashSlot *table, int64_t cap, const int64_t *offsets,
                      int64_t *out_probe, int64_t *out_build, void *stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_hash_probe_write, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), keys, n, table,
                     cap, offsets, out_probe, out_build);
  HIP_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------
// generic keys
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t value_hash64(const ColView &c, int64_t i) {
  if (c.valid != nullptr && c.valid[i] == 0) return 0x5bd1e9955bd1e995ULL;  // null token
  if (c.kind == static_cast<int>(ValueKind::VAR_BYTES)) {
    const int64_t b = c.offsets[i], e = c.offsets[i + 1];
    const uint32_t h1 = hashing::murmur3_32(c.data + b, e - b, 0u);
    const uint32_t h2 = hashing::murmur3_32(c.data + b, e - b, 0x9747b28cu);
    return ((uint64_t)h1 << 32) ^ h2 ^ (uint64_t)(e - b);
  }
  if (c.kind == static_cast<int>(ValueKind::FIXED_BYTES)) {
    const uint32_t h1 = hashing::murmur3_32(c.data + i * (int64_t)c.width, c.width, 0u);
    const uint32_t h2 = hashing::murmur3_32(c.data + i * (int64_t)c.width, c.width, 0x9747b28cu);
    return ((uint64_t)h1 << 32) ^ h2;
  }
  return hashing::fmix64((uint64_t)extend_bits(load_bits(c.data, i, c.width), c.width, c.kind));
}

__global__ void k_row_hash64(ColSet2 cols, int ncols, int64_t n, uint64_t *__restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    uint64_t h = 0x84222325cbf29ce4ULL;
    for (int c = 0; c < ncols; ++c) h = hashing::combine64(h, value_hash64(cols.c[c], i));
    out[i] = h;
  }
}

void row_hash64(const ColView *cols, int ncols, int64_t n, uint64_t *out, void *stream) {
  if (n == 0) return;
  CYLON_CHECK(ncols <= kMaxFusedCols, Code::Invalid, "too many key columns " << ncols);
  ColSet2 s;
  for (int c = 0; c < ncols; ++c) s.c[c] = cols[c];
  hipLaunchKernelGGL(k_row_hash64, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), s, ncols, n, out);
  HIP_LAUNCH_CHECK();
}

__global__ void k_key64(ColView c, int64_t n, int64_t *__restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    out[i] = extend_bits(load_bits(c.data, i, c.width), c.width, c.kind);
}

void key64_from_column(const ColView &col, int64_t n, int64_t *out, void *stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_key64, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), col, n, out);
  HIP_LAUNCH_CHECK();
}

__device__ __forceinline__ bool value_equal(const ColView &a, int64_t i, const ColView &b, int64_t j) {
  const bool va = a.valid == nullptr || a.valid[i] != 0;
  const bool vb = b.valid == nullptr || b.valid[j] != 0;
  if (!va || !vb) return va == vb;
  if (a.kind == static_cast<int>(ValueKind::VAR_BYTES)) {
    const int64_t ab = a.offsets[i], al = a.offsets[i + 1] - ab;
    const int64_t bb = b.offsets[j], bl = b.offsets[j + 1] - bb;
    if (al != bl) return false;
    for (int64_t k = 0; k < al; ++k)
      if (a.data[ab + k] != b.data[bb + k]) return false;
    return true;
  }
  if (a.kind == static_cast<int>(ValueKind::FIXED_BYTES)) {
    const int w = a.width;
    for (int k = 0; k < w; ++k)
      if (a.data[i * w + k] != b.data[j * w + k]) return false;
    return true;
  }
  const int64_t x = extend_bits(load_bits(a.data, i, a.width), a.width, a.kind);
  const int64_t y = extend_bits(load_bits(b.data, j, b.width), b.width, b.kind);
  if (a.kind == static_cast<int>(ValueKind::FLOAT)) {
    if (a.width == 8) {
      const double dx = __longlong_as_double(x), dy = __longlong_as_double(y);
      return dx == dy || (dx != dx && dy != dy);
    }
    if (a.width == 4) {
      const float fx = __int_as_float((int)x), fy = __int_as_float((int)y);
      return fx == fy || (fx != fx && fy != fy);
    }
  }
  return x == y;
}

__global__ void k_rows_equal(ColSet2 l, ColSet2 r, int ncols, const int64_t *__restrict__ li,
                             const int64_t *__restrict__ ri, int64_t m, uint8_t *__restrict__ eq) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride) {
    const int64_t a = li[j], b = ri[j];
    bool e = true;
    for (int c = 0; c < ncols && e; ++c) e = value_equal(l.c[c], a, r.c[c], b);
    eq[j] = e ? 1 : 0;
  }
}

void rows_equal(const ColView *l, const ColView *r, int ncols, const int64_t *li, const int64_t *ri, int64_t m,
                uint8_t *eq, void *stream) {
  if (m == 0) return;
  CYLON_CHECK(ncols <= kMaxFusedCols, Code::Invalid, "too many key columns " << ncols);
  ColSet2 a, b;
  for (int c = 0; c < ncols; ++c) {
    a.c[c] = l[c];
    b.c[c] = r[c];
  }
  hipLaunchKernelGGL(k_rows_equal, dim3(grid_for(m)), dim3(kBlock), 0, as_stream(stream), a, b, ncols, li, ri, m,
                     eq);
  HIP_LAUNCH_CHECK();
}

__global__ void k_radix_part_ids(const int64_t *__restrict__ keys, int64_t n, int bits, uint32_t *__restrict__ pid) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    pid[i] = hashing::radix_part_of((uint64_t)keys[i], bits);
}

void radix_partition_ids(const int64_t *keys, int64_t n, int bits, uint32_t *pid, void *stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_radix_part_ids, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), keys, n, bits, pid);
  HIP_LAUNCH_CHECK();
}

}  // namespace hip
}  // namespace cylon
