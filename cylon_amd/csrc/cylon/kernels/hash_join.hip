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
#include "radix_pass.hpp"

namespace cylon {
namespace hip {

struct ColSet2 {
  ColView c[kMaxFusedCols];
};

__global__ void k_table_init(HashSlot *table, int64_t tsize) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < tsize; i += stride) {
    HashSlot s;
    s.key = 0;
    s.row = -1;
    table[i] = s;
  }
}

void hash_table_init(HashSlot *table, int64_t tsize, void *stream) {
  hipLaunchKernelGGL(k_table_init, dim3(grid_for(tsize)), dim3(kBlock), 0, as_stream(stream), table, tsize);
  HIP_LAUNCH_CHECK();
}

__device__ __forceinline__ int64_t next_slot(int64_t s, int64_t tsize) { return (s + 1 == tsize) ? 0 : s + 1; }

// atomic build (small build sides): CAS on the row word claims a slot
__global__ void k_hash_build(const int64_t *__restrict__ keys, int64_t n, HashTableRef t) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t k = keys[i];
    int64_t slot = (int64_t)hashing::slot_of((uint64_t)k, t.shift);
    while (true) {
      unsigned long long *rowp = reinterpret_cast<unsigned long long *>(&t.slots[slot].row);
      const unsigned long long prev = atomicCAS(rowp, ~0ull, (unsigned long long)i);
      if (prev == ~0ull) {
        t.slots[slot].key = k;
        break;
      }
      slot = next_slot(slot, t.tsize);
    }
  }
}

void hash_build(const int64_t *keys, int64_t n, HashTableRef t, void *stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_hash_build, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), keys, n, t);
  HIP_LAUNCH_CHECK();
}

// ---- atomic-free build (large build sides) --------------------------------
// (1) LSD radix sort of (key, row) by the key's slot (SlotDigit, 8-bit staged
//     passes); (2) linear-probing placement of keys inserted in slot order is
//     pos_i = i + max_{j<=i}(slot_j - j): one inclusive max-scan; (3) plain,
//     sequential stores of the slots.  No atomics, no random writes.
__global__ void k_slot_minus_index(const uint64_t *__restrict__ skeys, int64_t n, int shift,
                                   int64_t *__restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    out[i] = (int64_t)hashing::slot_of(skeys[i], shift) - i;
}

int64_t hash_build_sorted_workspace(int64_t n) {
  return std::max(stable_rank_workspace(n, kRadixBuckets), max_scan_workspace(n));
}

int hash_build_sorted(const int64_t *keys, int64_t n, int shift, int64_t *ws, uint64_t *ka, int64_t *va,
                      uint64_t *kb, int64_t *vb, int64_t *maxpos, void *stream) {
  hipStream_t s = as_stream(stream);
  const int lg = 64 - shift;
  uint64_t *kbuf[2] = {ka, kb};
  int64_t *vbuf[2] = {va, vb};
  int cur = -1;
  for (int sh = 0; sh < lg; sh += kRadixBits) {
    const uint64_t *kin = cur < 0 ? reinterpret_cast<const uint64_t *>(keys) : kbuf[cur];
    const int64_t *vin = cur < 0 ? nullptr : vbuf[cur];
    const int nxt = cur < 0 ? 0 : cur ^ 1;
    radix_pass(SlotDigit{shift, sh}, kin, vin, kbuf[nxt], vbuf[nxt], n, ws, s);
    cur = nxt;
  }
  // pos_i = i + max_{j<=i}(slot_j - j), written into the other buffer's value array
  int64_t *t = vbuf[cur ^ 1];
  hipLaunchKernelGGL(k_slot_minus_index, dim3(grid_for(n)), dim3(kBlock), 0, s, kbuf[cur], n, shift, t);
  HIP_LAUNCH_CHECK();
  int64_t *pm = reinterpret_cast<int64_t *>(kbuf[cur ^ 1]);
  inclusive_max_scan(t, n, pm, ws, stream);
  HIP_CHECK(hipMemcpyAsync(maxpos, pm + n - 1, sizeof(int64_t), hipMemcpyDeviceToDevice, s));
  return cur;
}

__global__ void k_place(const uint64_t *__restrict__ skeys, const int64_t *__restrict__ srows,
                        const int64_t *__restrict__ pmax, int64_t n, HashSlot *__restrict__ slots) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    HashSlot v;
    v.key = (int64_t)skeys[i];
    v.row = srows[i];
    slots[pmax[i] + i] = v;
  }
}

void hash_table_place(const uint64_t *skeys, const int64_t *srows, const int64_t *pmax, int64_t n, HashTableRef t,
                      void *stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_place, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), skeys, srows, pmax, n, t.slots);
  HIP_LAUNCH_CHECK();
}

// ---- probes ---------------------------------------------------------------
__global__ void k_hash_probe_count(const int64_t *__restrict__ keys, int64_t n, HashTableRef t,
                                   int64_t *__restrict__ counts) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t k = keys[i];
    int64_t slot = (int64_t)hashing::slot_of((uint64_t)k, t.shift);
    int64_t c = 0;
    while (true) {
      const HashSlot s = t.slots[slot];
      if (s.row < 0) break;
      c += (s.key == k);
      slot = next_slot(slot, t.tsize);
    }
    counts[i] = c;
  }
}

void hash_probe_count(const int64_t *keys, int64_t n, HashTableRef t, int64_t *counts, void *stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_hash_probe_count, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), keys, n, t, counts);
  HIP_LAUNCH_CHECK();
}

__global__ void k_hash_probe_write(const int64_t *__restrict__ keys, int64_t n, HashTableRef t,
                                   const int64_t *__restrict__ offsets, int64_t *__restrict__ out_p,
                                   int64_t *__restrict__ out_b) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    int64_t o = offsets[i];
    const int64_t end = offsets[i + 1];
    if (o == end) continue;
    const int64_t k = keys[i];
    int64_t slot = (int64_t)hashing::slot_of((uint64_t)k, t.shift);
    while (o < end) {
      const HashSlot s = t.slots[slot];
      if (s.row < 0) break;
      if (s.key == k) {
        out_p[o] = i;
        out_b[o] = s.row;
        ++o;
      }
      slot = next_slot(slot, t.tsize);
    }
  }
}

void hash_probe_write(const int64_t *keys, int64_t n, HashTableRef t, const int64_t *offsets, int64_t *out_probe,
                      int64_t *out_build, void *stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_hash_probe_write, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), keys, n, t, offsets,
                     out_probe, out_build);
  HIP_LAUNCH_CHECK();
}

// Single-pass probe: each wave counts its matches, reserves output space with
// ONE atomic add (wave64 shuffle scan of the per-lane counts) and re-walks the
// chains (now L1/L2 hot) to write its pairs.  Output order across waves is not
// deterministic.  If the reservation exceeds `capacity` nothing more is
// written and the caller falls back to the exact two-pass probe.
__global__ __launch_bounds__(kBlock) void k_hash_probe_emit(const int64_t *__restrict__ keys, int64_t n,
                                                            HashTableRef t, int64_t capacity,
                                                            unsigned long long *counter, int64_t *__restrict__ out_p,
                                                            int64_t *__restrict__ out_b) {
  const int lane = lane_id();
  const int64_t wstride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t base = (int64_t)blockIdx.x * blockDim.x + (threadIdx.x & ~(kWave - 1)); base < n; base += wstride) {
    const int64_t i = base + lane;
    const bool active = i < n;
    int64_t k = 0, slot0 = 0, c = 0;
    if (active) {
      k = keys[i];
      slot0 = (int64_t)hashing::slot_of((uint64_t)k, t.shift);
      int64_t slot = slot0;
      while (true) {
        const HashSlot s = t.slots[slot];
        if (s.row < 0) break;
        c += (s.key == k);
        slot = next_slot(slot, t.tsize);
      }
    }
    int64_t inc = c;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
      const int64_t x = __shfl_up(inc, d, kWave);
      if (lane >= d) inc += x;
    }
    const int64_t total = __shfl(inc, kWave - 1, kWave);
    if (total == 0) continue;
    unsigned long long wbase = 0;
    if (lane == 0) wbase = atomicAdd(counter, (unsigned long long)total);
    wbase = __shfl(wbase, 0, kWave);
    if ((int64_t)wbase + total > capacity) continue;  // overflow: counted, not written
    int64_t o = (int64_t)wbase + inc - c;
    if (c > 0) {
      int64_t slot = slot0;
      int64_t left = c;
      while (left > 0) {
        const HashSlot s = t.slots[slot];
        if (s.key == k && s.row >= 0) {
          out_p[o] = i;
          out_b[o] = s.row;
          ++o;
          --left;
        }
        slot = next_slot(slot, t.tsize);
      }
    }
  }
}

void hash_probe_emit(const int64_t *keys, int64_t n, HashTableRef t, int64_t capacity, int64_t *counter,
                     int64_t *out_probe, int64_t *out_build, void *stream) {
  hipStream_t s = as_stream(stream);
  HIP_CHECK(hipMemsetAsync(counter, 0, sizeof(int64_t), s));
  if (n == 0) return;
  hipLaunchKernelGGL(k_hash_probe_emit, dim3(grid_for(n)), dim3(kBlock), 0, s, keys, n, t, capacity,
                     reinterpret_cast<unsigned long long *>(counter), out_probe, out_build);
  HIP_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------
// generic keys
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t value_hash64(const ColView &c, int64_t i) {
  if (c.valid != nullptr && c.valid[i] == 0) return 0x5bd1e9955bd1e995ULL;  // null token
  if (c.kind == static_cast<int>(ValueKind::VAR_BYTES)) {
    const int64_t b = c.offsets[i], e = c.offsets[i + 1];
    return hashing::bytes_hash64(c.data + b, e - b);
  }
  if (c.kind == static_cast<int>(ValueKind::FIXED_BYTES)) {
    return hashing::bytes_hash64(c.data + i * (int64_t)c.width, c.width);
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

// K5 exact composite key of several integer key columns (ops/join.cpp radix_keys): one pass reads
// every key column at its own width and writes the packed int64 -- the LDS radix join then moves
// ONE 8-byte key instead of the image plus each key column; unpack rebuilds the key columns of the
// join output from the composite the kernel wrote (one read, one write per key column).
struct CompositeSpec {
  ColView c[kMaxCompositeKeys];
  MutColView o[kMaxCompositeKeys];
  int64_t lo[kMaxCompositeKeys];
  uint64_t mask[kMaxCompositeKeys];
  int64_t ncode[kMaxCompositeKeys];  // field value of a null (-1: the column has no nulls)
  int shift[kMaxCompositeKeys];
};

template <int NK>
__global__ void k_composite_pack(CompositeSpec s, int64_t n, int64_t *__restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    uint64_t acc = 0;
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      uint64_t f = (uint64_t)(extend_bits(load_bits(s.c[k].data, i, s.c[k].width), s.c[k].width, s.c[k].kind) - s.lo[k]);
      if (s.ncode[k] >= 0 && s.c[k].valid && !s.c[k].valid[i]) f = (uint64_t)s.ncode[k];
      acc |= f << s.shift[k];
    }
    out[i] = (int64_t)acc;
  }
}

template <int NK>
__global__ void k_composite_unpack(CompositeSpec s, int64_t n, const int64_t *__restrict__ key) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint64_t v = (uint64_t)key[i];
#pragma unroll
    for (int k = 0; k < NK; ++k) {
      const uint64_t f = (v >> s.shift[k]) & s.mask[k];
      if (s.ncode[k] >= 0 && f == (uint64_t)s.ncode[k] && s.o[k].valid) s.o[k].valid[i] = 0;
      const uint64_t x = (uint64_t)s.lo[k] + f;
      switch (s.o[k].width) {
        case 1: s.o[k].data[i] = (uint8_t)x; break;
        case 2: reinterpret_cast<uint16_t *>(s.o[k].data)[i] = (uint16_t)x; break;
        case 4: reinterpret_cast<uint32_t *>(s.o[k].data)[i] = (uint32_t)x; break;
        default: reinterpret_cast<uint64_t *>(s.o[k].data)[i] = x; break;
      }
    }
  }
}

static CompositeSpec composite_spec(int nk, const int64_t *lo, const int *shift, const int *bits,
                                    const int64_t *ncode) {
  CYLON_CHECK(nk >= 1 && nk <= kMaxCompositeKeys, Code::Invalid, "composite key of " << nk << " columns");
  CompositeSpec s;
  for (int k = 0; k < nk; ++k) {
    s.lo[k] = lo[k];
    s.ncode[k] = ncode ? ncode[k] : -1;
    s.shift[k] = shift[k];
    s.mask[k] = bits ? (bits[k] >= 64 ? ~0ull : ((1ull << bits[k]) - 1)) : 0;
  }
  return s;
}

#define CYLON_NK_SWITCH(nk, KERNEL, ...)                                                                     \
  switch (nk) {                                                                                              \
    case 1: hipLaunchKernelGGL(KERNEL<1>, __VA_ARGS__); break;                                               \
    case 2: hipLaunchKernelGGL(KERNEL<2>, __VA_ARGS__); break;                                               \
    case 3: hipLaunchKernelGGL(KERNEL<3>, __VA_ARGS__); break;                                               \
    default: hipLaunchKernelGGL(KERNEL<4>, __VA_ARGS__); break;                                              \
  }

void composite_key_pack(const ColView *cols, int nk, const int64_t *lo, const int *shift, int64_t n, int64_t *out,
                        const int64_t *ncode, void *stream) {
  if (n == 0) return;
  CompositeSpec s = composite_spec(nk, lo, shift, nullptr, ncode);
  for (int k = 0; k < nk; ++k) s.c[k] = cols[k];
  CYLON_NK_SWITCH(nk, k_composite_pack, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), s, n, out);
  HIP_LAUNCH_CHECK();
}

void composite_key_unpack(const int64_t *key, int64_t n, int nk, const int64_t *lo, const int *shift, const int *bits,
                          const MutColView *out, const int64_t *ncode, void *stream) {
  if (n == 0) return;
  CompositeSpec s = composite_spec(nk, lo, shift, bits, ncode);
  for (int k = 0; k < nk; ++k) s.o[k] = out[k];
  CYLON_NK_SWITCH(nk, k_composite_unpack, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), s, n, key);
  HIP_LAUNCH_CHECK();
}
#undef CYLON_NK_SWITCH

// K8 float group key: the float64 image's bits with -0.0 -> +0.0 and every NaN -> one quiet NaN
// (float32 widened first), one read and one write (the torch where/isnan chain took ~5 passes)
__global__ void k_float_key_bits(ColView c, int64_t n, int64_t *__restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    double v = c.width == 8 ? reinterpret_cast<const double *>(c.data)[i]
                            : (double)reinterpret_cast<const float *>(c.data)[i];
    if (v == 0.0) v = 0.0;
    int64_t b = __double_as_longlong(v);
    if (v != v) b = 0x7ff8000000000000ll;
    out[i] = b;
  }
}

void float_key_bits(const ColView &c, int64_t n, int64_t *out, void *stream) {
  if (n == 0) return;
  CYLON_CHECK(c.width == 8 || c.width == 4, Code::Invalid, "float key of width " << c.width);
  hipLaunchKernelGGL(k_float_key_bits, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), c, n, out);
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

// this file's code object is loaded at context creation (preload_device_code), not on first use
void preload_hash_join() { preload_code(reinterpret_cast<const void *>(&k_table_init)); }

}  // namespace hip
}  // namespace cylon
