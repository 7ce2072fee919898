// CPU twins of the HIP primitives (kernels.hpp).  Same semantics and output
// order as the device versions; they run the engine on CPU tensors (gloo
// tests, BASELINE config 1) and serve as the in-tree oracle for the GPU
// numerics tests.
#include "strparse.hpp"
#include <algorithm>
#include <cstring>
#include <vector>
#include <cmath>

#include "kernels.hpp"
#include "../hash.hpp"
#include "../types.hpp"

namespace cylon {
namespace cpu {

namespace {

inline uint64_t load_bits(const uint8_t *base, int64_t i, int w) {
  switch (w) {
    case 1: return base[i];
    case 2: { uint16_t v; std::memcpy(&v, base + 2 * i, 2); return v; }
    case 4: { uint32_t v; std::memcpy(&v, base + 4 * i, 4); return v; }
    case 8: { uint64_t v; std::memcpy(&v, base + 8 * i, 8); return v; }
    default: return 0;
  }
}

inline int64_t extend_bits(uint64_t b, int w, int kind) {
  if (kind == static_cast<int>(ValueKind::SIGNED_INT)) {
    switch (w) {
      case 1: return (int64_t)(int8_t)b;
      case 2: return (int64_t)(int16_t)b;
      case 4: return (int64_t)(int32_t)b;
      default: return (int64_t)b;
    }
  }
  if (kind == static_cast<int>(ValueKind::FLOAT)) {
    if (w == 8 && b == 0x8000000000000000ull) return 0;
    if (w == 4 && b == 0x80000000ull) return 0;
    if (w == 2 && b == 0x8000ull) return 0;
  }
  return (int64_t)b;
}

inline uint32_t partition_f(const ColView &c, int64_t i) {
  if (c.valid != nullptr && c.valid[i] == 0) return 0u;
  if (c.kind == static_cast<int>(ValueKind::VAR_BYTES)) {
    const int64_t b = c.offsets[i], e = c.offsets[i + 1];
    return hashing::murmur3_32(c.data + b, e - b, 0u);
  }
  if (c.kind == static_cast<int>(ValueKind::FIXED_BYTES))
    return hashing::murmur3_32(c.data + i * (int64_t)c.width, c.width, 0u);
  const uint64_t bits = load_bits(c.data, i, c.width);
  if (c.kind == static_cast<int>(ValueKind::FLOAT)) {
    switch (c.width) {
      case 2: return hashing::murmur3_32_u16((uint16_t)bits);
      case 4: return hashing::murmur3_32_u32((uint32_t)bits);
      default: return hashing::murmur3_32_u64(bits);
    }
  }
  return (uint32_t)extend_bits(bits, c.width, c.kind);
}

inline void move_any(const uint8_t *src, int64_t si, uint8_t *dst, int64_t di, int w) {
  std::memcpy(dst + di * w, src + si * w, w);
}

inline uint64_t value_hash64(const ColView &c, int64_t i) {
  if (c.valid != nullptr && c.valid[i] == 0) return 0x5bd1e9955bd1e995ULL;
  if (c.kind == static_cast<int>(ValueKind::VAR_BYTES)) {
    const int64_t b = c.offsets[i], e = c.offsets[i + 1];
    return hashing::bytes_hash64(c.data + b, e - b);
  }
  if (c.kind == static_cast<int>(ValueKind::FIXED_BYTES)) {
    return hashing::bytes_hash64(c.data + i * (int64_t)c.width, c.width);
  }
  return hashing::fmix64((uint64_t)extend_bits(load_bits(c.data, i, c.width), c.width, c.kind));
}

inline bool value_equal(const ColView &a, int64_t i, const ColView &b, int64_t j) {
  const bool va = a.valid == nullptr || a.valid[i] != 0;
  const bool vb = b.valid == nullptr || b.valid[j] != 0;
  if (!va || !vb) return va == vb;
  if (a.kind == static_cast<int>(ValueKind::VAR_BYTES)) {
    const int64_t ab = a.offsets[i], al = a.offsets[i + 1] - ab;
    const int64_t bb = b.offsets[j], bl = b.offsets[j + 1] - bb;
    return al == bl && (al == 0 || std::memcmp(a.data + ab, b.data + bb, al) == 0);
  }
  if (a.kind == static_cast<int>(ValueKind::FIXED_BYTES))
    return std::memcmp(a.data + i * a.width, b.data + j * b.width, a.width) == 0;
  const int64_t x = extend_bits(load_bits(a.data, i, a.width), a.width, a.kind);
  const int64_t y = extend_bits(load_bits(b.data, j, b.width), b.width, b.kind);
  if (a.kind == static_cast<int>(ValueKind::FLOAT)) {
    if (a.width == 8) {
      double dx, dy;
      std::memcpy(&dx, &x, 8);
      std::memcpy(&dy, &y, 8);
      return dx == dy || (std::isnan(dx) && std::isnan(dy));
    }
    if (a.width == 4) {
      float fx, fy;
      uint32_t ux = (uint32_t)x, uy = (uint32_t)y;
      std::memcpy(&fx, &ux, 4);
      std::memcpy(&fy, &uy, 4);
      return fx == fy || (std::isnan(fx) && std::isnan(fy));
    }
  }
  return x == y;
}

}  // namespace

void row_partition_hash(const ColView *cols, int ncols, int64_t n, uint32_t *h, void *) {
  for (int64_t i = 0; i < n; ++i) {
    uint32_t acc = 0;
    for (int c = 0; c < ncols; ++c) acc = 31u * acc + partition_f(cols[c], i);
    h[i] = acc;
  }
}

void hash_to_partition(const uint32_t *h, int64_t n, uint32_t nparts, uint32_t *pid, int64_t *counts, void *) {
  std::memset(counts, 0, sizeof(int64_t) * nparts);
  for (int64_t i = 0; i < n; ++i) {
    const uint32_t p = hashing::partitioner(h[i], nparts);
    pid[i] = p;
    counts[p]++;
  }
}

int64_t partition_positions_workspace(int64_t, uint32_t nparts) { return nparts; }

void partition_positions(const uint32_t *pid, int64_t n, uint32_t nparts, int64_t *ws, int64_t *pos,
                         int64_t *counts, void *) {
  std::memset(counts, 0, sizeof(int64_t) * nparts);
  for (int64_t i = 0; i < n; ++i) counts[pid[i]]++;
  int64_t run = 0;
  for (uint32_t p = 0; p < nparts; ++p) {
    ws[p] = run;
    run += counts[p];
  }
  for (int64_t i = 0; i < n; ++i) pos[i] = ws[pid[i]]++;
}

void scatter_columns(const ColView *in, const MutColView *out, int ncols, const int64_t *pos, int64_t n, void *) {
  for (int c = 0; c < ncols; ++c) {
    const int w = in[c].width;
    for (int64_t i = 0; i < n; ++i) {
      const int64_t d = pos[i];
      move_any(in[c].data, i, out[c].data, d, w);
      if (out[c].valid) out[c].valid[d] = in[c].valid ? in[c].valid[i] : 1;
    }
  }
}

void scatter_var_lengths(const ColView &in, const int64_t *pos, int64_t n, int64_t *out_lens, void *) {
  for (int64_t i = 0; i < n; ++i) out_lens[pos[i]] = in.offsets[i + 1] - in.offsets[i];
}

void scatter_var_bytes(const ColView &in, const int64_t *pos, int64_t n, const int64_t *out_off,
                       uint8_t *out_bytes, uint8_t *out_valid, void *) {
  for (int64_t i = 0; i < n; ++i) {
    const int64_t d = pos[i];
    const int64_t sb = in.offsets[i], len = in.offsets[i + 1] - sb;
    if (len) std::memcpy(out_bytes + out_off[d], in.data + sb, len);
    if (out_valid) out_valid[d] = in.valid ? in.valid[i] : 1;
  }
}

void gather_columns(const ColView *in, const MutColView *out, int ncols, const int64_t *idx, int64_t m, void *) {
  for (int c = 0; c < ncols; ++c) {
    const int w = in[c].width;
    for (int64_t j = 0; j < m; ++j) {
      const int64_t s = idx[j];
      if (s >= 0)
        move_any(in[c].data, s, out[c].data, j, w);
      else
        std::memset(out[c].data + j * w, 0, w);
      if (out[c].valid) out[c].valid[j] = (s < 0) ? 0 : (in[c].valid ? in[c].valid[s] : 1);
    }
  }
}

// K15 string <-> number casts (twins of strcast.hip; the parsers are shared in strparse.hpp)
void str_to_i64(const ColView &c, int64_t n, int64_t *out, uint8_t *ok, void *) {
  for (int64_t i = 0; i < n; ++i) {
    int64_t v = 0;
    ok[i] = (!c.valid || c.valid[i]) ? strparse::sc_parse_i64(c.data + c.offsets[i], c.offsets[i + 1] - c.offsets[i], &v)
                                     : 1;
    out[i] = v;
  }
}

void str_to_f64(const ColView &c, int64_t n, double *out, uint8_t *ok, void *) {
  for (int64_t i = 0; i < n; ++i) {
    double v = 0.0;
    ok[i] = (!c.valid || c.valid[i]) ? strparse::sc_parse_f64(c.data + c.offsets[i], c.offsets[i + 1] - c.offsets[i], &v)
                                     : 1;
    out[i] = v;
  }
}

void i64_to_str_lengths(const int64_t *v, const uint8_t *valid, int64_t n, int64_t *lens, void *) {
  for (int64_t i = 0; i < n; ++i) lens[i] = (valid && !valid[i]) ? 0 : strparse::sc_i64_len(v[i]);
}

void i64_to_str_write(const int64_t *v, const uint8_t *valid, int64_t n, const int64_t *offs, uint8_t *bytes, void *) {
  for (int64_t i = 0; i < n; ++i)
    if (!valid || valid[i]) strparse::sc_i64_write(v[i], bytes + offs[i + 1]);
}

void select_var_lengths(const ColView &a, const ColView &b, int b_bcast, const uint8_t *cond, int64_t n,
                        int64_t *out_lens, void *) {
  for (int64_t i = 0; i < n; ++i) {
    const bool from_a = cond == nullptr || cond[i] != 0;
    const ColView &s = from_a ? a : b;
    const int64_t j = from_a || !b_bcast ? i : 0;
    out_lens[i] = s.offsets ? s.offsets[j + 1] - s.offsets[j] : 0;
  }
}

void select_var_bytes(const ColView &a, const ColView &b, int b_bcast, const uint8_t *cond, int64_t n,
                      const int64_t *out_off, uint8_t *out_bytes, uint8_t *out_valid, void *) {
  for (int64_t i = 0; i < n; ++i) {
    const bool from_a = cond == nullptr || cond[i] != 0;
    const ColView &s = from_a ? a : b;
    const int64_t j = from_a || !b_bcast ? i : 0;
    uint8_t valid = 0;
    if (s.offsets) {
      const int64_t sb = s.offsets[j], len = s.offsets[j + 1] - sb;
      if (len) std::memcpy(out_bytes + out_off[i], s.data + sb, len);
      valid = s.valid ? s.valid[j] : 1;
    }
    if (out_valid) out_valid[i] = valid;
  }
}

void gather_var_lengths(const ColView &in, const int64_t *idx, int64_t m, int64_t *out_lens, void *) {
  for (int64_t j = 0; j < m; ++j) {
    const int64_t s = idx[j];
    out_lens[j] = s < 0 ? 0 : in.offsets[s + 1] - in.offsets[s];
  }
}

void gather_var_bytes(const ColView &in, const int64_t *idx, int64_t m, const int64_t *out_off, int64_t,
                      uint8_t *out_bytes, uint8_t *out_valid, void *) {
  for (int64_t j = 0; j < m; ++j) {
    const int64_t s = idx[j];
    if (s >= 0) {
      const int64_t sb = in.offsets[s], len = in.offsets[s + 1] - sb;
      if (len) std::memcpy(out_bytes + out_off[j], in.data + sb, len);
    }
    if (out_valid) out_valid[j] = (s < 0) ? 0 : (in.valid ? in.valid[s] : 1);
  }
}

void row_hash64(const ColView *cols, int ncols, int64_t n, uint64_t *out, void *) {
  for (int64_t i = 0; i < n; ++i) {
    uint64_t h = 0x84222325cbf29ce4ULL;
    for (int c = 0; c < ncols; ++c) h = hashing::combine64(h, value_hash64(cols[c], i));
    out[i] = h;
  }
}

void key64_from_column(const ColView &col, int64_t n, int64_t *out, void *) {
  for (int64_t i = 0; i < n; ++i) out[i] = extend_bits(load_bits(col.data, i, col.width), col.width, col.kind);
}

void composite_key_pack(const ColView *cols, int nk, const int64_t *lo, const int *shift, int64_t n, int64_t *out,
                        const int64_t *ncode, void *) {
  for (int64_t i = 0; i < n; ++i) {
    uint64_t acc = 0;
    for (int k = 0; k < nk; ++k) {
      uint64_t f = (uint64_t)(extend_bits(load_bits(cols[k].data, i, cols[k].width), cols[k].width, cols[k].kind) - lo[k]);
      if (ncode && ncode[k] >= 0 && cols[k].valid && !cols[k].valid[i]) f = (uint64_t)ncode[k];
      acc |= f << shift[k];
    }
    out[i] = (int64_t)acc;
  }
}

void composite_key_unpack(const int64_t *key, int64_t n, int nk, const int64_t *lo, const int *shift, const int *bits,
                          const MutColView *out, const int64_t *ncode, void *) {
  for (int k = 0; k < nk; ++k) {
    const uint64_t mask = bits[k] >= 64 ? ~0ull : ((1ull << bits[k]) - 1);
    for (int64_t i = 0; i < n; ++i) {
      const uint64_t f = ((uint64_t)key[i] >> shift[k]) & mask;
      if (ncode && ncode[k] >= 0 && f == (uint64_t)ncode[k] && out[k].valid) out[k].valid[i] = 0;
      const uint64_t x = (uint64_t)lo[k] + f;
      std::memcpy(out[k].data + i * out[k].width, &x, out[k].width);  // little endian: the low bytes
    }
  }
}

void float_key_bits(const ColView &c, int64_t n, int64_t *out, void *) {
  for (int64_t i = 0; i < n; ++i) {
    double v = c.width == 8 ? reinterpret_cast<const double *>(c.data)[i]
                            : (double)reinterpret_cast<const float *>(c.data)[i];
    if (v == 0.0) v = 0.0;
    int64_t b;
    std::memcpy(&b, &v, 8);
    if (v != v) b = 0x7ff8000000000000ll;
    out[i] = b;
  }
}

void hash_table_init(HashSlot *table, int64_t tsize, void *) {
  for (int64_t i = 0; i < tsize; ++i) {
    table[i].key = 0;
    table[i].row = -1;
  }
}

static inline int64_t next_slot(int64_t s, int64_t tsize) { return (s + 1 == tsize) ? 0 : s + 1; }

void hash_build(const int64_t *keys, int64_t n, HashTableRef t, void *) {
  for (int64_t i = 0; i < n; ++i) {
    int64_t slot = (int64_t)hashing::slot_of((uint64_t)keys[i], t.shift);
    while (t.slots[slot].row >= 0) slot = next_slot(slot, t.tsize);
    t.slots[slot].row = i;
    t.slots[slot].key = keys[i];
  }
}

int64_t hash_build_sorted_workspace(int64_t) { return 1; }

int hash_build_sorted(const int64_t *keys, int64_t n, int shift, int64_t *, uint64_t *ka, int64_t *va, uint64_t *kb,
                      int64_t *vb, int64_t *maxpos, void *) {
  std::vector<int64_t> idx(n);
  for (int64_t i = 0; i < n; ++i) idx[i] = i;
  std::stable_sort(idx.begin(), idx.end(), [&](int64_t x, int64_t y) {
    return hashing::slot_of((uint64_t)keys[x], shift) < hashing::slot_of((uint64_t)keys[y], shift);
  });
  int64_t run = INT64_MIN;
  for (int64_t i = 0; i < n; ++i) {
    ka[i] = (uint64_t)keys[idx[i]];
    va[i] = idx[i];
    const int64_t t = (int64_t)hashing::slot_of(ka[i], shift) - i;
    run = t > run ? t : run;
    reinterpret_cast<int64_t *>(kb)[i] = run;
  }
  *maxpos = n ? reinterpret_cast<int64_t *>(kb)[n - 1] : 0;
  (void)vb;
  return 0;
}

void hash_table_place(const uint64_t *skeys, const int64_t *srows, const int64_t *pmax, int64_t n, HashTableRef t,
                      void *) {
  for (int64_t i = 0; i < n; ++i) {
    t.slots[pmax[i] + i].key = (int64_t)skeys[i];
    t.slots[pmax[i] + i].row = srows[i];
  }
}

void hash_probe_count(const int64_t *keys, int64_t n, HashTableRef t, int64_t *counts, void *) {
  for (int64_t i = 0; i < n; ++i) {
    const int64_t k = keys[i];
    int64_t slot = (int64_t)hashing::slot_of((uint64_t)k, t.shift);
    int64_t c = 0;
    while (t.slots[slot].row >= 0) {
      c += t.slots[slot].key == k;
      slot = next_slot(slot, t.tsize);
    }
    counts[i] = c;
  }
}

void hash_probe_write(const int64_t *keys, int64_t n, HashTableRef t, const int64_t *offsets, int64_t *out_p,
                      int64_t *out_b, void *) {
  for (int64_t i = 0; i < n; ++i) {
    int64_t o = offsets[i];
    const int64_t end = offsets[i + 1];
    if (o == end) continue;
    const int64_t k = keys[i];
    int64_t slot = (int64_t)hashing::slot_of((uint64_t)k, t.shift);
    while (o < end && t.slots[slot].row >= 0) {
      if (t.slots[slot].key == k) {
        out_p[o] = i;
        out_b[o] = t.slots[slot].row;
        ++o;
      }
      slot = next_slot(slot, t.tsize);
    }
  }
}

void hash_probe_emit(const int64_t *keys, int64_t n, HashTableRef t, int64_t capacity, int64_t *counter,
                     int64_t *out_p, int64_t *out_b, void *) {
  int64_t o = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t k = keys[i];
    int64_t slot = (int64_t)hashing::slot_of((uint64_t)k, t.shift);
    while (t.slots[slot].row >= 0) {
      if (t.slots[slot].key == k) {
        if (o < capacity) {
          out_p[o] = i;
          out_b[o] = t.slots[slot].row;
        }
        ++o;
      }
      slot = next_slot(slot, t.tsize);
    }
  }
  *counter = o;
}

int64_t max_scan_workspace(int64_t) { return 1; }

void inclusive_max_scan(const int64_t *in, int64_t n, int64_t *out, int64_t *, void *) {
  int64_t run = INT64_MIN;
  for (int64_t i = 0; i < n; ++i) {
    run = in[i] > run ? in[i] : run;
    out[i] = run;
  }
}

void rows_equal(const ColView *l, const ColView *r, int ncols, const int64_t *li, const int64_t *ri, int64_t m,
                uint8_t *eq, void *) {
  for (int64_t j = 0; j < m; ++j) {
    bool e = true;
    for (int c = 0; c < ncols && e; ++c) e = value_equal(l[c], li[j], r[c], ri[j]);
    eq[j] = e ? 1 : 0;
  }
}

void radix_partition_ids(const int64_t *keys, int64_t n, int bits, uint32_t *pid, void *) {
  for (int64_t i = 0; i < n; ++i) pid[i] = hashing::radix_part_of((uint64_t)keys[i], bits);
}

void mark_indices(const int64_t *idx, int64_t m, uint8_t *flags, void *) {
  for (int64_t j = 0; j < m; ++j)
    if (idx[j] >= 0) flags[idx[j]] = 1;
}

int64_t scan_workspace(int64_t) { return 1; }

void exclusive_scan(const int64_t *in, int64_t n, int64_t *out, int64_t *, void *) {
  int64_t run = 0;
  for (int64_t i = 0; i < n; ++i) {
    out[i] = run;
    run += in[i];
  }
  out[n] = run;
}

int64_t mask_to_indices_workspace(int64_t) { return 1; }

void mask_to_indices(const uint8_t *mask, int64_t n, bool invert, int64_t *, int64_t *out, int64_t *count, void *) {
  int64_t k = 0;
  for (int64_t i = 0; i < n; ++i)
    if ((mask[i] != 0) != invert) out[k++] = i;
  *count = k;
}

void iota(int64_t *out, int64_t n, int64_t start, void *) {
  for (int64_t i = 0; i < n; ++i) out[i] = start + i;
}

namespace {
inline uint64_t order_image(uint64_t bits, int w, int kind) {
  const int nb = 8 * w;
  const uint64_t mask = (nb == 64) ? ~0ull : ((1ull << nb) - 1);
  const uint64_t sign = 1ull << (nb - 1);
  bits &= mask;
  if (kind == static_cast<int>(ValueKind::SIGNED_INT)) return bits ^ sign;
  if (kind == static_cast<int>(ValueKind::FLOAT)) {
    if (bits == sign) bits = 0;
    const uint64_t exp_mask = (w == 8) ? 0x7ff0000000000000ull : (w == 4 ? 0x7f800000ull : 0x7c00ull);
    const uint64_t man_mask = (w == 8) ? 0x000fffffffffffffull : (w == 4 ? 0x007fffffull : 0x03ffull);
    if ((bits & exp_mask) == exp_mask && (bits & man_mask) != 0) bits = exp_mask | ((man_mask + 1) >> 1);
    return (bits & sign) ? (~bits & mask) : (bits | sign);
  }
  return bits;
}
}  // namespace

void sort_keys_from_column(const ColView &c, const int64_t *perm, int64_t n, bool desc, uint64_t *out, void *) {
  const int nb = 8 * c.width;
  const uint64_t mask = (nb == 64) ? ~0ull : ((1ull << nb) - 1);
  for (int64_t i = 0; i < n; ++i) {
    const int64_t s = perm ? perm[i] : i;
    const uint64_t bits = load_bits(c.data, s, c.width);
    uint64_t k = order_image(bits, c.width, c.kind);
    k = desc ? (~k & mask) : k;
    if (c.kind == static_cast<int>(ValueKind::FLOAT)) {  // NaN sorts last in both directions
      const bool nan = c.width == 8 ? ((bits & 0x7ff0000000000000ull) == 0x7ff0000000000000ull &&
                                       (bits & 0x000fffffffffffffull))
                       : c.width == 4 ? ((bits & 0x7f800000ull) == 0x7f800000ull && (bits & 0x007fffffull))
                                      : ((bits & 0x7c00ull) == 0x7c00ull && (bits & 0x03ffull));
      if (nan) k = mask;
    }
    if (c.valid != nullptr && c.valid[s] == 0) k = mask;  // nulls: constant image (see sort.hip)
    out[i] = k;
  }
}

int64_t radix_sort_workspace(int64_t n) { return 2 * n + 2; }

// CPU twin: LSD radix with 8-bit digits, identical (stable) result.
int radix_sort_pairs(uint64_t *keys, int64_t *vals, int64_t n, uint64_t *keys_alt, int64_t *vals_alt, int begin_bit,
                     int end_bit, int64_t *, void *) {
  if (n <= 1) return 0;
  uint64_t o = 0, a = ~0ull;
  for (int64_t i = 0; i < n; ++i) {
    o |= keys[i];
    a &= keys[i];
  }
  const uint64_t diff = o ^ a;
  int cur = 0;
  uint64_t *kb[2] = {keys, keys_alt};
  int64_t *vb[2] = {vals, vals_alt};
  std::vector<int64_t> cnt(257);
  for (int shift = begin_bit; shift < end_bit; shift += 8) {
    if (((diff >> shift) & 0xffull) == 0) continue;
    std::fill(cnt.begin(), cnt.end(), 0);
    const uint64_t *ki = kb[cur];
    const int64_t *vi = vb[cur];
    uint64_t *ko = kb[cur ^ 1];
    int64_t *vo = vb[cur ^ 1];
    for (int64_t i = 0; i < n; ++i) cnt[((ki[i] >> shift) & 0xff) + 1]++;
    for (int d = 0; d < 256; ++d) cnt[d + 1] += cnt[d];
    for (int64_t i = 0; i < n; ++i) {
      const int64_t d = cnt[(ki[i] >> shift) & 0xff]++;
      ko[d] = ki[i];
      vo[d] = vi[i];
    }
    cur ^= 1;
  }
  return cur;
}

void merge_join_count(const uint64_t *lk, int64_t nl, const uint64_t *rk, int64_t nr, int64_t *lo, int64_t *counts,
                      void *) {
  for (int64_t i = 0; i < nl; ++i) {
    const uint64_t *b = std::lower_bound(rk, rk + nr, lk[i]);
    const uint64_t *e = std::upper_bound(b, rk + nr, lk[i]);
    lo[i] = b - rk;
    counts[i] = e - b;
  }
}

void merge_join_write(const int64_t *lperm, int64_t nl, const int64_t *rperm, const int64_t *lo, const int64_t *offs,
                      int64_t *out_l, int64_t *out_r, void *) {
  for (int64_t i = 0; i < nl; ++i) {
    const int64_t o = offs[i], c = offs[i + 1] - o;
    for (int64_t k = 0; k < c; ++k) {
      out_l[o + k] = lperm[i];
      out_r[o + k] = rperm[lo[i] + k];
    }
  }
}

}  // namespace cpu
}  // namespace cylon

namespace cylon {
namespace cpu {

void sort_string_chunk_keys(const ColView &c, const int64_t *perm, int64_t n, int64_t chunk, bool desc, uint64_t *out,
                            void *) {
  for (int64_t i = 0; i < n; ++i) {
    const int64_t s = perm ? perm[i] : i;
    const int64_t b = c.offsets[s], len = c.offsets[s + 1] - b;
    uint64_t k = 0;
    if (chunk < 0) {
      k = (uint64_t)len;
    } else {
      for (int j = 0; j < 8; ++j) {
        const int64_t p = chunk * 8 + j;
        k = (k << 8) | (p < len ? (uint64_t)c.data[b + p] : 0ull);
      }
    }
    out[i] = (c.valid != nullptr && c.valid[s] == 0) ? ~0ull : (desc ? ~k : k);  // nulls: constant image
  }
}

void narrow_i64(const int64_t *in, int64_t n, int64_t base, uint32_t *out, void *) {
  for (int64_t i = 0; i < n; ++i) out[i] = (uint32_t)((uint64_t)in[i] - (uint64_t)base);
}

void widen_u32(const uint32_t *in, int64_t n, int64_t base, int64_t *out, void *) {
  for (int64_t i = 0; i < n; ++i) out[i] = (int64_t)((uint64_t)base + in[i]);
}

}  // namespace cpu
}  // namespace cylon

namespace cylon {
namespace cpu {

void batched_copy(const void *const *src, void *const *dst, const int64_t *bytes, int n, void *) {
  for (int i = 0; i < n; ++i)
    if (bytes[i] > 0) std::memcpy(dst[i], src[i], (size_t)bytes[i]);
}

}  // namespace cpu
}  // namespace cylon
