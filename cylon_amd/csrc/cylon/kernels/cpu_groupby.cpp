// CPU twins of the group-by / distinct / reduction primitives (groupby.hip).
#include <cmath>
#include <cstring>
#include <limits>

#include "kernels.hpp"
#include "../hash.hpp"
#include "../types.hpp"

namespace cylon {
namespace cpu {

namespace {
constexpr int64_t kSentinel = std::numeric_limits<int64_t>::min();

inline uint64_t load_bits(const uint8_t *base, int64_t i, int w) {
  uint64_t v = 0;
  std::memcpy(&v, base + i * w, w);
  return v;
}

inline int64_t extend(uint64_t b, int w, int kind) {
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

inline uint64_t img(uint64_t bits, int w, int kind) {
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

inline float half_to_float(uint16_t h) {
  const uint32_t s = (h >> 15) & 1, e = (h >> 10) & 0x1f, m = h & 0x3ff;
  float f;
  if (e == 0) f = std::ldexp((float)m, -24);
  else if (e == 31) f = m ? std::numeric_limits<float>::quiet_NaN() : std::numeric_limits<float>::infinity();
  else f = std::ldexp((float)(m | 0x400), (int)e - 25);
  return s ? -f : f;
}

inline double as_double(const ColView &c, int64_t i) {
  const uint64_t b = load_bits(c.data, i, c.width);
  if (c.kind == static_cast<int>(ValueKind::FLOAT)) {
    if (c.width == 8) {
      double d;
      std::memcpy(&d, &b, 8);
      return d;
    }
    if (c.width == 4) {
      float f;
      uint32_t u = (uint32_t)b;
      std::memcpy(&f, &u, 4);
      return f;
    }
    return half_to_float((uint16_t)b);
  }
  if (c.kind == static_cast<int>(ValueKind::SIGNED_INT)) return (double)extend(b, c.width, c.kind);
  return (double)b;
}

inline bool val_eq(const ColView &a, int64_t i, int64_t j) {
  const bool va = a.valid == nullptr || a.valid[i] != 0;
  const bool vb = a.valid == nullptr || a.valid[j] != 0;
  if (!va || !vb) return va == vb;
  if (a.kind == static_cast<int>(ValueKind::VAR_BYTES)) {
    const int64_t ab = a.offsets[i], al = a.offsets[i + 1] - ab;
    const int64_t bb = a.offsets[j], bl = a.offsets[j + 1] - bb;
    return al == bl && (al == 0 || std::memcmp(a.data + ab, a.data + bb, al) == 0);
  }
  if (a.kind == static_cast<int>(ValueKind::FIXED_BYTES))
    return std::memcmp(a.data + i * a.width, a.data + j * a.width, a.width) == 0;
  const int64_t x = extend(load_bits(a.data, i, a.width), a.width, a.kind);
  const int64_t y = extend(load_bits(a.data, j, a.width), a.width, a.kind);
  if (x == y) return true;
  if (a.kind == static_cast<int>(ValueKind::FLOAT)) {
    const double dx = as_double(a, i), dy = as_double(a, j);
    return std::isnan(dx) && std::isnan(dy);
  }
  return false;
}
}  // namespace

void group_insert(const int64_t *keys, int64_t n, int64_t *slot_keys, int64_t cap, int64_t *slot_of_row,
                  int64_t *slot_first, void *) {
  const uint64_t mask = (uint64_t)cap - 1;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t k = keys[i];
    int64_t slot;
    if (k == kSentinel) {
      slot = cap;
    } else {
      uint64_t h = hashing::fmix64((uint64_t)k) & mask;
      while (slot_keys[h] != k && slot_keys[h] != kSentinel) h = (h + 1) & mask;
      slot_keys[h] = k;
      slot = (int64_t)h;
    }
    slot_of_row[i] = slot;
    if (i < slot_first[slot]) slot_first[slot] = i;
  }
}

void mark_firsts(const int64_t *v, int64_t m, uint8_t *flags, void *) {
  for (int64_t j = 0; j < m; ++j)
    if (v[j] >= 0 && v[j] != std::numeric_limits<int64_t>::max()) flags[v[j]] = 1;
}

void scatter_iota(const int64_t *idx, int64_t m, int64_t *out, void *) {
  for (int64_t g = 0; g < m; ++g) out[idx[g]] = g;
}

void permute_assign(const int64_t *dst, const int64_t *src, const int64_t *table, int64_t n, int64_t *out, void *) {
  for (int64_t i = 0; i < n; ++i) out[dst[i]] = table[src ? src[i] : i];
}

void gather_chain2(const int64_t *a, const int64_t *b, const int64_t *c, int64_t n, int64_t *out, void *) {
  for (int64_t i = 0; i < n; ++i) out[i] = c[b[a[i]]];
}

void segment_heads(const ColView *cols, int ncols, const int64_t *perm, int64_t n, uint8_t *heads, void *) {
  for (int64_t i = 0; i < n; ++i) {
    bool h = (i == 0);
    for (int c = 0; c < ncols && !h; ++c) h = !val_eq(cols[c], perm[i], perm[i - 1]);
    heads[i] = h;
  }
}

void agg_accumulate(const int64_t *gid, int64_t n, int64_t, const ColView &v, int kind, void *acc,
                    const double *mean, void *) {
  double *fa = reinterpret_cast<double *>(acc);
  uint64_t *ua = reinterpret_cast<uint64_t *>(acc);
  for (int64_t i = 0; i < n; ++i) {
    if (v.valid && !v.valid[i]) continue;
    const int64_t g = gid ? gid[i] : 0;
    switch (kind) {
      case 0: fa[g] += as_double(v, i); break;
      case 1: ua[g] += (uint64_t)extend(load_bits(v.data, i, v.width), v.width, v.kind); break;
      case 2: {
        const uint64_t x = img(load_bits(v.data, i, v.width), v.width, v.kind);
        if (x < ua[g]) ua[g] = x;
        break;
      }
      case 3: {
        const uint64_t x = img(load_bits(v.data, i, v.width), v.width, v.kind);
        if (x > ua[g]) ua[g] = x;
        break;
      }
      case 4: ua[g] += 1; break;
      case 5: {
        const double d = as_double(v, i) - mean[g];
        fa[g] += d * d;
        break;
      }
    }
  }
}

void agg_unimage(const uint64_t *in, int64_t m, int w, int kind, uint8_t *out, void *) {
  const int nb = 8 * w;
  const uint64_t mask = (nb == 64) ? ~0ull : ((1ull << nb) - 1);
  const uint64_t sign = 1ull << (nb - 1);
  for (int64_t g = 0; g < m; ++g) {
    uint64_t b = in[g] & mask;
    if (kind == static_cast<int>(ValueKind::SIGNED_INT)) b ^= sign;
    else if (kind == static_cast<int>(ValueKind::FLOAT)) b = (b & sign) ? (b ^ sign) : (~b & mask);
    std::memcpy(out + g * w, &b, w);
  }
}

void group_quantile(const ColView &v, const int64_t *perm, const int64_t *offs, int64_t ngroups, double q, double *out,
                    uint8_t *valid, void *) {
  for (int64_t g = 0; g < ngroups; ++g) {
    const int64_t b = offs[g], cnt = offs[g + 1] - b;
    if (cnt == 0) {
      out[g] = 0;
      valid[g] = 0;
      continue;
    }
    const double np = (double)cnt * q, j = std::floor(np), gg = np - j;
    int64_t pos = (int64_t)j;
    if (pos >= cnt) pos = cnt - 1;
    out[g] = (gg == 0.0 && pos > 0) ? 0.5 * (as_double(v, perm[b + pos - 1]) + as_double(v, perm[b + pos]))
                                    : as_double(v, perm[b + pos]);
    valid[g] = 1;
  }
}

}  // namespace cpu
}  // namespace cylon
