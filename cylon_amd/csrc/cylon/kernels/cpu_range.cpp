// CPU twins of the K13 range-partition primitives (range.hip).
#include <cmath>
#include <cstring>
#include <limits>
#include <vector>

#include "kernels.hpp"
#include "../types.hpp"

namespace cylon {
namespace cpu {

namespace {
inline double value_as_double(const ColView &c, int64_t i) {
  uint64_t b = 0;
  std::memcpy(&b, c.data + i * c.width, c.width);
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
    const uint32_t s = (b >> 15) & 1, e = (b >> 10) & 0x1f, m = b & 0x3ff;
    double f = e == 0 ? std::ldexp((double)m, -24)
                      : (e == 31 ? (m ? NAN : INFINITY) : std::ldexp((double)(m | 0x400), (int)e - 25));
    return s ? -f : f;
  }
  if (c.kind == static_cast<int>(ValueKind::SIGNED_INT)) {
    switch (c.width) {
      case 1: return (double)(int8_t)b;
      case 2: return (double)(int16_t)b;
      case 4: return (double)(int32_t)b;
      default: return (double)(int64_t)b;
    }
  }
  return (double)b;
}

inline int64_t bin_pos(double v, double vmin, double vmax, int64_t nbins) {
  if (!(v >= vmin)) return 0;
  if (v >= vmax) return nbins + 1;
  int64_t b = 1 + (int64_t)std::floor((v - vmin) * (double)nbins / (vmax - vmin));
  return b > nbins ? nbins : b;
}
}  // namespace

void range_minmax(const ColView &c, const int64_t *idx, int64_t m, double *out, void *) {
  double lo = INFINITY, hi = -INFINITY;
  for (int64_t j = 0; j < m; ++j) {
    const int64_t i = idx ? idx[j] : j;
    if (c.valid && !c.valid[i]) continue;
    const double v = value_as_double(c, i);
    lo = std::fmin(lo, v);
    hi = std::fmax(hi, v);
  }
  out[0] = lo;
  out[1] = hi;
}

void range_histogram(const ColView &c, const int64_t *idx, int64_t m, double vmin, double vmax, int64_t nbins,
                     int64_t *hist, void *) {
  for (int64_t j = 0; j < m; ++j) hist[bin_pos(value_as_double(c, idx ? idx[j] : j), vmin, vmax, nbins)]++;
}

void range_partition(const ColView &c, int64_t n, double vmin, double vmax, int64_t nbins, const uint32_t *b2p,
                     uint32_t nparts, bool desc, uint32_t *pid, int64_t *counts, void *) {
  for (int64_t i = 0; i < n; ++i) {
    uint32_t p = b2p[bin_pos(value_as_double(c, i), vmin, vmax, nbins)];
    if (desc) p = nparts - 1 - p;
    pid[i] = p;
    counts[p]++;
  }
}

}  // namespace cpu
}  // namespace cylon

namespace cylon {
namespace cpu {

void splitter_partition(const uint64_t *const *images, const uint8_t *const *nulls, int nkeys, int64_t n,
                        int64_t gid0, const uint64_t *splitters, uint32_t nparts, uint32_t *pid, int64_t *counts,
                        void *) {
  const int stride = 2 * nkeys + 1;
  std::vector<uint64_t> k(stride);
  for (int64_t i = 0; i < n; ++i) {
    for (int c = 0; c < nkeys; ++c) {
      k[2 * c] = nulls[c] ? (uint64_t)(nulls[c][i] != 0) : 0ull;
      k[2 * c + 1] = images[c][i];
    }
    k[2 * nkeys] = (uint64_t)(gid0 + i);
    uint32_t lo = 0, hi = nparts - 1;
    while (lo < hi) {
      const uint32_t mid = (lo + hi) >> 1;
      const uint64_t *s = splitters + (int64_t)mid * stride;
      int cmp = 0;
      for (int w = 0; w < stride && cmp == 0; ++w) cmp = s[w] < k[w] ? -1 : (s[w] > k[w] ? 1 : 0);
      if (cmp < 0) lo = mid + 1; else hi = mid;
    }
    pid[i] = lo;
    ++counts[lo];
  }
}

}  // namespace cpu
}  // namespace cylon

namespace cylon {
namespace cpu {

// CPU twin of merge.hip k_merge_pairs: stable merge, A first on ties
void merge_sorted_pairs(const uint64_t *ak, const int64_t *ai, int64_t na, const uint64_t *bk, const int64_t *bi,
                        int64_t nb, uint64_t *ok, int64_t *oi, void *) {
  int64_t x = 0, y = 0, o = 0;
  while (x < na || y < nb) {
    const bool takea = x < na && (y >= nb || ak[x] <= bk[y]);
    ok[o] = takea ? ak[x] : bk[y];
    oi[o++] = takea ? ai[x++] : bi[y++];
  }
}

}  // namespace cpu
}  // namespace cylon
