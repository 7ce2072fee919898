// CPU twins of the K16 persistent index kernels (index.hip).
#include <algorithm>

#include "../hash.hpp"
#include "kernels.hpp"

namespace cylon {
namespace cpu {

void index_bounds(const uint64_t *sorted, int64_t n, const uint64_t *probe, int64_t m, int64_t *lo, int64_t *cnt,
                  void *) {
  for (int64_t i = 0; i < m; ++i) {
    auto r = std::equal_range(sorted, sorted + n, probe[i]);
    lo[i] = r.first - sorted;
    cnt[i] = r.second - r.first;
  }
}

void hash_index_build(const uint64_t *sorted, int64_t n, uint64_t *tkeys, int32_t *used, int64_t *tlo, int64_t *tcnt,
                      int64_t cap, void *) {
  for (int64_t i = 0; i < n; ++i) {
    if (i > 0 && sorted[i - 1] == sorted[i]) continue;
    const int64_t len = std::upper_bound(sorted + i, sorted + n, sorted[i]) - (sorted + i);
    uint64_t s = hashing::fmix64(sorted[i]) & (uint64_t)(cap - 1);
    while (used[s]) s = (s + 1) & (uint64_t)(cap - 1);
    used[s] = 1;
    tkeys[s] = sorted[i];
    tlo[s] = i;
    tcnt[s] = len;
  }
}

void hash_index_probe(const uint64_t *tkeys, const int32_t *used, const int64_t *tlo, const int64_t *tcnt, int64_t cap,
                      const uint64_t *probe, int64_t m, int64_t *lo, int64_t *cnt, void *) {
  for (int64_t i = 0; i < m; ++i) {
    uint64_t s = hashing::fmix64(probe[i]) & (uint64_t)(cap - 1);
    lo[i] = 0;
    cnt[i] = 0;
    for (int64_t p = 0; p < cap && used[s]; ++p) {
      if (tkeys[s] == probe[i]) {
        lo[i] = tlo[s];
        cnt[i] = tcnt[s];
        break;
      }
      s = (s + 1) & (uint64_t)(cap - 1);
    }
  }
}

void index_gather_positions(const int64_t *sorted_pos, const int64_t *lo, const int64_t *cnt, const int64_t *offs,
                            int64_t m, int64_t *out, void *) {
  for (int64_t i = 0; i < m; ++i)
    for (int64_t j = 0; j < cnt[i]; ++j) out[offs[i] + j] = sorted_pos[lo[i] + j];
}

static void bytes_of(const ColView &c, int64_t r, const uint8_t *&p, int64_t &len) {
  if (c.offsets) {
    p = c.data + c.offsets[r];
    len = c.offsets[r + 1] - c.offsets[r];
  } else {
    p = c.data + r * (int64_t)c.width;
    len = c.width;
  }
}

void index_verify_bytes(const ColView &col, const ColView &labels, const int64_t *sorted_pos, const int64_t *lo,
                        const int64_t *cnt, const int64_t *offs, int64_t m, uint8_t *keep, void *) {
  for (int64_t i = 0; i < m; ++i) {
    const uint8_t *lp;
    int64_t ll;
    bytes_of(labels, i, lp, ll);
    for (int64_t j = 0; j < cnt[i]; ++j) {
      const uint8_t *cp;
      int64_t cl;
      bytes_of(col, sorted_pos[lo[i] + j], cp, cl);
      keep[offs[i] + j] = cl == ll && (ll == 0 || std::equal(cp, cp + ll, lp)) ? 1 : 0;
    }
  }
}

}  // namespace cpu
}  // namespace cylon
