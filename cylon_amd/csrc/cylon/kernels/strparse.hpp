// String <-> number conversion of one value, shared by the HIP kernels (strcast.hip) and their
// CPU twins (cpu_kernels.cpp); see strcast.hip for the accepted syntax and the exact fast path.
#pragma once
#include <cstdint>

#include "../common.hpp"

namespace cylon {
namespace strparse {

CYLON_HD uint8_t sc_parse_i64(const uint8_t *s, int64_t len, int64_t *out) {
  if (len <= 0) return 0;
  int64_t i = 0;
  bool neg = false;
  if (s[0] == '-') {  // Arrow's integer parser: '-' only, no '+'
    neg = true;
    i = 1;
    if (len == 1) return 0;
  }
  if (len - i > 1 && s[i] == '0' && (s[i + 1] | 0x20) == 'x') return 2;  // hex: Arrow's host parser
  uint64_t v = 0;
  const uint64_t lim = neg ? (uint64_t)1 << 63 : ((uint64_t)1 << 63) - 1;
  for (; i < len; ++i) {
    const uint32_t d = (uint32_t)s[i] - '0';
    if (d > 9) return 0;
    if (v > (lim - d) / 10) return 0;  // overflow
    v = v * 10 + d;
  }
  *out = neg ? (int64_t)(0 - v) : (int64_t)v;
  return 1;
}

CYLON_HD uint8_t sc_parse_f64(const uint8_t *s, int64_t len, double *out) {
  if (len <= 0) return 0;
  int64_t i = 0;
  bool neg = false;
  if (s[0] == '+' || s[0] == '-') {
    neg = s[0] == '-';
    i = 1;
  }
  uint64_t m = 0;
  int sig = 0, exp10 = 0, digits = 0;
  bool dot = false;
  for (; i < len; ++i) {
    const uint8_t c = s[i];
    if (c == '.') {
      if (dot) return 0;
      dot = true;
      continue;
    }
    const uint32_t d = (uint32_t)c - '0';
    if (d > 9) break;
    ++digits;
    if (sig == 0 && d == 0) {  // leading zeros
      if (dot) --exp10;
      continue;
    }
    if (sig < 19) {
      m = m * 10 + d;
      ++sig;
      if (dot) --exp10;
    } else {
      if (!dot) ++exp10;  // dropped digit: the hard path keeps the value exact
      sig = 99;
    }
  }
  if (digits == 0) {
    // inf / infinity / nan spellings parse on the host
    const uint8_t c = i < len ? (uint8_t)(s[i] | 0x20) : 0;
    return (c == 'i' || c == 'n') ? 2 : 0;
  }
  if (i < len) {
    if ((s[i] | 0x20) != 'e') return 0;
    ++i;
    bool eneg = false;
    if (i < len && (s[i] == '+' || s[i] == '-')) {
      eneg = s[i] == '-';
      ++i;
    }
    if (i >= len) return 0;
    int e = 0;
    for (; i < len; ++i) {
      const uint32_t d = (uint32_t)s[i] - '0';
      if (d > 9) return 0;
      if (e < 100000) e = e * 10 + (int)d;
    }
    exp10 += eneg ? -e : e;
  }
  if (sig > 19 || m > ((uint64_t)1 << 53) || exp10 > 22 || exp10 < -22) return 2;
  const double p10[23] = {1e0,  1e1,  1e2,  1e3,  1e4,  1e5,  1e6,  1e7,  1e8,  1e9,  1e10, 1e11,
                          1e12, 1e13, 1e14, 1e15, 1e16, 1e17, 1e18, 1e19, 1e20, 1e21, 1e22};
  double v = (double)m;
  v = exp10 >= 0 ? v * p10[exp10] : v / p10[-exp10];
  *out = neg ? -v : v;
  return 1;
}

CYLON_HD int sc_i64_len(int64_t x) {
  uint64_t u = x < 0 ? 0 - (uint64_t)x : (uint64_t)x;
  int d = 1;
  while (u >= 10) {
    u /= 10;
    ++d;
  }
  return d + (x < 0 ? 1 : 0);
}

// writes the decimal digits of x so that they END at e (bytes [e - sc_i64_len(x), e))
CYLON_HD void sc_i64_write(int64_t x, uint8_t *e) {
  uint64_t u = x < 0 ? 0 - (uint64_t)x : (uint64_t)x;
  do {
    *--e = (uint8_t)('0' + u % 10);
    u /= 10;
  } while (u);
  if (x < 0) *--e = '-';
}

}  // namespace strparse
}  // namespace cylon
