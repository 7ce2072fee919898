// CPU twins of the validity bitmap kernels (bitmap.hip).
#include "kernels.hpp"

namespace cylon {
namespace cpu {

void pack_validity(const uint8_t *bytes, int64_t n, uint64_t *bitmap, int64_t *nulls, void *) {
  int64_t z = 0;
  for (int64_t w = 0; w < (n + 63) / 64; ++w) {
    uint64_t word = 0;
    for (int64_t b = 0; b < 64 && w * 64 + b < n; ++b) {
      if (bytes[w * 64 + b]) word |= 1ull << b;
      else ++z;
    }
    bitmap[w] = word;
  }
  *nulls += z;
}

void unpack_validity(const uint8_t *bits, int64_t bit_offset, int64_t n, uint8_t *bytes, void *) {
  for (int64_t i = 0; i < n; ++i) {
    const int64_t b = bit_offset + i;
    bytes[i] = (bits[b >> 3] >> (b & 7)) & 1;
  }
}

void pack_byte_columns(const uint8_t *const *cols, int k, int64_t n, uint64_t *const *words, void *) {
  for (int64_t i = 0; i < n; ++i)
    for (int w = 0; w < (k + 7) / 8; ++w) {
      uint64_t word = 0;
      for (int j = 0; j < 8 && 8 * w + j < k; ++j) word |= (uint64_t)cols[8 * w + j][i] << (8 * j);
      words[w][i] = word;
    }
}

void unpack_byte_columns(const uint64_t *const *words, int k, int64_t n, uint8_t *const *cols, void *) {
  for (int64_t i = 0; i < n; ++i)
    for (int w = 0; w < (k + 7) / 8; ++w)
      for (int j = 0; j < 8 && 8 * w + j < k; ++j) cols[8 * w + j][i] = (uint8_t)(words[w][i] >> (8 * j));
}

}  // namespace cpu
}  // namespace cylon
