// Hash functions shared by the HIP kernels and the CPU twins.
//
// Partitioning must be bit-identical to the reference so that per-rank golden
// files (data/output/*_{world}_{rank}.csv) stay valid:
//   * integer / bool / temporal keys: f(v) = (uint32)v       (ModuloPartitionKernel,
//     reference cpp/src/cylon/arrow/arrow_partition_kernels.cpp:67-115)
//   * float / double / binary / string: f(v) = MurmurHash3_x86_32(bytes, seed 0)
//     (arrow_partition_kernels.cpp:119-305, util/murmur3.cpp)
//   * multi-column chain: h = 31*h + f(v) ; p = h & (P-1) if P is a power of two
//     else h % P (arrow_partition_kernels.cpp:51-61, partition.cpp:118-166).
// Local hash tables use a separate 64-bit mixer (fmix64) so that hash-table slot
// selection is independent of the partition function.
#pragma once
#include "common.hpp"

namespace cylon {
namespace hashing {

CYLON_HD uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }

CYLON_HD uint32_t fmix32(uint32_t h) {
  h ^= h >> 16;
  h *= 0x85ebca6bu;
  h ^= h >> 13;
  h *= 0xc2b2ae35u;
  h ^= h >> 16;
  return h;
}

CYLON_HD uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdULL;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ULL;
  k ^= k >> 33;
  return k;
}

// inverse of fmix64: x ^= x >> 33 undoes itself (shift >= 32), the multipliers are odd (inverses mod 2^64)
CYLON_HD uint64_t fmix64_inv(uint64_t k) {
  k ^= k >> 33;
  k *= 0x9cb4b2f8129337dbULL;
  k ^= k >> 33;
  k *= 0x4f74430c22a54005ULL;
  k ^= k >> 33;
  return k;
}

// Invertible key of a fixed-length string of L bytes held as W = ceil(L / 8) little-endian words:
// h = fmix64(w0 ^ g), g a chain over L and words 1..W-1.  For fixed g, w0 -> h is a bijection, so
// (h, w1..w_{W-1}) determines the string: the join carries h as its key in place of w0
// (w0 = fmix64_inv(h) ^ g), and equal h + equal w1.. means equal strings.
CYLON_HD uint64_t word_key_seed(int64_t len) { return 0x9E3779B97F4A7C15ULL ^ (uint64_t)len; }
CYLON_HD uint64_t word_key_step(uint64_t g, uint64_t w) { return fmix64(g ^ w) + 0x632BE59BD9B4E019ULL; }

// 64-bit hash of a byte string (join / set-op keys of string, binary and fixed-size binary columns):
// a chain of fmix64 bijections over the little-endian 8-byte words, seeded with the length.  Two
// 32-bit murmur3 hashes with different seeds (round 4) are correlated on short keys: a 200M x 200M
// join on 16-byte keys saw 3 false matches, ~2^11 more than 64 independent bits give.
CYLON_HD uint64_t bytes_hash64(const uint8_t *p, int64_t len) {
  uint64_t h = 0x9E3779B97F4A7C15ULL ^ (uint64_t)len;
  int64_t i = 0;
  for (; i + 8 <= len; i += 8) {
    uint64_t w = 0;
    for (int b = 0; b < 8; ++b) w |= (uint64_t)p[i + b] << (8 * b);
    h = fmix64(h ^ w) + 0x632BE59BD9B4E019ULL;
  }
  uint64_t w = 0;
  for (int b = 0; i + b < len; ++b) w |= (uint64_t)p[i + b] << (8 * b);
  return fmix64(h ^ w ^ ((uint64_t)len << 56));
}

CYLON_HD uint32_t murmur_mix_k1(uint32_t k1) {
  k1 *= 0xcc9e2d51u;
  k1 = rotl32(k1, 15);
  k1 *= 0x1b873593u;
  return k1;
}

CYLON_HD uint32_t murmur_step(uint32_t h1, uint32_t k1) {
  h1 ^= murmur_mix_k1(k1);
  h1 = rotl32(h1, 13);
  return h1 * 5u + 0xe6546b64u;
}

// MurmurHash3_x86_32 over an arbitrary byte range (seed 0 in all callers).
CYLON_HD uint32_t murmur3_32(const uint8_t *data, int64_t len, uint32_t seed) {
  const int64_t nblocks = len / 4;
  uint32_t h1 = seed;
  for (int64_t i = 0; i < nblocks; ++i) {
    const uint8_t *p = data + i * 4;
    uint32_t k1 = (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) |
                  ((uint32_t)p[3] << 24);
    h1 = murmur_step(h1, k1);
  }
  const uint8_t *tail = data + nblocks * 4;
  uint32_t k1 = 0;
  switch (len & 3) {
    case 3: k1 ^= (uint32_t)tail[2] << 16;  // fallthrough
    case 2: k1 ^= (uint32_t)tail[1] << 8;   // fallthrough
    case 1:
      k1 ^= tail[0];
      h1 ^= murmur_mix_k1(k1);
  }
  h1 ^= (uint32_t)len;
  return fmix32(h1);
}

// Specialisations for 4- and 8-byte values held in registers (same result as
// murmur3_32 over their little-endian bytes).
CYLON_HD uint32_t murmur3_32_u32(uint32_t v) {
  uint32_t h1 = murmur_step(0u, v);
  h1 ^= 4u;
  return fmix32(h1);
}

CYLON_HD uint32_t murmur3_32_u64(uint64_t v) {
  uint32_t h1 = murmur_step(0u, (uint32_t)v);
  h1 = murmur_step(h1, (uint32_t)(v >> 32));
  h1 ^= 8u;
  return fmix32(h1);
}

CYLON_HD uint32_t murmur3_32_u16(uint16_t v) {
  uint32_t h1 = 0u;
  uint32_t k1 = (uint32_t)(v & 0xff) | ((uint32_t)(v >> 8) << 8);
  h1 ^= murmur_mix_k1(k1);
  h1 ^= 2u;
  return fmix32(h1);
}

// Slot of a 64-bit key in a power-of-two table of 2^(64-shift) slots: the TOP
// bits of the mixed key.  The join radix-partitions its inputs by the top
// bits of the same hash, so partition-major probe/build order walks the table
// front to back and the active window of the table stays cache resident.
CYLON_HD uint64_t slot_of(uint64_t k, int shift) { return fmix64(k) >> shift; }

// radix partition id of a key for 2^bits partitions (consistent with slot_of)
CYLON_HD uint32_t radix_part_of(uint64_t k, int bits) { return (uint32_t)(fmix64(k) >> (64 - bits)); }

CYLON_HD uint32_t partitioner(uint32_t h, uint32_t nparts) {
  return (nparts & (nparts - 1)) == 0 ? (h & (nparts - 1)) : (h % nparts);
}

// 64-bit row-hash combine used for multi-column / variable-width keys in the
// local relational kernels (join, group-by, set ops).  Not used for
// partitioning.
CYLON_HD uint64_t combine64(uint64_t h, uint64_t v) {
  return fmix64(h * 0x9E3779B97F4A7C15ULL + v + 0x632BE59BD9B4E019ULL);
}

}  // namespace hashing
}  // namespace cylon
