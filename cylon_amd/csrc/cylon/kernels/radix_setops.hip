// LDS radix distinct for set operations and unique (K10, gfx950).
//
// Reference behaviour: cpp/src/cylon/table.cpp:531-721 (Union / Subtract /
// Intersect insert row indices into a row-hash set with full-row equality;
// output = first occurrences in input order, left rows before right rows) and
// :923-999 (Unique keep first / last over a column subset).
//
// MI355X design (no sort, no global hash table):
//   1. k_so_hash_tiles: one pass over L ++ R writes a 64-bit row hash (NaN / -0.0 /
//      null canonicalised so that equal rows hash equal) and the global row id
//      (left rows 0..nl-1, right rows nl..n-1).
//   2. the (hash, row id) pairs are radix-partitioned by the top bits of
//      fmix64(hash) with the LDS-staged passes of radix_join.hip (16 bytes per
//      row move, not the table), so a partition's distinct hashes fit one LDS
//      table.  The passes are stable: inside a partition row ids ascend.
//   3. k_so_dedup, one partition per workgroup: phase 1 inserts every hash into
//      an LDS open-addressing table (64-bit LDS CAS) and folds the partition-local
//      position into the slot's representative (LDS atomicMin = first
//      occurrence, atomicMax = last) and the side flags (left / right row seen);
//      phase 2 revisits the rows: a row that is not its slot's representative is
//      compared column by column with the representative (random reads, one per
//      duplicate row); an unequal pair is a 64-bit hash collision and flags the
//      whole call for the exact fallback.  Each row's keep decision is written
//      to a byte mask indexed by row id only where it differs from the mask's
//      initial value (union: drop duplicates; subtract: drop left rows that
//      repeat or occur on the right; intersect: keep first left rows that occur
//      on the right), so mostly-distinct unions cost no scattered writes.
//      The count of such exceptions lets the host skip the compaction.
//   4. the host compacts the mask (ascending row ids = the reference's output
//      order) and gathers the surviving rows.
#include "device_common.hpp"

namespace cylon {
namespace hip {

constexpr int kSOThreads = 512;
// LDS table: 8 B hash + 4 B representative + 2 side bits per slot, 4096 slots ->
// 49 KB, several workgroups per CU.  Partitions of <= 2048 rows (load <= 0.5): 2^31
// rows take 20 partition bits (two 10-bit passes).  Measured alternative: 8192-row
// partitions in a 12288-slot table (one workgroup per CU) let 2^31 rows use two
// 9-bit passes (-8 ms per 1B x 1B union) but the dedup lost more (+10 ms).
constexpr int kSOSlots = 4096;
constexpr int64_t kSORowsPerPart = 2048;

struct SOColSet {
  ColView c[kMaxFusedCols];
};

// value hash with the equality semantics of value_equal (hash_join.hip): null ==
// null, NaN == NaN (any payload), -0.0 == 0.0
__device__ __forceinline__ uint64_t so_value_hash(const ColView &c, int64_t i) {
  if (c.valid != nullptr && c.valid[i] == 0) return 0x5bd1e9955bd1e995ULL;
  if (c.kind == static_cast<int>(ValueKind::VAR_BYTES)) {
    const int64_t b = c.offsets[i], e = c.offsets[i + 1];
    return hashing::bytes_hash64(c.data + b, e - b);
  }
  if (c.kind == static_cast<int>(ValueKind::FIXED_BYTES)) {
    return hashing::bytes_hash64(c.data + i * (int64_t)c.width, c.width);
  }
  uint64_t bits = (uint64_t)extend_bits(load_bits(c.data, i, c.width), c.width, c.kind);
  if (c.kind == static_cast<int>(ValueKind::FLOAT)) {
    bool nan = false;
    if (c.width == 8) nan = __longlong_as_double((long long)bits) != __longlong_as_double((long long)bits);
    else if (c.width == 4) nan = __int_as_float((int)bits) != __int_as_float((int)bits);
    else if (c.width == 2) nan = ((bits & 0x7c00u) == 0x7c00u) && (bits & 0x3ffu);
    if (nan) bits = 0x7ff8000000000000ull;
  }
  return hashing::fmix64(bits);
}

// Row hash of the concatenated L ++ R rows with the first partition pass's tile histogram (the
// prehist of ops/radix.cpp RadixPartition): 8192-row tiles (the XCD-tile passes' kRPTile), 16 rows
// per thread.  Every column of a row is loaded before any is hashed -- the per-column loop of
// k_so_hash waited one memory latency per column (4 per row: 1B-row union side 11.2 ms, 3.6 TB/s).
constexpr int kSHThreads = 512, kSHTile = 8192, kSHItems = kSHTile / kSHThreads;

// NC >= ncols columns held per row; the column sets live in device memory (cols[0] = L, cols[1] = R):
// their fields are wave-uniform scalar loads, and neither set is copied into registers or scratch
// W8: every column is a non-null 8-byte number -- one unconditional 8-byte load per column, all in
// flight together (the width switch of load_bits put a wait for each load at its join point)
template <int NC, bool W8>
__device__ __forceinline__ uint64_t so_row_hash(const SOColSet *__restrict__ S, int ncols, int64_t i) {
  uint64_t raw[NC];
  uint8_t vb[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    raw[c] = 0;
    vb[c] = 1;
    if (c < ncols) {
      const ColView &col = S->c[c];
      if (W8) {
        raw[c] = reinterpret_cast<const uint64_t *>(col.data)[i];
      } else {
        if (col.kind != static_cast<int>(ValueKind::VAR_BYTES) &&
            col.kind != static_cast<int>(ValueKind::FIXED_BYTES))
          raw[c] = load_bits(col.data, i, col.width);
        if (col.valid != nullptr) vb[c] = col.valid[i];
      }
    }
  }
  uint64_t x = 0x84222325cbf29ce4ULL;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    if (c < ncols) {
      const ColView &col = S->c[c];
      uint64_t hv;
      if (!W8 && vb[c] == 0) {
        hv = 0x5bd1e9955bd1e995ULL;
      } else if (!W8 && (col.kind == static_cast<int>(ValueKind::VAR_BYTES) ||
                         col.kind == static_cast<int>(ValueKind::FIXED_BYTES))) {
        hv = so_value_hash(col, i);
      } else {
        uint64_t bits = (uint64_t)extend_bits(raw[c], col.width, col.kind);
        if (col.kind == static_cast<int>(ValueKind::FLOAT)) {
          bool nan = false;
          if (col.width == 8) nan = __longlong_as_double((long long)bits) != __longlong_as_double((long long)bits);
          else if (col.width == 4) nan = __int_as_float((int)bits) != __int_as_float((int)bits);
          else if (col.width == 2) nan = ((bits & 0x7c00u) == 0x7c00u) && (bits & 0x3ffu);
          if (nan) bits = 0x7ff8000000000000ull;
        }
        hv = hashing::fmix64(bits);
      }
      x = hashing::combine64(x, hv);
    }
  }
  return x | 1ull;  // 0 marks an empty LDS slot
}

template <int NC, bool W8>
__global__ __launch_bounds__(kSHThreads) void k_so_hash_tiles(const SOColSet *__restrict__ cols, int ncols, int64_t nl,
                                                              int64_t n, uint64_t *__restrict__ h, int bits,
                                                              uint32_t dmask, int64_t ntiles,
                                                              uint16_t *__restrict__ th) {
  __shared__ uint32_t hist[1024];
  const uint32_t nb = dmask + 1u;
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    for (uint32_t p = threadIdx.x; p < nb; p += kSHThreads) hist[p] = 0u;
    __syncthreads();
    const int64_t r0 = t * kSHTile;
    // a tile wholly on one side reads that side's column set through a block-uniform pointer (scalar
    // loads); only the tile holding row nl chooses per row
    const int side = r0 + kSHTile <= nl ? 0 : (r0 >= nl ? 1 : 2);
    auto one = [&](int64_t i, const SOColSet *S, int64_t j) {
      const uint64_t x = so_row_hash<NC, W8>(S, ncols, j);
      h[i] = x;
      if (th != nullptr) atomicAdd(&hist[(uint32_t)(hashing::fmix64(x) >> (64 - bits)) & dmask], 1u);
    };
    if (W8 && side < 2) {
      // 8-byte columns of one side: the column pointers / kinds are block-uniform; four rows' loads of
      // every column are issued before any of them is hashed (one memory latency per four rows)
      const SOColSet *S = cols + side;
      const int64_t jo = side ? nl : 0;
      const uint64_t *cp[NC];
      int kind[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        cp[c] = c < ncols ? reinterpret_cast<const uint64_t *>(S->c[c].data) : nullptr;
        kind[c] = c < ncols ? S->c[c].kind : 0;
      }
      constexpr int B = 4;
      for (int u0 = 0; u0 < kSHItems; u0 += B) {
        uint64_t raw[B][NC];
#pragma unroll
        for (int q = 0; q < B; ++q) {
          const int64_t i = r0 + (u0 + q) * kSHThreads + threadIdx.x;
#pragma unroll
          for (int c = 0; c < NC; ++c) raw[q][c] = (c < ncols && i < n) ? cp[c][i - jo] : 0ull;
        }
#pragma unroll
        for (int q = 0; q < B; ++q) {
          const int64_t i = r0 + (u0 + q) * kSHThreads + threadIdx.x;
          if (i >= n) continue;
          uint64_t x = 0x84222325cbf29ce4ULL;
#pragma unroll
          for (int c = 0; c < NC; ++c) {
            if (c >= ncols) continue;
            uint64_t b = raw[q][c];
            if (kind[c] == static_cast<int>(ValueKind::FLOAT) &&
                __longlong_as_double((long long)b) != __longlong_as_double((long long)b))
              b = 0x7ff8000000000000ull;
            x = hashing::combine64(x, hashing::fmix64(b));
          }
          x |= 1ull;
          h[i] = x;
          if (th != nullptr) atomicAdd(&hist[(uint32_t)(hashing::fmix64(x) >> (64 - bits)) & dmask], 1u);
        }
      }
    } else if (side == 0) {
      for (int u = 0; u < kSHItems; ++u) {
        const int64_t i = r0 + u * kSHThreads + threadIdx.x;
        if (i < n) one(i, cols, i);
      }
    } else if (side == 1) {
      for (int u = 0; u < kSHItems; ++u) {
        const int64_t i = r0 + u * kSHThreads + threadIdx.x;
        if (i < n) one(i, cols + 1, i - nl);
      }
    } else {
      for (int u = 0; u < kSHItems; ++u) {
        const int64_t i = r0 + u * kSHThreads + threadIdx.x;
        if (i < n && i < nl) one(i, cols, i);
        if (i < n && i >= nl) one(i, cols + 1, i - nl);
      }
    }
    __syncthreads();
    if (th != nullptr)
      for (uint32_t p = threadIdx.x; p < nb; p += kSHThreads) th[t * nb + p] = (uint16_t)hist[p];
    __syncthreads();
  }
}

void setop_row_hash_tiles(const ColView *lcols, const ColView *rcols, int ncols, int64_t nl, int64_t n, uint64_t *h,
                          int bits, int digit_bits, uint16_t *th, void *colsets, void *stream) {
  if (n == 0) return;
  CYLON_CHECK(ncols >= 1 && ncols <= kMaxFusedCols && digit_bits >= 1 && digit_bits <= 10 && bits >= digit_bits &&
                  bits <= 64,
              Code::Invalid, "row hash tiles: " << ncols << " columns, digit " << digit_bits << " of " << bits);
  SOColSet hs[2];
  for (int c = 0; c < ncols; ++c) {
    hs[0].c[c] = lcols[c];
    hs[1].c[c] = rcols ? rcols[c] : lcols[c];
  }
  hipStream_t s = as_stream(stream);
  HIP_CHECK(hipMemcpyAsync(colsets, hs, sizeof(hs), hipMemcpyHostToDevice, s));
  HIP_CHECK(hipStreamSynchronize(s));  // (hs is pageable host memory on this stack frame)
  const SOColSet *d = reinterpret_cast<const SOColSet *>(colsets);
  const int64_t ntiles = (n + kSHTile - 1) / kSHTile;
  const int grid = (int)std::min<int64_t>(ntiles, (int64_t)kNumCUs * 4);
  const uint32_t dm = (1u << digit_bits) - 1u;
  bool w8 = true;
  for (int c = 0; c < ncols; ++c)
    for (const SOColSet &x : hs)
      w8 &= x.c[c].width == 8 && x.c[c].valid == nullptr && x.c[c].kind != static_cast<int>(ValueKind::VAR_BYTES) &&
            x.c[c].kind != static_cast<int>(ValueKind::FIXED_BYTES);
  if (w8 && ncols <= 4)
    hipLaunchKernelGGL((k_so_hash_tiles<4, true>), dim3(grid), dim3(kSHThreads), 0, s, d, ncols, nl, n, h, bits, dm,
                       ntiles, th);
  else if (w8 && ncols <= 8)
    hipLaunchKernelGGL((k_so_hash_tiles<8, true>), dim3(grid), dim3(kSHThreads), 0, s, d, ncols, nl, n, h, bits, dm,
                       ntiles, th);
  else if (ncols <= 4)
    hipLaunchKernelGGL((k_so_hash_tiles<4, false>), dim3(grid), dim3(kSHThreads), 0, s, d, ncols, nl, n, h, bits, dm,
                       ntiles, th);
  else if (ncols <= 8)
    hipLaunchKernelGGL((k_so_hash_tiles<8, false>), dim3(grid), dim3(kSHThreads), 0, s, d, ncols, nl, n, h, bits, dm,
                       ntiles, th);
  else
    hipLaunchKernelGGL((k_so_hash_tiles<kMaxFusedCols, false>), dim3(grid), dim3(kSHThreads), 0, s, d, ncols, nl, n, h,
                       bits, dm, ntiles, th);
  HIP_LAUNCH_CHECK();
}

int64_t setop_colsets_bytes() { return (int64_t)(2 * sizeof(SOColSet)); }

int64_t setop_rows_per_part() { return kSORowsPerPart; }

__device__ __forceinline__ bool so_value_equal(const ColView &a, int64_t i, const ColView &b, int64_t j) {
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
    for (int k = 0; k < a.width; ++k)
      if (a.data[i * a.width + k] != b.data[j * a.width + k]) return false;
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
    if (a.width == 2) {
      const bool nx = ((x & 0x7c00) == 0x7c00) && (x & 0x3ff), ny = ((y & 0x7c00) == 0x7c00) && (y & 0x3ff);
      return nx ? ny : (!ny && x == y);
    }
  }
  return x == y;
}

__device__ __forceinline__ bool so_rows_equal(const SOColSet &L, const SOColSet &R, int ncols, int64_t nl,
                                              int64_t a, int64_t b) {
  const SOColSet &A = a < nl ? L : R;
  const SOColSet &B = b < nl ? L : R;
  const int64_t ia = a < nl ? a : a - nl, ib = b < nl ? b : b - nl;
  for (int c = 0; c < ncols; ++c)
    if (!so_value_equal(A.c[c], ia, B.c[c], ib)) return false;
  return true;
}

enum SOOp : int { SO_DISTINCT = 0, SO_SUBTRACT = 1, SO_INTERSECT = 2 };

// slot of hash h (claims one in phase 1); -1 if the table is full
template <bool kInsert>
__device__ __forceinline__ int so_slot(unsigned long long *keys, uint64_t h) {
  uint32_t s = (uint32_t)(((uint64_t)(uint32_t)h * kSOSlots) >> 32);  // not a power of two: multiply-shift
  for (int probes = 0; probes < kSOSlots; ++probes) {
    const unsigned long long cur = keys[s];
    if (cur == h) return (int)s;
    if (cur == 0ull) {
      if (!kInsert) return -1;
      const unsigned long long prev = atomicCAS(&keys[s], 0ull, (unsigned long long)h);
      if (prev == 0ull || prev == h) return (int)s;
    }
    s = s + 1 == (uint32_t)kSOSlots ? 0u : s + 1;
  }
  return -1;
}

static_assert(kSORowsPerPart % kSOThreads == 0, "rows per thread");
constexpr int kSOItems = (int)(kSORowsPerPart / kSOThreads);  // rows per thread held in registers

__device__ __forceinline__ void so_load(const uint64_t *__restrict__ ph, const int64_t *__restrict__ prow,
                                        const int64_t *__restrict__ offs, int64_t p, int64_t &rb, int64_t &re,
                                        uint64_t *hv, int64_t *rv) {
  rb = offs[p];
  re = offs[p + 1];
#pragma unroll
  for (int k = 0; k < kSOItems; ++k) {
    const int64_t r = rb + threadIdx.x + k * kSOThreads;
    if (r < re) {
      hv[k] = ph[r];
      rv[k] = prow[r];
    }
  }
}

// One workgroup per partition at a time.  The partition's (hash, row) pairs are
// held in registers (8 per thread) and the next partition's are loaded while this
// one is deduplicated, so the global latency hides behind the LDS work of the two
// phases (rows beyond 8192 in a skewed partition are streamed from global).
__global__ __launch_bounds__(kSOThreads) __attribute__((amdgpu_waves_per_eu(6))) void k_so_dedup(const uint64_t *__restrict__ ph,
                                                         const int64_t *__restrict__ prow,
                                                         const int64_t *__restrict__ offs, int64_t nparts,
                                                         int64_t nl, int op, int keep_last, SOColSet L, SOColSet R,
                                                         int ncols, uint8_t *__restrict__ mask,
                                                         unsigned long long *exc, int *bad) {
  __shared__ unsigned long long keys[kSOSlots];
  __shared__ uint32_t rep[kSOSlots];
  __shared__ uint32_t side[kSOSlots / 16];  // 2 bits per slot: 1 = on the left, 2 = on the right
  __shared__ int sbad;
  const uint32_t rep_init = keep_last ? 0u : 0xffffffffu;
  // phase 1: insert, fold representative position and side flags
  auto insert = [&](uint64_t h, int64_t row, uint32_t local) -> int {
    const int s = so_slot<true>(keys, h);
    if (s < 0) {
      sbad = 1;
      return s;
    }
    if (keep_last) atomicMax(&rep[s], local);
    else atomicMin(&rep[s], local);
    if (op != SO_DISTINCT) atomicOr(&side[s >> 4], (row < nl ? 1u : 2u) << ((s & 15) * 2));
    return s;
  };
  // phase 2: verify duplicates against their representative, write mask exceptions
  // slot: the slot phase 1 claimed for this row (-1: look it up again)
  auto verify = [&](bool active, uint64_t h, int64_t row, uint32_t local, int64_t rb, int slot) {
    bool flip = false;
    if (active) {
      const int s = slot >= 0 ? slot : so_slot<false>(keys, h);
      const bool first = rep[s] == local;
      if (!first && !so_rows_equal(L, R, ncols, nl, row, prow[rb + rep[s]])) atomicExch(bad, 1);  // collision
      if (op == SO_DISTINCT) {
        flip = !first;  // default keep
        if (flip) mask[row] = 0;
      } else if (row < nl) {
        const bool on_right = ((side[s >> 4] >> ((s & 15) * 2)) & 2u) != 0;
        if (op == SO_SUBTRACT) {
          flip = !(first && !on_right);  // default keep
          if (flip) mask[row] = 0;
        } else {
          flip = first && on_right;  // default drop
          if (flip) mask[row] = 1;
        }
      }
    }
    const uint64_t b = __ballot(flip);
    if (lane_id() == 0 && b) atomicAdd(exc, (unsigned long long)__popcll(b));
  };
  int64_t p = blockIdx.x, nb = 0, ne = 0;
  uint64_t nh[kSOItems];
  int64_t nr[kSOItems];
  if (p < nparts) so_load(ph, prow, offs, p, nb, ne, nh, nr);
  for (; p < nparts; p += gridDim.x) {
    const int64_t rb = nb, re = ne;
    uint64_t hv[kSOItems];
    int64_t rv[kSOItems];
#pragma unroll
    for (int k = 0; k < kSOItems; ++k) {
      hv[k] = nh[k];
      rv[k] = nr[k];
    }
    if (p + gridDim.x < nparts) so_load(ph, prow, offs, p + gridDim.x, nb, ne, nh, nr);
    if (rb == re) continue;
    __syncthreads();  // previous partition done with the table
    for (int s = threadIdx.x; s < kSOSlots; s += blockDim.x) {
      keys[s] = 0ull;
      rep[s] = rep_init;
    }
    for (int s = threadIdx.x; s < kSOSlots / 16; s += blockDim.x) side[s] = 0u;
    if (threadIdx.x == 0) sbad = 0;
    __syncthreads();
    int sl[kSOItems];  // claimed slots: phase 2 does not probe again
#pragma unroll
    for (int k = 0; k < kSOItems; ++k) {
      const int64_t r = rb + threadIdx.x + k * kSOThreads;
      sl[k] = r < re ? insert(hv[k], rv[k], (uint32_t)(r - rb)) : -1;
    }
    for (int64_t r = rb + kSORowsPerPart + threadIdx.x; r < re; r += kSOThreads)
      insert(ph[r], prow[r], (uint32_t)(r - rb));
    __syncthreads();
    if (sbad) {
      if (threadIdx.x == 0) atomicExch(bad, 1);
      continue;
    }
#pragma unroll
    for (int k = 0; k < kSOItems; ++k) {
      const int64_t r = rb + threadIdx.x + k * kSOThreads;
      verify(r < re, hv[k], rv[k], (uint32_t)(r - rb), rb, sl[k]);
    }
    for (int64_t r0 = rb + kSORowsPerPart; r0 < re; r0 += kSOThreads) {  // wave-uniform trip count
      const int64_t r = r0 + threadIdx.x;
      const bool act = r < re;
      verify(act, act ? ph[r] : 0, act ? prow[r] : 0, (uint32_t)(r - rb), rb, -1);
    }
  }
}

void setop_dedup(const uint64_t *ph, const int64_t *prow, const int64_t *offs, int64_t nparts, int64_t nl, int op,
                 bool keep_last, const ColView *lcols, const ColView *rcols, int ncols, uint8_t *mask, int64_t *exc,
                 int *bad, void *stream) {
  hipStream_t s = as_stream(stream);
  HIP_CHECK(hipMemsetAsync(exc, 0, sizeof(int64_t), s));
  HIP_CHECK(hipMemsetAsync(bad, 0, sizeof(int), s));
  if (nparts == 0) return;
  CYLON_CHECK(ncols >= 1 && ncols <= kMaxFusedCols, Code::Invalid, "set operation over " << ncols << " columns");
  SOColSet L, R;
  for (int c = 0; c < ncols; ++c) {
    L.c[c] = lcols[c];
    R.c[c] = rcols ? rcols[c] : lcols[c];
  }
  const int grid = (int)std::min<int64_t>(nparts, (int64_t)kNumCUs * 16);
  hipLaunchKernelGGL(k_so_dedup, dim3(grid), dim3(kSOThreads), 0, s, ph, prow, offs, nparts, nl, op,
                     keep_last ? 1 : 0, L, R, ncols, mask, reinterpret_cast<unsigned long long *>(exc), bad);
  HIP_LAUNCH_CHECK();
}

// this file's code object is loaded at context creation (preload_device_code), not on first use
void preload_radix_setops() { preload_code(reinterpret_cast<const void *>(&k_so_hash_tiles<4, true>)); }

}  // namespace hip
}  // namespace cylon
