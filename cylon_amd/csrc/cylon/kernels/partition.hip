// K1/K2 partition hashing and K3 stable radix-partition scatter (gfx950).
//
// Reference semantics: cpp/src/cylon/arrow/arrow_partition_kernels.cpp:67-305
// (hash chain h = 31*h + f(v)), cpp/src/cylon/partition/partition.cpp:27-90
// (split into per-partition tables, order preserved inside a partition).
//
// MI355X design:
//   * row_partition_hash: one pass per key column over coalesced loads;
//     the chain stays in a uint32 per row.
//   * partition_positions: two kernels.  (1) per-block LDS histogram of pid;
//     (2) an exclusive scan of the partition-major block histogram (scan.hip);
//     (3) a stable rank kernel: inside a wave, lanes holding the same pid are
//     found with ceil(log2 P) 64-bit ballots (wave64 match), giving the
//     in-wave rank by one popcount; per-wave running counters live in LDS and
//     the cross-wave prefix is formed once per 2048-row sub-tile.  The result
//     is the destination of each row in partition-major order, so every
//     partition (and therefore every peer's slice in the RCCL shuffle) is one
//     contiguous range: no pack step before the all-to-all.
//   * scatter_columns: all fixed-width columns of a table in one launch,
//     destination read once per row.
#include "stable_rank.hpp"

namespace cylon {
namespace hip {

struct ColSet {
  ColView c[kMaxFusedCols];
};
struct MutColSet {
  MutColView c[kMaxFusedCols];
};

// ---------------------------------------------------------------------------
// K1 / K2
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t partition_f(const ColView &c, int64_t i) {
  if (c.valid != nullptr && c.valid[i] == 0) return 0u;
  const int kind = c.kind;
  if (kind == static_cast<int>(ValueKind::VAR_BYTES)) {
    const int64_t b = c.offsets[i], e = c.offsets[i + 1];
    return hashing::murmur3_32(c.data + b, e - b, 0u);
  }
  if (kind == static_cast<int>(ValueKind::FIXED_BYTES)) {
    return hashing::murmur3_32(c.data + i * (int64_t)c.width, c.width, 0u);
  }
  const uint64_t bits = load_bits(c.data, i, c.width);
  if (kind == static_cast<int>(ValueKind::FLOAT)) {
    switch (c.width) {
      case 2: return hashing::murmur3_32_u16((uint16_t)bits);
      case 4: return hashing::murmur3_32_u32((uint32_t)bits);
      default: return hashing::murmur3_32_u64(bits);
    }
  }
  // ModuloPartitionKernel: static_cast<uint32_t>(value)
  return (uint32_t)extend_bits(bits, c.width, kind);
}

__global__ void k_row_partition_hash(ColSet cols, int ncols, int64_t n, uint32_t *__restrict__ h) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    uint32_t acc = 0;
    for (int c = 0; c < ncols; ++c) acc = 31u * acc + partition_f(cols.c[c], i);
    h[i] = acc;
  }
}

void row_partition_hash(const ColView *cols, int ncols, int64_t n, uint32_t *h, void *stream) {
  if (n == 0) return;
  CYLON_CHECK(ncols <= kMaxFusedCols, Code::Invalid, "too many key columns " << ncols);
  ColSet s;
  for (int c = 0; c < ncols; ++c) s.c[c] = cols[c];
  hipLaunchKernelGGL(k_row_partition_hash, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), s,
                     ncols, n, h);
  HIP_LAUNCH_CHECK();
}

// pid + global histogram.  LDS histogram per block, one global atomic per
// (block, partition).
__global__ void k_hash_to_partition(const uint32_t *__restrict__ h, int64_t n, uint32_t nparts,
                                    uint32_t *__restrict__ pid, unsigned long long *counts) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  unsigned int *hist = reinterpret_cast<unsigned int *>(smem);
  const bool use_lds = nparts <= 8192;
  if (use_lds)
    for (uint32_t p = threadIdx.x; p < nparts; p += blockDim.x) hist[p] = 0;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint32_t p = hashing::partitioner(h[i], nparts);
    pid[i] = p;
    if (use_lds)
      atomicAdd(&hist[p], 1u);
    else
      atomicAdd(&counts[p], 1ull);
  }
  __syncthreads();
  if (use_lds)
    for (uint32_t p = threadIdx.x; p < nparts; p += blockDim.x)
      if (hist[p]) atomicAdd(&counts[p], (unsigned long long)hist[p]);
}

void hash_to_partition(const uint32_t *h, int64_t n, uint32_t nparts, uint32_t *pid, int64_t *counts,
                       void *stream) {
  HIP_CHECK(hipMemsetAsync(counts, 0, sizeof(int64_t) * nparts, as_stream(stream)));
  if (n == 0) return;
  size_t lds = nparts <= 8192 ? nparts * sizeof(unsigned int) : 0;
  hipLaunchKernelGGL(k_hash_to_partition, dim3(grid_for(n)), dim3(kBlock), lds, as_stream(stream), h,
                     n, nparts, pid, reinterpret_cast<unsigned long long *>(counts));
  HIP_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------
// K3: stable partition positions (stable_rank.hpp core, bucket = pid)
// ---------------------------------------------------------------------------
constexpr uint32_t kMaxPosParts = 4096;

struct PidDigit {
  const uint32_t *pid;
  __device__ __forceinline__ uint32_t operator()(int64_t i) const { return pid[i]; }
};
struct PosSink {
  int64_t *pos;
  __device__ __forceinline__ void operator()(int64_t i, int64_t d) const { pos[i] = d; }
};

int64_t partition_positions_workspace(int64_t n, uint32_t nparts) { return stable_rank_workspace(n, nparts); }

__global__ void k_counts_from_scan(const int64_t *bh_scan, int64_t nblocks, uint32_t nparts, int64_t *counts) {
  for (uint32_t p = blockIdx.x * blockDim.x + threadIdx.x; p < nparts; p += gridDim.x * blockDim.x)
    counts[p] = bh_scan[(int64_t)(p + 1) * nblocks] - bh_scan[(int64_t)p * nblocks];
}

void partition_positions(const uint32_t *pid, int64_t n, uint32_t nparts, int64_t *ws, int64_t *pos,
                         int64_t *counts, void *stream) {
  CYLON_CHECK(nparts >= 1 && nparts <= kMaxPosParts, Code::Invalid,
              "partition_positions supports 1.." << kMaxPosParts << " partitions, got " << nparts);
  hipStream_t s = as_stream(stream);
  if (n == 0) {
    HIP_CHECK(hipMemsetAsync(counts, 0, sizeof(int64_t) * nparts, s));
    return;
  }
  int64_t *bh_scan = nullptr;
  int64_t nblocks = 0;
  stable_rank_launch(PidDigit{pid}, PosSink{pos}, n, nparts, ws, s, &bh_scan, &nblocks);
  hipLaunchKernelGGL(k_counts_from_scan, dim3(grid_for(nparts)), dim3(kBlock), 0, s, (const int64_t *)bh_scan,
                     nblocks, nparts, counts);
  HIP_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------
// K3: scatter fixed-width columns (all columns of the table in one launch)
// ---------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ void move_elem(const uint8_t *src, int64_t si, uint8_t *dst, int64_t di) {
  reinterpret_cast<T *>(dst)[di] = reinterpret_cast<const T *>(src)[si];
}

__device__ __forceinline__ void move_any(const uint8_t *src, int64_t si, uint8_t *dst, int64_t di, int w) {
  switch (w) {
    case 1: move_elem<uint8_t>(src, si, dst, di); break;
    case 2: move_elem<uint16_t>(src, si, dst, di); break;
    case 4: move_elem<uint32_t>(src, si, dst, di); break;
    case 8: move_elem<uint64_t>(src, si, dst, di); break;
    case 16: move_elem<uint4>(src, si, dst, di); break;
    default:
      for (int b = 0; b < w; ++b) dst[di * w + b] = src[si * w + b];
  }
}

__global__ void k_scatter_columns(ColSet in, MutColSet out, int ncols, const int64_t *__restrict__ pos,
                                  int64_t n) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t d = pos[i];
    for (int c = 0; c < ncols; ++c) {
      move_any(in.c[c].data, i, out.c[c].data, d, in.c[c].width);
      if (out.c[c].valid) out.c[c].valid[d] = in.c[c].valid ? in.c[c].valid[i] : (uint8_t)1;
    }
  }
}

void scatter_columns(const ColView *in, const MutColView *out, int ncols, const int64_t *pos, int64_t n,
                     void *stream) {
  if (n == 0 || ncols == 0) return;
  for (int c0 = 0; c0 < ncols; c0 += kMaxFusedCols) {
    const int nc = (ncols - c0) < kMaxFusedCols ? (ncols - c0) : kMaxFusedCols;
    ColSet a;
    MutColSet b;
    for (int c = 0; c < nc; ++c) {
      a.c[c] = in[c0 + c];
      b.c[c] = out[c0 + c];
    }
    hipLaunchKernelGGL(k_scatter_columns, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), a, b, nc,
                       pos, n);
    HIP_LAUNCH_CHECK();
  }
}

__global__ void k_scatter_var_lengths(ColView in, const int64_t *__restrict__ pos, int64_t n,
                                      int64_t *__restrict__ out_lens) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    out_lens[pos[i]] = in.offsets[i + 1] - in.offsets[i];
}

void scatter_var_lengths(const ColView &in, const int64_t *pos, int64_t n, int64_t *out_lens, void *stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_scatter_var_lengths, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), in, pos, n,
                     out_lens);
  HIP_LAUNCH_CHECK();
}

// one wave per row: lanes copy the string bytes cooperatively
__global__ void k_scatter_var_bytes(ColView in, const int64_t *__restrict__ pos, int64_t n,
                                    const int64_t *__restrict__ out_off, uint8_t *__restrict__ out_bytes,
                                    uint8_t *__restrict__ out_valid) {
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x / kWave);
  const int lane = lane_id();
  for (int64_t i = (int64_t)blockIdx.x * (blockDim.x / kWave) + threadIdx.x / kWave; i < n; i += waves) {
    const int64_t d = pos[i];
    const int64_t sb = in.offsets[i], len = in.offsets[i + 1] - sb;
    const int64_t db = out_off[d];
    for (int64_t k = lane; k < len; k += kWave) out_bytes[db + k] = in.data[sb + k];
    if (lane == 0 && out_valid) out_valid[d] = in.valid ? in.valid[i] : (uint8_t)1;
  }
}

void scatter_var_bytes(const ColView &in, const int64_t *pos, int64_t n, const int64_t *out_offsets,
                       uint8_t *out_bytes, uint8_t *out_valid, void *stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_scatter_var_bytes, dim3(grid_for(n, kBlock / kWave)), dim3(kBlock), 0,
                     as_stream(stream), in, pos, n, out_offsets, out_bytes, out_valid);
  HIP_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------
// K4: gather with -1 -> null
// ---------------------------------------------------------------------------
__global__ void k_gather_columns(ColSet in, MutColSet out, int ncols, const int64_t *__restrict__ idx,
                                 int64_t m) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride) {
    const int64_t s = idx[j];
    for (int c = 0; c < ncols; ++c) {
      const int w = in.c[c].width;
      if (s >= 0) {
        move_any(in.c[c].data, s, out.c[c].data, j, w);
      } else {
        for (int b = 0; b < w; ++b) out.c[c].data[j * w + b] = 0;
      }
      if (out.c[c].valid)
        out.c[c].valid[j] = (s < 0) ? (uint8_t)0 : (in.c[c].valid ? in.c[c].valid[s] : (uint8_t)1);
    }
  }
}

void gather_columns(const ColView *in, const MutColView *out, int ncols, const int64_t *idx, int64_t m,
                    void *stream) {
  if (m == 0 || ncols == 0) return;
  for (int c0 = 0; c0 < ncols; c0 += kMaxFusedCols) {
    const int nc = (ncols - c0) < kMaxFusedCols ? (ncols - c0) : kMaxFusedCols;
    ColSet a;
    MutColSet b;
    for (int c = 0; c < nc; ++c) {
      a.c[c] = in[c0 + c];
      b.c[c] = out[c0 + c];
    }
    hipLaunchKernelGGL(k_gather_columns, dim3(grid_for(m)), dim3(kBlock), 0, as_stream(stream), a, b, nc, idx,
                       m);
    HIP_LAUNCH_CHECK();
  }
}

__global__ void k_gather_var_lengths(ColView in, const int64_t *__restrict__ idx, int64_t m,
                                     int64_t *__restrict__ out_lens) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; j < m; j += stride) {
    const int64_t s = idx[j];
    out_lens[j] = s < 0 ? 0 : in.offsets[s + 1] - in.offsets[s];
  }
}

void gather_var_lengths(const ColView &in, const int64_t *idx, int64_t m, int64_t *out_lens, void *stream) {
  if (m == 0) return;
  hipLaunchKernelGGL(k_gather_var_lengths, dim3(grid_for(m)), dim3(kBlock), 0, as_stream(stream), in, idx, m,
                     out_lens);
  HIP_LAUNCH_CHECK();
}

// G lanes per row (G from the mean row length: about 16 bytes per lane); 8-byte words where source
// and destination share their alignment mod 8, bytes elsewhere.  One wave per row (the old shape)
// left 48 of 64 lanes idle on 16-byte keys and ran at ~80 GB/s.
template <int G>
__global__ void k_gather_var_bytes(ColView in, const int64_t *__restrict__ idx, int64_t m,
                                   const int64_t *__restrict__ out_off, uint8_t *__restrict__ out_bytes,
                                   uint8_t *__restrict__ out_valid) {
  const int64_t groups = (int64_t)gridDim.x * (blockDim.x / G);
  const int sub = threadIdx.x % G;
  for (int64_t j = (int64_t)blockIdx.x * (blockDim.x / G) + threadIdx.x / G; j < m; j += groups) {
    const int64_t s = idx[j];
    if (s >= 0) {
      const int64_t sb = in.offsets[s], len = in.offsets[s + 1] - sb;
      const uint8_t *src = in.data + sb;
      uint8_t *dst = out_bytes + out_off[j];
      int64_t k0 = 0;
      if (len >= 16 && ((reinterpret_cast<uintptr_t>(src) ^ reinterpret_cast<uintptr_t>(dst)) & 7) == 0) {
        const int64_t head = (8 - (reinterpret_cast<uintptr_t>(dst) & 7)) & 7;
        for (int64_t k = sub; k < head; k += G) dst[k] = src[k];
        const int64_t words = (len - head) >> 3;
        const uint64_t *ws = reinterpret_cast<const uint64_t *>(src + head);
        uint64_t *wd = reinterpret_cast<uint64_t *>(dst + head);
        for (int64_t w = sub; w < words; w += G) wd[w] = ws[w];
        k0 = head + (words << 3);
      }
      for (int64_t k = k0 + sub; k < len; k += G) dst[k] = src[k];
    }
    if (sub == 0 && out_valid) out_valid[j] = (s < 0) ? (uint8_t)0 : (in.valid ? in.valid[s] : (uint8_t)1);
  }
}

void gather_var_bytes(const ColView &in, const int64_t *idx, int64_t m, const int64_t *out_offsets,
                      int64_t total_bytes, uint8_t *out_bytes, uint8_t *out_valid, void *stream) {
  if (m == 0) return;
  const int64_t mean = total_bytes / m;
  auto go = [&](auto kern, int g) {
    hipLaunchKernelGGL(kern, dim3(grid_for(m, kBlock / g)), dim3(kBlock), 0, as_stream(stream), in, idx, m,
                       out_offsets, out_bytes, out_valid);
  };
  if (mean <= 24)
    go(k_gather_var_bytes<1>, 1);
  else if (mean <= 96)
    go(k_gather_var_bytes<4>, 4);
  else if (mean <= 384)
    go(k_gather_var_bytes<16>, 16);
  else
    go(k_gather_var_bytes<kWave>, kWave);
  HIP_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------
// fixed-length strings <-> int64 word columns (ops/join.cpp: strings of L bytes travel through the
// radix join as ceil(L / 8) words); one row per thread, 8-byte accesses when L % 8 == 0
// ---------------------------------------------------------------------------
constexpr int kMaxWords = 8;
struct WordPtrs {
  int64_t *w[kMaxWords];
};
struct ConstWordPtrs {
  const int64_t *w[kMaxWords];
};

// hash (optional), inv = 0: the key row hash of a one-string-column key, hashing::combine64(seed,
// bytes_hash64(row)) as k_row_hash64 computes it, from the words in registers (bytes_hash64 folds
// the same little-endian words, the last one zero-padded) -- no second read of the bytes.
// inv = 1: hash = the invertible word key (hash.hpp word_key_*) and word 0 is not written.
__global__ void k_bytes_to_words(const uint8_t *__restrict__ bytes, int64_t n, int L, int W, int aligned8,
                                 WordPtrs out, uint64_t *__restrict__ hash, int inv) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint8_t *src = bytes + i * L;
    uint64_t h = hashing::word_key_seed(L), tail = 0, w0 = 0;
    for (int j = 0; j < W; ++j) {
      uint64_t v = 0;
      if (aligned8) {
        v = reinterpret_cast<const uint64_t *>(src)[j];
      } else {
        for (int b = 0; b < 8 && 8 * j + b < L; ++b) v |= (uint64_t)src[8 * j + b] << (8 * b);
      }
      if (inv) {
        if (j == 0) {
          w0 = v;
        } else {
          out.w[j][i] = (int64_t)v;
          h = hashing::word_key_step(h, v);
        }
        continue;
      }
      out.w[j][i] = (int64_t)v;
      if (8 * (j + 1) <= L) h = hashing::word_key_step(h, v);
      else tail = v;
    }
    if (inv) hash[i] = hashing::fmix64(w0 ^ h);
    else if (hash) hash[i] = hashing::combine64(0x84222325cbf29ce4ULL, hashing::fmix64(h ^ tail ^ ((uint64_t)L << 56)));
  }
}

// hash (optional): word 0 comes from the invertible word key, w0 = fmix64_inv(hash) ^ g(words 1..)
__global__ void k_words_to_bytes(ConstWordPtrs in, int64_t n, int L, int W, int aligned8,
                                 uint8_t *__restrict__ bytes, const uint64_t *__restrict__ hash) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    uint8_t *dst = bytes + i * L;
    auto put = [&](int j, uint64_t v) {
      if (aligned8) {
        reinterpret_cast<uint64_t *>(dst)[j] = v;
      } else {
        for (int b = 0; b < 8 && 8 * j + b < L; ++b) dst[8 * j + b] = (uint8_t)(v >> (8 * b));
      }
    };
    uint64_t g = hashing::word_key_seed(L);
    for (int j = hash ? 1 : 0; j < W; ++j) {
      const uint64_t v = (uint64_t)in.w[j][i];
      if (hash) g = hashing::word_key_step(g, v);
      put(j, v);
    }
    if (hash) put(0, hashing::fmix64_inv(hash[i]) ^ g);
  }
}

// bad[i] = 1 where both rows are present and any word differs
__global__ void k_words_mismatch(ConstWordPtrs a, ConstWordPtrs b, int W, const uint8_t *__restrict__ va,
                                 const uint8_t *__restrict__ vb, int64_t n, uint8_t *__restrict__ bad,
                                 unsigned long long *nbad) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  unsigned long long c = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    bool diff = false;
    for (int j = 0; j < W; ++j) diff |= a.w[j][i] != b.w[j][i];
    if (va && !va[i]) diff = false;
    if (vb && !vb[i]) diff = false;
    bad[i] = diff ? 1 : 0;
    c += diff ? 1ull : 0ull;
  }
  // the count rides along (no separate reduction over the flags): one atomic per wave that saw a row
  for (int d = kWave / 2; d > 0; d >>= 1) c += __shfl_xor(c, d, kWave);
  if ((threadIdx.x & (kWave - 1)) == 0 && c) atomicAdd(nbad, c);
}

// ---- variable-length strings as W zero-padded words + a length (the padded word key: the fixed-length
// invertible key of hash.hpp over W words, seeded with the row's own length).  A row's bytes are read
// as the aligned 8-byte words that hold at least one of its bytes (never past its last byte's word,
// so never into another page) and funnel-shifted into place.
// Text mode (text = 1: no row holds a zero byte -- *nul reports one if it does): the key is seeded
// with 0 instead of the length, which the zero padding then encodes (the string ends at the first
// zero byte), so no length column travels; words_to_var recomputes the lengths from the words.
__device__ __forceinline__ bool has_zero_byte(uint64_t v) {
  return ((v - 0x0101010101010101ull) & ~v & 0x8080808080808080ull) != 0;
}

__global__ void k_var_to_words(const uint8_t *__restrict__ bytes, const int64_t *__restrict__ offs, int64_t n, int W,
                               WordPtrs out, uint64_t *__restrict__ hash, int64_t *__restrict__ lens,
                               uint64_t *__restrict__ h2, int text, unsigned int *__restrict__ nul) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  bool anynul = false;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t o = offs[i], L = offs[i + 1] - o;
    const uintptr_t a = reinterpret_cast<uintptr_t>(bytes + o);
    const uint64_t *p = reinterpret_cast<const uint64_t *>(a & ~uintptr_t(7));
    const int sh = (int)(a & 7) * 8;
    const int64_t nw = ((int64_t)(a & 7) + L + 7) >> 3;  // aligned words holding the row's bytes
    uint64_t g = hashing::word_key_seed(text ? 0 : L), w0 = 0, s2 = 0xC2B2AE3D27D4EB4FULL ^ (uint64_t)L;
    uint64_t cur = nw > 0 ? p[0] : 0;
    for (int j = 0; j < W; ++j) {
      const uint64_t nxt = j + 1 < nw ? p[j + 1] : 0;
      uint64_t v = sh ? (cur >> sh) | (nxt << (64 - sh)) : cur;
      const int64_t rem = L - 8 * (int64_t)j;  // row bytes from word j on
      uint64_t keep = ~0ull;
      if (rem <= 0) keep = 0;
      else if (rem < 8) keep = (uint64_t(1) << (8 * rem)) - 1;
      v &= keep;
      if (nul && rem > 0) anynul |= has_zero_byte(v | ~keep);
      cur = nxt;
      if (j == 0) w0 = v;
      else {
        out.w[j][i] = (int64_t)v;
        g = hashing::word_key_step(g, v);
      }
      s2 = hashing::fmix64((s2 + v) * 0x87C37B91114253D5ULL) ^ 0x4CF5AD432745937FULL;
    }
    hash[i] = hashing::fmix64(w0 ^ g);
    if (lens) lens[i] = L;
    if (h2) h2[i] = s2;
  }
  if (anynul) atomicOr(nul, 1u);
}

// text mode: row lengths from the words (the first zero byte; w0 rebuilt from the key)
__global__ void k_padded_text_lens(ConstWordPtrs in, const uint64_t *__restrict__ hash, int64_t n, int W,
                                   int64_t *__restrict__ lens) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    uint64_t w[kMaxWords];
    uint64_t g = hashing::word_key_seed(0);
#pragma unroll
    for (int j = 1; j < kMaxWords; ++j) {
      w[j] = j < W ? (uint64_t)in.w[j][i] : 0;
      if (j < W) g = hashing::word_key_step(g, w[j]);
    }
    w[0] = hashing::fmix64_inv(hash[i]) ^ g;
    int64_t L = 8 * W;
    bool found = false;
#pragma unroll
    for (int j = 0; j < kMaxWords; ++j) {
      if (j >= W || found) continue;
      const uint64_t z = (w[j] - 0x0101010101010101ull) & ~w[j] & 0x8080808080808080ull;
      if (z) {  // (the lowest flagged byte is exact: the first zero byte)
        L = 8 * j + (__ffsll((long long)z) - 1) / 8;
        found = true;
      }
    }
    lens[i] = L;
  }
}

// nb <= 8 bytes of v at d with the widest naturally aligned stores
__device__ __forceinline__ void put_bytes(uint8_t *d, uint64_t v, int nb) {
  while (nb > 0) {
    const uintptr_t a = reinterpret_cast<uintptr_t>(d);
    if ((a & 7) == 0 && nb == 8) {
      *reinterpret_cast<uint64_t *>(d) = v;
      return;
    }
    if ((a & 3) == 0 && nb >= 4) {
      *reinterpret_cast<uint32_t *>(d) = (uint32_t)v;
      d += 4;
      v >>= 32;
      nb -= 4;
    } else if ((a & 1) == 0 && nb >= 2) {
      *reinterpret_cast<uint16_t *>(d) = (uint16_t)v;
      d += 2;
      v >>= 16;
      nb -= 2;
    } else {
      *d = (uint8_t)v;
      ++d;
      v >>= 8;
      --nb;
    }
  }
}

// A row of L bytes at dst (any alignment): the head up to dst's next 8-byte boundary, then aligned
// 8-byte stores of the words funnel-shifted by the head length, then the tail -- ~L / 8 + 4 stores
// instead of L byte stores (neighbouring rows share the head / tail words: no wider stores there).
__global__ void k_words_to_var(ConstWordPtrs in, const uint64_t *__restrict__ hash, const int64_t *__restrict__ lens,
                               const int64_t *__restrict__ ooffs, int64_t n, int W, int text,
                               uint8_t *__restrict__ bytes) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t L = lens[i];
    if (L <= 0) continue;
    uint8_t *dst = bytes + ooffs[i];
    uint64_t w[kMaxWords + 1];
    uint64_t g = hashing::word_key_seed(text ? 0 : L);
#pragma unroll
    for (int j = 1; j < kMaxWords; ++j) {
      w[j] = j < W ? (uint64_t)in.w[j][i] : 0;
      if (j < W) g = hashing::word_key_step(g, w[j]);
    }
    w[kMaxWords] = 0;
    w[0] = hashing::fmix64_inv(hash[i]) ^ g;
    const int h = (int)((8 - (reinterpret_cast<uintptr_t>(dst) & 7)) & 7);  // head bytes
    if (L <= h) {
      put_bytes(dst, w[0], (int)L);
      continue;
    }
    if (h) put_bytes(dst, w[0], h);
    const int64_t body = (L - h) >> 3;  // aligned 8-byte chunks
#pragma unroll
    for (int k = 0; k < kMaxWords; ++k) {
      if (k >= body) break;
      const uint64_t c = h ? (w[k] >> (8 * h)) | (w[k + 1] << (64 - 8 * h)) : w[k];
      *reinterpret_cast<uint64_t *>(dst + h + 8 * k) = c;
    }
    const int tail = (int)((L - h) & 7);
    if (tail) {
      uint64_t c = 0;
#pragma unroll
      for (int k = 0; k < kMaxWords; ++k)
        if (k == body) c = h ? (w[k] >> (8 * h)) | (w[k + 1] << (64 - 8 * h)) : w[k];
      put_bytes(dst + h + 8 * body, c, tail);
    }
  }
}

// two independent 64-bit hashes of rows of any length (the group-by's string key h and its check
// h2): different seeds, and h2 mixes with a different multiplier and an add instead of a xor
__global__ void k_var_hash2(const uint8_t *__restrict__ bytes, const int64_t *__restrict__ offs, int64_t n,
                            uint64_t *__restrict__ h1, uint64_t *__restrict__ h2, int pack_row) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t o = offs[i], L = offs[i + 1] - o;
    const uintptr_t a = reinterpret_cast<uintptr_t>(bytes + o);
    const uint64_t *p = reinterpret_cast<const uint64_t *>(a & ~uintptr_t(7));
    const int sh = (int)(a & 7) * 8;
    const int64_t nw = ((int64_t)(a & 7) + L + 7) >> 3, W = (L + 7) >> 3;
    uint64_t x = hashing::word_key_seed(L), y = 0xC2B2AE3D27D4EB4FULL ^ (uint64_t)L;
    uint64_t cur = nw > 0 ? p[0] : 0;
    for (int64_t j = 0; j < W; ++j) {
      const uint64_t nxt = j + 1 < nw ? p[j + 1] : 0;
      uint64_t v = sh ? (cur >> sh) | (nxt << (64 - sh)) : cur;
      const int64_t rem = L - 8 * j;
      if (rem < 8) v &= (uint64_t(1) << (8 * rem)) - 1;
      cur = nxt;
      x = hashing::word_key_step(x, v);
      y = hashing::fmix64((y + v) * 0x87C37B91114253D5ULL) ^ 0x4CF5AD432745937FULL;
    }
    h1[i] = hashing::fmix64(x);
    h2[i] = pack_row ? (y & 0xFFFFFFFF00000000ull) | (uint64_t)i : y;
  }
}

void var_hash2(const uint8_t *bytes, const int64_t *offs, int64_t n, uint64_t *h1, uint64_t *h2, void *stream,
               bool pack_row) {
  CYLON_CHECK(!pack_row || n <= (int64_t(1) << 32), Code::Invalid, "var_hash2: row numbers beyond 32 bits");
  if (n == 0) return;
  hipLaunchKernelGGL(k_var_hash2, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), bytes, offs, n, h1, h2,
                     pack_row ? 1 : 0);
  HIP_LAUNCH_CHECK();
}

void var_to_words(const uint8_t *bytes, const int64_t *offs, int64_t n, int W, int64_t *const *words, uint64_t *hash,
                  int64_t *lens, uint64_t *h2, void *stream, bool text, unsigned int *nul) {
  CYLON_CHECK(W >= 1 && W <= kMaxWords && hash && (lens || text), Code::Invalid, "padded string words: W " << W);
  if (n == 0) return;
  WordPtrs o{};
  for (int j = 1; j < W; ++j) o.w[j] = words[j];
  hipLaunchKernelGGL(k_var_to_words, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), bytes, offs, n, W, o, hash,
                     lens, h2, text ? 1 : 0, nul);
  HIP_LAUNCH_CHECK();
}

void padded_text_lens(const int64_t *const *words, const uint64_t *hash, int64_t n, int W, int64_t *lens,
                      void *stream) {
  CYLON_CHECK(W >= 1 && W <= kMaxWords && hash, Code::Invalid, "padded string words: W " << W);
  if (n == 0) return;
  ConstWordPtrs in{};
  for (int j = 1; j < W; ++j) in.w[j] = words[j];
  hipLaunchKernelGGL(k_padded_text_lens, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), in, hash, n, W, lens);
  HIP_LAUNCH_CHECK();
}

void words_to_var(const int64_t *const *words, const uint64_t *hash, const int64_t *lens, const int64_t *out_offs,
                  int64_t n, int W, uint8_t *bytes, void *stream, bool text) {
  CYLON_CHECK(W >= 1 && W <= kMaxWords && hash, Code::Invalid, "padded string words: W " << W);
  if (n == 0) return;
  ConstWordPtrs in{};
  for (int j = 1; j < W; ++j) in.w[j] = words[j];
  hipLaunchKernelGGL(k_words_to_var, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), in, hash, lens, out_offs,
                     n, W, text ? 1 : 0, bytes);
  HIP_LAUNCH_CHECK();
}

// mm[0] = min, mm[1] = max of the row lengths offs[i + 1] - offs[i] (mm preset to {~0, 0})
__global__ void k_len_minmax(const int64_t *__restrict__ offs, int64_t n, unsigned long long *mm) {
  unsigned long long lo = ~0ull, hi = 0ull;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const unsigned long long l = (unsigned long long)(offs[i + 1] - offs[i]);
    lo = l < lo ? l : lo;
    hi = l > hi ? l : hi;
  }
  for (int d = kWave / 2; d > 0; d >>= 1) {
    const unsigned long long a = __shfl_xor(lo, d, kWave), b = __shfl_xor(hi, d, kWave);
    lo = a < lo ? a : lo;
    hi = b > hi ? b : hi;
  }
  if (lane_id() == 0) {
    atomicMin(&mm[0], lo);
    atomicMax(&mm[1], hi);
  }
}

void var_len_minmax(const int64_t *offs, int64_t n, int64_t *mm, void *stream) {
  hipStream_t s = as_stream(stream);
  HIP_CHECK(hipMemsetAsync(mm, 0xff, sizeof(int64_t), s));  // min: all ones
  HIP_CHECK(hipMemsetAsync(mm + 1, 0, sizeof(int64_t), s));
  if (n > 0) {
    hipLaunchKernelGGL(k_len_minmax, dim3(grid_for(n)), dim3(kBlock), 0, s, offs, n,
                       reinterpret_cast<unsigned long long *>(mm));
    HIP_LAUNCH_CHECK();
  }
}

void bytes_to_words(const uint8_t *bytes, int64_t n, int L, int64_t *const *words, void *stream, uint64_t *hash,
                    bool inv) {
  const int W = (L + 7) / 8;
  CYLON_CHECK(L >= 1 && W <= kMaxWords, Code::Invalid, "string words: length " << L);
  CYLON_CHECK(!inv || hash, Code::Invalid, "string words: the invertible key needs its output");
  if (n == 0) return;
  WordPtrs o{};
  for (int j = inv ? 1 : 0; j < W; ++j) o.w[j] = words[j];
  const int al = (L & 7) == 0 && (reinterpret_cast<uintptr_t>(bytes) & 7) == 0;  // 8-byte accesses
  hipLaunchKernelGGL(k_bytes_to_words, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), bytes, n, L, W, al, o,
                     hash, inv ? 1 : 0);
  HIP_LAUNCH_CHECK();
}

void words_to_bytes(const int64_t *const *words, int64_t n, int L, uint8_t *bytes, void *stream,
                    const uint64_t *hash) {
  const int W = (L + 7) / 8;
  CYLON_CHECK(L >= 1 && W <= kMaxWords, Code::Invalid, "string words: length " << L);
  if (n == 0) return;
  ConstWordPtrs in{};
  for (int j = hash ? 1 : 0; j < W; ++j) in.w[j] = words[j];
  const int al = (L & 7) == 0 && (reinterpret_cast<uintptr_t>(bytes) & 7) == 0;
  hipLaunchKernelGGL(k_words_to_bytes, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), in, n, L, W, al, bytes,
                     hash);
  HIP_LAUNCH_CHECK();
}

void words_mismatch(const int64_t *const *a, const int64_t *const *b, int W, const uint8_t *va, const uint8_t *vb,
                    int64_t n, uint8_t *bad, int64_t *nbad, void *stream) {
  CYLON_CHECK(W >= 1 && W <= kMaxWords, Code::Invalid, "string words: " << W);
  HIP_CHECK(hipMemsetAsync(nbad, 0, sizeof(int64_t), as_stream(stream)));
  if (n == 0) return;
  ConstWordPtrs pa{}, pb{};
  for (int j = 0; j < W; ++j) {
    pa.w[j] = a[j];
    pb.w[j] = b[j];
  }
  hipLaunchKernelGGL(k_words_mismatch, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), pa, pb, W, va, vb, n,
                     bad, reinterpret_cast<unsigned long long *>(nbad));
  HIP_LAUNCH_CHECK();
}

// ---------------------------------------------------------------------------
// shuffle wire narrowing (int64 <-> uint32 offsets from a global base): two
// rows per thread with 16-byte accesses of the wide side when aligned
// ---------------------------------------------------------------------------
template <bool kVec>
__global__ void k_narrow_i64(const int64_t *__restrict__ in, int64_t n, int64_t base, uint32_t *__restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (kVec) {
    for (int64_t i = t0; i < (n >> 1); i += stride) {
      const longlong2 v = reinterpret_cast<const longlong2 *>(in)[i];
      reinterpret_cast<uint2 *>(out)[i] =
          make_uint2((uint32_t)((uint64_t)v.x - (uint64_t)base), (uint32_t)((uint64_t)v.y - (uint64_t)base));
    }
    if ((n & 1) && t0 == 0) out[n - 1] = (uint32_t)((uint64_t)in[n - 1] - (uint64_t)base);
  } else {
    for (int64_t i = t0; i < n; i += stride) out[i] = (uint32_t)((uint64_t)in[i] - (uint64_t)base);
  }
}

template <bool kVec>
__global__ void k_widen_u32(const uint32_t *__restrict__ in, int64_t n, int64_t base, int64_t *__restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (kVec) {
    for (int64_t i = t0; i < (n >> 1); i += stride) {
      const uint2 v = reinterpret_cast<const uint2 *>(in)[i];
      longlong2 o;
      o.x = (long long)((uint64_t)base + v.x);
      o.y = (long long)((uint64_t)base + v.y);
      reinterpret_cast<longlong2 *>(out)[i] = o;
    }
    if ((n & 1) && t0 == 0) out[n - 1] = (int64_t)((uint64_t)base + in[n - 1]);
  } else {
    for (int64_t i = t0; i < n; i += stride) out[i] = (int64_t)((uint64_t)base + in[i]);
  }
}

void narrow_i64(const int64_t *in, int64_t n, int64_t base, uint32_t *out, void *stream) {
  if (n == 0) return;
  const bool vec = reinterpret_cast<uintptr_t>(in) % 16 == 0 && reinterpret_cast<uintptr_t>(out) % 8 == 0;
  if (vec)
    hipLaunchKernelGGL(k_narrow_i64<true>, dim3(grid_for((n + 1) / 2)), dim3(kBlock), 0, as_stream(stream), in, n,
                       base, out);
  else
    hipLaunchKernelGGL(k_narrow_i64<false>, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), in, n, base, out);
  HIP_LAUNCH_CHECK();
}

void widen_u32(const uint32_t *in, int64_t n, int64_t base, int64_t *out, void *stream) {
  if (n == 0) return;
  const bool vec = reinterpret_cast<uintptr_t>(in) % 8 == 0 && reinterpret_cast<uintptr_t>(out) % 16 == 0;
  if (vec)
    hipLaunchKernelGGL(k_widen_u32<true>, dim3(grid_for((n + 1) / 2)), dim3(kBlock), 0, as_stream(stream), in, n,
                       base, out);
  else
    hipLaunchKernelGGL(k_widen_u32<false>, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), in, n, base, out);
  HIP_LAUNCH_CHECK();
}

// this file's code object is loaded at context creation (preload_device_code), not on first use
void preload_partition() { preload_code(reinterpret_cast<const void *>(&k_row_partition_hash)); }

}  // namespace hip
}  // namespace cylon
