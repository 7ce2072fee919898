// Operator-layer helpers: device dispatch between the HIP kernels and their CPU
// twins, stream lookup and scratch allocation through torch's caching
// allocator (stream ordered, so scratch tensors may be released as soon as the
// launches that use them are enqueued).
#pragma once
#include <functional>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <c10/hip/HIPGuard.h>

#include <vector>

#include "../column.hpp"
#include "../kernels/kernels.hpp"
#include "../table.hpp"

namespace cylon {
namespace ops {

struct Exec {
  at::Device device{at::kCPU};
  bool gpu = false;
  void *stream = nullptr;

  explicit Exec(at::Device d) : device(d), gpu(d.is_cuda()) {
    if (gpu) stream = reinterpret_cast<void *>(c10::hip::getCurrentHIPStream(d.index()).stream());
  }

  at::TensorOptions opts(at::ScalarType t) const { return at::TensorOptions().dtype(t).device(device); }
  at::Tensor empty_i64(int64_t n) const { return at::empty({n}, opts(at::kLong)); }
  at::Tensor empty_u32(int64_t n) const { return at::empty({n}, opts(at::kInt)); }
  at::Tensor empty_u8(int64_t n) const { return at::empty({n}, opts(at::kByte)); }
  at::Tensor zeros_u8(int64_t n) const { return at::zeros({n}, opts(at::kByte)); }
  at::Tensor empty_bytes(int64_t n) const { return at::empty({n}, opts(at::kByte)); }
};

// Call the same primitive on the device the Exec targets.
#define KCALL(ex, fn, ...) \
  ((ex).gpu ? ::cylon::hip::fn(__VA_ARGS__, (ex).stream) : ::cylon::cpu::fn(__VA_ARGS__, nullptr))

#define KSIZE(ex, fn, ...) ((ex).gpu ? ::cylon::hip::fn(__VA_ARGS__) : ::cylon::cpu::fn(__VA_ARGS__))

template <typename T>
inline T *ptr(const at::Tensor &t) {
  return t.numel() ? reinterpret_cast<T *>(t.data_ptr()) : nullptr;
}

// Read a single int64 element to the host (synchronises the stream).
inline int64_t read_i64(const at::Tensor &t, int64_t index) { return t[index].item<int64_t>(); }

inline std::vector<int64_t> to_host_vec(const at::Tensor &t) {
  at::Tensor h = t.to(at::kCPU).contiguous();
  return std::vector<int64_t>(h.data_ptr<int64_t>(), h.data_ptr<int64_t>() + h.numel());
}

// Radix-partition tensors by the top `bits` bits of fmix64(cols[0]) (cols[0] =
// int64 keys, widths 1/2/4/8 bytes) with LSD passes of <= 10 bits
// (radix_join.hip).  Returns the permuted tensors; *offs = partition offsets
// [2^bits + 1].  GPU only.  With `range` the partition is instead the order-
// preserving ((key ^ flip) - mn) >> rshift (key ranges in key order).
struct RangeSpec {
  uint64_t flip = 0, mn = 0;
  int rshift = 0;
};
// stable = false lets the first LSD pass rank with LDS atomics (rows of one partition
// come out in no particular order: the hash join only).
// keep_packed != nullptr: validity-style 1-byte columns that were packed 8 per 8-byte word
// for the passes stay packed -- their slots come back undefined, the words are appended
// to the result and *keep_packed lists the packed column indices in byte order.
// prehist (stable hash partitions): called before the first pass with the address of that pass's
// per-tile digit counts in its workspace and the pass's digit bits; it must fill column 0 (the keys)
// and those counts (radix_setops.hip setop_row_hash_tiles), which the first pass then does not recount.
using PrehistFn = std::function<void(int64_t *tile_counts, int digit_bits)>;
std::vector<at::Tensor> RadixPartition(const Exec &ex, std::vector<at::Tensor> cols, const std::vector<int> &widths,
                                       int bits, at::Tensor *offs, const RangeSpec *range = nullptr,
                                       std::vector<int> *keep_packed = nullptr, bool stable = true,
                                       const hip::NarrowKeys *nk = nullptr, const PrehistFn *prehist = nullptr);

// Chunk-major order of a table for the bounded-memory join: one exact pass of every column by the
// LOW cbits bits of fmix64(column 0 = the int64 key) (independent of the join partition's top bits);
// *offs (2^cbits + 1 rows) = each chunk's first row.  Validity bytes travel packed as for RadixPartition.
// key_into: write column 0 into this existing array (a later column group of the same table: the
// stable pass puts the keys exactly where the first group's pass did); offs may then be nullptr.
// stable: every pass over the same keys produces the same row order (column groups).
std::vector<at::Tensor> RadixChunkPartition(const Exec &ex, std::vector<at::Tensor> cols, const std::vector<int> &widths,
                                            int cbits, at::Tensor *offs, const at::Tensor *key_into = nullptr,
                                            bool stable = false);

// Hash-join partition in slot mode (MSD, two passes, no histogram before the second pass; see
// kernel_decls.inc radix_slot_rows_pass): partition p holds (*counts)[p] rows at row p * slot.
// Returns an empty vector (nothing launched) when the shape is not eligible; *overflow (int32
// device flag) is set when a partition did not fit its slot -- the result is then unusable and
// the caller partitions exactly instead.  keep_packed as for RadixPartition.
std::vector<at::Tensor> RadixPartitionSlotted(const Exec &ex, std::vector<at::Tensor> cols,
                                              const std::vector<int> &widths, int bits, int64_t slot,
                                              at::Tensor *counts, at::Tensor *overflow,
                                              std::vector<int> *keep_packed = nullptr,
                                              const hip::NarrowKeys *nk = nullptr);

// Row-moving passes (k_rows_pass) take their all-8-byte path only when every moved
// column is 8 bytes wide; validity bytes beside 8-byte columns therefore travel packed
// 8 per 8-byte word (bitmap.hip pack_byte_columns).  PackByteColumns rewrites
// cols/widths in place (kept columns first, then the words) when that applies;
// UnpackByteColumns restores the original column order.
struct BytePacking {
  std::vector<int> byte_idx, keep_idx;  // original positions
  std::vector<at::ScalarType> byte_dtype;  // 1-byte dtypes (uint8 validity, bool/int8 data)
  bool active = false;
  int words() const { return ((int)byte_idx.size() + 7) / 8; }
};
BytePacking PackByteColumns(const Exec &ex, std::vector<at::Tensor> &cols, std::vector<int> &widths, int64_t n);
std::vector<at::Tensor> UnpackByteColumns(const Exec &ex, const BytePacking &bp, std::vector<at::Tensor> cols,
                                          int64_t n);

// exclusive scan of int64 counts -> offsets[n+1]
inline at::Tensor exclusive_scan(const Exec &ex, const at::Tensor &counts) {
  const int64_t n = counts.numel();
  at::Tensor out = ex.empty_i64(n + 1);
  at::Tensor ws = ex.empty_i64(KSIZE(ex, scan_workspace, n));
  KCALL(ex, exclusive_scan, ptr<int64_t>(counts), n, ptr<int64_t>(out), ptr<int64_t>(ws));
  return out;
}

inline bool same_schema(const TablePtr &a, const TablePtr &b) {
  if (a->Columns() != b->Columns()) return false;
  for (int i = 0; i < a->Columns(); ++i)
    if (a->column(i).type != b->column(i).type) return false;
  return true;
}

std::vector<ColView> views(const TablePtr &t, const std::vector<int> &cols);

// stable LSD radix sort of (uint64 keys stored in an int64 tensor, int64 values); consumes its inputs
std::pair<at::Tensor, at::Tensor> RadixSortPairs(const Exec &ex, at::Tensor keys, at::Tensor vals, int end_bit);

}  // namespace ops
}  // namespace cylon
