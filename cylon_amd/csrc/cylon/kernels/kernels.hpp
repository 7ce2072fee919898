// Kernel-layer API (L3): raw-pointer primitives with identical signatures for
// the MI355X HIP implementation (namespace cylon::hip, *.hip files) and the CPU
// twin (namespace cylon::cpu, cpu_kernels.cpp).  The operator layer (ops/*.cpp)
// allocates every buffer through torch's stream-ordered caching allocator and
// dispatches on the tensor's device; kernels never allocate.
//
// Kernel inventory:
//   K1/K2 partition hash        -> row_partition_hash / hash_to_partition
//   K3    split / scatter       -> partition_positions + scatter_columns / scatter_var
//   K4    gather (-1 -> null)   -> gather_columns / gather_var
//   K5    hash join             -> hash_build / hash_probe_count / hash_probe_write
//   K6    radix sort            -> radix_sort_pairs (sort.hip)
//   K7    sort-merge join       -> merge_join_count / merge_join_write
//   K8/K9 group-by              -> groupby_* (groupby.hip)
//   K10   distinct / set ops    -> distinct_first / hash_set_*
//   K11   compaction            -> mask_to_indices
//   K12   reductions            -> reduce_column
//   K13   range partition       -> range_bins
//   K15   elementwise           -> elementwise.hip
#pragma once
#include "../common.hpp"

namespace cylon {

// Read-only column view handed to kernels.
struct ColView {
  const uint8_t *data = nullptr;     // fixed width values or var-width bytes
  const int64_t *offsets = nullptr;  // var width only (n + 1 entries)
  const uint8_t *valid = nullptr;    // optional byte mask, 1 = valid
  int32_t width = 0;                 // bytes per element, 0 for var width
  int32_t kind = 0;                  // ValueKind
};

struct MutColView {
  uint8_t *data = nullptr;
  int64_t *offsets = nullptr;
  uint8_t *valid = nullptr;
  int32_t width = 0;
  int32_t kind = 0;
};

// Hash-table slot for the join / group-by / distinct tables: 16 bytes, one
// global_load_dwordx4 per probe step.
struct alignas(16) HashSlot {
  int64_t key;
  int64_t row;  // -1 = empty
};

// A hash table: tsize slots; a key's home slot is slot_of(key, shift) < 2^(64-shift) <= tsize.
struct HashTableRef {
  HashSlot *slots;
  int64_t tsize;
  int shift;
};

constexpr int kMaxFusedCols = 16;  // columns handled by one multi-column launch
constexpr int kMaxCompositeKeys = 4;  // key columns of one composite join / group-by key

// buffers of one look-back LSD sort pass (radix_sort_lb_args; radix_join.hip "look-back sort passes")
struct SortLbArgs {
  const uint32_t *plan_in;  // this pass's chunk plan (nullptr: exact per-tile offsets)
  uint32_t *plan_out;       // the next pass's plan, counted by this pass (nullptr: last pass)
  uint32_t *state;          // [tile][nb] look-back words
  int64_t state_words;
  uint32_t *gcnt;           // [block][8][nbn] counts
  int64_t gcnt_words;
  unsigned int *err;        // look-back wait timed out
};

// Aggregation op ids, numerically identical to the reference
// (cpp/src/cylon/compute/aggregate_kernels.hpp:40-50).
// one accumulator of the LDS radix group-by (radix_groupby.hip)
struct RGAccDesc {
  const uint8_t *src;    // partitioned value column (nullptr: plain row count)
  const uint8_t *valid;  // partitioned validity bytes (nullptr: all valid)
  int kind;              // 0 SUM_F64, 1 SUM_I64, 2 MIN (order image), 3 MAX (order image), 4 COUNT,
                         // 5 M2 = sum of squared deviations from the group mean (VAR / STDDEV)
  int width, vkind;      // value width / ValueKind
  int sum_acc, cnt_acc;  // M2: the SUM_F64 and COUNT accumulators of the same column (their mean)
};

enum AggOp : int {
  AGG_SUM = 0,
  AGG_MIN = 1,
  AGG_MAX = 2,
  // COUNT = non-null values of the aggregated column, in the group-by and the scalar
  // aggregate alike.  The reference's scalar Count is the same (Arrow COUNT_NON_NULL,
  // compute/aggregates.cpp:55); its group-by CountKernel counts rows, nulls included
  // (compute/aggregate_kernels.hpp:438-440).  Deliberate pandas choice; identical on
  // non-null data (docs/semantics.md).
  AGG_COUNT = 3,
  AGG_MEAN = 4,
  AGG_VAR = 5,
  AGG_NUNIQUE = 6,
  AGG_QUANTILE = 7,
  AGG_STDDEV = 8,
};

namespace hip {
#include "kernel_decls.inc"
}  // namespace hip

namespace cpu {
#include "kernel_decls.inc"
}  // namespace cpu

}  // namespace cylon
