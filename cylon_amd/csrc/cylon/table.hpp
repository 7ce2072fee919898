// Table: the core data structure (L2), and the engine's operator API (L4/L5).
//
// Reference: cpp/src/cylon/table.hpp:46-468 (Table wraps arrow::Table; all
// relational operators are free functions over shared_ptr<Table>).
// Here a Table is a vector of device-resident Columns on the context's device
// (an MI355X under one-process-per-GPU), plus the reference's retain flag.
// Operators in namespace cylon::ops throw CylonError; the Status-returning
// reference-shaped API lives in api.hpp.
#pragma once
#include <functional>
#include <memory>
#include <optional>
#include <string>
#include <vector>

#include "column.hpp"
#include "ctx/cylon_context.hpp"
#include "join/join_config.hpp"

namespace cylon {

namespace indexing {
class BaseIndex;
}

class Table;
using TablePtr = std::shared_ptr<Table>;

class Table {
 public:
  Table(std::shared_ptr<CylonContext> ctx, std::vector<Column> columns);

  static TablePtr Make(std::shared_ptr<CylonContext> ctx, std::vector<Column> columns) {
    return std::make_shared<Table>(std::move(ctx), std::move(columns));
  }

  int64_t Rows() const { return rows_; }
  int32_t Columns() const { return static_cast<int32_t>(columns_.size()); }
  std::vector<std::string> ColumnNames() const;
  const std::vector<Column> &columns() const { return columns_; }
  const Column &column(int i) const;
  int ColumnIndex(const std::string &name) const;  // -1 if absent
  const std::shared_ptr<CylonContext> &GetContext() const { return ctx_; }
  at::Device device() const;

  void retainMemory(bool retain) { retain_ = retain; }
  bool IsRetain() const { return retain_; }
  void Clear() {
    columns_.clear();
    rows_ = 0;
  }
  // retain = false (reference table.cpp:150-154, :358-362): an operator that has consumed this
  // table's rows drops its buffers early, so the memory returns to the allocator while the operator
  // still runs.  The columns keep their name, type and nullability, with 0 rows (the table is
  // empty afterwards).  A no-op for retained tables.
  void ReleaseIfNotRetained();
  // retain = false: drop one buffer of column c (its data, or its validity) while an operator that
  // consumes the table column group by column group still runs; ReleaseIfNotRetained() finishes.
  void ReleaseBufferIfNotRetained(int c, bool validity);

  // total bytes of all buffers
  int64_t nbytes() const;
  TablePtr to(at::Device dev) const;

  // C27: the table's index (reference table.cpp:1001-1055 Set_Index / GetIndex / ResetIndex);
  // none = the implicit range index 0..rows-1
  void SetIndex(std::shared_ptr<indexing::BaseIndex> index) { index_ = std::move(index); }
  const std::shared_ptr<indexing::BaseIndex> &GetIndex() const { return index_; }
  void ResetIndex() { index_.reset(); }

 private:
  std::shared_ptr<CylonContext> ctx_;
  std::vector<Column> columns_;
  std::shared_ptr<indexing::BaseIndex> index_;
  int64_t rows_ = 0;
  bool retain_ = true;
};

// Sort options for DistributedSort (reference table.hpp:388-393).
struct SortOptions {
  // DistributedSort samples num_samples rows per rank (0 -> 256 x world) for its exact
  // splitters; MapToSortPartitions (the reference's bin histogram) uses both fields.
  uint32_t num_bins = 0;     // 0 -> 16 * world
  uint64_t num_samples = 0;  // 0 -> DistributedSort: 256 x world per rank; MapToSortPartitions: 1% of rows
  static SortOptions Defaults() { return SortOptions(); }
};

namespace ops {

// ---- plumbing -------------------------------------------------------------
TablePtr Gather(const TablePtr &t, const at::Tensor &idx);  // idx int64, -1 -> null row
TablePtr GatherNullable(const TablePtr &t, const at::Tensor &idx, bool may_null);
Column GatherColumn(const Column &c, const at::Tensor &idx);
// K15 string / binary select: row i = cond[i] ? a[i] : b[i] (b of one row: broadcast; no b: null)
Column SelectVar(const Column &a, const std::optional<Column> &b, const at::Tensor &cond);
// K15 casts between strings and numbers on the column's device (kernels/strcast.hip): string ->
// integer / floating column, nullopt when a float needs the host's correctly rounded parser
// (the caller then casts on the host); integer -> string.  Unparsable strings raise Invalid.
std::optional<Column> CastStringToNumber(const Column &c, const DataType &target);
Column CastIntegerToString(const Column &c, const DataType &target);
TablePtr Project(const TablePtr &t, const std::vector<int> &cols);
TablePtr Merge(const std::vector<TablePtr> &tables);  // vertical concat
TablePtr Slice(const TablePtr &t, int64_t offset, int64_t length);
TablePtr FilterByMask(const TablePtr &t, const at::Tensor &mask);  // uint8/bool mask
at::Tensor MaskToIndices(const at::Tensor &mask, bool invert = false);

// ---- partitioning (K1/K2/K3) --------------------------------------------
// pid[i] in [0, nparts) and per-partition row counts (host vector).
std::pair<at::Tensor, std::vector<int64_t>> MapToHashPartitions(const TablePtr &t, const std::vector<int> &cols,
                                                                uint32_t nparts);
// Reorders rows partition-major (stable); returns reordered table + counts.
std::pair<TablePtr, std::vector<int64_t>> PartitionReorder(const TablePtr &t, const at::Tensor &pid,
                                                           uint32_t nparts);
std::vector<TablePtr> Split(const TablePtr &t, const at::Tensor &pid, uint32_t nparts);
// the shuffle's partitioning: reference hash partition ids -> partition-major table + counts
// (one LDS-staged pass for a single non-null 8-byte integer key on the device)
std::pair<TablePtr, std::vector<int64_t>> ShufflePartition(const TablePtr &t, const std::vector<int> &hash_cols,
                                                           uint32_t nparts);
std::vector<TablePtr> HashPartition(const TablePtr &t, const std::vector<int> &cols, uint32_t nparts);

// ---- communication --------------------------------------------------------
// partition-major table + per-partition counts -> received table
TablePtr AllToAllTable(const TablePtr &partitioned, const std::vector<int64_t> &counts);
// Posted (non-blocking) form of AllToAllTable: the size / schema agreement collectives
// run now, the column all-to-alls are left in flight (RCCL: on its stream).
// PostedExchangeReady tests the transfers without blocking; FinishPostedExchange waits
// (stream-ordered on RCCL) and assembles the received table.
struct PostedExchange;
std::shared_ptr<PostedExchange> PostAllToAllTable(const TablePtr &partitioned, const std::vector<int64_t> &counts);
bool PostedExchangeReady(PostedExchange &x);
TablePtr FinishPostedExchange(PostedExchange &x);
TablePtr Shuffle(const TablePtr &t, const std::vector<int> &hash_cols);
// shuffle two tables with the second one's partitioning overlapped with the first's transfer
std::pair<TablePtr, TablePtr> ShufflePair(const TablePtr &a, const std::vector<int> &acols, const TablePtr &b,
                                          const std::vector<int> &bcols);
// pipelined shuffle of two tables in `chunks` hash-disjoint chunks: consume(k, a_k, b_k) runs
// on chunk k while the transfers of the later chunks are still in flight (fixed-width columns)
// chunk count for ShufflePairChunked (same on every rank; 1 = unchunked)
int ShuffleChunks(const TablePtr &a, const TablePtr &b);
void ShufflePairChunked(const TablePtr &a, const std::vector<int> &acols, const TablePtr &b,
                        const std::vector<int> &bcols, int chunks,
                        const std::function<void(int, const TablePtr &, const TablePtr &)> &consume);
// The binary operators' shuffle (DistributedJoin, distributed set operations): decides the chunk
// count itself and agrees on everything the exchange needs -- chunk count, per-chunk row counts of
// both tables, column nullability, narrowed wire columns -- in ONE all-gather of a per-rank
// descriptor before the first payload all-to-all is posted.  consume(k, K, a_k, b_k) runs once per
// chunk (K == 1: the whole shuffled pair).  Var-width tables take ShufflePair (K = 1).
void ShufflePairPlanned(const TablePtr &a, const std::vector<int> &acols, const TablePtr &b,
                        const std::vector<int> &bcols,
                        const std::function<void(int, int, const TablePtr &, const TablePtr &)> &consume);
// Stable merge of consecutive sorted runs of `runs` (run_rows[r] rows each, in order) by column
// `col` (pairwise merge-path rounds, kernels/merge.hip): the receive side of the pipelined sort.
TablePtr MergeSortedRuns(const TablePtr &runs, const std::vector<int64_t> &run_rows, int col, bool asc);
// Pipelined range exchange (distributed sort) of a table whose rows are ordered by destination
// sub-range: bounds has W*K + 1 entries and rows [bounds[d*K + k], bounds[d*K + k + 1]) go to rank
// d in chunk k.  One all-gather of (rows, nullability, sub-range counts) plans every chunk, all
// chunks are posted at once (the communicator runs them in order) and consume(k, K, runs,
// run_rows) receives chunk k -- the rows from every rank in rank order, run_rows[r] from rank r --
// while the later chunks are still in flight.  Fixed-width columns only.
void RangeExchange(const TablePtr &t, const std::vector<int64_t> &bounds, int K,
                   const std::function<void(int, int, const TablePtr &, const std::vector<int64_t> &)> &consume);
// single-table form (distributed group-by / unique): consume(k, K, t_k) per hash-disjoint chunk
void ShufflePlanned(const TablePtr &t, const std::vector<int> &cols,
                    const std::function<void(int, int, const TablePtr &)> &consume);

// ---- relational -----------------------------------------------------------
TablePtr Join(const TablePtr &left, const TablePtr &right, const join::config::JoinConfig &cfg);
TablePtr DistributedJoin(const TablePtr &left, const TablePtr &right, const join::config::JoinConfig &cfg);
// index pairs of a local join (li, ri; -1 for the unmatched side)
std::pair<at::Tensor, at::Tensor> JoinIndices(const TablePtr &left, const TablePtr &right,
                                              const join::config::JoinConfig &cfg);
// C27/K16: index row positions matching each label, grouped by label order then row order
at::Tensor IndexLookup(const std::shared_ptr<CylonContext> &ctx, const Column &index, const Column &labels);
// A/B hook of the stable hash partitions (ops/radix.cpp): digit bits per pass, 3..10 (default 10)
void SetPartitionDigitBits(int bits);

// grouping = true: only equal values must end adjacent (list columns then sort by their bytes)
at::Tensor SortIndices(const TablePtr &t, const std::vector<int> &cols, const std::vector<bool> &ascending,
                       bool grouping = false);
TablePtr Sort(const TablePtr &t, const std::vector<int> &cols, const std::vector<bool> &ascending);

}  // namespace ops
}  // namespace cylon
