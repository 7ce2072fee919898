// Persistent table indexes and the loc / iloc indexers (C27 / K16).
//
// Reference: cpp/src/cylon/indexing/index.hpp:22-700 (IndexingSchema; HashIndex =
// unordered_multimap value -> positions, built once; LinearIndex = scan per lookup;
// RangeIndex; BinaryTree / BTree declared but unimplemented), indexer.hpp:76-260
// (LocIndexer / ILocIndexer: loc by single value, value list or value range x single
// column, column range or column list), table.cpp:1001-1055 (Set_Index / ResetIndex).
//
// Device design: a Hash / BinaryTree / BTree index is built ONCE when it is set on a
// table -- the order images of the index column radix-sorted with their row numbers
// (stable), plus, for Hash, an open-addressing table over the distinct images -- and
// every lookup is a probe (or binary search) per label, a scan of the match counts and
// a coalesced gather of positions (kernels/index.hip).  Linear keeps the reference's
// per-lookup semantics (one device join of the labels against the column).  Results
// are in label order, then row order (pandas `loc`).  String / binary index columns:
// the Hash schema is persistent too (reference HashIndex<arrow::StringType>, index.hpp:222)
// -- the runs are keyed by 64-bit hashes of the bytes and a probe verifies every candidate's
// bytes against its label; the sorted schemas use the per-lookup join.
#pragma once
#include <memory>

#include "../table.hpp"

namespace cylon {
namespace indexing {

enum class IndexingSchema : int { Range = 0, Linear = 1, Hash = 2, BinaryTree = 3, BTree = 4 };

class BaseIndex {
 public:
  virtual ~BaseIndex() = default;
  virtual IndexingSchema GetSchema() const = 0;
  virtual int64_t Size() const = 0;
  // row positions matching each label (label order, then row order); int64 on the index device
  virtual at::Tensor LocationsOf(const Column &labels) const = 0;
  // rows [first row holding `start`, last row holding `end`] (reference LocIndexer range semantics)
  std::pair<int64_t, int64_t> RangeOf(const Column &start, const Column &end) const;
  // the indexed values (nullptr for a range index)
  virtual const Column *IndexColumn() const { return nullptr; }
};

class RangeIndex : public BaseIndex {
 public:
  RangeIndex(int64_t start, int64_t stop, int64_t step, at::Device dev)
      : start_(start), stop_(stop), step_(step), dev_(dev) {}
  IndexingSchema GetSchema() const override { return IndexingSchema::Range; }
  int64_t Size() const override;
  at::Tensor LocationsOf(const Column &labels) const override;

 private:
  int64_t start_, stop_, step_;
  at::Device dev_;
};

class LinearIndex : public BaseIndex {
 public:
  LinearIndex(std::shared_ptr<CylonContext> ctx, Column col) : ctx_(std::move(ctx)), col_(std::move(col)) {}
  IndexingSchema GetSchema() const override { return IndexingSchema::Linear; }
  int64_t Size() const override { return col_.length; }
  at::Tensor LocationsOf(const Column &labels) const override;
  const Column *IndexColumn() const override { return &col_; }

 protected:
  std::shared_ptr<CylonContext> ctx_;
  Column col_;
};

// sorted images + rows (BinaryTree / BTree schemas: binary search per label)
class SortedIndex : public LinearIndex {
 public:
  SortedIndex(std::shared_ptr<CylonContext> ctx, Column col, IndexingSchema schema);
  IndexingSchema GetSchema() const override { return schema_; }
  at::Tensor LocationsOf(const Column &labels) const override;
  int64_t BuiltRows() const { return sorted_img_.defined() ? sorted_img_.numel() : 0; }

 protected:
  at::Tensor LabelImages(const Column &labels) const;                // same transform as the index
  at::Tensor GatherRuns(const at::Tensor &lo, const at::Tensor &cnt) const;
  bool persistent() const { return sorted_img_.defined(); }
  IndexingSchema schema_;
  at::Tensor sorted_img_, sorted_pos_;
};

// sorted images + an open-addressing table of the distinct images (probe per label)
class HashIndex : public SortedIndex {
 public:
  HashIndex(std::shared_ptr<CylonContext> ctx, Column col);
  at::Tensor LocationsOf(const Column &labels) const override;
  int64_t Capacity() const { return cap_; }
  bool BytesKeyed() const { return bytes_; }

 private:
  bool bytes_ = false;  // run keys are 64-bit hashes of string / binary values (verified on probe)
  int64_t cap_ = 0;
  at::Tensor tkeys_, used_, tlo_, tcnt_;
};

// Index over column `col` of `t` with `schema` (Range ignores the column: 0..rows-1).
std::shared_ptr<BaseIndex> BuildIndex(const TablePtr &t, int col, IndexingSchema schema);

// Reference LocIndexer: label-based selection through the table's index.
class LocIndexer {
 public:
  explicit LocIndexer(IndexingSchema schema = IndexingSchema::Hash) : schema_(schema) {}
  // rows whose index value is one of `values`; `columns` empty = all columns
  TablePtr Loc(const TablePtr &in, const Column &values, const std::vector<int> &columns = {}) const;
  // rows from the first `start` to the last `end` (inclusive)
  TablePtr LocRange(const TablePtr &in, const Column &start, const Column &end,
                    const std::vector<int> &columns = {}) const;
  IndexingSchema GetSchema() const { return schema_; }

 private:
  std::shared_ptr<BaseIndex> index_of(const TablePtr &in) const;
  IndexingSchema schema_;
};

// Reference ILocIndexer: position-based selection.
class ILocIndexer {
 public:
  TablePtr ILoc(const TablePtr &in, const at::Tensor &positions, const std::vector<int> &columns = {}) const;
  TablePtr ILocRange(const TablePtr &in, int64_t start, int64_t end, const std::vector<int> &columns = {}) const;
};

}  // namespace indexing
}  // namespace cylon
