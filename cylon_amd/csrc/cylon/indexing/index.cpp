// Persistent indexes and loc / iloc (see index.hpp).
#include "index.hpp"

#include "../ops/util.hpp"
#include "../trace.hpp"

namespace cylon {
namespace indexing {

using ops::Exec;
using ops::ptr;

std::pair<int64_t, int64_t> BaseIndex::RangeOf(const Column &start, const Column &end) const {
  at::Tensor s = LocationsOf(start), e = LocationsOf(end);
  CYLON_CHECK(s.numel() > 0 && e.numel() > 0, Code::KeyError, "index range bounds not found");
  return {s.min().item<int64_t>(), e.max().item<int64_t>()};
}

// ---- range ------------------------------------------------------------------
int64_t RangeIndex::Size() const { return step_ > 0 ? std::max<int64_t>(0, (stop_ - start_ + step_ - 1) / step_) : 0; }

at::Tensor RangeIndex::LocationsOf(const Column &labels) const {
  at::Tensor v = labels.data.slice(0, 0, labels.length).to(dev_).to(at::kLong);
  at::Tensor ok = (v >= start_) & (v < stop_) & ((v - start_).remainder(step_) == 0);
  if (labels.nullable()) ok &= labels.validity.slice(0, 0, labels.length).to(dev_).ne(0);
  return ((v - start_) / step_).masked_select(ok).contiguous();
}

// ---- linear (per-lookup join, the reference's scan index) ------------------------
// Labels in the index column's type.  A label that the conversion does not carry exactly
// (2.5 against an integer index, 300 against int8, 2^53 + 1 against float64) matches nothing:
// it is marked null instead of matching the value it was rounded to.
static Column as_index_type(const Column &labels, const Column &index) {
  if (labels.type == index.type || index.is_var() || labels.is_var()) return labels.to(index.data.device());
  const at::Device dev = index.data.device();
  at::Tensor src = labels.data.slice(0, 0, labels.length).to(dev);
  at::Tensor d = src.to(storage_dtype(index.type));
  at::Tensor exact = d.to(src.scalar_type()).eq(src);
  if (at::isFloatingType(src.scalar_type()) || at::isFloatingType(d.scalar_type()))  // and back, in double
    exact &= d.to(at::kDouble).eq(src.to(at::kDouble));
  at::Tensor v = exact.to(at::kByte);
  if (labels.nullable()) v.mul_(labels.validity.slice(0, 0, labels.length).to(dev).ne(0).to(at::kByte));
  return Column(labels.name, index.type, labels.length, d, at::Tensor(), v);
}

at::Tensor LinearIndex::LocationsOf(const Column &labels) const {
  return ops::IndexLookup(ctx_, col_, as_index_type(labels, col_));
}

// ---- sorted (binary tree / b-tree schemas) --------------------------------------
SortedIndex::SortedIndex(std::shared_ptr<CylonContext> ctx, Column col, IndexingSchema schema)
    : LinearIndex(std::move(ctx), std::move(col)), schema_(schema) {
  if (col_.is_var() || col_.type.kind() == ValueKind::FIXED_BYTES) return;  // strings: per-lookup join
  Exec ex(col_.data.device());
  CYLON_PHASE("index.build", ex.device);
  // rows with a value (null index entries never match a label)
  at::Tensor rows = col_.nullable() ? ops::MaskToIndices(col_.validity.slice(0, 0, col_.length))
                                    : at::arange(col_.length, ex.opts(at::kLong));
  const int64_t n = rows.numel();
  at::Tensor img = ex.empty_i64(std::max<int64_t>(n, 1));
  if (n) KCALL(ex, sort_keys_from_column, col_.view(), ptr<int64_t>(rows), n, false, reinterpret_cast<uint64_t *>(ptr<int64_t>(img)));
  img = img.slice(0, 0, n);
  auto sorted = ops::RadixSortPairs(ex, img.contiguous(), rows.contiguous(), 8 * col_.type.width());
  sorted_img_ = sorted.first;
  sorted_pos_ = sorted.second;
  trace::add_counter("index.built_rows", n);
}

at::Tensor SortedIndex::LabelImages(const Column &labels) const {
  Column l = as_index_type(labels, col_);
  Exec ex(col_.data.device());
  at::Tensor img = ex.empty_i64(std::max<int64_t>(l.length, 1));
  if (l.length) KCALL(ex, sort_keys_from_column, l.view(), nullptr, l.length, false, reinterpret_cast<uint64_t *>(ptr<int64_t>(img)));
  return img.slice(0, 0, l.length);  // null labels get a zero count after the probe
}

at::Tensor SortedIndex::GatherRuns(const at::Tensor &lo, const at::Tensor &cnt) const {
  Exec ex(col_.data.device());
  const int64_t m = lo.numel();
  at::Tensor offs = ops::exclusive_scan(ex, cnt);
  const int64_t total = ops::read_i64(offs, m);
  at::Tensor out = ex.empty_i64(std::max<int64_t>(total, 1));
  KCALL(ex, index_gather_positions, ptr<int64_t>(sorted_pos_), ptr<int64_t>(lo), ptr<int64_t>(cnt), ptr<int64_t>(offs), m,
        ptr<int64_t>(out));
  return out.slice(0, 0, total);
}

static void zero_null_labels(const Column &labels, at::Tensor &cnt) {
  if (labels.nullable()) cnt.mul_(labels.validity.slice(0, 0, labels.length).to(cnt.device()).ne(0).to(at::kLong));
}

at::Tensor SortedIndex::LocationsOf(const Column &labels) const {
  if (!persistent()) return LinearIndex::LocationsOf(labels);
  Exec ex(col_.data.device());
  CYLON_PHASE("index.lookup", ex.device);
  at::Tensor img = LabelImages(labels);
  const int64_t m = img.numel();
  at::Tensor lo = ex.empty_i64(std::max<int64_t>(m, 1)).slice(0, 0, m), cnt = ex.empty_i64(std::max<int64_t>(m, 1)).slice(0, 0, m);
  KCALL(ex, index_bounds, reinterpret_cast<const uint64_t *>(ptr<int64_t>(sorted_img_)), sorted_img_.numel(),
        reinterpret_cast<const uint64_t *>(ptr<int64_t>(img)), m, ptr<int64_t>(lo), ptr<int64_t>(cnt));
  zero_null_labels(labels, cnt);
  return GatherRuns(lo, cnt);
}

// ---- hash --------------------------------------------------------------------------
// byte-keyed columns (strings, binary, fixed-size binary): the run keys are 64-bit hashes of the
// values (row_hash64), sorted with their rows; a probe verifies the bytes of every candidate
static bool bytes_keyed(const Column &c) { return c.is_var() || c.type.kind() == ValueKind::FIXED_BYTES; }

HashIndex::HashIndex(std::shared_ptr<CylonContext> ctx, Column col)
    : SortedIndex(std::move(ctx), std::move(col), IndexingSchema::Hash) {
  Exec ex(col_.data.device());
  if (bytes_keyed(col_)) {
    CYLON_PHASE("index.build", ex.device);
    const int64_t n = col_.length;
    at::Tensor h = ex.empty_i64(std::max<int64_t>(n, 1));
    const ColView v = col_.view();
    if (n) KCALL(ex, row_hash64, &v, 1, n, reinterpret_cast<uint64_t *>(ptr<int64_t>(h)));
    at::Tensor rows = col_.nullable() ? ops::MaskToIndices(col_.validity.slice(0, 0, n))
                                      : at::arange(n, ex.opts(at::kLong));
    auto sorted = ops::RadixSortPairs(ex, h.slice(0, 0, n).index_select(0, rows).contiguous(), rows.contiguous(), 64);
    sorted_img_ = sorted.first;
    sorted_pos_ = sorted.second;
    bytes_ = true;
    trace::add_counter("index.built_rows", rows.numel());
  }
  if (!persistent()) return;
  const int64_t n = sorted_img_.numel();
  cap_ = 16;
  while (cap_ < 2 * std::max<int64_t>(n, 1)) cap_ <<= 1;  // >= 2 x distinct images
  tkeys_ = ex.empty_i64(cap_);
  used_ = at::zeros({cap_}, ex.opts(at::kInt));
  tlo_ = ex.empty_i64(cap_);
  tcnt_ = ex.empty_i64(cap_);
  KCALL(ex, hash_index_build, reinterpret_cast<const uint64_t *>(ptr<int64_t>(sorted_img_)), n,
        reinterpret_cast<uint64_t *>(ptr<int64_t>(tkeys_)), ptr<int32_t>(used_), ptr<int64_t>(tlo_), ptr<int64_t>(tcnt_),
        cap_);
}

at::Tensor HashIndex::LocationsOf(const Column &labels) const {
  if (!persistent()) return LinearIndex::LocationsOf(labels);
  Exec ex(col_.data.device());
  CYLON_PHASE("index.lookup", ex.device);
  const bool bytes = bytes_;
  Column lab = bytes ? labels.to(col_.data.device()) : Column();
  CYLON_CHECK(!bytes || bytes_keyed(lab), Code::TypeError, "a string / binary index needs string / binary labels");
  at::Tensor img;
  if (bytes) {
    img = ex.empty_i64(std::max<int64_t>(lab.length, 1));
    const ColView lv = lab.view();
    if (lab.length) KCALL(ex, row_hash64, &lv, 1, lab.length, reinterpret_cast<uint64_t *>(ptr<int64_t>(img)));
    img = img.slice(0, 0, lab.length);
  } else {
    img = LabelImages(labels);
  }
  const int64_t m = img.numel();
  at::Tensor lo = ex.empty_i64(std::max<int64_t>(m, 1)).slice(0, 0, m), cnt = ex.empty_i64(std::max<int64_t>(m, 1)).slice(0, 0, m);
  KCALL(ex, hash_index_probe, reinterpret_cast<const uint64_t *>(ptr<int64_t>(tkeys_)), ptr<int32_t>(used_),
        ptr<int64_t>(tlo_), ptr<int64_t>(tcnt_), cap_, reinterpret_cast<const uint64_t *>(ptr<int64_t>(img)), m,
        ptr<int64_t>(lo), ptr<int64_t>(cnt));
  zero_null_labels(labels, cnt);
  if (!bytes) return GatherRuns(lo, cnt);
  // candidates share the label's 64-bit hash: keep those whose bytes equal the label's
  at::Tensor cand = GatherRuns(lo, cnt);
  at::Tensor offs = ops::exclusive_scan(ex, cnt);
  at::Tensor keep = at::empty({std::max<int64_t>(cand.numel(), 1)}, ex.opts(at::kByte));
  const ColView cv = col_.view(), lv = lab.view();
  KCALL(ex, index_verify_bytes, cv, lv, ptr<int64_t>(sorted_pos_), ptr<int64_t>(lo), ptr<int64_t>(cnt),
        ptr<int64_t>(offs), m, keep.data_ptr<uint8_t>());
  const int64_t k = cand.numel();
  if (k == 0) return cand;
  return cand.index_select(0, ops::MaskToIndices(keep.slice(0, 0, k)));
}

std::shared_ptr<BaseIndex> BuildIndex(const TablePtr &t, int col, IndexingSchema schema) {
  auto ctx = t->GetContext();
  switch (schema) {
    case IndexingSchema::Range: return std::make_shared<RangeIndex>(0, t->Rows(), 1, t->device());
    case IndexingSchema::Linear: return std::make_shared<LinearIndex>(ctx, t->column(col));
    case IndexingSchema::Hash: return std::make_shared<HashIndex>(ctx, t->column(col));
    case IndexingSchema::BinaryTree:
    case IndexingSchema::BTree: return std::make_shared<SortedIndex>(ctx, t->column(col), schema);
  }
  CYLON_THROW(Code::Invalid, "unknown indexing schema " << static_cast<int>(schema));
}

// ---- indexers ------------------------------------------------------------------------
static TablePtr select_rows(const TablePtr &in, const at::Tensor &pos, const std::vector<int> &columns) {
  TablePtr t = columns.empty() ? in : ops::Project(in, columns);
  return ops::Gather(t, pos.to(t->device()));
}

std::shared_ptr<BaseIndex> LocIndexer::index_of(const TablePtr &in) const {
  if (in->GetIndex()) return in->GetIndex();
  return std::make_shared<RangeIndex>(0, in->Rows(), 1, in->device());
}

TablePtr LocIndexer::Loc(const TablePtr &in, const Column &values, const std::vector<int> &columns) const {
  return select_rows(in, index_of(in)->LocationsOf(values), columns);
}

TablePtr LocIndexer::LocRange(const TablePtr &in, const Column &start, const Column &end,
                              const std::vector<int> &columns) const {
  auto r = index_of(in)->RangeOf(start, end);
  CYLON_CHECK(r.first <= r.second, Code::KeyError, "index range is empty (start after end)");
  return ops::Slice(columns.empty() ? in : ops::Project(in, columns), r.first, r.second - r.first + 1);
}

TablePtr ILocIndexer::ILoc(const TablePtr &in, const at::Tensor &positions, const std::vector<int> &columns) const {
  at::Tensor p = positions.to(at::kLong);
  CYLON_CHECK(p.numel() == 0 || (p.min().item<int64_t>() >= 0 && p.max().item<int64_t>() < in->Rows()),
              Code::IndexError, "iloc position out of range");
  return select_rows(in, p, columns);
}

TablePtr ILocIndexer::ILocRange(const TablePtr &in, int64_t start, int64_t end, const std::vector<int> &columns) const {
  CYLON_CHECK(start >= 0 && end <= in->Rows() && start <= end, Code::IndexError, "iloc range out of bounds");
  return ops::Slice(columns.empty() ? in : ops::Project(in, columns), start, end - start);
}

}  // namespace indexing
}  // namespace cylon
