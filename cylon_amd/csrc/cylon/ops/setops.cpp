// Set operations, unique and distributed sample sort.
//
// Reference: cpp/src/cylon/table.cpp:531-721 (Union / Subtract / Intersect with a
// row-hash set over all columns, distinct semantics), :727-785 (distributed set
// ops = shuffle on all columns + local op), :923-999 (Unique / DistributedUnique),
// :338-382 (DistributedSort: range partition on the first sort column, split,
// all-to-all, local sort), arrow_partition_kernels.cpp:334-455 (RangePartitionKernel).
//
// Device plan: every set operation is a group-id computation (K8/K10 hash set or
// the exact sort path) over the concatenation L ++ R, followed by per-group
// presence flags (mark_indices over the L and R slices of the group-id vector)
// and one gather of the selected first-occurrence rows.  Output keeps the input
// order of the surviving rows (first occurrences ascend).
#include <cmath>
#include <limits>

#include "relational.hpp"
#include "util.hpp"

namespace cylon {
namespace ops {

static std::vector<int> all_cols(const TablePtr &t) {
  std::vector<int> c(t->Columns());
  for (int i = 0; i < t->Columns(); ++i) c[i] = i;
  return c;
}

static void verify_schema(const TablePtr &l, const TablePtr &r) {
  CYLON_CHECK(same_schema(l, r), Code::Invalid, "set operation: tables must have the same schema");
}

TablePtr Unique(const TablePtr &t, const std::vector<int> &cols, bool keep_first) {
  if (t->Rows() == 0) return t;
  Exec ex(t->device());
  GroupInfo gi = GroupIds(t, cols.empty() ? all_cols(t) : cols);
  at::Tensor keep = gi.first_rows;
  if (!keep_first) {  // last occurrence: per-group max row id
    at::Tensor rows = ex.empty_i64(t->Rows());
    KCALL(ex, iota, ptr<int64_t>(rows), t->Rows(), 0);
    Column rc("r", DataType(Type::INT64), t->Rows(), rows);
    at::Tensor img = at::zeros({gi.ngroups}, ex.opts(at::kLong));
    KCALL(ex, agg_accumulate, ptr<int64_t>(gi.gid), t->Rows(), gi.ngroups, rc.view(), 3, img.data_ptr(), nullptr);
    at::Tensor last = at::bitwise_xor(img, at::full({1}, std::numeric_limits<int64_t>::min(), img.options()));
    keep = RadixSortPairs(ex, last.contiguous(), last.clone(), 64).first;
  }
  return GatherNullable(t, keep, false);
}

TablePtr DistributedUnique(const TablePtr &t, const std::vector<int> &cols, bool keep_first) {
  auto ctx = t->GetContext();
  const std::vector<int> c = cols.empty() ? all_cols(t) : cols;
  if (ctx->GetWorldSize() == 1) return Unique(t, c, keep_first);
  return Unique(Shuffle(t, c), c, keep_first);
}

enum class SetOp { UNION, SUBTRACT, INTERSECT };

static TablePtr set_op(const TablePtr &l, const TablePtr &r, SetOp op) {
  verify_schema(l, r);
  TablePtr m = Merge({l, r});
  if (m->Rows() == 0) return m;
  Exec ex(m->device());
  GroupInfo gi = GroupIds(m, all_cols(m));
  const int64_t nl = l->Rows(), nr = r->Rows();
  if (op == SetOp::UNION) return GatherNullable(m, gi.first_rows, false);
  at::Tensor in_l = ex.zeros_u8(gi.ngroups), in_r = ex.zeros_u8(gi.ngroups);
  KCALL(ex, mark_indices, ptr<int64_t>(gi.gid), nl, ptr<uint8_t>(in_l));
  if (nr) KCALL(ex, mark_indices, ptr<int64_t>(gi.gid) + nl, nr, ptr<uint8_t>(in_r));
  at::Tensor sel = (op == SetOp::SUBTRACT) ? (in_l.gt(0) & in_r.eq(0)) : (in_l.gt(0) & in_r.gt(0));
  at::Tensor groups = MaskToIndices(sel.to(at::kByte));
  at::Tensor rows = gi.first_rows.index_select(0, groups);
  return GatherNullable(m, rows, false);
}

TablePtr Union(const TablePtr &l, const TablePtr &r) { return set_op(l, r, SetOp::UNION); }
TablePtr Subtract(const TablePtr &l, const TablePtr &r) { return set_op(l, r, SetOp::SUBTRACT); }
TablePtr Intersect(const TablePtr &l, const TablePtr &r) { return set_op(l, r, SetOp::INTERSECT); }

static TablePtr dist_set_op(const TablePtr &l, const TablePtr &r, SetOp op) {
  verify_schema(l, r);
  auto ctx = l->GetContext();
  if (ctx->GetWorldSize() == 1) return set_op(l, r, op);
  const auto cols = all_cols(l);
  auto lr = ShufflePair(l, cols, r, cols);
  return set_op(lr.first, lr.second, op);
}

TablePtr DistributedUnion(const TablePtr &l, const TablePtr &r) { return dist_set_op(l, r, SetOp::UNION); }
TablePtr DistributedSubtract(const TablePtr &l, const TablePtr &r) { return dist_set_op(l, r, SetOp::SUBTRACT); }
TablePtr DistributedIntersect(const TablePtr &l, const TablePtr &r) { return dist_set_op(l, r, SetOp::INTERSECT); }

// ---------------------------------------------------------------------------
// K13 range partition + sample sort
// ---------------------------------------------------------------------------
std::pair<at::Tensor, std::vector<int64_t>> MapToSortPartitions(const TablePtr &t, int col, uint32_t nparts,
                                                                bool ascending, uint64_t num_samples,
                                                                uint32_t num_bins) {
  auto ctx = t->GetContext();
  const bool dist = ctx->GetWorldSize() > 1;
  auto comm = ctx->GetCommunicator();
  Exec ex(t->device());
  const Column &c = t->column(col);
  CYLON_CHECK(c.type.is_numeric(), Code::NotImplemented, "range partition needs a numeric column");
  const int64_t n = t->Rows();
  if (num_bins == 0) num_bins = 16 * nparts;                                            // partition.cpp:181-182
  if (num_samples == 0) num_samples = std::max<uint64_t>(1, (uint64_t)std::ceil(0.01 * (double)n));
  if (num_samples > (uint64_t)n) num_samples = n;
  // sample (uniform with replacement; the reference uses mt19937 per chunk)
  at::Tensor sample_idx;
  if ((int64_t)num_samples == n) {
    sample_idx = ex.empty_i64(n);
    KCALL(ex, iota, ptr<int64_t>(sample_idx), n, 0);
  } else {
    sample_idx = at::randint(0, std::max<int64_t>(n, 1), {(int64_t)num_samples}, ex.opts(at::kLong));
  }
  // min/max of the sample (global)
  at::Tensor mm = at::empty({2}, ex.opts(at::kDouble));
  KCALL(ex, range_minmax, c.view(), ptr<int64_t>(sample_idx), (int64_t)sample_idx.numel(), ptr<double>(mm));
  if (dist) {
    at::Tensor lo = mm.slice(0, 0, 1).clone(), hi = mm.slice(0, 1, 2).clone();
    comm->AllReduce(lo, net::ReduceOp::MIN);
    comm->AllReduce(hi, net::ReduceOp::MAX);
    mm = at::cat({lo, hi});
  }
  at::Tensor mmh = mm.to(at::kCPU);
  const double vmin = mmh[0].item<double>(), vmax = mmh[1].item<double>();
  // histogram of the sample over num_bins + 2 bins (global)
  at::Tensor hist = at::zeros({(int64_t)num_bins + 2}, ex.opts(at::kLong));
  KCALL(ex, range_histogram, c.view(), ptr<int64_t>(sample_idx), (int64_t)sample_idx.numel(), vmin, vmax,
        (int64_t)num_bins, ptr<int64_t>(hist));
  if (dist) comm->AllReduce(hist, net::ReduceOp::SUM);
  std::vector<int64_t> h = to_host_vec(hist);
  // quantile walk bins -> partitions (arrow_partition_kernels.cpp:418-435)
  int64_t total = 0;
  for (auto x : h) total += x;
  std::vector<uint32_t> b2p;
  const double quantile = 1.0 / nparts;
  double prefix = 0, target = quantile;
  uint32_t cur = 0;
  for (auto x : h) {
    b2p.push_back(cur);
    prefix += total ? (double)x / (double)total : 0.0;
    if (prefix > target) {
      cur += (cur < nparts - 1);
      target += quantile;
    }
  }
  at::Tensor b2p_t = at::from_blob(b2p.data(), {(int64_t)b2p.size()}, at::TensorOptions().dtype(at::kInt)).to(ex.device);
  at::Tensor pid = ex.empty_u32(n);
  at::Tensor counts = at::zeros({(int64_t)nparts}, ex.opts(at::kLong));
  KCALL(ex, range_partition, c.view(), n, vmin, vmax, (int64_t)num_bins,
        reinterpret_cast<const uint32_t *>(b2p_t.data_ptr()), nparts, !ascending, ptr<uint32_t>(pid),
        ptr<int64_t>(counts));
  return {pid, to_host_vec(counts)};
}

TablePtr DistributedSort(const TablePtr &t, const std::vector<int> &cols, const std::vector<bool> &ascending,
                         const SortOptions &opts) {
  auto ctx = t->GetContext();
  const int world = ctx->GetWorldSize();
  if (world == 1) return Sort(t, cols, ascending);
  CYLON_CHECK(!cols.empty(), Code::Invalid, "sort needs at least one column");
  const bool asc0 = ascending.empty() ? true : ascending[0];
  auto pm = MapToSortPartitions(t, cols[0], (uint32_t)world, asc0, opts.num_samples, opts.num_bins);
  auto reordered = PartitionReorder(t, pm.first, (uint32_t)world);
  TablePtr recv = AllToAllTable(reordered.first, reordered.second);
  return Sort(recv, cols, ascending);
}

}  // namespace ops
}  // namespace cylon
