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
#include <algorithm>
#include <cmath>
#include <limits>

#include "relational.hpp"
#include "../trace.hpp"
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

// ---------------------------------------------------------------------------
// K10 LDS radix distinct (radix_setops.hip): device path of union / subtract /
// intersect / unique for large inputs.  The surviving rows keep the reference's
// order (ascending row ids, left before right).  Returns nullptr when not
// eligible or when the kernel reports an LDS overflow / hash collision (the
// exact sort-based path then runs).
// ---------------------------------------------------------------------------
enum class SetOp { UNION, SUBTRACT, INTERSECT };

static int64_t radix_setop_min_rows() {
  const char *e = std::getenv("CYLON_RADIX_SETOP_MIN_ROWS");  // tuning / test knob
  return e ? std::atoll(e) : (int64_t(1) << 20);
}

// rows il of l followed by rows ir of r in one table (fixed-width columns: one
// output allocation, two gather launches)
static TablePtr gather_two(const TablePtr &l, const at::Tensor &il, const TablePtr &r, const at::Tensor &ir) {
  bool fixed = true;
  for (const auto &c : l->columns()) fixed &= !c.is_var();
  if (!fixed) return Merge({GatherNullable(l, il, false), GatherNullable(r, ir, false)});
  Exec ex(l->device());
  const int64_t kl = il.numel(), kr = ir.numel();
  std::vector<Column> out;
  std::vector<ColView> lin, rin;
  std::vector<MutColView> lo, ro;
  for (int c = 0; c < l->Columns(); ++c) {
    const Column &a = l->column(c), &b = r->column(c);
    Column o = make_fixed_column(a.name, a.type, kl + kr, ex.device, a.nullable() || b.nullable());
    MutColView m;
    m.data = kl + kr ? reinterpret_cast<uint8_t *>(o.data.data_ptr()) : nullptr;
    m.valid = o.validity.defined() ? ptr<uint8_t>(o.validity) : nullptr;
    m.width = a.type.width();
    m.kind = static_cast<int>(a.type.kind());
    lo.push_back(m);
    if (m.data) m.data += kl * m.width;
    if (m.valid) m.valid += kl;
    ro.push_back(m);
    lin.push_back(a.view());
    rin.push_back(b.view());
    out.push_back(std::move(o));
  }
  if (kl) KCALL(ex, gather_columns, lin.data(), lo.data(), (int)lin.size(), ptr<int64_t>(il), kl);
  if (kr) KCALL(ex, gather_columns, rin.data(), ro.data(), (int)rin.size(), ptr<int64_t>(ir), kr);
  return Table::Make(l->GetContext(), std::move(out));
}

static TablePtr radix_distinct(const TablePtr &l, const TablePtr &r, const std::vector<int> &cols, SetOp op,
                               bool keep_last) {
  if (!l->device().is_cuda()) return nullptr;
  const int64_t nl = l->Rows(), nr = r ? r->Rows() : 0, n = nl + nr;
  const int ncols = (int)cols.size();
  if (n < radix_setop_min_rows() || ncols < 1 || ncols > kMaxFusedCols) return nullptr;
  Exec ex(l->device());
  CYLON_PHASE("setop.radix", ex.device);
  std::vector<ColView> lv = views(l, cols), rv = r ? views(r, cols) : lv;
  at::Tensor h = ex.empty_i64(n), rid = ex.empty_i64(n);
  hip::setop_row_hash(lv.data(), ncols, nl, 0, reinterpret_cast<uint64_t *>(ptr<int64_t>(h)), ptr<int64_t>(rid),
                      ex.stream);
  if (nr) hip::setop_row_hash(rv.data(), ncols, nr, nl, reinterpret_cast<uint64_t *>(ptr<int64_t>(h)),
                              ptr<int64_t>(rid), ex.stream);
  int bits = 0;
  while ((n >> bits) > hip::setop_rows_per_part()) ++bits;
  at::Tensor offs;
  std::vector<at::Tensor> pr = RadixPartition(ex, {h, rid}, {8, 8}, bits, &offs);
  h = rid = at::Tensor();
  const int opi = op == SetOp::UNION ? 0 : (op == SetOp::SUBTRACT ? 1 : 2);
  const int64_t mlen = op == SetOp::UNION ? n : nl;
  at::Tensor mask = op == SetOp::INTERSECT ? ex.zeros_u8(mlen) : at::ones({mlen}, ex.opts(at::kByte));
  at::Tensor exc = ex.empty_i64(1);
  at::Tensor bad = at::empty({1}, ex.opts(at::kInt));
  hip::setop_dedup(reinterpret_cast<const uint64_t *>(ptr<int64_t>(pr[0])), ptr<int64_t>(pr[1]), ptr<int64_t>(offs),
                   int64_t(1) << bits, nl, opi, keep_last, lv.data(), r ? rv.data() : nullptr, ncols,
                   ptr<uint8_t>(mask), ptr<int64_t>(exc), bad.data_ptr<int>(), ex.stream);
  pr.clear();
  if (bad.item<int>() != 0) {
    trace::add_counter("setop.radix.fallback", 1);
    return nullptr;
  }
  const int64_t e = exc.item<int64_t>();
  trace::add_counter("setop.radix.exceptions", e);
  if (op == SetOp::UNION && e == 0) return r ? Merge({l, r}) : Slice(l, 0, nl);  // every row distinct
  if (op == SetOp::SUBTRACT && e == 0) return Slice(l, 0, nl);
  if (!r || op != SetOp::UNION) return GatherNullable(l, MaskToIndices(mask), false);
  return gather_two(l, MaskToIndices(mask.slice(0, 0, nl)), r, MaskToIndices(mask.slice(0, nl, n)));
}

TablePtr Unique(const TablePtr &t, const std::vector<int> &cols, bool keep_first) {
  if (t->Rows() == 0) return t;
  if (TablePtr out = radix_distinct(t, nullptr, cols.empty() ? all_cols(t) : cols, SetOp::UNION, !keep_first))
    return out;
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

static TablePtr set_op(const TablePtr &l, const TablePtr &r, SetOp op) {
  verify_schema(l, r);
  if (TablePtr out = radix_distinct(l, r, all_cols(l), op, false)) return out;
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
  const int K = ShuffleChunks(l, r);
  if (K > 1) {  // chunk k's local set operation overlaps the transfer of the later chunks
    std::vector<TablePtr> parts;
    ShufflePairChunked(l, cols, r, cols, K,
                       [&](int, const TablePtr &a, const TablePtr &b) { parts.push_back(set_op(a, b, op)); });
    return Merge(parts);
  }
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

// Exact sample-sort splitters (DistributedSort).  Every row gets the composite key
// (null_0, image_0, ..., null_K-1, image_K-1, gid) over ALL sort columns -- order
// images are the local sort's uint64 keys (direction applied, NaN last), nulls sort
// last, gid = the row's global number -- so keys are distinct and totally ordered
// exactly like the final order.  A random sample of each rank's keys is all-gathered,
// sorted on the host and cut at W-1 equal-count positions; rows are then assigned by
// binary search over these splitters.  Unlike the reference's equal-width bins over
// a double [min, max] (table.cpp:338-382, arrow_partition_kernels.cpp:334-455), no
// precision is lost for int64 keys, and equal keys may straddle ranks in gid order,
// so heavy skew (even a single repeated key) still splits evenly.  The local sort
// after the exchange is stable and receives pieces in rank order, which keeps equal
// keys in gid order: the distributed sort is globally stable.
static bool splitter_sort_eligible(const TablePtr &t, const std::vector<int> &cols, int world) {
  if (cols.empty() || cols.size() > 4 || world > 1024) return false;
  for (int c : cols) {
    const Column &col = t->column(c);
    if (col.is_var() || col.type.kind() == ValueKind::FIXED_BYTES || !col.type.is_numeric()) return false;
  }
  return true;
}

static TablePtr splitter_sort(const TablePtr &t, const std::vector<int> &cols, const std::vector<bool> &ascending,
                              const SortOptions &opts) {
  auto ctx = t->GetContext();
  auto comm = ctx->GetCommunicator();
  const int W = ctx->GetWorldSize();
  const int K = (int)cols.size();
  const int stride = 2 * K + 1;
  Exec ex(t->device());
  const int64_t n = t->Rows();
  std::vector<at::Tensor> imgs(K), nuls(K);
  std::vector<const uint64_t *> ip(K);
  std::vector<const uint8_t *> np(K, nullptr);
  {
    CYLON_PHASE("sort.dist.images", ex.device);
    for (int k = 0; k < K; ++k) {
      const Column &c = t->column(cols[k]);
      const bool asc = ascending.empty() ? true : (ascending.size() == 1 ? ascending[0] : ascending[k]);
      imgs[k] = ex.empty_i64(std::max<int64_t>(n, 1));
      if (n) KCALL(ex, sort_keys_from_column, c.view(), nullptr, n, !asc, reinterpret_cast<uint64_t *>(ptr<int64_t>(imgs[k])));
      ip[k] = reinterpret_cast<const uint64_t *>(imgs[k].data_ptr());
      if (c.nullable()) {
        nuls[k] = c.validity.slice(0, 0, n).eq(0).to(at::kByte).contiguous();
        np[k] = nuls[k].numel() ? nuls[k].data_ptr<uint8_t>() : nullptr;
      }
    }
  }
  // global row numbers: rank r's rows are gid0 .. gid0 + n - 1
  at::Tensor ns = comm->AllGather(at::full({1}, n, ex.opts(at::kLong))).to(at::kCPU);
  int64_t gid0 = 0;
  for (int r = 0; r < ctx->GetRank(); ++r) gid0 += ns[r].item<int64_t>();
  // sample -> all-gather -> host sort -> W-1 splitters
  const int64_t per = std::min<int64_t>(n, opts.num_samples ? (int64_t)opts.num_samples : 256 * (int64_t)W);
  at::Tensor idx = per == n ? at::arange(n, ex.opts(at::kLong))
                            : at::randint(0, std::max<int64_t>(n, 1), {per}, ex.opts(at::kLong));
  at::Tensor sample = at::empty({per, stride}, ex.opts(at::kLong));
  for (int k = 0; k < K; ++k) {
    sample.select(1, 2 * k).copy_(nuls[k].defined() ? nuls[k].index_select(0, idx).to(at::kLong)
                                                    : at::zeros({per}, ex.opts(at::kLong)));
    sample.select(1, 2 * k + 1).copy_(imgs[k].slice(0, 0, std::max<int64_t>(n, 1)).index_select(0, idx));
  }
  sample.select(1, 2 * K).copy_(idx + gid0);
  std::vector<at::Tensor> parts = comm->AllGatherV(sample.reshape({-1}));
  at::Tensor all = at::cat(parts).to(at::kCPU).contiguous();
  const int64_t S = all.numel() / stride;
  const uint64_t *sw = reinterpret_cast<const uint64_t *>(all.data_ptr<int64_t>());
  std::vector<int64_t> order(S);
  for (int64_t i = 0; i < S; ++i) order[i] = i;
  std::sort(order.begin(), order.end(), [&](int64_t a, int64_t b) {
    return std::lexicographical_compare(sw + a * stride, sw + (a + 1) * stride, sw + b * stride, sw + (b + 1) * stride);
  });
  std::vector<uint64_t> spl((size_t)(W - 1) * stride, ~0ull);
  for (int i = 0; i + 1 < W && S > 0; ++i) {
    const int64_t at_ = std::min<int64_t>(S - 1, (int64_t)(i + 1) * S / W);
    std::copy(sw + order[at_] * stride, sw + (order[at_] + 1) * stride, spl.begin() + (size_t)i * stride);
  }
  at::Tensor spl_t = at::from_blob(spl.data(), {(int64_t)spl.size()}, at::TensorOptions().dtype(at::kLong))
                         .to(ex.device)
                         .contiguous();
  at::Tensor pid = ex.empty_u32(std::max<int64_t>(n, 1));
  at::Tensor counts = at::zeros({W}, ex.opts(at::kLong));
  {
    CYLON_PHASE("sort.dist.partition", ex.device);
    KCALL(ex, splitter_partition, ip.data(), np.data(), K, n, gid0,
          reinterpret_cast<const uint64_t *>(ptr<int64_t>(spl_t)), (uint32_t)W, ptr<uint32_t>(pid),
          ptr<int64_t>(counts));
  }
  trace::add_counter("sort.dist.splitter_partitions", 1);
  auto reordered = PartitionReorder(t, pid.slice(0, 0, n), (uint32_t)W);
  TablePtr recv;
  {
    CYLON_PHASE("sort.dist.exchange", ex.device);
    recv = AllToAllTable(reordered.first, reordered.second);
  }
  return Sort(recv, cols, ascending);
}

TablePtr DistributedSort(const TablePtr &t, const std::vector<int> &cols, const std::vector<bool> &ascending,
                         const SortOptions &opts) {
  auto ctx = t->GetContext();
  const int world = ctx->GetWorldSize();
  if (world == 1) return Sort(t, cols, ascending);
  CYLON_CHECK(!cols.empty(), Code::Invalid, "sort needs at least one column");
  if (splitter_sort_eligible(t, cols, world)) return splitter_sort(t, cols, ascending, opts);
  // string / binary first column etc.: the reference's histogram partition on the first column
  const bool asc0 = ascending.empty() ? true : ascending[0];
  auto pm = MapToSortPartitions(t, cols[0], (uint32_t)world, asc0, opts.num_samples, opts.num_bins);
  auto reordered = PartitionReorder(t, pm.first, (uint32_t)world);
  TablePtr recv = AllToAllTable(reordered.first, reordered.second);
  return Sort(recv, cols, ascending);
}

}  // namespace ops
}  // namespace cylon
