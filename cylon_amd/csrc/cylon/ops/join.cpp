// Join (L3 local + L4 distributed).
//
// Reference: cpp/src/cylon/join/join.cpp:29-100 (JoinTables dispatch),
// hash_join.cpp:188-346, sort_join.cpp:576-722, join_utils.cpp:126-181
// (build_final_table: left columns ++ right columns, prefixed names, index -1
// -> null), table.cpp:428-502 (Join / DistributedJoin).
//
// Device plan for one local join:
//   1. key encoding: a single non-null fixed-width key column is used as-is
//      (int64 zero-copy, narrower types sign/zero-extended); otherwise a 64-bit
//      row hash over the key columns + a rows_equal confirmation pass.
//   2. hash: build the smaller side into the open-addressing multimap, probe
//      the other side (count, scan, write).
//      sort: radix-sort (key, row) of both sides and expand equal ranges
//      (sort_join.cpp).
//   3. outer completion: matched flags (mark_indices) + compaction of the
//      unmatched rows of the preserved side(s), appended with -1 partners.
//   4. materialisation: one fused gather launch per side (K4).
#include "util.hpp"
#include "../trace.hpp"

namespace cylon {
namespace ops {

using join::config::JoinAlgorithm;
using join::config::JoinConfig;
using join::config::JoinType;

// defined in sort_join.cpp
std::pair<at::Tensor, at::Tensor> SortJoinPairs(const Exec &ex, const at::Tensor &lkeys, const at::Tensor &rkeys);

static int64_t next_pow2(int64_t v) {
  int64_t p = 1;
  while (p < v) p <<= 1;
  return p;
}

struct KeyEncoding {
  at::Tensor keys;   // int64 per row
  bool exact;        // keys equal <=> rows equal
};

static bool simple_key(const Column &c) {
  return !c.nullable() && !c.is_var() && c.type.kind() != ValueKind::FIXED_BYTES && c.type.width() <= 8;
}

static KeyEncoding encode_keys(const Exec &ex, const TablePtr &t, const std::vector<int> &cols, bool exact_ok) {
  const int64_t n = t->Rows();
  if (exact_ok) {
    const Column &c = t->column(cols[0]);
    if (c.type.width() == 8 && c.type.kind() == ValueKind::SIGNED_INT) return {c.data.view(at::kLong), true};
    at::Tensor k = ex.empty_i64(n);
    KCALL(ex, key64_from_column, c.view(), n, ptr<int64_t>(k));
    return {k, true};
  }
  std::vector<ColView> v = views(t, cols);
  at::Tensor k = ex.empty_i64(n);
  KCALL(ex, row_hash64, v.data(), (int)v.size(), n, reinterpret_cast<uint64_t *>(ptr<int64_t>(k)));
  return {k, false};
}

// Build sides at least this large use the atomic-free sorted build (random
// 64-bit CAS into a table far beyond the caches runs at the memory-side atomic
// rate: 213 ms for 1B keys, profiles/); probe sides this large use the
// single-pass probe.
static constexpr int64_t kSortedBuildRows = int64_t(1) << 20;
static constexpr int64_t kEmitProbeRows = int64_t(1) << 22;

// inner-join index pairs on int64 keys via the K5 hash table (build = smaller side)
static std::pair<at::Tensor, at::Tensor> hash_join_pairs(const Exec &ex, const at::Tensor &lk, const at::Tensor &rk) {
  const bool build_left = lk.numel() < rk.numel();
  const at::Tensor &bk = build_left ? lk : rk;
  const at::Tensor &pk = build_left ? rk : lk;
  const int64_t nb = bk.numel(), np = pk.numel();
  const int64_t cap = next_pow2(std::max<int64_t>(2 * nb, 64));
  const int shift = 64 - __builtin_ctzll((unsigned long long)cap);
  at::Tensor table;
  HashTableRef t{nullptr, cap, shift};
  if (ex.gpu && nb >= kSortedBuildRows) {
    CYLON_PHASE("join.build.sorted", ex.device);
    // atomic-free build: radix sort (key,row) by slot, prefix-max placement, sequential stores
    at::Tensor ka = ex.empty_i64(nb), va = ex.empty_i64(nb), kb = ex.empty_i64(nb), vb = ex.empty_i64(nb);
    at::Tensor mp = ex.empty_i64(1);
    at::Tensor ws = ex.empty_i64(KSIZE(ex, hash_build_sorted_workspace, nb));
    const int which = KCALL(ex, hash_build_sorted, ptr<int64_t>(bk), nb, shift, ptr<int64_t>(ws),
                            reinterpret_cast<uint64_t *>(ptr<int64_t>(ka)), ptr<int64_t>(va),
                            reinterpret_cast<uint64_t *>(ptr<int64_t>(kb)), ptr<int64_t>(vb), ptr<int64_t>(mp));
    ws = at::Tensor();
    const int64_t maxpos = read_i64(mp, 0) + nb - 1;
    t.tsize = std::max<int64_t>(cap, maxpos + 2);
    table = at::empty({t.tsize * 2}, ex.opts(at::kLong));  // HashSlot = 2 x int64
    t.slots = reinterpret_cast<HashSlot *>(table.data_ptr());
    KCALL(ex, hash_table_init, t.slots, t.tsize);
    const at::Tensor &sk = which ? kb : ka;
    const at::Tensor &sr = which ? vb : va;
    const at::Tensor &pm = which ? ka : kb;
    KCALL(ex, hash_table_place, reinterpret_cast<const uint64_t *>(ptr<int64_t>(sk)), ptr<int64_t>(sr),
          ptr<int64_t>(pm), nb, t);
  } else {
    table = at::empty({cap * 2}, ex.opts(at::kLong));
    t.slots = reinterpret_cast<HashSlot *>(table.data_ptr());
    KCALL(ex, hash_table_init, t.slots, cap);
    KCALL(ex, hash_build, ptr<int64_t>(bk), nb, t);
  }
  if (ex.gpu && np >= kEmitProbeRows) {
    CYLON_PHASE("join.probe.emit", ex.device);
    // single-pass probe into an over-allocated pair buffer; exact two-pass fallback on overflow
    const int64_t capacity = np + np / 4 + 4096;
    at::Tensor po = ex.empty_i64(capacity), bo = ex.empty_i64(capacity), cnt = ex.empty_i64(1);
    KCALL(ex, hash_probe_emit, ptr<int64_t>(pk), np, t, capacity, ptr<int64_t>(cnt), ptr<int64_t>(po),
          ptr<int64_t>(bo));
    const int64_t m = read_i64(cnt, 0);
    if (m <= capacity) {
      po = po.slice(0, 0, m);
      bo = bo.slice(0, 0, m);
      return build_left ? std::make_pair(bo, po) : std::make_pair(po, bo);
    }
  }
  CYLON_PHASE("join.probe.twopass", ex.device);
  at::Tensor counts = ex.empty_i64(np);
  KCALL(ex, hash_probe_count, ptr<int64_t>(pk), np, t, ptr<int64_t>(counts));
  at::Tensor offs = exclusive_scan(ex, counts);
  counts = at::Tensor();
  const int64_t m = read_i64(offs, np);
  at::Tensor po = ex.empty_i64(m), bo = ex.empty_i64(m);
  KCALL(ex, hash_probe_write, ptr<int64_t>(pk), np, t, ptr<int64_t>(offs), ptr<int64_t>(po), ptr<int64_t>(bo));
  return build_left ? std::make_pair(bo, po) : std::make_pair(po, bo);
}

static std::pair<at::Tensor, at::Tensor> join_impl(TablePtr left, TablePtr right, const JoinConfig &cfg,
                                                   bool allow_reorder, TablePtr *lout, TablePtr *rout);

std::pair<at::Tensor, at::Tensor> JoinIndices(const TablePtr &left, const TablePtr &right, const JoinConfig &cfg) {
  return join_impl(left, right, cfg, false, nullptr, nullptr);
}

static std::pair<at::Tensor, at::Tensor> join_impl(TablePtr left, TablePtr right, const JoinConfig &cfg,
                                                   bool allow_reorder, TablePtr *lout, TablePtr *rout) {
  const auto &lc = cfg.GetLeftColumnIdx();
  const auto &rc = cfg.GetRightColumnIdx();
  CYLON_CHECK(lc.size() == rc.size(), Code::Invalid, "left/right key counts differ");
  CYLON_CHECK(left->device() == right->device(), Code::Invalid, "join inputs on different devices");
  for (size_t i = 0; i < lc.size(); ++i) {
    const auto &a = left->column(lc[i]).type;
    const auto &b = right->column(rc[i]).type;
    const bool both_int = a.kind() != ValueKind::FLOAT && b.kind() != ValueKind::FLOAT && a.width() <= 8 &&
                          b.width() <= 8 && !a.is_variable_width() && !b.is_variable_width() &&
                          a.kind() != ValueKind::FIXED_BYTES && b.kind() != ValueKind::FIXED_BYTES;
    CYLON_CHECK(a == b || both_int, Code::TypeError,
                "join key types differ: " << a.ToString() << " vs " << b.ToString());
  }
  Exec ex(left->device());
  const bool exact = lc.size() == 1 && simple_key(left->column(lc[0])) && simple_key(right->column(rc[0])) &&
                     left->column(lc[0]).type == right->column(rc[0]).type;
  KeyEncoding lk = encode_keys(ex, left, lc, exact);
  KeyEncoding rk = encode_keys(ex, right, rc, exact);
  (void)allow_reorder;  // hook for input reordering strategies (none profitable so far, see docs)
  if (lout) *lout = left;
  if (rout) *rout = right;

  std::pair<at::Tensor, at::Tensor> pr;
  if (cfg.GetAlgorithm() == JoinAlgorithm::SORT)
    pr = SortJoinPairs(ex, lk.keys, rk.keys);
  else
    pr = hash_join_pairs(ex, lk.keys, rk.keys);
  at::Tensor li = pr.first, ri = pr.second;

  if (!exact && li.numel() > 0) {  // confirm hash candidates
    std::vector<ColView> lv = views(left, lc), rv = views(right, rc);
    at::Tensor eq = ex.empty_u8(li.numel());
    KCALL(ex, rows_equal, lv.data(), rv.data(), (int)lv.size(), ptr<int64_t>(li), ptr<int64_t>(ri), li.numel(),
          ptr<uint8_t>(eq));
    at::Tensor keep = MaskToIndices(eq);
    if (keep.numel() != li.numel()) {
      li = li.index_select(0, keep);
      ri = ri.index_select(0, keep);
    }
  }

  const JoinType jt = cfg.GetType();
  std::vector<at::Tensor> lparts{li}, rparts{ri};
  if (jt == JoinType::LEFT || jt == JoinType::FULL_OUTER) {
    at::Tensor matched = ex.zeros_u8(left->Rows());
    KCALL(ex, mark_indices, ptr<int64_t>(li), li.numel(), ptr<uint8_t>(matched));
    at::Tensor um = MaskToIndices(matched, true);
    lparts.push_back(um);
    rparts.push_back(at::full({um.numel()}, -1, ex.opts(at::kLong)));
  }
  if (jt == JoinType::RIGHT || jt == JoinType::FULL_OUTER) {
    at::Tensor matched = ex.zeros_u8(right->Rows());
    KCALL(ex, mark_indices, ptr<int64_t>(ri), ri.numel(), ptr<uint8_t>(matched));
    at::Tensor um = MaskToIndices(matched, true);
    rparts.push_back(um);
    lparts.push_back(at::full({um.numel()}, -1, ex.opts(at::kLong)));
  }
  if (lparts.size() > 1) {
    li = at::cat(lparts);
    ri = at::cat(rparts);
  }
  return {li, ri};
}

TablePtr Join(const TablePtr &left, const TablePtr &right, const JoinConfig &cfg) {
  TablePtr l = left, r = right;
  auto idx = join_impl(left, right, cfg, true, &l, &r);
  const JoinType jt = cfg.GetType();
  const bool lnull = jt == JoinType::RIGHT || jt == JoinType::FULL_OUTER;
  const bool rnull = jt == JoinType::LEFT || jt == JoinType::FULL_OUTER;
  CYLON_PHASE("join.materialize", l->device());
  TablePtr lo = GatherNullable(l, idx.first, lnull);
  TablePtr ro = GatherNullable(r, idx.second, rnull);
  std::vector<Column> cols;
  cols.reserve(lo->Columns() + ro->Columns());
  for (const auto &c : lo->columns()) cols.push_back(c.with_name(cfg.GetLeftTablePrefix() + c.name));
  for (const auto &c : ro->columns()) cols.push_back(c.with_name(cfg.GetRightTablePrefix() + c.name));
  return Table::Make(left->GetContext(), std::move(cols));
}

TablePtr DistributedJoin(const TablePtr &left, const TablePtr &right, const JoinConfig &cfg) {
  auto ctx = left->GetContext();
  if (ctx->GetWorldSize() == 1) return Join(left, right, cfg);
  TablePtr l = Shuffle(left, cfg.GetLeftColumnIdx());
  TablePtr r = Shuffle(right, cfg.GetRightColumnIdx());
  return Join(l, r, cfg);
}

}  // namespace ops
}  // namespace cylon
