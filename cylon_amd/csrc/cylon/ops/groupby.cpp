// Group-by (hash and pipeline), two-phase distributed group-by and scalar
// aggregates.
//
// Reference: cpp/src/cylon/groupby/groupby.cpp:24-137 (DistributedHashGroupBy:
// local combine only when every op is SUM/MIN/MAX, then shuffle + final),
// hash_groupby.cpp:92-320, pipeline_groupby.cpp:131-256,
// compute/aggregates.cpp:26-152 (Sum/Count/Min/Max + MPI_Allreduce).
//
// Differences by design (documented in docs/semantics.md):
//   * every decomposable op (SUM, COUNT, MIN, MAX, MEAN, VAR, STDDEV) is
//     combined locally before the shuffle through partial states
//     (count, sum, M2, sum^2/count), so only #local-groups rows cross xGMI;
//   * output names carry a single prefix (the reference double-prefixes in
//     its two-phase path);
//   * COUNT counts non-null values (identical to the reference on non-null data).
#include "cylon/knobs.hpp"
#include <algorithm>
#include <cstdlib>
#include <limits>

#include "relational.hpp"
#include "util.hpp"
#include "../trace.hpp"

namespace cylon {
namespace ops {

static int64_t next_pow2(int64_t v) {
  int64_t p = 1;
  while (p < v) p <<= 1;
  return p;
}

static bool simple_key(const Column &c) {
  return !c.nullable() && !c.is_var() && c.type.kind() != ValueKind::FIXED_BYTES && c.type.width() <= 8;
}

static at::Tensor iota_t(const Exec &ex, int64_t n) {
  at::Tensor p = ex.empty_i64(n);
  KCALL(ex, iota, ptr<int64_t>(p), n, 0);
  return p;
}

const char *AggPrefix(int op) {
  switch (op) {
    case AGG_SUM: return "sum_";
    case AGG_MIN: return "min_";
    case AGG_MAX: return "max_";
    case AGG_COUNT: return "count_";
    case AGG_MEAN: return "mean_";
    case AGG_VAR: return "var_";
    case AGG_NUNIQUE: return "nunique_";
    case AGG_QUANTILE: return "quantile_";
    case AGG_STDDEV: return "std_";
  }
  return "agg_";
}

GroupInfo GroupIds(const TablePtr &t, const std::vector<int> &cols, bool presorted) {
  Exec ex(t->device());
  const int64_t n = t->Rows();
  GroupInfo gi;
  if (n == 0) {
    gi.gid = ex.empty_i64(0);
    gi.first_rows = ex.empty_i64(0);
    return gi;
  }
  if (!presorted && cols.size() == 1 && simple_key(t->column(cols[0]))) {
    const Column &c = t->column(cols[0]);
    at::Tensor keys;
    if (c.type.width() == 8 && c.type.kind() == ValueKind::SIGNED_INT) {
      keys = c.data.view(at::kLong);
    } else {
      keys = ex.empty_i64(n);
      KCALL(ex, key64_from_column, c.view(), n, ptr<int64_t>(keys));
    }
    const int64_t cap = next_pow2(std::max<int64_t>(2 * n, 64));
    at::Tensor slot_keys = at::full({cap}, std::numeric_limits<int64_t>::min(), ex.opts(at::kLong));
    at::Tensor slot_first = at::full({cap + 1}, std::numeric_limits<int64_t>::max(), ex.opts(at::kLong));
    at::Tensor slot_of_row = ex.empty_i64(n);
    KCALL(ex, group_insert, ptr<int64_t>(keys), n, ptr<int64_t>(slot_keys), cap, ptr<int64_t>(slot_of_row),
          ptr<int64_t>(slot_first));
    at::Tensor flags = ex.zeros_u8(n);
    KCALL(ex, mark_firsts, ptr<int64_t>(slot_first), cap + 1, ptr<uint8_t>(flags));
    gi.first_rows = MaskToIndices(flags);
    gi.ngroups = gi.first_rows.numel();
    at::Tensor gid_at_row = ex.empty_i64(n);
    KCALL(ex, scatter_iota, ptr<int64_t>(gi.first_rows), gi.ngroups, ptr<int64_t>(gid_at_row));
    gi.gid = ex.empty_i64(n);
    KCALL(ex, gather_chain2, ptr<int64_t>(slot_of_row), ptr<int64_t>(slot_first), ptr<int64_t>(gid_at_row), n,
          ptr<int64_t>(gi.gid));
    return gi;
  }
  // exact sort-based path (multi-column, strings, nullable keys, presorted input)
  at::Tensor perm = presorted ? iota_t(ex, n) : SortIndices(t, cols, {true}, true);
  std::vector<ColView> v = views(t, cols);
  at::Tensor heads = ex.empty_u8(n);
  KCALL(ex, segment_heads, v.data(), (int)v.size(), ptr<int64_t>(perm), n, ptr<uint8_t>(heads));
  at::Tensor head_pos = MaskToIndices(heads);
  const int64_t nruns = head_pos.numel();
  at::Tensor incl = exclusive_scan(ex, heads.to(at::kLong)).slice(0, 1, n + 1) - 1;  // run of each sorted position
  at::Tensor first_unsorted = perm.index_select(0, head_pos);
  at::Tensor gid_of_run;
  if (presorted) {
    gid_of_run = iota_t(ex, nruns);
    gi.first_rows = first_unsorted;
  } else {
    auto s = RadixSortPairs(ex, first_unsorted.clone(), iota_t(ex, nruns), 64);
    gi.first_rows = s.first;
    gid_of_run = ex.empty_i64(nruns);
    KCALL(ex, scatter_iota, ptr<int64_t>(s.second), nruns, ptr<int64_t>(gid_of_run));
  }
  gi.ngroups = nruns;
  gi.gid = ex.empty_i64(n);
  KCALL(ex, permute_assign, ptr<int64_t>(perm), ptr<int64_t>(incl.contiguous()), ptr<int64_t>(gid_of_run), n,
        ptr<int64_t>(gi.gid));
  return gi;
}

// ---------------------------------------------------------------------------
// per-group accumulators
// ---------------------------------------------------------------------------
namespace {

constexpr int kSumF = 0, kSumI = 1, kMin = 2, kMax = 3, kCount = 4, kM2 = 5;

struct Acc {
  const Exec &ex;
  const at::Tensor &gid;  // may be undefined for a single group
  int64_t n, ng;

  const int64_t *g() const { return gid.defined() ? ptr<int64_t>(gid) : nullptr; }

  at::Tensor run(const Column &c, int kind, const at::Tensor &mean = at::Tensor()) const {
    at::Tensor acc;
    if (kind == kSumF || kind == kM2) acc = at::zeros({ng}, ex.opts(at::kDouble));
    else if (kind == kMin) acc = at::full({ng}, -1, ex.opts(at::kLong));
    else acc = at::zeros({ng}, ex.opts(at::kLong));
    KCALL(ex, agg_accumulate, g(), n, ng, c.view(), kind, acc.data_ptr(),
          mean.defined() ? ptr<double>(mean) : nullptr);
    return acc;
  }
};

Column double_col(const std::string &name, at::Tensor v, at::Tensor valid = at::Tensor()) {
  return Column(name, DataType(Type::DOUBLE), v.numel(), v.contiguous(),
                at::Tensor(), valid.defined() ? valid.to(at::kByte).contiguous() : at::Tensor());
}

Column long_col(const std::string &name, at::Tensor v, Type t = Type::INT64) {
  return Column(name, DataType(t), v.numel(), v.contiguous());
}

Column minmax_col(const Exec &ex, const std::string &name, const Column &c, const at::Tensor &img,
                  const at::Tensor &count) {
  const int64_t ng = img.numel();
  Column out = make_fixed_column(name, c.type, ng, ex.device, c.nullable());
  KCALL(ex, agg_unimage, reinterpret_cast<const uint64_t *>(ptr<int64_t>(img)), ng, c.type.width(),
        static_cast<int>(c.type.kind()), reinterpret_cast<uint8_t *>(out.data.data_ptr()));
  if (c.nullable()) out.validity = (count > 0).to(at::kByte);
  return out;
}

Column column_from(const std::string &name, const at::Tensor &t) {
  return Column(name, DataType(Type::INT64), t.numel(), t);
}

TablePtr values_by_group(const TablePtr &t, const at::Tensor &gid, const Column &val) {
  std::vector<Column> cols{column_from("g", gid), val};
  return Table::Make(t->GetContext(), std::move(cols));
}

}  // namespace

static Column agg_column(const Exec &ex, const TablePtr &t, const GroupInfo &gi, const AggSpec &a) {
  const Column &c = t->column(a.col);
  const std::string name = std::string(AggPrefix(a.op)) + c.name;
  Acc acc{ex, gi.gid, t->Rows(), gi.ngroups};
  const bool is_float = c.type.kind() == ValueKind::FLOAT;
  const bool numeric = c.type.is_numeric();
  if (a.op != AGG_COUNT && a.op != AGG_NUNIQUE)
    CYLON_CHECK(numeric, Code::TypeError, "aggregation " << AggPrefix(a.op) << " needs a numeric column, got "
                                                         << c.type.ToString());
  switch (a.op) {
    case AGG_SUM:
      if (is_float) return double_col(name, acc.run(c, kSumF));
      return long_col(name, acc.run(c, kSumI),
                      c.type.kind() == ValueKind::UNSIGNED_INT ? Type::UINT64 : Type::INT64);
    case AGG_COUNT: return long_col(name, acc.run(c, kCount));
    case AGG_MIN:
    case AGG_MAX: {
      at::Tensor img = acc.run(c, a.op == AGG_MIN ? kMin : kMax);
      at::Tensor cnt = c.nullable() ? acc.run(c, kCount) : at::Tensor();
      return minmax_col(ex, name, c, img, cnt);
    }
    case AGG_MEAN: {
      at::Tensor s = acc.run(c, kSumF), n = acc.run(c, kCount);
      return double_col(name, s / n.to(at::kDouble), n > 0);
    }
    case AGG_VAR:
    case AGG_STDDEV: {
      at::Tensor s = acc.run(c, kSumF), n = acc.run(c, kCount).to(at::kDouble);
      at::Tensor mean = (s / n).contiguous();
      at::Tensor m2 = acc.run(c, kM2, mean);
      at::Tensor var = m2 / (n - a.ddof);
      at::Tensor valid = (n - a.ddof) > 0;
      return double_col(name, a.op == AGG_VAR ? var : var.sqrt(), valid);
    }
    case AGG_NUNIQUE:
    case AGG_QUANTILE: {
      at::Tensor gsub = gi.gid;
      Column vsub = c;
      if (c.nullable()) {  // both exclude nulls (pandas defaults)
        at::Tensor keep = MaskToIndices(c.validity);
        gsub = gi.gid.index_select(0, keep);
        vsub = GatherColumn(c, keep);
        vsub.validity = at::Tensor();
      }
      TablePtr tmp = values_by_group(t, gsub, vsub);
      Acc sub{ex, gsub, tmp->Rows(), gi.ngroups};
      if (a.op == AGG_NUNIQUE) {
        GroupInfo pairs = GroupIds(tmp, {0, 1});
        at::Tensor pg = gsub.index_select(0, pairs.first_rows);
        Acc pacc{ex, pg, pg.numel(), gi.ngroups};
        return long_col(name, pacc.run(column_from("g", pg), kCount));
      }
      at::Tensor perm = SortIndices(tmp, {0, 1}, {true});
      at::Tensor counts = sub.run(column_from("g", gsub), kCount);
      at::Tensor offs = exclusive_scan(ex, counts);
      at::Tensor out = ex.opts(at::kDouble).device().is_cuda() ? at::empty({gi.ngroups}, ex.opts(at::kDouble))
                                                               : at::empty({gi.ngroups}, ex.opts(at::kDouble));
      at::Tensor valid = ex.empty_u8(gi.ngroups);
      KCALL(ex, group_quantile, tmp->column(1).view(), ptr<int64_t>(perm), ptr<int64_t>(offs), gi.ngroups,
            a.quantile, ptr<double>(out), ptr<uint8_t>(valid));
      return double_col(name, out, valid);
    }
  }
  CYLON_THROW(Code::NotImplemented, "aggregation op " << a.op << " not supported");
}

// ---------------------------------------------------------------------------
// K8 LDS radix group-by (radix_groupby.hip): large inputs; keys: one integer key, one float key
// (canonical bits: -0.0 == +0.0, NaNs group together), or several non-null integer keys packed
// into one exact 63-bit composite; SUM / COUNT / MIN / MAX / MEAN / VAR / STDDEV (M2 from a
// second in-block pass over the partition's rows).  Groups come out in partition order (the
// hash path's first-occurrence order is not kept; the reference's hash group-by order is
// unspecified as well).  Returns nullptr when not eligible or when a partition overflows its
// LDS table.  Reference: groupby/hash_groupby.cpp:92-201, compute/aggregate_kernels.hpp:92-263.
static int64_t radix_groupby_min_rows() {
  return knobs::Int("RADIX_GROUPBY_MIN_ROWS", int64_t(1) << 22);
}

namespace {
// the group key as one int64 per row, and its inverse for the output key columns
struct GroupKey {
  at::Tensor k;                 // int64 [n]
  std::vector<int> cols;        // key columns
  std::vector<int64_t> lo;      // composite: per-column minimum
  std::vector<int> shift, bits; // composite: bit range of each column
  bool composite = false, fbits = false;
  // one fixed-length string key (wlen = L bytes): k is its invertible word key (hash.hpp word_key_*),
  // wmin / wmax the accumulators of MIN / MAX of its words 1..W-1 (equal in every group: exact)
  int64_t wlen = -1;
  std::vector<int> wmin, wmax;
  // any other string key: k is a 64-bit hash of the bytes; wmin[0] / wmax[0] the MIN / MAX of an
  // independent hash h2 (equal in every group: the groups are verified), rmin MIN of the row number
  bool hashed = false;
  int rmin = -1;
  bool null_group = false;  // nullable single integer key: null rows carry null_key (no valid key has it)
  int64_t null_key = 0;
  std::vector<int64_t> ncode;  // composite: field value of a null in key i (-1: the column has no nulls)
};
}  // namespace

static bool gb_int_key(const Column &c) {
  return simple_key(c) && (c.type.kind() == ValueKind::SIGNED_INT ||
                           (c.type.kind() == ValueKind::UNSIGNED_INT && c.type.width() < 8));
}

static bool group_key(const Exec &ex, const TablePtr &t, const std::vector<int> &keys, GroupKey &g) {
  g.cols = keys;
  const int64_t n = t->Rows();
  if (keys.size() == 1) {
    const Column &kc = t->column(keys[0]);
    const bool int_key = kc.type.kind() == ValueKind::SIGNED_INT || kc.type.kind() == ValueKind::UNSIGNED_INT;
    // a nullable integer key: its null rows form one group (as on the global path) under a key value
    // no valid row has -- one below the smallest valid key, or one above the largest
    const bool nullable_int = int_key && kc.nullable() && !kc.is_var() && kc.type.width() <= 8 &&
                              kc.data.element_size() == kc.type.width();
    if (!simple_key(kc) && !nullable_int) return false;
    if (int_key) {
      if (kc.type.width() == 8) {
        g.k = kc.data.view(at::kLong);
      } else {
        g.k = ex.empty_i64(n);
        hip::key64_from_column(kc.view(), n, ptr<int64_t>(g.k), ex.stream);
      }
      if (nullable_int) {
        const at::Tensor valid = kc.validity.slice(0, 0, n).ne(0);
        const at::Tensor lim = at::cat({at::where(valid, g.k, std::numeric_limits<int64_t>::max()).min().reshape({1}),
                                        at::where(valid, g.k, std::numeric_limits<int64_t>::min()).max().reshape({1})});
        const std::vector<int64_t> h = to_host_vec(lim);
        if (h[0] > std::numeric_limits<int64_t>::min()) g.null_key = h[0] - 1;
        else if (h[1] < std::numeric_limits<int64_t>::max()) g.null_key = h[1] + 1;
        else return false;  // every int64 value is a key: no free value for the null group
        g.k = at::where(valid, g.k, g.null_key);
        g.null_group = true;
      }
      return true;
    }
    if (kc.type.kind() == ValueKind::FLOAT && (kc.type.width() == 8 || kc.type.width() == 4)) {
      g.k = ex.empty_i64(n);  // -0.0 -> +0.0, NaNs -> one quiet NaN: one fused pass
      KCALL(ex, float_key_bits, kc.view(), n, ptr<int64_t>(g.k));
      g.fbits = true;
      return true;
    }
    return false;
  }
  std::vector<at::Tensor> mm;
  if ((int)keys.size() > kMaxCompositeKeys) return false;
  bool any_null = false;
  for (int c : keys) {
    const Column &kc = t->column(c);
    const bool nullable_int = kc.nullable() && !kc.is_var() && kc.type.width() <= 8 &&
                              kc.data.element_size() == kc.type.width() &&
                              (kc.type.kind() == ValueKind::SIGNED_INT ||
                               (kc.type.kind() == ValueKind::UNSIGNED_INT && kc.type.width() < 8));
    if (!gb_int_key(kc) && !nullable_int) return false;
    if (nullable_int) {  // span over the valid rows (a null takes the field value one past it)
      any_null = true;
      at::Tensor k = ex.empty_i64(n);
      hip::key64_from_column(kc.view(), n, ptr<int64_t>(k), ex.stream);
      const at::Tensor valid = kc.validity.slice(0, 0, n).ne(0);
      mm.push_back(at::where(valid, k, std::numeric_limits<int64_t>::max()).min().reshape({1}));
      mm.push_back(at::where(valid, k, std::numeric_limits<int64_t>::min()).max().reshape({1}));
      continue;
    }
    // span: min / max of the column itself (signed or byte storage), else of its 64-bit image
    const bool direct = kc.type.kind() == ValueKind::SIGNED_INT || kc.type.width() == 1;
    at::Tensor k = direct ? kc.data : ex.empty_i64(n);
    if (!direct) hip::key64_from_column(kc.view(), n, ptr<int64_t>(k), ex.stream);
    auto m2 = at::aminmax(k);
    mm.push_back(std::get<0>(m2).to(at::kLong).reshape({1}));
    mm.push_back(std::get<1>(m2).to(at::kLong).reshape({1}));
  }
  const std::vector<int64_t> h = to_host_vec(at::cat(mm));
  int total = 0;
  g.lo.resize(keys.size());
  g.bits.resize(keys.size());
  g.shift.resize(keys.size());
  g.ncode.assign(keys.size(), -1);
  for (size_t i = 0; i < keys.size(); ++i) {
    g.lo[i] = h[2 * i];
    if (h[2 * i + 1] < h[2 * i]) g.lo[i] = 0;  // every key of the column null
    uint64_t span = h[2 * i + 1] >= h[2 * i] ? (uint64_t)h[2 * i + 1] - (uint64_t)h[2 * i] : 0;
    if (t->column(keys[i]).nullable()) {
      if (span >= (uint64_t)std::numeric_limits<int64_t>::max()) return false;
      g.ncode[i] = (int64_t)span + 1;
      span += 1;
    }
    int b = 0;
    while (b < 64 && (span >> b) != 0) ++b;
    g.bits[i] = b;
    total += b;
  }
  if (total > 63) return false;
  for (size_t i = keys.size(), sh = 0; i-- > 0;) {
    g.shift[i] = (int)sh;
    sh += g.bits[i];
  }
  // one fused pass (composite_key_pack: each key column read once at its own width)
  g.k = ex.empty_i64(n);
  std::vector<ColView> v = views(t, keys);
  KCALL(ex, composite_key_pack, v.data(), (int)keys.size(), g.lo.data(), g.shift.data(), n, ptr<int64_t>(g.k),
        any_null ? g.ncode.data() : nullptr);
  g.composite = true;
  return true;
}

// output key columns of the groups from their int64 keys
static std::vector<Column> group_key_columns(const TablePtr &t, const GroupKey &g, const at::Tensor &gk) {
  std::vector<Column> out;
  const int64_t ng = gk.numel();
  if (g.composite) {
    for (size_t i = 0; i < g.cols.size(); ++i) {
      const Column &kc = t->column(g.cols[i]);
      const int64_t mask = g.bits[i] >= 63 ? std::numeric_limits<int64_t>::max() : (int64_t(1) << g.bits[i]) - 1;
      const at::Tensor f = at::bitwise_and(at::bitwise_right_shift(gk, (int64_t)g.shift[i]), mask);
      at::Tensor v = f + g.lo[i], valid;
      if (g.ncode[i] >= 0) {  // the null code: a null key, value unspecified
        valid = f.ne(g.ncode[i]).to(at::kByte);
        v = at::where(valid.to(at::kBool), v, at::zeros({1}, v.options()));
      }
      out.emplace_back(kc.name, kc.type, ng, v.to(kc.data.scalar_type()).contiguous(), at::Tensor(), valid);
    }
    return out;
  }
  const Column &kc = t->column(g.cols[0]);
  at::Tensor v = gk;
  if (g.fbits) v = gk.view(at::kDouble).to(kc.data.scalar_type());
  else if (kc.type.width() != 8) v = gk.to(kc.data.scalar_type());
  at::Tensor valid;
  if (g.null_group) {  // the null group's key slot: value unspecified, validity 0
    valid = gk.ne(g.null_key).to(at::kByte);
    v = at::where(valid.to(at::kBool), v, at::zeros({1}, v.options()));
  }
  out.emplace_back(kc.name, kc.type, ng, v.contiguous(), at::Tensor(), valid);
  return out;
}

// L when every row of c (a non-null string / binary column) holds L <= 64 bytes, else -1
static int64_t fixed_string_len(const Exec &ex, const Column &c) {
  if (c.nullable() || !(c.type.type == Type::STRING || c.type.type == Type::BINARY) || c.length == 0) return -1;
  at::Tensor mm = ex.empty_i64(2);
  hip::var_len_minmax(ptr<int64_t>(c.offsets), c.length, ptr<int64_t>(mm), ex.stream);
  const std::vector<int64_t> h = to_host_vec(mm);
  return h[0] == h[1] && h[0] > 0 && h[0] <= 64 ? h[0] : -1;
}

static TablePtr radix_groupby(const TablePtr &tin, const std::vector<int> &keys, const std::vector<AggSpec> &aggs,
                              bool hash_strings = false) {
  const int64_t n = tin->Rows();
  if (!tin->device().is_cuda() || n < radix_groupby_min_rows()) return nullptr;
  // A fixed-length string key groups by its invertible word key h (ops/join.cpp uses the same key):
  // equal h + equal words 1..W-1 means equal strings, so the words ride along as MIN and MAX
  // accumulators and the result is exact when MIN == MAX in every group (else: the exact path).
  // The output key bytes are rebuilt from h and the MIN words.
  //
  // Any other non-null string key (variable length, or words that would not fit the accumulator
  // planes) groups by a 64-bit hash h of its bytes, with MIN and MAX of one packed column -- the high
  // 32 bits of an independent hash h2 above the row number -- as accumulators: equal high halves of
  // MIN and MAX in every group mean all its rows agree on 96 hash bits (else: the exact path), and
  // the output key is the bytes of the row in MIN's low half (one gather of ng rows).  Reference:
  // hash_groupby.cpp:92-126 takes any key type.
  TablePtr t = tin;
  GroupKey gkey;
  int wfirst = -1;  // column of word 1 in the augmented table
  int hcol = -1;  // hashed string key: column of (h2 high half << 32 | row)
  at::Tensor wk;
  if (keys.size() == 1 && tin->column(keys[0]).is_var()) {
    const Column &kc = tin->column(keys[0]);
    if (kc.nullable() || !(kc.type.type == Type::STRING || kc.type.type == Type::BINARY)) return nullptr;
    Exec ex0(tin->device());
    if ((hash_strings || fixed_string_len(ex0, kc) < 0) && n <= (int64_t(1) << 32)) {
      // one column, (high 32 bits of h2) << 32 | row: MIN and MAX of it verify the group (equal high
      // halves: every row agrees on 64 + 32 hash bits) and MIN's low half is a representative row --
      // 8 B/row through the passes and one accumulator plane fewer than h2 + a row-number column
      at::Tensor h1 = ex0.empty_i64(n), h2 = ex0.empty_i64(n);
      hip::var_hash2(ptr<uint8_t>(kc.data), ptr<int64_t>(kc.offsets), n, reinterpret_cast<uint64_t *>(ptr<int64_t>(h1)),
                     reinterpret_cast<uint64_t *>(ptr<int64_t>(h2)), ex0.stream, true);
      std::vector<Column> cols = tin->columns();
      hcol = (int)cols.size();
      cols.emplace_back("__gh2row", DataType(Type::INT64), n, h2);
      t = Table::Make(tin->GetContext(), std::move(cols));
      gkey.hashed = true;
      gkey.cols = keys;
      gkey.k = h1;
    }
  }
  if (keys.size() == 1 && tin->column(keys[0]).is_var() && !gkey.hashed) {
    const Column &kc = tin->column(keys[0]);
    Exec ex0(tin->device());
    const int64_t L = fixed_string_len(ex0, kc);
    if (L < 0) return nullptr;
    const int64_t W = (L + 7) / 8;
    const int64_t o0 = read_i64(kc.offsets, 0);
    wk = ex0.empty_i64(n);
    std::vector<Column> cols = tin->columns();
    std::vector<int64_t *> wp{nullptr};
    wfirst = (int)cols.size();
    for (int64_t j = 1; j < W; ++j) {
      cols.emplace_back("__gw" + std::to_string(j), DataType(Type::INT64), n, ex0.empty_i64(n));
      wp.push_back(ptr<int64_t>(cols.back().data));
    }
    hip::bytes_to_words(ptr<uint8_t>(kc.data) + o0, n, (int)L, wp.data(), ex0.stream,
                        reinterpret_cast<uint64_t *>(ptr<int64_t>(wk)), true);
    t = Table::Make(tin->GetContext(), std::move(cols));
    gkey.wlen = L;
    gkey.cols = keys;
    gkey.k = wk;
  }
  struct Plan {
    int col, kind;  // kind: 0 SUMF 1 SUMI 2 MIN 3 MAX 4 CNT 5 M2
  };
  std::vector<Plan> plan;
  auto need = [&](int col, int kind) {
    for (size_t j = 0; j < plan.size(); ++j)
      if (plan[j].col == col && plan[j].kind == kind) return (int)j;
    plan.push_back({col, kind});
    return (int)plan.size() - 1;
  };
  struct Out {
    int op, col, a, b, c, ddof;  // accumulator indices (b: count for MEAN / VAR / nullable MIN,MAX; c: M2)
  };
  std::vector<Out> outs;
  for (const auto &a : aggs) {
    const Column &c = t->column(a.col);
    const int w = c.type.width();
    if (c.is_var() || c.type.kind() == ValueKind::FIXED_BYTES || !c.type.is_numeric() ||
        !(w == 1 || w == 2 || w == 4 || w == 8))
      return nullptr;
    const bool fl = c.type.kind() == ValueKind::FLOAT;
    switch (a.op) {
      case AGG_SUM: outs.push_back({a.op, a.col, need(a.col, fl ? 0 : 1), -1, -1, 0}); break;
      case AGG_COUNT: outs.push_back({a.op, a.col, need(a.col, 4), -1, -1, 0}); break;
      case AGG_MIN:
      case AGG_MAX:
        outs.push_back({a.op, a.col, need(a.col, a.op == AGG_MIN ? 2 : 3), c.nullable() ? need(a.col, 4) : -1, -1, 0});
        break;
      case AGG_MEAN: outs.push_back({a.op, a.col, need(a.col, 0), need(a.col, 4), -1, 0}); break;
      case AGG_VAR:
      case AGG_STDDEV: {
        const int sa = need(a.col, 0), ca = need(a.col, 4);
        outs.push_back({a.op, a.col, sa, ca, need(a.col, 5), a.ddof});
        break;
      }
      default: return nullptr;
    }
  }
  if (gkey.wlen > 0) {
    for (int c = wfirst; c < t->Columns(); ++c) {
      gkey.wmin.push_back(need(c, 2));
      gkey.wmax.push_back(need(c, 3));
    }
  }
  if (gkey.hashed) {
    gkey.wmin.push_back(need(hcol, 2));
    gkey.wmax.push_back(need(hcol, 3));
    gkey.rmin = gkey.wmin.back();  // (its low 32 bits: the row)
  }
  // the LDS aggregation kernels are instantiated with 1, 2, 3, 4 or 8 accumulator planes; a
  // fixed-length key whose MIN / MAX words do not fit beside the aggregates is hashed instead
  if (plan.size() > 8 && gkey.wlen > 0) {
    trace::add_counter("groupby.radix.word_key_too_wide", 1);
    return radix_groupby(tin, keys, aggs, true);
  }
  if (plan.empty() || plan.size() > 8) return nullptr;
  Exec ex(t->device());
  if (gkey.wlen < 0 && !gkey.hashed && !group_key(ex, t, keys, gkey)) return nullptr;
  const int nacc = (int)plan.size();
  const at::Tensor &kt = gkey.k;
  double est;
  {
    CYLON_PHASE("groupby.radix.estimate", ex.device);
    at::Tensor regs = at::empty({hip::distinct_estimate_workspace()}, ex.opts(at::kInt));
    est = hip::distinct_estimate(ptr<int64_t>(kt), n, reinterpret_cast<uint32_t *>(ptr<int32_t>(regs)), ex.stream);
  }
  const double target = 0.6 * (double)hip::radix_groupby_slots(nacc);  // mean distinct keys per partition
  int bits = 0;
  while (bits < 24 && est * 1.05 / (double)(int64_t(1) << bits) > target) ++bits;
  // partition set: key, each used value column, its validity
  std::vector<at::Tensor> cols{kt};
  std::vector<int> widths{8};
  std::vector<int> dslot(t->Columns(), -1), vslot(t->Columns(), -1);
  for (const auto &pl : plan) {
    const Column &c = t->column(pl.col);
    if (dslot[pl.col] < 0) {
      dslot[pl.col] = (int)cols.size();
      cols.push_back(c.data);
      widths.push_back(c.type.width());
      if (c.nullable()) {
        vslot[pl.col] = (int)cols.size();
        cols.push_back(c.validity);
        widths.push_back(1);
      }
    }
  }
  at::Tensor offs;
  if (bits > 0) {
    CYLON_PHASE("groupby.radix.partition", ex.device);
    cols = RadixPartition(ex, std::move(cols), widths, bits, &offs);
  } else {
    offs = at::tensor({int64_t(0), n}, at::TensorOptions().dtype(at::kLong)).to(ex.device);
  }
  const int64_t nparts = int64_t(1) << bits;
  std::vector<RGAccDesc> desc(nacc);
  for (int j = 0; j < nacc; ++j) {
    const Column &c = t->column(plan[j].col);
    desc[j].src = plan[j].kind == 4 ? nullptr : reinterpret_cast<const uint8_t *>(cols[dslot[plan[j].col]].data_ptr());
    desc[j].valid = vslot[plan[j].col] >= 0 ? cols[vslot[plan[j].col]].data_ptr<uint8_t>() : nullptr;
    desc[j].kind = plan[j].kind;
    desc[j].width = c.type.width();
    desc[j].vkind = static_cast<int>(c.type.kind());
    desc[j].sum_acc = desc[j].cnt_acc = 0;
    if (plan[j].kind == 5)
      for (int q = 0; q < nacc; ++q) {
        if (plan[q].col == plan[j].col && plan[q].kind == 0) desc[j].sum_acc = q;
        if (plan[q].col == plan[j].col && plan[q].kind == 4) desc[j].cnt_acc = q;
      }
  }
  at::Tensor okeys = ex.empty_i64(n), oacc = ex.empty_i64(hip::radix_groupby_planes(nacc) * n),
             gcount = ex.empty_i64(nparts);
  at::Tensor overflow = at::empty({1}, ex.opts(at::kInt));
  {
    CYLON_PHASE("groupby.radix.aggregate", ex.device);
    hip::radix_groupby_agg(ptr<int64_t>(cols[0]), ptr<int64_t>(offs), nparts, desc.data(), nacc, ptr<int64_t>(okeys),
                           reinterpret_cast<uint64_t *>(ptr<int64_t>(oacc)), n, ptr<int64_t>(gcount),
                           overflow.data_ptr<int>(), ex.stream);
  }
  if (hip::rp_take_order_violation(ex.stream)) {  // ranking guard of a stable pass fired
    trace::add_counter("groupby.radix.order_violation_fallback", 1);
    return nullptr;
  }
  const int ovf = overflow.item<int>();
  CYLON_CHECK((ovf & ~1) == 0, Code::ExecutionError,
              "radix group-by: inconsistent partition (flags " << ovf << ": 8 = offsets, 16 = groups > rows)");
  if (ovf != 0) {
    trace::add_counter("groupby.radix.overflow_fallback", 1);
    return nullptr;
  }
  at::Tensor goff = exclusive_scan(ex, gcount);
  const int64_t ng = read_i64(goff, nparts);
  at::Tensor gkeys = ex.empty_i64(ng), gacc = ex.empty_i64(std::max(1, nacc) * ng);
  if (ng > 0)
    hip::radix_groupby_pack(ptr<int64_t>(offs), ptr<int64_t>(goff), nparts, ptr<int64_t>(okeys),
                            reinterpret_cast<const uint64_t *>(ptr<int64_t>(oacc)), n, nacc, ptr<int64_t>(gkeys),
                            reinterpret_cast<uint64_t *>(ptr<int64_t>(gacc)), ng, ex.stream);
  trace::add_counter("groupby.radix.groups", ng);
  if (gkey.composite) trace::add_counter("groupby.radix.composite_key", 1);
  auto plane = [&](int j) { return gacc.slice(0, j * ng, (j + 1) * ng); };
  std::vector<Column> out;
  if (gkey.hashed) {
    const at::Tensor mn = minmax_col(ex, "", t->column(hcol), plane(gkey.wmin[0]).contiguous(), at::Tensor()).data;
    const at::Tensor mx = minmax_col(ex, "", t->column(hcol), plane(gkey.wmax[0]).contiguous(), at::Tensor()).data;
    if (ng > 0 && at::bitwise_right_shift(mn, 32).ne(at::bitwise_right_shift(mx, 32)).any().item<bool>()) {
      trace::add_counter("groupby.radix.string_hash_collision_fallback", 1);
      return nullptr;
    }
    const at::Tensor rep = at::bitwise_and(mn, 0xffffffffll);
    const Column &kc = t->column(keys[0]);
    out.push_back(Gather(Table::Make(t->GetContext(), {kc}), rep)->column(0));
    trace::add_counter("groupby.radix.hashed_string_key", 1);
  } else if (gkey.wlen > 0) {
    if (!gkey.wmin.empty()) {  // exact iff every group's words 1..W-1 agree (a 64-bit h collision: not)
      std::vector<at::Tensor> ne;
      for (size_t j = 0; j < gkey.wmin.size(); ++j) ne.push_back(plane(gkey.wmin[j]).ne(plane(gkey.wmax[j])).any());
      if (at::stack(ne).any().item<bool>()) {
        trace::add_counter("groupby.radix.word_key_collision_fallback", 1);
        return nullptr;
      }
    }
    const Column &kc = t->column(keys[0]);
    const int64_t L = gkey.wlen;
    std::vector<at::Tensor> wcols;  // the words from the MIN planes (which hold order images)
    std::vector<const int64_t *> wp{nullptr};
    for (size_t j = 0; j < gkey.wmin.size(); ++j) {
      wcols.push_back(minmax_col(ex, "", t->column(wfirst + (int)j), plane(gkey.wmin[j]).contiguous(), at::Tensor()).data);
      wp.push_back(ptr<int64_t>(wcols.back()));
    }
    at::Tensor bytes = ex.empty_bytes(std::max<int64_t>(1, ng * L));
    if (ng > 0)
      hip::words_to_bytes(wp.data(), ng, (int)L, ptr<uint8_t>(bytes), ex.stream,
                          reinterpret_cast<const uint64_t *>(ptr<int64_t>(gkeys)));
    out.emplace_back(kc.name, kc.type, ng, bytes.slice(0, 0, ng * L), at::arange(0, (ng + 1) * L, L, ex.opts(at::kLong)));
    trace::add_counter("groupby.radix.word_key", 1);
  } else {
    out = group_key_columns(t, gkey, gkeys);
  }
  for (const auto &o : outs) {
    const Column &c = t->column(o.col);
    const std::string name = std::string(AggPrefix(o.op)) + c.name;
    switch (o.op) {
      case AGG_SUM:
        if (c.type.kind() == ValueKind::FLOAT) out.push_back(double_col(name, plane(o.a).view(at::kDouble)));
        else
          out.push_back(long_col(name, plane(o.a),
                                 c.type.kind() == ValueKind::UNSIGNED_INT ? Type::UINT64 : Type::INT64));
        break;
      case AGG_COUNT: out.push_back(long_col(name, plane(o.a))); break;
      case AGG_MIN:
      case AGG_MAX: {
        at::Tensor cnt = o.b >= 0 ? plane(o.b) : at::Tensor();
        out.push_back(minmax_col(ex, name, c, plane(o.a).contiguous(), cnt));
        break;
      }
      case AGG_MEAN: {
        at::Tensor s = plane(o.a).view(at::kDouble), cnt = plane(o.b);
        out.push_back(double_col(name, s / cnt.to(at::kDouble), cnt > 0));
        break;
      }
      case AGG_VAR:
      case AGG_STDDEV: {
        at::Tensor m2 = plane(o.c).view(at::kDouble), cnt = plane(o.b).to(at::kDouble);
        at::Tensor var = m2 / (cnt - o.ddof);
        out.push_back(double_col(name, o.op == AGG_VAR ? var : var.sqrt(), (cnt - o.ddof) > 0));
        break;
      }
    }
  }
  return Table::Make(t->GetContext(), std::move(out));
}

static TablePtr groupby_with(const TablePtr &t, const std::vector<int> &keys, const std::vector<AggSpec> &aggs,
                             bool presorted);

// QUANTILE on the LDS radix path (one (column, q) aggregate): the rows (group key, value[, validity])
// are radix-partitioned by the key's hash into partitions of <= radix_quantile_capacity() rows, and
// one workgroup per partition sorts them in LDS by (key, value) and takes each group's quantile by
// the global path's type-2 rule (radix_groupby.hip k_rg_quantile).  nullptr when a partition
// overflows (a group -- or a hash bucket of groups -- beyond the capacity): the caller falls back.
// Reference: compute/aggregate_kernels.hpp:504-545 (QuantileKernel).
static TablePtr radix_quantile_bits(const TablePtr &t, const std::vector<int> &keys, const AggSpec &a, const GroupKey &gkey,
                                    int bits, const Column &c, int w, const std::vector<AggSpec> *fuse);

// fuse (optional): SUM / COUNT / MEAN / MIN / MAX aggregates of the quantile's own float64 column,
// computed by the quantile kernel from the same sorted rows (no second group-by and no join); their
// columns follow the quantile column in `fuse` order.
static TablePtr radix_quantile_table(const TablePtr &t, const std::vector<int> &keys, const AggSpec &a,
                                     const std::vector<AggSpec> *fuse = nullptr) {
  const Column &c = t->column(a.col);
  const int w = c.type.width();
  if (c.is_var() || c.type.kind() == ValueKind::FIXED_BYTES || !c.type.is_numeric() ||
      !(w == 1 || w == 2 || w == 4 || w == 8))
    return nullptr;
  Exec ex(t->device());
  GroupKey gkey;
  if (!group_key(ex, t, keys, gkey)) return nullptr;
  const int64_t n = t->Rows(), cap = hip::radix_quantile_capacity();
  // A partition holds Poisson(groups / P) whole groups of ~n / groups rows each, so its row count
  // varies with the group size: P comes from the distinct-key estimate (HyperLogLog), with the
  // groups' Poisson tail (6 sigma) inside the capacity -- 1B rows / 10M groups: 20 bits (two passes),
  // where a row-count rule (1907-row mean) overflowed.  Groups larger than half the capacity: global path.
  double groups;
  {
    at::Tensor regs = at::empty({hip::distinct_estimate_workspace()}, ex.opts(at::kInt));
    groups = std::max(1.0, hip::distinct_estimate(ptr<int64_t>(gkey.k), n, reinterpret_cast<uint32_t *>(ptr<int32_t>(regs)),
                                                  ex.stream));
  }
  const double grp_rows = (double)n / groups;
  if (grp_rows > 0.5 * (double)cap) return nullptr;
  auto fits = [&](int b) {
    const double lam = groups / (double)(int64_t(1) << b);
    return (double)n / (double)(int64_t(1) << b) <= 0.85 * (double)cap &&
           grp_rows * (lam + 6.0 * std::sqrt(lam) + 2.0) <= (double)cap;
  };
  int bits = 0;
  while (bits < 24 && !fits(bits)) ++bits;
  return radix_quantile_bits(t, keys, a, gkey, bits, c, w, fuse);
}

static TablePtr radix_quantile_bits(const TablePtr &t, const std::vector<int> &keys, const AggSpec &a, const GroupKey &gkey,
                                    int bits, const Column &c, int w, const std::vector<AggSpec> *fuse) {
  Exec ex(t->device());
  const int64_t n = t->Rows();
  std::vector<at::Tensor> cols{gkey.k, c.data};
  std::vector<int> widths{8, w};
  if (c.nullable()) {
    cols.push_back(c.validity);
    widths.push_back(1);
  }
  at::Tensor offs;
  if (bits > 0) {
    CYLON_PHASE("groupby.radix.quantile_partition", ex.device);
    cols = RadixPartition(ex, std::move(cols), widths, bits, &offs, nullptr, nullptr, false);
  } else {
    offs = at::tensor({int64_t(0), n}, at::TensorOptions().dtype(at::kLong)).to(ex.device);
  }
  const int64_t nparts = int64_t(1) << bits;
  const int planes = fuse ? 6 : 2;  // quantile, validity [, sum, count, min, max]
  at::Tensor okeys = ex.empty_i64(n), oacc = ex.empty_i64(planes * n), gcount = ex.empty_i64(nparts);
  at::Tensor overflow = at::empty({1}, ex.opts(at::kInt));
  {
    CYLON_PHASE("groupby.radix.quantile", ex.device);
    hip::radix_groupby_quantile(ptr<int64_t>(cols[0]), reinterpret_cast<const uint8_t *>(cols[1].data_ptr()), w,
                                static_cast<int>(c.type.kind()), c.nullable() ? cols[2].data_ptr<uint8_t>() : nullptr,
                                ptr<int64_t>(offs), nparts, bits, a.quantile, ptr<int64_t>(okeys),
                                reinterpret_cast<uint64_t *>(ptr<int64_t>(oacc)),
                                reinterpret_cast<uint64_t *>(ptr<int64_t>(oacc) + n), ptr<int64_t>(gcount),
                                overflow.data_ptr<int>(), ex.stream,
                                fuse ? reinterpret_cast<uint64_t *>(ptr<int64_t>(oacc) + 2 * n) : nullptr, n);
  }
  if (overflow.item<int>() != 0) {  // a partition beyond the LDS capacity: finer partitions, once
    if (bits <= 22) {
      trace::add_counter("groupby.radix.quantile_overflow_retry", 1);
      cols.clear();
      return radix_quantile_bits(t, keys, a, gkey, bits + 2, c, w, fuse);
    }
    trace::add_counter("groupby.radix.quantile_overflow_fallback", 1);
    return nullptr;
  }
  at::Tensor goff = exclusive_scan(ex, gcount);
  const int64_t ng = read_i64(goff, nparts);
  at::Tensor gkeys = ex.empty_i64(ng), gacc = ex.empty_i64(planes * ng);
  if (ng > 0)
    hip::radix_groupby_pack(ptr<int64_t>(offs), ptr<int64_t>(goff), nparts, ptr<int64_t>(okeys),
                            reinterpret_cast<const uint64_t *>(ptr<int64_t>(oacc)), n, planes, ptr<int64_t>(gkeys),
                            reinterpret_cast<uint64_t *>(ptr<int64_t>(gacc)), ng, ex.stream);
  std::vector<Column> out = group_key_columns(t, gkey, gkeys);
  auto plane = [&](int j) { return gacc.slice(0, j * ng, (j + 1) * ng); };
  out.push_back(double_col(std::string(AggPrefix(AGG_QUANTILE)) + c.name, plane(0).view(at::kDouble), plane(1).ne(0)));
  if (fuse) {
    const at::Tensor cnt = plane(3), some = cnt > 0;
    for (const AggSpec &f : *fuse) {
      const std::string name = std::string(AggPrefix(f.op)) + c.name;
      switch (f.op) {
        case AGG_SUM: out.push_back(double_col(name, plane(2).view(at::kDouble))); break;
        case AGG_COUNT: out.push_back(long_col(name, cnt)); break;
        case AGG_MEAN: out.push_back(double_col(name, plane(2).view(at::kDouble) / cnt.to(at::kDouble), some)); break;
        case AGG_MIN: out.push_back(double_col(name, plane(4).view(at::kDouble), c.nullable() ? some : at::Tensor())); break;
        case AGG_MAX: out.push_back(double_col(name, plane(5).view(at::kDouble), c.nullable() ? some : at::Tensor())); break;
        default: CYLON_THROW(Code::Invalid, "fused quantile aggregate " << f.op);
      }
    }
    trace::add_counter("groupby.radix.quantile_fused_aggs", (int64_t)fuse->size());
  }
  trace::add_counter("groupby.radix.quantile", 1);
  return Table::Make(t->GetContext(), std::move(out));
}

// NUNIQUE and QUANTILE on the LDS radix path, composed from radix group-bys: the other aggregates of
// the keys (one radix group-by); per NUNIQUE column x the distinct (keys, x) pairs with x non-null
// (a radix group-by on keys + x) counted per key (a group-by of those pairs); per QUANTILE aggregate
// the LDS-sorted partitions above.  A LEFT join of the first result with each such (keys, value)
// table on the keys puts them side by side (a group whose x is all null counts 0 / has a null
// quantile).  Output order: join order (group-by order is unspecified, docs/semantics.md).
static TablePtr radix_groupby_composed(const TablePtr &t, const std::vector<int> &keys,
                                       const std::vector<AggSpec> &aggs) {
  if (!t->device().is_cuda() || t->Rows() < radix_groupby_min_rows()) return nullptr;
  std::vector<AggSpec> rest;
  std::vector<int> nucols, qidx;  // NUNIQUE columns; indices of the QUANTILE aggregates
  for (size_t i = 0; i < aggs.size(); ++i) {
    const auto &a = aggs[i];
    if (a.op == AGG_QUANTILE) {
      qidx.push_back((int)i);
    } else if (a.op != AGG_NUNIQUE) {
      rest.push_back(a);
    } else if (std::find(nucols.begin(), nucols.end(), a.col) == nucols.end()) {
      if (std::find(keys.begin(), keys.end(), a.col) != keys.end()) return nullptr;  // (nunique of a key: 1)
      nucols.push_back(a.col);
    }
  }
  if (nucols.empty() && qidx.empty()) return nullptr;
  for (int k : keys)
    if (t->column(k).is_var() || (!nucols.empty() && t->column(k).nullable())) return nullptr;
  // one QUANTILE of a float64 column whose other aggregates are SUM / COUNT / MEAN / MIN / MAX of the
  // same column: the quantile kernel computes them all from its sorted rows (one partition of
  // (key, value), no second group-by, no join) -- the {sum, quantile} shape of the config-4 bench
  if (qidx.size() == 1 && nucols.empty() && !rest.empty()) {
    const int qc = aggs[(size_t)qidx[0]].col;
    bool fusable = t->column(qc).type.type == Type::DOUBLE;
    for (const auto &r : rest)
      fusable &= r.col == qc && (r.op == AGG_SUM || r.op == AGG_COUNT || r.op == AGG_MEAN || r.op == AGG_MIN ||
                                 r.op == AGG_MAX);
    if (fusable) {
      TablePtr ft = radix_quantile_table(t, keys, aggs[(size_t)qidx[0]], &rest);
      if (ft) {
        const int nk = (int)keys.size();
        std::vector<Column> out;
        for (int i = 0; i < nk; ++i) out.push_back(ft->column(i).with_name(t->column(keys[i]).name));
        int ri = 0;
        for (size_t i = 0; i < aggs.size(); ++i)
          out.push_back(ft->column(aggs[i].op == AGG_QUANTILE ? nk : nk + 1 + ri++));
        return Table::Make(t->GetContext(), std::move(out));
      }
    }
  }
  const int nk = (int)keys.size();
  std::vector<int> kidx(nk);
  for (int i = 0; i < nk; ++i) kidx[i] = i;
  // the base: the rest aggregates, or the first quantile table, or a COUNT carrying the groups
  TablePtr cur;
  std::vector<int> qpos(aggs.size(), -1);  // column of cur holding quantile aggregate i
  size_t qfirst = 0;
  if (!rest.empty()) {
    cur = radix_groupby(t, keys, rest);
  } else if (!qidx.empty()) {
    cur = radix_quantile_table(t, keys, aggs[(size_t)qidx[0]]);
    qpos[(size_t)qidx[0]] = nk;
    qfirst = 1;
  } else {
    cur = radix_groupby(t, keys, {AggSpec{keys[0], AGG_COUNT}});
  }
  if (!cur) return nullptr;
  for (size_t j = qfirst; j < qidx.size(); ++j) {
    TablePtr qt = radix_quantile_table(t, keys, aggs[(size_t)qidx[j]]);
    if (!qt) return nullptr;
    const int width = cur->Columns();
    cur = Join(cur, qt, join::config::JoinConfig::LeftJoin(kidx, kidx, join::config::HASH));
    qpos[(size_t)qidx[j]] = width + nk;
  }
  std::vector<int> nupos;  // column of cur holding the count of nucols[i]
  for (int x : nucols) {
    std::vector<int> pc(keys);
    pc.push_back(x);
    TablePtr pairs = Project(t, pc);
    if (t->column(x).nullable()) pairs = FilterByMask(pairs, t->column(x).validity);
    std::vector<int> pk(kidx);
    pk.push_back(nk);
    TablePtr distinct = groupby_with(pairs, pk, {AggSpec{nk, AGG_COUNT}}, false);
    TablePtr counts = groupby_with(Project(distinct, kidx), kidx, {AggSpec{0, AGG_COUNT}}, false);
    const int width = cur->Columns();
    cur = Join(cur, counts, join::config::JoinConfig::LeftJoin(kidx, kidx, join::config::HASH));
    nupos.push_back(width + nk);
  }
  if (!nucols.empty()) trace::add_counter("groupby.radix.nunique_columns", (int64_t)nucols.size());
  std::vector<Column> out;
  for (int i = 0; i < nk; ++i) out.push_back(cur->column(i).with_name(t->column(keys[i]).name));
  int ri = 0;
  for (size_t i = 0; i < aggs.size(); ++i) {
    const auto &a = aggs[i];
    if (a.op == AGG_QUANTILE) {
      out.push_back(cur->column(qpos[i]).with_name(std::string(AggPrefix(AGG_QUANTILE)) + t->column(a.col).name));
      continue;
    }
    if (a.op != AGG_NUNIQUE) {
      out.push_back(cur->column(nk + ri++));
      continue;
    }
    const size_t j = std::find(nucols.begin(), nucols.end(), a.col) - nucols.begin();
    Column c = cur->column(nupos[j]);
    at::Tensor v = c.nullable() ? c.data.masked_fill(c.validity == 0, 0) : c.data;
    out.emplace_back(std::string(AggPrefix(AGG_NUNIQUE)) + t->column(a.col).name, DataType(Type::INT64), c.length,
                     v.contiguous());
  }
  return Table::Make(t->GetContext(), std::move(out));
}

static TablePtr groupby_with(const TablePtr &t, const std::vector<int> &keys, const std::vector<AggSpec> &aggs,
                             bool presorted) {
  CYLON_CHECK(!keys.empty(), Code::Invalid, "group-by needs at least one key column");
  if (!presorted) {
    if (TablePtr r = radix_groupby(t, keys, aggs)) return r;
    if (TablePtr r = radix_groupby_composed(t, keys, aggs)) return r;
  }
  Exec ex(t->device());
  GroupInfo gi;
  {
    CYLON_PHASE("groupby.group_ids", ex.device);
    gi = GroupIds(t, keys, presorted);
  }
  CYLON_PHASE("groupby.aggregate", ex.device);
  TablePtr kt = GatherNullable(Project(t, keys), gi.first_rows, false);
  std::vector<Column> cols = kt->columns();
  for (const auto &a : aggs) cols.push_back(agg_column(ex, t, gi, a));
  return Table::Make(t->GetContext(), std::move(cols));
}

TablePtr HashGroupBy(const TablePtr &t, const std::vector<int> &keys, const std::vector<AggSpec> &aggs) {
  return groupby_with(t, keys, aggs, false);
}

TablePtr PipelineGroupBy(const TablePtr &t, const std::vector<int> &keys, const std::vector<AggSpec> &aggs) {
  return groupby_with(t, keys, aggs, true);
}

// ---------------------------------------------------------------------------
// distributed (two-phase with partial states)
// ---------------------------------------------------------------------------
static bool decomposable(int op) {
  return op == AGG_SUM || op == AGG_COUNT || op == AGG_MIN || op == AGG_MAX || op == AGG_MEAN || op == AGG_VAR ||
         op == AGG_STDDEV;
}

TablePtr DistributedHashGroupBy(const TablePtr &t, const std::vector<int> &keys, const std::vector<AggSpec> &aggs) {
  auto ctx = t->GetContext();
  if (!ctx->ShuffleRequired()) return HashGroupBy(t, keys, aggs);
  bool all_dec = true;
  for (const auto &a : aggs) all_dec &= decomposable(a.op);
  const int nk = (int)keys.size();
  std::vector<int> key_pos(nk);
  for (int i = 0; i < nk; ++i) key_pos[i] = i;

  if (!all_dec) {  // shuffle raw rows, aggregate once
    std::vector<int> cols = keys;
    std::vector<AggSpec> remapped;
    for (const auto &a : aggs) {
      AggSpec b = a;
      b.col = (int)cols.size();
      cols.push_back(a.col);
      remapped.push_back(b);
    }
    std::vector<TablePtr> parts;
    ShufflePlanned(Project(t, cols), key_pos,
                   [&](int, int, const TablePtr &sh) { parts.push_back(HashGroupBy(sh, key_pos, remapped)); });
    return parts.size() == 1 ? parts[0] : Merge(parts);
  }

  struct Plan {
    int op;
    int ddof;
    std::string name;
    std::vector<int> state_cols;  // positions in the partial table
  };
  std::vector<Plan> plans;
  std::vector<AggSpec> combine;  // phase-2 aggregations over the state columns
  TablePtr partial;

  // phase 1, fast form: SUM / COUNT / MIN / MAX / MEAN over non-null value columns
  // are their own partial states, so the local hash group-by produces them directly
  // (the LDS radix group-by on device tables, radix_groupby.hip) instead of the
  // global group-id path below.
  bool simple_states = true;
  for (const auto &a : aggs)
    simple_states &= (a.op == AGG_SUM || a.op == AGG_COUNT || a.op == AGG_MIN || a.op == AGG_MAX ||
                      a.op == AGG_MEAN) &&
                     !t->column(a.col).nullable();
  if (simple_states) {
    std::vector<AggSpec> st;
    for (const auto &a : aggs) {
      Plan p{a.op, a.ddof, std::string(AggPrefix(a.op)) + t->column(a.col).name, {}};
      auto add = [&](int op, int combine_op) {
        const int pos = nk + (int)st.size();
        st.push_back(AggSpec{a.col, op});
        p.state_cols.push_back(pos);
        combine.push_back(AggSpec{pos, combine_op});
      };
      if (a.op == AGG_MEAN) {
        add(AGG_SUM, AGG_SUM);
        add(AGG_COUNT, AGG_SUM);
      } else {
        add(a.op, a.op == AGG_COUNT ? AGG_SUM : a.op);
      }
      plans.push_back(std::move(p));
    }
    partial = HashGroupBy(t, keys, st);
  } else {
  // phase 1: local partial states
  Exec ex(t->device());
  GroupInfo gi = GroupIds(t, keys, false);
  TablePtr kt = GatherNullable(Project(t, keys), gi.first_rows, false);
  std::vector<Column> pcols = kt->columns();
  Acc acc{ex, gi.gid, t->Rows(), gi.ngroups};
  auto add_state = [&](Plan &p, Column c, int combine_op) {
    const int pos = (int)pcols.size();
    c.name = "__s" + std::to_string(pos);
    pcols.push_back(std::move(c));
    p.state_cols.push_back(pos);
    combine.push_back(AggSpec{pos, combine_op});
  };
  for (const auto &a : aggs) {
    const Column &c = t->column(a.col);
    Plan p{a.op, a.ddof, std::string(AggPrefix(a.op)) + c.name, {}};
    switch (a.op) {
      case AGG_SUM:
      case AGG_MIN:
      case AGG_MAX:
      case AGG_COUNT:
        add_state(p, agg_column(ex, t, gi, a), a.op == AGG_COUNT ? AGG_SUM : a.op);
        break;
      case AGG_MEAN:
        add_state(p, double_col("", acc.run(c, kSumF)), AGG_SUM);
        add_state(p, long_col("", acc.run(c, kCount)), AGG_SUM);
        break;
      default: {  // VAR / STDDEV: (count, sum, M2, sum^2/count)
        at::Tensor s = acc.run(c, kSumF), n = acc.run(c, kCount);
        at::Tensor nd = n.to(at::kDouble);
        at::Tensor mean = (s / nd).contiguous();
        at::Tensor m2 = at::nan_to_num(acc.run(c, kM2, mean), 0.0);
        at::Tensor q = at::nan_to_num(s * s / nd, 0.0);
        add_state(p, long_col("", n), AGG_SUM);
        add_state(p, double_col("", s), AGG_SUM);
        add_state(p, double_col("", m2), AGG_SUM);
        add_state(p, double_col("", q), AGG_SUM);
      }
    }
    plans.push_back(std::move(p));
  }
  partial = Table::Make(t->GetContext(), std::move(pcols));
  }  // generic phase 1
  // phase 2: shuffle partial rows by key and combine -- chunk by hash-disjoint chunk, so the
  // combine of chunk k runs while the later chunks are still on the wire
  std::vector<TablePtr> combined;
  ShufflePlanned(partial, key_pos, [&](int, int, const TablePtr &sh) {
    combined.push_back(HashGroupBy(sh, key_pos, combine));
  });
  TablePtr comb = combined.size() == 1 ? combined[0] : Merge(combined);
  std::vector<Column> out;
  for (int i = 0; i < nk; ++i) out.push_back(comb->column(i));
  int ci = nk;
  for (const auto &p : plans) {
    switch (p.op) {
      case AGG_SUM:
      case AGG_MIN:
      case AGG_MAX:
      case AGG_COUNT:
        out.push_back(comb->column(ci++).with_name(p.name));
        break;
      case AGG_MEAN: {
        at::Tensor s = comb->column(ci++).data.to(at::kDouble), n = comb->column(ci++).data.to(at::kDouble);
        out.push_back(double_col(p.name, s / n, n > 0));
        break;
      }
      default: {
        at::Tensor n = comb->column(ci++).data.to(at::kDouble);
        at::Tensor s = comb->column(ci++).data;
        at::Tensor m2 = comb->column(ci++).data;
        at::Tensor q = comb->column(ci++).data;
        at::Tensor mean = s / n;
        at::Tensor M2 = at::clamp_min(m2 + q - n * mean * mean, 0.0);
        at::Tensor var = M2 / (n - p.ddof);
        out.push_back(double_col(p.name, p.op == AGG_VAR ? var : var.sqrt(), (n - p.ddof) > 0));
      }
    }
  }
  return Table::Make(t->GetContext(), std::move(out));
}

TablePtr DistributedPipelineGroupBy(const TablePtr &t, const std::vector<int> &keys,
                                    const std::vector<AggSpec> &aggs) {
  auto ctx = t->GetContext();
  std::vector<int> cols = keys;
  std::vector<AggSpec> remapped;
  for (const auto &a : aggs) {
    AggSpec b = a;
    b.col = (int)cols.size();
    cols.push_back(a.col);
    remapped.push_back(b);
  }
  std::vector<int> key_pos(keys.size());
  for (size_t i = 0; i < keys.size(); ++i) key_pos[i] = (int)i;
  TablePtr p = Project(t, cols);
  if (ctx->GetWorldSize() > 1) p = Shuffle(p, key_pos);
  TablePtr sorted = Sort(p, key_pos, {true});
  return PipelineGroupBy(sorted, key_pos, remapped);
}

// ---------------------------------------------------------------------------
// scalar aggregates (K12 + allreduce)
// ---------------------------------------------------------------------------
TablePtr Aggregate(const TablePtr &t, int col, int op, double quantile, int ddof, bool distributed) {
  auto ctx = t->GetContext();
  const bool dist = distributed && ctx->GetWorldSize() > 1;
  auto comm = ctx->GetCommunicator();
  Exec ex(t->device());
  const Column &c = t->column(col);
  at::Tensor none;
  Acc acc{ex, none, t->Rows(), 1};
  auto allreduce = [&](at::Tensor x, net::ReduceOp o) {
    if (dist) comm->AllReduce(x, o);
    return x;
  };
  const bool is_float = c.type.kind() == ValueKind::FLOAT;
  std::vector<Column> out;
  switch (op) {
    case AGG_SUM:
      if (is_float) out.push_back(double_col(c.name, allreduce(acc.run(c, kSumF), net::ReduceOp::SUM)));
      else out.push_back(long_col(c.name, allreduce(acc.run(c, kSumI), net::ReduceOp::SUM)));
      break;
    case AGG_COUNT:
      out.push_back(long_col(c.name, allreduce(acc.run(c, kCount), net::ReduceOp::SUM)));
      break;
    case AGG_MIN:
    case AGG_MAX: {
      CYLON_CHECK(c.type.is_numeric(), Code::TypeError, "min/max need a numeric column");
      at::Tensor img = acc.run(c, op == AGG_MIN ? kMin : kMax);
      // unsigned image -> signed order for the collective
      at::Tensor flip = at::full({1}, std::numeric_limits<int64_t>::min(), img.options());
      at::Tensor s = at::bitwise_xor(img, flip);
      s = allreduce(s, op == AGG_MIN ? net::ReduceOp::MIN : net::ReduceOp::MAX);
      img = at::bitwise_xor(s, flip).contiguous();
      at::Tensor cnt = allreduce(acc.run(c, kCount), net::ReduceOp::SUM);
      Column mc = minmax_col(ex, c.name, c, img, cnt);
      if (!c.nullable()) mc.validity = (cnt > 0).to(at::kByte);
      out.push_back(mc);
      break;
    }
    case AGG_MEAN: {
      at::Tensor s = allreduce(acc.run(c, kSumF), net::ReduceOp::SUM);
      at::Tensor n = allreduce(acc.run(c, kCount), net::ReduceOp::SUM);
      out.push_back(double_col(c.name, s / n.to(at::kDouble), n > 0));
      break;
    }
    case AGG_VAR:
    case AGG_STDDEV: {
      at::Tensor s = allreduce(acc.run(c, kSumF), net::ReduceOp::SUM);
      at::Tensor n = allreduce(acc.run(c, kCount), net::ReduceOp::SUM).to(at::kDouble);
      at::Tensor mean = (s / n).contiguous();
      at::Tensor m2 = allreduce(acc.run(c, kM2, mean), net::ReduceOp::SUM);
      at::Tensor var = m2 / (n - ddof);
      out.push_back(double_col(c.name, op == AGG_VAR ? var : var.sqrt(), (n - ddof) > 0));
      break;
    }
    case AGG_NUNIQUE: {
      TablePtr one = Project(t, {col});
      if (c.nullable()) one = FilterByMask(one, c.validity);
      TablePtr u = dist ? DistributedUnique(one, {0}, true) : Unique(one, {0}, true);
      at::Tensor cnt = at::full({1}, u->Rows(), ex.opts(at::kLong));
      out.push_back(long_col(c.name, allreduce(cnt, net::ReduceOp::SUM)));
      break;
    }
    case AGG_QUANTILE: {
      TablePtr one = Project(t, {col});
      if (dist) {
        std::vector<Column> gathered;
        CYLON_CHECK(!c.is_var(), Code::TypeError, "quantile needs a numeric column");
        auto parts = comm->AllGatherV(c.data);
        at::Tensor all = at::cat(parts);
        at::Tensor valid;
        if (c.nullable()) valid = at::cat(comm->AllGatherV(c.validity));
        one = Table::Make(ctx, {Column(c.name, c.type, all.numel(), all, at::Tensor(), valid)});
      }
      at::Tensor zero = at::zeros({one->Rows()}, ex.opts(at::kLong));
      GroupInfo gi{zero, one->Rows() ? 1 : 0, at::Tensor()};
      if (one->Rows() == 0) {
        out.push_back(double_col(c.name, at::zeros({1}, ex.opts(at::kDouble)), at::zeros({1}, ex.opts(at::kByte))));
        break;
      }
      Column q = agg_column(ex, one, gi, AggSpec{0, AGG_QUANTILE, quantile, ddof});
      out.push_back(q.with_name(c.name));
      break;
    }
    default: CYLON_THROW(Code::NotImplemented, "aggregate op " << op);
  }
  return Table::Make(ctx, std::move(out));
}

}  // namespace ops
}  // namespace cylon
