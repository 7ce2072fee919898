// Table plumbing operators: gather (K4), compaction (K11), project, merge,
// slice.  Reference: cylon/util/copy_arrray.cpp:24-142 (copy_array_by_indices,
// -1 -> null), table.cpp:267-289 (Merge), :831-850 (Project), arrow Filter.
#include "util.hpp"

namespace cylon {
namespace ops {

std::vector<ColView> views(const TablePtr &t, const std::vector<int> &cols) {
  std::vector<ColView> v;
  v.reserve(cols.size());
  for (int c : cols) v.push_back(t->column(c).view());
  return v;
}

static Column gather_var(const Exec &ex, const Column &c, const at::Tensor &idx, bool may_null) {
  const int64_t m = idx.numel();
  ColView in = c.view();
  at::Tensor lens = ex.empty_i64(m);
  KCALL(ex, gather_var_lengths, in, ptr<int64_t>(idx), m, ptr<int64_t>(lens));
  at::Tensor offs = exclusive_scan(ex, lens);
  const int64_t total = read_i64(offs, m);
  at::Tensor bytes = ex.empty_bytes(total);
  at::Tensor valid;
  if (c.nullable() || may_null) valid = ex.empty_u8(m);
  KCALL(ex, gather_var_bytes, in, ptr<int64_t>(idx), m, ptr<int64_t>(offs), total, ptr<uint8_t>(bytes),
        valid.defined() ? ptr<uint8_t>(valid) : nullptr);
  return Column(c.name, c.type, m, bytes, offs, valid);
}

// K15 var-width select (string / binary where and fill_null; kernels/select.hip): row i is a[i]
// where cond[i], else b[i] (b one row long: broadcast; b undefined: null).  cond: bool or uint8
// tensor of a's length on any device (undefined: always a).
Column SelectVar(const Column &a, const std::optional<Column> &b, const at::Tensor &cond) {
  CYLON_CHECK(a.is_var(), Code::TypeError, "select_var: column " << a.name << " is not variable width");
  const int64_t n = a.length;
  Exec ex(a.device());
  if (b) {
    CYLON_CHECK(b->is_var() && b->type.kind() == a.type.kind(), Code::TypeError,
                "select_var: the other column must have the type of " << a.name);
    CYLON_CHECK(b->length == n || b->length == 1, Code::Invalid,
                "select_var: other has " << b->length << " rows, want " << n << " or 1");
    CYLON_CHECK(b->device() == a.device(), Code::Invalid, "select_var: columns on different devices");
  }
  at::Tensor c;
  if (cond.defined()) {
    CYLON_CHECK(cond.numel() == n, Code::Invalid, "select_var: condition has " << cond.numel() << " rows, want " << n);
    c = cond.to(ex.device, at::kByte).contiguous();
  }
  ColView av = a.view(), bv{};
  const int bcast = b && b->length == 1 && n != 1 ? 1 : 0;
  if (b) bv = b->view();
  const uint8_t *cp = c.defined() ? ptr<uint8_t>(c) : nullptr;
  at::Tensor lens = ex.empty_i64(n);
  KCALL(ex, select_var_lengths, av, bv, bcast, cp, n, ptr<int64_t>(lens));
  at::Tensor offs = exclusive_scan(ex, lens);
  const int64_t total = read_i64(offs, n);
  at::Tensor bytes = ex.empty_bytes(total);
  const bool may_null = a.nullable() || !b || b->nullable();
  at::Tensor valid = may_null ? ex.empty_u8(n) : at::Tensor();
  KCALL(ex, select_var_bytes, av, bv, bcast, cp, n, ptr<int64_t>(offs), ptr<uint8_t>(bytes),
        valid.defined() ? ptr<uint8_t>(valid) : nullptr);
  return Column(a.name, a.type, n, bytes, offs, valid);
}

std::optional<Column> CastStringToNumber(const Column &c, const DataType &target) {
  CYLON_CHECK(c.type.type == Type::STRING || c.type.type == Type::BINARY, Code::TypeError,
              "cast: column " << c.name << " is not a string column");
  const ValueKind k = target.kind();
  CYLON_CHECK(!target.is_variable_width() && (k == ValueKind::SIGNED_INT || k == ValueKind::UNSIGNED_INT ||
                                              k == ValueKind::FLOAT) && target.type != Type::BOOL,
              Code::TypeError, "cast: string -> " << target.ToString() << " is not a numeric cast");
  Exec ex(c.device());
  const int64_t n = c.length;
  at::Tensor ok = ex.empty_u8(std::max<int64_t>(n, 1));
  at::Tensor v;
  const bool fl = k == ValueKind::FLOAT;
  if (fl) {
    v = at::empty({n}, ex.opts(at::kDouble));
    KCALL(ex, str_to_f64, c.view(), n, ptr<double>(v), ptr<uint8_t>(ok));
  } else {
    v = ex.empty_i64(n);
    KCALL(ex, str_to_i64, c.view(), n, ptr<int64_t>(v), ptr<uint8_t>(ok));
  }
  if (n) {
    at::Tensor okn = ok.slice(0, 0, n);
    const std::vector<int64_t> st = to_host_vec(at::stack({(okn == 0).sum(), (okn == 2).sum()}));
    CYLON_CHECK(st[0] == 0, Code::Invalid, "cast: " << st[0] << " value(s) of column " << c.name
                                                     << " do not parse as " << target.ToString());
    if (st[1] != 0) return std::nullopt;  // host parser (hex integers, long or special floats)
  }
  at::Tensor live = c.nullable() ? v.masked_select(c.validity.to(at::kBool)) : v;
  if (!fl && target.width() < 8 && live.numel()) {  // range check of the narrower integer
    const std::vector<int64_t> mm = to_host_vec(at::stack({live.min(), live.max()}));
    const int bits = 8 * target.width();
    const int64_t lo = k == ValueKind::SIGNED_INT ? -(int64_t(1) << (bits - 1)) : 0;
    const int64_t hi = k == ValueKind::SIGNED_INT ? (int64_t(1) << (bits - 1)) - 1 : (int64_t(1) << bits) - 1;
    CYLON_CHECK(mm[0] >= lo && mm[1] <= hi, Code::Invalid,
                "cast: integer value out of range for " << target.ToString() << " in column " << c.name);
  }
  if (!fl && k == ValueKind::UNSIGNED_INT && live.numel())
    CYLON_CHECK(live.min().item<int64_t>() >= 0, Code::Invalid,
                "cast: negative value for " << target.ToString() << " in column " << c.name);
  at::Tensor out = v.to(storage_dtype(target)).contiguous();
  return Column(c.name, target, n, out, at::Tensor(), c.validity);
}

Column CastIntegerToString(const Column &c, const DataType &target) {
  CYLON_CHECK(target.type == Type::STRING, Code::TypeError, "cast: integer -> string only");
  CYLON_CHECK(!c.is_var() && (c.type.kind() == ValueKind::SIGNED_INT || c.type.kind() == ValueKind::UNSIGNED_INT) &&
                  c.type.type != Type::BOOL && !(c.type.kind() == ValueKind::UNSIGNED_INT && c.type.width() == 8) &&
                  c.type.type >= Type::UINT8 && c.type.type <= Type::INT64,
              Code::TypeError, "cast: " << c.type.ToString() << " -> string is not an integer cast");
  Exec ex(c.device());
  const int64_t n = c.length;
  at::Tensor v = c.data.to(at::kLong).contiguous();
  const uint8_t *valid = c.nullable() ? ptr<uint8_t>(c.validity) : nullptr;
  at::Tensor lens = ex.empty_i64(n);
  KCALL(ex, i64_to_str_lengths, ptr<int64_t>(v), valid, n, ptr<int64_t>(lens));
  at::Tensor offs = exclusive_scan(ex, lens);
  at::Tensor bytes = ex.empty_bytes(read_i64(offs, n));
  KCALL(ex, i64_to_str_write, ptr<int64_t>(v), valid, n, ptr<int64_t>(offs), ptr<uint8_t>(bytes));
  return Column(c.name, target, n, bytes, offs, c.validity);
}

// Gather every column of a table with one fused launch per 16 fixed-width
// columns; var-width columns take the two-pass path.
static std::vector<Column> gather_columns(const std::vector<Column> &cols, const at::Tensor &idx, bool may_null) {
  CYLON_CHECK(idx.scalar_type() == at::kLong, Code::TypeError, "gather index must be int64");
  std::vector<Column> out(cols.size());
  if (cols.empty()) return out;
  Exec ex(cols[0].device());
  at::Tensor ix = idx.device() == ex.device ? idx.contiguous() : idx.to(ex.device).contiguous();
  const int64_t m = ix.numel();
  std::vector<ColView> ins;
  std::vector<MutColView> outs;
  std::vector<size_t> fixed_pos;
  for (size_t i = 0; i < cols.size(); ++i) {
    const Column &c = cols[i];
    if (c.is_var()) {
      out[i] = gather_var(ex, c, ix, may_null);
      continue;
    }
    Column o = make_fixed_column(c.name, c.type, m, ex.device, c.nullable() || may_null);
    ColView v = c.view();
    MutColView mv;
    mv.data = m ? reinterpret_cast<uint8_t *>(o.data.data_ptr()) : nullptr;
    mv.valid = o.validity.defined() ? ptr<uint8_t>(o.validity) : nullptr;
    mv.width = v.width;
    mv.kind = v.kind;
    ins.push_back(v);
    outs.push_back(mv);
    fixed_pos.push_back(i);
    out[i] = std::move(o);
  }
  if (!ins.empty() && m > 0)
    KCALL(ex, gather_columns, ins.data(), outs.data(), (int)ins.size(), ptr<int64_t>(ix), m);
  return out;
}

Column GatherColumn(const Column &c, const at::Tensor &idx) { return gather_columns({c}, idx, true)[0]; }

TablePtr Gather(const TablePtr &t, const at::Tensor &idx) {
  // -1 entries make the output nullable only if the caller may pass them; we
  // check cheaply: int64 min over the index is one reduction.
  bool may_null = false;
  if (idx.numel() > 0) may_null = idx.min().item<int64_t>() < 0;
  return Table::Make(t->GetContext(), gather_columns(t->columns(), idx, may_null));
}

TablePtr GatherNullable(const TablePtr &t, const at::Tensor &idx, bool may_null) {
  return Table::Make(t->GetContext(), gather_columns(t->columns(), idx, may_null));
}

at::Tensor MaskToIndices(const at::Tensor &mask, bool invert) {
  Exec ex(mask.device());
  at::Tensor mk = mask.scalar_type() == at::kBool ? mask.view(at::kByte) : mask;
  CYLON_CHECK(mk.scalar_type() == at::kByte, Code::TypeError, "mask must be bool or uint8");
  mk = mk.contiguous();
  const int64_t n = mk.numel();
  at::Tensor ws = ex.empty_i64(KSIZE(ex, mask_to_indices_workspace, n));
  at::Tensor out = ex.empty_i64(n);
  at::Tensor cnt = ex.empty_i64(1);
  KCALL(ex, mask_to_indices, ptr<uint8_t>(mk), n, invert, ptr<int64_t>(ws), ptr<int64_t>(out), ptr<int64_t>(cnt));
  const int64_t k = read_i64(cnt, 0);
  return out.slice(0, 0, k);
}

TablePtr FilterByMask(const TablePtr &t, const at::Tensor &mask) {
  CYLON_CHECK(mask.numel() == t->Rows(), Code::Invalid,
              "mask length " << mask.numel() << " != table rows " << t->Rows());
  at::Tensor idx = MaskToIndices(mask.device() == t->device() ? mask : mask.to(t->device()));
  return GatherNullable(t, idx, false);
}

TablePtr Project(const TablePtr &t, const std::vector<int> &cols) {
  std::vector<Column> out;
  for (int c : cols) out.push_back(t->column(c));
  return Table::Make(t->GetContext(), std::move(out));
}

TablePtr Slice(const TablePtr &t, int64_t offset, int64_t length) {
  std::vector<Column> out;
  for (const auto &c : t->columns()) out.push_back(c.slice(offset, length));
  return Table::Make(t->GetContext(), std::move(out));
}

// Concatenation of contiguous buffers into one allocation: all parts of all columns
// are moved by ONE batched copy launch (kernels/copy.hip: 16-byte vectors, every copy
// in flight at once) -- at::cat's batched kernel and the runtime's blit copy both ran
// the 1B-row union's concatenation at ~2-2.4 TB/s (profiles/suite_cfg6_*).
struct CopyPlan {
  std::vector<const void *> src;
  std::vector<void *> dst;
  std::vector<int64_t> bytes;
  std::vector<at::Tensor> keep;  // contiguous copies of strided parts, alive until launch
};

static at::Tensor concat_buffers(const std::vector<at::Tensor> &parts, CopyPlan &plan) {
  int64_t n = 0;
  for (const auto &p : parts) n += p.numel();
  at::Tensor out = at::empty({n}, parts[0].options());
  const int64_t es = out.element_size();
  uint8_t *dst = n ? reinterpret_cast<uint8_t *>(out.data_ptr()) : nullptr;
  for (const auto &p0 : parts) {
    const at::Tensor p = p0.contiguous();
    const int64_t nb = p.numel() * es;
    if (nb == 0) continue;
    plan.keep.push_back(p);
    plan.src.push_back(p.data_ptr());
    plan.dst.push_back(dst);
    plan.bytes.push_back(nb);
    dst += nb;
  }
  return out;
}

static Column concat_columns(const std::vector<const Column *> &parts, CopyPlan &plan) {
  const Column &f = *parts[0];
  int64_t n = 0;
  bool nullable = false;
  for (auto *p : parts) {
    n += p->length;
    nullable |= p->nullable();
  }
  at::Tensor valid;
  if (nullable) {
    std::vector<at::Tensor> vs;
    for (auto *p : parts)
      vs.push_back(p->nullable() ? p->validity.slice(0, 0, p->length)
                                 : at::ones({p->length}, p->data.options().dtype(at::kByte)));
    valid = concat_buffers(vs, plan);
  }
  if (!f.is_var()) {
    std::vector<at::Tensor> ds;
    for (auto *p : parts) ds.push_back(p->data);
    return Column(f.name, f.type, n, concat_buffers(ds, plan), at::Tensor(), valid);
  }
  std::vector<at::Tensor> bs, os;
  int64_t base = 0;
  for (size_t i = 0; i < parts.size(); ++i) {
    const Column *p = parts[i];
    bs.push_back(p->data);
    at::Tensor o = p->offsets.slice(0, i == 0 ? 0 : 1, p->length + 1) + base;
    os.push_back(o);
    base += p->data.numel();
  }
  return Column(f.name, f.type, n, at::cat(bs), at::cat(os), valid);
}

TablePtr Merge(const std::vector<TablePtr> &tables) {
  CYLON_CHECK(!tables.empty(), Code::Invalid, "merge of zero tables");
  const TablePtr &f = tables[0];
  for (const auto &t : tables)
    CYLON_CHECK(same_schema(f, t), Code::Invalid, "merge: tables must have identical schemas");
  if (tables.size() == 1) return f;
  std::vector<Column> out;
  CopyPlan plan;
  for (int c = 0; c < f->Columns(); ++c) {
    std::vector<const Column *> parts;
    for (const auto &t : tables) parts.push_back(&t->column(c));
    out.push_back(concat_columns(parts, plan));
  }
  if (!plan.src.empty()) {
    Exec ex(f->device());
    KCALL(ex, batched_copy, plan.src.data(), plan.dst.data(), plan.bytes.data(), (int)plan.src.size());
  }
  return Table::Make(f->GetContext(), std::move(out));
}

}  // namespace ops
}  // namespace cylon
