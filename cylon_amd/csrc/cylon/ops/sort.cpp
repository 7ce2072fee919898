// Sorting (K6) and the sort-merge join pair generator (K7).
// Reference: cpp/src/cylon/table.cpp:291-328 (Sort), util/arrow_utils.cpp:30-108
// (SortTable / SortTableMultiColumns), join/sort_join.cpp:576-722.
//
// Multi-column order = LSD over columns: the permutation is refined by stable
// radix sorts from the least significant sort column to the most significant
// one.  Nulls sort last within each column (pandas na_position='last').
// Strings sort by stable passes over their length and then their 8-byte
// big-endian chunks from the last chunk to the first, which yields byte-wise
// lexicographic order.
#include "cylon/knobs.hpp"
#include <limits>
#include <cstdlib>

#include <atomic>
#include <cmath>

#include "util.hpp"
#include "../trace.hpp"

namespace cylon {
namespace ops {

std::pair<at::Tensor, at::Tensor> RadixSortPairs(const Exec &ex, at::Tensor keys, at::Tensor vals, int end_bit) {
  const int64_t n = keys.numel();
  at::Tensor ka = at::empty_like(keys), va = at::empty_like(vals);
  at::Tensor ws = ex.empty_i64(KSIZE(ex, radix_sort_workspace, n));
  const int which = KCALL(ex, radix_sort_pairs, reinterpret_cast<uint64_t *>(ptr<int64_t>(keys)), ptr<int64_t>(vals), n,
                          reinterpret_cast<uint64_t *>(ptr<int64_t>(ka)), ptr<int64_t>(va), 0, end_bit,
                          ptr<int64_t>(ws));
  return which ? std::make_pair(ka, va) : std::make_pair(keys, vals);
}

static at::Tensor iota(const Exec &ex, int64_t n) {
  at::Tensor p = ex.empty_i64(n);
  KCALL(ex, iota, ptr<int64_t>(p), n, 0);
  return p;
}

// stable: rows whose column value is null move to the end, order otherwise kept
static at::Tensor nulls_last(const Exec &ex, const Column &c, const at::Tensor &perm) {
  if (!c.nullable()) return perm;
  at::Tensor v = c.validity.index_select(0, perm);
  at::Tensor valid_pos = MaskToIndices(v, false);
  if (valid_pos.numel() == perm.numel()) return perm;
  at::Tensor null_pos = MaskToIndices(v, true);
  return at::cat({perm.index_select(0, valid_pos), perm.index_select(0, null_pos)});
}

static at::Tensor refine_by_column(const Exec &ex, const Column &c, at::Tensor perm, bool asc, bool grouping = false);

// bytes [off, off + width of t) of every row of a fixed-width column as a contiguous
// column of numeric type t (the validity of the source column)
static Column fixed_slice(const Column &c, int64_t off, const DataType &t) {
  const int64_t w = c.type.width(), n = c.length;
  at::Tensor b = c.data.view(at::kByte).slice(0, 0, n * w).reshape({n, w}).slice(1, off, off + t.width());
  return Column(c.name, t, n, b.contiguous().view(storage_dtype(t)).reshape({n}), at::Tensor(), c.validity);
}

// fixed-size binary: byte-wise (memcmp) order, through the variable-width path over
// synthetic offsets i * width.  DECIMAL (little-endian two's complement, 16 or 32
// bytes): numeric order -- LSD over 8-byte limbs, unsigned below the top limb, signed
// top limb.  FIXED_SIZE_LIST<numeric>: lexicographic element-wise numeric order --
// LSD over the elements.  (Byte order would put 256 before 1 and negatives last.)
static at::Tensor refine_fixed_bytes(const Exec &ex, const Column &c, at::Tensor perm, bool asc) {
  const int64_t w = c.type.width();
  if (c.type.type == Type::DECIMAL) {
    CYLON_CHECK(w % 8 == 0 && w >= 8, Code::NotImplemented, "sort by a decimal of " << w << " bytes");
    for (int64_t limb = 0; limb < w / 8; ++limb) {
      const bool top = limb == w / 8 - 1;
      perm = refine_by_column(ex, fixed_slice(c, 8 * limb, DataType(top ? Type::INT64 : Type::UINT64)), perm, asc);
    }
    return perm;
  }
  if (c.type.type == Type::FIXED_SIZE_LIST) {
    const DataType et(c.type.value_type);
    for (int64_t e = (int64_t)c.type.list_size - 1; e >= 0; --e)
      perm = refine_by_column(ex, fixed_slice(c, e * et.width(), et), perm, asc);
    return c.type.list_size > 0 ? perm : nulls_last(ex, c, perm);
  }
  at::Tensor offs = at::arange(0, (c.length + 1) * w, w, ex.opts(at::kLong));
  Column v(c.name, DataType(Type::BINARY), c.length, c.data, offs, c.validity);
  return refine_by_column(ex, v, std::move(perm), asc);
}

// grouping: the order only has to bring equal values together (group ids, distinct rows), so
// list columns may use their byte order there; a user-visible sort by a list column is refused
static at::Tensor refine_by_column(const Exec &ex, const Column &c, at::Tensor perm, bool asc, bool grouping) {
  const int64_t n = perm.numel();
  CYLON_CHECK(grouping || c.type.type != Type::LIST, Code::NotImplemented, "sort by a list column (" << c.name << ")");
  if (!c.is_var() && c.type.kind() == ValueKind::FIXED_BYTES) return refine_fixed_bytes(ex, c, std::move(perm), asc);
  if (!c.is_var()) {
    at::Tensor keys = ex.empty_i64(n);
    KCALL(ex, sort_keys_from_column, c.view(), ptr<int64_t>(perm), n, !asc,
          reinterpret_cast<uint64_t *>(ptr<int64_t>(keys)));
    perm = RadixSortPairs(ex, keys, perm, 8 * c.type.width()).second;
    return nulls_last(ex, c, perm);
  }
  // strings: length pass, then chunks from last to first
  at::Tensor lens = c.offsets.slice(0, 1, c.length + 1) - c.offsets.slice(0, 0, c.length);
  const int64_t maxlen = c.length ? lens.max().item<int64_t>() : 0;
  const int64_t nchunks = (maxlen + 7) / 8;
  for (int64_t ch = -1; ch < nchunks; ++ch) {
    const int64_t chunk = ch < 0 ? -1 : nchunks - 1 - ch;
    at::Tensor keys = ex.empty_i64(n);
    KCALL(ex, sort_string_chunk_keys, c.view(), ptr<int64_t>(perm), n, chunk, !asc,
          reinterpret_cast<uint64_t *>(ptr<int64_t>(keys)));
    perm = RadixSortPairs(ex, keys, perm, 64).second;
  }
  return nulls_last(ex, c, perm);
}

at::Tensor SortIndices(const TablePtr &t, const std::vector<int> &cols, const std::vector<bool> &ascending,
                       bool grouping) {
  CYLON_CHECK(!cols.empty(), Code::Invalid, "sort needs at least one column");
  CYLON_CHECK(ascending.size() == cols.size() || ascending.size() == 1, Code::Invalid,
              "ascending flags must match sort columns");
  Exec ex(t->device());
  CYLON_PHASE("sort.indices", ex.device);
  at::Tensor perm = iota(ex, t->Rows());
  for (int k = (int)cols.size() - 1; k >= 0; --k) {
    const bool asc = ascending.size() == 1 ? ascending[0] : ascending[k];
    perm = refine_by_column(ex, t->column(cols[k]), perm, asc, grouping);
  }
  return perm;
}

// Large single-key sorts on the GPU: LSD passes over the key's order image
// that move every column (radix_join.hip k_rows_pass with an image digit)
// instead of sorting (image, row) pairs and gathering each column at random
// afterwards (~50 G random accesses/s, profiles/membench.txt).  Constant
// leading/trailing bits of the image are skipped (OR ^ AND reduction).
static std::atomic<bool> g_msd_sort{true};  // A/B hook (SetMsdSort)
void SetMsdSort(bool on) { g_msd_sort.store(on); }
static bool msd_sort_on() { return g_msd_sort.load(); }

static int64_t radix_sort_min_rows() {
  return knobs::Int("RADIX_SORT_MIN_ROWS", int64_t(1) << 22);
}

// Keys-only sorts of 8-byte integers (a one-column table): two MSD slot passes over the top digits
// of image - min, then one LDS sort of every final partition by the bits below them
// (kernels/seg_sort.hip): the keys cross HBM three times instead of once per 9-bit LSD pass (seven
// for keys spanning 63 bits).  Every partition must fit the LDS (slot <= seg_sort_capacity()); keys
// whose top digits are skewed overflow a slot, and the LSD passes sort instead (nullptr).
static TablePtr radix_sort_keys_msd(const Exec &ex, const TablePtr &t, const Column &kc, uint64_t key_xor,
                                    uint64_t img_min, uint64_t img_max) {
  const int64_t n = t->Rows();
  if (img_max <= img_min || !hip::lds_lane_order_ok(ex.stream)) return nullptr;
  const int hr = 64 - __builtin_clzll(img_max - img_min);
  // the keys fill [0, span) of the digits' [0, 2^hr): a bucket of an occupied range holds 1 / fill
  // times the mean (keys in [-3e6, 3e6) x 977 span 33 bits at fill 0.68)
  const double fill = std::max(0.5, (double)(img_max - img_min) / std::ldexp(1.0, hr));
  auto slot_for = [](double mean) { return ((int64_t)(mean + 8.0 * std::sqrt(mean) + 64.0) + 7) & ~int64_t(7); };
  const int64_t cap = hip::seg_sort_capacity();
  auto mean_of = [&](int64_t buckets) { return (double)n / ((double)buckets * fill); };
  int bits = 11;
  while (bits < 19 && slot_for(mean_of(int64_t(1) << bits)) > cap) ++bits;
  const int64_t slot = slot_for(mean_of(int64_t(1) << bits));
  const int db2 = std::min(9, bits / 2), db1 = bits - db2;
  if (slot > cap || bits > hr || !hip::radix_slot_eligible(n, 1, db1, db2)) return nullptr;
  CYLON_PHASE("sort.radix_msd", ex.device);
  const int64_t nb1 = int64_t(1) << db1, nparts = int64_t(1) << bits, tail = hip::radix_slot_tile_rows();
  // first pass into (XCD, bucket) slots when the second pass's segment table holds 8 x 2^db1 of them,
  // else exact (2B keys: 19 bits = 10 + 9)
  const bool slot1 = hip::radix_slot_first_pass_ok(db1);
  const int64_t s1 = slot1 ? slot_for(mean_of(8 * nb1)) : 0;
  at::Tensor ovf = at::zeros({1}, ex.opts(at::kInt));
  unsigned int *ov = reinterpret_cast<unsigned int *>(ovf.data_ptr<int>());
  at::Tensor mid = ex.empty_i64(slot1 ? 8 * nb1 * s1 + tail : n), cnt1 = slot1 ? ex.empty_i64(8 * nb1) : at::Tensor();
  at::Tensor ws = ex.empty_i64(slot1 ? hip::radix_slot_workspace(db1, db2) : hip::radix_rows_pass_workspace(n, db1));
  hip::radix_sort_msd_first_pass(ptr<int64_t>(kc.data), n, hr, db1, db2, key_xor, img_min, ptr<int64_t>(mid), s1,
                                 ptr<int64_t>(ws), slot1 ? ptr<int64_t>(cnt1) : nullptr, ov, ex.stream);
  at::Tensor fin = ex.empty_i64(nparts * slot + tail), counts = ex.empty_i64(nparts);
  at::Tensor ws2 = ex.empty_i64(hip::radix_slot_workspace(db1, db2));
  hip::radix_sort_msd_second_pass(ptr<int64_t>(mid), n, hr, db1, db2, img_min, ptr<int64_t>(ws),
                                  slot1 ? ptr<int64_t>(cnt1) : nullptr, s1, ptr<int64_t>(fin), slot, ptr<int64_t>(ws2),
                                  ptr<int64_t>(counts), ov, ex.stream);
  mid = at::Tensor();
  if (ovf.item<int>() != 0) {  // a partition outgrew its slot: skewed top digits
    trace::add_counter("sort.radix.msd_slot_overflow", 1);
    return nullptr;
  }
  at::Tensor offs = exclusive_scan(ex, counts);
  at::Tensor out = at::empty_like(kc.data);
  hip::seg_sort_local(ptr<int64_t>(fin), ptr<int64_t>(counts), slot, nparts, ptr<int64_t>(offs), img_min, hr - bits,
                      key_xor, ptr<int64_t>(out), ex.stream);
  trace::add_counter("sort.radix.msd", 1);
  return Table::Make(t->GetContext(), {Column(kc.name, kc.type, n, out)});
}

static TablePtr radix_sort_table(const TablePtr &t, int col, bool asc) {
  const int64_t n = t->Rows();
  if (!t->device().is_cuda() || n < radix_sort_min_rows()) return nullptr;
  const Column &kc = t->column(col);
  if (kc.nullable() || kc.is_var() || kc.type.kind() == ValueKind::FIXED_BYTES) return nullptr;
  int slots = 1;
  for (const auto &c : t->columns()) {
    const int w = c.type.width();
    if (c.is_var() || c.type.kind() == ValueKind::FIXED_BYTES || !(w == 1 || w == 2 || w == 4 || w == 8) ||
        c.data.element_size() != w)
      return nullptr;
    slots += 1 + (c.nullable() ? 1 : 0);
  }
  if (slots > kMaxFusedCols) return nullptr;
  Exec ex(t->device());
  CYLON_PHASE("sort.radix_rows", ex.device);
  // an integer key is rebuilt from its image at the end instead of travelling too
  const bool key_from_image = kc.type.kind() == ValueKind::SIGNED_INT || kc.type.kind() == ValueKind::UNSIGNED_INT;
  // an 8-byte integer key's image is key ^ key_xor: the first pass reads the raw keys (its digit
  // XORs them) and stores images, so the image kernel only reduces (no 8 B/row image write)
  const uint64_t key_xor = (kc.type.kind() == ValueKind::SIGNED_INT ? (1ull << 63) : 0ull) ^ (asc ? 0ull : ~0ull);
  const bool raw_in = key_from_image && kc.type.width() == 8 && kc.data.is_contiguous() &&
                      kc.data.element_size() == 8;
  at::Tensor img = raw_in ? kc.data : ex.empty_i64(n);
  at::Tensor ws2 = ex.empty_i64(2);
  // raw 8-byte integer keys on the XCD-tile passes: one read gives the varying bits AND the first
  // pass's per-tile histogram (bits [0, 10) of the image), folded below when the pass digit starts
  // at bit 0 -- the separate reduction read every key once more (3.3 ms of a 2B-row sort)
  const bool prehist = raw_in && n > 0;
  at::Tensor pre_ws;
  uint64_t diff, img_min = 0, img_max = 0;
  if (prehist) {
    pre_ws = ex.empty_i64(hip::radix_sort_prehist_workspace(n));
    diff = hip::radix_sort_prehist(ptr<int64_t>(kc.data), n, key_xor, ptr<int64_t>(pre_ws), ex.stream, &img_min,
                                   &img_max);
  } else {
    diff = hip::sort_keys_varying_bits(kc.view(), n, !asc,
                                       raw_in ? nullptr : reinterpret_cast<uint64_t *>(ptr<int64_t>(img)),
                                       ptr<int64_t>(ws2), ex.stream);
  }
  if (prehist && diff != 0 && t->Columns() == 1 && key_from_image && msd_sort_on())
    if (TablePtr r = radix_sort_keys_msd(ex, t, kc, key_xor, img_min, img_max)) return r;
  std::vector<at::Tensor> cur{img};
  std::vector<int> widths{8};
  for (int ci = 0; ci < t->Columns(); ++ci) {
    const Column &c = t->column(ci);
    if (!(key_from_image && ci == col)) {
      cur.push_back(c.data);
      widths.push_back(c.type.width());
    }
    if (c.nullable()) {
      cur.push_back(c.validity);
      widths.push_back(1);
    }
  }
  // an 8-byte integer key comes back from its image by one XOR, applied by the last
  // pass as it stores column 0 (no separate un-image read + write of the key)
  const bool key_in_last_pass = key_from_image && kc.type.width() == 8 && diff != 0;
  // validity bytes of an otherwise all-8-byte table travel packed (8-byte pass path)
  BytePacking bp;
  if (diff != 0) bp = PackByteColumns(ex, cur, widths, n);
  if (diff != 0) {
    const int lo = __builtin_ctzll(diff);
    int hi = 64 - __builtin_clzll(diff);
    // digits of image - min when the keys span fewer bits than vary (every image agrees with the
    // minimum below bit lo, so image - min keeps those bits zero)
    uint64_t sub = 0;
    if (prehist && img_max > img_min) {
      const int hr = 64 - __builtin_clzll(img_max - img_min);
      if (hr < hi) {
        sub = img_min;
        hi = hr;
        trace::add_counter("sort.radix.sub_min", 1);
      }
    }
    const int npass = (hi - lo + 9) / 10;
    std::vector<int> shifts, dbits;
    int max_db = 0;
    for (int ps = 0, sh = lo; ps < npass; ++ps) {
      const int db = (hi - sh + (npass - ps) - 1) / (npass - ps);
      shifts.push_back(sh);
      dbits.push_back(db);
      max_db = std::max(max_db, db);
      sh += db;
    }
    at::Tensor ws;
    // each pass but the last writes the next pass's digits (2 B/row) as it stores the keys: the
    // next pass's tile histogram then reads those instead of the 8-byte keys (XCD-tile passes)
    // look-back passes (1-2 all-8-byte columns): no tile histograms and no next-digit array at all
    const bool lb_on = hip::radix_sort_lb_eligible(n, (int)cur.size(), widths.data(), dbits.data(), npass, ex.stream);
    const bool nd_on = !lb_on && npass > 1;
    at::Tensor nd = nd_on ? at::empty({n}, ex.opts(at::kShort)) : at::Tensor();
    at::Tensor lbws = lb_on ? ex.empty_i64(hip::radix_sort_lb_workspace(n)) : at::Tensor();
    if (lb_on) trace::add_counter("sort.radix.lookback", 1);
    int shift = lo;
    for (int ps = 0; ps < npass; ++ps) {
      const int db = dbits[ps];
      const int64_t wsn = hip::radix_rows_pass_workspace(n, db);
      if (!ws.defined() || ws.numel() < wsn) ws = ex.empty_i64(wsn);
      std::vector<at::Tensor> nxt;
      std::vector<const uint8_t *> in;
      std::vector<uint8_t *> out;
      for (auto &x : cur) {
        nxt.push_back(at::empty_like(x));
        in.push_back(reinterpret_cast<const uint8_t *>(x.data_ptr()));
        out.push_back(reinterpret_cast<uint8_t *>(nxt.back().data_ptr()));
      }
      // the XOR goes on the FINAL pass only: a pass reads column 0 as the order image it
      // ranks by, so an un-imaged key column must never be the input of another pass
      // raw_in: the first pass ranks key ^ key_xor and stores it (raw -> image); the last
      // pass XORs again (image -> raw); one pass does both (stores the raw key)
      const uint64_t flip = ps == 0 && raw_in ? key_xor : 0ull;
      const bool pre = prehist && ps == 0 && shift == 0 && db <= 10;
      if (pre) hip::radix_sort_prehist_fold(ptr<int64_t>(pre_ws), n, db, ptr<int64_t>(ws), ex.stream, sub);
      uint16_t *ndp = nd_on ? reinterpret_cast<uint16_t *>(nd.data_ptr()) : nullptr;
      SortLbArgs lba{};
      if (lb_on) lba = hip::radix_sort_lb_args(ptr<int64_t>(lbws), n, ps, npass, ex.stream);
      hip::radix_sort_rows_pass(ptr<int64_t>(cur[0]), n, shift, db, in.data(), out.data(), widths.data(),
                                (int)cur.size(), ptr<int64_t>(ws), ex.stream,
                                flip ^ (ps + 1 == npass && key_in_last_pass ? key_xor : 0ull), flip, pre,
                                ps > 0 ? ndp : nullptr, ps + 1 < npass ? ndp : nullptr, shift + db,
                                ps + 1 < npass ? dbits[ps + 1] : 0, sub, lb_on ? &lba : nullptr);
      if (ps == 0) pre_ws = at::Tensor();  // 10-bit tile histogram consumed
      cur = std::move(nxt);
      shift += db;
    }
    cur = UnpackByteColumns(ex, bp, std::move(cur), n);
    if (lb_on && hip::radix_sort_lb_failed(ptr<int64_t>(lbws), ex.stream)) {  // never expected
      trace::add_counter("sort.radix.lookback_timeout_fallback", 1);
      hip::rp_take_order_violation(ex.stream);
      return nullptr;
    }
    if (hip::rp_take_order_violation(ex.stream)) {  // ranking guard: index sort instead
      trace::add_counter("sort.radix.order_violation_fallback", 1);
      return nullptr;
    }
  }
  std::vector<Column> cols;
  size_t q = 1;
  for (int ci = 0; ci < t->Columns(); ++ci) {
    const Column &c = t->column(ci);
    at::Tensor d;
    if (key_in_last_pass && ci == col) {
      d = cur[0].view(c.data.scalar_type());
    } else if (raw_in && ci == col) {  // all keys equal (no pass ran): column 0 is still the raw key
      d = cur[0].view(c.data.scalar_type());
    } else if (key_from_image && ci == col) {
      at::Tensor im = cur[0];
      if (!asc) {
        const int nb = 8 * c.type.width();
        const int64_t mask = nb == 64 ? -1 : (int64_t)((1ull << nb) - 1);
        im = at::bitwise_and(at::bitwise_not(im), mask);
      }
      d = at::empty_like(c.data);
      hip::agg_unimage(reinterpret_cast<const uint64_t *>(ptr<int64_t>(im)), n, c.type.width(),
                       static_cast<int>(c.type.kind()), reinterpret_cast<uint8_t *>(d.data_ptr()), ex.stream);
    } else {
      d = cur[q++];
    }
    at::Tensor v = c.nullable() ? cur[q++] : at::Tensor();
    cols.emplace_back(c.name, c.type, n, d, at::Tensor(), v);
  }
  return Table::Make(t->GetContext(), std::move(cols));
}

// config "verify_sort" = "1" (or CYLON_VERIFY_SORT=1): one read of the first sort column's
// order images checks that the result is non-decreasing in the requested order
static void verify_sorted(const TablePtr &out, int col, bool asc) {
  auto ctx = out->GetContext();
  const std::string v = knobs::ConfigOr(ctx->GetConfig("verify_sort", ""), "VERIFY_SORT");
  if (v != "1" || out->Rows() < 2) return;
  Exec ex(out->device());
  const Column &c = out->column(col);
  const int64_t n = out->Rows();
  if (c.is_var() || c.type.kind() == ValueKind::FIXED_BYTES) return;
  at::Tensor img = ex.empty_i64(n);
  KCALL(ex, sort_keys_from_column, c.view(), nullptr, n, !asc, reinterpret_cast<uint64_t *>(ptr<int64_t>(img)));
  // unsigned order of the images = signed order after flipping the top bit; nulls sort last
  at::Tensor s = at::bitwise_xor(img, at::full({1}, std::numeric_limits<int64_t>::min(), img.options()));
  at::Tensor bad = s.slice(0, 1, n).lt(s.slice(0, 0, n - 1));
  if (c.nullable()) {
    at::Tensor valid = c.validity.slice(0, 0, n).to(at::kBool);
    bad = bad & valid.slice(0, 1, n) & valid.slice(0, 0, n - 1);
    bad = bad | (valid.slice(0, 1, n) & valid.slice(0, 0, n - 1).logical_not());  // a value after a null
  }
  CYLON_CHECK(!bad.any().item<bool>(), Code::ExecutionError, "sort verification failed on column " << c.name);
  trace::add_counter("sort.verified", 1);
}

TablePtr Sort(const TablePtr &t, const std::vector<int> &cols, const std::vector<bool> &ascending) {
  if (t->Rows() <= 1) return t;
  TablePtr out;
  if (cols.size() == 1) out = radix_sort_table(t, cols[0], ascending.empty() ? true : ascending[0]);
  if (!out) out = GatherNullable(t, SortIndices(t, cols, ascending), false);
  verify_sorted(out, cols[0], ascending.empty() ? true : ascending[0]);
  return out;
}

std::pair<at::Tensor, at::Tensor> SortJoinPairs(const Exec &ex, const at::Tensor &lkeys, const at::Tensor &rkeys) {
  const int64_t nl = lkeys.numel(), nr = rkeys.numel();
  auto ls = RadixSortPairs(ex, lkeys.clone(), iota(ex, nl), 64);
  auto rs = RadixSortPairs(ex, rkeys.clone(), iota(ex, nr), 64);
  at::Tensor lo = ex.empty_i64(nl), counts = ex.empty_i64(nl);
  KCALL(ex, merge_join_count, reinterpret_cast<const uint64_t *>(ptr<int64_t>(ls.first)), nl,
        reinterpret_cast<const uint64_t *>(ptr<int64_t>(rs.first)), nr, ptr<int64_t>(lo), ptr<int64_t>(counts));
  at::Tensor offs = exclusive_scan(ex, counts);
  const int64_t m = read_i64(offs, nl);
  at::Tensor ol = ex.empty_i64(m), orr = ex.empty_i64(m);
  KCALL(ex, merge_join_write, ptr<int64_t>(ls.second), nl, ptr<int64_t>(rs.second), ptr<int64_t>(lo),
        ptr<int64_t>(offs), ptr<int64_t>(ol), ptr<int64_t>(orr));
  return {ol, orr};
}

}  // namespace ops
}  // namespace cylon
