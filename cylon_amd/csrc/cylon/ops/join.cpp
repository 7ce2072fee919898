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
#include "cylon/knobs.hpp"
#include <algorithm>
#include <optional>
#include <array>
#include <cmath>
#include <cstdlib>
#include <limits>

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
// Global-table hash join (the path of joins the LDS radix join does not take).  Clustering-free
// directory: the build keys are sorted once, and the open-addressing table holds each DISTINCT key
// once with its head index h; key k's build rows are perm[hstart[h], hstart[h + 1]).  A hot key is
// one slot, so no probe ever walks through its duplicates (a row-per-slot linear-probing multimap
// puts a hot key's duplicates into every nearby key's probe path: primary clustering that grows
// with the hot run's length).  Probes find <= 1 directory entry; the (probe, head) pairs are then
// expanded into (probe, build row) pairs in probe-row order.  Reference: the unordered_multimap of
// join/hash_join.cpp:255-298.
static std::pair<at::Tensor, at::Tensor> hash_join_pairs(const Exec &ex, const at::Tensor &lk, const at::Tensor &rk) {
  const bool build_left = lk.numel() < rk.numel();
  const at::Tensor &bk0 = build_left ? lk : rk;
  const at::Tensor &pk = build_left ? rk : lk;
  const int64_t nb0 = bk0.numel(), np = pk.numel();
  at::Tensor sk, perm, hstart;
  bool distinct = false;
  {
    CYLON_PHASE("join.build.directory", ex.device);
    auto sr = at::sort(bk0);
    sk = std::get<0>(sr);
    perm = std::get<1>(sr);
    at::Tensor head = at::ones({nb0}, ex.opts(at::kBool));
    if (nb0 > 1) head.slice(0, 1, nb0).copy_(sk.slice(0, 1, nb0) != sk.slice(0, 0, nb0 - 1));
    // distinct build keys (the common case): the sorted keys ARE the directory and
    // every head is its own row -- no compaction, and the expansion below is one gather
    distinct = nb0 == 0 || head.all().item<bool>();
    if (!distinct) {
      at::Tensor hpos = head.nonzero().flatten();
      sk = sk.index_select(0, hpos);  // distinct keys, ascending
      hstart = at::cat({hpos, at::full({1}, nb0, ex.opts(at::kLong))});
    }
  }
  const at::Tensor &bk = sk;
  const int64_t nb = bk.numel();
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
    const at::Tensor &sk2 = which ? kb : ka;
    const at::Tensor &sr2 = which ? vb : va;
    const at::Tensor &pm = which ? ka : kb;
    KCALL(ex, hash_table_place, reinterpret_cast<const uint64_t *>(ptr<int64_t>(sk2)), ptr<int64_t>(sr2),
          ptr<int64_t>(pm), nb, t);
  } else {
    table = at::empty({cap * 2}, ex.opts(at::kLong));
    t.slots = reinterpret_cast<HashSlot *>(table.data_ptr());
    KCALL(ex, hash_table_init, t.slots, cap);
    KCALL(ex, hash_build, ptr<int64_t>(bk), nb, t);
  }
  // (probe row, head) pairs: at most one per probe row
  at::Tensor po, ho;
  if (ex.gpu && np >= kEmitProbeRows) {
    CYLON_PHASE("join.probe.emit", ex.device);
    const int64_t capacity = np + 4096;
    po = ex.empty_i64(capacity);
    ho = ex.empty_i64(capacity);
    at::Tensor cnt = ex.empty_i64(1);
    KCALL(ex, hash_probe_emit, ptr<int64_t>(pk), np, t, capacity, ptr<int64_t>(cnt), ptr<int64_t>(po),
          ptr<int64_t>(ho));
    const int64_t m = read_i64(cnt, 0);
    CYLON_CHECK(m <= np, Code::ExecutionError, "directory probe: " << m << " matches for " << np << " probe rows");
    po = po.slice(0, 0, m);
    ho = ho.slice(0, 0, m);
  } else {
    CYLON_PHASE("join.probe.twopass", ex.device);
    at::Tensor counts = ex.empty_i64(np);
    KCALL(ex, hash_probe_count, ptr<int64_t>(pk), np, t, ptr<int64_t>(counts));
    at::Tensor offs = exclusive_scan(ex, counts);
    counts = at::Tensor();
    const int64_t m = read_i64(offs, np);
    po = ex.empty_i64(m);
    ho = ex.empty_i64(m);
    KCALL(ex, hash_probe_write, ptr<int64_t>(pk), np, t, ptr<int64_t>(offs), ptr<int64_t>(po), ptr<int64_t>(ho));
  }
  table = at::Tensor();
  at::Tensor bo;
  {
    CYLON_PHASE("join.probe.expand", ex.device);
    if (distinct) return build_left ? std::make_pair(perm.index_select(0, ho), po)
                                    : std::make_pair(po, perm.index_select(0, ho));
    at::Tensor first = hstart.index_select(0, ho);
    at::Tensor cnt = hstart.index_select(0, ho + 1) - first;
    const int64_t m = po.numel() ? cnt.sum().item<int64_t>() : 0;
    if (m != po.numel()) {  // some key has duplicates: repeat each pair over its key's rows
      at::Tensor excl = cnt.cumsum(0) - cnt;
      po = po.repeat_interleave(cnt, 0, m);
      at::Tensor pos = (first - excl).repeat_interleave(cnt, 0, m) + at::arange(m, ex.opts(at::kLong));
      bo = perm.index_select(0, pos);
    } else {
      bo = perm.index_select(0, first);
    }
  }
  return build_left ? std::make_pair(bo, po) : std::make_pair(po, bo);
}

// ---------------------------------------------------------------------------
// K5 LDS radix join (radix_join.hip): partition both sides, all columns, into
// LDS-sized buckets and join bucket pairs inside one workgroup each, emitting
// the output columns directly.  Used on the GPU for large inner joins on one
// exact key where every column is fixed width <= 8 bytes.
// ---------------------------------------------------------------------------
static int64_t radix_join_min_rows() {
  return knobs::Int("RADIX_JOIN_MIN_ROWS", int64_t(1) << 22);
}

static constexpr int64_t kRadixRowsPerPart = 4096;  // avg build rows per partition (LDS table: 6144 max)

static bool radix_eligible(const TablePtr &t) {
  int slots = 1;
  for (const auto &c : t->columns()) {
    const int w = c.type.width();
    if (c.is_var() || c.type.kind() == ValueKind::FIXED_BYTES || !(w == 1 || w == 2 || w == 4 || w == 8) ||
        c.data.element_size() != w)
      return false;
    slots += 1 + (c.nullable() ? 1 : 0);
  }
  return slots <= kMaxFusedCols;
}

struct RadixSide {
  at::Tensor keys, offs;  // offs: partition offsets [2^bits + 1], or (slot > 0) rows per partition
  int64_t slot = 0;       // slot mode: partition p's rows start at p * slot (RadixPartitionSlotted)
  at::Tensor overflow;    // slot mode: int32 device flag, set when a partition outgrew its slot
  std::vector<at::Tensor> data, valid;  // per table column (valid undefined if not nullable or packed)
  std::vector<bool> is_key;             // data[c] is the (partitioned) key array itself
  // validity bytes kept packed 8 per 8-byte word (radix.cpp): vpos[c] = byte position of
  // column c's validity in the words (-1: not packed); the write kernel moves the words
  std::vector<int> vpos;
  std::vector<at::Tensor> vwords;
};

// partitioned key array (int64, or uint32 offsets when narrowed) as the kernels' pointer
static const int64_t *kptr(const at::Tensor &k) { return reinterpret_cast<const int64_t *>(k.data_ptr()); }

// rows of each partition / its first row in the partitioned arrays (slot mode: p * slot)
static at::Tensor part_counts(const RadixSide &s, int64_t nparts) {
  return s.slot ? s.offs.slice(0, 0, nparts) : s.offs.slice(0, 1, nparts + 1) - s.offs.slice(0, 0, nparts);
}
static at::Tensor part_starts(const RadixSide &s, int64_t nparts) {
  return s.slot ? at::arange(nparts, s.offs.options()) * s.slot : s.offs.slice(0, 0, nparts);
}

// the partition / write kernels move validity packed when every data column is 8 bytes wide
// (the all-8-byte kernel variants; byte runs of 1-byte validity columns cost 2x)
static bool packs_validity(const TablePtr &t) {
  bool any = false;
  for (const auto &c : t->columns()) {
    if (c.type.width() != 8) return false;
    any |= c.nullable();
  }
  return any;
}

// Partition every column of t (+ validity bytes) by the top `bits` bits of fmix64(key).
// slot > 0: try the slot-mode (histogram-free MSD) partition first
static RadixSide radix_partition(const Exec &ex, const TablePtr &t, const at::Tensor &keys, int bits,
                                 const RangeSpec *range = nullptr, int64_t slot = 0,
                                 const hip::NarrowKeys *nk = nullptr) {
  std::vector<at::Tensor> cur{keys};
  std::vector<int> widths{8};
  std::vector<int> dslot(t->Columns(), -1), vslot(t->Columns(), -1);
  for (int c = 0; c < t->Columns(); ++c) {
    const Column &col = t->column(c);
    if (col.type.width() == 8 && col.data.data_ptr() == keys.data_ptr()) {
      dslot[c] = 0;  // the key column itself
    } else {
      dslot[c] = (int)cur.size();
      cur.push_back(col.data);
      widths.push_back(col.type.width());
    }
    if (col.nullable()) {
      vslot[c] = (int)cur.size();
      cur.push_back(col.validity);
      widths.push_back(1);
    }
  }
  at::Tensor offs;
  const size_t nslots = cur.size();
  std::vector<int> packed;
  // hash partitions: the LDS join ignores row order inside a partition, so the first LSD pass
  // ranks with LDS atomics (later passes must keep its order)
  RadixSide s;
  std::vector<at::Tensor> sl;
  if (slot > 0 && !range)
    sl = RadixPartitionSlotted(ex, cur, widths, bits, slot, &offs, &s.overflow,
                               packs_validity(t) ? &packed : nullptr, nk);
  if (!sl.empty()) {
    cur = std::move(sl);
    s.slot = slot;
  } else {
    cur = RadixPartition(ex, std::move(cur), widths, bits, &offs, range, packs_validity(t) ? &packed : nullptr,
                         range != nullptr, nk);
  }
  s.keys = cur[0];
  s.offs = offs;
  for (size_t w = nslots; w < cur.size(); ++w) s.vwords.push_back(cur[w]);
  for (int c = 0; c < t->Columns(); ++c) {
    s.data.push_back(cur[dslot[c]]);
    const bool pk = vslot[c] >= 0 && !s.vwords.empty();
    s.valid.push_back(vslot[c] >= 0 && !pk ? cur[vslot[c]] : at::Tensor());
    int pos = -1;
    if (pk)
      for (size_t j = 0; j < packed.size(); ++j)
        if (packed[j] == vslot[c]) pos = (int)j;
    s.vpos.push_back(pos);
    s.is_key.push_back(dslot[c] == 0);
  }
  return s;
}

// Column pointer lists of one side for the write kernel (nullptr input = key column).
struct RadixCols {
  std::vector<const uint8_t *> in;
  std::vector<uint8_t *> out;
  std::vector<int> w;
};

static RadixCols radix_cols(const TablePtr &t, const RadixSide *s, const std::vector<Column> *outs,
                            int64_t out_off = 0, const std::vector<at::Tensor> *word_outs = nullptr) {
  RadixCols rc;
  const bool packed = s ? !s->vwords.empty() : packs_validity(t);
  int nnull = 0;
  for (int c = 0; c < t->Columns(); ++c) {
    const Column &col = t->column(c);
    rc.in.push_back(s && !s->is_key[c] ? reinterpret_cast<const uint8_t *>(s->data[c].data_ptr())
                                       : (s ? nullptr : reinterpret_cast<const uint8_t *>(1)));
    rc.out.push_back(outs ? reinterpret_cast<uint8_t *>((*outs)[c].data.data_ptr()) + out_off * col.type.width()
                          : nullptr);
    rc.w.push_back(col.type.width());
    if (col.nullable() && packed) {
      ++nnull;
    } else if (col.nullable()) {
      rc.in.push_back(s ? s->valid[c].data_ptr<uint8_t>() : reinterpret_cast<const uint8_t *>(1));
      rc.out.push_back(outs ? (*outs)[c].validity.data_ptr<uint8_t>() + out_off : nullptr);
      rc.w.push_back(1);
    }
  }
  if (packed) {  // the packed validity words, 8 bytes per row (outputs: temporary words)
    const int nw = (nnull + 7) / 8;
    for (int w = 0; w < nw; ++w) {
      rc.in.push_back(s ? reinterpret_cast<const uint8_t *>(s->vwords[w].data_ptr()) : reinterpret_cast<const uint8_t *>(1));
      rc.out.push_back(word_outs ? reinterpret_cast<uint8_t *>((*word_outs)[w].data_ptr()) : nullptr);
      rc.w.push_back(8);
    }
  }
  return rc;
}

// output validity of the packed columns from the written words (at row offset out_off)
static void unpack_validity_words(const Exec &ex, const TablePtr &t, const RadixSide &s,
                                  const std::vector<at::Tensor> &words, std::vector<Column> &outs, int64_t out_off,
                                  int64_t m) {
  if (s.vwords.empty() || m == 0) return;
  std::vector<uint8_t *> dst;
  for (int c = 0; c < t->Columns(); ++c)
    if (s.vpos[c] >= 0) dst.push_back(outs[c].validity.data_ptr<uint8_t>() + out_off);
  std::vector<const uint64_t *> wp;
  for (const auto &w : words) wp.push_back(reinterpret_cast<const uint64_t *>(w.data_ptr()));
  hip::unpack_byte_columns(wp.data(), (int)dst.size(), m, dst.data(), ex.stream);
}

// A bounded-memory join chunk partitioned outside radix_join (radix_join_chunked): both sides'
// partitions (narrowed keys), the chunk's partition bits and the narrowing base's source.
struct PrePartition {
  RadixSide L, R;
  int bits = 0;
  at::Tensor base_src;
  // set by radix_join (nothing written) when a side's slot pass overflowed: the flags ride with
  // radix_join's first host read instead of a read of their own
  mutable bool overflowed = false, overflow_l = false, overflow_r = false;
};

// Output accumulator of a chunked (pipelined) distributed join.  The radix join
// writes every chunk's rows straight into one set of output columns at the
// running row offset (capacity sized from the first chunk's output for all
// chunks, grown geometrically if a later chunk needs more), so the chunked join
// costs no concatenation pass; chunks that take another join path hand over
// whole tables, concatenated once at the end.
struct JoinSink {
  std::vector<Column> cols;  // left columns ++ right columns, `cap` rows each
  int64_t size = 0, cap = 0;
  int chunks_total = 1, chunks_done = 0;
  // the radix join's sampled skew check before its slot passes (off for the bounded-memory chunks:
  // a skewed chunk still completes -- an overflowing slot repartitions that side exactly)
  bool sample_skew = true;
  const PrePartition *pre = nullptr;  // this chunk arrives partitioned (radix_join skips its passes)
  std::vector<TablePtr> tables;

  // room for m more rows; returns the row offset to write at
  int64_t reserve(const Exec &ex, int64_t m, const std::vector<Column> &proto) {
    if (size + m > cap) {
      const int64_t left_chunks = std::max(1, chunks_total - chunks_done);
      const int64_t want = std::max(size + m + (m * (left_chunks - 1)) * 103 / 100 + 4096, 2 * cap);
      std::vector<Column> fresh;
      for (size_t c = 0; c < proto.size(); ++c) {
        Column n = make_fixed_column(proto[c].name, proto[c].type, want, ex.device, proto[c].nullable());
        if (size > 0) {
          n.data.slice(0, 0, size).copy_(cols[c].data.slice(0, 0, size));
          if (n.nullable()) n.validity.slice(0, 0, size).copy_(cols[c].validity.slice(0, 0, size));
        }
        fresh.push_back(std::move(n));
      }
      cols = std::move(fresh);
      cap = want;
    }
    const int64_t off = size;
    size += m;
    return off;
  }

  TablePtr finish(const std::shared_ptr<CylonContext> &ctx) {
    std::vector<TablePtr> parts;
    if (!cols.empty()) {
      std::vector<Column> out;
      for (const auto &c : cols) out.push_back(c.slice(0, size));
      parts.push_back(Table::Make(ctx, std::move(out)));
    }
    for (auto &t : tables) parts.push_back(t);
    if (parts.size() == 1) return parts[0];
    return Merge(parts);
  }
};

// Outer-join mode of the LDS join kernels (kernel_decls.inc radix_join_count): bit 0 = probe rows
// without a match are output rows, bit 1 = build rows without a match are.
static int outer_mode(JoinType jt, bool build_left) {
  const bool lp = jt == JoinType::LEFT || jt == JoinType::FULL_OUTER;
  const bool rp = jt == JoinType::RIGHT || jt == JoinType::FULL_OUTER;
  return ((build_left ? rp : lp) ? 1 : 0) | ((build_left ? lp : rp) ? 2 : 0);
}
static bool left_may_null(JoinType jt) { return jt == JoinType::RIGHT || jt == JoinType::FULL_OUTER; }
static bool right_may_null(JoinType jt) { return jt == JoinType::LEFT || jt == JoinType::FULL_OUTER; }

// validity of the output columns of a side that can be null: the side's presence bytes, AND the
// column's own validity where the input column was nullable.  Without a sink the columns of a
// non-nullable input share the presence bytes as their validity (no per-column copy: a 1B-row
// FULL OUTER join would otherwise hold 8 more bytes per output row); a sink's columns own theirs.
static void apply_presence(std::vector<Column> &cols, const TablePtr &in, const at::Tensor &pres, int64_t off,
                           int64_t m, bool share) {
  at::Tensor p = pres.slice(0, 0, m);
  for (int c = 0; c < in->Columns(); ++c) {
    if (share && !in->column(c).nullable()) {
      cols[c].validity = p;
      continue;
    }
    at::Tensor v = cols[c].validity.slice(0, off, off + m);
    if (in->column(c).nullable()) v.mul_(p);
    else v.copy_(p);
  }
}

// Returns nullptr when a build partition overflows the LDS capacity (heavy key
// skew / duplicates); the caller then runs the global-table join.  With a sink the
// rows are written into the sink's columns and the sink's table is returned.
// Every column of both tables is fixed width (radix_eligible); lk / rk are the int64 join keys
// (a key column itself, or the composite image of several key columns).  All four join types:
// the kernels emit unmatched rows of the preserved side(s) with presence bytes (outer_mode).
static TablePtr radix_join(const Exec &ex, const TablePtr &left, const TablePtr &right, at::Tensor lk, at::Tensor rk,
                           const JoinConfig &cfg, JoinSink *sink = nullptr, bool hashed_key = false) {
  const int64_t nl = left->Rows(), nr = right->Rows();
  const bool build_left = nl < nr;
  const TablePtr &bt = build_left ? left : right;
  const int64_t nb = std::min(nl, nr);
  const JoinType jt = cfg.GetType();
  const int oj = outer_mode(jt, build_left);
  const bool lnull = left_may_null(jt), rnull = right_may_null(jt);
  const PrePartition *pre = sink ? sink->pre : nullptr;  // (tables: schema only, partitions in pre)
  // LDS capacity from the build side's staged row width (key column counted once)
  RadixCols shape = radix_cols(bt, nullptr, nullptr);
  for (int c = 0, q = 0; c < bt->Columns(); ++c, ++q) {
    const Column &col = bt->column(c);
    const bool is_key = pre ? (build_left ? pre->L : pre->R).is_key[(size_t)c]
                            : col.type.width() == 8 && col.data.data_ptr() == (build_left ? lk : rk).data_ptr();
    if (is_key) shape.in[q] = nullptr;
    if (col.nullable() && !packs_validity(bt)) ++q;  // packed validity words sit after the columns
  }
  // Narrowed keys (kernel_decls.inc NarrowKeys): when each side's join key is its own int64 column,
  // the partitions carry it as a uint32 offset from base = (left key 0) - 2^31 -- 4 B/row less in
  // every pass write, the second pass's reads and the join kernel's reads (the headline's 1B x 1B
  // join: 16 of 128 bytes moved per row and side).  A key outside [base, base + 2^32) is detected
  // by the first pass, and the join repartitions without narrowing.
  auto own_key_column = [](const TablePtr &t, const at::Tensor &k) {
    int hits = 0;
    for (const auto &c : t->columns())
      hits += c.type.width() == 8 && c.data.data_ptr() == k.data_ptr() &&
              (c.type.kind() == ValueKind::SIGNED_INT || c.type.kind() == ValueKind::UNSIGNED_INT);
    return hits == 1;
  };
  // (a hashed key -- the invertible string word key a proxy carries as a column -- never fits 32 bits)
  bool narrow = pre != nullptr || (!hashed_key && nl > 0 && nr > 0 && lk.scalar_type() == at::kLong &&
                                   rk.scalar_type() == at::kLong && own_key_column(left, lk) && own_key_column(right, rk));
  at::Tensor narrow_bad = narrow ? at::zeros({1}, ex.opts(at::kInt)) : at::Tensor();
  // the narrowing base's source (left key 0), its own copy: a released input's key column goes away
  const at::Tensor base_src = pre ? pre->base_src : narrow ? lk.slice(0, 0, 1).clone() : at::Tensor();
  hip::NarrowKeys nk;
  if (narrow) {
    nk.base_src = ptr<int64_t>(base_src);
    nk.bad = reinterpret_cast<unsigned int *>(narrow_bad.data_ptr<int>());
  }
  int64_t cap = hip::radix_join_capacity(shape.w.data(), shape.in.data(), (int)shape.w.size(), (oj & 2) != 0,
                                         narrow ? 4 : 8);
  // fewest partition bits whose mean build partition sits 8 Poisson sigma (+16 rows) below the
  // LDS capacity: the largest of ~2^18 uniform partitions then fits with ~1e-10 failure odds (an
  // overflow only sends the join to the exact / global path).  1B rows: 18 bits -- two 9-bit
  // passes -- for inner joins (cap 4544) and build-preserving outer joins (cap 4408) alike.
  auto fits = [&](int64_t mean) { return (double)mean + 8.0 * std::sqrt((double)mean) + 16.0 <= (double)cap; };
  int bits = 0;
  while (bits < 24 && !fits((nb + (int64_t(1) << bits) - 1) >> bits)) ++bits;
  if (const int64_t xb = knobs::Int("RJ_EXTRA_BITS", 0))  // test knob: finer partitions
    bits = std::min(bits + (int)std::max<int64_t>(0, xb), 2 * 10);
  if (pre) bits = pre->bits;
  if (narrow && bits == 0 && !pre) {  // one partition: no pass runs, so nothing would narrow the keys
    narrow = false;
    nk = hip::NarrowKeys();
    cap = hip::radix_join_capacity(shape.w.data(), shape.in.data(), (int)shape.w.size(), (oj & 2) != 0, 8);
    while (bits < 24 && !fits((nb + (int64_t(1) << bits) - 1) >> bits)) ++bits;
  }
  const int64_t nparts = int64_t(1) << bits;
  // Slot mode for two-pass partitions (>= 11 bits): the second pass claims fixed-size partition
  // slots (mean + 8 sigma + 64 rows) instead of reading the keys once more for exact offsets
  // (k_rp_hist_tiles + scans + k_part_offsets, ~2 ms per 1B-row side).  A partition beyond its
  // slot (skewed keys) sends that side through the exact passes.  Test knob: CYLON_RJ_SLOT=0.
  const bool slot_on = knobs::Flag("RJ_SLOT", true);
  auto slot_of = [&](int64_t rows) -> int64_t {
    if (!slot_on || bits < 11) return 0;
    const double mean = (double)rows / (double)nparts;
    return ((int64_t)(mean + 8.0 * std::sqrt(mean) + 64.0) + 7) & ~int64_t(7);
  };
  auto key_col = [](const TablePtr &t, const at::Tensor &k) {
    int idx = -1, hits = 0;
    for (int c = 0; c < t->Columns(); ++c) {
      const Column &col = t->column(c);
      if (col.type.width() == 8 && col.data.data_ptr() == k.data_ptr() && !col.nullable() &&
          (col.type.kind() == ValueKind::SIGNED_INT || col.type.kind() == ValueKind::UNSIGNED_INT)) {
        idx = c;
        ++hits;
      }
    }
    return hits == 1 ? idx : -1;
  };
  const int kl = pre ? -1 : key_col(left, lk), kr = pre ? -1 : key_col(right, rk);
  // retain = false (reference table.cpp:150-154): an input is released as soon as nothing can need
  // it again -- its own passes fit their slots and no key of either side leaves the narrowed range
  // (else it would be repartitioned from the input) -- so its buffers are free before the other
  // side's passes and the output allocation (1B x 1B: ~64 GB lower peak).  Only the sink-less join
  // on partitions that can always complete releases (no global-table fallback needs the input later).
  const bool rel_l = !left->IsRetain() && !sink, rel_r = !right->IsRetain() && !sink;
  bool released_l = false, released_r = false;
  at::Tensor r_outside;  // narrowed keys: right keys outside [base, base + 2^32) (checked before releasing left)
  if (rel_l && narrow) {
    auto mm = at::aminmax(rk);
    const at::Tensor base = base_src - (int64_t(1) << 31);
    r_outside = at::logical_or(std::get<0>(mm) < base, (std::get<1>(mm) - base) > (int64_t)0xffffffffll).to(at::kInt);
  }
  auto release = [&](const TablePtr &t, at::Tensor &key) {
    t->ReleaseIfNotRetained();
    key = at::Tensor();
    trace::add_counter("join.radix.released_inputs", 1);
  };
  // Skewed partitions are handled per partition, not per join: a partition whose build side exceeds
  // the LDS capacity or whose probe side is hot (> 2 probe chunks) is skipped by the partition loop
  // and covered by split work items (kernel_decls.inc RJSplit): build chunks of <= cap rows x probe
  // chunks of pch rows, so a hot key costs its own rows, never the whole join (reference: one
  // unordered_multimap, join/hash_join.cpp:255-298).
  const int64_t np_rows = build_left ? nr : nl;
  const int64_t pch = std::max<int64_t>(int64_t(1) << 15, 8 * ((np_rows + nparts - 1) / nparts));
  const int64_t bmean = ((build_left ? nl : nr) + nparts - 1) / nparts;
  struct SkewMasks {
    at::Tensor bcnt, pcnt, heavy, mid, sums;  // sums: [heavy partitions, mid partitions] (device)
    int64_t cap = 0;
  };
  auto skew_masks = [&](const RadixSide &Bs, const RadixSide &Ps, int64_t cp) {
    SkewMasks k;
    k.cap = cp;
    const int64_t split_rows = std::max<int64_t>(8, std::min<int64_t>(cp, knobs::Int("RJ_SPLIT_ROWS", cp)));
    k.bcnt = part_counts(Bs, nparts);
    k.pcnt = part_counts(Ps, nparts);
    k.heavy = at::logical_or(k.bcnt > split_rows, k.pcnt > 2 * pch);
    // hot-ish partitions (far above the mean, not split) are counted exactly instead of sampled: a
    // sample that misses them under-estimates the output and costs a second write (skip = 2)
    k.mid = at::logical_and(k.heavy.logical_not(),
                            at::logical_or(k.pcnt > 4 * (np_rows + nparts - 1) / nparts + 1024, k.bcnt > 4 * bmean + 1024));
    k.sums = at::stack({k.heavy.sum(), k.mid.sum()});
    return k;
  };
  SkewMasks sk;  // computed with the partition flags' read when no side is repartitioned
  RadixSide L, R;
  if (pre) {
    L = pre->L;
    R = pre->R;
  } else {
    CYLON_PHASE("join.radix.partition", ex.device);
    const hip::NarrowKeys *nkp = narrow ? &nk : nullptr;
    // A side with a hot partition would overflow a slot and repartition exactly after both slot
    // passes (1B x 1B with 16 build keys x 200k duplicates: +48 ms): a histogram of ~1M sampled keys
    // (every stride-th) finds a partition far above the mean first, and that side starts exact.
    int64_t sl = slot_of(nl), sr = slot_of(nr);
    if ((sl || sr) && std::max(nl, nr) >= (int64_t(1) << 24) && (!sink || sink->sample_skew)) {
      auto sample = [&](const at::Tensor &k, int64_t rows, at::Tensor &h, int64_t &stride) {
        stride = std::max<int64_t>(1, rows >> 20);
        h = at::empty({nparts}, ex.opts(at::kInt));
        hip::radix_part_sample(ptr<int64_t>(k), rows, bits, stride, reinterpret_cast<uint32_t *>(h.data_ptr<int>()),
                               nkp, ex.stream);
      };
      at::Tensor hl, hr;
      int64_t stl = 1, str = 1;
      sample(lk, nl, hl, stl);
      sample(rk, nr, hr, str);
      at::Tensor mx = at::stack({hl.max(), hr.max()}).cpu();
      auto hot = [&](int64_t m, int64_t rows, int64_t stride) {
        const double mean = (double)((rows + stride - 1) / stride) / (double)nparts;
        return (double)m > 4.0 * mean + 32.0;
      };
      if (sl && hot(mx[0].item<int>(), nl, stl)) sl = 0;
      if (sr && hot(mx[1].item<int>(), nr, str)) sr = 0;
      if (!sl || !sr) trace::add_counter("join.radix.sampled_skew_sides", (sl ? 0 : 1) + (sr ? 0 : 1));
    }
    L = radix_partition(ex, left, lk, bits, nullptr, sl, nkp);
    if (rel_l) {
      at::Tensor z = at::zeros({1}, ex.opts(at::kInt));
      const int bad = at::cat({L.slot ? L.overflow.slice(0, 0, 1) : z, narrow ? narrow_bad : z,
                               r_outside.defined() ? r_outside.reshape({1}) : z}).sum().item<int>();
      if (bad == 0) {
        release(left, lk);
        released_l = true;
      }
    }
    R = radix_partition(ex, right, rk, bits, nullptr, sr, nkp);
    if (rel_r) {
      at::Tensor z = at::zeros({1}, ex.opts(at::kInt));
      const int bad = at::cat({R.slot ? R.overflow.slice(0, 0, 1) : z, narrow ? narrow_bad : z}).sum().item<int>();
      if (bad == 0) {
        release(right, rk);
        released_r = true;
      }
    }
    if (L.slot || R.slot || narrow) {  // a side whose partition outgrew a slot is partitioned exactly
      at::Tensor z = at::zeros({}, ex.opts(at::kInt));
      // the skew masks of the partitions as they stand ride in the same copy (used when no side is
      // repartitioned below: one host sync instead of two)
      sk = skew_masks(build_left ? L : R, build_left ? R : L, cap);
      at::Tensor f = at::cat({at::stack({L.slot ? L.overflow[0] : z, R.slot ? R.overflow[0] : z,
                                         narrow ? narrow_bad[0] : z}).to(at::kLong),
                              sk.sums}).cpu();
      bool redo = f[2].item<int64_t>() != 0;
      if (redo) {  // a key outside the uint32 offset range: both sides as int64 keys
        trace::add_counter("join.radix.narrow_fallback", 1);
        narrow = false;  // (8-byte keys: the smaller LDS capacity; fuller partitions become split items)
        cap = hip::radix_join_capacity(shape.w.data(), shape.in.data(), (int)shape.w.size(), (oj & 2) != 0, 8);
        L = radix_partition(ex, left, lk, bits, nullptr, slot_of(nl));
        R = radix_partition(ex, right, rk, bits, nullptr, slot_of(nr));
        if (L.slot || R.slot)
          f = at::stack({L.slot ? L.overflow[0] : z, R.slot ? R.overflow[0] : z, z}).to(at::kLong).cpu();
      }
      nkp = narrow ? &nk : nullptr;
      if (f[0].item<int64_t>()) {
        trace::add_counter("join.radix.slot_overflow", 1);
        L = radix_partition(ex, left, lk, bits, nullptr, 0, nkp);
        redo = true;
      }
      if (f[1].item<int64_t>()) {
        trace::add_counter("join.radix.slot_overflow", 1);
        R = radix_partition(ex, right, rk, bits, nullptr, 0, nkp);
        redo = true;
      }
      if (redo) sk = SkewMasks();
      else sk.sums = f.slice(0, 3, 5);  // (host copy of the sums)
      trace::add_counter("join.radix.slot_sides", (L.slot ? 1 : 0) + (R.slot ? 1 : 0));
      if (narrow) trace::add_counter("join.radix.narrow_keys", 1);
    }
  }
  RadixSide &B = build_left ? L : R;
  RadixSide &P = build_left ? R : L;
  const int64_t *nbase = narrow ? ptr<int64_t>(base_src) : nullptr;  // the join kernels' narrowed-key base
  // (a released input can no longer feed a fallback: the remaining failure exits raise instead)
  const bool released = released_l || released_r;
  auto fail = [&](const char *why) -> TablePtr {
    CYLON_CHECK(!released, Code::ExecutionError,
                "radix join with a released (retain = false) input could not complete: " << why);
    return nullptr;
  };
  // Inner joins keyed on one integer column per side (the partitioned key itself, same type, no
  // nulls): the two key values of every output row are equal, so the build side's output key
  // column is the probe side's -- one buffer behind both (columns are immutable): 8 B/row less
  // written and allocated (1B x 1B: 8 GB).  A/B knob: CYLON_RJ_SHARE_KEY=0.
  const bool share_key = oj == 0 && !sink && kl >= 0 && kr >= 0 && left->column(kl).type == right->column(kr).type &&
                         knobs::Flag("RJ_SHARE_KEY", true);
  const int bkc = build_left ? kl : kr;  // the build side's key column (not written when shared)
  const int64_t split_rows = std::max<int64_t>(8, std::min<int64_t>(cap, knobs::Int("RJ_SPLIT_ROWS", cap)));
  if (!sk.heavy.defined() || sk.cap != cap) sk = skew_masks(B, P, cap);
  const at::Tensor &bcnt = sk.bcnt, &pcnt = sk.pcnt, &heavy = sk.heavy, &mid = sk.mid;
  at::Tensor skip = heavy.to(at::kByte), skip_sample = at::logical_or(heavy, mid).to(at::kByte);
  at::Tensor hm;
  if (pre) {  // the prepartitioned sides' slot overflow flags in the same copy
    hm = at::cat({sk.sums.to(at::kLong), pre->L.overflow.to(at::kLong), pre->R.overflow.to(at::kLong)}).cpu();
    pre->overflow_l = hm[2].item<int64_t>() != 0;
    pre->overflow_r = hm[3].item<int64_t>() != 0;
    if (pre->overflow_l || pre->overflow_r) {
      pre->overflowed = true;
      return nullptr;
    }
  } else {
    hm = sk.sums.is_cuda() ? sk.sums.cpu() : sk.sums;
  }
  const int64_t nheavy = hm[0].item<int64_t>(), nmid = hm[1].item<int64_t>();
  std::vector<int64_t> items, emits;  // kRJItemWords per item
  int64_t emit_bound = 0;
  if (nheavy > 0) {
    at::Tensor hidx = heavy.nonzero().flatten();
    at::Tensor info = at::stack({part_starts(P, nparts).index_select(0, hidx), pcnt.index_select(0, hidx),
                                 part_starts(B, nparts).index_select(0, hidx), bcnt.index_select(0, hidx)},
                                1)
                          .cpu()
                          .contiguous();
    const int64_t *h = info.data_ptr<int64_t>();
    std::vector<std::array<int64_t, hip::kRJItemWords>> work;
    for (int64_t i = 0; i < nheavy; ++i) {
      const int64_t lb0 = h[4 * i], nl0 = h[4 * i + 1], rb0 = h[4 * i + 2], nr0 = h[4 * i + 3];
      const int64_t nbc = std::max<int64_t>(1, (nr0 + split_rows - 1) / split_rows);
      const int64_t npc = nl0 > 2 * pch ? (nl0 + pch - 1) / pch : 1;
      // a side split into several items learns "unmatched" only from all of them: deferred
      const bool pdef = (oj & 1) && nbc > 1, bdef = (oj & 2) && npc > 1;
      const int64_t fl = (pdef ? hip::kRJItemPDefer : 0) | (bdef ? hip::kRJItemBDefer : 0);
      for (int64_t bc = 0; bc < nbc; ++bc)
        for (int64_t pc = 0; pc < npc; ++pc) {
          const int64_t b0 = nr0 * bc / nbc, b1 = nr0 * (bc + 1) / nbc, p0 = nl0 * pc / npc, p1 = nl0 * (pc + 1) / npc;
          if (b1 > b0 || p1 > p0) work.push_back({lb0 + p0, p1 - p0, rb0 + b0, b1 - b0, fl});
        }
      if (pdef) {
        for (int64_t pc = 0; pc < npc; ++pc)
          emits.insert(emits.end(), {lb0 + nl0 * pc / npc, nl0 * (pc + 1) / npc - nl0 * pc / npc, 0, 0,
                                     (int64_t)hip::kRJItemPEmit});
        emit_bound += nl0;
      }
      if (bdef) {
        for (int64_t bc = 0; bc < nbc; ++bc)
          emits.insert(emits.end(), {0, 0, rb0 + nr0 * bc / nbc, nr0 * (bc + 1) / nbc - nr0 * bc / nbc,
                                     (int64_t)hip::kRJItemBEmit});
        emit_bound += nr0;
      }
    }
    // heaviest items first: they lead the write kernel's grid-stride order
    std::stable_sort(work.begin(), work.end(), [](const auto &a, const auto &b) {
      return a[1] * std::max<int64_t>(1, a[3]) > b[1] * std::max<int64_t>(1, b[3]);
    });
    for (const auto &w : work) items.insert(items.end(), w.begin(), w.end());
    trace::add_counter("join.radix.split_partitions", nheavy);
    trace::add_counter("join.radix.split_items", (int64_t)work.size());
  }
  const int64_t nitems = (int64_t)items.size() / hip::kRJItemWords, nemits = (int64_t)emits.size() / hip::kRJItemWords;
  at::Tensor items_d = nitems ? at::tensor(items, at::TensorOptions().dtype(at::kLong)).to(ex.device) : at::Tensor();
  at::Tensor emits_d = nemits ? at::tensor(emits, at::TensorOptions().dtype(at::kLong)).to(ex.device) : at::Tensor();
  at::Tensor gprobe, gbuild;  // matched flags of the deferred sides (per partitioned row)
  for (int64_t i = 0; i < nitems; ++i) {
    const int64_t f = items[i * hip::kRJItemWords + 4];
    if ((f & hip::kRJItemPDefer) && !gprobe.defined()) gprobe = at::zeros({std::max<int64_t>(1, P.keys.numel())}, ex.opts(at::kByte));
    if ((f & hip::kRJItemBDefer) && !gbuild.defined()) gbuild = at::zeros({std::max<int64_t>(1, B.keys.numel())}, ex.opts(at::kByte));
  }
  hip::RJSplit split_main, split_emit;
  split_main.skip = nheavy ? skip.data_ptr<uint8_t>() : nullptr;
  at::Tensor mid_items;  // count-only items of the skip = 2 partitions
  if (nmid > 0) {
    at::Tensor midx = mid.nonzero().flatten();
    mid_items = at::stack({part_starts(P, nparts).index_select(0, midx), pcnt.index_select(0, midx),
                           part_starts(B, nparts).index_select(0, midx), bcnt.index_select(0, midx),
                           at::zeros({nmid}, ex.opts(at::kLong))},
                          1)
                    .contiguous();
    trace::add_counter("join.radix.exact_counted_partitions", nmid);
  }
  split_main.items = nitems ? ptr<int64_t>(items_d) : nullptr;
  split_main.nitems = nitems;
  split_main.gprobe = gprobe.defined() ? gprobe.data_ptr<uint8_t>() : nullptr;
  split_main.gbuild = gbuild.defined() ? gbuild.data_ptr<uint8_t>() : nullptr;
  split_emit = split_main;
  split_emit.skip = nullptr;
  split_emit.items = nemits ? ptr<int64_t>(emits_d) : nullptr;
  split_emit.nitems = nemits;
  // Output size.  Exact mode: a count kernel over every partition, a scan, then the write
  // kernel at the scanned offsets.  Fused mode (default): the count kernel runs on every
  // 32nd partition only, the output is allocated for the extrapolated size + 2 % (partitions
  // are hash-uniform: the estimate's standard error is ~0.03 % at 1B rows), and the write
  // kernel counts each partition's matches itself and claims its output rows with one
  // atomic.  A claim past the allocation makes the kernel report the exact total instead,
  // and the write runs again into an exact allocation (skewed keys); the row order differs
  // between runs either way (docs/semantics.md).
  // test / A-B knobs: CYLON_RJ_EXACT_COUNT=1 (count kernel over every partition),
  // CYLON_RJ_FUSED_MIN_PARTS (default 4096), CYLON_RJ_ESTIMATE_SCALE (scales the estimate: < 1
  // forces the exact rerun)
  const bool exact_count = knobs::Flag("RJ_EXACT_COUNT", false);
  const int64_t fused_min = knobs::Int("RJ_FUSED_MIN_PARTS", 4096);
  const char *es = knobs::Get("RJ_ESTIMATE_SCALE");
  const double est_scale = es ? std::atof(es) : 1.0;
  int64_t stride = exact_count || nparts < fused_min ? 1 : std::min<int64_t>(32, std::max<int64_t>(1, nparts / 64));
  at::Tensor counts;
  at::Tensor overflow = at::empty({1}, ex.opts(at::kInt));
  at::Tensor out_offs;
  int64_t m = 0, alloc = 0;
  {
    CYLON_PHASE("join.radix.count", ex.device);
    // the partition count skips split partitions (items are counted below); the sampled count also
    // the hot-ish ones (counted exactly below)
    hip::RJSplit skip_only;
    auto count = [&](int64_t st) {
      skip_only.skip = st > 1 && nmid ? skip_sample.data_ptr<uint8_t>() : split_main.skip;
      counts = ex.empty_i64((nparts + st - 1) / st);
      hip::radix_join_count(kptr(P.keys), ptr<int64_t>(P.offs), kptr(B.keys), ptr<int64_t>(B.offs),
                            nparts, cap, ptr<int64_t>(counts), overflow.data_ptr<int>(), ex.stream, st, oj, P.slot,
                            B.slot, &skip_only, nbase);
    };
    count(stride);
    // the ranking guard of the stable (second and later) partition passes: its device flag travels
    // in the same copy as the count results (one host sync instead of two)
    const at::Tensor oflag = at::from_blob(hip::rp_order_flag(), {1}, ex.opts(at::kInt)).to(at::kLong);
    auto order_violation = [&](int64_t flag) {
      if (!flag) return false;
      hip::rp_note_order_violation(ex.stream);
      trace::add_counter("join.radix.order_violation_fallback", 1);
      return true;
    };
    int64_t ssum = 0, sover = 0;  // the sample's total and overflow flag (one read for both uses)
    if (stride > 1) {
      // Skew check of the sample: extrapolating a hot key's partition 32x would over-allocate
      // (ADVICE r03), so a sample whose largest partition output is far above its mean is
      // counted exactly instead.
      at::Tensor st = at::stack({counts.sum(), counts.max(), overflow.to(at::kLong)[0], oflag[0]}).cpu();
      if (order_violation(st[3].item<int64_t>())) return fail("order violation");
      ssum = st[0].item<int64_t>();
      sover = st[2].item<int64_t>();
      const int64_t smax = st[1].item<int64_t>();
      const int64_t nsample = counts.numel();
      if (sover == 0 && smax > 16 * (ssum / std::max<int64_t>(1, nsample)) + 65536) {
        trace::add_counter("join.radix.skewed_sample_exact_count", 1);
        stride = 1;
        count(1);
      }
    }
    if (stride == 1) {
      out_offs = exclusive_scan(ex, counts);
      at::Tensor tail = at::cat({out_offs.slice(0, nparts, nparts + 1), overflow.to(at::kLong), oflag}).cpu();
      if (order_violation(tail[2].item<int64_t>())) return fail("order violation");
      m = tail[0].item<int64_t>();
      if (tail[1].item<int64_t>() != 0) {
        trace::add_counter("join.radix.overflow_fallback", 1);
        return fail("overflow");
      }
      alloc = m;
    } else {
      if (sover != 0) {  // a sampled partition already overflows the LDS (or is misplaced)
        trace::add_counter("join.radix.overflow_fallback", 1);
        return fail("overflow");
      }
      const double est = (double)ssum * (double)nparts / (double)counts.numel();
      // skewed inputs (split or exactly counted partitions exist): the sampled rest still holds
      // moderately hot keys, so its estimate gets 10 % slack instead of 2 % (memory, not a rewrite)
      const double slack = nheavy + nmid > 0 ? 1.10 : 1.02;
      alloc = (int64_t)(est * slack * est_scale) + (est_scale < 1.0 ? 0 : 65536);
      trace::add_counter("join.radix.estimated_rows", (int64_t)est);
    }
    if (nmid > 0 && stride > 1) {  // the partitions left out of the sample, counted exactly
      at::Tensor mc = ex.empty_i64(nmid);
      hip::RJSplit only;
      only.items = ptr<int64_t>(mid_items);
      only.nitems = nmid;
      hip::radix_join_count(kptr(P.keys), ptr<int64_t>(P.offs), kptr(B.keys), ptr<int64_t>(B.offs),
                            0, cap, ptr<int64_t>(mc), overflow.data_ptr<int>(), ex.stream, 1, oj, P.slot, B.slot,
                            &only, nbase);
      alloc += mc.sum().item<int64_t>();
    }
    if (nitems > 0) {  // split items: counted exactly (their deferred rows bounded), cursor mode
      at::Tensor ic = ex.empty_i64(nitems);
      hip::RJSplit only = split_main;
      only.skip = nullptr;
      hip::radix_join_count(kptr(P.keys), ptr<int64_t>(P.offs), kptr(B.keys), ptr<int64_t>(B.offs),
                            0, cap, ptr<int64_t>(ic), overflow.data_ptr<int>(), ex.stream, 1, oj, P.slot, B.slot,
                            &only, nbase);
      const int64_t exact_items = ic.sum().item<int64_t>();
      alloc = (stride == 1 ? m : alloc) + exact_items + emit_bound;
      stride = 2;  // (cursor mode below)
      out_offs = at::Tensor();
    }
  }
  CYLON_PHASE("join.radix.write", ex.device);
  std::vector<Column> lcols, rcols;
  std::vector<at::Tensor> lwords, rwords;
  at::Tensor ppres, bpres;  // presence bytes of the probe / build side (outer joins)
  int64_t off = 0;
  auto allocate = [&](int64_t rows) {
    lcols.clear();
    rcols.clear();
    if (sink) {
      std::vector<Column> proto;  // (the proto's validity only says whether the column is nullable)
      for (const auto &col : left->columns())
        proto.emplace_back(cfg.GetLeftTablePrefix() + col.name, col.type, 0, col.data, at::Tensor(),
                           col.nullable() || lnull ? col.data : at::Tensor());
      for (const auto &col : right->columns())
        proto.emplace_back(cfg.GetRightTablePrefix() + col.name, col.type, 0, col.data, at::Tensor(),
                           col.nullable() || rnull ? col.data : at::Tensor());
      off = sink->reserve(ex, rows, proto);
      lcols.assign(sink->cols.begin(), sink->cols.begin() + left->Columns());
      rcols.assign(sink->cols.begin() + left->Columns(), sink->cols.end());
    } else {
      for (int c = 0; c < left->Columns(); ++c) {  // (null-side validity: apply_presence)
        const Column &col = left->column(c);
        const bool shared = share_key && build_left && c == bkc;
        lcols.push_back(make_fixed_column(cfg.GetLeftTablePrefix() + col.name, col.type, shared ? 0 : rows,
                                          ex.device, col.nullable()));
      }
      for (int c = 0; c < right->Columns(); ++c) {
        const Column &col = right->column(c);
        const bool shared = share_key && !build_left && c == bkc;
        rcols.push_back(make_fixed_column(cfg.GetRightTablePrefix() + col.name, col.type, shared ? 0 : rows,
                                          ex.device, col.nullable()));
      }
    }
    auto word_outs = [&](const RadixSide &sd) {
      std::vector<at::Tensor> w;
      for (size_t i = 0; i < sd.vwords.size(); ++i) w.push_back(ex.empty_i64(std::max<int64_t>(rows, 1)));
      return w;
    };
    lwords = word_outs(L);
    rwords = word_outs(R);
    if (oj & 2) ppres = ex.empty_u8(std::max<int64_t>(rows, 1));
    if (oj & 1) bpres = ex.empty_u8(std::max<int64_t>(rows, 1));
  };
  auto write = [&](int64_t rows, const int64_t *offs, int64_t *cursor) {
    RadixCols pc = build_left ? radix_cols(right, &R, &rcols, off, &rwords) : radix_cols(left, &L, &lcols, off, &lwords);
    RadixCols bc = build_left ? radix_cols(left, &L, &lcols, off, &lwords) : radix_cols(right, &R, &rcols, off, &rwords);
    if (share_key) {  // the build key column's entry (after any unpacked validity entries before it)
      int q = 0;
      for (int c = 0; c < bkc; ++c) q += 1 + (bt->column(c).nullable() && B.vwords.empty());
      bc.in.erase(bc.in.begin() + q);
      bc.out.erase(bc.out.begin() + q);
      bc.w.erase(bc.w.begin() + q);
    }
    // probe-side columns are streamed from HBM; the key column (in == nullptr) is written from
    // the probe key the kernel already holds
    int pkey = -1;
    for (size_t q = 0; q < pc.in.size(); ++q)
      if (!pc.in[q]) {
        pc.in[q] = reinterpret_cast<const uint8_t *>(P.keys.data_ptr());
        if (pkey < 0) pkey = (int)q;
      }
    hip::radix_join_write(kptr(P.keys), ptr<int64_t>(P.offs), kptr(B.keys), ptr<int64_t>(B.offs),
                          nparts, cap, offs, pc.in.data(), pc.out.data(), pc.w.data(), (int)pc.in.size(),
                          bc.in.data(), bc.out.data(), bc.w.data(), (int)bc.in.size(), ex.stream, cursor, rows,
                          overflow.data_ptr<int>(), pkey, oj, ppres.defined() ? ppres.data_ptr<uint8_t>() : nullptr,
                          bpres.defined() ? bpres.data_ptr<uint8_t>() : nullptr, P.slot, B.slot, &split_main, nbase);
    if (nemits > 0)  // the deferred sides' unmatched rows, after every item recorded its matches
      hip::radix_join_write(kptr(P.keys), ptr<int64_t>(P.offs), kptr(B.keys), ptr<int64_t>(B.offs),
                            0, cap, nullptr, pc.in.data(), pc.out.data(), pc.w.data(), (int)pc.in.size(),
                            bc.in.data(), bc.out.data(), bc.w.data(), (int)bc.in.size(), ex.stream, cursor, rows,
                            overflow.data_ptr<int>(), pkey, oj, ppres.defined() ? ppres.data_ptr<uint8_t>() : nullptr,
                            bpres.defined() ? bpres.data_ptr<uint8_t>() : nullptr, P.slot, B.slot, &split_emit, nbase);
  };
  if (stride == 1) {
    allocate(m);
    if (m > 0) write(m, ptr<int64_t>(out_offs), nullptr);
  } else {
    at::Tensor cursor = at::zeros({1}, ex.opts(at::kLong));
    overflow.zero_();
    allocate(alloc);
    write(alloc, nullptr, ptr<int64_t>(cursor));
    at::Tensor res = at::cat({cursor, overflow.to(at::kLong)}).cpu();
    m = res[0].item<int64_t>();
    const int64_t flags = res[1].item<int64_t>();
    if (flags & 1) {  // a build partition beyond the LDS capacity: global-table join instead
      if (sink) sink->size = off;
      trace::add_counter("join.radix.overflow_fallback", 1);
      return fail("overflow");
    }
    if (flags & 2) {  // the estimate was short: write again into an exact allocation
      trace::add_counter("join.radix.estimate_rerun", 1);
      if (sink) sink->size = off;
      cursor.zero_();
      overflow.zero_();
      if (gprobe.defined()) gprobe.zero_();
      if (gbuild.defined()) gbuild.zero_();
      allocate(m);
      write(m, nullptr, ptr<int64_t>(cursor));
      CYLON_CHECK(at::cat({cursor, overflow.to(at::kLong)}).cpu().equal(at::tensor({m, (int64_t)0})),
                  Code::ExecutionError, "radix join: exact rerun did not match its own count");
    } else if (sink) {
      sink->size = off + m;  // give back the estimate's slack
    }
    if (!sink) {
      for (auto &c : lcols)
        if (c.length > 0) c = c.slice(0, m);
      for (auto &c : rcols)
        if (c.length > 0) c = c.slice(0, m);
    }
  }
  if (share_key) {
    Column &dst = build_left ? lcols[kl] : rcols[kr];
    const Column &src = build_left ? rcols[kr] : lcols[kl];
    dst.data = src.data;
    dst.length = src.length;
    trace::add_counter("join.radix.shared_key_column", 1);
  }
  if (m > 0) {
    unpack_validity_words(ex, left, L, lwords, lcols, off, m);
    unpack_validity_words(ex, right, R, rwords, rcols, off, m);
  }
  {  // outer joins: the null side's validity from the presence bytes
    const at::Tensor &lpres = build_left ? bpres : ppres, &rpres = build_left ? ppres : bpres;
    if (lnull) apply_presence(lcols, left, lpres, off, m, sink == nullptr);
    if (rnull) apply_presence(rcols, right, rpres, off, m, sink == nullptr);
  }
  trace::add_counter("join.radix.rows_out", m);
  if (oj) trace::add_counter("join.radix.outer", oj);
  if (sink) return Table::Make(left->GetContext(), sink->cols);
  for (auto &c : rcols) lcols.push_back(std::move(c));
  return Table::Make(left->GetContext(), std::move(lcols));
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

// K7 sort-merge join on row-sorted tables (device, large inner joins on one exact
// integer key, algorithm = SORT).  Both relations are first sorted by the key with
// the row-moving LSD passes of ops::Sort (every column moves with the key, constant
// key bits skipped), so the merge's index pairs are monotone in both tables and
// the final gathers stream through HBM instead of touching it at random (the
// pair-sort + gather form spends most of its time in those random gathers).  The
// output comes out ordered by key, as the reference's sort join does.
static TablePtr sorted_merge_join(const Exec &ex, const TablePtr &left, const TablePtr &right,
                                  const JoinConfig &cfg) {
  const int lc = cfg.GetLeftColumnIdx()[0], rc = cfg.GetRightColumnIdx()[0];
  TablePtr ls, rs;
  {
    CYLON_PHASE("join.sortmerge.sort", ex.device);
    ls = Sort(left, {lc}, {true});
    rs = Sort(right, {rc}, {true});
  }
  // merge_join_* compare keys as uint64: the sign-flipped image of a signed key is
  // ordered like the key itself
  auto image = [&](const TablePtr &t, int c) {
    KeyEncoding k = encode_keys(ex, t, {c}, true);
    return t->column(c).type.kind() == ValueKind::SIGNED_INT
               ? at::bitwise_xor(k.keys, at::full({1}, std::numeric_limits<int64_t>::min(), k.keys.options()))
               : k.keys;
  };
  at::Tensor lk = image(ls, lc), rk = image(rs, rc);
  const int64_t nl = ls->Rows(), nr = rs->Rows();
  at::Tensor li, ri;
  {
    CYLON_PHASE("join.sortmerge.merge", ex.device);
    at::Tensor lo = ex.empty_i64(nl), counts = ex.empty_i64(nl);
    KCALL(ex, merge_join_count, reinterpret_cast<const uint64_t *>(ptr<int64_t>(lk)), nl,
          reinterpret_cast<const uint64_t *>(ptr<int64_t>(rk)), nr, ptr<int64_t>(lo), ptr<int64_t>(counts));
    at::Tensor offs = exclusive_scan(ex, counts);
    const int64_t m = read_i64(offs, nl);
    at::Tensor lperm = ex.empty_i64(nl), rperm = ex.empty_i64(nr);
    KCALL(ex, iota, ptr<int64_t>(lperm), nl, 0);
    KCALL(ex, iota, ptr<int64_t>(rperm), nr, 0);
    li = ex.empty_i64(m);
    ri = ex.empty_i64(m);
    KCALL(ex, merge_join_write, ptr<int64_t>(lperm), nl, ptr<int64_t>(rperm), ptr<int64_t>(lo), ptr<int64_t>(offs),
          ptr<int64_t>(li), ptr<int64_t>(ri));
  }
  CYLON_PHASE("join.sortmerge.materialize", ex.device);
  TablePtr lo = GatherNullable(ls, li, false);
  TablePtr ro = GatherNullable(rs, ri, false);
  std::vector<Column> cols;
  for (const auto &c : lo->columns()) cols.push_back(c.with_name(cfg.GetLeftTablePrefix() + c.name));
  for (const auto &c : ro->columns()) cols.push_back(c.with_name(cfg.GetRightTablePrefix() + c.name));
  trace::add_counter("join.sortmerge.rows_out", li.numel());
  return Table::Make(left->GetContext(), std::move(cols));
}

// K7 range join (device, inner, one signed integer key, algorithm = SORT): both
// relations are radix-partitioned into key ranges in key order (RangeSpec), each
// partition holding 2^rshift consecutive key values (rshift <= 12), and each
// partition is joined in LDS by exact key offset, emitting its rows in key order
// (radix_join.hip k_rg_*).  Same passes as the hash radix join, no full sort.
// Returns nullptr when the keys are too sparse for 12-bit partitions or a
// partition overflows (skew): the caller then runs sorted_merge_join.
static bool range_join_enabled() {
  return knobs::Flag("RANGE_JOIN", true);  // test knob: 0 = sort-merge path only
}

static TablePtr range_join(const Exec &ex, const TablePtr &left, const TablePtr &right, const JoinConfig &cfg) {
  const int lc = cfg.GetLeftColumnIdx()[0], rc = cfg.GetRightColumnIdx()[0];
  if (left->column(lc).type.kind() != ValueKind::SIGNED_INT) return nullptr;
  const int64_t nl = left->Rows(), nr = right->Rows();
  KeyEncoding lk = encode_keys(ex, left, {lc}, true), rk = encode_keys(ex, right, {rc}, true);
  at::Tensor mm = at::stack({lk.keys.min(), lk.keys.max(), rk.keys.min(), rk.keys.max()}).to(at::kCPU);
  const int64_t *h = mm.data_ptr<int64_t>();
  const int64_t kmin = std::min(h[0], h[2]), kmax = std::max(h[1], h[3]);
  const uint64_t span = (uint64_t)kmax - (uint64_t)kmin;  // signed range as an unsigned count
  int span_bits = 0;
  while (span_bits < 64 && (span >> span_bits) != 0) ++span_bits;
  // ~half the LDS capacity per side and partition on average: far below the cap for uniform keys
  const int64_t target = hip::range_join_max_rows() / 2;
  int bits = 0;
  while ((std::max(nl, nr) >> bits) > target) ++bits;
  // sparse keys: up to 16x more (smaller) partitions than the row count asks for keep
  // each partition's key range within the 4096 exact-offset buckets
  const int maxs = hip::range_join_max_shift();
  if (span_bits - bits > maxs && span_bits - maxs <= bits + 4) bits = span_bits - maxs;
  const int rshift = std::max(0, span_bits - bits);
  if (rshift > maxs) {
    trace::add_counter("join.range.sparse_fallback", 1);
    return nullptr;
  }
  const int pbits = span_bits - rshift;
  RangeSpec spec;
  spec.flip = uint64_t(1) << 63;  // signed -> order-preserving unsigned image
  spec.mn = (uint64_t)kmin ^ spec.flip;
  spec.rshift = rshift;
  const int64_t nparts = int64_t(1) << pbits;
  RadixSide L, R;
  {
    CYLON_PHASE("join.range.partition", ex.device);
    L = radix_partition(ex, left, lk.keys, pbits, &spec);
    R = radix_partition(ex, right, rk.keys, pbits, &spec);
  }
  at::Tensor counts = ex.empty_i64(nparts);
  at::Tensor overflow = at::empty({1}, ex.opts(at::kInt));
  {
    CYLON_PHASE("join.range.count", ex.device);
    hip::range_join_count(ptr<int64_t>(L.keys), ptr<int64_t>(L.offs), ptr<int64_t>(R.keys), ptr<int64_t>(R.offs),
                          nparts, spec.flip, spec.mn, rshift, ptr<int64_t>(counts), overflow.data_ptr<int>(),
                          ex.stream);
  }
  if (overflow.item<int>() != 0) {
    trace::add_counter("join.range.overflow_fallback", 1);
    return nullptr;
  }
  at::Tensor out_offs = exclusive_scan(ex, counts);
  const int64_t m = read_i64(out_offs, nparts);
  CYLON_PHASE("join.range.write", ex.device);
  std::vector<Column> lcols, rcols;
  for (const auto &col : left->columns())
    lcols.push_back(make_fixed_column(cfg.GetLeftTablePrefix() + col.name, col.type, m, ex.device, col.nullable()));
  for (const auto &col : right->columns())
    rcols.push_back(make_fixed_column(cfg.GetRightTablePrefix() + col.name, col.type, m, ex.device, col.nullable()));
  if (m > 0) {
    std::vector<at::Tensor> lwords, rwords;
    for (size_t i = 0; i < L.vwords.size(); ++i) lwords.push_back(ex.empty_i64(m));
    for (size_t i = 0; i < R.vwords.size(); ++i) rwords.push_back(ex.empty_i64(m));
    RadixCols a = radix_cols(left, &L, &lcols, 0, &lwords), b = radix_cols(right, &R, &rcols, 0, &rwords);
    for (auto &q : a.in)
      if (!q) q = reinterpret_cast<const uint8_t *>(L.keys.data_ptr());
    for (auto &q : b.in)
      if (!q) q = reinterpret_cast<const uint8_t *>(R.keys.data_ptr());
    hip::range_join_write(ptr<int64_t>(L.keys), ptr<int64_t>(L.offs), ptr<int64_t>(R.keys), ptr<int64_t>(R.offs),
                          nparts, spec.flip, spec.mn, rshift, ptr<int64_t>(out_offs), a.in.data(), a.out.data(),
                          a.w.data(), (int)a.in.size(), b.in.data(), b.out.data(), b.w.data(), (int)b.in.size(),
                          ex.stream);
    unpack_validity_words(ex, left, L, lwords, lcols, 0, m);
    unpack_validity_words(ex, right, R, rwords, rcols, 0, m);
  }
  trace::add_counter("join.range.rows_out", m);
  for (auto &c : rcols) lcols.push_back(std::move(c));
  return Table::Make(left->GetContext(), std::move(lcols));
}

// Keys of the LDS radix join (K5).  One simple key column: the column itself.  Several non-null
// integer key columns: one EXACT composite -- each column's offset from its two-relation minimum,
// packed into 63 bits when the spans fit -- or else a 64-bit row hash whose matches are verified
// on the output (reference multi-key join: hash_join.cpp:92-186, TwoTableRowIndexHash).
struct RadixKeys {
  at::Tensor l, r;
  bool ok = false, verify = false;
  bool composite = false;  // l / r are exact composites: key column i = lo[i] + ((key >> shift[i]) & 2^bits[i]-1)
  std::vector<int64_t> lo;
  std::vector<int> shift, bits;
  std::vector<int64_t> ncode;  // composite: field value of a null in key i (-1: no nulls on either side)
  bool nulls = false;
  // one fixed-length string key per side: l / r are its invertible word keys (hash.hpp word_key_*,
  // carried by the proxies as a column in place of word 0) and lwords / rwords its words 1..W-1,
  // all from one read of the bytes
  std::vector<at::Tensor> lwords, rwords;
  int64_t wlen = -1;
  // one variable-length string key per side, every row <= 64 bytes: W = vw zero-padded words, l / r
  // the padded word keys (word 0's stand-in), lwords / rwords words 1..W-1, llen / rlen the lengths
  int vw = 0;
  at::Tensor llen, rlen;
  bool vtext = false;  // text mode (no zero bytes on either side): no length columns (partition.hip)
};

static int64_t fixed_var_len(const Exec &ex, const Column &c);
static std::vector<at::Tensor> var_to_words(const Exec &ex, const Column &c, int64_t L, at::Tensor *hash = nullptr,
                                            bool inv = false);
static std::pair<int64_t, int64_t> var_len_range(const Exec &ex, const Column &c);
static std::vector<at::Tensor> var_to_padded(const Exec &ex, const Column &c, int W, at::Tensor *key,
                                             at::Tensor *lens, unsigned int *nul = nullptr);

static bool int_key(const Column &c) {
  return simple_key(c) && (c.type.kind() == ValueKind::SIGNED_INT ||
                           (c.type.kind() == ValueKind::UNSIGNED_INT && c.type.width() < 8));
}

// an integer key column that may hold nulls (fixed width <= 8, dense storage): packable into an exact
// composite with one field value reserved for null, so nulls match nulls (docs/semantics.md)
static bool nullable_int_key(const Column &c) {
  return c.nullable() && !c.is_var() && c.type.kind() != ValueKind::FIXED_BYTES && c.type.width() <= 8 &&
         c.data.element_size() == c.type.width() &&
         (c.type.kind() == ValueKind::SIGNED_INT || (c.type.kind() == ValueKind::UNSIGNED_INT && c.type.width() < 8));
}

static RadixKeys radix_keys(const Exec &ex, const TablePtr &left, const TablePtr &right, const JoinConfig &cfg,
                            bool words_ok) {
  const auto &lc = cfg.GetLeftColumnIdx();
  const auto &rc = cfg.GetRightColumnIdx();
  RadixKeys k;
  if (lc.size() == 1) {
    const Column &a = left->column(lc[0]), &b = right->column(rc[0]);
    if (simple_key(a) && simple_key(b) && a.type == b.type) {
      k.l = encode_keys(ex, left, lc, true).keys;
      k.r = encode_keys(ex, right, rc, true).keys;
      k.ok = true;
      return k;
    }
  }
  bool packable = lc.size() <= (size_t)kMaxCompositeKeys;
  // non-null string / binary / fixed-size binary key columns join through the verified row hash
  // (their bytes travel as gathered var-width columns; reference arrow_partition_kernels.cpp:243-305)
  auto hashed_ok = [](const Column &c) {
    return !c.nullable() && (c.is_var() || c.type.kind() == ValueKind::FIXED_BYTES);
  };
  for (size_t i = 0; i < lc.size(); ++i) {
    const Column &a = left->column(lc[i]), &b = right->column(rc[i]);
    if (!(a.type == b.type)) return k;
    const bool na = nullable_int_key(a), nb = nullable_int_key(b);
    if ((!simple_key(a) && !na && !hashed_ok(a)) || (!simple_key(b) && !nb && !hashed_ok(b))) return k;
    k.nulls = k.nulls || na || nb;
    packable = packable && (int_key(a) || na) && (int_key(b) || nb);
    if (hashed_ok(a)) trace::add_counter("join.radix.var_key", 1);
  }
  if (k.nulls && !packable) return k;  // nullable keys only as an exact composite
  k.ok = true;
  if (packable) {
    // per-key span over both relations (signed / byte storage: min / max of the column itself,
    // wider unsigned storage through its 64-bit image)
    auto span_of = [&](const Column &c, const TablePtr &t, int col) -> at::Tensor {
      if (c.data.numel() == 0)
        return at::tensor({std::numeric_limits<int64_t>::max(), std::numeric_limits<int64_t>::min()},
                          ex.opts(at::kLong));
      if (c.nullable()) {  // over the valid rows only (all null: an empty span)
        at::Tensor x = ex.empty_i64(t->Rows());
        hip::key64_from_column(c.view(), t->Rows(), ptr<int64_t>(x), ex.stream);
        const at::Tensor valid = c.validity.slice(0, 0, t->Rows()).ne(0);
        return at::stack({at::where(valid, x, std::numeric_limits<int64_t>::max()).min(),
                          at::where(valid, x, std::numeric_limits<int64_t>::min()).max()});
      }
      const bool direct = c.type.kind() == ValueKind::SIGNED_INT || c.type.width() == 1;
      at::Tensor x = direct ? c.data : encode_keys(ex, t, {col}, true).keys;
      auto m2 = at::aminmax(x);
      return at::stack({std::get<0>(m2).to(at::kLong), std::get<1>(m2).to(at::kLong)});
    };
    std::vector<at::Tensor> mm;
    for (size_t i = 0; i < lc.size(); ++i) {
      mm.push_back(span_of(left->column(lc[i]), left, lc[i]));
      mm.push_back(span_of(right->column(rc[i]), right, rc[i]));
    }
    const std::vector<int64_t> h = to_host_vec(at::cat(mm));
    const size_t nk = lc.size();
    k.lo.resize(nk);
    k.bits.resize(nk);
    k.shift.resize(nk);
    k.ncode.assign(nk, -1);
    int total = 0;
    for (size_t i = 0; i < nk; ++i) {
      k.lo[i] = std::min(h[4 * i], h[4 * i + 2]);
      const int64_t hi = std::max(h[4 * i + 1], h[4 * i + 3]);
      if (hi < k.lo[i]) k.lo[i] = 0;  // no valid key on either side
      uint64_t span = hi >= k.lo[i] ? (uint64_t)hi - (uint64_t)k.lo[i] : 0;
      if (left->column(lc[i]).nullable() || right->column(rc[i]).nullable()) {
        if (span >= (uint64_t)std::numeric_limits<int64_t>::max()) return k.ok = false, k;  // no free field value
        k.ncode[i] = (int64_t)span + 1;  // one past the largest valid field
        span += 1;
      }
      int b = 0;
      while (b < 64 && (span >> b) != 0) ++b;
      k.bits[i] = b;
      total += b;
    }
    if (total > 63 && k.nulls) return k.ok = false, k;  // nullable keys only as an exact composite
    if (total <= 63) {  // exact: key i occupies its own bit range (the last key the lowest bits)
      for (size_t i = nk, sh = 0; i-- > 0;) {
        k.shift[i] = (int)sh;
        sh += k.bits[i];
      }
      auto pack = [&](const TablePtr &t, const std::vector<int> &cols) {
        std::vector<ColView> v = views(t, cols);
        at::Tensor out = ex.empty_i64(t->Rows());
        KCALL(ex, composite_key_pack, v.data(), (int)nk, k.lo.data(), k.shift.data(), t->Rows(), ptr<int64_t>(out),
              k.nulls ? k.ncode.data() : nullptr);
        return out;
      };
      k.l = pack(left, lc);
      k.r = pack(right, rc);
      k.composite = true;
      trace::add_counter("join.radix.composite_key", 1);
      return k;
    }
  }
  k.verify = true;
  if (words_ok && lc.size() == 1 && left->device().is_cuda()) {
    // one fixed-length string key per side: its invertible word key (the join key, standing in for
    // word 0) and words 1..W-1 come out of one read of the bytes (the proxies below carry them)
    const int64_t L = fixed_var_len(ex, left->column(lc[0]));
    if (L > 0 && fixed_var_len(ex, right->column(rc[0])) == L) {
      k.wlen = L;
      k.lwords = var_to_words(ex, left->column(lc[0]), L, &k.l, true);
      k.rwords = var_to_words(ex, right->column(rc[0]), L, &k.r, true);
      trace::add_counter("join.radix.hashed_key", 1);
      return k;
    }
    // variable-length rows of <= 64 bytes: zero-padded words + the length (the padded word key seeds
    // its chain with the row's length, so equal keys + equal words 1..W-1 + equal lengths <=> equal
    // strings), no row-number gather of the key bytes after the join
    const Column &a = left->column(lc[0]), &b = right->column(rc[0]);
    if (a.is_var() && b.is_var() && knobs::Flag("RJ_VAR_WORDS", true)) {
      const auto ra = var_len_range(ex, a), rb = var_len_range(ex, b);
      const int64_t hi = std::max(ra.second, rb.second);
      if (ra.first >= 0 && rb.first >= 0 && hi <= 64) {
        k.vw = (int)std::max<int64_t>(1, (hi + 7) / 8);
        // text mode first (no zero byte in any row: the padding encodes the length, no length
        // column travels); a zero byte on either side redoes both sides with lengths
        at::Tensor nul = at::zeros({1}, ex.opts(at::kInt));
        unsigned int *np = reinterpret_cast<unsigned int *>(nul.data_ptr<int>());
        k.lwords = var_to_padded(ex, a, k.vw, &k.l, nullptr, np);
        k.rwords = var_to_padded(ex, b, k.vw, &k.r, nullptr, np);
        k.vtext = nul.item<int>() == 0;
        if (!k.vtext) {
          k.lwords = var_to_padded(ex, a, k.vw, &k.l, &k.llen);
          k.rwords = var_to_padded(ex, b, k.vw, &k.r, &k.rlen);
        }
        trace::add_counter(k.vtext ? "join.radix.var_word_key_text" : "join.radix.var_word_key", 1);
        return k;
      }
    }
  }
  k.l = encode_keys(ex, left, lc, false).keys;  // row hash of the key columns
  k.r = encode_keys(ex, right, rc, false).keys;
  trace::add_counter("join.radix.hashed_key", 1);
  return k;
}

// Rows of a hashed-key radix join whose key columns differ (64-bit key-hash collisions), as a bool
// mask, or an undefined tensor when there are none.  Rows where both sides are present only (outer
// rows carry one null side); row-wise equality of every key type (strings / binary byte-wise) by
// the rows_equal kernel.
static at::Tensor key_mismatches(const TablePtr &out, const JoinConfig &cfg, int nleft) {
  const auto &lc = cfg.GetLeftColumnIdx();
  const auto &rc = cfg.GetRightColumnIdx();
  const int64_t m = out->Rows();
  if (m == 0) return at::Tensor();
  Exec ex(out->device());
  std::vector<int> lcols(lc.begin(), lc.end()), rcols;
  for (int c : rc) rcols.push_back(nleft + c);
  std::vector<ColView> lv = views(out, lcols), rv = views(out, rcols);
  at::Tensor idx = at::arange(m, ex.opts(at::kLong));
  at::Tensor eq = ex.empty_u8(m);
  KCALL(ex, rows_equal, lv.data(), rv.data(), (int)lv.size(), ptr<int64_t>(idx), ptr<int64_t>(idx), m,
        ptr<uint8_t>(eq));
  at::Tensor bad = eq.eq(0);
  for (size_t i = 0; i < lc.size(); ++i) {  // compare where both sides hold a row
    const Column &a = out->column(lc[i]), &b = out->column(nleft + rc[i]);
    if (a.nullable()) bad.logical_and_(a.validity.slice(0, 0, m));
    if (b.nullable()) bad.logical_and_(b.validity.slice(0, 0, m));
  }
  return bad.any().item<bool>() ? bad : at::Tensor();
}

// A collision pairs rows whose keys differ: an inner join drops those rows; any other join type
// redoes the join on the exact path (nullptr), since a falsely matched row may owe an unmatched one.
static TablePtr drop_false_matches(const TablePtr &out, const JoinConfig &cfg, int nleft) {
  at::Tensor bad = key_mismatches(out, cfg, nleft);
  if (!bad.defined()) return out;
  const int64_t n = bad.sum().item<int64_t>();
  if (cfg.GetType() != JoinType::INNER) {
    trace::add_counter("join.radix.hash_collision_fallback", n);
    return nullptr;
  }
  trace::add_counter("join.radix.hash_collision_dropped", n);
  return FilterByMask(out, bad.logical_not());
}

// ---------------------------------------------------------------------------
// Bounded memory.  radix_join's working set -- both sides' partitioned copies (the
// second pass's slots) plus the first pass's transient copy of one side -- and its output are sized
// against the device headroom (free HBM + the caching allocator's cached blocks; config
// "memory_budget_mb" caps it).  When they do not fit, the join runs in C key-hash chunks: rows whose
// multiplicative key hash falls in chunk c are gathered from both sides, partitioned and joined into
// ONE output sink allocated for the whole result, so the peak is inputs + output + ~1/C of the
// working set (plus the chunk copies) instead of inputs + output + the whole working set.  The
// output size is estimated from an exactly joined 1/1024 key-hash sample when it matters.
// Reference: the retain=false release of shuffled inputs, table.cpp:150-155.
// ---------------------------------------------------------------------------
static int64_t radix_row_bytes(const TablePtr &t) {
  int64_t b = 0;
  for (const auto &c : t->columns()) b += c.type.width() + (c.nullable() ? 1 : 0);
  return std::max<int64_t>(b, 8);
}

static at::Tensor key_chunk_ids(const at::Tensor &k, int64_t C) {  // independent of fmix64 / fmix32 bits
  at::Tensor h = k * (int64_t)0x9E3779B97F4A7C15ull;
  return at::bitwise_and(at::bitwise_right_shift(h, 32), 0x7fffffff).remainder(C);
}

static int radix_join_chunks(const Exec &ex, const TablePtr &l, const TablePtr &r, const at::Tensor &lk,
                             const at::Tensor &rk, JoinType jt) {
  if (!ex.gpu) return 1;
  const int64_t head = l->GetContext()->DeviceHeadroom();
  if (head <= 0) return 1;
  const int64_t nl = l->Rows(), nr = r->Rows();
  const int64_t bl = radix_row_bytes(l) * nl, br = radix_row_bytes(r) * nr;
  const int64_t work = (int64_t)(1.17 * (double)(bl + br)) + (int64_t)(1.03 * (double)std::max(bl, br));
  const int64_t out_row = radix_row_bytes(l) + radix_row_bytes(r);
  const double budget = 0.92 * (double)head;
  // one output row per row of the larger side, with room to spare (plus every preserved row of an
  // outer join): no estimate needed
  const int64_t outer_rows = (jt == JoinType::LEFT || jt == JoinType::FULL_OUTER ? nl : 0) +
                             (jt == JoinType::RIGHT || jt == JoinType::FULL_OUTER ? nr : 0);
  if ((double)work + (1.5 * (double)std::max(nl, nr) + (double)outer_rows) * (double)out_row <= budget) return 1;
  int64_t est = 0;
  {  // exact join of a 1/1024 hash sample of both key sets, scaled up
    at::Tensor sl = at::bitwise_and(at::bitwise_right_shift(lk * (int64_t)0x632BE59BD9B4E019ll, 40), 1023).eq(0);
    at::Tensor sr = at::bitwise_and(at::bitwise_right_shift(rk * (int64_t)0x632BE59BD9B4E019ll, 40), 1023).eq(0);
    auto pr = hash_join_pairs(ex, lk.masked_select(sl), rk.masked_select(sr));
    est = (int64_t)(1.1 * 1024.0 * (double)pr.first.numel()) + 65536;
  }
  // the sample counts matched pairs only: an outer join also emits its preserved side's unmatched
  // rows -- up to all of them (a low-match join), so they are added in full
  est += outer_rows;
  const double out_bytes = (double)est * (double)out_row;
  if ((double)work + out_bytes <= budget) return 1;
  const double room = budget - out_bytes;
  const int C = room <= 0 ? 64 : (int)std::min<double>(64.0, std::ceil((double)(work + bl + br) / room));
  trace::add_counter("join.radix.memory_chunks", C);
  trace::add_counter("join.radix.estimated_output_rows", est);
  return std::max(C, 2);
}

// Bounded memory with retain = false and an int64 key column per side: the chunk pass IS the join's
// first radix pass -- every column moved once by the HIGH db1 bits of the narrowed partition hash
// (exact, so each first-level bucket is a contiguous row range; column groups with stable passes as
// in the chunk-major path, releasing each group's input buffers) -- and chunk c is a range of
// consecutive first-level buckets.  Per chunk only the slot second pass runs (radix_slot_segment_pass
// over its buckets) and radix_join joins the prepartitioned chunk into the sink (JoinSink::pre):
// the rows cross HBM in two passes, as in the unbounded join, instead of three (chunk-major pass +
// the chunk's own two passes).  nullptr when not applicable (the caller takes the chunk-major path).
static TablePtr radix_join_first_pass_chunks(const Exec &ex, const TablePtr &l, const TablePtr &r, const at::Tensor &lk,
                                             const at::Tensor &rk, int lkc, int rkc, const JoinConfig &cfg, int C,
                                             bool hashed_key) {
  if (l->IsRetain() || r->IsRetain() || hashed_key || lkc < 0 || rkc < 0 || lk.scalar_type() != at::kLong ||
      rk.scalar_type() != at::kLong || !knobs::Flag("RJ_FIRST_PASS_CHUNKS", true))
    return nullptr;
  // (nullable columns take the chunk-major path: radix_join sizes the LDS rows for packed validity
  // words, which these partitions do not carry)
  for (const TablePtr &t : {l, r})
    for (const auto &c : t->columns())
      if (c.is_var() || c.type.width() > 8 || c.nullable()) return nullptr;
  const int64_t nl = l->Rows(), nr = r->Rows();
  if (nl < (int64_t(1) << 20) || nr < (int64_t(1) << 20)) return nullptr;
  // the narrowed-key range, checked before anything is released: [base, base + 2^32), base = (left
  // key 0) - 2^31, as in radix_join
  const at::Tensor base_src = lk.slice(0, 0, 1).clone();
  {
    auto ml = at::aminmax(lk), mr = at::aminmax(rk);
    const at::Tensor h = at::stack({std::get<0>(ml), std::get<1>(ml), std::get<0>(mr), std::get<1>(mr), base_src[0]}).cpu();
    const int64_t base = h[4].item<int64_t>() - (int64_t(1) << 31);
    for (int i = 0; i < 4; ++i) {
      const int64_t v = h[i].item<int64_t>();
      if (v < base || (uint64_t)(v - base) > 0xffffffffull) return nullptr;
    }
  }
  // partition bits as radix_join chooses them for the whole join (narrowed keys)
  const bool build_left = nl < nr;
  const TablePtr &bt = build_left ? l : r;
  const int bkc = build_left ? lkc : rkc;
  const int oj = outer_mode(cfg.GetType(), build_left);
  RadixCols shape = radix_cols(bt, nullptr, nullptr);
  for (int c = 0, q = 0; c < bt->Columns(); ++c, ++q) {
    if (c == bkc) shape.in[q] = nullptr;
    if (bt->column(c).nullable() && !packs_validity(bt)) ++q;
  }
  const int64_t cap = hip::radix_join_capacity(shape.w.data(), shape.in.data(), (int)shape.w.size(), (oj & 2) != 0, 4);
  const int64_t nb = std::min(nl, nr);
  auto fits = [&](int64_t mean) { return (double)mean + 8.0 * std::sqrt((double)mean) + 16.0 <= (double)cap; };
  int bits = 0;
  while (bits < 24 && !fits((nb + (int64_t(1) << bits) - 1) >> bits)) ++bits;
  if (const int64_t xb = knobs::Int("RJ_EXTRA_BITS", 0))  // test knob: finer partitions (as radix_join)
    bits = std::min(bits + (int)std::max<int64_t>(0, xb), 2 * 10);
  const int db2 = std::min(9, bits / 2), db1 = bits - db2;
  if (bits < 11 || db1 > 10) return nullptr;
  int cbits = 1;  // chunks: twice what the retained-input budget asks for, as the chunk-major path
  while ((1 << cbits) < 2 * C) ++cbits;
  cbits = std::min(cbits, db1);
  const int gbits = db1 - cbits;  // first-level buckets per chunk: 2^gbits
  if ((1 << gbits) > 4096) return nullptr;
  at::Tensor narrow_bad = at::zeros({1}, ex.opts(at::kInt));
  hip::NarrowKeys nk;
  nk.base_src = ptr<int64_t>(base_src);
  nk.bad = reinterpret_cast<unsigned int *>(narrow_bad.data_ptr<int>());
  // ---- first pass of each side, column group by column group
  struct First {
    at::Tensor keys;                     // uint32 offsets, first-level bucket order
    std::vector<at::Tensor> data, valid;  // per column (data of the key column: undefined)
    std::vector<int64_t> boff;            // 2^db1 + 1 bucket starts
    at::Tensor boff_dev;                  // the same on the device
    int64_t n = 0;
  };
  auto first_pass = [&](const TablePtr &t, const at::Tensor &k, int kc) {
    First f;
    f.n = t->Rows();
    f.data.resize((size_t)t->Columns());
    f.valid.resize((size_t)t->Columns());
    std::vector<std::pair<int, bool>> ent;
    for (int c = 0; c < t->Columns(); ++c) {
      if (c != kc) ent.push_back({c, false});
      if (t->column(c).nullable()) ent.push_back({c, true});
    }
    constexpr size_t kGroup = 3;
    const size_t ngroups = std::max<size_t>(1, (ent.size() + kGroup - 1) / kGroup);
    const bool stable = ngroups > 1;
    f.keys = at::empty({f.n}, ex.opts(at::kInt));
    at::Tensor ws = ex.empty_i64(hip::radix_rows_pass_workspace(f.n, db1));
    for (size_t g = 0; g < ngroups; ++g) {
      const size_t e0 = ent.size() * g / ngroups, e1 = ent.size() * (g + 1) / ngroups;
      std::vector<const uint8_t *> in{reinterpret_cast<const uint8_t *>(k.data_ptr())};
      std::vector<uint8_t *> out{reinterpret_cast<uint8_t *>(f.keys.data_ptr())};
      std::vector<int> widths{8};
      for (size_t e = e0; e < e1; ++e) {
        const Column &col = t->column(ent[e].first);
        const at::Tensor &src = ent[e].second ? col.validity : col.data;
        at::Tensor dst = at::empty_like(src);
        in.push_back(reinterpret_cast<const uint8_t *>(src.data_ptr()));
        out.push_back(reinterpret_cast<uint8_t *>(dst.data_ptr()));
        widths.push_back(ent[e].second ? 1 : col.type.width());
        (ent[e].second ? f.valid : f.data)[(size_t)ent[e].first] = dst;
      }
      hip::radix_rows_pass(reinterpret_cast<const int64_t *>(k.data_ptr()), f.n, bits, db2, db1, in.data(), out.data(),
                           widths.data(), (int)in.size(), ptr<int64_t>(ws), ex.stream, stable, nullptr, 0, &nk);
      if (stable)
        for (size_t e = e0; e < e1; ++e) t->ReleaseBufferIfNotRetained(ent[e].first, ent[e].second);
    }
    at::Tensor offs = ex.empty_i64((int64_t(1) << db1) + 1);
    hip::radix_part_offsets32(reinterpret_cast<const uint32_t *>(f.keys.data_ptr()), f.n, db1, ptr<int64_t>(offs),
                              ex.stream);
    f.boff = to_host_vec(offs);
    f.boff_dev = offs;
    return f;
  };
  First fl = first_pass(l, lk, lkc);
  l->ReleaseIfNotRetained();
  First fr = first_pass(r, rk, rkc);
  r->ReleaseIfNotRetained();
  trace::add_counter("join.radix.released_inputs", 2);
  trace::add_counter("join.radix.first_pass_chunks", int64_t(1) << cbits);
  CYLON_CHECK(narrow_bad.item<int>() == 0, Code::ExecutionError, "first-pass chunks: a key left the narrowed range");
  // schema tables of a chunk (names, types, nullability; the data lives in the partitions)
  auto schema = [&](const TablePtr &t, int64_t rows) {
    std::vector<Column> cols;
    for (const auto &c : t->columns())
      cols.emplace_back(c.name, c.type, rows, at::empty({0}, c.data.options()), at::Tensor(),
                        c.nullable() ? at::empty({0}, ex.opts(at::kByte)) : at::Tensor());
    return Table::Make(t->GetContext(), std::move(cols));
  };
  const int64_t nparts = int64_t(1) << bits;
  auto slot_of = [&](int64_t rows) {
    const double mean = (double)rows / (double)nparts;
    return ((int64_t)(mean + 8.0 * std::sqrt(mean) + 64.0) + 7) & ~int64_t(7);
  };
  // second pass of one side's chunk [b0, b1) of first-level buckets -> its RadixSide
  auto second_pass = [&](const TablePtr &t, const First &f, int kc, int64_t b0, int64_t b1, int64_t slot) {
    const int64_t r0 = f.boff[(size_t)b0], r1 = f.boff[(size_t)b1], n = r1 - r0;
    const int nseg = (int)(b1 - b0);
    const int64_t nslots = int64_t(nseg) << db2;
    RadixSide s;
    std::vector<const uint8_t *> in{reinterpret_cast<const uint8_t *>(ptr<int32_t>(f.keys) + r0)};
    std::vector<int> widths{4};
    std::vector<std::pair<int, bool>> ent;
    for (int c = 0; c < t->Columns(); ++c) {
      if (c != kc) ent.push_back({c, false});
      if (t->column(c).nullable()) ent.push_back({c, true});
    }
    for (const auto &e : ent) {
      const at::Tensor &src = e.second ? f.valid[(size_t)e.first] : f.data[(size_t)e.first];
      const int w = e.second ? 1 : t->column(e.first).type.width();
      in.push_back(reinterpret_cast<const uint8_t *>(src.data_ptr()) + r0 * w);
      widths.push_back(w);
    }
    s.data.assign((size_t)t->Columns(), at::Tensor());
    s.valid.assign((size_t)t->Columns(), at::Tensor());
    s.is_key.assign((size_t)t->Columns(), false);
    s.vpos.assign((size_t)t->Columns(), -1);
    if (n == 0) {  // (an empty chunk side: empty partitions)
      s.keys = at::empty({0}, ex.opts(at::kInt));
      s.offs = at::zeros({nslots}, ex.opts(at::kLong));
      s.slot = 1;
      s.overflow = at::zeros({1}, ex.opts(at::kInt));
      for (int c = 0; c < t->Columns(); ++c) {
        s.is_key[(size_t)c] = c == kc;
        s.data[(size_t)c] = c == kc ? s.keys : at::empty({0}, t->column(c).data.options());
        if (t->column(c).nullable()) s.valid[(size_t)c] = at::empty({0}, ex.opts(at::kByte));
      }
      return s;
    }
    const at::Tensor bb = (f.boff_dev.slice(0, b0, b1) - r0).to(at::kInt);  // (device: no host copy per chunk)
    const int64_t rows = nslots * slot + hip::radix_slot_tile_rows();
    std::vector<at::Tensor> fin;
    std::vector<uint8_t *> out;
    fin.push_back(at::empty({rows}, ex.opts(at::kInt)));
    out.push_back(reinterpret_cast<uint8_t *>(fin.back().data_ptr()));
    for (const auto &e : ent) {
      const at::Tensor &src = e.second ? f.valid[(size_t)e.first] : f.data[(size_t)e.first];
      fin.push_back(at::empty({rows}, src.options()));
      out.push_back(reinterpret_cast<uint8_t *>(fin.back().data_ptr()));
    }
    int fbits = 0;
    while ((1 << fbits) < nseg) ++fbits;
    at::Tensor ws = ex.empty_i64(hip::radix_slot_workspace(std::max(1, fbits), db2));
    s.offs = ex.empty_i64(nslots);
    s.overflow = at::zeros({1}, ex.opts(at::kInt));
    hip::NarrowKeys nk2 = nk;
    nk2.kin4 = 1;
    hip::radix_slot_segment_pass(reinterpret_cast<const uint32_t *>(ptr<int32_t>(f.keys) + r0), n, bits, db2, in.data(),
                                 out.data(), widths.data(), (int)in.size(),
                                 reinterpret_cast<const uint32_t *>(bb.data_ptr<int>()), nseg, slot, ptr<int64_t>(ws),
                                 ptr<int64_t>(s.offs), reinterpret_cast<unsigned int *>(s.overflow.data_ptr<int>()),
                                 ex.stream, &nk2);
    s.slot = slot;
    s.keys = fin[0];
    for (int c = 0; c < t->Columns(); ++c) {
      s.is_key[(size_t)c] = c == kc;
      if (c == kc) s.data[(size_t)c] = s.keys;
    }
    for (size_t j = 0; j < ent.size(); ++j) (ent[j].second ? s.valid : s.data)[(size_t)ent[j].first] = fin[1 + j];
    return s;
  };
  JoinSink sink;
  sink.chunks_total = 1 << cbits;
  sink.sample_skew = false;
  const int64_t ls = slot_of(nl), rs = slot_of(nr);
  for (int64_t c = 0; c < (int64_t(1) << cbits); ++c) {
    const int64_t b0 = c << gbits, b1 = (c + 1) << gbits;
    PrePartition pp;
    pp.bits = gbits + db2;
    pp.base_src = base_src;
    int64_t lslot = ls, rslot = rs;
    const TablePtr ls_t = schema(l, fl.boff[(size_t)b1] - fl.boff[(size_t)b0]);
    const TablePtr rs_t = schema(r, fr.boff[(size_t)b1] - fr.boff[(size_t)b0]);
    for (int attempt = 0;; ++attempt) {
      pp.L = second_pass(l, fl, lkc, b0, b1, lslot);
      pp.R = second_pass(r, fr, rkc, b0, b1, rslot);
      pp.overflowed = false;
      sink.pre = &pp;
      const bool done = radix_join(ex, ls_t, rs_t, pp.L.keys, pp.R.keys, cfg, &sink) != nullptr;
      sink.pre = nullptr;
      if (done) break;
      CYLON_CHECK(pp.overflowed && attempt == 0, Code::ExecutionError,
                  "radix join of a first-pass chunk of released (retain = false) inputs did not complete");
      // a partition beyond its slot (skewed keys; radix_join saw the flags and wrote nothing): the
      // overflowing side again with slots as large as the chunk's largest first-level bucket (which
      // bounds every partition of the chunk)
      trace::add_counter("join.radix.slot_overflow", 1);
      auto widest = [&](const First &f) {
        int64_t m = 0;
        for (int64_t b = b0; b < b1; ++b) m = std::max(m, f.boff[(size_t)b + 1] - f.boff[(size_t)b]);
        return (m + 7) & ~int64_t(7);
      };
      if (pp.overflow_l) lslot = std::max<int64_t>(lslot, widest(fl));
      if (pp.overflow_r) rslot = std::max<int64_t>(rslot, widest(fr));
    }
    ++sink.chunks_done;
  }
  return sink.finish(l->GetContext());
}

// the radix join in C key-hash chunks into one sink (see above); nullptr if a chunk's radix join fails
static TablePtr radix_join_chunked(const Exec &ex, const TablePtr &l, const TablePtr &r, const at::Tensor &lk,
                                   const at::Tensor &rk, const JoinConfig &cfg, int C, bool hashed_key = false) {
  auto key_col = [](const TablePtr &t, const at::Tensor &k) {
    for (int c = 0; c < t->Columns(); ++c)
      if (t->column(c).data.defined() && t->column(c).data.data_ptr() == k.data_ptr()) return c;
    return -1;
  };
  const int lkc = key_col(l, lk), rkc = key_col(r, rk);
  if (TablePtr t = radix_join_first_pass_chunks(ex, l, r, lk, rk, lkc, rkc, cfg, C, hashed_key)) return t;
  // retain = false on both inputs: one chunk-major pass per side (radix.cpp RadixChunkPartition: every
  // column, chunk = the LOW bits of fmix64(key)) whose input is released right after it, so each chunk
  // is a contiguous slice and the inputs are read once -- instead of a chunk-id filter + row gather
  // per chunk, whose gathers touch nearly every cache line of the inputs C times
  if (!l->IsRetain() && !r->IsRetain() && C <= 1024) {
    int cbits = 1;  // (twice the chunks the retained-input budget asks for: the copies and the output
    while ((1 << cbits) < 2 * C) ++cbits;  // hold ~inputs + output, so each chunk's working set must be small)
    const int64_t C2 = int64_t(1) << cbits;
    // Column groups: a pass moves the key plus <= kGroup other buffers, and the group's input buffers
    // are released before the next group's pass, so the side's copy reuses its own input's memory
    // (peak: the inputs + one group's copies, not the inputs + a whole second copy).  With several
    // groups the passes rank stably (exact tile offsets, stable in-tile order): every group's rows
    // land where the first group's did, the later passes rewriting the same keys in place.
    constexpr size_t kGroup = 3;
    auto chunk_major = [&](const TablePtr &t, const at::Tensor &k, int kc, at::Tensor &kout, std::vector<int64_t> &offs) {
      std::vector<std::pair<int, bool>> ent;  // (column, validity?) of every buffer that moves with the key
      for (int c = 0; c < t->Columns(); ++c) {
        if (c != kc) ent.push_back({c, false});
        if (t->column(c).nullable()) ent.push_back({c, true});
      }
      const size_t ngroups = std::max<size_t>(1, (ent.size() + kGroup - 1) / kGroup);
      const bool stable = ngroups > 1;
      std::vector<at::Tensor> dout(t->Columns()), vout(t->Columns());
      at::Tensor o;
      for (size_t g = 0; g < ngroups; ++g) {
        const size_t e0 = ent.size() * g / ngroups, e1 = ent.size() * (g + 1) / ngroups;
        std::vector<at::Tensor> sub{k};
        std::vector<int> widths{8};
        for (size_t e = e0; e < e1; ++e) {
          const Column &col = t->column(ent[e].first);
          sub.push_back(ent[e].second ? col.validity : col.data);
          widths.push_back(ent[e].second ? 1 : col.type.width());
        }
        std::vector<at::Tensor> res =
            RadixChunkPartition(ex, std::move(sub), widths, cbits, g == 0 ? &o : nullptr, g == 0 ? nullptr : &kout, stable);
        if (g == 0) kout = res[0];
        for (size_t e = e0; e < e1; ++e) {
          (ent[e].second ? vout : dout)[(size_t)ent[e].first] = res[1 + e - e0];
          if (stable) t->ReleaseBufferIfNotRetained(ent[e].first, ent[e].second);
        }
      }
      offs = to_host_vec(o);
      std::vector<Column> cols;
      for (int c = 0; c < t->Columns(); ++c) {
        const Column &col = t->column(c);
        at::Tensor d = c == kc ? kout : dout[(size_t)c];
        if (c == kc && d.scalar_type() != col.data.scalar_type()) d = d.view(col.data.scalar_type());
        cols.emplace_back(col.name, col.type, kout.numel(), d, at::Tensor(), vout[(size_t)c]);
      }
      TablePtr res = Table::Make(t->GetContext(), std::move(cols));
      t->ReleaseIfNotRetained();
      trace::add_counter("join.radix.released_inputs", 1);
      if (stable) trace::add_counter("join.radix.chunk_pass_groups", (int64_t)ngroups);
      return res;
    };
    at::Tensor lkp, rkp;
    std::vector<int64_t> lo, ro;
    TablePtr lp = chunk_major(l, lk, lkc, lkp, lo);
    TablePtr rp = chunk_major(r, rk, rkc, rkp, ro);
    trace::add_counter("join.radix.chunk_pass", 2);
    JoinSink sink;
    sink.chunks_total = (int)C2;
    sink.sample_skew = false;
    auto slice_tab = [&](const TablePtr &t, int64_t a, int64_t b) {
      std::vector<Column> cols;
      for (const auto &c : t->columns()) cols.push_back(c.slice(a, b - a));
      return Table::Make(t->GetContext(), std::move(cols));
    };
    for (int64_t c = 0; c < C2; ++c) {
      TablePtr lc = slice_tab(lp, lo[c], lo[c + 1]), rc = slice_tab(rp, ro[c], ro[c + 1]);
      const at::Tensor lkc_t = lkc >= 0 ? lc->column(lkc).data.view(at::kLong) : lkp.slice(0, lo[c], lo[c + 1]);
      const at::Tensor rkc_t = rkc >= 0 ? rc->column(rkc).data.view(at::kLong) : rkp.slice(0, ro[c], ro[c + 1]);
      CYLON_CHECK(radix_join(ex, lc, rc, lkc_t, rkc_t, cfg, &sink, hashed_key), Code::ExecutionError,
                  "radix join of a chunk of released (retain = false) inputs did not complete");
      ++sink.chunks_done;
    }
    return sink.finish(l->GetContext());
  }
  const at::Tensor cl = key_chunk_ids(lk, C), cr = key_chunk_ids(rk, C);
  JoinSink sink;
  sink.chunks_total = C;
  for (int c = 0; c < C; ++c) {
    at::Tensor il = cl.eq(c).nonzero().flatten(), ir = cr.eq(c).nonzero().flatten();
    TablePtr lc = Gather(l, il), rc = Gather(r, ir);
    const at::Tensor lkc_t = lkc >= 0 ? lc->column(lkc).data : lk.index_select(0, il);
    const at::Tensor rkc_t = rkc >= 0 ? rc->column(rkc).data : rk.index_select(0, ir);
    il = at::Tensor();
    ir = at::Tensor();
    if (!radix_join(ex, lc, rc, lkc_t, rkc_t, cfg, &sink, hashed_key)) return nullptr;
    ++sink.chunks_done;
  }
  return sink.finish(l->GetContext());
}

// Fixed-length strings / binaries (every row L <= 64 bytes, no nulls) travel through the radix join
// as ceil(L / 8) int64 word columns -- moved by the partition passes and the write kernel like any
// payload -- instead of a row number and a gather by it afterwards (random reads at ~50 G accesses/s:
// a 200M x 200M join on 16-byte string keys spent 26 of its 62 ms gathering, profiles/r05).
static int64_t fixed_var_len(const Exec &ex, const Column &c) {  // L, or -1
  if (c.nullable() || !(c.type.type == Type::STRING || c.type.type == Type::BINARY) || c.length == 0) return -1;
  at::Tensor mm = ex.empty_i64(2);
  hip::var_len_minmax(ptr<int64_t>(c.offsets), c.length, ptr<int64_t>(mm), ex.stream);
  at::Tensor h = mm.cpu();
  const int64_t lo = h[0].item<int64_t>(), hi = h[1].item<int64_t>();
  return lo == hi && lo > 0 && lo <= 64 ? lo : -1;
}

// words 0..W-1 (inv: words 1..W-1, *hash = the invertible word key that stands in for word 0)
static std::vector<at::Tensor> var_to_words(const Exec &ex, const Column &c, int64_t L, at::Tensor *hash, bool inv) {
  const int64_t n = c.length, W = (L + 7) / 8;
  if (hash) *hash = ex.empty_i64(n);
  const int64_t o0 = c.offsets.slice(0, 0, 1).cpu().item<int64_t>();
  std::vector<at::Tensor> out;
  std::vector<int64_t *> wp;
  if (inv) wp.push_back(nullptr);
  for (int64_t j = inv ? 1 : 0; j < W; ++j) {
    out.push_back(ex.empty_i64(n));
    wp.push_back(ptr<int64_t>(out.back()));
  }
  hip::bytes_to_words(ptr<uint8_t>(c.data) + o0, n, (int)L, wp.data(), ex.stream,
                      hash ? reinterpret_cast<uint64_t *>(ptr<int64_t>(*hash)) : nullptr, inv);
  return out;
}

// {min, max} row length of a non-null string / binary column, or {-1, -1}
static std::pair<int64_t, int64_t> var_len_range(const Exec &ex, const Column &c) {
  if (c.nullable() || !(c.type.type == Type::STRING || c.type.type == Type::BINARY)) return {-1, -1};
  if (c.length == 0) return {0, 0};
  at::Tensor mm = ex.empty_i64(2);
  hip::var_len_minmax(ptr<int64_t>(c.offsets), c.length, ptr<int64_t>(mm), ex.stream);
  const std::vector<int64_t> h = to_host_vec(mm);
  return {h[0], h[1]};
}

// a variable-length column (rows <= 8 W bytes) as W zero-padded words: *key = the padded word key
// (word 0's stand-in), *lens = the row lengths; returns words 1..W-1.  One read of the bytes.
static std::vector<at::Tensor> var_to_padded(const Exec &ex, const Column &c, int W, at::Tensor *key,
                                             at::Tensor *lens, unsigned int *nul) {
  const int64_t n = c.length;
  *key = ex.empty_i64(n);
  if (lens) *lens = ex.empty_i64(n);
  std::vector<at::Tensor> out;
  std::vector<int64_t *> wp{nullptr};
  for (int j = 1; j < W; ++j) {
    out.push_back(ex.empty_i64(n));
    wp.push_back(ptr<int64_t>(out.back()));
  }
  hip::var_to_words(ptr<uint8_t>(c.data), ptr<int64_t>(c.offsets), n, W, wp.data(),
                    reinterpret_cast<uint64_t *>(ptr<int64_t>(*key)), lens ? ptr<int64_t>(*lens) : nullptr, nullptr,
                    ex.stream, lens == nullptr, nul);
  return out;
}

// wc = {padded word key, words 1..W-1[, lengths]} of m rows -> a string / binary column (rows whose
// key column is null -- an outer join's absent side -- become null, zero bytes).  Text mode (no
// length column): the lengths come from the words.
static Column padded_to_var(const Exec &ex, const std::string &name, const DataType &type,
                            const std::vector<Column> &wc, int W, bool text) {
  const Column &kc = wc[0];
  const int64_t m = kc.length;
  at::Tensor lens;
  if (text) {
    lens = ex.empty_i64(std::max<int64_t>(m, 1)).slice(0, 0, m);
    std::vector<const int64_t *> wp;
    for (int j = 0; j < W; ++j) wp.push_back(ptr<int64_t>(wc[(size_t)j].data));
    hip::padded_text_lens(wp.data(), reinterpret_cast<const uint64_t *>(wp[0]), m, W, ptr<int64_t>(lens), ex.stream);
  } else {
    lens = wc[(size_t)W].data.slice(0, 0, m);
  }
  if (kc.nullable()) lens = at::where(kc.validity.slice(0, 0, m).to(at::kBool), lens, at::zeros({1}, lens.options()));
  // offsets = the device exclusive scan of the lengths (offs[m] = total): no zero fill + ATen cumsum
  at::Tensor offs = m ? exclusive_scan(ex, lens.contiguous()) : at::zeros({1}, ex.opts(at::kLong));
  const int64_t nbytes = m ? read_i64(offs, m) : 0;
  at::Tensor bytes = ex.empty_bytes(std::max<int64_t>(1, nbytes));
  std::vector<const int64_t *> wp;
  for (int j = 0; j < W; ++j) wp.push_back(ptr<int64_t>(wc[(size_t)j].data));
  hip::words_to_var(wp.data(), reinterpret_cast<const uint64_t *>(wp[0]), ptr<int64_t>(lens),
                    ptr<int64_t>(offs), m, W, ptr<uint8_t>(bytes), ex.stream, text);
  return Column(name, type, m, bytes.slice(0, 0, nbytes), offs, kc.validity);
}

// wc = the word columns 0..W-1 (inv: wc[0] = the invertible word key, wc[1..] = words 1..W-1)
static Column words_to_var(const Exec &ex, const std::string &name, const DataType &type,
                           const std::vector<Column> &wc, int64_t L, bool inv = false) {
  const int64_t m = wc[0].length;
  std::vector<const int64_t *> wp;
  for (const auto &c : wc) wp.push_back(ptr<int64_t>(c.data));
  at::Tensor bytes = ex.empty_bytes(std::max<int64_t>(1, m * L));
  hip::words_to_bytes(wp.data(), m, (int)L, ptr<uint8_t>(bytes), ex.stream,
                      inv ? reinterpret_cast<const uint64_t *>(wp[0]) : nullptr);
  at::Tensor offs = at::arange(0, (m + 1) * L, L, ex.opts(at::kLong));
  // (a null row of an outer join keeps L zero bytes under its null: Arrow allows any length there)
  return Column(name, type, m, bytes.slice(0, 0, m * L), offs, wc[0].validity);
}

// LDS radix join of any large device join (every type, one or several keys, var-width payload
// columns); nullptr when ineligible or when the kernels report an overflow / collision.  Tables
// with string / binary / list columns join their fixed-width columns plus a row-number column,
// and the var-width columns are gathered by those row numbers afterwards (two-pass offsets +
// bytes gather, row -1 -> null).  Exact composite keys (no sink): the proxy tables carry the
// composite in place of the key columns, so the passes and the write kernel move one 8-byte key
// (as in the one-key join), and composite_key_unpack rebuilds the key columns of the output.
static TablePtr radix_join_any(const Exec &ex, const TablePtr &left, const TablePtr &right, const JoinConfig &cfg,
                               JoinSink *sink) {
  std::optional<trace::Phase> keys_phase;
  keys_phase.emplace("join.radix.keys", ex.device);  // key encoding + proxies (ends before the join)
  RadixKeys k = radix_keys(ex, left, right, cfg, sink == nullptr);  // (a sink takes no var-width keys)
  if (!k.ok) return nullptr;
  auto var_col = [](const Column &c) { return c.is_var() || c.type.kind() == ValueKind::FIXED_BYTES; };
  auto has_var = [&](const TablePtr &t) {
    for (const auto &c : t->columns())
      if (var_col(c)) return true;
    return false;
  };
  const bool lvar = has_var(left), rvar = has_var(right);
  // a chunked distributed join writes into its sink: fixed-width tables on exact keys only
  if ((lvar || rvar || k.verify) && sink) return nullptr;
  const bool ckey = k.composite && !sink;
  const auto &lc = cfg.GetLeftColumnIdx();
  const auto &rc = cfg.GetRightColumnIdx();
  // proxy of a side: [composite key] + its fixed-width non-key columns + the word columns of its
  // fixed-length strings [+ the row number, when other var-width columns are gathered by it];
  // pos[c] = proxy column of the side's column c (-1: rebuilt from the key or gathered);
  // wlen[c] = L of a column carried as words (from proxy column pos[c]), else -1
  static const std::string kRow = "__cylon_row", kKey = "__cylon_key";
  // vwid[c] = W of a variable-length key carried as W padded words + its length column
  auto proxy = [&](const TablePtr &t, bool &var, const std::vector<int> &keys, const at::Tensor &img,
                   std::vector<int> &pos, std::vector<int64_t> &wlen, std::vector<int> &vwid,
                   const std::vector<at::Tensor> &kwords, const at::Tensor &klens) {
    pos.assign(t->Columns(), -1);
    wlen.assign(t->Columns(), -1);
    vwid.assign(t->Columns(), 0);
    std::vector<Column> cols;
    if (ckey) cols.emplace_back(kKey, DataType(Type::INT64), t->Rows(), img);
    var = false;
    for (int c = 0; c < t->Columns(); ++c) {
      const Column &col = t->column(c);
      if (ckey && std::find(keys.begin(), keys.end(), c) != keys.end()) continue;
      if (var_col(col)) {
        if (k.vw > 0 && c == keys[0]) {  // padded word key, words 1..W-1, length (radix_keys)
          vwid[c] = k.vw;
          pos[c] = (int)cols.size();
          cols.emplace_back("__cylon_wk" + std::to_string(c), DataType(Type::INT64), t->Rows(), img);
          for (size_t j = 0; j < kwords.size(); ++j)
            cols.emplace_back("__cylon_w" + std::to_string(c) + "_" + std::to_string(j + 1), DataType(Type::INT64),
                              t->Rows(), kwords[j]);
          if (!k.vtext) cols.emplace_back("__cylon_wl" + std::to_string(c), DataType(Type::INT64), t->Rows(), klens);
          continue;
        }
        const bool kw = k.wlen > 0 && c == keys[0];  // the key's word key + words from radix_keys
        const int64_t L = kw ? k.wlen : fixed_var_len(ex, col);
        if (L < 0) {
          var = true;
          continue;
        }
        wlen[c] = L;
        pos[c] = (int)cols.size();
        // the key's word key is the join key itself (no pass moves it twice), then words 1..W-1
        if (kw) cols.emplace_back("__cylon_wk" + std::to_string(c), DataType(Type::INT64), t->Rows(), img);
        std::vector<at::Tensor> w = kw ? kwords : var_to_words(ex, col, L);
        for (size_t j = 0; j < w.size(); ++j)
          cols.emplace_back("__cylon_w" + std::to_string(c) + "_" + std::to_string(j + (kw ? 1 : 0)),
                            DataType(Type::INT64), t->Rows(), w[j]);
        continue;
      }
      pos[c] = (int)cols.size();
      cols.push_back(col);
    }
    if (var) cols.emplace_back(kRow, DataType(Type::INT64), t->Rows(), at::arange(t->Rows(), ex.opts(at::kLong)));
    return Table::Make(t->GetContext(), std::move(cols));
  };
  std::vector<int> lpos, rpos, lvw, rvw;
  std::vector<int64_t> lwlen, rwlen;
  const bool lpx = lvar || ckey, rpx = rvar || ckey;
  bool lgather = false, rgather = false;  // var-width columns gathered by row number after the join
  TablePtr lp = lpx ? proxy(left, lgather, lc, k.l, lpos, lwlen, lvw, k.lwords, k.llen) : left;
  TablePtr rp = rpx ? proxy(right, rgather, rc, k.r, rpos, rwlen, rvw, k.rwords, k.rlen) : right;
  if (lpx || rpx) {
    int64_t nw = 0;
    for (int64_t L : lwlen) nw += L > 0;
    for (int64_t L : rwlen) nw += L > 0;
    for (int W : lvw) nw += W > 0;
    for (int W : rvw) nw += W > 0;
    if (nw) trace::add_counter("join.radix.word_columns", nw);
  }
  if (!radix_eligible(lp) || !radix_eligible(rp)) return nullptr;
  keys_phase.reset();
  const int mchunks = sink ? 1 : radix_join_chunks(ex, lp, rp, k.l, k.r, cfg.GetType());
  TablePtr out = mchunks > 1 ? radix_join_chunked(ex, lp, rp, k.l, k.r, cfg, mchunks, k.verify)
                             : radix_join(ex, lp, rp, std::move(k.l), std::move(k.r), cfg, sink, k.verify);
  if (!out) return nullptr;
  if (k.verify && !lvar && !rvar) return drop_false_matches(out, cfg, left->Columns());
  if (!lpx && !rpx) return out;
  CYLON_PHASE("join.radix.rebuild", ex.device);  // word / proxy columns back to the output columns
  const JoinType jt = cfg.GetType();
  // Inner join on one fixed-length string key per side (same type and length, no nulls): the key
  // words are verified equal row by row below, so the right output key column is the left one's
  // bytes and offsets (one words -> bytes conversion; CYLON_RJ_SHARE_KEY=0 converts both).
  const bool share_skey = jt == JoinType::INNER && k.verify && lc.size() == 1 && lpx && rpx &&
                          ((lwlen[lc[0]] > 0 && lwlen[lc[0]] == rwlen[rc[0]]) || (lvw[lc[0]] > 0 && lvw[lc[0]] == rvw[rc[0]])) &&
                          left->column(lc[0]).type == right->column(rc[0]).type &&
                          !left->column(lc[0]).nullable() && !right->column(rc[0]).nullable() &&
                          knobs::Flag("RJ_SHARE_KEY", true);
  auto side = [&](const TablePtr &orig, bool px, bool var, const std::vector<int> &pos, const std::vector<int64_t> &wlen,
                  const std::vector<int> &vwid, const std::vector<int> &keys, int first, int np, bool may_null,
                  const std::string &prefix, int skip_col) {
    std::vector<Column> cols(orig->Columns());
    if (!px) {
      for (int c = 0; c < orig->Columns(); ++c) cols[c] = out->column(first + c);
      return cols;
    }
    for (int c = 0; c < orig->Columns(); ++c) {
      if (pos[c] < 0 || c == skip_col) continue;
      if (vwid[c] > 0) {  // a variable-length string from its padded words + length
        std::vector<Column> wc;
        for (int j = 0; j < vwid[c] + (k.vtext ? 0 : 1); ++j) wc.push_back(out->column(first + pos[c] + j));
        cols[c] = padded_to_var(ex, prefix + orig->column(c).name, orig->column(c).type, wc, vwid[c], k.vtext);
        continue;
      }
      if (wlen[c] > 0) {  // a fixed-length string from its word columns
        const int64_t L = wlen[c];
        std::vector<Column> wc;
        for (int64_t j = 0; j < (L + 7) / 8; ++j) wc.push_back(out->column(first + pos[c] + (int)j));
        cols[c] = words_to_var(ex, prefix + orig->column(c).name, orig->column(c).type, wc, L,
                               k.wlen > 0 && c == keys[0]);
      } else {
        cols[c] = out->column(first + pos[c]);
      }
    }
    if (ckey) {  // the key columns from the composite (its validity: the side's presence)
      const Column &img = out->column(first);
      std::vector<MutColView> mv;
      for (size_t i = 0; i < keys.size(); ++i) {
        const Column &kc = orig->column(keys[i]);
        Column o = make_fixed_column(prefix + kc.name, kc.type, img.length, ex.device, false);
        o.validity = img.validity;
        MutColView v;
        if (k.ncode[i] >= 0) {  // nulls come back where the field holds the null code (own validity)
          o.validity = img.validity.defined() ? img.validity.clone() : at::ones({img.length}, ex.opts(at::kByte));
          v.valid = img.length ? o.validity.data_ptr<uint8_t>() : nullptr;
        }
        v.data = reinterpret_cast<uint8_t *>(ptr<uint8_t>(o.data.view(at::kByte)));
        v.width = kc.type.width();
        v.kind = static_cast<int>(kc.type.kind());
        mv.push_back(v);
        cols[keys[i]] = std::move(o);
      }
      KCALL(ex, composite_key_unpack, ptr<int64_t>(img.data), img.length, (int)keys.size(), k.lo.data(),
            k.shift.data(), k.bits.data(), mv.data(), k.nulls ? k.ncode.data() : nullptr);
      trace::add_counter("join.radix.composite_unpacked", (int64_t)keys.size());
    }
    if (!var) return cols;
    const Column &rid = out->column(first + np - 1);
    at::Tensor idx = rid.nullable() ? at::where(rid.validity.to(at::kBool), rid.data, at::full({1}, -1, rid.data.options()))
                                    : rid.data;
    std::vector<Column> vcols;
    std::vector<int> vpos;
    for (int c = 0; c < orig->Columns(); ++c)
      if (var_col(orig->column(c))) {
        vcols.push_back(orig->column(c));
        vpos.push_back(c);
      }
    TablePtr g = GatherNullable(Table::Make(orig->GetContext(), vcols), idx.contiguous(), may_null);
    for (size_t j = 0; j < vpos.size(); ++j) cols[vpos[j]] = g->column((int)j).with_name(prefix + g->column((int)j).name);
    return cols;
  };
  std::vector<Column> all = side(left, lpx, lgather, lpos, lwlen, lvw, lc, 0, lp->Columns(), left_may_null(jt),
                                cfg.GetLeftTablePrefix(), -1);
  std::vector<Column> rcols = side(right, rpx, rgather, rpos, rwlen, rvw, rc, lp->Columns(), rp->Columns(),
                                   right_may_null(jt), cfg.GetRightTablePrefix(), share_skey ? rc[0] : -1);
  if (share_skey) {
    rcols[rc[0]] = all[lc[0]].with_name(cfg.GetRightTablePrefix() + right->column(rc[0]).name);
    trace::add_counter("join.radix.shared_key_column", 1);
  }
  for (auto &c : rcols) all.push_back(std::move(c));
  TablePtr res = Table::Make(left->GetContext(), std::move(all));
  if (lgather || rgather) trace::add_counter("join.radix.var_gather", 1);
  if (!k.verify) return res;
  // keys that are all fixed-length strings: compare their word columns (8 bytes per compare)
  bool words = lpx && rpx;
  for (size_t i = 0; words && i < lc.size(); ++i)
    words = (lwlen[lc[i]] > 0 && lwlen[lc[i]] == rwlen[rc[i]]) || (lvw[lc[i]] > 0 && lvw[lc[i]] == rvw[rc[i]]);
  if (!words) return drop_false_matches(res, cfg, left->Columns());
  const int64_t m = out->Rows();
  if (m == 0) return res;
  std::vector<const int64_t *> aw, bw;
  const int rfirst = lp->Columns();
  // (a word-key column: the key words 1..W-1 -- equal word keys were matched, so word 0 is equal too;
  // a padded word key: words 1..W-1 and the length, which seeds the key's chain)
  for (size_t i = 0; i < lc.size(); ++i) {
    const int64_t nwc = lvw[lc[i]] > 0 ? lvw[lc[i]] + (k.vtext ? 0 : 1) : (lwlen[lc[i]] + 7) / 8;
    for (int64_t j = (k.wlen > 0 || k.vw > 0) ? 1 : 0; j < nwc; ++j) {
      aw.push_back(ptr<int64_t>(out->column(lpos[lc[i]] + (int)j).data));
      bw.push_back(ptr<int64_t>(out->column(rfirst + rpos[rc[i]] + (int)j).data));
    }
  }
  if (aw.empty()) return res;  // an L <= 8 word key is the string itself: no false matches
  if (aw.size() > 8) return drop_false_matches(res, cfg, left->Columns());
  const Column &lw = out->column(lpos[lc[0]]), &rw = out->column(rfirst + rpos[rc[0]]);
  at::Tensor badb = ex.empty_u8(m);  // both sides present and some key word differs
  at::Tensor nbadd = ex.empty_i64(1);
  hip::words_mismatch(aw.data(), bw.data(), (int)aw.size(), lw.nullable() ? ptr<uint8_t>(lw.validity) : nullptr,
                      rw.nullable() ? ptr<uint8_t>(rw.validity) : nullptr, m, ptr<uint8_t>(badb), ptr<int64_t>(nbadd),
                      ex.stream);
  const int64_t nbad = nbadd.item<int64_t>();
  if (nbad == 0) return res;
  at::Tensor bad = badb.to(at::kBool);
  if (jt != JoinType::INNER) {
    trace::add_counter("join.radix.hash_collision_fallback", nbad);
    return nullptr;
  }
  trace::add_counter("join.radix.hash_collision_dropped", nbad);
  return FilterByMask(res, bad.logical_not());
}

// Local join.  With a sink (chunked distributed join) the radix path writes into
// the sink and nullptr is returned; other paths return their table.
static TablePtr join_local(const TablePtr &left, const TablePtr &right, const JoinConfig &cfg, JoinSink *sink) {
  const bool big = left->device().is_cuda() && std::min(left->Rows(), right->Rows()) >= radix_join_min_rows();
  const JoinType jt = cfg.GetType();
  if (big && jt == JoinType::INNER && cfg.GetAlgorithm() == JoinAlgorithm::SORT &&
      cfg.GetLeftColumnIdx().size() == 1 && radix_eligible(left) && radix_eligible(right)) {
    const Column &a = left->column(cfg.GetLeftColumnIdx()[0]);
    const Column &b = right->column(cfg.GetRightColumnIdx()[0]);
    if (simple_key(a) && simple_key(b) && a.type == b.type && a.type.kind() != ValueKind::FLOAT) {
      Exec ex(left->device());
      if (range_join_enabled())
        if (TablePtr out = range_join(ex, left, right, cfg)) return out;
      return sorted_merge_join(ex, left, right, cfg);
    }
  }
  // the LDS radix hash join: hash joins of every type, and sort-algorithm outer / multi-key
  // joins (their output order is unspecified, docs/semantics.md)
  if (big && (cfg.GetAlgorithm() == JoinAlgorithm::HASH || jt != JoinType::INNER ||
              cfg.GetLeftColumnIdx().size() > 1)) {
    Exec ex(left->device());
    if (TablePtr out = radix_join_any(ex, left, right, cfg, sink)) return sink ? nullptr : out;
  }
  TablePtr l = left, r = right;
  auto idx = join_impl(left, right, cfg, true, &l, &r);
  const bool lnull = left_may_null(jt);
  const bool rnull = right_may_null(jt);
  CYLON_PHASE("join.materialize", l->device());
  TablePtr lo = GatherNullable(l, idx.first, lnull);
  TablePtr ro = GatherNullable(r, idx.second, rnull);
  std::vector<Column> cols;
  cols.reserve(lo->Columns() + ro->Columns());
  for (const auto &c : lo->columns()) cols.push_back(c.with_name(cfg.GetLeftTablePrefix() + c.name));
  for (const auto &c : ro->columns()) cols.push_back(c.with_name(cfg.GetRightTablePrefix() + c.name));
  return Table::Make(left->GetContext(), std::move(cols));
}

TablePtr Join(const TablePtr &left, const TablePtr &right, const JoinConfig &cfg) {
  return join_local(left, right, cfg, nullptr);
}

TablePtr DistributedJoin(const TablePtr &left, const TablePtr &right, const JoinConfig &cfg) {
  auto ctx = left->GetContext();
  if (!ctx->ShuffleRequired()) return Join(left, right, cfg);
  JoinSink sink;
  TablePtr whole;
  ShufflePairPlanned(left, cfg.GetLeftColumnIdx(), right, cfg.GetRightColumnIdx(),
                     [&](int, int K, const TablePtr &l, const TablePtr &r) {
                       if (K == 1) {  // unchunked: the shuffled pair is joined as a whole
                         whole = Join(l, r, cfg);
                         return;
                       }
                       sink.chunks_total = K;
                       if (TablePtr t = join_local(l, r, cfg, &sink)) sink.tables.push_back(t);
                       ++sink.chunks_done;
                     });
  return whole ? whole : sink.finish(ctx);
}

}  // namespace ops
}  // namespace cylon
