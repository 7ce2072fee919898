// Shared radix partitioning driver for the LDS radix join and group-by
// (kernels: radix_join.hip k_rp_hist / k_rows_pass / k_part_offsets).
#include "cylon/knobs.hpp"
#include <algorithm>
#include <cmath>
#include <cstdlib>

#include <atomic>

#include "util.hpp"
#include "../trace.hpp"

namespace cylon {
namespace ops {

BytePacking PackByteColumns(const Exec &ex, std::vector<at::Tensor> &cur, std::vector<int> &widths, int64_t n) {
  BytePacking bp;
  bool others8 = true;
  for (size_t i = 0; i < cur.size(); ++i) {
    if (i > 0 && widths[i] == 1) {
      bp.byte_idx.push_back((int)i);
      bp.byte_dtype.push_back(cur[i].scalar_type());
    } else {
      bp.keep_idx.push_back((int)i);
      others8 &= widths[i] == 8;
    }
  }
  bp.active = !bp.byte_idx.empty() && others8 && n > 0;
  if (!bp.active) return bp;
  const int k = (int)bp.byte_idx.size(), nw = bp.words();
  std::vector<const uint8_t *> src;
  for (int i : bp.byte_idx) src.push_back(reinterpret_cast<const uint8_t *>(cur[i].data_ptr()));
  std::vector<at::Tensor> packed;
  std::vector<int> pw;
  for (int i : bp.keep_idx) {
    packed.push_back(cur[i]);
    pw.push_back(widths[i]);
  }
  std::vector<uint64_t *> wp;
  for (int w = 0; w < nw; ++w) {
    packed.push_back(ex.empty_i64(n));
    pw.push_back(8);
    wp.push_back(reinterpret_cast<uint64_t *>(packed.back().data_ptr()));
  }
  hip::pack_byte_columns(src.data(), k, n, wp.data(), ex.stream);
  cur = std::move(packed);
  widths = std::move(pw);
  return bp;
}

std::vector<at::Tensor> UnpackByteColumns(const Exec &ex, const BytePacking &bp, std::vector<at::Tensor> cur,
                                          int64_t n) {
  if (!bp.active) return cur;
  const int k = (int)bp.byte_idx.size(), nw = bp.words();
  const size_t nk = bp.keep_idx.size();
  std::vector<at::Tensor> out(nk + k);
  for (size_t j = 0; j < nk; ++j) out[bp.keep_idx[j]] = cur[j];
  std::vector<const uint64_t *> wp;
  for (int w = 0; w < nw; ++w) wp.push_back(reinterpret_cast<const uint64_t *>(cur[nk + w].data_ptr()));
  std::vector<uint8_t *> dst;
  for (int j = 0; j < k; ++j) {
    at::Tensor b = ex.empty_u8(n);
    dst.push_back(b.data_ptr<uint8_t>());
    out[bp.byte_idx[j]] = b.view(bp.byte_dtype[j]);
  }
  hip::unpack_byte_columns(wp.data(), k, n, dst.data(), ex.stream);
  return out;
}



static thread_local bool tl_partition_lb_off = false;  // set while a look-back fallback repartitions
static std::atomic<int> g_max_digit_bits{10};  // A/B hook (SetPartitionDigitBits): digit bits per pass

void SetPartitionDigitBits(int bits) { g_max_digit_bits.store(bits >= 3 && bits <= 10 ? bits : 10); }

std::vector<at::Tensor> RadixPartition(const Exec &ex, std::vector<at::Tensor> cur, const std::vector<int> &widths,
                                       int bits, at::Tensor *offs, const RangeSpec *range,
                                       std::vector<int> *keep_packed, bool stable, const hip::NarrowKeys *nk,
                                       const PrehistFn *prehist) {
  CYLON_CHECK(ex.gpu, Code::Invalid, "RadixPartition is a device path");
  CYLON_CHECK(!cur.empty() && cur.size() == widths.size() && widths[0] == 8, Code::Invalid,
              "RadixPartition: column 0 must be the int64 key");
  const int64_t n = cur[0].numel();
  for (size_t c = 1; c < cur.size(); ++c)
    CYLON_CHECK(cur[c].defined() || (widths[c] == 8 && !range), Code::Invalid,
                "RadixPartition: only 8-byte hash-partition columns may be generated row ids");
  // look-back passes (stable hash partitions of 1-2 all-8-byte columns, as for the sort): the first
  // pass counts (chunk, next digit) and the later ones take their offsets by look-back, without a
  // tile histogram (1B-row group-by 24.2 / 25.3 -> 23.3 / 24.0 ms, profiles/r04/partition_lookback_ab.txt).
  // Test knob CYLON_PARTITION_LOOKBACK=0 returns to the exact tile histograms.
  if (nk && !nk->base_src) nk = nullptr;
  CYLON_CHECK(!(nk && range), Code::Invalid, "RadixPartition: narrowed keys are hash partitions");
  const bool lb_want = !range && !nk && stable && !tl_partition_lb_off && knobs::Flag("PARTITION_LOOKBACK", true) &&
                       !knobs::Flag("RP_DEBUG_UNSTABLE", false);
  const std::vector<at::Tensor> orig = lb_want ? cur : std::vector<at::Tensor>();  // for the (never seen) fallback
  // Nullable payloads made a 200M join 24.8 -> 47.8 ms with unpacked validity bytes
  // (16-B byte runs per pass instead of 128-B runs); packed: 30.2 ms.
  std::vector<int> pw = widths;
  const BytePacking bp = PackByteColumns(ex, cur, pw, n);
  const int max_db = g_max_digit_bits.load();  // digit bits per pass
  const int npass = (bits + max_db - 1) / max_db;
  int shift = 0;
  at::Tensor ws;
  std::vector<int> dbits;
  for (int ps = 0, sh = 0; ps < npass; ++ps) {
    dbits.push_back((bits - sh + (npass - ps) - 1) / (npass - ps));
    sh += dbits.back();
  }
  const bool lb_on = lb_want && hip::radix_sort_lb_eligible(n, (int)cur.size(), pw.data(), dbits.data(), npass,
                                                            ex.stream);
  at::Tensor lbws = lb_on ? ex.empty_i64(hip::radix_sort_lb_workspace(n)) : at::Tensor();
  if (lb_on) trace::add_counter("partition.radix.lookback", 1);
  // exact XCD-tile passes after the first: the previous pass writes every stored key's next digit
  // (2 B/row), so this pass's tile histogram reads 2 bytes per row instead of the 8-byte key
  const bool nd_on = !range && !nk && !lb_on && npass > 1;
  at::Tensor nd = nd_on ? at::empty({n}, ex.opts(at::kShort)) : at::Tensor();
  uint16_t *ndp = nd_on ? reinterpret_cast<uint16_t *>(nd.data_ptr()) : nullptr;
  for (int ps = 0; ps < npass; ++ps) {
    const int db = dbits[ps];
    const int64_t wsn = hip::radix_rows_pass_workspace(n, db);
    if (!ws.defined() || ws.numel() < wsn) ws = ex.empty_i64(wsn);
    // the caller's producer kernel (a row hash) already counted the first pass's tile digits
    const bool pre = ps == 0 && prehist && !range && !nk;
    if (pre) (*prehist)(ptr<int64_t>(ws) + hip::radix_rows_pass_th_offset(n, db), db);
    std::vector<at::Tensor> nxt;
    std::vector<const uint8_t *> in;
    std::vector<uint8_t *> out;
    std::vector<int> pwp = pw;  // narrowed keys: column 0 is 4 bytes wide after the first pass
    if (nk && ps > 0) pwp[0] = 4;
    for (size_t c = 0; c < cur.size(); ++c) {
      const at::Tensor &x = cur[c];
      // an undefined tensor is a row-id column: generated by the first pass (radix_rows_pass)
      nxt.push_back(nk && c == 0 ? at::empty({n}, ex.opts(at::kInt)) : (x.defined() ? at::empty_like(x) : ex.empty_i64(n)));
      in.push_back(x.defined() ? reinterpret_cast<const uint8_t *>(x.data_ptr()) : nullptr);
      out.push_back(reinterpret_cast<uint8_t *>(nxt.back().data_ptr()));
    }
    if (range)
      hip::radix_range_rows_pass(reinterpret_cast<const int64_t *>(cur[0].data_ptr()), n, range->flip, range->mn,
                                 range->rshift, shift, db, in.data(), out.data(), pw.data(), (int)cur.size(),
                                 ptr<int64_t>(ws), ex.stream);
    else {
      SortLbArgs lba{};
      if (lb_on) lba = hip::radix_sort_lb_args(ptr<int64_t>(lbws), n, ps, npass, ex.stream);
      hip::NarrowKeys nkp;
      if (nk) {
        nkp = *nk;
        nkp.kin4 = ps > 0;
      }
      hip::radix_rows_pass(reinterpret_cast<const int64_t *>(cur[0].data_ptr()), n, bits, shift, db, in.data(),
                           out.data(), pwp.data(), (int)cur.size(), ptr<int64_t>(ws), ex.stream,
                           stable || ps > 0,  // LSD: every pass after the first keeps the order it receives
                           lb_on ? &lba : nullptr, ps + 1 < npass ? dbits[ps + 1] : 0, nk ? &nkp : nullptr, pre,
                           nd_on && ps > 0 ? ndp : nullptr, nd_on && ps + 1 < npass ? ndp : nullptr);
    }
    cur = std::move(nxt);
    shift += db;
  }
  if (lb_on && hip::radix_sort_lb_failed(ptr<int64_t>(lbws), ex.stream)) {  // a look-back wait gave up
    trace::add_counter("partition.radix.lookback_timeout_fallback", 1);
    cur.clear();
    tl_partition_lb_off = true;  // the exact passes, once
    std::vector<at::Tensor> r = RadixPartition(ex, orig, widths, bits, offs, range, keep_packed, stable);
    tl_partition_lb_off = false;
    return r;
  }
  for (auto &x : cur)  // no pass ran (bits == 0): row ids are still to be made
    if (!x.defined()) x = at::arange(n, ex.opts(at::kLong));
  if (bp.active && keep_packed) {  // caller consumes the words: undefined byte slots + words appended
    std::vector<at::Tensor> out(bp.keep_idx.size() + bp.byte_idx.size());
    for (size_t j = 0; j < bp.keep_idx.size(); ++j) out[bp.keep_idx[j]] = cur[j];
    for (int w = 0; w < bp.words(); ++w) out.push_back(cur[bp.keep_idx.size() + w]);
    *keep_packed = bp.byte_idx;
    cur = std::move(out);
  } else {
    cur = UnpackByteColumns(ex, bp, std::move(cur), n);
  }
  *offs = ex.empty_i64((int64_t(1) << bits) + 1);
  if (keep_packed && !bp.active) keep_packed->clear();
  if (range)
    hip::radix_range_part_offsets(ptr<int64_t>(cur[0]), n, range->flip, range->mn, range->rshift, bits,
                                  ptr<int64_t>(*offs), ex.stream);
  else if (nk && npass > 0)
    hip::radix_part_offsets32(reinterpret_cast<const uint32_t *>(cur[0].data_ptr()), n, bits, ptr<int64_t>(*offs),
                              ex.stream);
  else
    hip::radix_part_offsets(ptr<int64_t>(cur[0]), n, bits, ptr<int64_t>(*offs), ex.stream);
  return cur;
}

std::vector<at::Tensor> RadixChunkPartition(const Exec &ex, std::vector<at::Tensor> cur, const std::vector<int> &widths,
                                            int cbits, at::Tensor *offs, const at::Tensor *key_into, bool stable) {
  CYLON_CHECK(ex.gpu && !cur.empty() && cur.size() == widths.size() && widths[0] == 8, Code::Invalid,
              "RadixChunkPartition arguments");
  const int64_t n = cur[0].numel();
  CYLON_CHECK(!key_into || key_into->numel() == n, Code::Invalid, "RadixChunkPartition: key output size");
  std::vector<int> pw = widths;
  const BytePacking bp = PackByteColumns(ex, cur, pw, n);
  CYLON_CHECK(cur.size() <= 16, Code::Invalid, "RadixChunkPartition: " << cur.size() << " columns in one pass");
  at::Tensor ws = ex.empty_i64(hip::radix_rows_pass_workspace(n, cbits));
  std::vector<at::Tensor> nxt;
  std::vector<const uint8_t *> in;
  std::vector<uint8_t *> out;
  for (size_t c = 0; c < cur.size(); ++c) {
    nxt.push_back(c == 0 && key_into ? *key_into : at::empty_like(cur[c]));
    in.push_back(reinterpret_cast<const uint8_t *>(cur[c].data_ptr()));
    out.push_back(reinterpret_cast<uint8_t *>(nxt.back().data_ptr()));
  }
  if (offs) *offs = ex.empty_i64((int64_t(1) << cbits) + 1);
  hip::radix_chunk_pass(reinterpret_cast<const int64_t *>(cur[0].data_ptr()), n, cbits, in.data(), out.data(),
                        pw.data(), (int)cur.size(), ptr<int64_t>(ws), offs ? ptr<int64_t>(*offs) : nullptr, ex.stream,
                        stable);
  cur.clear();
  return UnpackByteColumns(ex, bp, std::move(nxt), n);
}

std::vector<at::Tensor> RadixPartitionSlotted(const Exec &ex, std::vector<at::Tensor> cur,
                                              const std::vector<int> &widths, int bits, int64_t slot,
                                              at::Tensor *counts, at::Tensor *overflow,
                                              std::vector<int> *keep_packed, const hip::NarrowKeys *nk) {
  if (nk && !nk->base_src) nk = nullptr;
  CYLON_CHECK(ex.gpu && !cur.empty() && cur.size() == widths.size() && widths[0] == 8 && slot > 0, Code::Invalid,
              "RadixPartitionSlotted arguments");
  const int64_t n = cur[0].numel();
  // second (low) digit <= 9 bits, first (high) digit <= 10 bits: 11 .. 19 partition bits
  const int db2 = std::min(9, bits / 2), db1 = bits - db2;
  if (bits < 2 || db1 > 10) return {};
  // (the block size of the unstable pass does not depend on the column count)
  if (!hip::radix_slot_eligible(n, (int)cur.size(), db1, db2)) return {};
  std::vector<int> pw = widths;
  const BytePacking bp = PackByteColumns(ex, cur, pw, n);
  // pass 1: the HIGH digit -- histogram-free into (bucket, XCD) slots when 8 x 2^db1 segments fit
  // the second pass's LDS segment table, else with exact per-tile offsets (XT, bucket bases kept
  // in ws1)
  const bool slot1 = hip::radix_slot_first_pass_ok(db1);
  at::Tensor ws1 = slot1 ? ex.empty_i64(hip::radix_slot_workspace(db1, db2))
                         : ex.empty_i64(hip::radix_rows_pass_workspace(n, db1));
  const int64_t nb1 = int64_t(1) << db1;
  const double mean1 = (double)n / (double)(8 * nb1);
  const int64_t s1 = slot1 ? (((int64_t)(mean1 + 8.0 * std::sqrt(mean1) + 64.0) + 7) & ~int64_t(7)) : 0;
  const int64_t rows1 = slot1 ? 8 * nb1 * s1 + hip::radix_slot_tile_rows() : n;
  at::Tensor cnt1 = slot1 ? ex.empty_i64(8 * nb1) : at::Tensor();
  *overflow = at::zeros({1}, ex.opts(at::kInt));
  unsigned int *ovf = reinterpret_cast<unsigned int *>(overflow->data_ptr<int>());
  // The first pass's output (freed when the second pass is done) is ONE allocation carved into its
  // columns: the caching allocator then splits that cached block for the join's output columns.
  // Column-sized blocks were each ~1 % smaller than an output column (slot padding 1.6 % vs the
  // output estimate's 2 % slack), so the 1B x 1B join's output reserved 25 GB of fresh memory next to
  // 28 GB of unusable cached blocks (peak reserved 207 GB for 181 GB allocated).
  std::vector<at::Tensor> mid;
  std::vector<const uint8_t *> in;
  std::vector<uint8_t *> out;
  {
    std::vector<at::ScalarType> dt;
    std::vector<int64_t> at_byte;
    int64_t total = 0;
    for (const at::Tensor &x : cur) {
      dt.push_back(nk && dt.empty() ? at::kInt : (x.defined() ? x.scalar_type() : at::kLong));
      at_byte.push_back(total);
      total += (rows1 * (int64_t)c10::elementSize(dt.back()) + 255) & ~int64_t(255);
    }
    at::Tensor block = ex.empty_bytes(total);
    for (size_t c = 0; c < cur.size(); ++c) {
      const int64_t es = (int64_t)c10::elementSize(dt[c]);
      mid.push_back(block.slice(0, at_byte[c], at_byte[c] + rows1 * es).view(dt[c]));
      in.push_back(cur[c].defined() ? reinterpret_cast<const uint8_t *>(cur[c].data_ptr()) : nullptr);
      out.push_back(reinterpret_cast<uint8_t *>(mid.back().data_ptr()));
    }
  }
  if (slot1) {
    for (size_t c = 0; c < cur.size(); ++c)  // (the slot pass reads every column: row ids made here)
      if (!in[c]) {
        cur[c] = at::arange(n, ex.opts(at::kLong));
        in[c] = reinterpret_cast<const uint8_t *>(cur[c].data_ptr());
      }
    hip::radix_slot_first_pass(reinterpret_cast<const int64_t *>(cur[0].data_ptr()), n, bits, db1, db2, in.data(),
                               out.data(), pw.data(), (int)cur.size(), s1, ptr<int64_t>(ws1), ptr<int64_t>(cnt1), ovf,
                               ex.stream, nk);
  } else {
    hip::radix_rows_pass(reinterpret_cast<const int64_t *>(cur[0].data_ptr()), n, bits, db2, db1, in.data(),
                         out.data(), pw.data(), (int)cur.size(), ptr<int64_t>(ws1), ex.stream, false, nullptr, 0, nk);
  }
  cur.clear();
  // pass 2: the low digit inside each first-pass bucket, into the partition slots
  const int64_t nparts = int64_t(1) << bits;
  const int64_t rows = nparts * slot + hip::radix_slot_tile_rows();
  std::vector<at::Tensor> fin;
  in.clear();
  out.clear();
  for (const at::Tensor &x : mid) {
    fin.push_back(at::empty({rows}, x.options()));
    in.push_back(reinterpret_cast<const uint8_t *>(x.data_ptr()));
    out.push_back(reinterpret_cast<uint8_t *>(fin.back().data_ptr()));
  }
  at::Tensor ws2 = ex.empty_i64(hip::radix_slot_workspace(db1, db2));
  *counts = ex.empty_i64(nparts);
  hip::NarrowKeys nk2;
  std::vector<int> pw2 = pw;
  if (nk) {
    nk2 = *nk;
    nk2.kin4 = 1;
    pw2[0] = 4;
  }
  hip::radix_slot_rows_pass(reinterpret_cast<const int64_t *>(mid[0].data_ptr()), n, bits, db1, db2, in.data(),
                            out.data(), pw2.data(), (int)mid.size(), ptr<int64_t>(ws1),
                            slot1 ? ptr<int64_t>(cnt1) : nullptr, s1, slot, ptr<int64_t>(ws2), ptr<int64_t>(*counts),
                            ovf, ex.stream, nk ? &nk2 : nullptr);
  mid.clear();
  if (bp.active && keep_packed) {
    std::vector<at::Tensor> res(bp.keep_idx.size() + bp.byte_idx.size());
    for (size_t j = 0; j < bp.keep_idx.size(); ++j) res[bp.keep_idx[j]] = fin[j];
    for (int w = 0; w < bp.words(); ++w) res.push_back(fin[bp.keep_idx.size() + w]);
    *keep_packed = bp.byte_idx;
    return res;
  }
  if (keep_packed) keep_packed->clear();
  return UnpackByteColumns(ex, bp, std::move(fin), rows);
}

}  // namespace ops
}  // namespace cylon
