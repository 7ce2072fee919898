// Shared radix partitioning driver for the LDS radix join and group-by
// (kernels: radix_join.hip k_rp_hist / k_rows_pass / k_part_offsets).
#include <algorithm>
#include <cstdlib>

#include "util.hpp"

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
  static const bool enabled = [] {  // A/B knob (tools/nullable_probe.py)
    const char *e = std::getenv("CYLON_PACK_VALIDITY");
    return !(e && e[0] == '0');
  }();
  bp.active = enabled && !bp.byte_idx.empty() && others8 && n > 0;
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

static int max_digit_bits() {  // digit bits per pass (<= 10); tuning knob
  static const int v = [] {
    const char *e = std::getenv("CYLON_RADIX_DIGIT_BITS");
    return e ? std::max(1, std::min(10, std::atoi(e))) : 10;
  }();
  return v;
}

int RadixFirstDigitBits(int bits) {
  const int npass = (bits + max_digit_bits() - 1) / max_digit_bits();
  return npass ? (bits + npass - 1) / npass : 0;
}

at::Tensor RadixNarrowPrehist(const Exec &ex, const at::Tensor &keys, int bits, const at::Tensor &mm) {
  const int db = RadixFirstDigitBits(bits);
  const int64_t n = keys.numel();
  at::Tensor ws = ex.empty_i64(hip::radix_rows_pass_workspace(n, db));
  hip::radix_narrow_prehist(ptr<int64_t>(keys), n, bits, db, ptr<int64_t>(ws), ptr<int64_t>(mm), ex.stream);
  return ws;
}

std::vector<at::Tensor> RadixPartition(const Exec &ex, std::vector<at::Tensor> cur, const std::vector<int> &widths,
                                       int bits, at::Tensor *offs, const RangeSpec *range,
                                       std::vector<int> *keep_packed, bool stable, at::Tensor *narrow_ws) {
  const bool narrow = narrow_ws != nullptr;
  CYLON_CHECK(!narrow || (!range && bits > 0), Code::Invalid, "RadixPartition: narrow keys need hash partitions");
  CYLON_CHECK(ex.gpu, Code::Invalid, "RadixPartition is a device path");
  CYLON_CHECK(!cur.empty() && cur.size() == widths.size() && widths[0] == 8, Code::Invalid,
              "RadixPartition: column 0 must be the int64 key");
  const int64_t n = cur[0].numel();
  for (size_t c = 1; c < cur.size(); ++c)
    CYLON_CHECK(cur[c].defined() || (widths[c] == 8 && !range), Code::Invalid,
                "RadixPartition: only 8-byte hash-partition columns may be generated row ids");
  // Nullable payloads made a 200M join 24.8 -> 47.8 ms with unpacked validity bytes
  // (16-B byte runs per pass instead of 128-B runs); packed: 30.2 ms.
  std::vector<int> pw = widths;
  const BytePacking bp = PackByteColumns(ex, cur, pw, n);
  const int max_db = max_digit_bits();
  const int npass = (bits + max_db - 1) / max_db;
  std::vector<int> shifts, dbits;
  int lb_bits = 0;
  for (int ps = 0, sh = 0; ps < npass; ++ps) {
    const int db = (bits - sh + (npass - ps) - 1) / (npass - ps);
    shifts.push_back(sh);
    dbits.push_back(db);
    lb_bits = std::max(lb_bits, db);
    sh += db;
  }
  // chained-scan passes (kernels/radix_join.hip k_lb_hist): one read of the keys counts the
  // digits of every pass instead of a histogram kernel before each pass
  const bool lbm = npass >= 2 && n > 0 && hip::radix_lookback_enabled() && !narrow;
  at::Tensor lbws;
  if (lbm) {
    lbws = ex.empty_i64(hip::radix_lb_workspace(n, lb_bits));
    const int64_t *k0 = reinterpret_cast<const int64_t *>(cur[0].data_ptr());
    if (range)
      hip::radix_lb_prepare_range(k0, n, range->flip, range->mn, range->rshift, shifts.data(), dbits.data(), npass,
                                  lb_bits, ptr<int64_t>(lbws), ex.stream);
    else
      hip::radix_lb_prepare_part(k0, n, bits, shifts.data(), dbits.data(), npass, lb_bits, ptr<int64_t>(lbws),
                                 ex.stream);
  }
  int64_t *lbp = lbm ? ptr<int64_t>(lbws) : nullptr;
  int shift = 0;
  at::Tensor ws;
  for (int ps = 0; ps < npass; ++ps) {
    const int db = dbits[ps];
    const int64_t wsn = lbm ? 1 : hip::radix_rows_pass_workspace(n, db);
    if (!ws.defined() || ws.numel() < wsn) ws = ex.empty_i64(wsn);
    std::vector<at::Tensor> nxt;
    std::vector<const uint8_t *> in;
    std::vector<uint8_t *> out;
    for (size_t c = 0; c < cur.size(); ++c) {
      const at::Tensor &x = cur[c];
      // an undefined tensor is a row-id column: generated by the first pass (radix_rows_pass)
      nxt.push_back(narrow && c == 0 ? at::empty({n}, ex.opts(at::kInt))
                                     : (x.defined() ? at::empty_like(x) : ex.empty_i64(n)));
      in.push_back(x.defined() ? reinterpret_cast<const uint8_t *>(x.data_ptr()) : nullptr);
      out.push_back(reinterpret_cast<uint8_t *>(nxt.back().data_ptr()));
    }
    if (narrow) {
      CYLON_CHECK(ps > 0 || db == RadixFirstDigitBits(bits), Code::Invalid, "narrow prehist digit");
      std::vector<int> nw = pw;
      nw[0] = 4;
      hip::radix_narrow_rows_pass(cur[0].data_ptr(), ps == 0 ? 8 : 4, n, bits, shift, db, in.data(), out.data(),
                                  nw.data(), (int)cur.size(), ps == 0 ? ptr<int64_t>(*narrow_ws) : ptr<int64_t>(ws),
                                  ex.stream, stable || ps > 0, ps == 0);
    } else if (range)
      hip::radix_range_rows_pass(reinterpret_cast<const int64_t *>(cur[0].data_ptr()), n, range->flip, range->mn,
                                 range->rshift, shift, db, in.data(), out.data(), pw.data(), (int)cur.size(),
                                 ptr<int64_t>(ws), ex.stream, lbp, ps, lb_bits);
    else
      hip::radix_rows_pass(reinterpret_cast<const int64_t *>(cur[0].data_ptr()), n, bits, shift, db, in.data(),
                           out.data(), pw.data(), (int)cur.size(), ptr<int64_t>(ws), ex.stream,
                           stable || ps > 0,  // LSD: every pass after the first keeps the order it receives
                           lbp, ps, lb_bits);
    cur = std::move(nxt);
    shift += db;
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
  if (narrow)
    hip::radix_narrow_part_offsets(reinterpret_cast<const uint32_t *>(cur[0].data_ptr()), n, bits,
                                   ptr<int64_t>(*offs), ex.stream);
  else if (range)
    hip::radix_range_part_offsets(ptr<int64_t>(cur[0]), n, range->flip, range->mn, range->rshift, bits,
                                  ptr<int64_t>(*offs), ex.stream);
  else
    hip::radix_part_offsets(ptr<int64_t>(cur[0]), n, bits, ptr<int64_t>(*offs), ex.stream);
  return cur;
}

}  // namespace ops
}  // namespace cylon
