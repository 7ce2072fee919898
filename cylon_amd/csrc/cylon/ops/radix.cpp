// Shared radix partitioning driver for the LDS radix join and group-by
// (kernels: radix_join.hip k_rp_hist / k_rows_pass / k_part_offsets).
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

std::vector<at::Tensor> RadixPartition(const Exec &ex, std::vector<at::Tensor> cur, const std::vector<int> &widths,
                                       int bits, at::Tensor *offs, const RangeSpec *range,
                                       std::vector<int> *keep_packed, bool stable) {
  CYLON_CHECK(ex.gpu, Code::Invalid, "RadixPartition is a device path");
  CYLON_CHECK(!cur.empty() && cur.size() == widths.size() && widths[0] == 8, Code::Invalid,
              "RadixPartition: column 0 must be the int64 key");
  const int64_t n = cur[0].numel();
  // Nullable payloads made a 200M join 24.8 -> 47.8 ms with unpacked validity bytes
  // (16-B byte runs per pass instead of 128-B runs); packed: 30.2 ms.
  std::vector<int> pw = widths;
  const BytePacking bp = PackByteColumns(ex, cur, pw, n);
  static const int max_db = [] {  // digit bits per pass (<= 10); tuning knob
    const char *e = std::getenv("CYLON_RADIX_DIGIT_BITS");
    return e ? std::max(1, std::min(10, std::atoi(e))) : 10;
  }();
  const int npass = (bits + max_db - 1) / max_db;
  int shift = 0;
  at::Tensor ws;
  for (int ps = 0; ps < npass; ++ps) {
    const int db = (bits - shift + (npass - ps) - 1) / (npass - ps);
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
    if (range)
      hip::radix_range_rows_pass(reinterpret_cast<const int64_t *>(cur[0].data_ptr()), n, range->flip, range->mn,
                                 range->rshift, shift, db, in.data(), out.data(), pw.data(), (int)cur.size(),
                                 ptr<int64_t>(ws), ex.stream);
    else
      hip::radix_rows_pass(reinterpret_cast<const int64_t *>(cur[0].data_ptr()), n, bits, shift, db, in.data(),
                           out.data(), pw.data(), (int)cur.size(), ptr<int64_t>(ws), ex.stream,
                           stable || ps > 0);  // LSD: every pass after the first keeps the order it receives
    cur = std::move(nxt);
    shift += db;
  }
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
  else
    hip::radix_part_offsets(ptr<int64_t>(cur[0]), n, bits, ptr<int64_t>(*offs), ex.stream);
  return cur;
}

}  // namespace ops
}  // namespace cylon
