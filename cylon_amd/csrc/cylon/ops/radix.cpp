// Shared radix partitioning driver for the LDS radix join and group-by
// (kernels: radix_join.hip k_rp_hist / k_rows_pass / k_part_offsets).
#include <cstdlib>

#include "util.hpp"

namespace cylon {
namespace ops {

std::vector<at::Tensor> RadixPartition(const Exec &ex, std::vector<at::Tensor> cur, const std::vector<int> &widths,
                                       int bits, at::Tensor *offs, const RangeSpec *range,
                                       std::vector<int> *keep_packed) {
  CYLON_CHECK(ex.gpu, Code::Invalid, "RadixPartition is a device path");
  CYLON_CHECK(!cur.empty() && cur.size() == widths.size() && widths[0] == 8, Code::Invalid,
              "RadixPartition: column 0 must be the int64 key");
  const int64_t n = cur[0].numel();
  // Validity (1-byte) columns next to 8-byte columns travel packed, 8 per 8-byte word:
  // every pass then takes the all-8-byte path and writes 128-B runs instead of 16-B
  // byte runs (nullable payloads made a 200M join 24.8 -> 47.8 ms unpacked).
  std::vector<int> byte_idx, keep_idx;
  bool others8 = true;
  for (size_t i = 0; i < cur.size(); ++i) {
    if (i > 0 && widths[i] == 1) byte_idx.push_back((int)i);
    else {
      keep_idx.push_back((int)i);
      others8 &= widths[i] == 8;
    }
  }
  const bool pack = !byte_idx.empty() && others8 && n > 0;
  std::vector<int> pw = widths;
  if (pack) {
    const int k = (int)byte_idx.size(), nw = (k + 7) / 8;
    std::vector<const uint8_t *> bp;
    for (int i : byte_idx) bp.push_back(reinterpret_cast<const uint8_t *>(cur[i].data_ptr()));
    std::vector<at::Tensor> words;
    std::vector<uint64_t *> wp;
    for (int w = 0; w < nw; ++w) {
      words.push_back(ex.empty_i64(n));
      wp.push_back(reinterpret_cast<uint64_t *>(words.back().data_ptr()));
    }
    hip::pack_byte_columns(bp.data(), k, n, wp.data(), ex.stream);
    std::vector<at::Tensor> packed;
    pw.clear();
    for (int i : keep_idx) {
      packed.push_back(cur[i]);
      pw.push_back(widths[i]);
    }
    for (auto &w : words) {
      packed.push_back(w);
      pw.push_back(8);
    }
    cur = std::move(packed);
  }
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
                           out.data(), pw.data(), (int)cur.size(), ptr<int64_t>(ws), ex.stream);
    cur = std::move(nxt);
    shift += db;
  }
  if (pack && keep_packed) {  // caller consumes the words: undefined byte slots + words appended
    const int nw = ((int)byte_idx.size() + 7) / 8;
    std::vector<at::Tensor> out(keep_idx.size() + byte_idx.size());
    for (size_t j = 0; j < keep_idx.size(); ++j) out[keep_idx[j]] = cur[j];
    for (int w = 0; w < nw; ++w) out.push_back(cur[keep_idx.size() + w]);
    *keep_packed = byte_idx;
    cur = std::move(out);
  } else if (pack) {  // unpack into 1-byte columns, original order
    const int k = (int)byte_idx.size(), nw = (k + 7) / 8;
    std::vector<at::Tensor> out(keep_idx.size() + byte_idx.size());
    for (size_t j = 0; j < keep_idx.size(); ++j) out[keep_idx[j]] = cur[j];
    std::vector<const uint64_t *> wp;
    for (int w = 0; w < nw; ++w) wp.push_back(reinterpret_cast<const uint64_t *>(cur[keep_idx.size() + w].data_ptr()));
    std::vector<uint8_t *> bp;
    for (int i : byte_idx) {
      out[i] = ex.empty_u8(n);
      bp.push_back(out[i].data_ptr<uint8_t>());
    }
    hip::unpack_byte_columns(wp.data(), k, n, bp.data(), ex.stream);
    cur = std::move(out);
  }
  *offs = ex.empty_i64((int64_t(1) << bits) + 1);
  if (keep_packed && !pack) keep_packed->clear();
  if (range)
    hip::radix_range_part_offsets(ptr<int64_t>(cur[0]), n, range->flip, range->mn, range->rshift, bits,
                                  ptr<int64_t>(*offs), ex.stream);
  else
    hip::radix_part_offsets(ptr<int64_t>(cur[0]), n, bits, ptr<int64_t>(*offs), ex.stream);
  return cur;
}

}  // namespace ops
}  // namespace cylon
