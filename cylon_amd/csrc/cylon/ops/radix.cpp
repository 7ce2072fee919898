// Shared radix partitioning driver for the LDS radix join and group-by
// (kernels: radix_join.hip k_rp_hist / k_rows_pass / k_part_offsets).
#include <cstdlib>

#include "util.hpp"

namespace cylon {
namespace ops {

std::vector<at::Tensor> RadixPartition(const Exec &ex, std::vector<at::Tensor> cur, const std::vector<int> &widths,
                                       int bits, at::Tensor *offs, const RangeSpec *range) {
  CYLON_CHECK(ex.gpu, Code::Invalid, "RadixPartition is a device path");
  CYLON_CHECK(!cur.empty() && cur.size() == widths.size() && widths[0] == 8, Code::Invalid,
              "RadixPartition: column 0 must be the int64 key");
  const int64_t n = cur[0].numel();
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
                                 range->rshift, shift, db, in.data(), out.data(), widths.data(), (int)cur.size(),
                                 ptr<int64_t>(ws), ex.stream);
    else
      hip::radix_rows_pass(reinterpret_cast<const int64_t *>(cur[0].data_ptr()), n, bits, shift, db, in.data(),
                           out.data(), widths.data(), (int)cur.size(), ptr<int64_t>(ws), ex.stream);
    cur = std::move(nxt);
    shift += db;
  }
  *offs = ex.empty_i64((int64_t(1) << bits) + 1);
  if (range)
    hip::radix_range_part_offsets(ptr<int64_t>(cur[0]), n, range->flip, range->mn, range->rshift, bits,
                                  ptr<int64_t>(*offs), ex.stream);
  else
    hip::radix_part_offsets(ptr<int64_t>(cur[0]), n, bits, ptr<int64_t>(*offs), ex.stream);
  return cur;
}

}  // namespace ops
}  // namespace cylon
