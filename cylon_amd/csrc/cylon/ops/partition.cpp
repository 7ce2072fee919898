// Partition module (L4): hash partition ids, stable partition-major reorder,
// split.  Reference: cpp/src/cylon/partition/partition.cpp:27-217,
// cpp/src/cylon/table.cpp:384-405 (HashPartition).
#include "util.hpp"

namespace cylon {
namespace ops {

std::pair<at::Tensor, std::vector<int64_t>> MapToHashPartitions(const TablePtr &t, const std::vector<int> &cols,
                                                                uint32_t nparts) {
  CYLON_CHECK(nparts >= 1, Code::Invalid, "number of partitions must be >= 1");
  CYLON_CHECK(!cols.empty(), Code::Invalid, "hash partition needs at least one column");
  Exec ex(t->device());
  const int64_t n = t->Rows();
  std::vector<ColView> v = views(t, cols);
  at::Tensor h = ex.empty_u32(n);
  at::Tensor pid = ex.empty_u32(n);
  at::Tensor counts = ex.empty_i64(nparts);
  KCALL(ex, row_partition_hash, v.data(), (int)v.size(), n, ptr<uint32_t>(h));
  KCALL(ex, hash_to_partition, ptr<uint32_t>(h), n, nparts, ptr<uint32_t>(pid), ptr<int64_t>(counts));
  return {pid, to_host_vec(counts)};
}

std::pair<TablePtr, std::vector<int64_t>> PartitionReorder(const TablePtr &t, const at::Tensor &pid,
                                                           uint32_t nparts) {
  Exec ex(t->device());
  const int64_t n = t->Rows();
  CYLON_CHECK(pid.numel() == n, Code::Invalid, "partition id vector length != rows");
  at::Tensor ws = ex.empty_i64(KSIZE(ex, partition_positions_workspace, n, nparts));
  at::Tensor pos = ex.empty_i64(n);
  at::Tensor counts = ex.empty_i64(nparts);
  KCALL(ex, partition_positions, ptr<uint32_t>(pid), n, nparts, ptr<int64_t>(ws), ptr<int64_t>(pos),
        ptr<int64_t>(counts));

  std::vector<Column> out(t->Columns());
  std::vector<ColView> ins;
  std::vector<MutColView> outs;
  for (int i = 0; i < t->Columns(); ++i) {
    const Column &c = t->column(i);
    if (c.is_var()) {
      ColView in = c.view();
      at::Tensor lens = ex.empty_i64(n);
      KCALL(ex, scatter_var_lengths, in, ptr<int64_t>(pos), n, ptr<int64_t>(lens));
      at::Tensor offs = exclusive_scan(ex, lens);
      at::Tensor bytes = ex.empty_bytes(c.data.numel());
      at::Tensor valid;
      if (c.nullable()) valid = ex.empty_u8(n);
      KCALL(ex, scatter_var_bytes, in, ptr<int64_t>(pos), n, ptr<int64_t>(offs), ptr<uint8_t>(bytes),
            valid.defined() ? ptr<uint8_t>(valid) : nullptr);
      out[i] = Column(c.name, c.type, n, bytes, offs, valid);
      continue;
    }
    Column o = make_fixed_column(c.name, c.type, n, ex.device, c.nullable());
    MutColView mv;
    mv.data = n ? reinterpret_cast<uint8_t *>(o.data.data_ptr()) : nullptr;
    mv.valid = o.validity.defined() ? ptr<uint8_t>(o.validity) : nullptr;
    mv.width = c.type.width();
    mv.kind = static_cast<int>(c.type.kind());
    ins.push_back(c.view());
    outs.push_back(mv);
    out[i] = std::move(o);
  }
  if (!ins.empty() && n > 0) KCALL(ex, scatter_columns, ins.data(), outs.data(), (int)ins.size(), ptr<int64_t>(pos), n);
  return {Table::Make(t->GetContext(), std::move(out)), to_host_vec(counts)};
}

std::vector<TablePtr> Split(const TablePtr &t, const at::Tensor &pid, uint32_t nparts) {
  auto r = PartitionReorder(t, pid, nparts);
  std::vector<TablePtr> parts;
  int64_t off = 0;
  for (uint32_t p = 0; p < nparts; ++p) {
    parts.push_back(Slice(r.first, off, r.second[p]));
    off += r.second[p];
  }
  return parts;
}

std::vector<TablePtr> HashPartition(const TablePtr &t, const std::vector<int> &cols, uint32_t nparts) {
  auto m = MapToHashPartitions(t, cols, nparts);
  return Split(t, m.first, nparts);
}

}  // namespace ops
}  // namespace cylon
