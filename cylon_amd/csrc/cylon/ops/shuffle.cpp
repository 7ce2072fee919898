// Shuffle (L4 + L1): hash partition -> partition-major reorder -> one
// all_to_all_v per column buffer over the communicator (RCCL/xGMI on MI355X).
//
// Reference: cpp/src/cylon/table.cpp:67-179 (all_to_all_arrow_tables,
// shuffle_table_by_hashing), arrow/arrow_all_to_all.cpp (per-buffer header +
// payload protocol).  Partition -> rank mapping is identical: partition i goes
// to rank i when P == world, else to rank i*world/P (table.cpp:89-106).
#include "util.hpp"
#include "../trace.hpp"

namespace cylon {
namespace ops {

static at::Tensor hash_pids(const TablePtr &t, const std::vector<int> &cols, uint32_t nparts) {
  Exec ex(t->device());
  const int64_t n = t->Rows();
  std::vector<ColView> v = views(t, cols);
  at::Tensor h = ex.empty_u32(n);
  at::Tensor pid = ex.empty_u32(n);
  at::Tensor counts = ex.empty_i64(nparts);
  KCALL(ex, row_partition_hash, v.data(), (int)v.size(), n, ptr<uint32_t>(h));
  KCALL(ex, hash_to_partition, ptr<uint32_t>(h), n, nparts, ptr<uint32_t>(pid), ptr<int64_t>(counts));
  return pid;
}

TablePtr AllToAllTable(const TablePtr &part, const std::vector<int64_t> &counts) {
  auto ctx = part->GetContext();
  auto comm = ctx->GetCommunicator();
  const int world = ctx->GetWorldSize();
  if (world == 1 || !ctx->IsDistributed()) return part;
  const size_t P = counts.size();

  // rows per destination rank (partition-major order keeps each rank contiguous)
  std::vector<int64_t> send_rows(world, 0);
  for (size_t i = 0; i < P; ++i) {
    const size_t target = (P == (size_t)world) ? i : i * world / P;
    send_rows[target] += counts[i];
  }
  std::vector<int64_t> recv_rows = comm->ExchangeCounts(send_rows);
  int64_t total = 0;
  for (auto r : recv_rows) total += r;

  // schema-level nullability must agree across ranks
  const int ncols = part->Columns();
  at::Tensor flags = at::zeros({std::max(ncols, 1)}, at::TensorOptions().dtype(at::kInt));
  for (int c = 0; c < ncols; ++c) flags[c] = part->column(c).nullable() ? 1 : 0;
  at::Tensor gflags = flags.to(part->device());
  comm->AllReduce(gflags, net::ReduceOp::MAX);
  std::vector<int64_t> nullable = to_host_vec(gflags.to(at::kLong));

  Exec ex(part->device());
  std::vector<Column> out;
  for (int c = 0; c < ncols; ++c) {
    const Column &col = part->column(c);
    at::Tensor valid;
    if (nullable[c]) {
      at::Tensor v = col.nullable() ? col.validity : at::ones({col.length}, ex.opts(at::kByte));
      valid = comm->AllToAllV(v, send_rows, recv_rows);
    }
    if (!col.is_var()) {
      const int64_t per = col.type.kind() == ValueKind::FIXED_BYTES ? col.type.width() : 1;
      std::vector<int64_t> sc(send_rows), rc(recv_rows);
      for (auto &x : sc) x *= per;
      for (auto &x : rc) x *= per;
      at::Tensor d = comm->AllToAllV(col.data, sc, rc);
      out.emplace_back(col.name, col.type, total, d, at::Tensor(), valid);
      continue;
    }
    // var width: lengths, then bytes
    at::Tensor lens = col.offsets.slice(0, 1, col.length + 1) - col.offsets.slice(0, 0, col.length);
    at::Tensor rlens = comm->AllToAllV(lens.contiguous(), send_rows, recv_rows);
    std::vector<int64_t> send_bytes(world, 0);
    {
      at::Tensor ho = col.offsets.to(at::kCPU);
      const int64_t *o = ho.data_ptr<int64_t>();
      int64_t row = 0;
      for (int r = 0; r < world; ++r) {
        send_bytes[r] = o[row + send_rows[r]] - o[row];
        row += send_rows[r];
      }
    }
    std::vector<int64_t> recv_bytes = comm->ExchangeCounts(send_bytes);
    at::Tensor bytes = comm->AllToAllV(col.data, send_bytes, recv_bytes);
    at::Tensor offs = exclusive_scan(ex, rlens.contiguous());
    out.emplace_back(col.name, col.type, total, bytes, offs, valid);
  }
  return Table::Make(ctx, std::move(out));
}

TablePtr Shuffle(const TablePtr &t, const std::vector<int> &hash_cols) {
  auto ctx = t->GetContext();
  const int world = ctx->GetWorldSize();
  if (world == 1) return t;
  std::pair<TablePtr, std::vector<int64_t>> r;
  {
    CYLON_PHASE("shuffle.partition", t->device());
    at::Tensor pid = hash_pids(t, hash_cols, (uint32_t)world);
    r = PartitionReorder(t, pid, (uint32_t)world);
  }
  CYLON_PHASE("shuffle.exchange", t->device());
  trace::add_counter("shuffle.rows_in", t->Rows());
  trace::add_counter("shuffle.bytes_in", t->nbytes());
  TablePtr out = AllToAllTable(r.first, r.second);
  trace::add_counter("shuffle.rows_out", out->Rows());
  return out;
}

}  // namespace ops
}  // namespace cylon
