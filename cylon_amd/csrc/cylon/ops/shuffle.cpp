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

// A table whose column buffers are in flight (posted all-to-alls).
struct PendingTable {
  std::shared_ptr<CylonContext> ctx;
  int64_t total = 0;
  struct Col {
    const Column *src;
    at::Tensor data, valid, rlens;  // receive buffers (rlens: var-width lengths)
  };
  std::vector<Col> cols;
  std::vector<std::shared_ptr<net::P2PRequest>> reqs;
  TablePtr passthrough;  // world 1
};

static PendingTable AllToAllBegin(const TablePtr &part, const std::vector<int64_t> &counts) {
  PendingTable pt;
  auto ctx = part->GetContext();
  pt.ctx = ctx;
  auto comm = ctx->GetCommunicator();
  const int world = ctx->GetWorldSize();
  if (world == 1 || !ctx->IsDistributed()) {
    pt.passthrough = part;
    return pt;
  }
  const size_t P = counts.size();

  // rows per destination rank (partition-major order keeps each rank contiguous)
  std::vector<int64_t> send_rows(world, 0);
  for (size_t i = 0; i < P; ++i) {
    const size_t target = (P == (size_t)world) ? i : i * world / P;
    send_rows[target] += counts[i];
  }
  std::vector<int64_t> recv_rows = comm->ExchangeCounts(send_rows);
  for (auto r : recv_rows) pt.total += r;

  // schema-level nullability must agree across ranks
  const int ncols = part->Columns();
  at::Tensor flags = at::zeros({std::max(ncols, 1)}, at::TensorOptions().dtype(at::kInt));
  for (int c = 0; c < ncols; ++c) flags[c] = part->column(c).nullable() ? 1 : 0;
  at::Tensor gflags = flags.to(part->device());
  comm->AllReduce(gflags, net::ReduceOp::MAX);
  std::vector<int64_t> nullable = to_host_vec(gflags.to(at::kLong));

  Exec ex(part->device());
  auto post = [&](const at::Tensor &t, const std::vector<int64_t> &sc, const std::vector<int64_t> &rc) {
    auto r = comm->AllToAllVAsync(t, sc, rc);
    pt.reqs.push_back(r.second);
    return r.first;
  };
  for (int c = 0; c < ncols; ++c) {
    const Column &col = part->column(c);
    PendingTable::Col pc;
    pc.src = &col;
    if (nullable[c]) {
      at::Tensor v = col.nullable() ? col.validity : at::ones({col.length}, ex.opts(at::kByte));
      pc.valid = post(v, send_rows, recv_rows);
    }
    if (!col.is_var()) {
      const int64_t per = col.type.kind() == ValueKind::FIXED_BYTES ? col.type.width() : 1;
      std::vector<int64_t> sc(send_rows), rc(recv_rows);
      for (auto &x : sc) x *= per;
      for (auto &x : rc) x *= per;
      pc.data = post(col.data, sc, rc);
    } else {  // var width: lengths, then bytes
      at::Tensor lens = col.offsets.slice(0, 1, col.length + 1) - col.offsets.slice(0, 0, col.length);
      pc.rlens = post(lens.contiguous(), send_rows, recv_rows);
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
      pc.data = post(col.data, send_bytes, recv_bytes);
    }
    pt.cols.push_back(pc);
  }
  return pt;
}

static TablePtr AllToAllFinish(PendingTable &pt) {
  if (pt.passthrough) return pt.passthrough;
  for (auto &r : pt.reqs) r->Wait();
  std::vector<Column> out;
  for (auto &pc : pt.cols) {
    const Column &col = *pc.src;
    if (!col.is_var()) {
      out.emplace_back(col.name, col.type, pt.total, pc.data, at::Tensor(), pc.valid);
    } else {
      Exec ex(pc.rlens.device());
      at::Tensor offs = exclusive_scan(ex, pc.rlens.contiguous());
      out.emplace_back(col.name, col.type, pt.total, pc.data, offs, pc.valid);
    }
  }
  return Table::Make(pt.ctx, std::move(out));
}

TablePtr AllToAllTable(const TablePtr &part, const std::vector<int64_t> &counts) {
  PendingTable pt = AllToAllBegin(part, counts);
  return AllToAllFinish(pt);
}

static std::pair<TablePtr, std::vector<int64_t>> shuffle_partition(const TablePtr &t,
                                                                   const std::vector<int> &hash_cols, int world) {
  CYLON_PHASE("shuffle.partition", t->device());
  at::Tensor pid = hash_pids(t, hash_cols, (uint32_t)world);
  return PartitionReorder(t, pid, (uint32_t)world);
}

TablePtr Shuffle(const TablePtr &t, const std::vector<int> &hash_cols) {
  auto ctx = t->GetContext();
  const int world = ctx->GetWorldSize();
  if (world == 1) return t;
  auto r = shuffle_partition(t, hash_cols, world);
  CYLON_PHASE("shuffle.exchange", t->device());
  trace::add_counter("shuffle.rows_in", t->Rows());
  trace::add_counter("shuffle.bytes_in", t->nbytes());
  TablePtr out = AllToAllTable(r.first, r.second);
  trace::add_counter("shuffle.rows_out", out->Rows());
  return out;
}

// Both relations of a distributed binary operator: the second table's partitioning
// kernels are enqueued while the first table's all-to-alls are in flight on the
// communicator's stream, and the two transfers are waited for only at the end.
std::pair<TablePtr, TablePtr> ShufflePair(const TablePtr &a, const std::vector<int> &acols, const TablePtr &b,
                                          const std::vector<int> &bcols) {
  auto ctx = a->GetContext();
  const int world = ctx->GetWorldSize();
  if (world == 1) return {a, b};
  auto ra = shuffle_partition(a, acols, world);
  PendingTable pa;
  {
    CYLON_PHASE("shuffle.exchange", a->device());
    pa = AllToAllBegin(ra.first, ra.second);
  }
  auto rb = shuffle_partition(b, bcols, world);
  PendingTable pb;
  {
    CYLON_PHASE("shuffle.exchange", b->device());
    pb = AllToAllBegin(rb.first, rb.second);
  }
  trace::add_counter("shuffle.rows_in", a->Rows() + b->Rows());
  trace::add_counter("shuffle.bytes_in", a->nbytes() + b->nbytes());
  TablePtr oa = AllToAllFinish(pa), ob = AllToAllFinish(pb);
  trace::add_counter("shuffle.rows_out", oa->Rows() + ob->Rows());
  return {oa, ob};
}

}  // namespace ops
}  // namespace cylon
