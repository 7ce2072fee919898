// Shuffle (L4 + L1): hash partition -> partition-major reorder -> one
// all_to_all_v per column buffer over the communicator (RCCL/xGMI on MI355X).
//
// Reference: cpp/src/cylon/table.cpp:67-179 (all_to_all_arrow_tables,
// shuffle_table_by_hashing), arrow/arrow_all_to_all.cpp (per-buffer header +
// payload protocol).  Partition -> rank mapping is identical: partition i goes
// to rank i when P == world, else to rank i*world/P (table.cpp:89-106).
#include "cylon/knobs.hpp"
#include <limits>

#include "util.hpp"
#include "../trace.hpp"

namespace cylon {
namespace ops {

// partition ids + per-partition row counts (device tensor)
static std::pair<at::Tensor, at::Tensor> hash_pids_counts(const TablePtr &t, const std::vector<int> &cols,
                                                          uint32_t nparts) {
  Exec ex(t->device());
  const int64_t n = t->Rows();
  std::vector<ColView> v = views(t, cols);
  at::Tensor h = ex.empty_u32(n);
  at::Tensor pid = ex.empty_u32(n);
  at::Tensor counts = ex.empty_i64(nparts);
  KCALL(ex, row_partition_hash, v.data(), (int)v.size(), n, ptr<uint32_t>(h));
  KCALL(ex, hash_to_partition, ptr<uint32_t>(h), n, nparts, ptr<uint32_t>(pid), ptr<int64_t>(counts));
  return {pid, counts};
}

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

// ---------------------------------------------------------------------------
// Fast shuffle partition (radix_join.hip ModDigit pass): when the partition key
// is one non-null 8-byte integer column of a device table whose columns are all
// 1/2/4/8 bytes wide, the reference partition id is (uint32)key % P and a single
// LDS-staged pass moves the whole table into partition-major order (one read and
// one write per buffer, long write runs for P <= 1024) instead of pid + hash
// arrays, a ballot ranking and a per-row scatter.
// ---------------------------------------------------------------------------
static bool mod_pass_eligible(const TablePtr &t, const std::vector<int> &cols, uint32_t P) {
  if (!t->device().is_cuda() || cols.size() != 1 || P > 1024 || t->Rows() == 0) return false;
  const Column &k = t->column(cols[0]);
  if (k.nullable() || k.is_var() || k.type.width() != 8 || k.data.element_size() != 8 ||
      (k.type.kind() != ValueKind::SIGNED_INT && k.type.kind() != ValueKind::UNSIGNED_INT))
    return false;
  int slots = 1;
  for (int c = 0; c < t->Columns(); ++c) {
    const Column &col = t->column(c);
    const int w = col.type.width();
    if (col.is_var() || col.type.kind() == ValueKind::FIXED_BYTES || !(w == 1 || w == 2 || w == 4 || w == 8) ||
        col.data.element_size() != w)
      return false;
    slots += (c == cols[0] ? 0 : 1) + (col.nullable() ? 1 : 0);
  }
  return slots <= kMaxFusedCols;
}

static std::vector<int64_t> mod_counts(const TablePtr &t, int key, uint32_t P) {
  Exec ex(t->device());
  at::Tensor counts = ex.empty_i64(P);
  hip::mod_partition_counts(reinterpret_cast<const int64_t *>(t->column(key).data.data_ptr()), t->Rows(), P,
                            ptr<int64_t>(counts), ex.stream);
  return to_host_vec(counts);
}

static TablePtr mod_reorder(const TablePtr &t, int key, uint32_t P) {
  Exec ex(t->device());
  const int64_t n = t->Rows();
  const Column &kc = t->column(key);
  std::vector<at::Tensor> src{kc.data};
  std::vector<int> widths{8};
  std::vector<int> dslot(t->Columns(), 0), vslot(t->Columns(), -1);
  auto add = [&](const at::Tensor &x, int w) {
    src.push_back(x);
    widths.push_back(w);
    return (int)src.size() - 1;
  };
  for (int c = 0; c < t->Columns(); ++c) {
    const Column &col = t->column(c);
    if (c != key) dslot[c] = add(col.data, col.type.width());
    if (col.nullable()) vslot[c] = add(col.validity, 1);
  }
  // validity bytes travel packed so a nullable all-8-byte table keeps the 8-byte path
  const BytePacking bp = PackByteColumns(ex, src, widths, n);
  std::vector<at::Tensor> out;
  std::vector<const uint8_t *> in;
  std::vector<uint8_t *> outp;
  for (auto &x : src) {
    out.push_back(at::empty_like(x));
    in.push_back(reinterpret_cast<const uint8_t *>(x.data_ptr()));
    outp.push_back(reinterpret_cast<uint8_t *>(out.back().data_ptr()));
  }
  at::Tensor ws = ex.empty_i64(hip::radix_mod_rows_pass_workspace(n, P));
  hip::radix_mod_rows_pass(reinterpret_cast<const int64_t *>(in[0]), n, P, in.data(), outp.data(), widths.data(),
                           (int)in.size(), ptr<int64_t>(ws), ex.stream);
  out = UnpackByteColumns(ex, bp, std::move(out), n);
  std::vector<Column> cols;
  for (int c = 0; c < t->Columns(); ++c) {
    const Column &col = t->column(c);
    cols.emplace_back(col.name, col.type, n, out[dslot[c]], at::Tensor(), vslot[c] >= 0 ? out[vslot[c]] : at::Tensor());
  }
  return Table::Make(t->GetContext(), std::move(cols));
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
  TablePtr keep;         // the sent table (its buffers must outlive the posted transfers)
  TablePtr passthrough;  // world 1
  std::vector<int64_t> wire_base;  // per column: narrowed on the wire (see WirePlan) -> base, else unset
  std::vector<bool> wire_narrow;
  std::vector<DataType> wire_type;  // original column types
};

// Wire format of a shuffled table: 8-byte signed integer columns whose global
// value range fits 32 bits travel as uint32 offsets from the global minimum
// (frame of reference), so e.g. the headline join's int64 key costs 4 of the
// 32 bytes a row puts on xGMI instead of 8; the receiver widens them back.
// Config "shuffle_narrow" = "0" (or CYLON_SHUFFLE_NARROW=0) turns it off.
struct WirePlan {
  std::vector<bool> narrow;
  std::vector<int64_t> base;
  bool any() const {
    for (bool b : narrow)
      if (b) return true;
    return false;
  }
};

static bool narrow_candidate(const Column &c) {
  return !c.is_var() && c.type.kind() == ValueKind::SIGNED_INT && c.type.width() == 8 &&
         c.data.scalar_type() == at::kLong;
}

static std::vector<WirePlan> plan_wire(const std::vector<TablePtr> &ts) {
  std::vector<WirePlan> plans(ts.size());
  for (size_t i = 0; i < ts.size(); ++i) {
    plans[i].narrow.assign(ts[i]->Columns(), false);
    plans[i].base.assign(ts[i]->Columns(), 0);
  }
  auto ctx = ts[0]->GetContext();
  const std::string v = knobs::ConfigOr(ctx->GetConfig("shuffle_narrow", ""), "SHUFFLE_NARROW");
  if (v == "0") return plans;
  std::vector<std::pair<size_t, int>> cand;
  for (size_t i = 0; i < ts.size(); ++i)
    for (int c = 0; c < ts[i]->Columns(); ++c)
      if (narrow_candidate(ts[i]->column(c))) cand.push_back({i, c});
  if (cand.empty()) return plans;
  const at::Device dev = ts[0]->device();
  std::vector<at::Tensor> lo, hi;
  for (auto &ic : cand) {
    const Column &c = ts[ic.first]->column(ic.second);
    if (c.length == 0) {
      lo.push_back(at::full({1}, std::numeric_limits<int64_t>::max(), at::TensorOptions().dtype(at::kLong).device(dev)));
      hi.push_back(at::full({1}, std::numeric_limits<int64_t>::min(), at::TensorOptions().dtype(at::kLong).device(dev)));
    } else {
      auto mm = at::aminmax(c.data.slice(0, 0, c.length));
      lo.push_back(std::get<0>(mm).reshape({1}));
      hi.push_back(std::get<1>(mm).reshape({1}));
    }
  }
  at::Tensor mins = at::cat(lo), maxs = at::cat(hi);
  auto comm = ctx->GetCommunicator();
  comm->AllReduce(mins, net::ReduceOp::MIN);
  comm->AllReduce(maxs, net::ReduceOp::MAX);
  const std::vector<int64_t> hmin = to_host_vec(mins), hmax = to_host_vec(maxs);
  for (size_t j = 0; j < cand.size(); ++j) {
    if (hmax[j] < hmin[j]) continue;  // no rows anywhere
    if ((uint64_t)hmax[j] - (uint64_t)hmin[j] > 0xffffffffull) continue;
    plans[cand[j].first].narrow[cand[j].second] = true;
    plans[cand[j].first].base[cand[j].second] = hmin[j];
    trace::add_counter("shuffle.narrowed_columns", 1);
  }
  return plans;
}

// narrowed columns replaced by int32-stored offsets (same names)
static TablePtr to_wire(const TablePtr &t, const WirePlan &p) {
  if (!p.any()) return t;
  Exec ex(t->device());
  std::vector<Column> cols;
  for (int c = 0; c < t->Columns(); ++c) {
    const Column &col = t->column(c);
    if (!p.narrow[c]) {
      cols.push_back(col);
      continue;
    }
    at::Tensor w = at::empty({col.length}, ex.opts(at::kInt));
    KCALL(ex, narrow_i64, ptr<int64_t>(col.data), col.length, p.base[c], reinterpret_cast<uint32_t *>(ptr<int32_t>(w)));
    cols.emplace_back(col.name, DataType(Type::UINT32), col.length, w, at::Tensor(), col.validity);
  }
  return Table::Make(t->GetContext(), std::move(cols));
}

static void attach_plan(PendingTable &pt, const TablePtr &orig, const WirePlan &p) {
  if (!p.any()) return;
  pt.wire_narrow = p.narrow;
  pt.wire_base = p.base;
  for (const auto &c : orig->columns()) pt.wire_type.push_back(c.type);
}

// schema-level nullability of every column, agreed across ranks (one all-reduce
// for any number of tables with the same column count)
static std::vector<int64_t> agree_nullability(const std::vector<TablePtr> &ts) {
  auto ctx = ts[0]->GetContext();
  std::vector<int> off;
  int total = 0;
  for (auto &t : ts) {
    off.push_back(total);
    total += t->Columns();
  }
  at::Tensor flags = at::zeros({std::max(total, 1)}, at::TensorOptions().dtype(at::kInt));
  for (size_t i = 0; i < ts.size(); ++i)
    for (int c = 0; c < ts[i]->Columns(); ++c) flags[off[i] + c] = ts[i]->column(c).nullable() ? 1 : 0;
  at::Tensor g = flags.to(ts[0]->device());
  ctx->GetCommunicator()->AllReduce(g, net::ReduceOp::MAX);
  return to_host_vec(g.to(at::kLong));
}

// Posts one all-to-all per column buffer of `part` (rows already grouped by
// destination rank, send_rows[r] rows for rank r) and returns without waiting.
// nullable[c] is the cross-rank agreed nullability of column c.
static PendingTable AllToAllPost(const TablePtr &part, const std::vector<int64_t> &send_rows,
                                 const std::vector<int64_t> &recv_rows, const std::vector<int64_t> &nullable) {
  PendingTable pt;
  auto ctx = part->GetContext();
  pt.ctx = ctx;
  auto comm = ctx->GetCommunicator();
  const int world = ctx->GetWorldSize();
  for (auto r : recv_rows) pt.total += r;
  Exec ex(part->device());
  auto post = [&](const at::Tensor &t, const std::vector<int64_t> &sc, const std::vector<int64_t> &rc) {
    auto r = comm->AllToAllVAsync(t, sc, rc);
    pt.reqs.push_back(r.second);
    return r.first;
  };
  for (int c = 0; c < part->Columns(); ++c) {
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
  pt.keep = part;
  return pt;
}

// requests of a just-posted exchange that are still running (Test() == false): the
// transfer is asynchronous to the host and to the kernels enqueued after it
static void count_pending(const PendingTable &pt) {
  if (!trace::enabled()) return;
  int64_t pending = 0;
  for (auto &r : pt.reqs) pending += r->Test() ? 0 : 1;
  trace::add_counter("shuffle.requests_posted", (int64_t)pt.reqs.size());
  trace::add_counter("shuffle.requests_pending_after_post", pending);
}

static PendingTable AllToAllBegin(const TablePtr &part, const std::vector<int64_t> &counts) {
  auto ctx = part->GetContext();
  const int world = ctx->GetWorldSize();
  if (!ctx->ShuffleRequired()) {
    PendingTable pt;
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
  std::vector<int64_t> recv_rows = ctx->GetCommunicator()->ExchangeCounts(send_rows);
  const std::vector<int64_t> nullable = agree_nullability({part});
  const WirePlan plan = plan_wire({part})[0];
  PendingTable pt = AllToAllPost(to_wire(part, plan), send_rows, recv_rows, nullable);
  attach_plan(pt, part, plan);
  count_pending(pt);
  return pt;
}

static TablePtr AllToAllFinish(PendingTable &pt) {
  if (pt.passthrough) return pt.passthrough;
  // a request still in flight when its consumer arrives means the transfer overlapped the
  // work enqueued since it was posted (the wait below is a stream wait on RCCL, not a block)
  int64_t in_flight = 0;
  for (auto &r : pt.reqs) in_flight += r->Test() ? 0 : 1;
  trace::add_counter("shuffle.requests_waited", (int64_t)pt.reqs.size());
  trace::add_counter("shuffle.requests_in_flight_at_wait", in_flight);
  for (auto &r : pt.reqs) r->Wait();
  std::vector<Column> out;
  for (size_t c = 0; c < pt.cols.size(); ++c) {
    auto &pc = pt.cols[c];
    const Column &col = *pc.src;
    if (!pt.wire_narrow.empty() && pt.wire_narrow[c]) {  // widen back to int64
      Exec ex(pc.data.device());
      at::Tensor w = ex.empty_i64(pt.total);
      KCALL(ex, widen_u32, reinterpret_cast<const uint32_t *>(ptr<int32_t>(pc.data)), pt.total, pt.wire_base[c],
            ptr<int64_t>(w));
      out.emplace_back(col.name, pt.wire_type[c], pt.total, w, at::Tensor(), pc.valid);
    } else if (!col.is_var()) {
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

struct PostedExchange {
  PendingTable pt;
};

std::shared_ptr<PostedExchange> PostAllToAllTable(const TablePtr &part, const std::vector<int64_t> &counts) {
  auto x = std::make_shared<PostedExchange>();
  x->pt = AllToAllBegin(part, counts);
  return x;
}

bool PostedExchangeReady(PostedExchange &x) {
  if (x.pt.passthrough) return true;
  for (auto &r : x.pt.reqs)
    if (!r->Test()) return false;
  return true;
}

TablePtr FinishPostedExchange(PostedExchange &x) { return AllToAllFinish(x.pt); }

std::pair<TablePtr, std::vector<int64_t>> ShufflePartition(const TablePtr &t, const std::vector<int> &hash_cols,
                                                           uint32_t nparts) {
  if (mod_pass_eligible(t, hash_cols, nparts)) return {mod_reorder(t, hash_cols[0], nparts), mod_counts(t, hash_cols[0], nparts)};
  return PartitionReorder(t, hash_pids(t, hash_cols, nparts), nparts);
}

static std::pair<TablePtr, std::vector<int64_t>> shuffle_partition(const TablePtr &t,
                                                                   const std::vector<int> &hash_cols, int world) {
  CYLON_PHASE("shuffle.partition", t->device());
  if (mod_pass_eligible(t, hash_cols, (uint32_t)world)) {
    std::vector<int64_t> counts = mod_counts(t, hash_cols[0], (uint32_t)world);
    return {mod_reorder(t, hash_cols[0], (uint32_t)world), counts};
  }
  at::Tensor pid = hash_pids(t, hash_cols, (uint32_t)world);
  return PartitionReorder(t, pid, (uint32_t)world);
}

static void planned_shuffle(const std::vector<TablePtr> &ts, const std::vector<std::vector<int>> &tcols,
                            bool allow_chunks,
                            const std::function<void(int, int, const std::vector<TablePtr> &)> &consume);

TablePtr Shuffle(const TablePtr &t, const std::vector<int> &hash_cols) {
  auto ctx = t->GetContext();
  const int world = ctx->GetWorldSize();
  if (!ctx->ShuffleRequired()) return t;
  bool var = false;
  for (const auto &c : t->columns()) var |= c.is_var();
  if (!var) {  // fixed width: one planning collective (ShufflePairPlanned's descriptor), one post
    TablePtr out;
    planned_shuffle({t}, {hash_cols}, false, [&](int, int, const std::vector<TablePtr> &r) { out = r[0]; });
    return out;
  }
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
  if (!ctx->ShuffleRequired()) return {a, b};
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

namespace cylon {
namespace ops {

// Number of hash chunks for a pipelined binary operator (identical on every
// rank: config / environment, or the global row count).  Context config
// "shuffle_chunks" (or CYLON_SHUFFLE_CHUNKS) forces a value; by default device
// tables with >= 2^24 rows per rank per relation are shuffled in 4 chunks, so
// that three quarters of the local operator overlap the RCCL transfer.
int ShuffleChunks(const TablePtr &a, const TablePtr &b) {
  auto ctx = a->GetContext();
  for (const TablePtr &t : {a, b})
    for (const auto &c : t->columns())
      if (c.is_var()) return 1;
  const std::string v = knobs::ConfigOr(ctx->GetConfig("shuffle_chunks", ""), "SHUFFLE_CHUNKS");
  if (!v.empty()) return std::max(1, std::min(64, std::atoi(v.c_str())));
  if (!a->device().is_cuda() || !ctx->ShuffleRequired()) return 1;
  at::Tensor rows = at::tensor({std::min(a->Rows(), b->Rows())}, at::TensorOptions().dtype(at::kLong)).to(a->device());
  ctx->GetCommunicator()->AllReduce(rows, net::ReduceOp::MIN);
  return rows.item<int64_t>() >= (int64_t(1) << 24) ? 4 : 1;
}

// Pipelined shuffle of two relations in K hash-disjoint chunks.
//
// Rows are partitioned once into W*K partitions with the reference's partition
// hash h (pid = h % (W*K) = W*chunk + rank, chunk = (h / W) % K), so the rank
// a row goes to is h % W exactly as in the unchunked shuffle, and a chunk is a
// contiguous, rank-grouped row range of the reordered table.  The counts of
// every chunk and both tables are exchanged in one all-to-all, then every
// chunk's column all-to-alls are posted at once: RCCL runs them back to back on
// its own stream while `consume(k, a_k, b_k)` processes chunk k on the compute
// stream as soon as chunk k has landed (the request waits are stream waits on
// RCCL, not host blocks), so the local work on chunk k overlaps the xGMI
// transfer of chunks k+1..K-1.  Equal keys hash to the same chunk, which makes
// any per-key operator (join of every type, set ops) chunk-separable.
// Fixed-width columns only (var-width columns would need a synchronous byte
// count exchange per chunk).
void ShufflePairChunked(const TablePtr &a, const std::vector<int> &acols, const TablePtr &b,
                        const std::vector<int> &bcols, int chunks,
                        const std::function<void(int, const TablePtr &, const TablePtr &)> &consume) {
  auto ctx = a->GetContext();
  const int W = ctx->GetWorldSize();
  const int K = std::max(1, chunks);
  for (const TablePtr &t : {a, b})
    for (const auto &c : t->columns())
      CYLON_CHECK(!c.is_var(), Code::Invalid, "chunked shuffle supports fixed-width columns only");
  const uint32_t P = (uint32_t)W * (uint32_t)K;
  if (!ctx->ShuffleRequired()) {
    auto ra = PartitionReorder(a, hash_pids(a, acols, P), P);
    auto rb = PartitionReorder(b, hash_pids(b, bcols, P), P);
    int64_t oa = 0, ob = 0;
    for (int k = 0; k < K; ++k) {
      const int64_t na = ra.second[k], nb = rb.second[k];
      consume(k, Slice(ra.first, oa, na), Slice(rb.first, ob, nb));
      oa += na;
      ob += nb;
    }
    return;
  }
  auto comm = ctx->GetCommunicator();
  // partition ids and counts of both tables first (cheap), so that one count exchange
  // serves every chunk and b's reorder can run while a's first chunk is on the wire
  std::pair<at::Tensor, at::Tensor> ha, hb;
  const bool fast_a = mod_pass_eligible(a, acols, P), fast_b = mod_pass_eligible(b, bcols, P);
  std::vector<int64_t> ca, cb;
  {
    CYLON_PHASE("shuffle.partition", a->device());
    if (fast_a) ca = mod_counts(a, acols[0], P);
    else ha = hash_pids_counts(a, acols, P);
    if (fast_b) cb = mod_counts(b, bcols[0], P);
    else hb = hash_pids_counts(b, bcols, P);
  }
  if (!fast_a) ca = to_host_vec(ha.second);
  if (!fast_b) cb = to_host_vec(hb.second);
  trace::add_counter("shuffle.fast_partition", (fast_a ? 1 : 0) + (fast_b ? 1 : 0));
  // block r of the exchange = [a chunks 0..K-1, b chunks 0..K-1] for rank r
  std::vector<int64_t> sendc((size_t)W * 2 * K), recvc;
  for (int r = 0; r < W; ++r)
    for (int k = 0; k < K; ++k) {
      sendc[(size_t)r * 2 * K + k] = ca[(size_t)k * W + r];
      sendc[(size_t)r * 2 * K + K + k] = cb[(size_t)k * W + r];
    }
  {
    at::Tensor s = at::tensor(sendc, at::TensorOptions().dtype(at::kLong)).to(a->device());
    std::vector<int64_t> per(W, 2 * K);
    recvc = to_host_vec(comm->AllToAllV(s, per, per));
  }
  const std::vector<int64_t> nullable = agree_nullability({a, b});
  const std::vector<WirePlan> plans = plan_wire({a, b});
  const std::vector<int64_t> na_flags(nullable.begin(), nullable.begin() + a->Columns());
  const std::vector<int64_t> nb_flags(nullable.begin() + a->Columns(), nullable.end());

  std::vector<PendingTable> pa(K), pb(K);
  std::vector<int64_t> offa(K + 1, 0), offb(K + 1, 0);
  auto post = [&](const TablePtr &part, const std::vector<int64_t> &cnt, int side, int k,
                  const std::vector<int64_t> &flags, std::vector<int64_t> &off) -> PendingTable {
    std::vector<int64_t> sc(W), rc(W);
    int64_t tot = 0;
    for (int r = 0; r < W; ++r) {
      sc[r] = cnt[(size_t)k * W + r];
      rc[r] = recvc[(size_t)r * 2 * K + side * K + k];
      tot += sc[r];
    }
    off[k + 1] = off[k] + tot;
    PendingTable pt = AllToAllPost(Slice(part, off[k], tot), sc, rc, flags);
    attach_plan(pt, side == 0 ? a : b, plans[side]);
    count_pending(pt);
    return pt;
  };
  TablePtr pta, ptb;
  {
    CYLON_PHASE("shuffle.reorder+post", a->device());
    pta = to_wire(fast_a ? mod_reorder(a, acols[0], P) : PartitionReorder(a, ha.first, P).first, plans[0]);
    ha = {};
    pa[0] = post(pta, ca, 0, 0, na_flags, offa);  // a's chunk 0 transfers while b is reordered
    ptb = to_wire(fast_b ? mod_reorder(b, bcols[0], P) : PartitionReorder(b, hb.first, P).first, plans[1]);
    hb = {};
    pb[0] = post(ptb, cb, 1, 0, nb_flags, offb);
    for (int k = 1; k < K; ++k) {
      pa[k] = post(pta, ca, 0, k, na_flags, offa);
      pb[k] = post(ptb, cb, 1, k, nb_flags, offb);
    }
  }
  trace::add_counter("shuffle.rows_in", a->Rows() + b->Rows());
  trace::add_counter("shuffle.bytes_in", a->nbytes() + b->nbytes());
  trace::add_counter("shuffle.chunks", K);
  for (int k = 0; k < K; ++k) {
    TablePtr ta, tb;
    {
      CYLON_PHASE("shuffle.wait", a->device());
      ta = AllToAllFinish(pa[k]);
      tb = AllToAllFinish(pb[k]);
    }
    pa[k] = PendingTable();
    pb[k] = PendingTable();
    trace::add_counter("shuffle.rows_out", ta->Rows() + tb->Rows());
    consume(k, ta, tb);
  }
}


// ---------------------------------------------------------------------------
// ShufflePairPlanned: one host-synchronous collective before the first payload post.
//
// The row counts are computed for P = W * Kc partitions (chunk-major pid = h % P, so the
// destination rank is pid % W = h % W), which serves both outcomes: K = Kc chunks use them
// directly, K = 1 sums a rank's Kc chunk counts.  Every rank's descriptor
//   [rows_a, rows_b | nullable flags of a's and b's columns | min, max of every narrowable
//    int64 column | counts_a[P] | counts_b[P]]
// is all-gathered once; K (the reference-compatible default: 4 chunks when every rank holds
// >= 2^24 rows per relation on a GPU, else 1; config shuffle_chunks forces it), the receive
// counts, the agreed nullability and the wire narrowing are then derived identically on every
// rank from the gathered matrix, with no further collective before the payload all-to-alls.
// ---------------------------------------------------------------------------
static at::Tensor counts_device(const TablePtr &t, const std::vector<int> &cols, uint32_t P, bool fast) {
  Exec ex(t->device());
  if (fast) {
    at::Tensor c = ex.empty_i64(P);
    hip::mod_partition_counts(reinterpret_cast<const int64_t *>(t->column(cols[0]).data.data_ptr()), t->Rows(), P,
                              ptr<int64_t>(c), ex.stream);
    return c;
  }
  return hash_pids_counts(t, cols, P).second;
}


// ---------------------------------------------------------------------------
// Gapped exchange layout of one relation (planned_shuffle).  The sender's rows are laid out in
// partition-major order (pid = chunk * W + rank, the reference's modulo partition refined into K
// hash chunks) with, right after each chunk's OWN bucket, a receive region for the rows the other
// ranks send this rank in that chunk:
//   chunk k: [bucket (k,0)] ... [bucket (k,me)] [recv from 0 .. W-1, r != me] [bucket (k,me+1)] ...
// so chunk k's input to the local operator is the contiguous range [own rows | received rows]:
// the own partition never crosses the communicator (reference: table.cpp:89-106 keeps its piece
// off MPI) and received rows land where the operator reads them (no concatenation copy).  The
// reorder pass writes the gaps itself (kernels/radix_join.hip k_ts_offsets `extra`).  With
// config shuffle_self_rccl=1 the own bucket is sent to this rank as well and chunk k's input is
// its receive region alone (test knob: RCCL kernels run at world 1).
// ---------------------------------------------------------------------------
struct GapPlan {
  int W = 1, K = 1, me = 0;
  bool self_wire = false;
  int64_t total = 0;                                     // rows of a layout column
  std::vector<int64_t> bucket_base;                      // [W*K] first layout row of each partition
  std::vector<uint32_t> extra;                           // [2^bits(W*K)] gap rows before each bucket
  std::vector<int64_t> recv_base, recv_rows;             // [K] receive region of chunk k
  std::vector<std::vector<int64_t>> send_off, send_cnt;  // [K][W] (layout rows)
  std::vector<std::vector<int64_t>> recv_off, recv_cnt;  // [K][W]
  std::vector<int64_t> in_off, in_rows;                  // [K] chunk k's input range
  std::vector<int64_t> wire_rows;                        // [K] rows ANY rank puts on the wire in chunk k
};

static GapPlan gap_plan(int W, int K, int me, bool self_wire, const std::function<int64_t(int, int, int)> &cnt,
                        uint32_t P) {
  GapPlan g;
  g.W = W;
  g.K = K;
  g.me = me;
  g.self_wire = self_wire;
  uint32_t nbk = 1;
  while (nbk < P) nbk <<= 1;
  g.bucket_base.assign(P, 0);
  g.extra.assign(std::max<uint32_t>(nbk, 2), 0);
  g.recv_base.assign(K, 0);
  g.recv_rows.assign(K, 0);
  g.send_off.assign(K, std::vector<int64_t>(W, 0));
  g.send_cnt = g.recv_off = g.recv_cnt = g.send_off;
  g.in_off.assign(K, 0);
  g.in_rows.assign(K, 0);
  // the skip-the-collective decision must be the same on every rank: computed from the
  // whole gathered count matrix, not from this rank's own sends and receives
  g.wire_rows.assign(K, 0);
  for (int k = 0; k < K; ++k)
    for (int from = 0; from < W; ++from)
      for (int to = 0; to < W; ++to)
        if (from != to || self_wire) g.wire_rows[k] += cnt(k, from, to);
  int64_t row = 0, own = 0;  // own: rows of the sender's buckets placed so far
  for (int k = 0; k < K; ++k)
    for (int r = 0; r < W; ++r) {
      const uint32_t pid = (uint32_t)k * W + r;
      g.bucket_base[pid] = row;
      g.extra[pid] = (uint32_t)(row - own);
      const int64_t c = cnt(k, me, r);
      g.send_off[k][r] = row;
      g.send_cnt[k][r] = (r == me && !self_wire) ? 0 : c;
      row += c;
      own += c;
      if (r != me) continue;
      g.recv_base[k] = row;
      for (int src = 0; src < W; ++src) {
        g.recv_off[k][src] = row;
        g.recv_cnt[k][src] = (src == me && !self_wire) ? 0 : cnt(k, src, me);
        row += g.recv_cnt[k][src];
      }
      g.recv_rows[k] = row - g.recv_base[k];
      g.in_off[k] = self_wire ? g.recv_base[k] : g.bucket_base[pid];
      g.in_rows[k] = g.recv_rows[k] + (self_wire ? 0 : c);
    }
  for (uint32_t p = P; p < (uint32_t)g.extra.size(); ++p) g.extra[p] = (uint32_t)(row - own);  // unused digits
  g.total = row;
  return g;
}

// ts[i] reordered into its gapped layout (columns of g.total rows; agreed-nullable columns get a
// validity buffer whatever this rank holds).  Fast path: ONE LDS-staged mod-partition pass writes
// the gaps itself; otherwise a partition-major reorder is copied bucket-range by bucket-range.
static TablePtr layout_reorder(const TablePtr &t, const std::vector<int> &kcols, uint32_t P, const GapPlan &g,
                               const std::vector<int64_t> &nullable, bool fast, bool *used_fast,
                               const at::Tensor &pid_pre = at::Tensor()) {
  Exec ex(t->device());
  const int64_t n = t->Rows();
  *used_fast = false;
  if (fast && n > 0 && g.total < (int64_t(1) << 32)) {
    const int key = kcols[0];
    const Column &kc = t->column(key);
    std::vector<at::Tensor> src{kc.data};
    std::vector<int> widths{8};
    std::vector<int> dslot(t->Columns(), 0), vslot(t->Columns(), -1);
    for (int c = 0; c < t->Columns(); ++c) {
      const Column &col = t->column(c);
      if (c != key) {
        dslot[c] = (int)src.size();
        src.push_back(col.data);
        widths.push_back(col.type.width());
      }
      if (col.nullable()) {
        vslot[c] = (int)src.size();
        src.push_back(col.validity);
        widths.push_back(1);
      }
    }
    const BytePacking bp = PackByteColumns(ex, src, widths, n);
    std::vector<at::Tensor> out;
    std::vector<const uint8_t *> in;
    std::vector<uint8_t *> outp;
    for (auto &x : src) {
      out.push_back(at::empty({g.total}, x.options()));
      in.push_back(reinterpret_cast<const uint8_t *>(x.data_ptr()));
      outp.push_back(reinterpret_cast<uint8_t *>(out.back().data_ptr()));
    }
    at::Tensor ws = ex.empty_i64(hip::radix_mod_rows_pass_workspace(n, P));
    at::Tensor extra = at::from_blob(const_cast<uint32_t *>(g.extra.data()), {(int64_t)g.extra.size()},
                                     at::TensorOptions().dtype(at::kInt))
                           .to(ex.device);
    if (hip::radix_mod_rows_pass_gapped(reinterpret_cast<const int64_t *>(in[0]), n, P, in.data(), outp.data(),
                                        widths.data(), (int)in.size(), ptr<int64_t>(ws), ex.stream,
                                        reinterpret_cast<const uint32_t *>(ptr<int32_t>(extra)), g.total)) {
      out = UnpackByteColumns(ex, bp, std::move(out), g.total);
      std::vector<Column> cols;
      for (int c = 0; c < t->Columns(); ++c) {
        const Column &col = t->column(c);
        at::Tensor v = vslot[c] >= 0 ? out[vslot[c]] : at::Tensor();
        if (!v.defined() && nullable[c]) v = at::ones({g.total}, ex.opts(at::kByte));
        cols.emplace_back(col.name, col.type, g.total, out[dslot[c]], at::Tensor(), v);
      }
      *used_fast = true;
      trace::add_counter("shuffle.gapped_pass", 1);
      return Table::Make(t->GetContext(), std::move(cols));
    }
  }
  // partition-major reorder, then two range copies per chunk (buckets up to the own one, the rest)
  trace::add_counter("shuffle.gapped_copy", 1);
  std::pair<TablePtr, std::vector<int64_t>> ro =
      fast ? std::make_pair(mod_reorder(t, kcols[0], P), std::vector<int64_t>())
           : PartitionReorder(t, pid_pre.defined() ? pid_pre : hash_pids(t, kcols, P), P);
  std::vector<Column> cols;
  for (int c = 0; c < t->Columns(); ++c) {
    const Column &col = t->column(c);
    Column o = make_fixed_column(col.name, col.type, g.total, ex.device, nullable[c] != 0);
    if (o.nullable()) o.validity.fill_(1);
    cols.push_back(std::move(o));
  }
  TablePtr lay = Table::Make(t->GetContext(), cols);
  int64_t src_row = 0;
  for (int k = 0; k < g.K; ++k)
    for (int part = 0; part < 2; ++part) {
      const int r0 = part == 0 ? 0 : g.me + 1, r1 = part == 0 ? g.me + 1 : g.W;
      if (r0 >= r1) continue;
      const int64_t dst = g.bucket_base[(size_t)k * g.W + r0];
      int64_t len = 0;
      for (int r = r0; r < r1; ++r) len += (r == g.me && !g.self_wire) ? g.in_rows[k] - g.recv_rows[k] : g.send_cnt[k][r];
      if (len == 0) continue;
      for (int c = 0; c < t->Columns(); ++c) {
        Column d = lay->column(c).slice(dst, len);
        Column sc = ro.first->column(c).slice(src_row, len);
        d.data.copy_(sc.data);
        if (d.nullable() && sc.nullable()) d.validity.copy_(sc.validity);
      }
      src_row += len;
    }
  return lay;
}

struct GapPending {
  std::vector<std::shared_ptr<net::P2PRequest>> reqs;
  std::vector<std::pair<int, at::Tensor>> widen;  // (column, received narrowed values of chunk k)
};

// posts chunk k of a gapped layout: one segment all-to-all per column buffer
static GapPending post_gapped(const TablePtr &lay, const GapPlan &g, int k, const WirePlan &plan,
                              const std::vector<at::Tensor> &wire, const std::vector<int64_t> &nullable,
                              int skip_col = -1) {
  GapPending pd;
  auto comm = lay->GetContext()->GetCommunicator();
  // nothing crosses the wire in chunk k on ANY rank (world 1 with the own rows local): every rank
  // skips the collectives together; otherwise every rank posts, with zero counts where it is idle
  if (g.wire_rows[k] == 0) return pd;
  Exec ex(lay->device());
  auto scaled = [](std::vector<int64_t> v, int64_t per, int64_t minus) {
    for (auto &x : v) x = (x - minus) * per;
    return v;
  };
  for (int c = 0; c < lay->Columns(); ++c) {
    if (c == skip_col) continue;  // (a proxy's source-row column is used by the sender only)
    const Column &col = lay->column(c);
    const int64_t per = col.type.kind() == ValueKind::FIXED_BYTES ? col.type.width() : 1;
    if (nullable[c])
      pd.reqs.push_back(comm->AllToAllVSegmentsAsync(col.validity, g.send_off[k], g.send_cnt[k], col.validity,
                                                     g.recv_off[k], g.recv_cnt[k]));
    if (!plan.narrow.empty() && plan.narrow[c]) {
      at::Tensor tmp = at::empty({std::max<int64_t>(g.recv_rows[k], 1)}, ex.opts(at::kInt));
      pd.reqs.push_back(comm->AllToAllVSegmentsAsync(wire[c], g.send_off[k], g.send_cnt[k], tmp,
                                                     scaled(g.recv_off[k], 1, g.recv_base[k]), g.recv_cnt[k]));
      pd.widen.push_back({c, tmp});
    } else {
      pd.reqs.push_back(comm->AllToAllVSegmentsAsync(col.data, scaled(g.send_off[k], per, 0), scaled(g.send_cnt[k], per, 0),
                                                     col.data, scaled(g.recv_off[k], per, 0),
                                                     scaled(g.recv_cnt[k], per, 0)));
    }
  }
  if (trace::enabled()) {
    int64_t pending = 0;
    for (auto &r : pd.reqs) pending += r->Test() ? 0 : 1;
    trace::add_counter("shuffle.requests_posted", (int64_t)pd.reqs.size());
    trace::add_counter("shuffle.requests_pending_after_post", pending);
  }
  return pd;
}

// waits for chunk k (stream waits on RCCL), widens narrowed columns into place, returns the input
static TablePtr finish_gapped(const TablePtr &lay, const GapPlan &g, int k, GapPending &pd, const WirePlan &plan) {
  int64_t in_flight = 0;
  for (auto &r : pd.reqs) in_flight += r->Test() ? 0 : 1;
  trace::add_counter("shuffle.requests_waited", (int64_t)pd.reqs.size());
  trace::add_counter("shuffle.requests_in_flight_at_wait", in_flight);
  for (auto &r : pd.reqs) r->Wait();
  Exec ex(lay->device());
  for (auto &w : pd.widen) {
    const Column &col = lay->column(w.first);
    if (g.recv_rows[k] > 0)
      KCALL(ex, widen_u32, reinterpret_cast<const uint32_t *>(ptr<int32_t>(w.second)), g.recv_rows[k],
            plan.base[w.first], ptr<int64_t>(col.data) + g.recv_base[k]);
  }
  return Slice(lay, g.in_off[k], g.in_rows[k]);
}

// ts: one or two tables (the binary operators shuffle both relations in one plan).
static void planned_shuffle(const std::vector<TablePtr> &ts, const std::vector<std::vector<int>> &tcols,
                            bool allow_chunks,
                            const std::function<void(int, int, const std::vector<TablePtr> &)> &consume) {
  const int NT = (int)ts.size();
  auto ctx = ts[0]->GetContext();
  if (!ctx->ShuffleRequired()) {
    consume(0, 1, ts);
    return;
  }
  // Var-width (string / binary) columns: the planned exchange moves a fixed-width PROXY of the table
  // -- var column c replaced by its int64 lengths (with c's validity), plus a source-row column used
  // only on the sending side -- and each var column's bytes in a gapped byte layout of its own
  // (same partition order, receive regions sized by per-partition byte counts that travel in the
  // one descriptor), posted per chunk like the rows.  Chunk k's var column is its received bytes
  // with offsets from the chunk's lengths.  Reference: arrow_all_to_all.cpp (lengths + bytes).
  struct VarSpec {
    std::vector<int> vcols;  // var-width column indices
    int rid = -1;            // proxy column of the source row
    TablePtr orig;
    at::Tensor pid;          // partition ids of the original rows (W * Kc partitions)
  };
  std::vector<VarSpec> vs(NT);
  std::vector<TablePtr> tsp(ts);  // the tables as exchanged (proxies for var-width tables)
  int nvar = 0;
  for (int i = 0; i < NT; ++i) {
    for (int c = 0; c < ts[i]->Columns(); ++c)
      if (ts[i]->column(c).is_var()) vs[i].vcols.push_back(c);
    if (vs[i].vcols.empty()) continue;
    nvar += (int)vs[i].vcols.size();
    vs[i].orig = ts[i];
    Exec ex(ts[i]->device());
    const int64_t n = ts[i]->Rows();
    std::vector<Column> pc;
    for (int c = 0; c < ts[i]->Columns(); ++c) {
      const Column &col = ts[i]->column(c);
      if (!col.is_var()) {
        pc.push_back(col);
        continue;
      }
      at::Tensor lens = col.offsets.slice(0, 1, n + 1) - col.offsets.slice(0, 0, n);
      pc.emplace_back(col.name, DataType(Type::INT64), n, lens.contiguous(), at::Tensor(), col.validity);
    }
    vs[i].rid = (int)pc.size();
    pc.emplace_back("__cylon_row", DataType(Type::INT64), n, at::arange(n, ex.opts(at::kLong)));
    tsp[i] = Table::Make(ts[i]->GetContext(), std::move(pc));
  }
  const int W = ctx->GetWorldSize(), me = ctx->GetRank();
  const std::string v = knobs::ConfigOr(ctx->GetConfig("shuffle_chunks", ""), "SHUFFLE_CHUNKS");
  const int forced = !allow_chunks ? 1 : (v.empty() ? 0 : std::max(1, std::min(64, std::atoi(v.c_str()))));
  // 8 chunks on the device: the first chunk's exchange (the only one with no join to hide behind)
  // is 1/8 of the traffic; the self-wire trace overlaps 82.5 % of the RCCL time at 8 chunks vs
  // 70.1 % at 4, and the step is 7 % faster (profiles/r04/rccl_selfwire_k*_overlap.txt)
  const int Kc = forced ? forced : (ts[0]->device().is_cuda() ? 8 : 1);
  const uint32_t P = (uint32_t)W * (uint32_t)Kc;
  const at::Device dev = ts[0]->device();
  const auto lopt = at::TensorOptions().dtype(at::kLong).device(dev);
  // ---- the descriptor (assembled on the device: no sync before the all-gather)
  std::vector<at::Tensor> parts;
  std::vector<int64_t> rows, nflags;
  for (const TablePtr &t : tsp) rows.push_back(t->Rows());
  for (const TablePtr &t : tsp)
    for (const auto &c : t->columns()) nflags.push_back(c.nullable() ? 1 : 0);
  parts.push_back(at::tensor(rows, at::TensorOptions().dtype(at::kLong)).to(dev));
  parts.push_back(at::tensor(nflags, at::TensorOptions().dtype(at::kLong)).to(dev));
  const std::string nv = knobs::ConfigOr(ctx->GetConfig("shuffle_narrow", ""), "SHUFFLE_NARROW");
  std::vector<std::pair<int, int>> cand;  // (table, column) narrowable on the wire
  if (nv != "0")
    for (int side = 0; side < NT; ++side)
      for (int c = 0; c < tsp[side]->Columns(); ++c)
        if (c != vs[side].rid && narrow_candidate(tsp[side]->column(c))) cand.push_back({side, c});
  std::vector<bool> fast(NT);
  std::vector<at::Tensor> vbytes;  // per var column: bytes per partition
  std::vector<at::Tensor> counts(NT), key_mm(NT);  // key_mm: the fast count kernel's key min / max
  {
    CYLON_PHASE("shuffle.partition", dev);
    for (int i = 0; i < NT; ++i) {
      fast[i] = vs[i].vcols.empty() && mod_pass_eligible(ts[i], tcols[i], P);
      if (vs[i].vcols.empty()) {
        if (fast[i]) {  // counts and, for a narrowable key, its range from ONE read of the keys
          Exec ex(dev);
          counts[i] = ex.empty_i64(P);
          const bool kmm = std::find(cand.begin(), cand.end(), std::make_pair(i, tcols[i][0])) != cand.end();
          if (kmm) key_mm[i] = ex.empty_i64(2);
          hip::mod_partition_counts(reinterpret_cast<const int64_t *>(ts[i]->column(tcols[i][0]).data.data_ptr()),
                                    ts[i]->Rows(), P, ptr<int64_t>(counts[i]), ex.stream,
                                    kmm ? ptr<int64_t>(key_mm[i]) : nullptr);
        } else {
          counts[i] = counts_device(ts[i], tcols[i], P, false);
        }
        continue;
      }
      auto pc = hash_pids_counts(ts[i], tcols[i], P);  // the ORIGINAL key columns (a var key hashes its bytes)
      vs[i].pid = pc.first;
      counts[i] = pc.second;
      const at::Tensor pid64 = pc.first.to(at::kLong);
      for (int c : vs[i].vcols) {
        const Column &col = ts[i]->column(c);
        const int64_t n = ts[i]->Rows();
        at::Tensor lens = col.offsets.slice(0, 1, n + 1) - col.offsets.slice(0, 0, n);
        vbytes.push_back(at::zeros({(int64_t)P}, lens.options()).index_add_(0, pid64, lens));
      }
    }
  }
  for (auto &sc : cand) {
    const Column &c = tsp[sc.first]->column(sc.second);
    if (c.length == 0) {
      parts.push_back(at::tensor({std::numeric_limits<int64_t>::max(), std::numeric_limits<int64_t>::min()}, lopt));
    } else if (key_mm[sc.first].defined() && sc.second == tcols[sc.first][0]) {
      parts.push_back(key_mm[sc.first]);
      trace::add_counter("shuffle.fused_key_minmax", 1);
    } else {
      auto mm = at::aminmax(c.data.slice(0, 0, c.length));
      parts.push_back(at::stack({std::get<0>(mm), std::get<1>(mm)}));
    }
  }
  for (auto &cn : counts) parts.push_back(cn);
  for (auto &b : vbytes) parts.push_back(b);
  at::Tensor desc = at::cat(parts);
  const int64_t D = desc.numel();
  at::Tensor all;
  {
    CYLON_PHASE("shuffle.plan", dev);
    all = ctx->GetCommunicator()->AllGather(desc).to(at::kCPU).contiguous();
  }
  trace::add_counter("shuffle.plan_collectives", 1);
  const int64_t *g = all.data_ptr<int64_t>();  // W x D
  std::vector<int> ncols(NT), coff(NT + 1, 0);
  for (int i = 0; i < NT; ++i) {
    ncols[i] = tsp[i]->Columns();
    coff[i + 1] = coff[i] + ncols[i];
  }
  const int64_t off_null = NT, off_mm = off_null + coff[NT], off_cnt = off_mm + 2 * (int64_t)cand.size();
  const int64_t off_vb = off_cnt + (int64_t)NT * P;  // then P byte counts per var column
  CYLON_CHECK(off_vb + (int64_t)nvar * P == D, Code::ExecutionError, "shuffle descriptor layout");
  // own rows through the communicator as well (test knob: keeps the RCCL kernels running at world 1)
  const std::string sw = knobs::ConfigOr(ctx->GetConfig("shuffle_self_rccl", ""), "SHUFFLE_SELF_RCCL");
  const bool self_wire = sw == "1";
  int K = Kc;
  if (!forced) {  // chunked when every rank holds >= 2^24 rows of every table
    int64_t mn = std::numeric_limits<int64_t>::max();
    for (int r = 0; r < W; ++r)
      for (int i = 0; i < NT; ++i) mn = std::min(mn, g[r * D + i]);
    K = mn >= (int64_t(1) << 24) ? Kc : 1;
    // nothing crosses the wire at world 1 (the own partition stays in place): no transfer to overlap
    if (W == 1 && !self_wire) K = 1;
  }
  std::vector<int64_t> nullable(coff[NT], 0);
  for (int r = 0; r < W; ++r)
    for (int c = 0; c < coff[NT]; ++c) nullable[c] |= g[r * D + off_null + c];
  std::vector<WirePlan> plans(NT);
  for (int i = 0; i < NT; ++i) {
    plans[i].narrow.assign(ncols[i], false);
    plans[i].base.assign(ncols[i], 0);
  }
  for (size_t j = 0; j < cand.size(); ++j) {
    int64_t lo = std::numeric_limits<int64_t>::max(), hi = std::numeric_limits<int64_t>::min();
    for (int r = 0; r < W; ++r) {
      lo = std::min(lo, g[r * D + off_mm + 2 * j]);
      hi = std::max(hi, g[r * D + off_mm + 2 * j + 1]);
    }
    if (hi < lo || (uint64_t)hi - (uint64_t)lo > 0xffffffffull) continue;
    plans[cand[j].first].narrow[cand[j].second] = true;
    plans[cand[j].first].base[cand[j].second] = lo;
    trace::add_counter("shuffle.narrowed_columns", 1);
  }
  // rows this rank sends to / receives from rank r in chunk k (K = 1: a rank's Kc counts summed)
  auto cnt = [&](int side, int k, int from, int to) -> int64_t {
    const int64_t *c = g + (int64_t)from * D + off_cnt + (int64_t)side * P;
    if (K == Kc) return c[(int64_t)k * W + to];
    int64_t s = 0;
    for (int q = 0; q < Kc; ++q) s += c[(int64_t)q * W + to];
    return s;
  };
  // bytes of var column v (global index over the tables' var columns) this rank sends / receives
  auto cntb = [&](int v, int k, int from, int to) -> int64_t {
    const int64_t *c = g + (int64_t)from * D + off_vb + (int64_t)v * P;
    if (K == Kc) return c[(int64_t)k * W + to];
    int64_t s = 0;
    for (int q = 0; q < Kc; ++q) s += c[(int64_t)q * W + to];
    return s;
  };
  const uint32_t PK = (uint32_t)W * (uint32_t)K;
  if (PK == 1 && !self_wire) {  // world 1, one chunk: every row is already where it is consumed
    trace::add_counter("shuffle.self_rows_kept_local", ts[0]->Rows() + (NT > 1 ? ts[1]->Rows() : 0));
    trace::add_counter("shuffle.chunks", 1);
    consume(0, 1, ts);
    return;
  }
  std::vector<GapPlan> gp;
  for (int i = 0; i < NT; ++i)
    gp.push_back(gap_plan(W, K, me, self_wire, [&](int k, int from, int to) { return cnt(i, k, from, to); }, PK));
  // per var column: its gapped byte layout (plan in bytes) and the byte buffer
  std::vector<GapPlan> gpb;
  std::vector<at::Tensor> vbuf;
  std::vector<int> vfirst(NT, 0);  // first global var index of table i
  for (int i = 0, v = 0; i < NT; ++i) {
    vfirst[i] = v;
    for (size_t j = 0; j < vs[i].vcols.size(); ++j, ++v)
      gpb.push_back(gap_plan(W, K, me, self_wire, [&, v](int k, int from, int to) { return cntb(v, k, from, to); }, PK));
  }
  vbuf.resize(gpb.size());
  std::vector<TablePtr> lay(NT);
  std::vector<std::vector<GapPending>> pend(NT, std::vector<GapPending>(K));
  std::vector<std::vector<at::Tensor>> wire(NT);  // per column: narrowed send buffer (or undefined)
  auto post = [&](int side, int k) {
    const std::vector<int64_t> flags(nullable.begin() + coff[side], nullable.begin() + coff[side + 1]);
    pend[side][k] = post_gapped(lay[side], gp[side], k, plans[side], wire[side], flags, vs[side].rid);
    for (size_t j = 0; j < vs[side].vcols.size(); ++j) {  // the var columns' bytes of chunk k
      const int v = vfirst[side] + (int)j;
      if (gpb[v].wire_rows[k] == 0) continue;  // (agreed on every rank)
      pend[side][k].reqs.push_back(ctx->GetCommunicator()->AllToAllVSegmentsAsync(
          vbuf[v], gpb[v].send_off[k], gpb[v].send_cnt[k], vbuf[v], gpb[v].recv_off[k], gpb[v].recv_cnt[k]));
    }
  };
  int nfast = 0;
  {
    CYLON_PHASE("shuffle.reorder+post", dev);
    for (int i = 0; i < NT; ++i) {  // table i's first chunk transfers while table i+1 is reordered
      const std::vector<int64_t> flags(nullable.begin() + coff[i], nullable.begin() + coff[i + 1]);
      bool fastpath = false;
      const bool var_t = !vs[i].vcols.empty();
      lay[i] = layout_reorder(tsp[i], tcols[i], PK, gp[i], flags,
                              !var_t && (K == Kc ? fast[i] : mod_pass_eligible(ts[i], tcols[i], PK)), &fastpath,
                              var_t ? (K == Kc ? vs[i].pid : hash_pids(ts[i], tcols[i], PK)) : at::Tensor());
      nfast += fastpath ? 1 : 0;
      if (var_t) {  // each var column's bytes, gathered in the layout's bucket order into its byte layout
        Exec ex(dev);
        std::vector<at::Tensor> idxs;
        const at::Tensor &rid = lay[i]->column(vs[i].rid).data;
        for (int k = 0; k < K; ++k)
          for (int r = 0; r < W; ++r)
            if (const int64_t nr = cnt(i, k, me, r)) {
              const int64_t b0 = gp[i].bucket_base[(size_t)k * W + r];
              idxs.push_back(rid.slice(0, b0, b0 + nr));
            }
        const at::Tensor idx = idxs.empty() ? ex.empty_i64(0) : at::cat(idxs);
        for (size_t j = 0; j < vs[i].vcols.size(); ++j) {
          const int v = vfirst[i] + (int)j;
          const Column &vc = vs[i].orig->column(vs[i].vcols[j]);
          const TablePtr gt = Gather(Table::Make(ctx, {Column(vc.name, vc.type, vc.length, vc.data, vc.offsets)}), idx);
          const at::Tensor &gb = gt->column(0).data;
          vbuf[v] = at::empty({std::max<int64_t>(gpb[v].total, 1)}, ex.opts(at::kByte));
          int64_t cur = 0;
          for (int k = 0; k < K; ++k)
            for (int r = 0; r < W; ++r)
              if (const int64_t nb = cntb(v, k, me, r)) {
                const int64_t b0 = gpb[v].bucket_base[(size_t)k * W + r];
                vbuf[v].slice(0, b0, b0 + nb).copy_(gb.slice(0, cur, cur + nb));
                cur += nb;
              }
        }
        trace::add_counter("shuffle.var_columns_planned", (int64_t)vs[i].vcols.size());
      }
      wire[i].assign(tsp[i]->Columns(), at::Tensor());
      for (int c = 0; c < tsp[i]->Columns(); ++c)
        if (plans[i].narrow[c]) {  // narrowed copies of the rows that are sent (not the own rows)
          const Column &col = lay[i]->column(c);
          Exec ex(dev);
          wire[i][c] = at::empty({col.length}, ex.opts(at::kInt));
          for (int k = 0; k < K; ++k)
            for (int r = 0; r < W; ++r)
              if (const int64_t cnt_kr = gp[i].send_cnt[k][r]) {
                const int64_t o = gp[i].send_off[k][r];
                KCALL(ex, narrow_i64, ptr<int64_t>(col.data) + o, cnt_kr, plans[i].base[c],
                      reinterpret_cast<uint32_t *>(ptr<int32_t>(wire[i][c])) + o);
              }
        }
      post(i, 0);
    }
    for (int k = 1; k < K; ++k)
      for (int i = 0; i < NT; ++i) post(i, k);
  }
  int64_t rows_in = 0, bytes_in = 0, self_rows = 0;
  for (const TablePtr &t : ts) {
    rows_in += t->Rows();
    bytes_in += t->nbytes();
  }
  for (int i = 0; i < NT; ++i)
    for (int k = 0; k < K; ++k) self_rows += self_wire ? 0 : cnt(i, k, me, me);
  trace::add_counter("shuffle.fast_partition", nfast);
  trace::add_counter("shuffle.rows_in", rows_in);
  trace::add_counter("shuffle.bytes_in", bytes_in);
  trace::add_counter("shuffle.self_rows_kept_local", self_rows);
  trace::add_counter("shuffle.chunks", K);
  for (int k = 0; k < K; ++k) {
    std::vector<TablePtr> got(NT);
    {
      CYLON_PHASE("shuffle.wait", dev);
      for (int i = 0; i < NT; ++i) got[i] = finish_gapped(lay[i], gp[i], k, pend[i][k], plans[i]);
    }
    int64_t rows_out = 0;
    for (int i = 0; i < NT; ++i) {
      pend[i][k] = GapPending();
      rows_out += got[i]->Rows();
      if (vs[i].vcols.empty()) continue;
      // back to the original schema: lengths -> offsets over the chunk's bytes, source rows dropped
      Exec ex(dev);
      std::vector<Column> oc;
      for (int c = 0, j = 0; c < vs[i].orig->Columns(); ++c) {
        const Column &pcol = got[i]->column(c);
        if (j < (int)vs[i].vcols.size() && vs[i].vcols[j] == c) {
          const GapPlan &gb = gpb[vfirst[i] + j];
          at::Tensor offs = exclusive_scan(ex, pcol.data.contiguous());
          at::Tensor bytes = vbuf[vfirst[i] + j].slice(0, gb.in_off[k], gb.in_off[k] + gb.in_rows[k]);
          oc.emplace_back(pcol.name, vs[i].orig->column(c).type, pcol.length, bytes, offs, pcol.validity);
          ++j;
        } else {
          oc.push_back(pcol);
        }
      }
      got[i] = Table::Make(ctx, std::move(oc));
    }
    trace::add_counter("shuffle.rows_out", rows_out);
    consume(k, K, got);
  }
}

void RangeExchange(const TablePtr &t, const std::vector<int64_t> &bounds, int K,
                   const std::function<void(int, int, const TablePtr &, const std::vector<int64_t> &)> &consume) {
  auto ctx = t->GetContext();
  const int W = ctx->GetWorldSize(), me = ctx->GetRank();
  CYLON_CHECK(K >= 1 && (int64_t)bounds.size() == (int64_t)W * K + 1, Code::Invalid, "range exchange bounds");
  for (const auto &c : t->columns())
    CYLON_CHECK(!c.is_var(), Code::NotImplemented, "range exchange: fixed-width columns only");
  const at::Device dev = t->device();
  // descriptor: rows | nullable flag per column | rows per (destination, chunk)
  std::vector<int64_t> desc{t->Rows()};
  for (const auto &c : t->columns()) desc.push_back(c.nullable() ? 1 : 0);
  for (int64_t i = 0; i < (int64_t)W * K; ++i) desc.push_back(bounds[i + 1] - bounds[i]);
  const int64_t D = (int64_t)desc.size();
  at::Tensor all;
  {
    CYLON_PHASE("shuffle.plan", dev);
    all = ctx->GetCommunicator()->AllGather(at::tensor(desc, at::TensorOptions().dtype(at::kLong)).to(dev))
              .to(at::kCPU)
              .contiguous();
  }
  trace::add_counter("shuffle.plan_collectives", 1);
  const int64_t *g = all.data_ptr<int64_t>();
  const int nc = t->Columns();
  std::vector<int64_t> nullable(nc, 0);
  for (int r = 0; r < W; ++r)
    for (int c = 0; c < nc; ++c) nullable[c] |= g[r * D + 1 + c];
  auto cnt = [&](int from, int to, int k) { return g[(int64_t)from * D + 1 + nc + (int64_t)to * K + k]; };
  std::vector<PendingTable> pend(K);
  std::vector<std::vector<int64_t>> runs(K, std::vector<int64_t>(W));
  {
    CYLON_PHASE("shuffle.reorder+post", dev);
    for (int k = 0; k < K; ++k) {
      std::vector<int64_t> sc(W), rc(W);
      std::vector<TablePtr> pieces;
      for (int d = 0; d < W; ++d) {
        sc[d] = cnt(me, d, k);
        rc[d] = cnt(d, me, k);
        runs[k][d] = rc[d];
        pieces.push_back(Slice(t, bounds[(int64_t)d * K + k], sc[d]));
      }
      // K == 1: the destination ranges are already consecutive rows (no copy)
      TablePtr send = K == 1 ? t : Merge(pieces);
      pend[k] = AllToAllPost(send, sc, rc, nullable);
      count_pending(pend[k]);
    }
  }
  trace::add_counter("shuffle.chunks", K);
  for (int k = 0; k < K; ++k) {
    TablePtr got;
    {
      CYLON_PHASE("shuffle.wait", dev);
      got = AllToAllFinish(pend[k]);
    }
    pend[k] = PendingTable();
    trace::add_counter("shuffle.rows_out", got->Rows());
    consume(k, K, got, runs[k]);
  }
}

void ShufflePairPlanned(const TablePtr &a, const std::vector<int> &acols, const TablePtr &b,
                        const std::vector<int> &bcols,
                        const std::function<void(int, int, const TablePtr &, const TablePtr &)> &consume) {
  planned_shuffle({a, b}, {acols, bcols}, true,
                  [&](int k, int K, const std::vector<TablePtr> &t) { consume(k, K, t[0], t[1]); });
}

void ShufflePlanned(const TablePtr &t, const std::vector<int> &cols,
                    const std::function<void(int, int, const TablePtr &)> &consume) {
  planned_shuffle({t}, {cols}, true, [&](int k, int K, const std::vector<TablePtr> &r) { consume(k, K, r[0]); });
}

}  // namespace ops
}  // namespace cylon
