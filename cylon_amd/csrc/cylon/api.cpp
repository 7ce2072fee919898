// Status-returning API, table registry, Row/Select and the all-to-all classes (see api.hpp).
#include "api.hpp"

#include <iostream>
#include <mutex>

#include "ops/util.hpp"

namespace cylon {

namespace {
template <class F>
Status guard(F &&f) {
  try {
    f();
    return Status::OK();
  } catch (const CylonError &e) {
    return Status(e.code(), e.what());
  } catch (const std::exception &e) {
    return Status(Code::UnknownError, e.what());
  }
}
}  // namespace

Status FromCSV(const std::shared_ptr<CylonContext> &ctx, const std::string &path, TablePtr &out,
               const io::CSVReadOptions &options) {
  return guard([&] { out = io::ReadCSV(ctx, path, options); });
}
Status FromCSV(const std::shared_ptr<CylonContext> &ctx, const std::vector<std::string> &paths,
               std::vector<TablePtr> &out, const io::CSVReadOptions &options) {
  return guard([&] { out = io::ReadCSVs(ctx, paths, options); });
}
Status WriteCSV(const TablePtr &t, const std::string &path, const io::CSVWriteOptions &options) {
  return guard([&] { io::WriteCSV(t, path, options); });
}
Status FromParquet(const std::shared_ptr<CylonContext> &ctx, const std::string &path, TablePtr &out,
                   const io::ParquetOptions &options) {
  return guard([&] { out = io::ReadParquet(ctx, path, options); });
}
Status FromParquet(const std::shared_ptr<CylonContext> &ctx, const std::vector<std::string> &paths,
                   std::vector<TablePtr> &out, const io::ParquetOptions &options) {
  return guard([&] { out = io::ReadParquets(ctx, paths, options); });
}
Status WriteParquet(const TablePtr &t, const std::string &path, const io::ParquetOptions &options) {
  return guard([&] { io::WriteParquet(t, path, options); });
}

Status Join(const TablePtr &l, const TablePtr &r, const join::config::JoinConfig &cfg, TablePtr &out) {
  return guard([&] { out = ops::Join(l, r, cfg); });
}
Status DistributedJoin(const TablePtr &l, const TablePtr &r, const join::config::JoinConfig &cfg, TablePtr &out) {
  return guard([&] { out = ops::DistributedJoin(l, r, cfg); });
}
Status Union(const TablePtr &a, const TablePtr &b, TablePtr &out) { return guard([&] { out = ops::Union(a, b); }); }
Status Subtract(const TablePtr &a, const TablePtr &b, TablePtr &out) {
  return guard([&] { out = ops::Subtract(a, b); });
}
Status Intersect(const TablePtr &a, const TablePtr &b, TablePtr &out) {
  return guard([&] { out = ops::Intersect(a, b); });
}
Status DistributedUnion(const TablePtr &a, const TablePtr &b, TablePtr &out) {
  return guard([&] { out = ops::DistributedUnion(a, b); });
}
Status DistributedSubtract(const TablePtr &a, const TablePtr &b, TablePtr &out) {
  return guard([&] { out = ops::DistributedSubtract(a, b); });
}
Status DistributedIntersect(const TablePtr &a, const TablePtr &b, TablePtr &out) {
  return guard([&] { out = ops::DistributedIntersect(a, b); });
}
Status Project(const TablePtr &t, const std::vector<int32_t> &cols, TablePtr &out) {
  return guard([&] { out = ops::Project(t, std::vector<int>(cols.begin(), cols.end())); });
}
Status Merge(const std::vector<TablePtr> &tables, TablePtr &out) { return guard([&] { out = ops::Merge(tables); }); }
Status Sort(const TablePtr &t, int col, TablePtr &out, bool asc) {
  return guard([&] { out = ops::Sort(t, {col}, {asc}); });
}
Status Sort(const TablePtr &t, const std::vector<int32_t> &cols, TablePtr &out, const std::vector<bool> &dirs) {
  return guard([&] { out = ops::Sort(t, std::vector<int>(cols.begin(), cols.end()), dirs); });
}
Status DistributedSort(const TablePtr &t, const std::vector<int32_t> &cols, TablePtr &out,
                       const std::vector<bool> &dirs, SortOptions opts) {
  return guard([&] { out = ops::DistributedSort(t, std::vector<int>(cols.begin(), cols.end()), dirs, opts); });
}
Status Shuffle(const TablePtr &t, const std::vector<int> &cols, TablePtr &out) {
  return guard([&] { out = ops::Shuffle(t, cols); });
}
Status HashPartition(const TablePtr &t, const std::vector<int> &cols, int n, std::map<int, TablePtr> *out) {
  return guard([&] {
    auto parts = ops::HashPartition(t, cols, (uint32_t)n);
    out->clear();
    for (int i = 0; i < n; ++i) (*out)[i] = parts[i];
  });
}
Status Unique(const TablePtr &t, const std::vector<int> &cols, TablePtr &out, bool first) {
  return guard([&] { out = ops::Unique(t, cols, first); });
}
Status DistributedUnique(const TablePtr &t, const std::vector<int> &cols, TablePtr &out) {
  return guard([&] { out = ops::DistributedUnique(t, cols, true); });
}

// ---- Row / Select ----------------------------------------------------------------
bool Row::IsNull(int col) const {
  const Column &c = t_->column(col);
  return c.nullable() && c.validity.data_ptr<uint8_t>()[row_] == 0;
}

const uint8_t *Row::raw(int col, int *width) const {
  const Column &c = t_->column(col);
  CYLON_CHECK(!c.is_var(), Code::TypeError, "column " << c.name << " is variable width");
  CYLON_CHECK(row_ >= 0 && row_ < c.length, Code::IndexError, "row " << row_ << " out of range");
  *width = c.type.width();
  return static_cast<const uint8_t *>(c.data.data_ptr()) + row_ * (int64_t)(*width);
}

int64_t Row::GetInt64(int col) const {
  int w = 0;
  const uint8_t *p = raw(col, &w);
  const ValueKind k = t_->column(col).type.kind();
  CYLON_CHECK(k == ValueKind::SIGNED_INT || k == ValueKind::UNSIGNED_INT, Code::TypeError,
              "column " << t_->column(col).name << " is not an integer column");
  if (k == ValueKind::UNSIGNED_INT) return (int64_t)GetUInt64(col);
  switch (w) {
    case 1: return *reinterpret_cast<const int8_t *>(p);
    case 2: return *reinterpret_cast<const int16_t *>(p);
    case 4: return *reinterpret_cast<const int32_t *>(p);
    default: return *reinterpret_cast<const int64_t *>(p);
  }
}

uint64_t Row::GetUInt64(int col) const {
  int w = 0;
  const uint8_t *p = raw(col, &w);
  switch (w) {
    case 1: return *p;
    case 2: return *reinterpret_cast<const uint16_t *>(p);
    case 4: return *reinterpret_cast<const uint32_t *>(p);
    default: return *reinterpret_cast<const uint64_t *>(p);
  }
}

double Row::GetDouble(int col) const {
  const Column &c = t_->column(col);
  if (c.type.kind() != ValueKind::FLOAT) return c.type.kind() == ValueKind::UNSIGNED_INT ? (double)GetUInt64(col)
                                                                                         : (double)GetInt64(col);
  int w = 0;
  const uint8_t *p = raw(col, &w);
  if (w == 8) return *reinterpret_cast<const double *>(p);
  if (w == 4) return *reinterpret_cast<const float *>(p);
  return (double)c.data.slice(0, row_, row_ + 1).to(at::kDouble).item<double>();  // half
}

bool Row::GetBool(int col) const { return GetUInt64(col) != 0; }

const uint8_t *Row::GetFixedBinary(int col) const {
  int w = 0;
  return raw(col, &w);
}

std::string Row::GetString(int col) const {
  const Column &c = t_->column(col);
  CYLON_CHECK(c.is_var(), Code::TypeError, "column " << c.name << " is not a string column");
  const int64_t *o = c.offsets.data_ptr<int64_t>();
  const char *d = reinterpret_cast<const char *>(c.data.data_ptr<uint8_t>());
  return std::string(d + o[row_], d + o[row_ + 1]);
}

Status Select(const TablePtr &t, const std::function<bool(const Row &)> &pred, TablePtr &out) {
  return guard([&] {
    TablePtr host = t->device().is_cpu() ? t : t->to(at::Device(at::kCPU));
    at::Tensor mask = at::zeros({t->Rows()}, at::TensorOptions().dtype(at::kByte));
    uint8_t *m = mask.data_ptr<uint8_t>();
    for (int64_t i = 0; i < t->Rows(); ++i) m[i] = pred(Row(host, i)) ? 1 : 0;
    out = ops::FilterByMask(t, mask.to(t->device()));
  });
}

// ---- group-by / aggregates ----------------------------------------------------------
static std::vector<ops::AggSpec> specs(const std::vector<int32_t> &cols, const std::vector<AggOp> &ops_) {
  std::vector<ops::AggSpec> s;
  for (size_t i = 0; i < cols.size(); ++i) s.push_back(ops::AggSpec{cols[i], ops_[i]});
  return s;
}

Status DistributedHashGroupBy(const TablePtr &t, const std::vector<int32_t> &idx, const std::vector<int32_t> &cols,
                              const std::vector<AggOp> &ops_, TablePtr &out) {
  return guard([&] {
    CYLON_CHECK(cols.size() == ops_.size(), Code::Invalid, "aggregate columns and ops differ in length");
    out = ops::DistributedHashGroupBy(t, std::vector<int>(idx.begin(), idx.end()), specs(cols, ops_));
  });
}

Status DistributedPipelineGroupBy(const TablePtr &t, int32_t idx, const std::vector<int32_t> &cols,
                                  const std::vector<AggOp> &ops_, TablePtr &out) {
  return guard([&] { out = ops::DistributedPipelineGroupBy(t, {idx}, specs(cols, ops_)); });
}

namespace compute {
Status Sum(const TablePtr &t, int32_t col, TablePtr &out) {
  return guard([&] { out = ops::Aggregate(t, col, AGG_SUM, 0.5, 1, true); });
}
Status Count(const TablePtr &t, int32_t col, TablePtr &out) {
  return guard([&] { out = ops::Aggregate(t, col, AGG_COUNT, 0.5, 1, true); });
}
Status Min(const TablePtr &t, int32_t col, TablePtr &out) {
  return guard([&] { out = ops::Aggregate(t, col, AGG_MIN, 0.5, 1, true); });
}
Status Max(const TablePtr &t, int32_t col, TablePtr &out) {
  return guard([&] { out = ops::Aggregate(t, col, AGG_MAX, 0.5, 1, true); });
}
Status MinMax(const TablePtr &t, int32_t col, TablePtr &out) {
  return guard([&] {
    TablePtr mn = ops::Aggregate(t, col, AGG_MIN, 0.5, 1, true);
    TablePtr mx = ops::Aggregate(t, col, AGG_MAX, 0.5, 1, true);
    out = Table::Make(t->GetContext(), {mn->column(0).with_name("min"), mx->column(0).with_name("max")});
  });
}
}  // namespace compute

// ---- registry ------------------------------------------------------------------------
namespace {
std::mutex g_registry_mu;
std::map<std::string, TablePtr> &registry() {
  static std::map<std::string, TablePtr> r;
  return r;
}
}  // namespace

void PutTable(const std::string &id, const TablePtr &table) {
  std::lock_guard<std::mutex> lk(g_registry_mu);
  registry()[id] = table;
}

TablePtr GetTable(const std::string &id) {
  std::lock_guard<std::mutex> lk(g_registry_mu);
  auto it = registry().find(id);
  CYLON_CHECK(it != registry().end(), Code::KeyError, "no table with id '" << id << "'");
  return it->second;
}

void RemoveTable(const std::string &id) {
  std::lock_guard<std::mutex> lk(g_registry_mu);
  registry().erase(id);
}

std::vector<std::string> ListTables() {
  std::lock_guard<std::mutex> lk(g_registry_mu);
  std::vector<std::string> ids;
  for (auto &kv : registry()) ids.push_back(kv.first);
  return ids;
}

Status JoinTables(const std::string &l, const std::string &r, const join::config::JoinConfig &cfg,
                  const std::string &dest) {
  return guard([&] { PutTable(dest, ops::Join(GetTable(l), GetTable(r), cfg)); });
}

Status DistributedJoinTables(const std::string &l, const std::string &r, const join::config::JoinConfig &cfg,
                             const std::string &dest) {
  return guard([&] { PutTable(dest, ops::DistributedJoin(GetTable(l), GetTable(r), cfg)); });
}

Status UnionTables(const std::string &a, const std::string &b, const std::string &dest, bool distributed) {
  return guard([&] {
    PutTable(dest, distributed ? ops::DistributedUnion(GetTable(a), GetTable(b)) : ops::Union(GetTable(a), GetTable(b)));
  });
}

Status SortTable(const std::string &id, int col, const std::string &dest, bool asc) {
  return guard([&] { PutTable(dest, ops::Sort(GetTable(id), {col}, {asc})); });
}

int64_t RowCount(const std::string &id) { return GetTable(id)->Rows(); }
int32_t ColumnCount(const std::string &id) { return GetTable(id)->Columns(); }
std::vector<std::string> ColumnNames(const std::string &id) { return GetTable(id)->ColumnNames(); }

Status ReadCSV(const std::shared_ptr<CylonContext> &ctx, const std::string &path, const std::string &id,
               const io::CSVReadOptions &options) {
  return guard([&] { PutTable(id, io::ReadCSV(ctx, path, options)); });
}
Status ReadCSV(const std::shared_ptr<CylonContext> &ctx, const std::vector<std::string> &paths,
               const std::vector<std::string> &ids, const io::CSVReadOptions &options) {
  return guard([&] {
    CYLON_CHECK(paths.size() == ids.size(), Code::Invalid, paths.size() << " paths for " << ids.size() << " ids");
    auto ts = io::ReadCSVs(ctx, paths, options);
    for (size_t i = 0; i < ts.size(); ++i) PutTable(ids[i], ts[i]);
  });
}
Status WriteCSV(const std::string &id, const std::string &path, const io::CSVWriteOptions &options) {
  return guard([&] { io::WriteCSV(GetTable(id), path, options); });
}
Status ReadParquet(const std::shared_ptr<CylonContext> &ctx, const std::string &path, const std::string &id,
                   const io::ParquetOptions &options) {
  return guard([&] { PutTable(id, io::ReadParquet(ctx, path, options)); });
}
Status ReadParquet(const std::shared_ptr<CylonContext> &ctx, const std::vector<std::string> &paths,
                   const std::vector<std::string> &ids, const io::ParquetOptions &options) {
  return guard([&] {
    CYLON_CHECK(paths.size() == ids.size(), Code::Invalid, paths.size() << " paths for " << ids.size() << " ids");
    auto ts = io::ReadParquets(ctx, paths, options);
    for (size_t i = 0; i < ts.size(); ++i) PutTable(ids[i], ts[i]);
  });
}
Status WriteParquet(const std::string &id, const std::string &path, const io::ParquetOptions &options) {
  return guard([&] { io::WriteParquet(GetTable(id), path, options); });
}
Status SubtractTables(const std::string &a, const std::string &b, const std::string &dest, bool distributed) {
  return guard([&] {
    PutTable(dest, distributed ? ops::DistributedSubtract(GetTable(a), GetTable(b)) : ops::Subtract(GetTable(a), GetTable(b)));
  });
}
Status IntersectTables(const std::string &a, const std::string &b, const std::string &dest, bool distributed) {
  return guard([&] {
    PutTable(dest, distributed ? ops::DistributedIntersect(GetTable(a), GetTable(b))
                               : ops::Intersect(GetTable(a), GetTable(b)));
  });
}
Status MergeTables(const std::vector<std::string> &ids, const std::string &dest) {
  return guard([&] {
    std::vector<TablePtr> ts;
    for (const auto &id : ids) ts.push_back(GetTable(id));
    PutTable(dest, ops::Merge(ts));
  });
}
Status HashPartitionTable(const std::string &id, const std::vector<int> &hash_columns, int num_partitions,
                          std::unordered_map<int, std::string> *out) {
  return guard([&] {
    auto parts = ops::HashPartition(GetTable(id), hash_columns, (uint32_t)num_partitions);
    for (size_t p = 0; p < parts.size(); ++p) {
      const std::string pid = id + "_" + std::to_string(p);
      PutTable(pid, parts[p]);
      if (out) (*out)[(int)p] = pid;
    }
  });
}
Status SelectTable(const std::string &id, const std::function<bool(const Row &)> &selector, const std::string &dest) {
  TablePtr out;
  Status s = guard([&] { GetTable(id); });
  if (!s.is_ok()) return s;
  s = Select(GetTable(id), selector, out);
  if (s.is_ok()) PutTable(dest, out);
  return s;
}
Status ProjectTable(const std::string &id, const std::vector<int64_t> &columns, const std::string &dest) {
  return guard([&] {
    std::vector<int> cols(columns.begin(), columns.end());
    PutTable(dest, ops::Project(GetTable(id), cols));
  });
}
Status PrintToOStream(const TablePtr &t, int col1, int col2, int64_t row1, int64_t row2, std::ostream &out,
                      char delimiter, bool use_custom_header, const std::vector<std::string> &headers) {
  return guard([&] { io::PrintToOStream(t, col1, col2, row1, row2, out, delimiter, use_custom_header, headers); });
}
Status Print(const TablePtr &t, int col1, int col2, int64_t row1, int64_t row2) {
  return PrintToOStream(t, col1, col2, row1, row2, std::cout);
}
Status Print(const std::string &id, int col1, int col2, int64_t row1, int64_t row2) {
  return guard([&] { io::PrintToOStream(GetTable(id), col1, col2, row1, row2, std::cout); });
}
Status PrintToOStream(const std::string &id, int col1, int col2, int64_t row1, int64_t row2, std::ostream &out,
                      char delimiter, bool use_custom_header, const std::vector<std::string> &headers) {
  return guard([&] {
    io::PrintToOStream(GetTable(id), col1, col2, row1, row2, out, delimiter, use_custom_header, headers);
  });
}

// ---- TableAllToAll --------------------------------------------------------------------
TableAllToAll::TableAllToAll(std::shared_ptr<CylonContext> ctx, TableCallback callback)
    : ctx_(std::move(ctx)), cb_(std::move(callback)) {
  pending_.resize(ctx_->GetWorldSize());
  refs_.resize(ctx_->GetWorldSize());
}

int TableAllToAll::insert(const TablePtr &table, int32_t target, int32_t reference) {
  CYLON_CHECK(!finished_, Code::Invalid, "insert after finish()");
  CYLON_CHECK(target >= 0 && target < (int)pending_.size(), Code::IndexError, "target " << target);
  pending_[target].push_back(table);
  refs_[target].push_back(reference);
  return 1;
}

bool TableAllToAll::isComplete() {
  if (done_) return true;
  if (!finished_) return false;
  const int world = ctx_->GetWorldSize();
  auto comm = ctx_->GetCommunicator();
  TablePtr tmpl;
  for (auto &v : pending_)
    if (!v.empty()) tmpl = v[0];
  CYLON_CHECK(tmpl != nullptr, Code::Invalid, "TableAllToAll: nothing inserted on rank " << ctx_->GetRank());
  // metadata per target: [npieces, rows_0, ref_0, rows_1, ref_1, ...]
  std::vector<int64_t> meta, meta_counts(world), row_counts(world);
  std::vector<TablePtr> ordered;
  for (int t = 0; t < world; ++t) {
    meta.push_back((int64_t)pending_[t].size());
    int64_t rows = 0;
    for (size_t k = 0; k < pending_[t].size(); ++k) {
      meta.push_back(pending_[t][k]->Rows());
      meta.push_back(refs_[t][k]);
      rows += pending_[t][k]->Rows();
    }
    meta_counts[t] = 1 + 2 * (int64_t)pending_[t].size();
    row_counts[t] = rows;
    ordered.push_back(pending_[t].empty() ? ops::Slice(tmpl, 0, 0) : ops::Merge(pending_[t]));
  }
  TablePtr all = ops::Merge(ordered);
  at::Tensor meta_t = at::tensor(meta, at::TensorOptions().dtype(at::kLong));
  std::vector<int64_t> recv_meta_counts = comm->ExchangeCounts(meta_counts);
  at::Tensor recv_meta = world > 1 ? comm->AllToAllV(meta_t, meta_counts, recv_meta_counts).to(at::kCPU) : meta_t;
  TablePtr recv = ops::AllToAllTable(all, row_counts);
  // split the received table per source and per piece
  const int64_t *m = recv_meta.data_ptr<int64_t>();
  int64_t mi = 0, off = 0;
  for (int s = 0; s < world; ++s) {
    const int64_t np = m[mi++];
    for (int64_t k = 0; k < np; ++k) {
      const int64_t rows = m[mi++];
      const int ref = (int)m[mi++];
      cb_(s, ops::Slice(recv, off, rows), ref);
      off += rows;
    }
  }
  pending_.assign(world, {});
  refs_.assign(world, {});
  done_ = true;
  return true;
}

}  // namespace cylon
