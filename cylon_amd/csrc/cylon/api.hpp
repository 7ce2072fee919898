// Status-returning C++ API with the reference's shapes (L5).
//
// Reference: cpp/src/cylon/table.hpp:215-468 (free functions over
// shared_ptr<Table> with out-parameters), table_api.hpp:38-195 (string-ID
// registry used by the JNI layer), status.hpp, compute/aggregates.hpp,
// groupby/groupby.hpp, arrow/arrow_all_to_all.hpp (insert/finish/isComplete).
// Internally every call forwards to the throwing operators in cylon::ops and
// converts CylonError into a Status.
#pragma once
#include <chrono>
#include <thread>
#include <functional>
#include <map>
#include <memory>
#include <ostream>
#include <string>
#include <unordered_map>
#include <vector>

#include "io/arrow_io.hpp"
#include "io/csv.hpp"
#include "ops/relational.hpp"
#include "table.hpp"

namespace cylon {

class Status {
 public:
  Status() : code_(Code::OK) {}
  Status(int code, std::string msg) : code_(code), msg_(std::move(msg)) {}
  explicit Status(Code code) : code_(code) {}
  static Status OK() { return Status(); }
  int get_code() const { return code_; }
  bool is_ok() const { return code_ == Code::OK; }
  const std::string &get_msg() const { return msg_; }

 private:
  int code_;
  std::string msg_;
};

// ---- relational --------------------------------------------------------------
Status Join(const TablePtr &left, const TablePtr &right, const join::config::JoinConfig &cfg, TablePtr &out);
Status DistributedJoin(const TablePtr &left, const TablePtr &right, const join::config::JoinConfig &cfg,
                       TablePtr &out);
Status Union(const TablePtr &a, const TablePtr &b, TablePtr &out);
Status Subtract(const TablePtr &a, const TablePtr &b, TablePtr &out);
Status Intersect(const TablePtr &a, const TablePtr &b, TablePtr &out);
Status DistributedUnion(const TablePtr &a, const TablePtr &b, TablePtr &out);
Status DistributedSubtract(const TablePtr &a, const TablePtr &b, TablePtr &out);
Status DistributedIntersect(const TablePtr &a, const TablePtr &b, TablePtr &out);
Status Project(const TablePtr &t, const std::vector<int32_t> &cols, TablePtr &out);
Status Merge(const std::vector<TablePtr> &tables, TablePtr &out);
Status Sort(const TablePtr &t, int sort_column, TablePtr &out, bool ascending = true);
Status Sort(const TablePtr &t, const std::vector<int32_t> &cols, TablePtr &out, const std::vector<bool> &dirs);
Status DistributedSort(const TablePtr &t, const std::vector<int32_t> &cols, TablePtr &out,
                       const std::vector<bool> &dirs, SortOptions opts = SortOptions::Defaults());
Status Shuffle(const TablePtr &t, const std::vector<int> &hash_cols, TablePtr &out);
Status HashPartition(const TablePtr &t, const std::vector<int> &hash_cols, int num_partitions,
                     std::map<int, TablePtr> *out);
Status Unique(const TablePtr &t, const std::vector<int> &cols, TablePtr &out, bool first = true);
Status DistributedUnique(const TablePtr &t, const std::vector<int> &cols, TablePtr &out);

// ---- I/O (reference table.hpp FromCSV / WriteCSV / FromParquet / WriteParquet) --------
Status FromCSV(const std::shared_ptr<CylonContext> &ctx, const std::string &path, TablePtr &out,
               const io::CSVReadOptions &options = io::CSVReadOptions());
// several files concurrently (one thread per file); out[i] <- paths[i]
Status FromCSV(const std::shared_ptr<CylonContext> &ctx, const std::vector<std::string> &paths,
               std::vector<TablePtr> &out, const io::CSVReadOptions &options = io::CSVReadOptions());
Status WriteCSV(const TablePtr &t, const std::string &path,
                const io::CSVWriteOptions &options = io::CSVWriteOptions());
Status FromParquet(const std::shared_ptr<CylonContext> &ctx, const std::string &path, TablePtr &out,
                   const io::ParquetOptions &options = io::ParquetOptions());
Status FromParquet(const std::shared_ptr<CylonContext> &ctx, const std::vector<std::string> &paths,
                   std::vector<TablePtr> &out, const io::ParquetOptions &options = io::ParquetOptions());
Status WriteParquet(const TablePtr &t, const std::string &path,
                    const io::ParquetOptions &options = io::ParquetOptions());

// Row-predicate selection (reference table.cpp:504-529, row.hpp:23-52): the predicate
// sees a host Row view; accessors read the host buffers directly (no per-row allocation).
class Row {
 public:
  Row(const TablePtr &host_table, int64_t row) : t_(host_table), row_(row) {}
  void SetIndex(int64_t row) { row_ = row; }
  int64_t RowIndex() const { return row_; }
  bool IsNull(int col) const;
  int8_t GetInt8(int col) const { return (int8_t)GetInt64(col); }
  uint8_t GetUInt8(int col) const { return (uint8_t)GetUInt64(col); }
  int16_t GetInt16(int col) const { return (int16_t)GetInt64(col); }
  uint16_t GetUInt16(int col) const { return (uint16_t)GetUInt64(col); }
  int32_t GetInt32(int col) const { return (int32_t)GetInt64(col); }
  uint32_t GetUInt32(int col) const { return (uint32_t)GetUInt64(col); }
  int64_t GetInt64(int col) const;    // any integer / temporal type, sign-extended
  uint64_t GetUInt64(int col) const;  // any integer type, zero-extended
  float GetHalfFloat(int col) const { return (float)GetDouble(col); }
  float GetFloat(int col) const { return (float)GetDouble(col); }
  double GetDouble(int col) const;    // any numeric type
  bool GetBool(int col) const;
  std::string GetString(int col) const;
  const uint8_t *GetFixedBinary(int col) const;  // FIXED_SIZE_BINARY / DECIMAL bytes
  int32_t GetDate32(int col) const { return (int32_t)GetInt64(col); }
  int64_t GetDate64(int col) const { return GetInt64(col); }
  int64_t GetTimestamp(int col) const { return GetInt64(col); }
  int32_t Time32(int col) const { return (int32_t)GetInt64(col); }
  int64_t Time64(int col) const { return GetInt64(col); }
  const uint8_t *Decimal(int col) const { return GetFixedBinary(col); }

 private:
  const uint8_t *raw(int col, int *width) const;
  TablePtr t_;
  int64_t row_;
};
Status Select(const TablePtr &t, const std::function<bool(const Row &)> &predicate, TablePtr &out);

// ---- group-by / aggregates ------------------------------------------------------
Status DistributedHashGroupBy(const TablePtr &t, const std::vector<int32_t> &idx_cols,
                              const std::vector<int32_t> &aggregate_cols, const std::vector<AggOp> &ops,
                              TablePtr &out);
Status DistributedPipelineGroupBy(const TablePtr &t, int32_t idx_col, const std::vector<int32_t> &aggregate_cols,
                                  const std::vector<AggOp> &ops, TablePtr &out);
namespace compute {
Status Sum(const TablePtr &t, int32_t col, TablePtr &out);
Status Count(const TablePtr &t, int32_t col, TablePtr &out);
Status Min(const TablePtr &t, int32_t col, TablePtr &out);
Status Max(const TablePtr &t, int32_t col, TablePtr &out);
Status MinMax(const TablePtr &t, int32_t col, TablePtr &out);  // 1 row, columns min, max
}  // namespace compute

// ---- printing (reference table.hpp Print / PrintToOStream) -----------------------------
// columns [col1, col2) x rows [row1, row2) as delimited text; negative ends = to the last one
Status PrintToOStream(const TablePtr &t, int col1, int col2, int64_t row1, int64_t row2, std::ostream &out,
                      char delimiter = ',', bool use_custom_header = false,
                      const std::vector<std::string> &headers = {});
Status Print(const TablePtr &t, int col1 = 0, int col2 = -1, int64_t row1 = 0, int64_t row2 = -1);

// ---- string-ID table registry (reference table_api.cpp:34-61) --------------------
void PutTable(const std::string &id, const TablePtr &table);
TablePtr GetTable(const std::string &id);
void RemoveTable(const std::string &id);
std::vector<std::string> ListTables();
Status JoinTables(const std::string &left_id, const std::string &right_id, const join::config::JoinConfig &cfg,
                  const std::string &dest_id);
Status DistributedJoinTables(const std::string &left_id, const std::string &right_id,
                             const join::config::JoinConfig &cfg, const std::string &dest_id);
Status UnionTables(const std::string &a, const std::string &b, const std::string &dest, bool distributed);
Status SortTable(const std::string &id, int col, const std::string &dest, bool ascending);
int64_t RowCount(const std::string &id);
int32_t ColumnCount(const std::string &id);
std::vector<std::string> ColumnNames(const std::string &id);
// registry versions of the remaining table_api.hpp calls (reference table_api.hpp:40-195)
Status ReadCSV(const std::shared_ptr<CylonContext> &ctx, const std::string &path, const std::string &id,
               const io::CSVReadOptions &options = io::CSVReadOptions());
Status ReadCSV(const std::shared_ptr<CylonContext> &ctx, const std::vector<std::string> &paths,
               const std::vector<std::string> &ids, const io::CSVReadOptions &options = io::CSVReadOptions());
Status WriteCSV(const std::string &id, const std::string &path,
                const io::CSVWriteOptions &options = io::CSVWriteOptions());
Status ReadParquet(const std::shared_ptr<CylonContext> &ctx, const std::string &path, const std::string &id,
                   const io::ParquetOptions &options = io::ParquetOptions());
Status ReadParquet(const std::shared_ptr<CylonContext> &ctx, const std::vector<std::string> &paths,
                   const std::vector<std::string> &ids, const io::ParquetOptions &options = io::ParquetOptions());
Status WriteParquet(const std::string &id, const std::string &path,
                    const io::ParquetOptions &options = io::ParquetOptions());
Status SubtractTables(const std::string &a, const std::string &b, const std::string &dest, bool distributed);
Status IntersectTables(const std::string &a, const std::string &b, const std::string &dest, bool distributed);
Status MergeTables(const std::vector<std::string> &ids, const std::string &dest);
// partition p -> id "<id>_<p>" registered and returned in *out
Status HashPartitionTable(const std::string &id, const std::vector<int> &hash_columns, int num_partitions,
                          std::unordered_map<int, std::string> *out);
Status SelectTable(const std::string &id, const std::function<bool(const Row &)> &selector,
                   const std::string &dest);
Status ProjectTable(const std::string &id, const std::vector<int64_t> &columns, const std::string &dest);
Status Print(const std::string &id, int col1, int col2, int64_t row1, int64_t row2);
Status PrintToOStream(const std::string &id, int col1, int col2, int64_t row1, int64_t row2, std::ostream &out,
                      char delimiter = ',', bool use_custom_header = false,
                      const std::vector<std::string> &headers = {});

// ---- table all-to-all with the reference's insert/finish/isComplete protocol ----
// (arrow/arrow_all_to_all.hpp:101-253).  Tables inserted per target are batched;
// the exchange is one size exchange + per-buffer RCCL all-to-all issued by the
// first isComplete() after finish(); then the callback sees one table per source.
using TableCallback = std::function<bool(int source, const TablePtr &table, int reference)>;

class TableAllToAll {
 public:
  TableAllToAll(std::shared_ptr<CylonContext> ctx, TableCallback callback);
  int insert(const TablePtr &table, int32_t target, int32_t reference = 0);
  void finish() { finished_ = true; }
  bool isComplete();
  void close() {}

 private:
  std::shared_ptr<CylonContext> ctx_;
  TableCallback cb_;
  std::vector<std::vector<TablePtr>> pending_;
  std::vector<std::vector<int32_t>> refs_;  // per target, parallel to pending_
  bool finished_ = false;
  bool done_ = false;
};

// Task-level all-to-all (reference arrow_task_all_to_all.h:23-73): logical tasks
// mapped to workers; a task's table goes to the worker owning the target task.
struct LogicalTaskPlan {
  std::vector<int> task_to_worker;  // task id -> worker rank
};

class TaskAllToAll {
 public:
  TaskAllToAll(std::shared_ptr<CylonContext> ctx, LogicalTaskPlan plan, TableCallback callback)
      : plan_(std::move(plan)), inner_(std::move(ctx), std::move(callback)) {}
  int insert(const TablePtr &table, int target_task) {
    return inner_.insert(table, plan_.task_to_worker.at(target_task), target_task);
  }
  void finish() { inner_.finish(); }
  bool isComplete() { return inner_.isComplete(); }
  // Bounded wait (the reference busy-spins forever, arrow_task_all_to_all.cpp): a peer
  // that never delivers surfaces as ExecutionError after `timeout_s` seconds instead of
  // hanging the rank; polling backs off to 50 us sleeps after the first sweeps.
  void WaitForCompletion(double timeout_s = 600.0) {
    finish();
    const auto t0 = std::chrono::steady_clock::now();
    for (int64_t sweep = 0; !isComplete(); ++sweep) {
      const double el = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
      CYLON_CHECK(el < timeout_s, Code::ExecutionError,
                  "task all-to-all incomplete after " << timeout_s << " s (" << sweep << " progress sweeps)");
      if (sweep > 1024) std::this_thread::sleep_for(std::chrono::microseconds(50));
    }
  }

 private:
  LogicalTaskPlan plan_;
  TableAllToAll inner_;
};

}  // namespace cylon
