// String-ID table API example (reference: cpp/src/cylon/table_api.hpp, used by the Java
// binding; cpp/src/examples/select_example.cpp, project_example.cpp, partition_example.cpp).
//   usage: registry_example <device> <csv1> <csv2> <out_dir>
// Prints "name value" lines: row counts of every derived table, a selected row's typed
// fields, and the first rows of the join as CSV text (PrintToOStream).
#include <cstdio>
#include <sstream>
#include <unordered_map>

#include "cylon/api.hpp"

namespace jc = cylon::join::config;

#define CHECK_OK(expr)                                                        \
  do {                                                                        \
    cylon::Status _s = (expr);                                                \
    if (!_s.is_ok()) {                                                        \
      std::fprintf(stderr, "%s failed: %s\n", #expr, _s.get_msg().c_str());  \
      return 1;                                                               \
    }                                                                         \
  } while (0)

int main(int argc, char **argv) {
  if (argc < 5) return 2;
  auto ctx = cylon::CylonContext::Init(at::Device(std::string(argv[1])));
  const std::string out = argv[4];
  CHECK_OK(cylon::ReadCSV(ctx, std::vector<std::string>{argv[2], argv[3]}, {"a", "b"}));
  CHECK_OK(cylon::JoinTables("a", "b", jc::JoinConfig::InnerJoin(0, 0, jc::HASH, "l_", "r_"), "j"));
  CHECK_OK(cylon::SubtractTables("a", "b", "s", false));
  CHECK_OK(cylon::IntersectTables("a", "b", "i", false));
  CHECK_OK(cylon::MergeTables({"a", "b"}, "m"));
  CHECK_OK(cylon::ProjectTable("j", {0, 1}, "p"));
  // rows whose first column is even
  CHECK_OK(cylon::SelectTable("a", [](const cylon::Row &r) { return r.GetInt64(0) % 2 == 0; }, "sel"));
  std::unordered_map<int, std::string> parts;
  CHECK_OK(cylon::HashPartitionTable("a", {0}, 3, &parts));
  int64_t part_rows = 0;
  for (auto &kv : parts) part_rows += cylon::RowCount(kv.second);
  for (const char *id : {"a", "b", "j", "s", "i", "m", "p", "sel"})
    std::printf("%s %lld\n", id, static_cast<long long>(cylon::RowCount(id)));
  std::printf("partitions %zu\npartition_rows %lld\n", parts.size(), static_cast<long long>(part_rows));
  std::printf("p_columns %zu\n", cylon::ColumnNames("p").size());
  // typed accessors on the first selected row (host view)
  cylon::TablePtr sel = cylon::GetTable("sel");
  if (sel->Rows() > 0) {
    cylon::TablePtr host = sel->to(at::Device(at::kCPU));
    cylon::Row row(host, 0);
    std::printf("sel_first_even %d\n", static_cast<int>(row.GetInt64(0) % 2 == 0));
  }
  std::ostringstream text;
  CHECK_OK(cylon::PrintToOStream("j", 0, -1, 0, 3, text));
  int lines = 0;
  for (char c : text.str()) lines += c == '\n';
  std::printf("printed_lines %d\n", lines);
  CHECK_OK(cylon::WriteParquet("j", out + "/j.parquet"));
  CHECK_OK(cylon::ReadParquet(ctx, out + "/j.parquet", "j2"));
  std::printf("j2 %lld\n", static_cast<long long>(cylon::RowCount("j2")));
  return 0;
}
