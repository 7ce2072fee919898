// Native CSV reader / writer (C25).
//
// Reference: cpp/src/cylon/io/arrow_io.cpp:33-61 (mmap + arrow::csv::TableReader),
// csv_read_config.hpp:27-150 (options), csv_write_config.hpp:24-48,
// table.cpp:181-200 (FromCSV), 244-253 (WriteCSV), 791-829 (one thread per file).
//
// Host-side parser: the file is memory-mapped, split into line-aligned chunks
// parsed by a thread pool in two passes (type inference, then conversion into
// the final column buffers at prefix-summed row offsets); the resulting
// columns are moved to the context's device in one copy per buffer.  Types
// are inferred like Arrow's CSV reader for the common cases: int64, then
// boolean (true/false spellings), then double, else string; the default null
// spellings follow Arrow's and string columns are never null unless
// strings_can_be_null is set.
#pragma once
#include <ostream>
#include <string>
#include <vector>

#include "../table.hpp"

namespace cylon {
namespace io {

struct CSVReadOptions {
  char delimiter = ',';
  bool header = true;                     // first (non-skipped) row holds column names
  bool autogenerate_column_names = false; // f0, f1, ... (implies no header row)
  std::vector<std::string> column_names;  // explicit names (implies no header row)
  int64_t skip_rows = 0;
  bool ignore_empty_lines = true;
  std::vector<std::string> include_columns;  // subset / order of columns to keep
  std::vector<std::string> null_values;      // empty -> Arrow's defaults
  std::vector<std::string> true_values{"1", "True", "TRUE", "true"};
  std::vector<std::string> false_values{"0", "False", "FALSE", "false"};
  bool strings_can_be_null = false;
  bool quoting = true;
  char quote_char = '"';
  bool double_quote = true;
  int threads = 0;  // 0 -> hardware concurrency (capped at 16)
};

struct CSVWriteOptions {
  char delimiter = ',';
  std::vector<std::string> column_names;  // header override
};

TablePtr ReadCSV(const std::shared_ptr<CylonContext> &ctx, const std::string &path, const CSVReadOptions &opts);
// several files concurrently, one thread per file (reference table.cpp:799-829)
std::vector<TablePtr> ReadCSVs(const std::shared_ptr<CylonContext> &ctx, const std::vector<std::string> &paths,
                               const CSVReadOptions &opts);
void WriteCSV(const TablePtr &table, const std::string &path, const CSVWriteOptions &opts);
// columns [col1, col2) x rows [row1, row2) as CSV text (negative ends = to the last one);
// reference table.hpp PrintToOStream / Print
void PrintToOStream(const TablePtr &table, int col1, int col2, int64_t row1, int64_t row2, std::ostream &out,
                    char delimiter = ',', bool use_custom_header = false,
                    const std::vector<std::string> &headers = {});

}  // namespace io
}  // namespace cylon
