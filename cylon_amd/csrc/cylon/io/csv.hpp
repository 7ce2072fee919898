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
#include <unordered_map>
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
  bool include_missing_columns = false;      // absent include_columns -> all-null columns
  std::vector<std::string> null_values;      // empty -> Arrow's defaults
  std::vector<std::string> true_values{"1", "True", "TRUE", "true"};
  std::vector<std::string> false_values{"0", "False", "FALSE", "false"};
  bool strings_can_be_null = false;
  bool quoting = true;
  char quote_char = '"';
  bool double_quote = true;
  bool escaping = false;         // escape_char makes the next character literal
  char escape_char = '\\';
  bool newlines_in_values = false;  // quoted values may span lines (single-threaded line scan)
  std::unordered_map<std::string, DataType> column_types;  // overrides inference per column
  int threads = 0;               // 0 -> hardware concurrency (capped at 16)
  bool use_threads = true;       // false -> one parser thread
  bool concurrent_file_reads = true;  // ReadCSVs: one thread per file
  int32_t block_size = 1 << 20;  // minimum bytes per parser thread

  // Builder form of the reference's CSVReadOptions (csv_read_config.hpp:27-150).
  CSVReadOptions &ConcurrentFileReads(bool v) { concurrent_file_reads = v; return *this; }
  bool IsConcurrentFileReads() const { return concurrent_file_reads; }
  CSVReadOptions &UseThreads(bool v) { use_threads = v; return *this; }
  CSVReadOptions &WithDelimiter(char d) { delimiter = d; return *this; }
  CSVReadOptions &IgnoreEmptyLines() { ignore_empty_lines = true; return *this; }
  CSVReadOptions &AutoGenerateColumnNames() { autogenerate_column_names = true; return *this; }
  CSVReadOptions &ColumnNames(const std::vector<std::string> &names) { column_names = names; return *this; }
  CSVReadOptions &BlockSize(int32_t b) { block_size = b; return *this; }
  CSVReadOptions &UseQuoting() { quoting = true; return *this; }
  CSVReadOptions &WithQuoteChar(char q) { quote_char = q; quoting = true; return *this; }
  CSVReadOptions &DoubleQuote() { double_quote = true; return *this; }
  CSVReadOptions &UseEscaping() { escaping = true; return *this; }
  CSVReadOptions &EscapingCharacter(char c) { escape_char = c; escaping = true; return *this; }
  CSVReadOptions &HasNewLinesInValues() { newlines_in_values = true; return *this; }
  CSVReadOptions &SkipRows(int32_t n) { skip_rows = n; return *this; }
  CSVReadOptions &WithColumnTypes(const std::unordered_map<std::string, DataType> &t) {
    column_types = t;
    return *this;
  }
  CSVReadOptions &NullValues(const std::vector<std::string> &v) { null_values = v; return *this; }
  CSVReadOptions &TrueValues(const std::vector<std::string> &v) { true_values = v; return *this; }
  CSVReadOptions &FalseValues(const std::vector<std::string> &v) { false_values = v; return *this; }
  CSVReadOptions &StringsCanBeNull() { strings_can_be_null = true; return *this; }
  CSVReadOptions &IncludeColumns(const std::vector<std::string> &c) { include_columns = c; return *this; }
  CSVReadOptions &IncludeMissingColumns() { include_missing_columns = true; return *this; }
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
