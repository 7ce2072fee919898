// Native Arrow C++ bridge and Parquet I/O (C25 Parquet, C26 Arrow<->Cylon).
//
// Reference: cpp/src/cylon/io/arrow_io.cpp (readers), parquet_config.hpp:24-53
// (ParquetOptions: concurrent file reads, chunk size, writer properties),
// table.cpp:205-242 (FromParquet, one thread per file) and :1117-1126
// (WriteParquet), arrow/arrow_types.cpp (Arrow <-> Cylon type mapping).
//
// The engine links the Arrow / Parquet C++ libraries that ship with pyarrow
// (same image on every box).  Arrow tables are host-resident: conversion copies
// each buffer once to the context's device (fixed-width values as-is, Arrow
// validity bitmaps expanded to byte masks, 32-bit string offsets widened to the
// engine's 64-bit ones) and back for writing.
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "../table.hpp"

namespace arrow {
class Table;
}

namespace cylon {
namespace io {

struct ParquetOptions {
  bool concurrent_file_reads = true;  // one thread per file in ReadParquets
  int64_t chunk_size = 1 << 20;       // rows per row group when writing
  std::string compression = "snappy"; // snappy | zstd | gzip | lz4 | brotli | none
  std::vector<std::string> columns;   // read: subset / order (empty = all)
  bool use_threads = true;            // Arrow's column-parallel decoding
};

// Arrow C++ table <-> engine table (device = the context's device)
TablePtr FromArrowTable(const std::shared_ptr<CylonContext> &ctx, const std::shared_ptr<arrow::Table> &table);
std::shared_ptr<arrow::Table> ToArrowTable(const TablePtr &table);

TablePtr ReadParquet(const std::shared_ptr<CylonContext> &ctx, const std::string &path, const ParquetOptions &opts);
std::vector<TablePtr> ReadParquets(const std::shared_ptr<CylonContext> &ctx, const std::vector<std::string> &paths,
                                   const ParquetOptions &opts);
void WriteParquet(const TablePtr &table, const std::string &path, const ParquetOptions &opts);

}  // namespace io
}  // namespace cylon
