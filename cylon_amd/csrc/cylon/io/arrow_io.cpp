// Native Arrow C++ bridge and Parquet I/O (see arrow_io.hpp).
#include "arrow_io.hpp"

#include <algorithm>
#include <functional>

#include <arrow/api.h>
#include <arrow/io/file.h>
#include <parquet/arrow/reader.h>
#include <parquet/arrow/writer.h>
#include <parquet/properties.h>

#include <cstring>
#include <thread>

namespace cylon {
namespace io {

namespace {

template <typename T>
T ok_or_throw(arrow::Result<T> r, const char *what) {
  CYLON_CHECK(r.ok(), Code::IOError, what << ": " << r.status().ToString());
  return std::move(r).ValueOrDie();
}

void check(const arrow::Status &s, const char *what) {
  CYLON_CHECK(s.ok(), Code::IOError, what << ": " << s.ToString());
}

TimeUnit unit_of(arrow::TimeUnit::type u) {
  switch (u) {
    case arrow::TimeUnit::SECOND: return TimeUnit::SECOND;
    case arrow::TimeUnit::MILLI: return TimeUnit::MILLI;
    case arrow::TimeUnit::MICRO: return TimeUnit::MICRO;
    default: return TimeUnit::NANO;
  }
}

arrow::TimeUnit::type arrow_unit(TimeUnit u) {
  switch (u) {
    case TimeUnit::SECOND: return arrow::TimeUnit::SECOND;
    case TimeUnit::MILLI: return arrow::TimeUnit::MILLI;
    case TimeUnit::MICRO: return arrow::TimeUnit::MICRO;
    default: return arrow::TimeUnit::NANO;
  }
}

// Arrow type -> engine type (reference arrow/arrow_types.cpp validateArrowTableTypes allowlist)
DataType to_cylon(const arrow::DataType &t) {
  using arrow::Type;
  switch (t.id()) {
    case Type::BOOL: return DataType(cylon::Type::BOOL);
    case Type::UINT8: return DataType(cylon::Type::UINT8);
    case Type::INT8: return DataType(cylon::Type::INT8);
    case Type::UINT16: return DataType(cylon::Type::UINT16);
    case Type::INT16: return DataType(cylon::Type::INT16);
    case Type::UINT32: return DataType(cylon::Type::UINT32);
    case Type::INT32: return DataType(cylon::Type::INT32);
    case Type::UINT64: return DataType(cylon::Type::UINT64);
    case Type::INT64: return DataType(cylon::Type::INT64);
    case Type::HALF_FLOAT: return DataType(cylon::Type::HALF_FLOAT);
    case Type::FLOAT: return DataType(cylon::Type::FLOAT);
    case Type::DOUBLE: return DataType(cylon::Type::DOUBLE);
    case Type::STRING:
    case Type::LARGE_STRING: return DataType(cylon::Type::STRING);
    case Type::BINARY:
    case Type::LARGE_BINARY: return DataType(cylon::Type::BINARY);
    case Type::FIXED_SIZE_BINARY:
      return DataType::FixedSizeBinary(static_cast<const arrow::FixedSizeBinaryType &>(t).byte_width());
    case Type::DECIMAL128:
    case Type::DECIMAL256: {
      const auto &dt = static_cast<const arrow::DecimalType &>(t);
      DataType d(cylon::Type::DECIMAL, dt.byte_width());
      d.precision = dt.precision();
      d.scale = dt.scale();
      return d;
    }
    case Type::DATE32: return DataType(cylon::Type::DATE32);
    case Type::DATE64: return DataType(cylon::Type::DATE64);
    case Type::TIMESTAMP: {
      const auto &ts = static_cast<const arrow::TimestampType &>(t);
      return DataType::Timestamp(unit_of(ts.unit()), ts.timezone());
    }
    case Type::TIME32: {
      DataType d(cylon::Type::TIME32);
      d.unit = unit_of(static_cast<const arrow::Time32Type &>(t).unit());
      return d;
    }
    case Type::TIME64: {
      DataType d(cylon::Type::TIME64);
      d.unit = unit_of(static_cast<const arrow::Time64Type &>(t).unit());
      return d;
    }
    case Type::DURATION: {
      DataType d(cylon::Type::DURATION);
      d.unit = unit_of(static_cast<const arrow::DurationType &>(t).unit());
      return d;
    }
    case Type::LIST:
    case Type::LARGE_LIST:
      return DataType::List(to_cylon(*static_cast<const arrow::BaseListType &>(t).value_type()).type);
    case Type::FIXED_SIZE_LIST: {
      const auto &fl = static_cast<const arrow::FixedSizeListType &>(t);
      return DataType::FixedSizeList(to_cylon(*fl.value_type()).type, fl.list_size());
    }
    default: CYLON_THROW(Code::NotImplemented, "arrow type " << t.ToString() << " is not supported");
  }
}

std::shared_ptr<arrow::DataType> to_arrow(const DataType &t, bool large_var) {
  switch (t.type) {
    case cylon::Type::BOOL: return arrow::boolean();
    case cylon::Type::UINT8: return arrow::uint8();
    case cylon::Type::INT8: return arrow::int8();
    case cylon::Type::UINT16: return arrow::uint16();
    case cylon::Type::INT16: return arrow::int16();
    case cylon::Type::UINT32: return arrow::uint32();
    case cylon::Type::INT32: return arrow::int32();
    case cylon::Type::UINT64: return arrow::uint64();
    case cylon::Type::INT64: return arrow::int64();
    case cylon::Type::HALF_FLOAT: return arrow::float16();
    case cylon::Type::FLOAT: return arrow::float32();
    case cylon::Type::DOUBLE: return arrow::float64();
    case cylon::Type::STRING: return large_var ? arrow::large_utf8() : arrow::utf8();
    case cylon::Type::BINARY: return large_var ? arrow::large_binary() : arrow::binary();
    case cylon::Type::FIXED_SIZE_BINARY: return arrow::fixed_size_binary(t.byte_width);
    case cylon::Type::DATE32: return arrow::date32();
    case cylon::Type::DATE64: return arrow::date64();
    case cylon::Type::TIMESTAMP: return arrow::timestamp(arrow_unit(t.unit), t.timezone);
    case cylon::Type::TIME32: return arrow::time32(arrow_unit(t.unit));
    case cylon::Type::TIME64: return arrow::time64(arrow_unit(t.unit));
    case cylon::Type::DURATION: return arrow::duration(arrow_unit(t.unit));
    case cylon::Type::DECIMAL:
      if (t.byte_width == 32) return arrow::decimal256(t.precision ? t.precision : 76, t.scale);
      return arrow::decimal128(t.precision ? t.precision : 38, t.scale);
    case cylon::Type::LIST:
      return large_var ? arrow::large_list(to_arrow(DataType(t.value_type), false))
                       : arrow::list(to_arrow(DataType(t.value_type), false));
    case cylon::Type::FIXED_SIZE_LIST: return arrow::fixed_size_list(to_arrow(DataType(t.value_type), false), t.list_size);
    default: CYLON_THROW(Code::NotImplemented, "type " << static_cast<int>(t.type) << " has no Arrow mapping");
  }
}

at::Tensor host_bytes(int64_t n) { return at::empty({n}, at::TensorOptions().dtype(at::kByte)); }

// Arrow validity bitmap (with the array's bit offset) -> byte mask; undefined if no nulls
at::Tensor validity_bytes(const arrow::ArrayData &d) {
  if (d.GetNullCount() == 0 || d.buffers.empty() || !d.buffers[0]) return at::Tensor();
  at::Tensor v = host_bytes(d.length);
  uint8_t *o = v.data_ptr<uint8_t>();
  const uint8_t *bits = d.buffers[0]->data();
  for (int64_t i = 0; i < d.length; ++i) o[i] = arrow::bit_util::GetBit(bits, d.offset + i) ? 1 : 0;
  return v;
}

// element nulls are only representable under null rows (their bytes are never read)
void check_list_children(const arrow::ArrayData &d, const arrow::ArrayData &child, int64_t first, int64_t count,
                         const std::function<int64_t(int64_t)> &row_of, const std::string &name) {
  if (child.GetNullCount() == 0 || !child.buffers[0]) return;
  const uint8_t *cb = child.buffers[0]->data();
  const uint8_t *pb = d.buffers[0] ? d.buffers[0]->data() : nullptr;
  for (int64_t e = 0; e < count; ++e)
    if (!arrow::bit_util::GetBit(cb, child.offset + first + e)) {
      const int64_t r = row_of(e);
      CYLON_CHECK(pb && !arrow::bit_util::GetBit(pb, d.offset + r), Code::NotImplemented,
                  "column " << name << ": null list elements are not supported");
    }
}

Column list_column_from_array(const std::string &name, const arrow::ArrayData &d, const DataType &t,
                              at::Tensor valid, const at::Device &dev) {
  const int64_t n = d.length, w = t.value_width();
  const arrow::ArrayData &child = *d.child_data[0];
  if (t.type == cylon::Type::FIXED_SIZE_LIST) {
    const int64_t k = t.list_size;
    check_list_children(d, child, d.offset * k, n * k, [k](int64_t e) { return e / k; }, name);
    at::Tensor bytes = host_bytes(n * k * w);
    if (n * k) std::memcpy(bytes.data_ptr<uint8_t>(), child.buffers[1]->data() + (child.offset + d.offset * k) * w, n * k * w);
    return Column(name, t, n, bytes.to(dev), at::Tensor(), valid.defined() ? valid.to(dev) : valid);
  }
  const bool large = d.type->id() == arrow::Type::LARGE_LIST;
  at::Tensor offs = at::empty({n + 1}, at::TensorOptions().dtype(at::kLong));
  int64_t *o = offs.data_ptr<int64_t>();
  for (int64_t i = 0; i <= n; ++i) o[i] = large ? d.GetValues<int64_t>(1)[i] : (int64_t)d.GetValues<int32_t>(1)[i];
  const int64_t first = o[0], last = o[n];
  check_list_children(d, child, first, last - first, [o, n](int64_t e) {
    return (int64_t)(std::upper_bound(o, o + n + 1, o[0] + e) - o) - 1;
  }, name);
  for (int64_t i = 0; i <= n; ++i) o[i] = (o[i] - first) * w;  // element offsets -> byte offsets
  at::Tensor bytes = host_bytes((last - first) * w);
  if (last > first) std::memcpy(bytes.data_ptr<uint8_t>(), child.buffers[1]->data() + (child.offset + first) * w, (last - first) * w);
  return Column(name, t, n, bytes.to(dev), offs.to(dev), valid.defined() ? valid.to(dev) : valid);
}

Column column_from_array(const std::string &name, const arrow::Array &arr, const at::Device &dev) {
  const arrow::ArrayData &d = *arr.data();
  const DataType t = to_cylon(*arr.type());
  const int64_t n = d.length;
  at::Tensor valid = validity_bytes(d);
  if (t.is_list()) return list_column_from_array(name, d, t, valid, dev);
  if (t.is_variable_width()) {
    const bool large = arr.type_id() == arrow::Type::LARGE_STRING || arr.type_id() == arrow::Type::LARGE_BINARY;
    at::Tensor offs = at::empty({n + 1}, at::TensorOptions().dtype(at::kLong));
    int64_t *o = offs.data_ptr<int64_t>();
    int64_t first = 0, last = 0;
    if (large) {
      const int64_t *src = d.GetValues<int64_t>(1);
      first = src[0];
      for (int64_t i = 0; i <= n; ++i) o[i] = src[i] - first;
      last = src[n];
    } else {
      const int32_t *src = d.GetValues<int32_t>(1);
      first = src[0];
      for (int64_t i = 0; i <= n; ++i) o[i] = (int64_t)src[i] - first;
      last = src[n];
    }
    at::Tensor bytes = host_bytes(last - first);
    if (last > first) std::memcpy(bytes.data_ptr<uint8_t>(), d.buffers[2]->data() + first, last - first);
    return Column(name, t, n, bytes.to(dev), offs.to(dev), valid.defined() ? valid.to(dev) : valid);
  }
  Column c = make_fixed_column(name, t, n, at::Device(at::kCPU), false);
  if (t.type == cylon::Type::BOOL) {  // bit-packed values -> bytes
    uint8_t *o = reinterpret_cast<uint8_t *>(c.data.data_ptr());
    const uint8_t *bits = d.buffers[1]->data();
    for (int64_t i = 0; i < n; ++i) o[i] = arrow::bit_util::GetBit(bits, d.offset + i) ? 1 : 0;
  } else if (n > 0) {
    const int w = t.width();
    std::memcpy(c.data.data_ptr(), d.buffers[1]->data() + d.offset * (int64_t)w, (size_t)n * w);
  }
  return Column(name, t, n, c.data.to(dev), at::Tensor(), valid.defined() ? valid.to(dev) : valid);
}

std::shared_ptr<arrow::Buffer> to_buffer(const at::Tensor &host) {
  const int64_t nb = host.numel() * host.element_size();
  auto buf = ok_or_throw(arrow::AllocateBuffer(nb), "arrow buffer");
  if (nb) std::memcpy(buf->mutable_data(), host.data_ptr(), nb);
  return std::shared_ptr<arrow::Buffer>(std::move(buf));
}

std::shared_ptr<arrow::Buffer> pack_bits(const uint8_t *bytes, int64_t n, int64_t *nulls) {
  auto buf = ok_or_throw(arrow::AllocateBitmap(n), "arrow bitmap");
  uint8_t *bits = buf->mutable_data();
  std::memset(bits, 0, arrow::bit_util::BytesForBits(n));
  int64_t z = 0;
  for (int64_t i = 0; i < n; ++i) {
    if (bytes[i]) arrow::bit_util::SetBit(bits, i);
    else ++z;
  }
  if (nulls) *nulls = z;
  return std::shared_ptr<arrow::Buffer>(std::move(buf));
}

std::shared_ptr<arrow::Array> array_from_column(const Column &col) {
  const int64_t n = col.length;
  int64_t nulls = 0;
  std::shared_ptr<arrow::Buffer> validity;
  if (col.nullable()) {
    at::Tensor v = col.validity.to(at::kCPU).contiguous();
    validity = pack_bits(v.data_ptr<uint8_t>(), n, &nulls);
    if (nulls == 0) validity = nullptr;
  }
  if (col.type.is_list()) {  // child values (numeric) + element offsets / fixed rows
    const int64_t w = col.type.value_width();
    auto elem = to_arrow(DataType(col.type.value_type), false);
    at::Tensor bytes = col.data.to(at::kCPU).contiguous();
    if (col.type.type == cylon::Type::FIXED_SIZE_LIST) {
      const int64_t k = col.type.list_size;
      auto child = arrow::ArrayData::Make(elem, n * k, {nullptr, to_buffer(bytes.slice(0, 0, n * k * w).contiguous())}, 0);
      return arrow::MakeArray(arrow::ArrayData::Make(to_arrow(col.type, false), n, {validity}, {child}, nulls));
    }
    at::Tensor o = col.offsets.to(at::kCPU).contiguous();
    const int64_t base = o[0].item<int64_t>(), total = o[n].item<int64_t>() - base;
    const bool large = total / w > (int64_t)INT32_MAX;
    at::Tensor eo = (o - base).div(w, "trunc");
    std::shared_ptr<arrow::Buffer> obuf = large ? to_buffer(eo.contiguous()) : to_buffer(eo.to(at::kInt).contiguous());
    auto child = arrow::ArrayData::Make(elem, total / w, {nullptr, to_buffer(bytes.slice(0, base, base + total).contiguous())}, 0);
    return arrow::MakeArray(arrow::ArrayData::Make(to_arrow(col.type, large), n, {validity, obuf}, {child}, nulls));
  }
  if (col.is_var()) {
    at::Tensor o = col.offsets.to(at::kCPU).contiguous();
    const int64_t *off = o.data_ptr<int64_t>();
    const int64_t base = off[0], total = off[n] - off[0];
    const bool large = total > (int64_t)INT32_MAX;
    std::shared_ptr<arrow::Buffer> obuf;
    if (large) {
      at::Tensor lo = o - base;
      obuf = to_buffer(lo);
    } else {
      at::Tensor so = (o - base).to(at::kInt);
      obuf = to_buffer(so);
    }
    at::Tensor bytes = col.data.to(at::kCPU).contiguous().slice(0, base, base + total);
    auto data = arrow::ArrayData::Make(to_arrow(col.type, large), n, {validity, obuf, to_buffer(bytes.contiguous())},
                                       nulls);
    return arrow::MakeArray(data);
  }
  at::Tensor host = col.data.to(at::kCPU).contiguous();
  std::shared_ptr<arrow::Buffer> values;
  if (col.type.type == cylon::Type::BOOL) {
    at::Tensor b = host.to(at::kByte);
    values = pack_bits(b.data_ptr<uint8_t>(), n, nullptr);
  } else {
    values = to_buffer(host);
  }
  auto data = arrow::ArrayData::Make(to_arrow(col.type, false), n, {validity, values}, nulls);
  return arrow::MakeArray(data);
}

arrow::Compression::type compression_of(const std::string &c) {
  if (c == "snappy") return arrow::Compression::SNAPPY;
  if (c == "zstd") return arrow::Compression::ZSTD;
  if (c == "gzip") return arrow::Compression::GZIP;
  if (c == "lz4") return arrow::Compression::LZ4;
  if (c == "brotli") return arrow::Compression::BROTLI;
  if (c == "none" || c == "uncompressed" || c.empty()) return arrow::Compression::UNCOMPRESSED;
  CYLON_THROW(Code::Invalid, "unknown parquet compression " << c);
}

}  // namespace

TablePtr FromArrowTable(const std::shared_ptr<CylonContext> &ctx, const std::shared_ptr<arrow::Table> &table) {
  auto combined = ok_or_throw(table->CombineChunks(), "combine chunks");
  const at::Device dev(ctx->GetDevice());
  std::vector<Column> cols;
  for (int i = 0; i < combined->num_columns(); ++i) {
    const auto &chunked = combined->column(i);
    std::shared_ptr<arrow::Array> arr;
    if (chunked->num_chunks() == 1) arr = chunked->chunk(0);
    else arr = ok_or_throw(arrow::MakeArrayOfNull(chunked->type(), 0), "empty column");
    cols.push_back(column_from_array(combined->field(i)->name(), *arr, dev));
  }
  return Table::Make(ctx, std::move(cols));
}

std::shared_ptr<arrow::Table> ToArrowTable(const TablePtr &table) {
  std::vector<std::shared_ptr<arrow::Field>> fields;
  std::vector<std::shared_ptr<arrow::Array>> arrays;
  for (const auto &c : table->columns()) {
    arrays.push_back(array_from_column(c));
    fields.push_back(arrow::field(c.name, arrays.back()->type(), true));
  }
  return arrow::Table::Make(arrow::schema(fields), arrays, table->Rows());
}

TablePtr ReadParquet(const std::shared_ptr<CylonContext> &ctx, const std::string &path, const ParquetOptions &opts) {
  auto file = ok_or_throw(arrow::io::ReadableFile::Open(path), "open parquet file");
  auto reader = ok_or_throw(parquet::arrow::OpenFile(file, arrow::default_memory_pool()), "parquet reader");
  reader->set_use_threads(opts.use_threads);
  std::shared_ptr<arrow::Table> t;
  if (opts.columns.empty()) {
    t = ok_or_throw(reader->ReadTable(), "read parquet");
  } else {
    std::shared_ptr<arrow::Schema> schema;
    check(reader->GetSchema(&schema), "parquet schema");
    std::vector<int> idx;
    for (const auto &name : opts.columns) {
      const int i = schema->GetFieldIndex(name);
      CYLON_CHECK(i >= 0, Code::KeyError, "parquet file " << path << " has no column " << name);
      idx.push_back(i);
    }
    t = ok_or_throw(reader->ReadTable(idx), "read parquet");
  }
  return FromArrowTable(ctx, t);
}

std::vector<TablePtr> ReadParquets(const std::shared_ptr<CylonContext> &ctx, const std::vector<std::string> &paths,
                                   const ParquetOptions &opts) {
  std::vector<TablePtr> out(paths.size());
  if (!opts.concurrent_file_reads || paths.size() < 2) {
    for (size_t i = 0; i < paths.size(); ++i) out[i] = ReadParquet(ctx, paths[i], opts);
    return out;
  }
  std::vector<std::exception_ptr> errs(paths.size());
  std::vector<std::thread> th;
  for (size_t i = 0; i < paths.size(); ++i)
    th.emplace_back([&, i] {
      try {
        out[i] = ReadParquet(ctx, paths[i], opts);
      } catch (...) {
        errs[i] = std::current_exception();
      }
    });
  for (auto &t : th) t.join();
  for (auto &e : errs)
    if (e) std::rethrow_exception(e);
  return out;
}

void WriteParquet(const TablePtr &table, const std::string &path, const ParquetOptions &opts) {
  auto t = ToArrowTable(table);
  auto out = ok_or_throw(arrow::io::FileOutputStream::Open(path), "open parquet output");
  auto props = parquet::WriterProperties::Builder().compression(compression_of(opts.compression))->build();
  // store the Arrow schema too (types Parquet has no logical type for, e.g. duration, round-trip)
  auto arrow_props = parquet::ArrowWriterProperties::Builder().store_schema()->build();
  check(parquet::arrow::WriteTable(*t, arrow::default_memory_pool(), out, std::max<int64_t>(1, opts.chunk_size), props,
                                   arrow_props),
        "write parquet");
  check(out->Close(), "close parquet output");
}

}  // namespace io
}  // namespace cylon
