// Logical data types of the engine.
//
// The Type enum keeps the reference's numbering (cpp/src/cylon/data_types.hpp:26-100)
// so that code written against the reference's Type/Layout constants keeps its
// meaning.  Physical storage is device-resident and Arrow-like:
//   * fixed width  -> one contiguous buffer of n * byte_width bytes
//   * STRING/BINARY -> int64 offsets[n+1] + uint8 bytes   (always 64-bit offsets)
//   * LIST<numeric> -> the same var-width layout: int64 BYTE offsets[n+1] + the child
//                      values' bytes (Arrow's element offsets x element width), so every
//                      gather / shuffle / join materialisation path moves lists as it
//                      moves binary values (reference: arrow_types.cpp:83-111 accepts
//                      list<numeric>, copy_arrray.cpp:113-139,222-281 gathers it)
//   * FIXED_SIZE_LIST<numeric, k> -> fixed width k x element width bytes per row
//   * validity      -> optional uint8 byte-mask (1 = valid)
// Byte masks instead of bit-packed validity keep the scatter/gather kernels
// free of read-modify-write bit updates; Arrow bitmaps are produced at the
// host boundary (Table.to_arrow).
#pragma once
#include "common.hpp"

namespace cylon {

enum class Type : int {
  BOOL = 0,
  UINT8,
  INT8,
  UINT16,
  INT16,
  UINT32,
  INT32,
  UINT64,
  INT64,
  HALF_FLOAT,
  FLOAT,
  DOUBLE,
  STRING,
  BINARY,
  FIXED_SIZE_BINARY,
  DATE32,
  DATE64,
  TIMESTAMP,
  TIME32,
  TIME64,
  INTERVAL,
  DECIMAL,
  LIST,
  EXTENSION,
  FIXED_SIZE_LIST,
  DURATION,
};

enum class Layout : int { FIXED_WIDTH = 1, VARIABLE_WIDTH = 2 };

enum class TimeUnit : int { SECOND = 0, MILLI = 1, MICRO = 2, NANO = 3 };

// Kernel-level classification of a value for hashing / comparison.
enum class ValueKind : int {
  SIGNED_INT = 0,    // two's complement integer (also temporal types)
  UNSIGNED_INT = 1,  // unsigned integer and bool
  FLOAT = 2,         // IEEE float (half, float, double)
  FIXED_BYTES = 3,   // fixed-size binary / decimal: memcmp order
  VAR_BYTES = 4,     // string / binary: offsets + bytes
};

struct DataType {
  Type type = Type::INT64;
  int32_t byte_width = 0;  // only used by FIXED_SIZE_BINARY / DECIMAL
  TimeUnit unit = TimeUnit::MILLI;
  std::string timezone;
  Type value_type = Type::INT64;  // LIST / FIXED_SIZE_LIST element type (numeric)
  int32_t list_size = 0;          // FIXED_SIZE_LIST elements per row
  int32_t precision = 0;          // DECIMAL precision / scale (0, 0 = unknown: decimal(38, 0))
  int32_t scale = 0;

  DataType() = default;
  explicit DataType(Type t) : type(t) {}
  DataType(Type t, int32_t bw) : type(t), byte_width(bw) {}

  static DataType FixedSizeBinary(int32_t w) { return DataType(Type::FIXED_SIZE_BINARY, w); }
  static DataType List(Type elem) {
    DataType d(Type::LIST);
    d.value_type = elem;
    d.check_list();
    return d;
  }
  static DataType FixedSizeList(Type elem, int32_t size) {
    DataType d(Type::FIXED_SIZE_LIST);
    d.value_type = elem;
    d.list_size = size;
    d.check_list();
    return d;
  }
  bool is_list() const { return type == Type::LIST || type == Type::FIXED_SIZE_LIST; }
  // element width of a list type (numeric elements only)
  int32_t value_width() const { return DataType(value_type).width(); }
  void check_list() const {
    CYLON_CHECK(DataType(value_type).is_numeric(), Code::NotImplemented,
                "list columns support numeric elements only, not type " << static_cast<int>(value_type));
    CYLON_CHECK(type != Type::FIXED_SIZE_LIST || list_size >= 0, Code::Invalid, "negative list size");
  }
  static DataType Timestamp(TimeUnit u, std::string tz = "") {
    DataType d(Type::TIMESTAMP);
    d.unit = u;
    d.timezone = std::move(tz);
    return d;
  }

  bool operator==(const DataType &o) const {
    return type == o.type && width() == o.width() && unit == o.unit && (!is_list() || value_type == o.value_type);
  }
  bool operator!=(const DataType &o) const { return !(*this == o); }

  Layout layout() const { return is_variable_width() ? Layout::VARIABLE_WIDTH : Layout::FIXED_WIDTH; }

  bool is_variable_width() const { return type == Type::STRING || type == Type::BINARY || type == Type::LIST; }

  // physical bytes per element for fixed width types; 0 for var width
  int32_t width() const {
    switch (type) {
      case Type::BOOL:
      case Type::UINT8:
      case Type::INT8: return 1;
      case Type::UINT16:
      case Type::INT16:
      case Type::HALF_FLOAT: return 2;
      case Type::UINT32:
      case Type::INT32:
      case Type::FLOAT:
      case Type::DATE32:
      case Type::TIME32: return 4;
      case Type::UINT64:
      case Type::INT64:
      case Type::DOUBLE:
      case Type::DATE64:
      case Type::TIMESTAMP:
      case Type::TIME64:
      case Type::DURATION: return 8;
      case Type::FIXED_SIZE_BINARY:
      case Type::DECIMAL: return byte_width;
      case Type::FIXED_SIZE_LIST: return list_size * value_width();
      case Type::STRING:
      case Type::BINARY:
      case Type::LIST: return 0;
      default: CYLON_THROW(Code::NotImplemented, "type " << static_cast<int>(type) << " is not supported");
    }
  }

  ValueKind kind() const {
    switch (type) {
      case Type::BOOL:
      case Type::UINT8:
      case Type::UINT16:
      case Type::UINT32:
      case Type::UINT64: return ValueKind::UNSIGNED_INT;
      case Type::INT8:
      case Type::INT16:
      case Type::INT32:
      case Type::INT64:
      case Type::DATE32:
      case Type::DATE64:
      case Type::TIMESTAMP:
      case Type::TIME32:
      case Type::TIME64:
      case Type::DURATION: return ValueKind::SIGNED_INT;
      case Type::HALF_FLOAT:
      case Type::FLOAT:
      case Type::DOUBLE: return ValueKind::FLOAT;
      case Type::FIXED_SIZE_BINARY:
      case Type::DECIMAL:
      case Type::FIXED_SIZE_LIST: return ValueKind::FIXED_BYTES;
      case Type::STRING:
      case Type::BINARY:
      case Type::LIST: return ValueKind::VAR_BYTES;
      default: CYLON_THROW(Code::NotImplemented, "type " << static_cast<int>(type) << " is not supported");
    }
  }

  bool is_numeric() const {
    auto k = kind();
    return (k == ValueKind::SIGNED_INT || k == ValueKind::UNSIGNED_INT || k == ValueKind::FLOAT);
  }

  std::string ToString() const;
};

const char *TypeName(Type t);

}  // namespace cylon
