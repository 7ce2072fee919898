// Logical data types of the engine.
//
// The Type enum keeps the reference's numbering (cpp/src/cylon/data_types.hpp:26-100)
// so that code written against the reference's Type/Layout constants keeps its
// meaning.  Physical storage is device-resident and Arrow-like:
//   * fixed width  -> one contiguous buffer of n * byte_width bytes
//   * STRING/BINARY -> int64 offsets[n+1] + uint8 bytes   (always 64-bit offsets)
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

  DataType() = default;
  explicit DataType(Type t) : type(t) {}
  DataType(Type t, int32_t bw) : type(t), byte_width(bw) {}

  static DataType FixedSizeBinary(int32_t w) { return DataType(Type::FIXED_SIZE_BINARY, w); }
  static DataType Timestamp(TimeUnit u, std::string tz = "") {
    DataType d(Type::TIMESTAMP);
    d.unit = u;
    d.timezone = std::move(tz);
    return d;
  }

  bool operator==(const DataType &o) const {
    return type == o.type && width() == o.width() && unit == o.unit;
  }
  bool operator!=(const DataType &o) const { return !(*this == o); }

  Layout layout() const { return is_variable_width() ? Layout::VARIABLE_WIDTH : Layout::FIXED_WIDTH; }

  bool is_variable_width() const { return type == Type::STRING || type == Type::BINARY; }

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
      case Type::STRING:
      case Type::BINARY: return 0;
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
      case Type::DECIMAL: return ValueKind::FIXED_BYTES;
      case Type::STRING:
      case Type::BINARY: return ValueKind::VAR_BYTES;
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
