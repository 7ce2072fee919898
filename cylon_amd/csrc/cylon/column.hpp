// Device-resident column (L2 data model).
//
// Reference: cpp/src/cylon/column.hpp:31-104 (Column wraps an arrow::ChunkedArray).
// Here a column is always a single contiguous chunk owned by torch tensors so
// that storage comes from the HIP stream-ordered caching allocator and can be
// handed to RCCL, DLPack and the HIP kernels without copies.
#pragma once
#include <ATen/ATen.h>

#include <string>
#include <vector>

#include "types.hpp"
#include "kernels/kernels.hpp"

namespace cylon {

struct Column {
  std::string name;
  DataType type;
  int64_t length = 0;
  at::Tensor data;      // fixed width: typed tensor [length] or uint8 [length*w]; var width: uint8 bytes
  at::Tensor offsets;   // var width only: int64 [length + 1]
  at::Tensor validity;  // optional uint8 [length], 1 = valid

  Column() = default;
  Column(std::string n, DataType t, int64_t len, at::Tensor d, at::Tensor o = at::Tensor(),
         at::Tensor v = at::Tensor())
      : name(std::move(n)), type(std::move(t)), length(len), data(std::move(d)), offsets(std::move(o)),
        validity(std::move(v)) {}

  bool is_var() const { return type.is_variable_width(); }
  bool nullable() const { return validity.defined(); }
  at::Device device() const { return data.device(); }
  bool on_gpu() const { return data.is_cuda(); }

  ColView view() const {
    ColView v;
    v.data = data.defined() && data.numel() > 0 ? reinterpret_cast<const uint8_t *>(data.data_ptr()) : nullptr;
    v.offsets = is_var() ? offsets.data_ptr<int64_t>() : nullptr;
    v.valid = validity.defined() ? validity.data_ptr<uint8_t>() : nullptr;
    v.width = is_var() ? 0 : type.width();
    v.kind = static_cast<int>(type.kind());
    return v;
  }

  int64_t null_count() const;
  int64_t nbytes() const;
  Column to(at::Device dev, bool non_blocking = false) const;
  Column with_name(const std::string &n) const {
    Column c = *this;
    c.name = n;
    return c;
  }
  Column slice(int64_t offset, int64_t len) const;
};

// torch dtype used to store a fixed width cylon type
at::ScalarType storage_dtype(const DataType &t);

// Allocate an uninitialised fixed-width / var-width column on a device.
Column make_fixed_column(const std::string &name, const DataType &t, int64_t n, at::Device dev, bool nullable);

}  // namespace cylon
