// Memory pool abstraction (C2).
//
// Reference: cpp/src/cylon/ctx/memory_pool.hpp:25-66 (Allocate / Reallocate /
// Free / bytes_allocated / max_memory / backend_name) and
// arrow_memory_pool_utils.hpp:25-61 (ProxyMemoryPool adapting it to Arrow).
// Here the default pools are
//   * DeviceMemoryPool: HBM through the HIP caching allocator of the
//     context's device (the same allocator every table buffer comes from, so
//     pool-allocated scratch and table columns share one budget of 288 GB);
//   * HostMemoryPool: 64-byte aligned host memory (the reference's default).
// A custom pool can be installed on a context (CylonContext::SetMemoryPool);
// ProxyAllocator exposes any pool as an at::Allocator so tensors (and hence
// table columns) can be carved from it.
#pragma once
#include <ATen/ATen.h>

#include <atomic>
#include <cstdint>
#include <memory>
#include <string>

namespace cylon {

class MemoryPool {
 public:
  virtual ~MemoryPool() = default;
  // allocate `size` bytes (64-byte aligned); throws CylonError(OutOfMemory) on failure
  virtual uint8_t *Allocate(int64_t size) = 0;
  // grow/shrink an allocation, preserving min(old, new) bytes
  virtual uint8_t *Reallocate(uint8_t *ptr, int64_t old_size, int64_t new_size) = 0;
  virtual void Free(uint8_t *ptr, int64_t size) = 0;
  virtual int64_t bytes_allocated() const = 0;
  virtual int64_t max_memory() const = 0;
  virtual std::string backend_name() const = 0;
  virtual at::Device device() const = 0;
};

// Byte accounting shared by the built-in pools.
class CountingPool : public MemoryPool {
 public:
  int64_t bytes_allocated() const override { return bytes_.load(); }
  int64_t max_memory() const override { return peak_.load(); }

 protected:
  void on_alloc(int64_t n);
  void on_free(int64_t n) { bytes_ -= n; }

 private:
  std::atomic<int64_t> bytes_{0}, peak_{0};
};

class HostMemoryPool : public CountingPool {
 public:
  uint8_t *Allocate(int64_t size) override;
  uint8_t *Reallocate(uint8_t *ptr, int64_t old_size, int64_t new_size) override;
  void Free(uint8_t *ptr, int64_t size) override;
  std::string backend_name() const override { return "host"; }
  at::Device device() const override { return at::Device(at::kCPU); }
};

class DeviceMemoryPool : public CountingPool {
 public:
  explicit DeviceMemoryPool(at::Device dev) : dev_(dev) {}
  uint8_t *Allocate(int64_t size) override;
  uint8_t *Reallocate(uint8_t *ptr, int64_t old_size, int64_t new_size) override;
  void Free(uint8_t *ptr, int64_t size) override;
  std::string backend_name() const override { return "hip_caching_allocator"; }
  at::Device device() const override { return dev_; }

 private:
  at::Device dev_;
};

std::shared_ptr<MemoryPool> DefaultMemoryPool(at::Device dev);

// at::Allocator over a MemoryPool: tensors whose storage comes from the pool.
at::Tensor EmptyFromPool(const std::shared_ptr<MemoryPool> &pool, at::IntArrayRef sizes, at::ScalarType dtype);

}  // namespace cylon
