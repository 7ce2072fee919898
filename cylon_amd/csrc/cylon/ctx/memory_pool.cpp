// Memory pools (C2): see memory_pool.hpp.
#include "memory_pool.hpp"

#include <c10/hip/HIPCachingAllocator.h>
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>

#include "../common.hpp"

namespace cylon {

void CountingPool::on_alloc(int64_t n) {
  const int64_t now = bytes_ += n;
  int64_t p = peak_.load();
  while (now > p && !peak_.compare_exchange_weak(p, now)) {
  }
}

uint8_t *HostMemoryPool::Allocate(int64_t size) {
  if (size == 0) return nullptr;
  void *p = nullptr;
  if (posix_memalign(&p, 64, (size_t)size) != 0 || !p)
    CYLON_THROW(Code::OutOfMemory, "host pool: cannot allocate " << size << " bytes");
  on_alloc(size);
  return static_cast<uint8_t *>(p);
}

uint8_t *HostMemoryPool::Reallocate(uint8_t *ptr, int64_t old_size, int64_t new_size) {
  uint8_t *q = Allocate(new_size);
  if (ptr && q) std::memcpy(q, ptr, (size_t)std::min(old_size, new_size));
  Free(ptr, old_size);
  return q;
}

void HostMemoryPool::Free(uint8_t *ptr, int64_t size) {
  if (!ptr) return;
  std::free(ptr);
  on_free(size);
}

uint8_t *DeviceMemoryPool::Allocate(int64_t size) {
  if (size == 0) return nullptr;
  c10::DeviceGuard g(dev_);
  void *p = c10::hip::HIPCachingAllocator::raw_alloc((size_t)size);
  if (!p) CYLON_THROW(Code::OutOfMemory, "device pool: cannot allocate " << size << " bytes");
  on_alloc(size);
  return static_cast<uint8_t *>(p);
}

uint8_t *DeviceMemoryPool::Reallocate(uint8_t *ptr, int64_t old_size, int64_t new_size) {
  uint8_t *q = Allocate(new_size);
  if (ptr && q) {
    c10::DeviceGuard g(dev_);
    if (hipMemcpy(q, ptr, (size_t)std::min(old_size, new_size), hipMemcpyDeviceToDevice) != hipSuccess)
      CYLON_THROW(Code::ExecutionError, "device pool: reallocate copy failed");
  }
  Free(ptr, old_size);
  return q;
}

void DeviceMemoryPool::Free(uint8_t *ptr, int64_t size) {
  if (!ptr) return;
  c10::DeviceGuard g(dev_);
  c10::hip::HIPCachingAllocator::raw_delete(ptr);
  on_free(size);
}

std::shared_ptr<MemoryPool> DefaultMemoryPool(at::Device dev) {
  if (dev.is_cuda()) return std::make_shared<DeviceMemoryPool>(dev);
  return std::make_shared<HostMemoryPool>();
}

namespace {
struct PoolCtx {
  std::shared_ptr<MemoryPool> pool;
  uint8_t *ptr;
  int64_t size;
};
void pool_deleter(void *ctx) {
  auto *c = static_cast<PoolCtx *>(ctx);
  c->pool->Free(c->ptr, c->size);
  delete c;
}
}  // namespace

at::Tensor EmptyFromPool(const std::shared_ptr<MemoryPool> &pool, at::IntArrayRef sizes, at::ScalarType dtype) {
  int64_t numel = 1;
  for (auto s : sizes) numel *= s;
  const int64_t bytes = numel * (int64_t)c10::elementSize(dtype);
  uint8_t *p = pool->Allocate(std::max<int64_t>(bytes, 1));
  auto *ctx = new PoolCtx{pool, p, std::max<int64_t>(bytes, 1)};
  at::DataPtr dp(p, ctx, &pool_deleter, pool->device());
  at::Storage st(at::Storage::use_byte_size_t(), bytes, std::move(dp), /*allocator=*/nullptr, /*resizable=*/false);
  return at::empty({0}, at::TensorOptions().dtype(dtype).device(pool->device())).set_(st, 0, sizes);
}

}  // namespace cylon
