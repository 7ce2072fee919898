// Microbenchmark: semi-join key filter primitives on one MI355X.
// Build: atomicOr of n random keys into a bitmap over [0, range); probe: test n keys.
// Also a byte-map variant (plain byte stores, no atomics).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

__global__ void gen(int64_t *k, int64_t n, int64_t range, uint64_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t x = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
    x ^= x >> 33; x *= 0xff51afd7ed558ccdull; x ^= x >> 33; x *= 0xc4ceb9fe1a85ec53ull; x ^= x >> 33;
    k[i] = (int64_t)(x % (uint64_t)range);
  }
}
__global__ void build(const int64_t *k, int64_t n, uint32_t *bm) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t v = (uint64_t)k[i];
    atomicOr(&bm[v >> 5], 1u << (v & 31));
  }
}
__global__ void build_bytes(const int64_t *k, int64_t n, uint8_t *bm) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    bm[k[i]] = 1;
}
__global__ void probe(const int64_t *k, int64_t n, const uint32_t *bm, uint8_t *out) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t v = (uint64_t)k[i];
    out[i] = (bm[v >> 5] >> (v & 31)) & 1u;
  }
}

int main() {
  const int64_t n = 500000000, range = 990000000;
  int64_t *k; uint32_t *bm; uint8_t *bb, *out;
  CK(hipMalloc(&k, n * 8)); CK(hipMalloc(&bm, (range / 32 + 1) * 4)); CK(hipMalloc(&bb, range)); CK(hipMalloc(&out, n));
  hipLaunchKernelGGL(gen, dim3(4096), dim3(256), 0, 0, k, n, range, 12345ull);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int grid : {2048, 8192, 65536}) {
    for (int rep = 0; rep < 2; ++rep) {
      CK(hipMemset(bm, 0, (range / 32 + 1) * 4));
      hipEventRecord(a);
      hipLaunchKernelGGL(build, dim3(grid), dim3(256), 0, 0, k, n, bm);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b);
      hipEventRecord(a);
      hipLaunchKernelGGL(probe, dim3(grid), dim3(256), 0, 0, k, n, bm, out);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms2; hipEventElapsedTime(&ms2, a, b);
      hipEventRecord(a);
      hipLaunchKernelGGL(build_bytes, dim3(grid), dim3(256), 0, 0, k, n, bb);
      hipEventRecord(b); hipEventSynchronize(b);
      float ms3; hipEventElapsedTime(&ms3, a, b);
      if (rep) printf("grid %6d: bitmap build %.2f ms (%.1f G/s)  probe %.2f ms (%.1f G/s)  bytemap build %.2f ms\n", grid, ms,
                      n / ms / 1e6, ms2, n / ms2 / 1e6, ms3);
    }
  }
  return 0;
}
