// Infinity Cache (MALL, 256 MiB) residency microbenchmark: ping-pong copies A -> B -> A of a
// working set of S bytes (16-byte vector loads / stores, grid-stride), S from 16 MiB to 8 GiB,
// and a read-only re-read of S bytes.  If copies whose in + out fit the 256 MiB die cache run
// much faster than HBM-sized ones, a sort that finishes small segments while they are resident
// (MSD first pass, then per-segment LSD passes) can beat whole-array LSD passes.
// Build: hipcc --offload-arch=gfx950 -O3 tools/mallbench.hip -o tools/mallbench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      fprintf(stderr, "HIP %s at %d\n", hipGetErrorString(e), __LINE__);   \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

__global__ void k_copy(const int4 *__restrict__ in, int4 *__restrict__ out, long n) {
  const long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = in[i];
}

__global__ void k_read(const int4 *__restrict__ in, long n, int *sink) {
  const long stride = (long)gridDim.x * blockDim.x;
  int acc = 0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const int4 v = in[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678) sink[0] = acc;
}

int main() {
  const size_t maxb = size_t(8) << 30;
  int4 *a, *b;
  int *sink;
  CK(hipMalloc(&a, maxb));
  CK(hipMalloc(&b, maxb));
  CK(hipMalloc(&sink, 4));
  CK(hipMemset(a, 1, maxb));
  CK(hipMemset(b, 2, maxb));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (size_t s = size_t(16) << 20; s <= maxb; s <<= 1) {
    const long n = (long)(s / 16);
    const int grid = 256 * 8;
    const int reps = (int)std::max<size_t>(4, (size_t(64) << 30) / s);
    for (int w = 0; w < 2; ++w) hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, w ? b : a, w ? a : b, n);
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, r & 1 ? b : a, r & 1 ? a : b, n);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double cp = 2.0 * s * reps / (ms * 1e-3) / 1e12;
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, a, n, sink);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    CK(hipEventElapsedTime(&ms, e0, e1));
    const double rd = 1.0 * s * reps / (ms * 1e-3) / 1e12;
    printf("working set %7.0f MiB: ping-pong copy %.2f TB/s (read+write), re-read %.2f TB/s, %d reps\n",
           s / 1048576.0, cp, rd, reps);
    fflush(stdout);
  }
  return 0;
}
