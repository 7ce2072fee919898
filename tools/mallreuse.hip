// Infinity Cache (MALL) go / no-go for a MALL-resident second radix pass.
//
// The join's second partition pass writes 56 GB that the join kernel reads straight back.  If the
// pass and the join ran per GROUP of first-level buckets through one reused scratch buffer small
// enough to stay in the 256 MiB MALL, those 112 GB would not cross HBM.  This models exactly that
// traffic with plain streaming kernels (16-B vector accesses, grid-stride, 2048 blocks):
//   P(g): read  S bytes of `in`  at group g  -> write S bytes of mid
//   J(g): read  S bytes of mid               -> write S bytes of `out` at group g
// for G groups covering T bytes, in four schedules:
//   whole   : one P over all T bytes into a T-byte mid, then one J  (today's structure)
//   fresh   : per group, mid = a fresh T-byte array region (no reuse; launch-count control)
//   reuse   : per group, mid = ONE S-byte scratch buffer (MALL-resident if it survives)
//   reuse2s : double-buffered scratch, P(g+1) on stream 1 overlapping J(g) on stream 0
// Build: hipcc --offload-arch=gfx950 -O3 tools/mallreuse.hip -o tools/mallreuse
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                            \
  do {                                                                   \
    hipError_t e = (x);                                                  \
    if (e != hipSuccess) {                                               \
      fprintf(stderr, "HIP %s at %d\n", hipGetErrorString(e), __LINE__); \
      exit(1);                                                           \
    }                                                                    \
  } while (0)

__global__ __launch_bounds__(256) void k_copy(const int4 *__restrict__ in, int4 *__restrict__ out, long n) {
  const long stride = (long)gridDim.x * blockDim.x;
  long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {  // four loads in flight per thread
    const int4 a = in[i], b = in[i + stride], c = in[i + 2 * stride], d = in[i + 3 * stride];
    out[i] = a;
    out[i + stride] = b;
    out[i + 2 * stride] = c;
    out[i + 3 * stride] = d;
  }
  for (; i < n; i += stride) out[i] = in[i];
}

static float elapsed(hipEvent_t a, hipEvent_t b) {
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms;
}

int main(int argc, char **argv) {
  const size_t T = (argc > 1 ? (size_t)atol(argv[1]) : 16) << 30;  // GiB per array
  int4 *in, *mid, *out;
  CK(hipMalloc(&in, T));
  CK(hipMalloc(&mid, T));
  CK(hipMalloc(&out, T));
  CK(hipMemset(in, 1, T));
  CK(hipMemset(mid, 2, T));
  CK(hipMemset(out, 3, T));
  hipStream_t s0, s1;
  CK(hipStreamCreateWithFlags(&s0, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int grid = 2048;
  auto copy = [&](const int4 *src, int4 *dst, size_t bytes, hipStream_t s) {
    hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, s, src, dst, (long)(bytes / 16));
  };
  const double tb = 4.0 * T / 1e12;  // bytes every schedule moves through the kernels (2 reads + 2 writes)
  printf("# T = %zu GiB per array; rates = 4T / time (P + J reads and writes)\n", T >> 30);
  for (int rep = 0; rep < 2; ++rep) {
    // whole
    copy(in, mid, T, s0);
    copy(mid, out, T, s0);
    CK(hipStreamSynchronize(s0));
    CK(hipEventRecord(e0, s0));
    copy(in, mid, T, s0);
    copy(mid, out, T, s0);
    CK(hipEventRecord(e1, s0));
    CK(hipEventSynchronize(e1));
    float ms = elapsed(e0, e1);
    printf("whole                 %8.2f ms  %.2f TB/s\n", ms, tb / (ms * 1e-3));
    for (size_t S = size_t(16) << 20; S <= (size_t(256) << 20); S <<= 1) {
      const size_t G = T / S;
      const char *names[3] = {"fresh", "reuse", "reuse2s"};
      for (int mode = 0; mode < 3; ++mode) {
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0, s0));
        hipEvent_t done[2];
        CK(hipEventCreateWithFlags(&done[0], hipEventDisableTiming));
        CK(hipEventCreateWithFlags(&done[1], hipEventDisableTiming));
        for (size_t g = 0; g < G; ++g) {
          const int4 *src = in + g * (S / 16);
          int4 *dst = out + g * (S / 16);
          if (mode == 0) {
            int4 *m = mid + g * (S / 16);
            copy(src, m, S, s0);
            copy(m, dst, S, s0);
          } else if (mode == 1) {
            copy(src, mid, S, s0);
            copy(mid, dst, S, s0);
          } else {
            // P(g) on s1 into buffer g & 1 once J(g - 2) released it; J(g) on s0 after P(g)
            int4 *m = mid + (g & 1) * (S / 16);
            if (g >= 2) CK(hipStreamWaitEvent(s1, done[g & 1], 0));
            else if (g == 0) {
              CK(hipEventRecord(done[0], s0));
              CK(hipStreamWaitEvent(s1, done[0], 0));
            }
            copy(src, m, S, s1);
            hipEvent_t pe;
            CK(hipEventCreateWithFlags(&pe, hipEventDisableTiming));
            CK(hipEventRecord(pe, s1));
            CK(hipStreamWaitEvent(s0, pe, 0));
            CK(hipEventDestroy(pe));
            copy(m, dst, S, s0);
            CK(hipEventRecord(done[g & 1], s0));
          }
        }
        CK(hipEventRecord(e1, s0));
        CK(hipEventSynchronize(e1));
        ms = elapsed(e0, e1);
        printf("%-8s S=%4zu MiB  %8.2f ms  %.2f TB/s  (%zu groups)\n", names[mode], S >> 20, ms, tb / (ms * 1e-3), G);
        fflush(stdout);
        CK(hipEventDestroy(done[0]));
        CK(hipEventDestroy(done[1]));
      }
    }
  }
  return 0;
}
