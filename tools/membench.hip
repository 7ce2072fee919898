// Memory-system microbenchmarks for the join design (MI355X / gfx950).
//   1. streaming copy of 4 int64 columns -> 4 columns, columns allocated
//      separately (power-of-two spaced) vs one allocation with staggered offsets
//   2. same with the row index permuted inside 8192-row tiles (partition pass read side)
//   3. random 8-byte reads inside a window of W bytes (TLB / cache reach)
// Build: hipcc --offload-arch=gfx950 -O3 tools/membench.hip -o build/membench
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e = (x);                                                          \
    if (e != hipSuccess) {                                                       \
      fprintf(stderr, "HIP %s at %d\n", hipGetErrorString(e), __LINE__);         \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)

struct Cols {
  const long *in[4];
  long *out[4];
};

__global__ void k_copy4(Cols c, long n, int perm) {
  long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    long s = i;
    if (perm) s = (i & ~8191L) | ((i * 2654435761L) & 8191L);
    long v0 = c.in[0][s], v1 = c.in[1][s], v2 = c.in[2][s], v3 = c.in[3][s];
    c.out[0][i] = v0;
    c.out[1][i] = v1;
    c.out[2][i] = v2;
    c.out[3][i] = v3;
  }
}

// radix-pass write pattern: every 8192-row tile sends one run of R rows to each of 8192/R buckets
template <bool NT>
__global__ void k_scatter_runs(Cols c, long n, int R) {
  const long nb = 8192 / R, bsize = n / nb;
  long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const long tile = i >> 13, j = i & 8191;
    const long d = (j / R) * bsize + tile * R + (j % R);
    long v0 = c.in[0][i], v1 = c.in[1][i], v2 = c.in[2][i], v3 = c.in[3][i];
    if (NT) {
      __builtin_nontemporal_store(v0, &c.out[0][d]);
      __builtin_nontemporal_store(v1, &c.out[1][d]);
      __builtin_nontemporal_store(v2, &c.out[2][d]);
      __builtin_nontemporal_store(v3, &c.out[3][d]);
    } else {
      c.out[0][d] = v0;
      c.out[1][d] = v1;
      c.out[2][d] = v2;
      c.out[3][d] = v3;
    }
  }
}

__global__ void k_copy1(const long *in, long *out, long n) {
  long stride = (long)gridDim.x * blockDim.x;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) out[i] = in[i];
}

__global__ void k_rand(const long *in, long window_elems, long nreads, long *sink) {
  long stride = (long)gridDim.x * blockDim.x;
  long acc = 0;
  for (long i = (long)blockIdx.x * blockDim.x + threadIdx.x; i < nreads; i += stride) {
    unsigned long h = (unsigned long)i * 0x9E3779B97F4A7C15ull;
    h ^= h >> 29;
    h *= 0xBF58476D1CE4E5B9ull;
    h ^= h >> 32;
    acc += in[h % (unsigned long)window_elems];
  }
  if (acc == 42) sink[0] = acc;
}

static float timeit(void (*f)(void *), void *arg, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  f(arg);
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r) f(arg);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

struct CopyArg {
  Cols c;
  long n;
  int perm;
};
static void run_copy(void *p) {
  CopyArg *a = (CopyArg *)p;
  hipLaunchKernelGGL(k_copy4, dim3(4096), dim3(256), 0, 0, a->c, a->n, a->perm);
}
struct ScatArg {
  Cols c;
  long n;
  int R;
  bool nt;
};
static void run_scat(void *p) {
  ScatArg *a = (ScatArg *)p;
  if (a->nt)
    hipLaunchKernelGGL(k_scatter_runs<true>, dim3(4096), dim3(256), 0, 0, a->c, a->n, a->R);
  else
    hipLaunchKernelGGL(k_scatter_runs<false>, dim3(4096), dim3(256), 0, 0, a->c, a->n, a->R);
}
struct Copy1Arg {
  const long *in;
  long *out;
  long n;
};
static void run_copy1(void *p) {
  Copy1Arg *a = (Copy1Arg *)p;
  hipLaunchKernelGGL(k_copy1, dim3(4096), dim3(256), 0, 0, a->in, a->out, a->n);
}
struct RandArg {
  const long *in;
  long w, nreads;
  long *sink;
};
static void run_rand(void *p) {
  RandArg *a = (RandArg *)p;
  hipLaunchKernelGGL(k_rand, dim3(8192), dim3(256), 0, 0, a->in, a->w, a->nreads, a->sink);
}

int main(int argc, char **argv) {
  const long n = argc > 1 ? atol(argv[1]) : (1L << 28);  // rows per column
  const size_t bytes = n * sizeof(long);
  printf("rows per column %ld (%.2f GB)\n", n, bytes / 1e9);
  // separate allocations
  std::vector<long *> sep(8);
  for (auto &p : sep) {
    CK(hipMalloc(&p, bytes));
    CK(hipMemset(p, 1, bytes));
  }
  // one allocation, staggered
  long *big;
  const size_t pad = (1 << 20) + 4096 * 3;
  CK(hipMalloc(&big, 8 * (bytes + 8 * pad)));
  CK(hipMemset(big, 1, 8 * (bytes + 8 * pad)));
  std::vector<long *> stg(8);
  for (int c = 0; c < 8; ++c) stg[c] = (long *)((char *)big + c * (bytes + pad * (c + 1)));

  Copy1Arg c1{sep[0], sep[1], n};
  float ms = timeit(run_copy1, &c1, 5);
  printf("copy1 sequential: %.3f ms  %.2f TB/s\n", ms, 2.0 * bytes / ms / 1e9);
  for (int perm = 0; perm < 2; ++perm) {
    for (int lay = 0; lay < 2; ++lay) {
      std::vector<long *> &v = lay ? stg : sep;
      CopyArg a;
      for (int c = 0; c < 4; ++c) {
        a.c.in[c] = v[c];
        a.c.out[c] = v[4 + c];
      }
      a.n = n;
      a.perm = perm;
      ms = timeit(run_copy, &a, 5);
      printf("copy4 %s %s: %.3f ms  %.2f TB/s\n", perm ? "tile-permuted" : "sequential", lay ? "staggered" : "separate",
             ms, 8.0 * bytes / ms / 1e9);
      fflush(stdout);
    }
  }
  for (int nt = 0; nt < 2; ++nt)
    for (int R = 2; R <= 128; R *= 2) {
      ScatArg a;
      for (int c = 0; c < 4; ++c) {
        a.c.in[c] = sep[c];
        a.c.out[c] = sep[4 + c];
      }
      a.n = n;
      a.R = R;
      a.nt = nt;
      ms = timeit(run_scat, &a, 3);
      printf("scatter runs of %3d rows (%4d buckets) %s: %.3f ms  %.2f TB/s\n", R, 8192 / R, nt ? "nt   " : "plain", ms,
             8.0 * bytes / ms / 1e9);
      fflush(stdout);
    }
  long *sink;
  CK(hipMalloc(&sink, 8));
  for (long w = 1L << 20; w <= (long)bytes * 8; w <<= 2) {
    RandArg r{big, w / 8, 1L << 27, sink};
    ms = timeit(run_rand, &r, 3);
    printf("random 8B reads, window %8.1f MB: %.3f ms  %.2f Greads/s\n", w / 1e6, ms, (1L << 27) / ms / 1e6);
    fflush(stdout);
  }
  return 0;
}
