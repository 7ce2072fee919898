// Probe: do same-address LDS atomics of one wave64 instruction return in lane order?
// Each wave owns packed 16-bit bucket counters (two per 32-bit word, as the radix
// pass keeps them); every round each lane adds 1 to the counter of a pseudo-random
// bucket and compares the returned count with the stable rank computed by ballots
// (count before the round + #lower lanes with the same bucket).  Buckets are drawn
// from small ranges to force many same-address (and same-word) collisions.
// Build: hipcc --offload-arch=gfx950 -O3 tools/lds_atomic_order.hip -o /tmp/lds_atomic_order
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int kThreads = 1024, kWaves = kThreads / 64, kMaxBuckets = 1024;

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352dU;
  x ^= x >> 15;
  x *= 0x846ca68bU;
  x ^= x >> 16;
  return x;
}

__global__ __launch_bounds__(kThreads) void k_probe(int rounds, int nbits, unsigned long long *bad,
                                                    unsigned long long *checked) {
  __shared__ uint32_t cnt[kWaves * kMaxBuckets / 2];
  const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  const uint32_t nb = 1u << nbits;
  uint32_t *mine = cnt + wave * (kMaxBuckets / 2);
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  unsigned long long nbad = 0, nchk = 0;
  for (int r0 = 0; r0 < rounds; r0 += 256) {  // counters restart every 256 rounds (16-bit halves)
    for (uint32_t q = lane; q < kMaxBuckets / 2; q += 64) mine[q] = 0;
    __builtin_amdgcn_wave_barrier();
    for (int r = r0; r < r0 + 256 && r < rounds; ++r) {
      const uint32_t b = mix((uint32_t)(blockIdx.x * 7919u + threadIdx.x * 104729u + (uint32_t)r * 1299709u)) & (nb - 1);
      // stable expectation by ballots
      uint64_t m = ~0ull;
      for (int bit = 0; bit < nbits; ++bit) {
        const uint32_t x = (b >> bit) & 1u;
        const uint64_t bb = __ballot(x);
        m &= x ? bb : ~bb;
      }
      const uint32_t sh = (b & 1u) * 16u;
      const uint32_t before = (mine[b >> 1] >> sh) & 0xffffu;
      __builtin_amdgcn_wave_barrier();
      const uint32_t old = atomicAdd(&mine[b >> 1], 1u << sh);
      __builtin_amdgcn_wave_barrier();
      const uint32_t got = (old >> sh) & 0xffffu;
      const uint32_t want = before + (uint32_t)__popcll(m & lt);
      nbad += got != want;
      ++nchk;
    }
  }
  atomicAdd(bad, nbad);
  atomicAdd(checked, nchk);
}

int main(int argc, char **argv) {
  const int rounds = argc > 1 ? std::atoi(argv[1]) : 4096;
  unsigned long long *d;
  hipMalloc(&d, 2 * sizeof(unsigned long long));
  int fails = 0;
  for (int nbits : {1, 3, 6, 9, 10}) {
    hipMemset(d, 0, 2 * sizeof(unsigned long long));
    hipLaunchKernelGGL(k_probe, dim3(2048), dim3(kThreads), 0, 0, rounds, nbits, d, d + 1);
    unsigned long long h[2];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    std::printf("buckets=%5u lane-ops checked=%llu out-of-lane-order=%llu\n", 1u << nbits, h[1], h[0]);
    fails += h[0] != 0;
  }
  hipFree(d);
  return fails ? 1 : 0;
}
