// Stable merge of two sorted runs of (uint64 order image, int64 payload) pairs: the receive
// side of the pipelined distributed sort (ops/setops.cpp merge_sorted_chunk) merges the W
// sorted runs it receives per chunk pairwise instead of radix-sorting them again.
//
// Merge path (Odeh, Green, Mwassi, Shmueli, Birk: "Merge Path - Parallel Merging Made Simple"):
// output position d splits into a from A and d - a from B, a = the number of A elements among
// the first d outputs, found by a binary search along the cross diagonal.  A block owns 2048
// consecutive outputs: it finds its two diagonal splits, stages the at most 2048 inputs it
// needs (A then B, coalesced) in LDS, and every thread merges 8 consecutive outputs from its
// own LDS split -- sequential LDS reads, one coalesced 8-B store per output per lane group.
// Ties take A first: A is the run of the lower rank, so equal keys keep rank order (stable).
#include "device_common.hpp"

namespace cylon {
namespace hip {

constexpr int kMgThreads = 256;
constexpr int kMgItems = 8;
constexpr int kMgTile = kMgThreads * kMgItems;

// number of A elements among the first d outputs (A wins ties)
template <class LA, class LB>
__device__ __forceinline__ int64_t merge_split(LA a, int64_t na, LB b, int64_t nb, int64_t d) {
  int64_t lo = d > nb ? d - nb : 0, hi = d < na ? d : na;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (a(mid) <= b(d - 1 - mid)) lo = mid + 1; else hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(kMgThreads) void k_merge_pairs(const uint64_t *__restrict__ ak,
                                                            const int64_t *__restrict__ ai, int64_t na,
                                                            const uint64_t *__restrict__ bk,
                                                            const int64_t *__restrict__ bi, int64_t nb,
                                                            uint64_t *__restrict__ ok, int64_t *__restrict__ oi) {
  __shared__ uint64_t sk[kMgTile];
  __shared__ int64_t si[kMgTile];
  __shared__ int64_t split[2];
  const int64_t n = na + nb;
  const int64_t d0 = (int64_t)blockIdx.x * kMgTile, d1 = d0 + kMgTile < n ? d0 + kMgTile : n;
  if (threadIdx.x < 2) {
    auto ga = [&](int64_t i) { return ak[i]; };
    auto gb = [&](int64_t i) { return bk[i]; };
    split[threadIdx.x] = merge_split(ga, na, gb, nb, threadIdx.x == 0 ? d0 : d1);
  }
  __syncthreads();
  const int64_t a0 = split[0], a1 = split[1];
  const int64_t b0 = d0 - a0, b1 = d1 - a1;
  const int la = (int)(a1 - a0), lb = (int)(b1 - b0);
  for (int t = threadIdx.x; t < la + lb; t += kMgThreads) {  // A's slice, then B's
    const bool fa = t < la;
    sk[t] = fa ? ak[a0 + t] : bk[b0 + t - la];
    si[t] = fa ? ai[a0 + t] : bi[b0 + t - la];
  }
  __syncthreads();
  const int dl = threadIdx.x * kMgItems;
  const int nout = la + lb;  // == d1 - d0
  const int mine = dl < nout ? (nout - dl < kMgItems ? nout - dl : kMgItems) : 0;
  uint64_t rk[kMgItems];
  int64_t ri[kMgItems];
  if (mine > 0) {
    auto la_ = [&](int64_t i) { return sk[i]; };
    auto lb_ = [&](int64_t i) { return sk[la + i]; };
    int x = (int)merge_split(la_, la, lb_, lb, dl), y = dl - x;
#pragma unroll
    for (int j = 0; j < kMgItems; ++j) {
      if (j < mine) {
        const bool takea = x < la && (y >= lb || sk[x] <= sk[la + y]);
        const int src = takea ? x : la + y;
        rk[j] = sk[src];
        ri[j] = si[src];
        x += takea ? 1 : 0;
        y += takea ? 0 : 1;
      }
    }
  }
  __syncthreads();  // the tile's inputs are consumed: reuse the stage for coalesced stores
#pragma unroll
  for (int j = 0; j < kMgItems; ++j)
    if (j < mine) {
      sk[dl + j] = rk[j];
      si[dl + j] = ri[j];
    }
  __syncthreads();
  for (int t = threadIdx.x; t < nout; t += kMgThreads) {
    ok[d0 + t] = sk[t];
    oi[d0 + t] = si[t];
  }
}

void merge_sorted_pairs(const uint64_t *ak, const int64_t *ai, int64_t na, const uint64_t *bk, const int64_t *bi,
                        int64_t nb, uint64_t *ok, int64_t *oi, void *stream) {
  const int64_t n = na + nb;
  if (n == 0) return;
  const int64_t blocks = (n + kMgTile - 1) / kMgTile;
  hipLaunchKernelGGL(k_merge_pairs, dim3((unsigned)blocks), dim3(kMgThreads), 0, as_stream(stream), ak, ai, na, bk,
                     bi, nb, ok, oi);
  HIP_LAUNCH_CHECK();
}

// this file's code object is loaded at context creation (preload_device_code), not on first use
void preload_merge() { preload_code(reinterpret_cast<const void *>(&k_merge_pairs)); }

}  // namespace hip
}  // namespace cylon
