// Host -> HBM ingest of pageable host buffers (Arrow / numpy memory) through pinned staging.
//
// The reference builds Arrow arrays in host memory and never leaves it
// (cpp/src/cylon/arrow/arrow_builder.cpp:31-161).  Here every from-Arrow column crosses
// PCIe once; a pageable torch `.to(device)` copies through the driver's small bounce buffers
// synchronously.  StagedH2D instead keeps a per-device ring of pinned buffers: host worker
// threads copy chunk k+1 of the source into one ring slot while the DMA engine moves chunk k
// out of another (hipMemcpyAsync on a dedicated non-blocking copy stream), and the caller's
// stream waits on the last copy with an event -- the host returns as soon as the source bytes
// are staged, the device work that consumes the column is ordered after the DMA.
#pragma once
#include <cstddef>
#include <cstdint>

namespace cylon {
namespace io {

struct H2DStats {
  int64_t bytes = 0;
  int64_t chunks = 0;
  double seconds = 0;  // host time of the call (staging copies + DMA issue)
};

// Copy `bytes` from host `src` (any memory) to device pointer `dst` on `device`; the current
// stream of that device waits for the copy.  threads <= 0: default worker count.
void StagedH2D(const void *src, void *dst, size_t bytes, int device, int threads = 0, H2DStats *stats = nullptr);

// Chunk size and ring depth of the staging buffers (CYLON_H2D_CHUNK_MB, default 32; 4 slots).
size_t StagedH2DChunkBytes();

}  // namespace io
}  // namespace cylon
