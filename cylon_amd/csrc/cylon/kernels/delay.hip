// Timed device delay (test transport support, net/async_delay_communicator.cpp): one
// wave spins on the constant wall clock (s_memrealtime, hipDeviceAttributeWallClockRate) with s_sleep between reads,
// so a posted transfer's completion event fires `us` microseconds after the
// stream reaches it.  The loop ends for every lane at the same clock bound.
#include "device_common.hpp"

namespace cylon {
namespace hip {

__global__ __launch_bounds__(64) void k_spin_delay(uint64_t ticks) {
  const uint64_t t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(32);
}

void spin_delay_us(double us, void *stream) {
  int dev = 0, khz = 0;
  HIP_CHECK(hipGetDevice(&dev));
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess || khz <= 0) khz = 100000;
  const uint64_t ticks = (uint64_t)(us < 0 ? 0.0 : us * (double)khz / 1000.0);
  hipLaunchKernelGGL(k_spin_delay, dim3(1), dim3(64), 0, as_stream(stream), ticks);
  HIP_LAUNCH_CHECK();
}

// this file's code object is loaded at context creation (preload_device_code), not on first use
void preload_delay() { preload_code(reinterpret_cast<const void *>(&k_spin_delay)); }

}  // namespace hip
}  // namespace cylon
