// K15 string <-> number casts on the device (gfx950): Table.astype between string columns and
// integer / floating columns without a host round trip through Arrow.
//   * string -> int64: optional '-' + decimal digits (Arrow's strict integer parser: no '+', no
//     spaces, no empty strings), overflow detected; ok[i] = 0 marks a row that does not parse,
//     ok[i] = 2 a hex literal (Arrow's host parser takes those).
//   * string -> float64: [+-] digits [. digits] [(e|E) [+-] digits].  Clinger's fast path is
//     exact: a mantissa of <= 19 significant digits that is < 2^53 times a power of ten |e| <= 22
//     (both exactly representable) rounds once, i.e. correctly.  Anything else that parses
//     (longer mantissas, large exponents, inf / nan spellings) reports ok[i] = 2 and the caller
//     converts that column on the host with Arrow -- results never depend on the path.
//   * int64 -> string: lengths, device scan, digits (one thread per row).
// Reference: pycylon Table.astype (python/pycylon/pycylon/data/table.pyx:2188-2232), Arrow cast
// kernels on the host.
#include "device_common.hpp"
#include "strparse.hpp"

namespace cylon {
namespace hip {

using strparse::sc_i64_len;
using strparse::sc_parse_f64;
using strparse::sc_parse_i64;

__global__ void k_str_to_i64(ColView c, int64_t n, int64_t *__restrict__ out, uint8_t *__restrict__ ok) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    int64_t v = 0;
    uint8_t r = 1;
    if (!c.valid || c.valid[i]) r = sc_parse_i64(c.data + c.offsets[i], c.offsets[i + 1] - c.offsets[i], &v);
    out[i] = v;
    ok[i] = r;
  }
}

__global__ void k_str_to_f64(ColView c, int64_t n, double *__restrict__ out, uint8_t *__restrict__ ok) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    double v = 0.0;
    uint8_t r = 1;
    if (!c.valid || c.valid[i]) r = sc_parse_f64(c.data + c.offsets[i], c.offsets[i + 1] - c.offsets[i], &v);
    out[i] = v;
    ok[i] = r;
  }
}

__global__ void k_i64_to_str_lengths(const int64_t *__restrict__ v, const uint8_t *__restrict__ valid, int64_t n,
                                     int64_t *__restrict__ lens) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
    lens[i] = (valid && !valid[i]) ? 0 : sc_i64_len(v[i]);
}

__global__ void k_i64_to_str_write(const int64_t *__restrict__ v, const uint8_t *__restrict__ valid, int64_t n,
                                   const int64_t *__restrict__ offs, uint8_t *__restrict__ bytes) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    if (valid && !valid[i]) continue;
    strparse::sc_i64_write(v[i], bytes + offs[i + 1]);
  }
}

void str_to_i64(const ColView &c, int64_t n, int64_t *out, uint8_t *ok, void *stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_str_to_i64, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), c, n, out, ok);
  HIP_LAUNCH_CHECK();
}

void str_to_f64(const ColView &c, int64_t n, double *out, uint8_t *ok, void *stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_str_to_f64, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), c, n, out, ok);
  HIP_LAUNCH_CHECK();
}

void i64_to_str_lengths(const int64_t *v, const uint8_t *valid, int64_t n, int64_t *lens, void *stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_i64_to_str_lengths, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), v, valid, n, lens);
  HIP_LAUNCH_CHECK();
}

void i64_to_str_write(const int64_t *v, const uint8_t *valid, int64_t n, const int64_t *offs, uint8_t *bytes,
                      void *stream) {
  if (n == 0) return;
  hipLaunchKernelGGL(k_i64_to_str_write, dim3(grid_for(n)), dim3(kBlock), 0, as_stream(stream), v, valid, n, offs,
                     bytes);
  HIP_LAUNCH_CHECK();
}

// this file's code object is loaded at context creation (preload_device_code), not on first use
void preload_strcast() { preload_code(reinterpret_cast<const void *>(&k_str_to_i64)); }

}  // namespace hip
}  // namespace cylon
