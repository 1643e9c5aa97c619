// Random-row gather for the FETCH_SIZE / random-access calibration
// (benchmarks/pmc_calibrate.py --op rgather128 / rgather64): every thread
// copies U rows' 16-B chunks, all U loads issued before the stores, so a
// wave keeps U x 64 random 16-B pieces in flight.  Not part of the library;
// built by benchmarks/calib/build.sh into libcalib.so.
#include <hip/hip_runtime.h>
#include <cstdint>

namespace {
constexpr int U = 8;
__global__ void __launch_bounds__(256) k_rgather(const float4* __restrict__ table, const int64_t* __restrict__ idx,
                                                 int64_t nidx, int row16, float4* __restrict__ out) {
  const int64_t chunks = nidx * row16;
  const int64_t t0 = ((int64_t)blockIdx.x * 256 + threadIdx.x);
  const int64_t stride = (int64_t)gridDim.x * 256;
  float4 v[U];
  int64_t dst[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int64_t t = t0 + u * stride;
    dst[u] = t < chunks ? t : -1;
    const int64_t r = t < chunks ? t / row16 : 0;
    const int c = (int)(t - r * row16);
    v[u] = table[idx[r] * row16 + (t < chunks ? c : 0)];
  }
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (dst[u] >= 0) out[dst[u]] = v[u];
}
}  // namespace

extern "C" int calib_rgather(const void* table, const int64_t* idx, int64_t nidx, int row_bytes, void* out,
                             void* stream) {
  const int row16 = row_bytes / 16;
  const int64_t chunks = nidx * row16;
  const int64_t grid = (chunks + 256LL * U - 1) / (256LL * U);
  k_rgather<<<(unsigned)grid, 256, 0, (hipStream_t)stream>>>((const float4*)table, idx, nidx, row16, (float4*)out);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
