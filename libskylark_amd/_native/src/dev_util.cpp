// Device memory / stream helpers of the C ABI (so a C caller of the
// interpreter-free device paths needs nothing but this library): allocation,
// copies, fills, stream sync.  kind: 0 host->device, 1 device->host,
// 2 device->device.
#include <hip/hip_runtime.h>

#include "sl_common.hpp"

SL_API int sl_dev_malloc(int64_t bytes, void** out) {
  *out = nullptr;
  if (bytes <= 0) return SL_OK;
  SL_HIP_CHECK(hipMalloc(out, (size_t)bytes));
  return SL_OK;
}

SL_API int sl_dev_free(void* p) {
  if (p) SL_HIP_CHECK(hipFree(p));
  return SL_OK;
}

SL_API int sl_dev_memcpy(void* dst, const void* src, int64_t bytes, int kind, void* stream) {
  if (bytes <= 0) return SL_OK;
  const hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice : kind == 1 ? hipMemcpyDeviceToHost
                                                                        : hipMemcpyDeviceToDevice;
  SL_HIP_CHECK(hipMemcpyAsync(dst, src, (size_t)bytes, k, (hipStream_t)stream));
  if (kind != 2) SL_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
  return SL_OK;
}

SL_API int sl_dev_memset(void* dst, int value, int64_t bytes, void* stream) {
  if (bytes <= 0) return SL_OK;
  SL_HIP_CHECK(hipMemsetAsync(dst, value, (size_t)bytes, (hipStream_t)stream));
  return SL_OK;
}

SL_API int sl_dev_sync(void* stream) {
  SL_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
  return SL_OK;
}

SL_API int sl_dev_set_device(int dev) {
  SL_HIP_CHECK(hipSetDevice(dev));
  return SL_OK;
}
