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

// rows x width_bytes block between pitched buffers (pitches in bytes), same kinds
SL_API int sl_dev_memcpy2d(void* dst, int64_t dpitch, const void* src, int64_t spitch, int64_t width_bytes,
                           int64_t rows, int kind, void* stream) {
  if (rows <= 0 || width_bytes <= 0) return SL_OK;
  const hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice : kind == 1 ? hipMemcpyDeviceToHost
                                                                        : hipMemcpyDeviceToDevice;
  SL_HIP_CHECK(hipMemcpy2DAsync(dst, (size_t)dpitch, src, (size_t)spitch, (size_t)width_bytes, (size_t)rows, k,
                                (hipStream_t)stream));
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

// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, device):
// a process that drives several GPUs (sl_dev_set_device) sets it on each.
#include <mutex>
#include <set>
#include <utility>

int sl_lds_attr(const void* fn, int bytes) {
  static std::mutex mu;
  static std::set<std::pair<const void*, int>> done;
  int dev = 0;
  SL_HIP_CHECK(hipGetDevice(&dev));
  std::lock_guard<std::mutex> g(mu);
  if (done.count({fn, dev})) return SL_OK;
  SL_HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  done.insert({fn, dev});
  return SL_OK;
}
