// Shared helpers for the libskylark_amd native library (gfx950 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stddef.h>

#define SL_API extern "C" __attribute__((visibility("default")))

// dtype codes shared with Python (libskylark_amd/ops/_lib.py)
enum SlDtype : int { SL_F32 = 0, SL_F64 = 1, SL_BF16 = 2, SL_F16 = 3 };

// error codes (mirrors the reference's exception codes, base/exception.hpp)
enum SlError : int {
  SL_OK = 0,
  SL_ERR_GENERIC = 100,
  SL_ERR_UNSUPPORTED = 103,
  SL_ERR_DIMENSION = 104,
  SL_ERR_HIP = 106,
  SL_ERR_INVALID = 109,
};

#define SL_HIP_CHECK(expr)                                   \
  do {                                                        \
    hipError_t _e = (expr);                                   \
    if (_e != hipSuccess) { sl_set_last_error(hipGetErrorString(_e)); return SL_ERR_HIP; } \
  } while (0)

#define SL_LAUNCH_CHECK() SL_HIP_CHECK(hipGetLastError())

void sl_set_last_error(const char* msg);

// hipFuncSetAttribute(MaxDynamicSharedMemorySize, bytes) once per (kernel, device)
int sl_lds_attr(const void* fn, int bytes);
#define SL_LDS_ATTR(fn, bytes)                                   \
  do {                                                           \
    const int _rc = sl_lds_attr((const void*)(fn), (int)(bytes)); \
    if (_rc != SL_OK) return _rc;                                \
  } while (0)

typedef uint16_t bf16_t;

__host__ __device__ __forceinline__ float bf16_to_f(bf16_t v) {
  union { uint32_t u; float f; } c;
  c.u = ((uint32_t)v) << 16;
  return c.f;
}
__host__ __device__ __forceinline__ bf16_t f_to_bf16(float f) {
  union { uint32_t u; float f; } c;
  c.f = f;
  uint32_t u = c.u;
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return (bf16_t)((u >> 16) | 0x40);  // NaN stays NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (bf16_t)(u >> 16);
}

template <typename T> struct Cvt;
template <> struct Cvt<float> {
  __host__ __device__ static float to_f(float v) { return v; }
  __host__ __device__ static float from_f(float v) { return v; }
  __host__ __device__ static double to_d(float v) { return v; }
  __host__ __device__ static float from_d(double v) { return (float)v; }
};
template <> struct Cvt<double> {
  __host__ __device__ static float to_f(double v) { return (float)v; }
  __host__ __device__ static double from_f(float v) { return v; }
  __host__ __device__ static double to_d(double v) { return v; }
  __host__ __device__ static double from_d(double v) { return v; }
};
template <> struct Cvt<bf16_t> {
  __host__ __device__ static float to_f(bf16_t v) { return bf16_to_f(v); }
  __host__ __device__ static bf16_t from_f(float v) { return f_to_bf16(v); }
  __host__ __device__ static double to_d(bf16_t v) { return bf16_to_f(v); }
  __host__ __device__ static bf16_t from_d(double v) { return f_to_bf16((float)v); }
};

// Grid sizing for grid-stride memory-bound kernels: enough blocks to fill the
// 256 CUs several times over, capped (Guideline 11 of the CDNA HIP guide).
static inline unsigned sl_grid_for(size_t work, unsigned block, unsigned cap = 2048) {
  size_t g = (work + block - 1) / block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (unsigned)g;
}

#define SL_DISPATCH_FLOAT(dtype, T, ...)                      \
  switch (dtype) {                                            \
    case SL_F32: { typedef float T; __VA_ARGS__; break; }     \
    case SL_F64: { typedef double T; __VA_ARGS__; break; }    \
    case SL_BF16: { typedef bf16_t T; __VA_ARGS__; break; }   \
    default: sl_set_last_error("unsupported dtype"); return SL_ERR_UNSUPPORTED; \
  }
