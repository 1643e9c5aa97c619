// Counter-based random streams for libskylark_amd (host + gfx950 device).
//
// Behavioural parity target: libSkylark's context/random-array model
// (reference base/randgen.hpp:17-122, base/context.hpp:94-165):
//   * a stream is (seed, counter); allocating `size` samples reserves the
//     counter range [counter, counter + size) and advances the counter;
//   * element i of an allocated array is a pure function of
//     (seed, base + i), so any GPU / rank can realise any entry of a random
//     matrix without communication.
//
// The generator is Threefry-2x64 with 13 rounds (Random123 constants), keyed
// by {seed, 0} and counted by {base + i, j}: j = 0, 1, ... indexes further
// 128-bit blocks of the same element (rejection samplers such as the gamma /
// chi-squared draw use more than one block).  The samplers on top are our
// own, documented below; they do not reproduce Boost.Random bit-for-bit (see
// SURVEY.md 5.4), but the counter/key layout is the reference's.
//
// Everything here is `__host__ __device__` so the CPU plumbing path and the
// HIP kernels share one definition.
#pragma once
#include <stdint.h>
#include <math.h>

#if defined(__HIPCC__)
#define SL_HD __host__ __device__ __forceinline__
#else
#define SL_HD inline
#endif

namespace sl {

// ---------------------------------------------------------------- Threefry
struct u64x2 { uint64_t x, y; };

SL_HD uint64_t rotl64(uint64_t v, int r) { return (v << r) | (v >> (64 - r)); }

// rotl64 by a constant: on the device two v_alignbit_b32 (a funnel shift of
// the two 32-bit halves; the generic form compiled to a 64-bit shift, a
// 32-bit shift and two ORs), the same bits
template <int R>
SL_HD uint64_t rotl64c(uint64_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
  if constexpr (R == 32) {
    return ((uint64_t)lo << 32) | hi;
  } else if constexpr (R < 32) {
    const uint32_t nh = __builtin_amdgcn_alignbit(hi, lo, 32 - R);
    const uint32_t nl = __builtin_amdgcn_alignbit(lo, hi, 32 - R);
    return ((uint64_t)nh << 32) | nl;
  } else {   // rotate the swapped halves by R - 32
    const uint32_t nh = __builtin_amdgcn_alignbit(lo, hi, 64 - R);
    const uint32_t nl = __builtin_amdgcn_alignbit(hi, lo, 64 - R);
    return ((uint64_t)nh << 32) | nl;
  }
#else
  return rotl64(v, R);
#endif
}

// Threefry-2x64-13.  Rotation constants R_64x2 and key-schedule parity are the
// published Random123 / Skein values.
SL_HD u64x2 threefry2x64_13(uint64_t c0, uint64_t c1, uint64_t k0, uint64_t k1) {
  const uint64_t k2 = 0x1BD11BDAA9FC1A22ULL ^ k0 ^ k1;
  uint64_t x0 = c0 + k0, x1 = c1 + k1;
#define SL_TF_R(r) { x0 += x1; x1 = rotl64c<r>(x1); x1 ^= x0; }
  SL_TF_R(16) SL_TF_R(42) SL_TF_R(12) SL_TF_R(31)
  x0 += k1; x1 += k2 + 1;
  SL_TF_R(16) SL_TF_R(32) SL_TF_R(24) SL_TF_R(21)
  x0 += k2; x1 += k0 + 2;
  SL_TF_R(16) SL_TF_R(42) SL_TF_R(12) SL_TF_R(31)
  x0 += k0; x1 += k1 + 3;
  SL_TF_R(16)
#undef SL_TF_R
  return {x0, x1};
}

SL_HD u64x2 stream_block(uint64_t seed, uint64_t idx, uint64_t sub = 0) {
  return threefry2x64_13(idx, sub, seed, 0ULL);
}

// -------------------------------------------------------- bit -> uniform
// Uniforms on the OPEN interval (0,1): never 0 (safe for log), never 1.
SL_HD double u01_d(uint64_t b) { return ((double)(b >> 11) + 0.5) * 0x1.0p-53; }
SL_HD float u01_f(uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  // the 24-bit value through ONE 32-bit convert (the compiler folded the cast
  // back into its 64-bit -> f32 sequence, five instructions), same value
  const uint32_t x = (uint32_t)(b >> 32) >> 8;
  float f;
  asm("v_cvt_f32_u32 %0, %1" : "=v"(f) : "v"(x));
  return (f + 0.5f) * 0x1.0p-24f;
#else
  return ((float)(uint32_t)(b >> 40) + 0.5f) * 0x1.0p-24f;
#endif
}

// Unbiased-enough uniform integer in [lo, hi] via 64x64->128 multiply-high
// (bias < range / 2^64).
SL_HD uint64_t mulhi64(uint64_t a, uint64_t b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __umul64hi(a, b);
#else
  return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}
SL_HD int64_t uniform_int(uint64_t b, int64_t lo, int64_t hi) {
  uint64_t range = (uint64_t)(hi - lo) + 1ULL;
  return lo + (int64_t)mulhi64(b, range);
}

// ------------------------------------------------------------ samplers
// Distribution ids are part of the C ABI (capi) and the Python layer.
enum Dist : int {
  DIST_NORMAL = 0,      // N(0,1)
  DIST_CAUCHY = 1,      // standard Cauchy
  DIST_RADEMACHER = 2,  // +-1
  DIST_UNIFORM = 3,     // U(a, b)           (p0 = a, p1 = b)
  DIST_EXPONENTIAL = 4, // Exp(1)
  DIST_LEVY = 5,        // standard Levy = 1 / Z^2 (reference: 1/Gamma(1/2, 2))
  DIST_CHISQ = 6,       // chi-squared, p0 = degrees of freedom
  DIST_UNIFORM_INT = 7, // integer in [p0, p1]
  DIST_WZT = 8,         // +-(1/E)^(1/p), p0 = p  (Woodruff-Zhang value)
  DIST_SPARSE_SIGN = 9, // +-1/sqrt(d) w.p. d/2 each, else 0; p0 = d (sparse JL, Achlioptas / Li et al.)
};

// Normal: Box-Muller on the two 64-bit words of element idx's first block.
SL_HD double normal_d(uint64_t seed, uint64_t idx) {
  u64x2 b = stream_block(seed, idx);
  double r = sqrt(-2.0 * log(u01_d(b.x)));
  return r * cos(6.283185307179586476925 * u01_d(b.y));
}

SL_HD float normal_f(uint64_t seed, uint64_t idx) {
  u64x2 b = stream_block(seed, idx);
#if defined(__HIP_DEVICE_COMPILE__)
  // v_log_f32 is log2; v_cos_f32 takes revolutions (x * 2pi).
  float r = __builtin_sqrtf(-2.0f * 0.69314718056f * __builtin_amdgcn_logf(u01_f(b.x)));
  return r * __builtin_amdgcn_cosf(u01_f(b.y));
#else
  float r = sqrtf(-2.0f * logf(u01_f(b.x)));
  return r * cosf(6.2831853071795865f * u01_f(b.y));
#endif
}

// Marsaglia-Tsang gamma(shape, 1) for shape >= 1; uses blocks sub = 0, 1, ...
SL_HD double gamma_d(uint64_t seed, uint64_t idx, double shape) {
  double boost = 1.0;
  uint64_t sub = 0;
  if (shape < 1.0) {
    // gamma(a) = gamma(a+1) * U^(1/a): U from a dedicated block.
    u64x2 b = stream_block(seed, idx, 0x7fffffffULL);
    boost = pow(u01_d(b.x), 1.0 / shape);
    shape += 1.0;
  }
  const double d = shape - 1.0 / 3.0, c = 1.0 / sqrt(9.0 * d);
  for (int it = 0; it < 64; ++it) {
    u64x2 b0 = stream_block(seed, idx, sub++);
    u64x2 b1 = stream_block(seed, idx, sub++);
    double z = sqrt(-2.0 * log(u01_d(b0.x))) * cos(6.283185307179586 * u01_d(b0.y));
    double v = 1.0 + c * z;
    if (v <= 0.0) continue;
    v = v * v * v;
    double u = u01_d(b1.x);
    if (log(u) < 0.5 * z * z + d - d * v + d * log(v)) return boost * d * v;
  }
  return boost * d;  // practically unreachable (acceptance > 0.95 per try)
}

SL_HD double sample_d(int dist, uint64_t seed, uint64_t idx, double p0, double p1) {
  switch (dist) {
    case DIST_NORMAL: return normal_d(seed, idx);
    case DIST_CAUCHY: {
      u64x2 b = stream_block(seed, idx);
      return tan(3.14159265358979323846 * (u01_d(b.x) - 0.5));
    }
    case DIST_RADEMACHER: {
      u64x2 b = stream_block(seed, idx);
      return (b.x >> 63) ? 1.0 : -1.0;
    }
    case DIST_UNIFORM: {
      u64x2 b = stream_block(seed, idx);
      return p0 + (p1 - p0) * u01_d(b.x);
    }
    case DIST_EXPONENTIAL: {
      u64x2 b = stream_block(seed, idx);
      return -log(u01_d(b.x));
    }
    case DIST_LEVY: {
      double z = normal_d(seed, idx);
      return 1.0 / (z * z);
    }
    case DIST_CHISQ: return 2.0 * gamma_d(seed, idx, 0.5 * p0);
    case DIST_UNIFORM_INT: {
      u64x2 b = stream_block(seed, idx);
      return (double)uniform_int(b.x, (int64_t)p0, (int64_t)p1);
    }
    case DIST_WZT: {
      u64x2 b = stream_block(seed, idx);
      double e = -log(u01_d(b.x));
      double v = pow(1.0 / e, 1.0 / p0);
      return (b.y >> 63) ? v : -v;
    }
    case DIST_SPARSE_SIGN: {
      u64x2 b = stream_block(seed, idx);
      double u = u01_d(b.x);
      if (u >= p0) return 0.0;
      return (u < 0.5 * p0 ? -1.0 : 1.0) / sqrt(p0);
    }
  }
  return 0.0;
}

// Single-precision fast path used inside GEMM prologues.  Distributions
// without a dedicated float sampler go through the double one.
SL_HD float sample_f(int dist, uint64_t seed, uint64_t idx, float p0, float p1) {
  switch (dist) {
    case DIST_NORMAL: return normal_f(seed, idx);
    case DIST_RADEMACHER: {
      u64x2 b = stream_block(seed, idx);
      return (b.x >> 63) ? 1.0f : -1.0f;
    }
    case DIST_CAUCHY: {
      u64x2 b = stream_block(seed, idx);
#if defined(__HIP_DEVICE_COMPILE__)
      // tan(pi (u - 1/2)) = sin / cos with revolutions = (u - 1/2)/2
      float t = 0.5f * (u01_f(b.x) - 0.5f);
      return __builtin_amdgcn_sinf(t) / __builtin_amdgcn_cosf(t);
#else
      return tanf(3.14159265358979f * (u01_f(b.x) - 0.5f));
#endif
    }
    case DIST_UNIFORM: {
      u64x2 b = stream_block(seed, idx);
      return p0 + (p1 - p0) * u01_f(b.x);
    }
    case DIST_SPARSE_SIGN: {
      u64x2 b = stream_block(seed, idx);
      float u = u01_f(b.x);
      if (u >= p0) return 0.0f;
      return (u < 0.5f * p0 ? -1.0f : 1.0f) * __builtin_sqrtf(1.0f / p0);
    }
    default: return (float)sample_d(dist, seed, idx, p0, p1);
  }
}

// ---------------------------------------------------------- Halton (QMC)
// Leaped Halton sequence (reference base/quasirand.hpp:35-60):
// coordinate(idx, i) = RadicalInverse(prime_i, idx * leap).
SL_HD double radical_inverse(uint64_t base, uint64_t n) {
  double inv = 1.0 / (double)base, f = inv, r = 0.0;
  while (n > 0) {
    r += f * (double)(n % base);
    n /= base;
    f *= inv;
  }
  return r;
}

}  // namespace sl
