// Random-matrix realisation kernels (reference: base/random_matrices.hpp:23-171,
// sketch/dense_transform_data.hpp:79-101, base/randgen.hpp:98-116).
//
// Element (r, c) of a strided 2-D view receives
//     scale * sample(dist, seed, base + (r0 + r) * ir + (c0 + c) * ic)
// i.e. the stream index is computed from GLOBAL coordinates, so a row/column
// shard on any GPU reproduces exactly the entries of the unsharded matrix.
#include "sl_common.hpp"
#include "sl_rng.hpp"
#include <thread>
#include <vector>
#include <string.h>

static thread_local char g_last_error[512] = "";
void sl_set_last_error(const char* msg) {
  strncpy(g_last_error, msg, sizeof(g_last_error) - 1);
  g_last_error[sizeof(g_last_error) - 1] = 0;
}
SL_API const char* sl_last_error() { return g_last_error; }

struct FillArgs {
  int dist;
  uint64_t seed, base;
  int64_t rows, cols, sr, sc;  // view shape and element strides
  int64_t r0, c0, ir, ic;      // global offsets and stream strides
  double p0, p1, scale;
};

template <typename T, bool FAST>
__global__ void __launch_bounds__(256) k_fill_random(T* __restrict__ out, FillArgs a) {
  const int64_t total = a.rows * a.cols;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    // iterate the faster-varying output dimension fastest for coalescing
    int64_t r, c;
    if (a.sc == 1 || (a.sr != 1 && a.sc < a.sr)) { r = t / a.cols; c = t - r * a.cols; }
    else { c = t / a.rows; r = t - c * a.rows; }
    uint64_t idx = a.base + (uint64_t)((a.r0 + r) * a.ir + (a.c0 + c) * a.ic);
    if (FAST) {
      float v = sl::sample_f(a.dist, a.seed, idx, (float)a.p0, (float)a.p1);
      out[r * a.sr + c * a.sc] = Cvt<T>::from_f((float)a.scale * v);
    } else {
      double v = sl::sample_d(a.dist, a.seed, idx, a.p0, a.p1);
      out[r * a.sr + c * a.sc] = Cvt<T>::from_d(a.scale * v);
    }
  }
}

// Fast N(0,1) realisation for views whose fast dimension is contiguous (the
// dense-sketch panels: LSRN's 2e4 x 1.3e4 bf16 panels, 2.5e10 normals per
// 1.25e6-row sketch).  Same samples bit for bit as k_fill_random<T, true>;
// what changes is the index arithmetic: each thread owns 8 consecutive
// elements of one line (one 32-bit divide per 8 samples instead of a 64-bit
// divide + multiplies per sample), the stream index advances by an add, and
// the 8 results leave as one 16-B (bf16) or two 16-B (f32) stores.
template <typename T>
__global__ void __launch_bounds__(256) k_fill_normal_lines(T* __restrict__ out, uint64_t seed, uint64_t base0,
                                                           uint32_t nlines, uint32_t ngrp, int64_t nfast, int64_t ld,
                                                           int64_t s_line, int64_t s_fast, float scale) {
  const uint32_t total = nlines * ngrp;
  for (uint32_t t = blockIdx.x * 256u + threadIdx.x; t < total; t += gridDim.x * 256u) {
    const uint32_t l = t / ngrp, g = t - l * ngrp;
    const int64_t f = (int64_t)g * 8;
    uint64_t idx = base0 + (uint64_t)((int64_t)l * s_line + f * s_fast);
    float v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[j] = scale * sl::normal_f(seed, idx);
      idx += (uint64_t)s_fast;
    }
    T* p = out + (int64_t)l * ld + f;
    if (f + 8 <= nfast && (((uintptr_t)p) & 15) == 0) {
      if constexpr (sizeof(T) == 2) {
        // hardware round-to-nearest-even pairs (v_cvt_pk_bf16_f32): the same
        // bits as f_to_bf16's software RNE for the finite normals here
        typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
        typedef __attribute__((ext_vector_type(2))) float f32x2_t;
        uint32_t w[4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
          w[j] = __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2_t){v[2 * j], v[2 * j + 1]}, bf16x2_t));
        *(uint4*)p = make_uint4(w[0], w[1], w[2], w[3]);
      } else {
        *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
        *(float4*)(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (f + j < nfast) p[j] = Cvt<T>::from_f(v[j]);
    }
  }
}


// precise != 0 forces the double-precision sampler for fp32/bf16 outputs.
SL_API int sl_fill_random(void* out, int dtype, int dist, uint64_t seed, uint64_t base,
                          int64_t rows, int64_t cols, int64_t sr, int64_t sc, int64_t r0,
                          int64_t c0, int64_t ir, int64_t ic, double p0, double p1,
                          double scale, int precise, void* stream) {
  if (rows <= 0 || cols <= 0) return SL_OK;
  FillArgs a{dist, seed, base, rows, cols, sr, sc, r0, c0, ir, ic, p0, p1, scale};
  unsigned grid = sl_grid_for((size_t)(rows * cols), 256, 4096);
  hipStream_t s = (hipStream_t)stream;
  if (dist == sl::DIST_NORMAL && !precise && (dtype == SL_F32 || dtype == SL_BF16) && (sc == 1 || sr == 1)) {
    // lines = the slow dimension, fast = the contiguous one
    const bool rowmajor = sc == 1 && (sr != 1 || cols >= rows);
    const int64_t nlines = rowmajor ? rows : cols, nfast = rowmajor ? cols : rows;
    const int64_t ld = rowmajor ? sr : sc, s_line = rowmajor ? ir : ic, s_fast = rowmajor ? ic : ir;
    const int64_t ngrp = (nfast + 7) / 8;
    if (nlines * ngrp < (int64_t)0x7fffffff) {
      const uint64_t base0 = base + (uint64_t)(r0 * ir + c0 * ic);
      const unsigned g2 = sl_grid_for((size_t)(nlines * ngrp), 256, 8192);
      if (dtype == SL_F32)
        k_fill_normal_lines<float><<<g2, 256, 0, s>>>((float*)out, seed, base0, (uint32_t)nlines, (uint32_t)ngrp, nfast,
                                                      ld, s_line, s_fast, (float)scale);
      else
        k_fill_normal_lines<bf16_t><<<g2, 256, 0, s>>>((bf16_t*)out, seed, base0, (uint32_t)nlines, (uint32_t)ngrp,
                                                       nfast, ld, s_line, s_fast, (float)scale);
      SL_LAUNCH_CHECK();
      return SL_OK;
    }
  }
  SL_DISPATCH_FLOAT(dtype, T, {
    if (dtype == SL_F64 || precise)
      k_fill_random<T, false><<<grid, 256, 0, s>>>((T*)out, a);
    else
      k_fill_random<T, true><<<grid, 256, 0, s>>>((T*)out, a);
  });
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// Host implementation (CPU plumbing path, reference-compatible layouts).
template <typename T>
static void host_fill(T* out, const FillArgs& a, bool fast) {
  const int64_t total = a.rows * a.cols;
  unsigned nt = std::thread::hardware_concurrency();
  if (nt < 1) nt = 1;
  if (nt > 16) nt = 16;
  if (total < 65536) nt = 1;
  auto work = [&](int64_t lo, int64_t hi) {
    for (int64_t t = lo; t < hi; ++t) {
      int64_t r = t / a.cols, c = t - r * a.cols;
      uint64_t idx = a.base + (uint64_t)((a.r0 + r) * a.ir + (a.c0 + c) * a.ic);
      if (fast)
        out[r * a.sr + c * a.sc] = Cvt<T>::from_f((float)a.scale * sl::sample_f(a.dist, a.seed, idx, (float)a.p0, (float)a.p1));
      else
        out[r * a.sr + c * a.sc] = Cvt<T>::from_d(a.scale * sl::sample_d(a.dist, a.seed, idx, a.p0, a.p1));
    }
  };
  if (nt == 1) { work(0, total); return; }
  std::vector<std::thread> th;
  int64_t chunk = (total + nt - 1) / nt;
  for (unsigned i = 0; i < nt; ++i) {
    int64_t lo = i * chunk, hi = lo + chunk < total ? lo + chunk : total;
    if (lo < hi) th.emplace_back(work, lo, hi);
  }
  for (auto& t : th) t.join();
}

SL_API int sl_fill_random_host(void* out, int dtype, int dist, uint64_t seed, uint64_t base,
                               int64_t rows, int64_t cols, int64_t sr, int64_t sc, int64_t r0,
                               int64_t c0, int64_t ir, int64_t ic, double p0, double p1,
                               double scale, int precise) {
  if (rows <= 0 || cols <= 0) return SL_OK;
  FillArgs a{dist, seed, base, rows, cols, sr, sc, r0, c0, ir, ic, p0, p1, scale};
  bool fast = !(dtype == SL_F64 || precise);
  SL_DISPATCH_FLOAT(dtype, T, { host_fill<T>((T*)out, a, fast); });
  return SL_OK;
}

// Uniform integers in [lo, hi] for stream slots base .. base + n - 1.
__global__ void k_random_int(int64_t* __restrict__ out, uint64_t seed, uint64_t base, int64_t n,
                             int64_t lo, int64_t hi) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    sl::u64x2 b = sl::stream_block(seed, base + (uint64_t)i);
    out[i] = sl::uniform_int(b.x, lo, hi);
  }
}

SL_API int sl_random_int(int64_t* out, uint64_t seed, uint64_t base, int64_t n, int64_t lo,
                         int64_t hi, void* stream) {
  if (n <= 0) return SL_OK;
  k_random_int<<<sl_grid_for(n, 256), 256, 0, (hipStream_t)stream>>>(out, seed, base, n, lo, hi);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

SL_API int sl_random_int_host(int64_t* out, uint64_t seed, uint64_t base, int64_t n, int64_t lo,
                              int64_t hi) {
  for (int64_t i = 0; i < n; ++i) {
    sl::u64x2 b = sl::stream_block(seed, base + (uint64_t)i);
    out[i] = sl::uniform_int(b.x, lo, hi);
  }
  return SL_OK;
}

// Raw Threefry blocks (tests: host == device bitwise, known-answer vectors).
__global__ void k_threefry(uint64_t* out, uint64_t seed, uint64_t base, int64_t n) {
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) {
    sl::u64x2 b = sl::stream_block(seed, base + (uint64_t)i);
    out[2 * i] = b.x;
    out[2 * i + 1] = b.y;
  }
}
SL_API int sl_threefry(uint64_t* out, uint64_t seed, uint64_t base, int64_t n, void* stream) {
  if (n <= 0) return SL_OK;
  k_threefry<<<(unsigned)((n + 255) / 256), 256, 0, (hipStream_t)stream>>>(out, seed, base, n);
  SL_LAUNCH_CHECK();
  return SL_OK;
}
SL_API int sl_threefry_host(uint64_t* out, uint64_t c0, uint64_t c1, uint64_t k0, uint64_t k1) {
  sl::u64x2 b = sl::threefry2x64_13(c0, c1, k0, k1);
  out[0] = b.x;
  out[1] = b.y;
  return SL_OK;
}

// Leaped Halton block: out[i, d] = RadicalInverse(prime[d], (skip + i) * leap).
__global__ void k_halton(double* out, const int64_t* primes, int64_t n, int64_t d, int64_t skip,
                         int64_t leap) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n * d) {
    int64_t i = t / d, j = t - i * d;
    out[t] = sl::radical_inverse((uint64_t)primes[j], (uint64_t)((skip + i) * leap));
  }
}
SL_API int sl_halton_host(double* out, const int64_t* primes, int64_t n, int64_t d, int64_t skip,
                          int64_t leap) {
  for (int64_t i = 0; i < n; ++i)
    for (int64_t j = 0; j < d; ++j)
      out[i * d + j] = sl::radical_inverse((uint64_t)primes[j], (uint64_t)((skip + i) * leap));
  return SL_OK;
}
SL_API int sl_halton(double* out, const int64_t* primes, int64_t n, int64_t d, int64_t skip,
                     int64_t leap, void* stream) {
  if (n * d <= 0) return SL_OK;
  k_halton<<<(unsigned)((n * d + 255) / 256), 256, 0, (hipStream_t)stream>>>(out, primes, n, d, skip, leap);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

SL_API int sl_version() { return 1; }

// Inside-out Fisher-Yates draws (reference sketch/UST_data.hpp:88-96):
// out[i] = uniform_int(0, i) from stream slot base + i.
SL_API int sl_uniform_prefix_host(int64_t* out, uint64_t seed, uint64_t base, int64_t n) {
  for (int64_t i = 0; i < n; ++i) {
    sl::u64x2 b = sl::stream_block(seed, base + (uint64_t)i);
    out[i] = sl::uniform_int(b.x, 0, i);
  }
  return SL_OK;
}
