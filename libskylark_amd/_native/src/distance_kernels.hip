// Kernel-Gram building blocks (reference ml/kernels.hpp gram/symmetric_gram,
// base/distance.hpp Euclidean / L1 / exp-semigroup distance matrices).
//
// Points are ROWS (X is m x d, Y is n x d, row-major, leading dims ldx/ldy);
// K is m x n row-major.
//
// * sl_pairwise_map: non-GEMM distances (L1: sum_k |x_k - y_k|, semigroup:
//   sum_k sqrt(x_k + y_k)) with an optional fused exp(-scale * D) epilogue
//   (Laplacian / exp-semigroup kernels).  These are VALU-bound: 64x64 output
//   tile per 256-thread workgroup, 4x4 micro-tile per thread, 32-wide d slabs
//   staged through LDS transposed (stride 65 -> conflict-free stores; reads
//   are a 4-address broadcast for X and 16 consecutive words for Y).
// * sl_gram_map: in-place epilogue over a GEMM result G = X Y^T (hipBLASLt /
//   MFMA): Gaussian exp(-(|x|^2 + |y|^2 - 2 G) * a) with the distance clamped
//   at 0, polynomial (a G + c)^q; one vectorised pass over K.
#include "sl_common.hpp"

namespace {

enum { PW_L1 = 0, PW_SEMIGROUP = 1 };
enum { GM_GAUSSIAN = 0, GM_POLYNOMIAL = 1, GM_EXPNEG = 2, GM_MATERN05 = 3, GM_MATERN15 = 4, GM_MATERN25 = 5 };

constexpr int TB = 64;   // output tile edge
constexpr int KC = 32;   // d slab
constexpr int LDS_LD = TB + 1;

template <typename T>
__device__ __forceinline__ T dev_sqrt(T x);
template <>
__device__ __forceinline__ float dev_sqrt<float>(float x) { return __builtin_sqrtf(x); }
template <>
__device__ __forceinline__ double dev_sqrt<double>(double x) { return __builtin_sqrt(x); }

template <typename T, int MODE, bool EXP>
__global__ void __launch_bounds__(256)
k_pairwise(const T* __restrict__ X, const T* __restrict__ Y, T* __restrict__ K, int64_t m, int64_t n,
           int64_t d, int64_t ldx, int64_t sdx, int64_t ldy, int64_t sdy, int64_t ldk, double scale) {
  __shared__ T xs[KC][LDS_LD];
  __shared__ T ys[KC][LDS_LD];
  const int tid = threadIdx.x;
  const int tx = tid & 15, ty = tid >> 4;
  const int64_t r0 = (int64_t)blockIdx.y * TB, c0 = (int64_t)blockIdx.x * TB;
  T acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = T(0);

  for (int64_t k0 = 0; k0 < d; k0 += KC) {
    // stage: 64 rows x 32 k of X and of Y; consecutive threads walk k (coalesced)
    // every load issued unconditionally from a clamped address, then zeroed:
    // `cond ? X[..] : 0` compiled to one exec-masked branch per load, each
    // waiting for its own load
    constexpr int NE = (TB * KC) / 256;
    T xl[NE], yl[NE];
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      const int flat = e * 256 + tid;
      const int kk = flat & (KC - 1), rr = flat / KC;
      const int64_t gk = k0 + kk < d ? k0 + kk : d - 1;
      const int64_t gx = r0 + rr < m ? r0 + rr : m - 1, gy = c0 + rr < n ? c0 + rr : n - 1;
      xl[e] = X[gx * ldx + gk * sdx];
      yl[e] = Y[gy * ldy + gk * sdy];
    }
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      asm volatile("" : "+v"(xl[e]));
      asm volatile("" : "+v"(yl[e]));
    }
#pragma unroll
    for (int e = 0; e < NE; ++e) {
      const int flat = e * 256 + tid;
      const int kk = flat & (KC - 1), rr = flat / KC;
      const bool kok = k0 + kk < d;
      xs[kk][rr] = (kok && r0 + rr < m) ? xl[e] : T(0);
      ys[kk][rr] = (kok && c0 + rr < n) ? yl[e] : T(0);
    }
    __syncthreads();
    const int kmax = (int)((d - k0) < KC ? (d - k0) : KC);
    for (int kk = 0; kk < kmax; ++kk) {
      T xv[4], yv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) xv[i] = xs[kk][ty + 16 * i];
#pragma unroll
      for (int j = 0; j < 4; ++j) yv[j] = ys[kk][tx + 16 * j];
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (MODE == PW_L1) acc[i][j] += __builtin_fabs(xv[i] - yv[j]);
          else acc[i][j] += dev_sqrt<T>(__builtin_fabs(xv[i] + yv[j]));
        }
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t r = r0 + ty + 16 * i;
    if (r >= m) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t c = c0 + tx + 16 * j;
      if (c >= n) continue;
      T v = acc[i][j];
      if (EXP) v = (sizeof(T) == 8) ? (T)exp(-scale * (double)v) : (T)__expf(-(float)scale * (float)v);
      K[r * ldk + c] = v;
    }
  }
}

template <typename T, int KIND>
__global__ void __launch_bounds__(256)
k_gram_map(T* __restrict__ K, int64_t m, int64_t n, int64_t ldk, const T* __restrict__ xn,
           const T* __restrict__ yn, double a, double c, double q) {
  const int64_t total = m * n;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = t / n, col = t - r * n;
    T* p = K + r * ldk + col;
    const T g = *p;
    if (KIND == GM_GAUSSIAN) {
      T dist = xn[r] + yn[col] - T(2) * g;
      dist = dist > T(0) ? dist : T(0);
      *p = (sizeof(T) == 8) ? (T)exp(-a * (double)dist) : (T)__expf(-(float)a * (float)dist);
    } else if (KIND == GM_POLYNOMIAL) {
      const double base = a * (double)g + c;
      *p = (sizeof(T) == 8) ? (T)pow(base, q) : (T)powf((float)base, (float)q);
    } else if (KIND == GM_EXPNEG) {
      *p = (sizeof(T) == 8) ? (T)exp(-a * (double)g) : (T)__expf(-(float)a * (float)g);
    } else {
      // Matern nu = 1/2, 3/2, 5/2 of r = |x - y| / l (a = 1 / l)
      double d2 = (double)xn[r] + (double)yn[col] - 2.0 * (double)g;
      const double rr = sqrt(d2 > 0.0 ? d2 : 0.0) * a;
      double v;
      if (KIND == GM_MATERN05) v = exp(-rr);
      else if (KIND == GM_MATERN15) { const double t = 1.7320508075688772 * rr; v = (1.0 + t) * exp(-t); }
      else { const double t = 2.23606797749979 * rr; v = (1.0 + t + t * t / 3.0) * exp(-t); }
      *p = (T)v;
    }
  }
}

template <typename T>
int launch_pairwise(const T* X, const T* Y, T* K, int64_t m, int64_t n, int64_t d, int64_t ldx, int64_t sdx,
                    int64_t ldy, int64_t sdy, int64_t ldk, int mode, double scale, hipStream_t s) {
  dim3 grid((unsigned)((n + TB - 1) / TB), (unsigned)((m + TB - 1) / TB));
  const bool ex = scale > 0;
#define SL_PW(MODE, EX) k_pairwise<T, MODE, EX><<<grid, 256, 0, s>>>(X, Y, K, m, n, d, ldx, sdx, ldy, sdy, ldk, scale)
  if (mode == PW_L1) {
    if (ex) SL_PW(PW_L1, true);
    else SL_PW(PW_L1, false);
  } else {
    if (ex) SL_PW(PW_SEMIGROUP, true);
    else SL_PW(PW_SEMIGROUP, false);
  }
#undef SL_PW
  return SL_OK;
}

// squared norms of m points (point stride sp, coordinate stride sd)
template <typename T>
__global__ void __launch_bounds__(256) k_point_sqnorms(const T* __restrict__ X, int64_t m, int64_t d, int64_t sp,
                                                       int64_t sd, T* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= m) return;
  double a = 0.0;
  for (int64_t c = lane; c < d; c += 64) {
    const double v = (double)X[i * sp + c * sd];
    a += v * v;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) a += __shfl_xor(a, o);
  if (lane == 0) out[i] = (T)a;
}

}  // namespace

// mode 0 = L1, 1 = exp-semigroup; scale > 0 fuses K = exp(-scale * D).
SL_API int sl_pairwise_map(const void* X, const void* Y, void* K, int dtype, int64_t m, int64_t n, int64_t d,
                           int64_t ldx, int64_t ldy, int64_t ldk, int mode, double scale, void* stream) {
  if (m <= 0 || n <= 0) return SL_OK;
  if ((m + TB - 1) / TB > 65535) { sl_set_last_error("pairwise: too many rows"); return SL_ERR_DIMENSION; }
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SL_F32)
    launch_pairwise<float>((const float*)X, (const float*)Y, (float*)K, m, n, d, ldx, 1, ldy, 1, ldk, mode, scale, s);
  else if (dtype == SL_F64)
    launch_pairwise<double>((const double*)X, (const double*)Y, (double*)K, m, n, d, ldx, 1, ldy, 1, ldk, mode, scale,
                            s);
  else
    { sl_set_last_error("pairwise: dtype must be f32/f64"); return SL_ERR_UNSUPPORTED; }
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// As sl_pairwise_map with general operand strides: point i, coordinate c of X
// at X[i * ldx + c * sdx] (columns-as-points operands need no transpose copy).
SL_API int sl_pairwise_map_strided(const void* X, int64_t ldx, int64_t sdx, const void* Y, int64_t ldy, int64_t sdy,
                                   void* K, int64_t ldk, int dtype, int64_t m, int64_t n, int64_t d, int mode,
                                   double scale, void* stream) {
  if (m <= 0 || n <= 0) return SL_OK;
  if ((m + TB - 1) / TB > 65535) { sl_set_last_error("pairwise: too many rows"); return SL_ERR_DIMENSION; }
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SL_F32)
    launch_pairwise<float>((const float*)X, (const float*)Y, (float*)K, m, n, d, ldx, sdx, ldy, sdy, ldk, mode, scale,
                           s);
  else if (dtype == SL_F64)
    launch_pairwise<double>((const double*)X, (const double*)Y, (double*)K, m, n, d, ldx, sdx, ldy, sdy, ldk, mode,
                            scale, s);
  else
    { sl_set_last_error("pairwise: dtype must be f32/f64"); return SL_ERR_UNSUPPORTED; }
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// out[i] = |x_i|^2 for m points of dimension d (point stride sp, coordinate stride sd)
SL_API int sl_point_sqnorms(const void* X, int dtype, int64_t m, int64_t d, int64_t sp, int64_t sd, void* out,
                            void* stream) {
  if (m <= 0) return SL_OK;
  const unsigned g = (unsigned)((m + 3) / 4);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SL_F32) k_point_sqnorms<float><<<g, 256, 0, s>>>((const float*)X, m, d, sp, sd, (float*)out);
  else if (dtype == SL_F64) k_point_sqnorms<double><<<g, 256, 0, s>>>((const double*)X, m, d, sp, sd, (double*)out);
  else { sl_set_last_error("point_sqnorms: dtype must be f32/f64"); return SL_ERR_UNSUPPORTED; }
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// kind 0 Gaussian (needs xn, yn = squared row norms; a = 1/(2 sigma^2)),
// kind 1 polynomial (a = gamma, c, q), kind 2 exp(-a K), kinds 3/4/5 Matern
// nu = 1/2, 3/2, 5/2 (xn, yn; a = 1/l).
SL_API int sl_gram_map(void* K, int dtype, int64_t m, int64_t n, int64_t ldk, const void* xn, const void* yn,
                       int kind, double a, double c, double q, void* stream) {
  if (m * n <= 0) return SL_OK;
  unsigned grid = sl_grid_for((size_t)(m * n), 256, 8192);
  hipStream_t s = (hipStream_t)stream;
#define SL_GM(T)                                                                                     \
  do {                                                                                               \
    if (kind == GM_GAUSSIAN)                                                                         \
      k_gram_map<T, GM_GAUSSIAN><<<grid, 256, 0, s>>>((T*)K, m, n, ldk, (const T*)xn, (const T*)yn, a, c, q); \
    else if (kind == GM_POLYNOMIAL)                                                                  \
      k_gram_map<T, GM_POLYNOMIAL><<<grid, 256, 0, s>>>((T*)K, m, n, ldk, (const T*)xn, (const T*)yn, a, c, q); \
    else if (kind == GM_MATERN05)                                                                    \
      k_gram_map<T, GM_MATERN05><<<grid, 256, 0, s>>>((T*)K, m, n, ldk, (const T*)xn, (const T*)yn, a, c, q); \
    else if (kind == GM_MATERN15)                                                                    \
      k_gram_map<T, GM_MATERN15><<<grid, 256, 0, s>>>((T*)K, m, n, ldk, (const T*)xn, (const T*)yn, a, c, q); \
    else if (kind == GM_MATERN25)                                                                    \
      k_gram_map<T, GM_MATERN25><<<grid, 256, 0, s>>>((T*)K, m, n, ldk, (const T*)xn, (const T*)yn, a, c, q); \
    else                                                                                             \
      k_gram_map<T, GM_EXPNEG><<<grid, 256, 0, s>>>((T*)K, m, n, ldk, (const T*)xn, (const T*)yn, a, c, q); \
  } while (0)
  if (dtype == SL_F32) SL_GM(float);
  else if (dtype == SL_F64) SL_GM(double);
  else { sl_set_last_error("gram_map: dtype must be f32/f64"); return SL_ERR_UNSUPPORTED; }
#undef SL_GM
  SL_LAUNCH_CHECK();
  return SL_OK;
}
