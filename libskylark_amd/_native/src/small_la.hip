// Small dense factorisations that stay on the GPU (k <= 64): no host round
// trip inside power / Krylov iterations.
//
//   sl_small_chol_inv: G (k x k, f64, SPD) -> R upper (G = R^T R), R^{-1} (f64)
//                      and an f32 copy of R^{-1}; status[0] |= 1 when a pivot
//                      is not positive (the pivot is then replaced by a large
//                      value, which zeroes that direction, and the caller
//                      re-runs the robust host path after checking status).
//   sl_small_matmul:   C = A B for small f64 matrices (one workgroup).
//
// One workgroup of 256 threads, matrices in LDS, right-looking Cholesky with
// one barrier per column, column-parallel back substitution for R^{-1}.
// Reference counterpart: El::Cholesky / El::Trsm on [*,*] matrices inside
// nla/svd.hpp and ml/krr.hpp.
#include "sl_common.hpp"

namespace {
constexpr int KM = 64;
int g_chol_impl = 0;

__global__ void __launch_bounds__(256)
k_small_chol_inv(const double* __restrict__ G, int k, int ldg, double* __restrict__ R, double* __restrict__ Rinv,
                 float* __restrict__ Rinv32, int* __restrict__ status) {
  __shared__ double a[KM][KM + 1];
  __shared__ double x[KM][KM + 1];
  __shared__ int bad;
  const int t = threadIdx.x;
  if (t == 0) bad = 0;
  for (int e = t; e < k * k; e += 256) {
    const int i = e / k, j = e % k;
    a[i][j] = 0.5 * (G[i * ldg + j] + G[j * ldg + i]);
  }
  __syncthreads();
  double dmax = 0.0;
  for (int i = 0; i < k; ++i) dmax = fmax(dmax, fabs(a[i][i]));
  // right-looking Cholesky: a becomes L (lower) in place
  for (int j = 0; j < k; ++j) {
    if (t == 0) {
      double d = a[j][j];
      if (!(d > 1e-14 * dmax)) {  // also catches NaN
        bad = 1;
        d = 1e300;  // kill this direction
      }
      a[j][j] = sqrt(d);
    }
    __syncthreads();
    const double piv = a[j][j];
    for (int i = j + 1 + t; i < k; i += 256) a[i][j] /= piv;
    __syncthreads();
    // trailing update a[i][c] -= a[i][j] a[c][j], c <= i, i,c > j
    const int rem = k - j - 1;
    for (int e = t; e < rem * rem; e += 256) {
      const int i = j + 1 + e / rem, c = j + 1 + e % rem;
      if (c <= i) a[i][c] -= a[i][j] * a[c][j];
    }
    __syncthreads();
  }
  // X = L^{-1} by right-looking elimination (every step updates all remaining
  // entries in parallel: no serial dependency chain per thread); then
  // R^{-1} = (L^T)^{-1} = X^T.
  for (int e = t; e < k * k; e += 256) x[e / k][e % k] = (e / k == e % k) ? 1.0 : 0.0;
  __syncthreads();
  for (int j = 0; j < k; ++j) {
    const double inv = 1.0 / a[j][j];
    for (int c = t; c <= j; c += 256) x[j][c] *= inv;
    __syncthreads();
    const int rows = k - j - 1, cols = j + 1;
    for (int e = t; e < rows * cols; e += 256) {
      const int i = j + 1 + e / cols, c = e % cols;
      x[i][c] -= a[i][j] * x[j][c];
    }
    __syncthreads();
  }
  for (int e = t; e < k * k; e += 256) {
    const int i = e / k, j = e % k;
    const double r = (j >= i) ? a[j][i] : 0.0;
    if (R) R[i * k + j] = r;
    const double xi = (j >= i) ? x[j][i] : 0.0;  // R^{-1}[i][j] = (L^{-1})[j][i]
    if (Rinv) Rinv[i * k + j] = xi;
    if (Rinv32) Rinv32[i * k + j] = (float)xi;
  }
  if (t == 0 && bad && status) atomicOr(status, 1);
}

// Single-wave variant (k <= K <= 64): lane i keeps row i of the matrix in
// registers, every column broadcast is a pair of v_readlane_b32 (no LDS, no
// barriers), loops fully unrolled over the compile-time K.  Right-looking
// Cholesky, then X = L^{-1} by right-looking elimination, R = L^T, R^{-1} = X^T.
__device__ __forceinline__ double bcast(double v, int src) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, src);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), src);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

template <int K>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1)))
k_wave_chol_inv(const double* __restrict__ G, int k, int ldg, double* __restrict__ R, double* __restrict__ Rinv,
                float* __restrict__ Rinv32, int* __restrict__ status) {
  const int i = threadIdx.x;
  double a[K], x[K];
#pragma unroll
  for (int c = 0; c < K; ++c) {
    double v = 0.0;
    if (i < k && c < k) v = 0.5 * (G[i * ldg + c] + G[c * ldg + i]);
    else if (i == c) v = 1.0;  // identity padding keeps the factorisation regular
    a[c] = v;
    x[c] = (i == c) ? 1.0 : 0.0;
  }
  double dmax = 0.0;
#pragma unroll
  for (int c = 0; c < K; ++c) dmax = fmax(dmax, fabs(bcast(a[c], c)));
  int bad = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    double d = bcast(a[j], j);
    if (!(d > 1e-14 * dmax)) {
      bad |= (j < k);
      d = 1e300;
    }
    const double piv = sqrt(d);
    const double inv = 1.0 / piv;
    if (i == j) a[j] = piv;
    if (i > j) a[j] *= inv;
#pragma unroll
    for (int c = j + 1; c < K; ++c) {
      const double lcj = bcast(a[j], c);
      if (i > j) a[c] -= a[j] * lcj;
    }
  }
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const double ljj = bcast(a[j], j);
    if (i == j) {
#pragma unroll
      for (int c = 0; c <= j; ++c) x[c] /= ljj;
    }
#pragma unroll
    for (int c = 0; c <= j; ++c) {
      const double xjc = bcast(x[c], j);
      if (i > j) x[c] -= a[j] * xjc;
    }
  }
  if (i < k) {
#pragma unroll
    for (int c = 0; c < K; ++c) {
      if (c < k) {
        const double l = (c <= i) ? a[c] : 0.0;   // L[i][c] = R[c][i]
        const double xi = (c <= i) ? x[c] : 0.0;  // X[i][c] = R^{-1}[c][i]
        if (R) R[c * k + i] = l;
        if (Rinv) Rinv[c * k + i] = xi;
        if (Rinv32) Rinv32[c * k + i] = (float)xi;
      }
    }
  }
  if (i == 0 && bad && status) atomicOr(status, 1);
}

__global__ void __launch_bounds__(256)
k_small_matmul(const double* __restrict__ A, const double* __restrict__ B, double* __restrict__ C, int m, int kk,
               int n, float* __restrict__ C32) {
  for (int e = blockIdx.x * 256 + threadIdx.x; e < m * n; e += gridDim.x * 256) {
    const int i = e / n, j = e % n;
    double s = 0.0;
    for (int l = 0; l < kk; ++l) s += A[i * kk + l] * B[l * n + j];
    if (C) C[e] = s;
    if (C32) C32[e] = (float)s;
  }
}
}  // namespace

SL_API int sl_small_chol_inv(const double* G, int k, int ldg, double* R, double* Rinv, float* Rinv32, int* status,
                             void* stream) {
  if (k < 1 || k > KM) {
    sl_set_last_error("small_chol_inv: 1 <= k <= 64");
    return SL_ERR_UNSUPPORTED;
  }
  hipStream_t s = (hipStream_t)stream;
  if (g_chol_impl == 1)
    k_small_chol_inv<<<1, 256, 0, s>>>(G, k, ldg, R, Rinv, Rinv32, status);
  else if (k <= 16)
    k_wave_chol_inv<16><<<1, 64, 0, s>>>(G, k, ldg, R, Rinv, Rinv32, status);
  else if (k <= 32)
    k_wave_chol_inv<32><<<1, 64, 0, s>>>(G, k, ldg, R, Rinv, Rinv32, status);
  else if (k <= 48)
    k_wave_chol_inv<48><<<1, 64, 0, s>>>(G, k, ldg, R, Rinv, Rinv32, status);
  else
    k_wave_chol_inv<64><<<1, 64, 0, s>>>(G, k, ldg, R, Rinv, Rinv32, status);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// tuning/testing hook: 0 = single-wave register kernel (default), 1 = LDS workgroup kernel
SL_API int sl_small_chol_impl(int impl) {
  g_chol_impl = impl;
  return SL_OK;
}

SL_API int sl_small_matmul(const double* A, const double* B, double* C, int m, int kk, int n, float* C32,
                           void* stream) {
  if (m <= 0 || n <= 0) return SL_OK;
  int blocks = (m * n + 255) / 256;
  if (blocks > 1024) blocks = 1024;
  k_small_matmul<<<blocks, 256, 0, (hipStream_t)stream>>>(A, B, C, m, kk, n, C32);
  SL_LAUNCH_CHECK();
  return SL_OK;
}
