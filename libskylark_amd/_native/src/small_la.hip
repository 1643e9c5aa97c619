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
#include "sl_wave_la.hpp"
#include <stdlib.h>

namespace {
constexpr int KM = 64;
int g_chol_impl = -1;  // -1: read SL_CHOL_IMPL once (default 0)

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

// Workgroup variant with ONE barrier per elimination step.  Cholesky: step j
// reads the (already updated) pivot a[j][j], updates the trailing matrix
// from the UNSCALED column j (a[i][c] -= a[i][j] a[c][j] / d), and scales
// column j of the previous step (never read again) in the same phase.
// Inverse X = L^{-1}: step j subtracts L[i][j] * (x[j][c] / L[j][j]) from the
// rows below using the unscaled row j, and scales row j-1 meanwhile.
__global__ void __launch_bounds__(256)
k_small_chol_inv1b(const double* __restrict__ G, int k, int ldg, double* __restrict__ R, double* __restrict__ Rinv,
                   float* __restrict__ Rinv32, int* __restrict__ status) {
  __shared__ double a[KM][KM + 1];
  __shared__ double x[KM][KM + 1];
  const int t = threadIdx.x;
  for (int e = t; e < k * k; e += 256) {
    const int i = e / k, j = e % k;
    a[i][j] = 0.5 * (G[i * ldg + j] + G[j * ldg + i]);
    x[i][j] = (i == j) ? 1.0 : 0.0;
  }
  __syncthreads();
  double dmax = 0.0;
  for (int i = 0; i < k; ++i) dmax = fmax(dmax, fabs(a[i][i]));
  int bad = 0;
  double pinv_prev = 0.0;  // 1/sqrt(d_{j-1}) for the deferred column scaling
  for (int j = 0; j <= k; ++j) {
    double d = 1.0, dinv = 0.0, pinv = 0.0;
    if (j < k) {
      d = a[j][j];
      if (!(d > 1e-14 * dmax)) {
        bad = 1;
        d = 1e300;
      }
      dinv = 1.0 / d;
      pinv = sqrt(dinv);
    }
    // deferred scaling of column j-1 (rows > j-1) and its pivot
    if (j > 0) {
      const int jp = j - 1;
      for (int i = jp + 1 + t; i < k; i += 256) a[i][jp] *= pinv_prev;
      if (t == 0) a[jp][jp] = 1.0 / pinv_prev;  // sqrt(d) (or 1e150 for a killed pivot)
    }
    if (j < k) {
      const int rem = k - j - 1;
      for (int e = t; e < rem * rem; e += 256) {
        const int i = j + 1 + e / rem, c = j + 1 + e % rem;
        if (c <= i) a[i][c] -= a[i][j] * a[c][j] * dinv;
      }
    }
    pinv_prev = pinv;
    __syncthreads();
  }
  // a now holds L (lower, diagonal sqrt(d_j)).
  for (int j = 0; j <= k; ++j) {
    if (j > 0) {  // scale row j-1 of X by 1 / L[j-1][j-1]
      const int jp = j - 1;
      const double inv = 1.0 / a[jp][jp];
      for (int c = t; c <= jp; c += 256) x[jp][c] *= inv;
    }
    if (j < k) {
      const double inv = 1.0 / a[j][j];
      const int rows = k - j - 1, cols = j + 1;
      for (int e = t; e < rows * cols; e += 256) {
        const int i = j + 1 + e / cols, c = e % cols;
        x[i][c] -= a[i][j] * (x[j][c] * inv);
      }
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

// Single-wave variant (k <= K <= 64), no barriers:
//   Cholesky: lane i keeps row i of the matrix in registers; per column j the
//   pivot column is published through a 64-double LDS vector and read back as
//   wave-uniform (broadcast) LDS reads, so the k dependent steps cost a few
//   LDS round trips each instead of long v_readlane chains.
//   Inverse:  L is written to LDS once; lane c then forward-substitutes
//   column c of X = L^{-1} (all columns in parallel) with broadcast reads of
//   L.  R = L^T, R^{-1} = X^T.  Loops are unrolled over the compile-time K so
//   the per-lane rows stay in registers.
template <int K>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1)))
k_wave_chol_inv(const double* __restrict__ G, int k, int ldg, double* __restrict__ R, double* __restrict__ Rinv,
                float* __restrict__ Rinv32, int* __restrict__ status) {
  __shared__ double colv[64];
  __shared__ double L[K][K + 1];
  const int i = threadIdx.x;
  double a[K];
#pragma unroll
  for (int c = 0; c < K; ++c) {
    double v = 0.0;
    if (i < k && c < k) v = 0.5 * (G[i * ldg + c] + G[c * ldg + i]);
    else if (i == c) v = 1.0;  // identity padding keeps the factorisation regular
    a[c] = v;
  }
  // max diagonal (for the relative pivot test)
  double diag = 0.0;
#pragma unroll
  for (int c = 0; c < K; ++c)
    if (i == c) diag = a[c];
  colv[i] = fabs(diag);
  double dmax = 0.0;
#pragma unroll
  for (int c = 0; c < K; ++c) dmax = fmax(dmax, colv[c]);
  int bad = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    colv[i] = a[j];
    double d = colv[j];
    if (!(d > 1e-14 * dmax)) {
      bad |= (j < k);
      d = 1e300;
    }
    const double piv = sqrt(d);
    const double lij = (i == j) ? piv : a[j] / piv;
    a[j] = (i >= j) ? lij : a[j];
    colv[i] = lij;
#pragma unroll
    for (int c = j + 1; c < K; ++c) {
      const double lcj = colv[c];
      if (i > j) a[c] -= lij * lcj;
    }
  }
  if (i < K) {
#pragma unroll
    for (int c = 0; c < K; ++c) L[i][c] = (c <= i) ? a[c] : 0.0;
  }
  // column c = i of X = L^{-1}: x_r = (delta_rc - sum_{c<=s<r} L[r][s] x_s) / L[r][r]
  double x[K];
#pragma unroll
  for (int r = 0; r < K; ++r) {
    double acc = (r == i) ? 1.0 : 0.0;
#pragma unroll
    for (int s2 = 0; s2 < r; ++s2) acc -= L[r][s2] * x[s2];
    x[r] = (r >= i) ? acc / L[r][r] : 0.0;
  }
  if (i < k) {
#pragma unroll
    for (int c = 0; c < K; ++c) {
      if (c < k) {
        const double l = (c <= i) ? a[c] : 0.0;  // L[i][c] = R[c][i]
        if (R) R[c * k + i] = l;
        if (Rinv) Rinv[i * k + c] = x[c];      // X[c][i] = R^{-1}[i][c]
        if (Rinv32) Rinv32[i * k + c] = (float)x[c];
      }
    }
  }
  if (i == 0 && bad && status) atomicOr(status, 1);
}

// Compact single-wave variant: the same algorithm with the matrix in LDS and
// rolled loops (a few hundred bytes of code instead of tens of KB of fully
// unrolled straight-line code, which a cold instruction cache fetches at
// every launch).  Lane i owns row i during the factorisation and column i
// of X = L^{-1} during the inversion; all cross-lane values are wave-uniform
// LDS broadcast reads, and one wave needs no barriers.
__global__ void __launch_bounds__(64)
k_wave_chol_inv_rolled(const double* __restrict__ G, int k, int ldg, double* __restrict__ R,
                       double* __restrict__ Rinv, float* __restrict__ Rinv32, int* __restrict__ status) {
  __shared__ double a[KM][KM + 1];
  __shared__ double x[KM][KM + 1];
  const int i = threadIdx.x;
  double dmax = 0.0;
  if (i < k) {
    for (int c = 0; c < k; ++c) a[i][c] = 0.5 * (G[i * ldg + c] + G[c * ldg + i]);
  }
  for (int c = 0; c < k; ++c) dmax = fmax(dmax, fabs(a[c][c]));
  int bad = 0;
  for (int j = 0; j < k; ++j) {
    double d = a[j][j];
    if (!(d > 1e-14 * dmax)) {
      bad = 1;
      d = 1e300;
    }
    const double piv = sqrt(d);
    const double inv = 1.0 / piv;
    double lij = 0.0;
    if (i > j && i < k) {
      lij = a[i][j] * inv;
      a[i][j] = lij;
    }
    if (i == j) a[j][j] = piv;
    if (i > j && i < k) {
#pragma unroll 4
      for (int c = j + 1; c <= i; ++c) a[i][c] -= lij * a[c][j];
    }
  }
  // X = L^{-1}, lane c owns column c
  for (int r = 0; r < k; ++r) {
    double acc = (r == i) ? 1.0 : 0.0;
#pragma unroll 4
    for (int s2 = 0; s2 < r; ++s2) acc -= a[r][s2] * ((s2 >= i) ? x[s2][i] : 0.0);
    if (i < k) x[r][i] = (r >= i) ? acc / a[r][r] : 0.0;
  }
  if (i < k) {
    for (int c = 0; c < k; ++c) {
      const double l = (c <= i) ? a[i][c] : 0.0;  // L[i][c] = R[c][i]
      if (R) R[c * k + i] = l;
      const double xi = x[c][i];                    // X[c][i] = R^{-1}[i][c]
      if (Rinv) Rinv[i * k + c] = xi;
      if (Rinv32) Rinv32[i * k + c] = (float)xi;
    }
  }
  if (i == 0 && bad && status) atomicOr(status, 1);
}

// Register-resident elimination of the augmented matrix [G | I] (impl 5):
// Gaussian elimination without pivoting turns [G | I] into [D L_u^T | L_u^{-1}]
// (G = L_u D L_u^T), so R = D^{-1/2} (left part) and R^{-1} = (right part)^T
// D^{-1/2} come out of ONE k-step elimination instead of a factorisation
// followed by a triangular inversion.  The 64 x 128 augmented matrix lives in
// registers, 2-D cyclic over a 16 x 16 thread grid (32 doubles per thread).
// The trailing block stays symmetric, so the multipliers of step j are the
// pivot row itself: step j publishes row j (final from then on) into its own
// LDS slot, one barrier, and every thread reads the 13 values it needs.  No
// slot is ever rewritten, so one barrier per step is race free, and the slots
// hold the whole eliminated matrix for the final output pass.
// KA = padded size (16, 32, 48 or 64): thread (tr, tc) of the 16 x 16 grid
// holds rows tr + 16 a and columns tc + 16 b of both halves (NA = KA / 16 of
// each), so a k = 40 matrix does 9 + 9 FMAs per thread per step instead of
// the 64-padded 16 + 16; the pivot reciprocal is v_rcp_f64 + one Newton step.
template <int KA>
__global__ void __launch_bounds__(256)
k_aug_elim_chol_inv(const double* __restrict__ G, int k, int ldg, double* __restrict__ R,
                    double* __restrict__ Rinv, float* __restrict__ Rinv32, int* __restrict__ status) {
  constexpr int NA = KA / 16;
  __shared__ double rows[KA][2 * KA];
  __shared__ double dsh[KA];
  const int t = threadIdx.x, tr = t >> 4, tc = t & 15;
  __shared__ double diag[KA];
  double m[NA][2 * NA];
  // diagonal staged through LDS: a rolled loop of k global loads here waited
  // on one load at a time (~0.7 us each -> most of the kernel's 37 us)
  if (t < k) diag[t] = fabs(G[t * ldg + t]);
#pragma unroll
  for (int a = 0; a < NA; ++a) {
    const int i = tr + 16 * a;
#pragma unroll
    for (int b = 0; b < NA; ++b) {
      const int c = tc + 16 * b;
      double v = (i == c) ? 1.0 : 0.0;
      if (i < k && c < k) v = 0.5 * (G[i * ldg + c] + G[c * ldg + i]);
      m[a][b] = v;
      m[a][NA + b] = (i == c) ? 1.0 : 0.0;
    }
  }
  __syncthreads();
  double dmax = 0.0;
  for (int c = 0; c < k; ++c) dmax = fmax(dmax, diag[c]);
  int bad = 0;
  for (int j = 0; j < k; ++j) {
    const int ja = j >> 4;
    if (tr == (j & 15)) {
#pragma unroll
      for (int a = 0; a < NA; ++a)
        if (a == ja) {
#pragma unroll
          for (int b = 0; b < NA; ++b) {
            rows[j][tc + 16 * b] = m[a][b];
            rows[j][KA + tc + 16 * b] = m[a][NA + b];
          }
        }
    }
    __syncthreads();
    double d = rows[j][j];
    if (!(d > 1e-14 * dmax)) {  // also catches NaN: kill this direction
      bad = 1;
      d = 1e300;
    }
    double dinv = __builtin_amdgcn_rcp(d);
    dinv = fma(fma(-d, dinv, 1.0), dinv, dinv);
    double mult[NA], rv[2 * NA];
#pragma unroll
    for (int a = 0; a < NA; ++a) {
      const int i = tr + 16 * a;
      mult[a] = (i > j) ? rows[j][i] * dinv : 0.0;
    }
#pragma unroll
    for (int b = 0; b < NA; ++b) {
      rv[b] = rows[j][tc + 16 * b];
      rv[NA + b] = rows[j][KA + tc + 16 * b];
    }
#pragma unroll
    for (int a = 0; a < NA; ++a)
#pragma unroll
      for (int b = 0; b < 2 * NA; ++b) m[a][b] = fma(-mult[a], rv[b], m[a][b]);
    if (t == j) dsh[j] = d;
  }
  __syncthreads();
  // R[i][c] = U[i][c] / sqrt(d_i) (c >= i; the diagonal is sqrt(d_i) itself, which also
  // gives 1e150 for a killed pivot); R^{-1}[i][c] = X[c][i] / sqrt(d_c) (c >= i).
  for (int e = t; e < k * k; e += 256) {
    const int i = e / k, c = e % k;
    double r = 0.0, ri = 0.0;
    if (c >= i) {
      const double si = sqrt(dsh[i]);
      r = (c == i) ? si : rows[i][c] / si;
      ri = rows[c][KA + i] / sqrt(dsh[c]);
    }
    if (R) R[e] = r;
    if (Rinv) Rinv[e] = ri;
    if (Rinv32) Rinv32[e] = (float)ri;
  }
  if (t == 0 && bad && status) atomicOr(status, 1);
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
  if (g_chol_impl < 0) {
    const char* e = getenv("SL_CHOL_IMPL");
    g_chol_impl = e ? atoi(e) : 0;
  }
  // measured on MI355X (rocprof, k x k f64): k<=16 single wave 10 us; k=40:
  // workgroup 61 us vs wave 57; k=64: wave 95 vs workgroup 121 -> pick per size
  int impl = g_chol_impl;
  if (impl == 0) impl = 5;
  if (impl == 5) {
    if (k <= 16) k_aug_elim_chol_inv<16><<<1, 256, 0, s>>>(G, k, ldg, R, Rinv, Rinv32, status);
    else if (k <= 32) k_aug_elim_chol_inv<32><<<1, 256, 0, s>>>(G, k, ldg, R, Rinv, Rinv32, status);
    else if (k <= 48) k_aug_elim_chol_inv<48><<<1, 256, 0, s>>>(G, k, ldg, R, Rinv, Rinv32, status);
    else k_aug_elim_chol_inv<64><<<1, 256, 0, s>>>(G, k, ldg, R, Rinv, Rinv32, status);
  }
  else if (impl == 1)
    k_small_chol_inv<<<1, 256, 0, s>>>(G, k, ldg, R, Rinv, Rinv32, status);
  else if (impl == 4)
    k_small_chol_inv1b<<<1, 256, 0, s>>>(G, k, ldg, R, Rinv, Rinv32, status);
  else if (impl == 2)
    k_wave_chol_inv_rolled<<<1, 64, 0, s>>>(G, k, ldg, R, Rinv, Rinv32, status);
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

// tuning/testing hook: 0 = auto (default), 1 = LDS workgroup kernel, 2 = single-wave rolled LDS
// kernel, 3 = single-wave register kernel, 4 = one-barrier-per-step workgroup kernel,
// 5 = register-resident augmented elimination
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

// ------------------------------------------------------------------------
// X = R^{-1} (upper) of G = R^T R (k <= 64) by one wave with the matrix in
// registers (sl_wave_la.hpp wave_chol_inv: in-place LDL^T of [G | I]); the
// kernel the randSVD pass boundaries run, as a standalone launch.  Status
// bit 1: a pivot at or below 1e-13 max G_ii was dropped.
namespace {
template <int K>
__global__ void __launch_bounds__(64) k_chol_inv_wave(const double* __restrict__ G, int k, int ldg,
                                                      double* __restrict__ X, int* __restrict__ status) {
  __shared__ __attribute__((aligned(16))) double fsh[192];
  __shared__ int st;
  if (threadIdx.x == 0) st = 0;
  __syncthreads();
  slw::wave_chol_inv<K>(G, ldg, X, k, k, fsh, &st);
  __syncthreads();
  if (threadIdx.x == 0 && status && st) atomicOr(status, st);
}
}  // namespace

SL_API int sl_chol_inv_wave(const double* G, int k, int ldg, double* X, int* status, void* stream) {
  if (k < 1 || k > 64 || ldg < k) { sl_set_last_error("chol_inv_wave: 1 <= k <= 64"); return SL_ERR_DIMENSION; }
  hipStream_t s = (hipStream_t)stream;
  if (k <= 16) k_chol_inv_wave<16><<<1, 64, 0, s>>>(G, k, ldg, X, status);
  else if (k <= 32) k_chol_inv_wave<32><<<1, 64, 0, s>>>(G, k, ldg, X, status);
  else if (k <= 40) k_chol_inv_wave<40><<<1, 64, 0, s>>>(G, k, ldg, X, status);
  else if (k <= 48) k_chol_inv_wave<48><<<1, 64, 0, s>>>(G, k, ldg, X, status);
  else k_chol_inv_wave<64><<<1, 64, 0, s>>>(G, k, ldg, X, status);
  SL_LAUNCH_CHECK();
  return SL_OK;
}
