// Small dense factorisations that stay on the GPU (k <= 64): no host round
// trip inside power / Krylov iterations.
//
//   sl_small_chol_inv: G (k x k, f64, SPD) -> R upper (G = R^T R), R^{-1} (f64)
//                      and an f32 copy of R^{-1}; status[0] |= 1 when a pivot
//                      is not positive (the pivot is then replaced by a large
//                      value, which zeroes that direction, and the caller
//                      re-runs the robust host path after checking status).
//                      One register-resident elimination of [G | I] on a
//                      256-thread workgroup (k_aug_elim_chol_inv below).
//   sl_chol_inv_wave:  the same factor on ONE wave (sl_wave_la.hpp), the
//                      kernel the randSVD pass boundaries run.
//   sl_small_matmul:   C = A B for small f64 matrices (one workgroup).
// Reference counterpart: El::Cholesky / El::Trsm on [*,*] matrices inside
// nla/svd.hpp and ml/krr.hpp.
#include "sl_common.hpp"
#include "sl_wave_la.hpp"
#include <stdlib.h>

namespace {
constexpr int KM = 64;

// Register-resident elimination of the augmented matrix [G | I]:
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
  // register-resident augmented elimination, padded to the next multiple of 16
  // (measured on MI355X against the earlier LDS workgroup and single-wave
  // variants, profiles/small_la_stamps_r3*.jsonl)
  if (k <= 16) k_aug_elim_chol_inv<16><<<1, 256, 0, s>>>(G, k, ldg, R, Rinv, Rinv32, status);
  else if (k <= 32) k_aug_elim_chol_inv<32><<<1, 256, 0, s>>>(G, k, ldg, R, Rinv, Rinv32, status);
  else if (k <= 48) k_aug_elim_chol_inv<48><<<1, 256, 0, s>>>(G, k, ldg, R, Rinv, Rinv32, status);
  else k_aug_elim_chol_inv<64><<<1, 256, 0, s>>>(G, k, ldg, R, Rinv, Rinv32, status);
  SL_LAUNCH_CHECK();
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
// V: 0 one wave, 1 rows over 4 waves, 2 / 3 two pivots per step over 4 / 8
// waves, 4 / 5 four pivots per step over 4 / 8 waves
template <int K, int V>
__global__ void __launch_bounds__(V == 3 || V == 5 ? 512 : 256) k_chol_inv_wave(const double* __restrict__ G, int k, int ldg,
                                                       double* __restrict__ X, int* __restrict__ status) {
  __shared__ __attribute__((aligned(16))) double fsh[576];
  __shared__ int st;
  if (threadIdx.x == 0) st = 0;
  __syncthreads();
  if constexpr (V == 1) slw::wg_chol_inv<K, 4>(G, ldg, X, k, k, fsh, &st);
  else if constexpr (V == 2) slw::wg_chol_invB<K, 4, 2>(G, ldg, X, k, k, fsh, &st);
  else if constexpr (V == 3) slw::wg_chol_invB<K, 8, 2>(G, ldg, X, k, k, fsh, &st);
  else if constexpr (V == 4) slw::wg_chol_invB<K, 4, 4>(G, ldg, X, k, k, fsh, &st);
  else if constexpr (V == 5) slw::wg_chol_invB<K, 8, 4>(G, ldg, X, k, k, fsh, &st);
  else if (threadIdx.x < 64) slw::wave_chol_inv<K>(G, ldg, X, k, k, fsh, &st);
  __syncthreads();
  if (threadIdx.x == 0 && status && st) atomicOr(status, st);
}
// 4: four pivots per step, rows over 4 waves (default: k = 40 12.5 us, k = 64
// 24.7 us against 14.0 / 40.4 for one pivot per step, profiles/r6/chol_wave_ab.jsonl);
// 1: one pivot per step over 4 waves for K <= 48 (64 on one wave), 0: one wave,
// 2 / 3 / 5: two pivots over 4 / 8 waves, four over 8 (A/B)
int g_chol_variant = 4;

// 64 < k <= 128: rows of [G | I] over NG = 8 row groups of two waves each,
// four pivots per block (sl_wave_la.hpp wg_chol_invW)
template <int K>
__global__ void __launch_bounds__(1024) k_chol_inv_wide(const double* __restrict__ G, int k, int ldg,
                                                        double* __restrict__ X, int* __restrict__ status) {
  __shared__ __attribute__((aligned(16))) double fsh[2 * 4 * 128 + 136];
  __shared__ int st;
  if (threadIdx.x == 0) st = 0;
  __syncthreads();
  slw::wg_chol_invW<K, 8, 4>(G, ldg, X, k, k, fsh, &st);
  __syncthreads();
  if (threadIdx.x == 0 && status && st) atomicOr(status, st);
}
}  // namespace

SL_API void sl_chol_inv_set_variant(int v) { g_chol_variant = v; }

SL_API int sl_chol_inv_wave(const double* G, int k, int ldg, double* X, int* status, void* stream) {
  if (k < 1 || k > 128 || ldg < k) { sl_set_last_error("chol_inv_wave: 1 <= k <= 128"); return SL_ERR_DIMENSION; }
  hipStream_t s = (hipStream_t)stream;
  if (k > 64) {
    if (k <= 96) k_chol_inv_wide<96><<<1, 1024, 0, s>>>(G, k, ldg, X, status);
    else k_chol_inv_wide<128><<<1, 1024, 0, s>>>(G, k, ldg, X, status);
    SL_LAUNCH_CHECK();
    return SL_OK;
  }
#define SL_CIW(KK)                                                                                      \
  if (g_chol_variant == 5) k_chol_inv_wave<KK, 5><<<1, 512, 0, s>>>(G, k, ldg, X, status);               \
  else if (g_chol_variant == 4) k_chol_inv_wave<KK, 4><<<1, 256, 0, s>>>(G, k, ldg, X, status);          \
  else if (g_chol_variant == 3) k_chol_inv_wave<KK, 3><<<1, 512, 0, s>>>(G, k, ldg, X, status);          \
  else if (g_chol_variant == 2) k_chol_inv_wave<KK, 2><<<1, 256, 0, s>>>(G, k, ldg, X, status);          \
  else if (g_chol_variant && KK <= 48) k_chol_inv_wave<KK, 1><<<1, 256, 0, s>>>(G, k, ldg, X, status);   \
  else k_chol_inv_wave<KK, 0><<<1, 64, 0, s>>>(G, k, ldg, X, status);
  if (k <= 16) { SL_CIW(16) }
  else if (k <= 32) { SL_CIW(32) }
  else if (k <= 40) { SL_CIW(40) }
  else if (k <= 48) { SL_CIW(48) }
  else { SL_CIW(64) }
#undef SL_CIW
  SL_LAUNCH_CHECK();
  return SL_OK;
}
