// Device NLA drivers of the C API's host-operand ("Matrix") paths, column-major
// like the reference's El::Matrix, every step on the GPU (rocBLAS GEMMs /
// GEMVs, rocSOLVER QR / eigensolver / SVD, small kernels here):
//
//   sl_nat_sym_rsvd     ApproximateSymmetricSVD (reference nla/svd.hpp:321-392;
//                       runtime nla/svd.py approximate_symmetric_svd): Gaussian
//                       Omega from the context stream (entry (i, j) at
//                       base + i + j n), Symm power iterations with Householder
//                       orthonormalisation, Rayleigh-Ritz with rocSOLVER syevd,
//                       eigenpairs by SIGNED value, descending
//   sl_nat_blendenpik   FasterLeastSquares (reference nla/least_squares.hpp,
//                       algorithms/regression/accelerated_*_Elemental.hpp;
//                       runtime algorithms/regression.py "blendenpik"): up to
//                       three FJLT sketches of 4n rows, R from Householder QR of
//                       S A, 1-norm condition check, preconditioned LSQR with
//                       the runtime's stopping rules (algorithms/krylov.py
//                       lsqr); exact SVD solve when every sketch is singular
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <vector>

#include "sl_blas.hpp"
#include "sl_common.hpp"
#include "sl_rng.hpp"

SL_API int sl_fill_random(void* out, int dtype, int dist, uint64_t seed, uint64_t base, int64_t rows, int64_t cols,
                          int64_t sr, int64_t sc, int64_t r0, int64_t c0, int64_t ir, int64_t ic, double p0, double p1,
                          double scale, int precise, void* stream);
SL_API int sl_symmetrize(const void* A, int dtype, int64_t n, int64_t lda, int lower, void* out, int64_t ldo,
                         void* stream);
SL_API int sl_dct2_rows(const int64_t* rows, int64_t S, int64_t N, const double* d, double scale, void* out,
                        int dtype, int64_t ld, int transpose, void* stream);
SL_API int sl_comm_all_reduce(void* comm, const void* send, void* recv, int64_t count, int dtype, int op,
                              void* stream);

namespace {

// column-major C (M x N) = op(A) op(B) (+ beta C) via the row-major wrapper
int gemm_cm(bool ta, bool tb, int64_t M, int64_t N, int64_t K, const double* A, int64_t lda, const double* B,
            int64_t ldb, double beta, double* C, int64_t ldc, hipStream_t s) {
  return slb_gemm(SL_F64, tb, ta, N, M, K, 1.0, B, ldb, A, lda, beta, C, ldc, s);
}

__global__ void k_sym_avg(double* B, int k) {
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < k * k; t += gridDim.x * blockDim.x) {
    const int i = t % k, j = t / k;
    if (i > j) {
      const double v = 0.5 * (B[i + j * k] + B[j + i * k]);
      B[i + j * k] = v;
      B[j + i * k] = v;
    }
  }
}

// V[:, j] = T[:, r - 1 - j] (reverse the ascending eigen order), s[j] = w[k - 1 - j]
__global__ void k_reverse_cols(const double* T, int64_t n, int r, double* V, int64_t ldv, const double* w, int k,
                               double* s) {
  const int64_t tot = n * r;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < tot; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = t % n, j = t / n;
    V[i + j * ldv] = T[i + (r - 1 - j) * n];
    if (i == 0) s[j] = w[k - 1 - j];
  }
}

// y = a x + b y
__global__ void k_axpby(int64_t n, double a, const double* x, double b, double* y) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (int64_t)gridDim.x * blockDim.x)
    y[t] = a * x[t] + b * y[t];
}

// R (n x n, ld n) = upper triangle of QR (ld lda), zeros below
__global__ void k_upper(const double* QR, int64_t lda, int64_t n, double* R) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n * n; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = t % n, j = t / n;
    R[i + j * n] = i <= j ? QR[i + j * lda] : 0.0;
  }
}

// column absolute sums (1-norm per column) of the column-major n x n T
__global__ void k_colabs(const double* T, int64_t n, double* out) {
  const int64_t j = blockIdx.x;
  double acc = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += blockDim.x) acc += fabs(T[i + j * n]);
  __shared__ double red[256];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[j] = red[0];
}

// X (n x nrhs) = V diag(sinv) U^T B: W = U^T B scaled by sinv rows
__global__ void k_scale_rows(double* W, int64_t r, int64_t c, int64_t ld, const double* s, double tol) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < r * c; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = t % r, j = t / r;
    W[i + j * ld] = s[i] > tol ? W[i + j * ld] / s[i] : 0.0;
  }
}

unsigned grid_of(int64_t n) { return (unsigned)std::min<int64_t>((n + 255) / 256 > 0 ? (n + 255) / 256 : 1, 8192); }

struct DevBuf {
  void* p = nullptr;
  explicit DevBuf(size_t bytes) {
    if (hipMalloc(&p, bytes ? bytes : 8) != hipSuccess) p = nullptr;
  }
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  double* d() const { return (double*)p; }
};

#define NAT_TRY(expr)                  \
  do {                                 \
    const int _rc = (expr);            \
    if (_rc != SL_OK) return _rc;      \
  } while (0)

int orth_inplace(double* X, int64_t m, int k, double* tau, hipStream_t s) {
  NAT_TRY(slb_dgeqrf_cm((int)m, k, X, (int)m, tau, s));
  return slb_dorgqr_cm((int)m, k, k, X, (int)m, tau, s);
}

}  // namespace

// A: column-major n x n (lda), only the `lower` (1) / upper (0) triangle read;
// V (n x rank, ldv) and s (rank) written, column-major, device memory.
SL_API int sl_nat_sym_rsvd(const double* A, int64_t n, int64_t lda, int lower, int k, int rank, int iters,
                           int skip_qr, uint64_t seed, uint64_t base, double* V, int64_t ldv, double* s_out,
                           void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (n < 1 || k < rank || rank < 1 || k > n) {
    sl_set_last_error("sym_rsvd: needs 1 <= rank <= k <= n");
    return SL_ERR_INVALID;
  }
  if (!slb_solver_available()) {
    sl_set_last_error("sym_rsvd: rocBLAS / rocSOLVER not available");
    return SL_ERR_UNSUPPORTED;
  }
  DevBuf As(sizeof(double) * n * n), X(sizeof(double) * n * k), Y(sizeof(double) * n * k), tau(sizeof(double) * k),
      Bk(sizeof(double) * k * k), w(sizeof(double) * k), E(sizeof(double) * k), T(sizeof(double) * n * rank),
      info(sizeof(int) * 4);
  if (!As.p || !X.p || !Y.p || !tau.p || !Bk.p || !w.p || !E.p || !T.p || !info.p) {
    sl_set_last_error("sym_rsvd: device allocation failed");
    return SL_ERR_HIP;
  }
  NAT_TRY(sl_symmetrize(A, SL_F64, n, lda, lower, As.p, n, s));
  NAT_TRY(sl_fill_random(X.p, SL_F64, sl::DIST_NORMAL, seed, base, n, k, 1, n, 0, 0, 1, n, 0.0, 0.0, 1.0, 1, s));
  NAT_TRY(gemm_cm(false, false, n, k, n, As.d(), n, X.d(), n, 0.0, Y.d(), n, s));   // V = A Omega
  for (int it = 0; it < iters; ++it) {
    if (!skip_qr) NAT_TRY(orth_inplace(Y.d(), n, k, tau.d(), s));
    NAT_TRY(gemm_cm(false, false, n, k, n, As.d(), n, Y.d(), n, 0.0, X.d(), n, s));
    std::swap(X.p, Y.p);
  }
  NAT_TRY(orth_inplace(Y.d(), n, k, tau.d(), s));                                      // Q
  NAT_TRY(gemm_cm(false, false, n, k, n, As.d(), n, Y.d(), n, 0.0, X.d(), n, s));      // U = A Q
  NAT_TRY(gemm_cm(true, false, k, k, n, Y.d(), n, X.d(), n, 0.0, Bk.d(), k, s));       // B = Q^T U
  k_sym_avg<<<grid_of((int64_t)k * k), 256, 0, s>>>(Bk.d(), k);
  SL_LAUNCH_CHECK();
  NAT_TRY(slb_dsyevd(k, Bk.d(), k, w.d(), E.d(), (int*)info.p, s));                    // ascending
  // T = Q E[:, k - rank : k], then columns reversed (descending signed order)
  NAT_TRY(gemm_cm(false, false, n, rank, k, Y.d(), n, Bk.d() + (int64_t)(k - rank) * k, k, 0.0, T.d(), n, s));
  k_reverse_cols<<<grid_of(n * rank), 256, 0, s>>>(T.d(), n, rank, V, ldv, w.d(), k, s_out);
  SL_LAUNCH_CHECK();
  int hinfo = 0;
  SL_HIP_CHECK(hipMemcpyAsync(&hinfo, info.p, sizeof(int), hipMemcpyDeviceToHost, s));
  SL_HIP_CHECK(hipStreamSynchronize(s));
  if (hinfo != 0) {
    sl_set_last_error("sym_rsvd: syevd did not converge");
    return SL_ERR_GENERIC;
  }
  return SL_OK;
}

namespace {

// T (m x n row-major, ld n) = the stored triangle of this rank's rows [r0, r0
// + m) of a symmetric A (row-major shard R, ld ldr): lower keeps columns j <=
// r0 + i, upper j >= r0 + i
__global__ void k_tri_rows(const double* __restrict__ R, int64_t ldr, int64_t m, int64_t n, int64_t r0, int lower,
                           double* __restrict__ T) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < m * n; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = t / n, j = t - i * n;
    const bool keep = lower ? j <= r0 + i : j >= r0 + i;
    T[t] = keep ? R[i * ldr + j] : 0.0;
  }
}

// F (n x k col-major) rows r0 .. r0 + m += P (m x k col-major) - diag(T) X rows
__global__ void k_fold_rows(double* __restrict__ F, int64_t n, int64_t m, int k, int64_t r0,
                            const double* __restrict__ P, const double* __restrict__ T, const double* __restrict__ X) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < m * k; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = t % m, c = t / m;
    const int64_t g = r0 + i;
    F[g + c * n] += P[i + c * m] - T[i * n + g] * X[g + c * n];
  }
}

}  // namespace

// ApproximateSymmetricSVD of a row-distributed symmetric A: this rank holds
// rows [r0, r0 + m) of the n x n A (row-major shard, ld ldr), only its lower
// (1) / upper (0) triangle read.  A X = L X + L^T X - D X over the stored
// triangle L: each rank forms its rows of L X - D X and its partial L^T X,
// and ONE n x k all-reduce per application of A gives A X on every rank; the
// orthonormalisation, the k x k Rayleigh-Ritz and V (n x rank, col-major,
// ldv) / s are replicated.  Same operator stream as sl_nat_sym_rsvd (the
// same Omega at base), so one rank reproduces the host-operand call.
SL_API int sl_nat_sym_rsvd_comm(const double* R, int64_t m, int64_t n, int64_t ldr, int64_t r0, int lower, int k,
                                int rank, int iters, int skip_qr, uint64_t seed, uint64_t base, double* V, int64_t ldv,
                                double* s_out, void* comm, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (n < 1 || k < rank || rank < 1 || k > n || m < 0 || r0 < 0 || r0 + m > n) {
    sl_set_last_error("sym_rsvd: needs 1 <= rank <= k <= n and a row range inside n");
    return SL_ERR_INVALID;
  }
  if (!slb_solver_available()) {
    sl_set_last_error("sym_rsvd: rocBLAS / rocSOLVER not available");
    return SL_ERR_UNSUPPORTED;
  }
  DevBuf T(sizeof(double) * std::max<int64_t>(1, m * n)), X(sizeof(double) * n * k), Y(sizeof(double) * n * k),
      P(sizeof(double) * std::max<int64_t>(1, m * k)), tau(sizeof(double) * k), Bk(sizeof(double) * k * k),
      w(sizeof(double) * k), E(sizeof(double) * k), T2(sizeof(double) * n * rank), info(sizeof(int) * 4);
  if (!T.p || !X.p || !Y.p || !P.p || !tau.p || !Bk.p || !w.p || !E.p || !T2.p || !info.p) {
    sl_set_last_error("sym_rsvd: device allocation failed");
    return SL_ERR_HIP;
  }
  if (m > 0) {
    k_tri_rows<<<grid_of(m * n), 256, 0, s>>>(R, ldr, m, n, r0, lower, T.d());
    SL_LAUNCH_CHECK();
  }
  // out (n x k col-major, every rank) = A in (n x k col-major, every rank)
  auto apply = [&](const double* in, double* out) -> int {
    if (m > 0) {
      NAT_TRY(gemm_cm(true, false, m, k, n, T.d(), n, in, n, 0.0, P.d(), m, s));        // rows of L X
      NAT_TRY(gemm_cm(false, false, n, k, m, T.d(), n, in + r0, n, 0.0, out, n, s));     // partial L^T X
      k_fold_rows<<<grid_of(m * k), 256, 0, s>>>(out, n, m, k, r0, P.d(), T.d(), in);
      SL_LAUNCH_CHECK();
    } else {
      SL_HIP_CHECK(hipMemsetAsync(out, 0, sizeof(double) * n * k, s));
    }
    if (!comm) return SL_OK;
    return sl_comm_all_reduce(comm, out, out, n * k, SL_F64, 0, s);
  };
  NAT_TRY(sl_fill_random(X.p, SL_F64, sl::DIST_NORMAL, seed, base, n, k, 1, n, 0, 0, 1, n, 0.0, 0.0, 1.0, 1, s));
  NAT_TRY(apply(X.d(), Y.d()));                                                          // Y = A Omega
  for (int it = 0; it < iters; ++it) {
    if (!skip_qr) NAT_TRY(orth_inplace(Y.d(), n, k, tau.d(), s));
    NAT_TRY(apply(Y.d(), X.d()));
    std::swap(X.p, Y.p);
  }
  NAT_TRY(orth_inplace(Y.d(), n, k, tau.d(), s));                                        // Q
  NAT_TRY(apply(Y.d(), X.d()));                                                          // U = A Q
  NAT_TRY(gemm_cm(true, false, k, k, n, Y.d(), n, X.d(), n, 0.0, Bk.d(), k, s));         // B = Q^T U
  k_sym_avg<<<grid_of((int64_t)k * k), 256, 0, s>>>(Bk.d(), k);
  SL_LAUNCH_CHECK();
  NAT_TRY(slb_dsyevd(k, Bk.d(), k, w.d(), E.d(), (int*)info.p, s));
  NAT_TRY(gemm_cm(false, false, n, rank, k, Y.d(), n, Bk.d() + (int64_t)(k - rank) * k, k, 0.0, T2.d(), n, s));
  k_reverse_cols<<<grid_of(n * rank), 256, 0, s>>>(T2.d(), n, rank, V, ldv, w.d(), k, s_out);
  SL_LAUNCH_CHECK();
  int hinfo = 0;
  SL_HIP_CHECK(hipMemcpyAsync(&hinfo, info.p, sizeof(int), hipMemcpyDeviceToHost, s));
  SL_HIP_CHECK(hipStreamSynchronize(s));
  if (hinfo != 0) {
    sl_set_last_error("sym_rsvd: syevd did not converge");
    return SL_ERR_GENERIC;
  }
  return SL_OK;
}

namespace {

// Row distribution of the least-squares operand: this rank holds rows
// [r0, r0 + m) of the mg-row A and B; comm (sl_comm_*) sums over the ranks,
// null = one rank.  Every n-vector / n x n quantity is replicated and, the
// sums being identical on every rank, bit-equal across ranks.
struct Dist {
  void* comm = nullptr;
  int64_t mg = 0, r0 = 0;
  double* scal = nullptr;   // device scratch (1 double) for scalar sums
};

int dsum(const Dist& D, double* dev, int64_t count, hipStream_t s) {
  if (!D.comm) return SL_OK;
  return sl_comm_all_reduce(D.comm, dev, dev, count, SL_F64, 0, s);
}

// 2-norm of a row-distributed vector (m local entries)
int nrm2_rows(const Dist& D, int64_t m, const double* u, double* out, hipStream_t s) {
  NAT_TRY(slb_dnrm2((int)m, u, out, s));
  if (!D.comm) return SL_OK;
  double sq = (*out) * (*out);
  SL_HIP_CHECK(hipMemcpyAsync(D.scal, &sq, sizeof(double), hipMemcpyHostToDevice, s));
  NAT_TRY(dsum(D, D.scal, 1, s));
  SL_HIP_CHECK(hipMemcpyAsync(&sq, D.scal, sizeof(double), hipMemcpyDeviceToHost, s));
  SL_HIP_CHECK(hipStreamSynchronize(s));
  *out = std::sqrt(sq);
  return SL_OK;
}

// runtime lsqr (algorithms/krylov.py) for one right-hand side, preconditioned
// by P = R^{-1} (explicit Rinv when given, else triangular solves with R); A,
// b, u row-distributed per D (m local rows), x, v, w, z, t replicated
int lsqr_one(const Dist& D, const double* A, int64_t m, int64_t n, int64_t lda, const double* b, double* x,
             const double* R, const double* Rinv, double tol, int iter_lim, int* code, double* u, double* v, double* w,
             double* z, double* t, hipStream_t s) {
  const double eps = 32 * DBL_EPSILON;
  if (tol < eps) tol = eps;
  if (tol >= 1.0) tol = 1 - eps;
  if (iter_lim < 0) iter_lim = std::max<int64_t>(20, 2 * std::min(D.mg, n));
  auto P = [&](double* vec) -> int {   // vec = R^{-1} vec (z = P v)
    if (Rinv) {
      NAT_TRY(slb_dgemv_cm(false, (int)n, (int)n, 1.0, Rinv, (int)n, vec, 0.0, t, s));
      SL_HIP_CHECK(hipMemcpyAsync(vec, t, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
      return SL_OK;
    }
    return slb_dtrsv_upper_cm(false, (int)n, R, (int)n, vec, s);
  };
  SL_HIP_CHECK(hipMemcpyAsync(u, b, sizeof(double) * m, hipMemcpyDeviceToDevice, s));
  SL_HIP_CHECK(hipMemsetAsync(x, 0, sizeof(double) * n, s));
  double beta = 0, alpha = 0;
  NAT_TRY(nrm2_rows(D, m, u, &beta, s));
  k_axpby<<<grid_of(m), 256, 0, s>>>(m, 0.0, u, 1.0 / std::max(beta, DBL_MIN), u);
  // v = P^T A^T u
  NAT_TRY(slb_dgemv_cm(true, (int)m, (int)n, 1.0, A, (int)lda, u, 0.0, t, s));
  NAT_TRY(dsum(D, t, n, s));
  if (Rinv) {
    NAT_TRY(slb_dgemv_cm(true, (int)n, (int)n, 1.0, Rinv, (int)n, t, 0.0, v, s));
  } else {
    SL_HIP_CHECK(hipMemcpyAsync(v, t, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
    NAT_TRY(slb_dtrsv_upper_cm(true, (int)n, R, (int)n, v, s));
  }
  NAT_TRY(slb_dnrm2((int)n, v, &alpha, s));
  k_axpby<<<grid_of(n), 256, 0, s>>>(n, 0.0, v, 1.0 / std::max(alpha, DBL_MIN), v);
  SL_HIP_CHECK(hipMemcpyAsync(z, v, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
  NAT_TRY(P(z));
  SL_HIP_CHECK(hipMemcpyAsync(w, z, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
  double nrm_a = 0, cnd_a = 0, sq_d = 0, nrm_r = beta, nrm_x = 0, sq_x = 0;
  const double nrm_ar_0 = alpha * beta;
  double phibar = beta, rhobar = alpha, cs2 = -1, sn2 = 0, zz = 0;
  int stag = 0;
  if (nrm_ar_0 == 0) {
    *code = -1;
    return SL_OK;
  }
  *code = -6;
  for (int itn = 0; itn < iter_lim; ++itn) {
    NAT_TRY(slb_dgemv_cm(false, (int)m, (int)n, 1.0, A, (int)lda, z, -alpha, u, s));   // u = A z - alpha u
    NAT_TRY(nrm2_rows(D, m, u, &beta, s));
    k_axpby<<<grid_of(m), 256, 0, s>>>(m, 0.0, u, 1.0 / beta, u);
    nrm_a = std::sqrt(nrm_a * nrm_a + alpha * alpha + beta * beta);
    NAT_TRY(slb_dgemv_cm(true, (int)m, (int)n, 1.0, A, (int)lda, u, 0.0, t, s));        // t = A^T u
    NAT_TRY(dsum(D, t, n, s));
    if (Rinv) {
      NAT_TRY(slb_dgemv_cm(true, (int)n, (int)n, 1.0, Rinv, (int)n, t, -beta, v, s));   // v = P^T t - beta v
    } else {
      NAT_TRY(slb_dtrsv_upper_cm(true, (int)n, R, (int)n, t, s));
      k_axpby<<<grid_of(n), 256, 0, s>>>(n, 1.0, t, -beta, v);
    }
    NAT_TRY(slb_dnrm2((int)n, v, &alpha, s));
    k_axpby<<<grid_of(n), 256, 0, s>>>(n, 0.0, v, 1.0 / alpha, v);
    SL_HIP_CHECK(hipMemcpyAsync(z, v, sizeof(double) * n, hipMemcpyDeviceToDevice, s));
    NAT_TRY(P(z));
    const double rho = std::sqrt(rhobar * rhobar + beta * beta);
    const double cs = rhobar / rho, sn = beta / rho, theta = sn * alpha;
    rhobar = -cs * alpha;
    const double phi = cs * phibar;
    phibar = sn * phibar;
    k_axpby<<<grid_of(n), 256, 0, s>>>(n, phi / rho, w, 1.0, x);        // x += (phi / rho) w
    k_axpby<<<grid_of(n), 256, 0, s>>>(n, 1.0, z, -theta / rho, w);     // w = z - (theta / rho) w
    nrm_r = phibar;
    const double nrm_ar = std::fabs(phibar * alpha * cs);
    const bool s1 = nrm_ar < tol * nrm_ar_0;
    const bool s2 = nrm_ar < eps * nrm_a * nrm_r;
    double nrm_w = 0;
    NAT_TRY(slb_dnrm2((int)n, w, &nrm_w, s));
    sq_d += (nrm_w * nrm_w) / (rho * rho);
    cnd_a = nrm_a * std::sqrt(sq_d);
    const bool s3 = cnd_a > 1.0 / eps;
    stag = std::fabs(phi / rho) * nrm_w < eps * nrm_x ? stag + 1 : 0;
    const bool s5 = stag >= 3;
    const double delta = sn2 * rho, gambar = -cs2 * rho, rhs = phi - delta * zz, zbar = rhs / gambar;
    nrm_x = std::sqrt(sq_x + zbar * zbar);
    const double gamma = std::sqrt(gambar * gambar + theta * theta);
    cs2 = gambar / gamma;
    sn2 = theta / gamma;
    zz = rhs / gamma;
    sq_x += zz * zz;
    if (s1) { *code = -2; break; }
    if (s2) { *code = -3; break; }
    if (s3) { *code = -4; break; }
    if (s5) { *code = -5; break; }
  }
  SL_LAUNCH_CHECK();
  return SL_OK;
}

}  // namespace

// min ||A X - B|| with A and B row-distributed: this rank holds rows [r0, r0
// + m) of the mg x n A (column-major, lda) and of B (ldb); X (n x nrhs, ldx)
// comes out the same on every rank.  The FJLT sketch draws the operator over
// all mg rows (so every rank count gives the one-rank sketch), each rank
// applies its columns of it and the t x n partial sketches are summed; LSQR
// sums A^T u and ||u||^2 over the ranks (comm: sl_comm_*, null = one rank).
SL_API int sl_nat_blendenpik_comm(const double* A, int64_t m, int64_t n, int64_t lda, const double* B, int nrhs,
                                  int64_t ldb, double* X, int64_t ldx, int64_t mg, int64_t r0, void* comm,
                                  uint64_t seed, uint64_t* ctr, double tol, int iter_lim, int* code, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (mg < 1 || n < 1 || n > mg || m < 0 || r0 < 0 || r0 + m > mg) {
    sl_set_last_error("blendenpik: needs mg >= n >= 1 (an overdetermined system) and a row range inside it");
    return SL_ERR_INVALID;
  }
  if (!slb_solver_available()) {
    sl_set_last_error("blendenpik: rocBLAS / rocSOLVER not available");
    return SL_ERR_UNSUPPORTED;
  }
  DevBuf scal(sizeof(double));
  Dist D;
  D.comm = comm;
  D.mg = mg;
  D.r0 = r0;
  D.scal = scal.d();
  const int64_t t = 4 * n;
  const double scale = std::sqrt((double)mg / (double)t);
  DevBuf dD(sizeof(double) * mg), dsamp(sizeof(int64_t) * t), SA(sizeof(double) * t * n), tau(sizeof(double) * n),
      R(sizeof(double) * n * n), Ri(sizeof(double) * n * n), nrm(sizeof(double) * 2 * n), info(sizeof(int) * 4);
  if (!dD.p || !dsamp.p || !SA.p || !tau.p || !R.p || !Ri.p || !nrm.p || !info.p) {
    sl_set_last_error("blendenpik: device allocation failed");
    return SL_ERR_HIP;
  }
  const int64_t PB = std::max<int64_t>(1, std::min<int64_t>(t, (int64_t(1) << 25) / mg));   // operator rows per panel
  DevBuf panel(sizeof(double) * PB * mg);
  if (!panel.p) {
    sl_set_last_error("blendenpik: device allocation failed");
    return SL_ERR_HIP;
  }
  bool ok = false;
  double kappa = HUGE_VAL;
  std::vector<double> hD((size_t)mg);
  std::vector<int64_t> hs((size_t)t);
  for (int attempt = 0; attempt < 3 && !ok; ++attempt) {
    // FJLT(mg, t) from the stream: mg Rademacher signs, then t sample rows
    const uint64_t c = *ctr;
    for (int64_t i = 0; i < mg; ++i) hD[(size_t)i] = sl::sample_d(sl::DIST_RADEMACHER, seed, c + (uint64_t)i, 0, 0);
    for (int64_t j = 0; j < t; ++j)
      hs[(size_t)j] = sl::uniform_int(sl::stream_block(seed, c + (uint64_t)(mg + j)).x, 0, mg - 1);
    *ctr = c + (uint64_t)(mg + t);
    SL_HIP_CHECK(hipMemcpyAsync(dD.p, hD.data(), sizeof(double) * mg, hipMemcpyHostToDevice, s));
    SL_HIP_CHECK(hipMemcpyAsync(dsamp.p, hs.data(), sizeof(int64_t) * t, hipMemcpyHostToDevice, s));
    // S A (t x n, ld t) = (operator rows) A, panel by panel of operator rows;
    // a panel is the pb x mg column-major operator block (ld pb), this rank's
    // columns r0 .. r0 + m of it against its rows of A
    if (m == 0) SL_HIP_CHECK(hipMemsetAsync(SA.p, 0, sizeof(double) * t * n, s));
    for (int64_t j0 = 0; j0 < t && m > 0; j0 += PB) {
      const int64_t pb = std::min(PB, t - j0);
      NAT_TRY(sl_dct2_rows((const int64_t*)dsamp.p + j0, pb, mg, dD.d(), scale, panel.p, SL_F64, pb, 1, s));
      NAT_TRY(gemm_cm(false, false, pb, n, m, panel.d() + r0 * pb, pb, A, lda, 0.0, SA.d() + j0, t, s));
    }
    NAT_TRY(dsum(D, SA.d(), t * n, s));
    NAT_TRY(slb_dgeqrf_cm((int)t, (int)n, SA.d(), (int)t, tau.d(), s));
    k_upper<<<grid_of(n * n), 256, 0, s>>>(SA.d(), t, n, R.d());
    SL_LAUNCH_CHECK();
    SL_HIP_CHECK(hipMemcpyAsync(Ri.p, R.p, sizeof(double) * n * n, hipMemcpyDeviceToDevice, s));
    NAT_TRY(slb_dtrtri_upper_cm((int)n, Ri.d(), (int)n, (int*)info.p, s));
    k_colabs<<<(unsigned)n, 256, 0, s>>>(R.d(), n, nrm.d());
    k_colabs<<<(unsigned)n, 256, 0, s>>>(Ri.d(), n, nrm.d() + n);
    SL_LAUNCH_CHECK();
    std::vector<double> h((size_t)(2 * n));
    int hinfo = 0;
    SL_HIP_CHECK(hipMemcpyAsync(h.data(), nrm.p, sizeof(double) * 2 * n, hipMemcpyDeviceToHost, s));
    SL_HIP_CHECK(hipMemcpyAsync(&hinfo, info.p, sizeof(int), hipMemcpyDeviceToHost, s));
    SL_HIP_CHECK(hipStreamSynchronize(s));
    double n1 = 0, n2 = 0;
    for (int64_t j = 0; j < n; ++j) {
      n1 = std::max(n1, h[(size_t)j]);
      n2 = std::max(n2, h[(size_t)(n + j)]);
    }
    kappa = hinfo == 0 ? n1 * n2 : HUGE_VAL;
    ok = std::isfinite(kappa) && kappa < 1e14;
  }
  if (!ok) {
    // reference: an exact solver when the sketch never yields a usable R (the
    // whole A and B on every rank: each rank's rows placed in zeros, summed)
    const int64_t r = n;
    DevBuf Ac(sizeof(double) * mg * n), Bc(sizeof(double) * mg * nrhs), U(sizeof(double) * mg * r),
        VT(sizeof(double) * r * n), sv(sizeof(double) * r), E(sizeof(double) * r), W(sizeof(double) * r * nrhs);
    if (!Ac.p || !Bc.p || !U.p || !VT.p || !sv.p || !E.p || !W.p) {
      sl_set_last_error("blendenpik: device allocation failed");
      return SL_ERR_HIP;
    }
    SL_HIP_CHECK(hipMemsetAsync(Ac.p, 0, sizeof(double) * mg * n, s));
    SL_HIP_CHECK(hipMemsetAsync(Bc.p, 0, sizeof(double) * mg * nrhs, s));
    if (m > 0) {
      SL_HIP_CHECK(hipMemcpy2DAsync(Ac.d() + r0, sizeof(double) * mg, A, sizeof(double) * lda, sizeof(double) * m, n,
                                    hipMemcpyDeviceToDevice, s));
      SL_HIP_CHECK(hipMemcpy2DAsync(Bc.d() + r0, sizeof(double) * mg, B, sizeof(double) * ldb, sizeof(double) * m, nrhs,
                                    hipMemcpyDeviceToDevice, s));
    }
    NAT_TRY(dsum(D, Ac.d(), mg * n, s));
    NAT_TRY(dsum(D, Bc.d(), mg * nrhs, s));
    NAT_TRY(slb_dgesvd_cm((int)mg, (int)n, Ac.d(), (int)mg, sv.d(), U.d(), (int)mg, VT.d(), (int)r, E.d(),
                          (int*)info.p, s));
    double smax = 0;
    SL_HIP_CHECK(hipMemcpyAsync(&smax, sv.p, sizeof(double), hipMemcpyDeviceToHost, s));
    SL_HIP_CHECK(hipStreamSynchronize(s));
    const double cut = smax * (double)std::max(mg, n) * DBL_EPSILON;
    NAT_TRY(gemm_cm(true, false, r, nrhs, mg, U.d(), mg, Bc.d(), mg, 0.0, W.d(), r, s));
    k_scale_rows<<<grid_of(r * nrhs), 256, 0, s>>>(W.d(), r, nrhs, r, sv.d(), cut);
    SL_LAUNCH_CHECK();
    NAT_TRY(gemm_cm(true, false, n, nrhs, r, VT.d(), r, W.d(), r, 0.0, X, ldx, s));
    SL_HIP_CHECK(hipStreamSynchronize(s));
    *code = -7;
    return SL_OK;
  }
  DevBuf u(sizeof(double) * std::max<int64_t>(m, 1)), v(sizeof(double) * n), w(sizeof(double) * n),
      z(sizeof(double) * n), tv(sizeof(double) * std::max(m, n));
  if (!u.p || !v.p || !w.p || !z.p || !tv.p) {
    sl_set_last_error("blendenpik: device allocation failed");
    return SL_ERR_HIP;
  }
  // explicit R^{-1} while it stays accurate (error ~ kappa eps), else solves
  const double* Rinv = kappa < 1e7 ? Ri.d() : nullptr;
  for (int j = 0; j < nrhs; ++j)
    NAT_TRY(lsqr_one(D, A, m, n, lda, B + (int64_t)j * ldb, X + (int64_t)j * ldx, R.d(), Rinv, tol, iter_lim, code,
                     u.d(), v.d(), w.d(), z.d(), tv.d(), s));
  SL_HIP_CHECK(hipStreamSynchronize(s));
  return SL_OK;
}

// min ||A X - B||: A column-major m x n (lda), B m x nrhs (ldb), X n x nrhs
// (ldx), device memory.  *ctr: the context counter (advanced by m + 4n per
// sketch drawn, as the runtime's FJLT draws); *code: the last column's LSQR
// code (-1 zero rhs, -2 / -3 converged, -4 ill-conditioned, -5 stagnation,
// -6 iteration limit, -7 exact SVD fallback).
SL_API int sl_nat_blendenpik(const double* A, int64_t m, int64_t n, int64_t lda, const double* B, int nrhs,
                             int64_t ldb, double* X, int64_t ldx, uint64_t seed, uint64_t* ctr, double tol,
                             int iter_lim, int* code, void* stream) {
  return sl_nat_blendenpik_comm(A, m, n, lda, B, nrhs, ldb, X, ldx, m, 0, nullptr, seed, ctr, tol, iter_lim, code,
                                stream);
}
