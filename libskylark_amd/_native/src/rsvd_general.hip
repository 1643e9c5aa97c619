// General-precision randomized SVD engine (reference nla/svd.hpp:222-318
// ApproximateSVD with the power iteration of :71-149, templated there over
// the operand type, double by default): f32 / f64 / bf16 row-distributed A,
// any n (the bf16 fused engine, rsvd_engine.cpp, covers n <= 1024, k <= 48),
// k <= 128, every stage on the device with no host round trip.
//
// One call = 2 q + 3 segments on a HIP stream (sl_rsvd_gen_num_segments),
// driven by one loop (Python _GenPlan, C sl_rsvd_gen_run_comm) that sums the
// span sl_rsvd_gen_reduce_span(i) of WG across ranks after each segment:
//   seg 2 j      [j > 0: H = W^T W, R^{-1} (Cholesky, pivot dropping),
//                Z = W R^{-1}] then Y = A Z and Y^T Y (f64) -> WG[n k :]
//   seg 2 j + 1  Ry = R^{-1} of Y^T Y, Q = Y Ry, W = A^T Q -> WG[0 : n k]
//                (j = q also G = Q^T Q -> WG[n k :])
//   seg 2 q + 2  the core: Rt^{-1} of G, C = Rt^{-T} W^T W Rt^{-1}, its top
//                r + 1 eigenpairs, M = Rt^{-1} Ub_r, N = M S^{-1}, s
// then the finish (V = W N, U = Q M) into the caller's buffers.  Y and W are
// both re-orthonormalised, as the reference's power iteration does after
// every application of A (W = A^T A Z without it squares the condition
// number, and the trailing wanted directions drowned at k = 128).
// f32 / f64 A with k <= 64 ("hand" plans) run every product on hand-written
// kernels: the two products over A per pass on the matrix cores in A's own
// precision (rsvd_stream.hip: sl_ts_az, sl_ts_atq), the m x k / n x k / k x k
// ones on sl_ts_xm64 / sl_ts_gram64 / sl_ts_small / sl_tsk_f32_xm /
// sl_tsk_gram64, the CholeskyQR factors and the core eigensolver on the
// one-wave kernels of sl_wave_la.hpp (sl_chol_inv_wave, sl_sym_eig_tridiag;
// Jacobi re-solve when flagged) -- no rocBLAS / rocSOLVER call.  f32 / f64 A
// with 64 < k <= 128 ("big" plans) run the same products on the same kernels
// at six / eight column tiles (the m x k by k x k ones -- Q = Y R^{-1}, Z = W
// R^{-1}, V = W N, U = Q M -- on sl_ts_az with the tall factor as its "A",
// the Grams on sl_ts_gram_w, the k x k ones on sl_ts_small's tiled form, the
// CholeskyQR factors on the two-waves-per-row register kernel); only their
// core eigensolver stays on rocSOLVER syevd.  bf16 A (n > 1024) keeps its two
// products over A on rocBLAS bf16 GEMMs (Y = A Z, and W = A^T [Q_hi Q_lo] as
// ONE product over the side-by-side split planes, so each pass reads A twice,
// not three times); every other product of its call is on the hand-written
// kernels above.  W, H, G and the core are f64 whatever A's precision.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <new>
#include <type_traits>

#include "sl_blas.hpp"
#include "sl_common.hpp"
#include "sl_rng.hpp"

SL_API int sl_chol_inv_wave(const double* G, int k, int ldg, double* X, int* status, void* stream);
SL_API int sl_sym_eig_tridiag(const double* C, int k, int ldc, int r, double* out, int want_sqrt, int* status,
                              void* stream);
SL_API int sl_sym_eig_topr_if(const double* C, int k, int ldc, int r, double* out, int want_sqrt, int max_sweeps,
                              const int* flag, void* stream);
SL_API int sl_fill_random(void* out, int dtype, int dist, uint64_t seed, uint64_t base, int64_t rows, int64_t cols,
                          int64_t sr, int64_t sc, int64_t r0, int64_t c0, int64_t ir, int64_t ic, double p0, double p1,
                          double scale, int precise, void* stream);
SL_API int64_t sl_tsk_gram64_workspace(int64_t m, int k);
SL_API int sl_tsk_gram64(const float* Y, int64_t m, int k, int64_t ldy, double* G, void* ws, void* stream);
SL_API int sl_comm_all_reduce(void* comm, const void* send, void* recv, int64_t count, int dtype, int op,
                              void* stream);
SL_API int sl_ts_az(const void* A, int64_t m, int64_t n, int64_t lda, const void* Z, int k, void* Y, int64_t ldy,
                    int dt, void* stream);
SL_API int64_t sl_ts_atq_workspace(int64_t m, int64_t n, int k, int dt);
SL_API int sl_ts_atq(const void* A, int64_t m, int64_t n, int64_t lda, const void* Q, int k, double* W, int ldw,
                     void* ws, int dt, void* stream);
SL_API int sl_ts_xm64(const double* X, int64_t rows, int k, int64_t ldx, const double* Mm, int k2, void* out,
                      int64_t ldo, int out_dt, void* stream);
SL_API int64_t sl_ts_gram64_workspace(int64_t rows, int k);
SL_API int sl_ts_gram64(const double* X, int64_t rows, int k, int64_t ldx, double* G, int ldg, void* ws,
                        void* stream);
SL_API int sl_ts_small(int ta, int tb, int mr, int nc, int kd, const double* A, int lda, const double* B, int ldb,
                       double* C, int ldc, void* stream);
SL_API int sl_ts_gram_w(const void* X, int dt, int64_t rows, int k, int64_t ldx, double* G, int ldg, void* ws,
                        void* stream);
SL_API int sl_tsk_f32_xm(const float* Y, int64_t m, int k, int64_t ldy, const float* M, int k2, float* out,
                         int64_t ldo, double* G, void* ws, void* stream);

namespace {

enum : int { ST_PIVOT = 1, ST_NONFINITE = 2, ST_NOCONV = 4, ST_RANK = 8 };

template <typename T> __device__ __forceinline__ double ld_d(const T* p) { return (double)*p; }
template <> __device__ __forceinline__ double ld_d<bf16_t>(const bf16_t* p) { return (double)bf16_to_f(*p); }
template <typename T> __device__ __forceinline__ void st_d(T* p, double v) { *p = (T)v; }
template <> __device__ __forceinline__ void st_d<bf16_t>(bf16_t* p, double v) { *p = f_to_bf16((float)v); }

// out (rows x cols, ldo) = in (rows x cols, ldi), converted
template <typename TI, typename TO>
__global__ void __launch_bounds__(256) k_cast2d(const TI* __restrict__ in, int64_t ldi, int64_t rows, int cols,
                                               TO* __restrict__ out, int64_t ldo, int* zero_word) {
  if (zero_word && blockIdx.x == 0 && threadIdx.x == 0) *zero_word = 0;
  const int64_t tot = rows * cols;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < tot; t += (int64_t)gridDim.x * 256) {
    const int64_t i = t / cols;
    const int j = (int)(t - i * cols);
    st_d<TO>(out + i * ldo + j, ld_d<TI>(in + i * ldi + j));
  }
}

// FJLT operator of the rowwise sketch A Omega^T as Z (n x k, row-major):
// Z[i][j] = scale * d_i * c_{p_j} cos(pi p_j (2 i + 1) / 2n), d the n
// Rademacher signs at stream offset baseD, p_j the k sampled DCT-II
// frequencies at baseS (reference FJLT_data.hpp:79-86; the same operator as
// the fused engine's k_fjlt_zt, transposed and in full precision)
template <typename T>
__global__ void __launch_bounds__(256) k_fjlt_z(uint64_t seed, uint64_t baseD, uint64_t baseS, double scale, int k,
                                               int64_t n, T* __restrict__ Z) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * k) return;
  const int64_t i = t / k;
  const int j = (int)(t - i * k);
  const int64_t p = sl::uniform_int(sl::stream_block(seed, baseS + (uint64_t)j).x, 0, n - 1);
  const double d = (sl::stream_block(seed, baseD + (uint64_t)i).x >> 63) ? 1.0 : -1.0;
  const int64_t a = (p * (2 * i + 1)) % (4 * n);
  const double w = 3.14159265358979323846 / (2.0 * (double)n);
  const double c0 = sqrt(1.0 / (double)n), c1 = sqrt(2.0 / (double)n);
  st_d<T>(Z + t, cos(w * (double)a) * (p == 0 ? c0 : c1) * scale * d);
}

// bf16 hi / lo planes of an f32 m x k matrix side by side in hl (m x 2k):
// hi = bf16(y) in columns [0, k), lo = bf16(y - hi) in [k, 2k), and y <- hi +
// lo (exact in f32): the rows the bf16 products actually see
__global__ void __launch_bounds__(256) k_split_bf16(float* __restrict__ y, int64_t m, int k, bf16_t* __restrict__ hl) {
  const int64_t tot = m * k;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < tot; t += (int64_t)gridDim.x * 256) {
    const int64_t i = t / k;
    const int j = (int)(t - i * k);
    const float v = y[t];
    const bf16_t h = f_to_bf16(v);
    const bf16_t l = f_to_bf16(v - bf16_to_f(h));
    hl[i * 2 * k + j] = h;
    hl[i * 2 * k + k + j] = l;
    y[t] = bf16_to_f(h) + bf16_to_f(l);
  }
}

// out (f64, tot) = sum of np slabs (stride tot) of T; zero_word cleared when given
template <typename T>
__global__ void __launch_bounds__(256) k_sum_parts(const T* __restrict__ parts, int np, int64_t tot,
                                                   double* __restrict__ out, int* zero_word) {
  if (zero_word && blockIdx.x == 0 && threadIdx.x == 0) *zero_word = 0;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < tot; e += (int64_t)gridDim.x * blockDim.x) {
    double acc = 0.0;
    for (int p_ = 0; p_ < np; ++p_) acc += (double)parts[(int64_t)p_ * tot + e];
    out[e] = acc;
  }
}

// the core's epilogue: eig = [Ub_r (k x r); s (r)] from the eigensolver.
// s_out (r, dtype T), N = M S^{-1} (k x r f64) from M (k x r f64), rank / finiteness status
template <typename T>
__global__ void __launch_bounds__(256) k_core_epi(const double* __restrict__ eig, int k, int r,
                                                  const double* __restrict__ M, double* __restrict__ N,
                                                  T* __restrict__ Md, int* __restrict__ status) {
  const double* s = eig + k * r;
  for (int e = threadIdx.x; e < k * r; e += 256) {
    const int c = e % r;
    const double sv = s[c];
    N[e] = sv > 0.0 ? M[e] / sv : 0.0;
    st_d<T>(Md + e, M[e]);
  }
  if (threadIdx.x == 0) {
    int st = 0;
    for (int c = 0; c < r; ++c) {
      if (!(s[c] > 0.0)) st |= ST_RANK;
      if (!(s[c] == s[c])) st |= ST_NONFINITE;
    }
    if (st) atomicOr(status, st);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) k_store_s(const double* __restrict__ s, int r, T* __restrict__ out) {
  if ((int)threadIdx.x < r) st_d<T>(out + threadIdx.x, s[threadIdx.x]);
}

// Cholesky statuses (dropped pivots / rocSOLVER infos) and eigensolver
// statuses -> the call's status word.  st[2]: the Jacobi re-solve of a core
// the tridiagonal path flagged (st[1]) ran out of sweeps; st[12]: rocSOLVER
// syevd info (k > 64).  Both mean the core's eigenpairs did not converge.
__global__ void k_status_merge(int* __restrict__ st) {
  if (threadIdx.x == 0) {
    int v = 0;
    for (int i = 4; i < 12; ++i) v |= st[i] ? ST_PIVOT : 0;
    if (st[2] || st[12]) v |= ST_NOCONV;
    if (v) atomicOr(st, v);
  }
}

int64_t align256(int64_t b) { return (b + 255) & ~(int64_t)255; }

// A/B knob (plans created after setting it): 1 = the hand-written products
// over A for f32 / f64 at any k <= 128 (default), 0 = rocBLAS past k = 64
int g_gen_big = 1;

// A/B knob (plans created after setting it): bf16 A's A^T [Q_hi Q_lo] as a
// strided batch of row-chunk products (split K; 1, default) or one product (0)
int g_bf16_split = 1;

size_t esize(int dt) { return dt == SL_F64 ? 8 : dt == SL_F32 ? 4 : 2; }

struct GPlan {
  int64_t m = 0, n = 0, lda = 0;
  int k = 0, r = 0, q = 0, dt = SL_F32;
  char* base = nullptr;
  void* Z = nullptr;       // n x k (dt)
  void* Y = nullptr;       // m x k (dt; f32 when A is bf16)
  void* Yh = nullptr;      // bf16 A: hi / lo planes of Q side by side (m x 2k bf16)
  void* Wt = nullptr;      // bf16 A: n x 2k f32 pass output (A^T [Q_hi Q_lo])
  void* Qb = nullptr;      // m x k orthonormalised Y (dt; f32 when A is bf16): the basis U is formed from
  void* Rf = nullptr;      // k x k f32 copy of R^{-1} (f32 / bf16 A)
  double* WG = nullptr;    // [W (n x k); G (k x k)] f64
  double* Zf = nullptr;    // n x k f64
  double* H = nullptr;     // k x k
  double* Ri = nullptr;    // k x k
  double* T1 = nullptr;    // k x k
  double* Cc = nullptr;    // k x k
  double* eig = nullptr;   // k r + r (+ k for syevd eigenvalues, k scratch)
  double* M = nullptr;     // k x r
  double* N = nullptr;     // k x r
  void* Md = nullptr;      // k x r (dt of U)
  double* Vf = nullptr;    // n x r
  void* gws = nullptr;     // f32 Gram workspace
  void* parts = nullptr;   // f32 / f64 A: per-row-chunk partials of A^T Y (np + 1 slabs of n x k, dt)
  int np = 0;              // row chunks of ch rows (+ one for the remainder)
  int64_t ch = 0;
  int* st = nullptr;       // [0] status, [1..2] eig status, [4..11] chol statuses / infos (4 / 6 inter, 8 core, 10 Y)
  // hand: f32 / f64 A with k <= 64 -- every product on the hand-written
  // kernels (rsvd_stream.hip, tsk_f32_kernels.hip), no rocBLAS / rocSOLVER
  bool hand = false;
  // big: f32 / f64 A (k <= 128) -- the two products over A per pass on the
  // hand-written kernels (sl_ts_az / sl_ts_atq; KT = 6 / 8 column tiles past
  // k = 64), whatever runs the k x k algebra
  bool big = false;
  void* atqw = nullptr;    // big: A^T Q row-group slabs
  void* g64w = nullptr;    // f64 Gram slabs (W^T W; Y^T Y of f64 A)
  // sketch of the call
  int sk = 0;              // 0 none, 1 FJLT, 2 dense
  uint64_t seed = 0, b0 = 0, b1 = 0;
  double p0 = 0, p1 = 0, scale = 1;
  int dist = 0;
};

template <typename F>
int dispatch_dt(int dt, F f) {
  if (dt == SL_F32) return f((float*)nullptr);
  if (dt == SL_F64) return f((double*)nullptr);
  return f((bf16_t*)nullptr);
}

unsigned grid_of(int64_t tot) {
  int64_t g = (tot + 255) / 256;
  return (unsigned)(g < 1 ? 1 : (g > 4096 ? 4096 : g));
}

// X = R^{-1} of the SPD k x k G (row-major f64) by the register Cholesky
// kernels (k <= 64: sl_wave_la.hpp wg_chol_invB; 64 < k <= 128: two waves per
// row, wg_chol_invW), pivots at or below 1e-13 max G_ii dropped (zero row /
// column, status bit ST_PIVOT via st).  (64 < k <= 128 ran eigen-whitening on
// rocSOLVER syevd before: ~2.4 ms per factor, four factors per q = 1 call.)
int chol_inv(GPlan* p, const double* G, double* X, int* st, hipStream_t s) {
  return sl_chol_inv_wave(G, p->k, p->k, X, st, s);
}

// the sketch operator of the call into Z (dt)
int make_z(GPlan* p, hipStream_t s) {
  const int64_t tot = p->n * p->k;
  if (p->sk == 1) {
    return dispatch_dt(p->dt, [&](auto* tag) {
      using T = std::remove_pointer_t<decltype(tag)>;
      k_fjlt_z<T><<<(unsigned)((tot + 255) / 256), 256, 0, s>>>(p->seed, p->b0, p->b1, p->scale, p->k, p->n, (T*)p->Z);
      SL_LAUNCH_CHECK();
      return SL_OK;
    });
  }
  if (p->sk == 2) {
    // dense: Z[i][j] = scale * dist(seed, base + i k + j) (column-major k x n stream of S = Z^T)
    int rc = sl_fill_random(p->Zf, SL_F64, p->dist, p->seed, p->b0, p->n, p->k, p->k, 1, 0, 0, p->k, 1, p->p0, p->p1,
                            p->scale, 1, s);
    if (rc != SL_OK) return rc;
    return dispatch_dt(p->dt, [&](auto* tag) {
      using T = std::remove_pointer_t<decltype(tag)>;
      k_cast2d<double, T><<<grid_of(tot), 256, 0, s>>>(p->Zf, p->k, p->n, p->k, (T*)p->Z, p->k, nullptr);
      SL_LAUNCH_CHECK();
      return SL_OK;
    });
  }
  return SL_OK;   // Z set explicitly
}

// G (k x k f64) = Yb^T Yb of an m x k matrix in the pass precision (f64, or
// f32 for f32 / bf16 A), f64 products and sums: the matrix-core Gram kernels
// (k <= 64: sl_ts_gram64 / sl_tsk_gram64; 64 < k <= 128: sl_ts_gram_w)
int gram(GPlan* p, const void* Yb, double* G, hipStream_t s) {
  const int64_t m = p->m;
  const int k = p->k;
  if (k > 64) return sl_ts_gram_w(Yb, p->dt == SL_F64 ? SL_F64 : SL_F32, m, k, k, G, k, p->g64w, s);
  if (p->dt == SL_F64) return sl_ts_gram64((const double*)Yb, m, k, k, G, k, p->g64w, s);
  return sl_tsk_gram64((const float*)Yb, m, k, k, G, p->gws, s);
}

// first half of pass i: Y = A Z and its Gram Y^T Y -> WG[n k :] (all-reduced
// across ranks before the second half)
int apply_z(GPlan* p, const void* A, hipStream_t s) {
  const int dt = p->dt == SL_BF16 ? SL_BF16 : p->dt;
  int rc = p->big ? sl_ts_az(A, p->m, p->n, p->lda, p->Z, p->k, p->Y, p->k, dt, s)
                   : slb_gemm(dt, false, false, p->m, p->k, p->n, 1.0, A, p->lda, p->Z, p->k, 0.0, p->Y, p->k, s);
  if (rc != SL_OK) return rc;
  return gram(p, p->Y, p->WG + p->n * p->k, s);
}

// Qb = Y Ry (Ry = R^{-1} in p->Ri): the hand-written tall-skinny kernels --
// k <= 64 sl_ts_xm64 (f64) / sl_tsk_f32_xm (f32 Y: f32 and bf16 A), past 64
// sl_ts_az with Y as its operand (big plans and bf16 A); rocBLAS only for the
// k > 64 library A/B (g_gen_big = 0)
int q_from_y(GPlan* p, hipStream_t s) {
  const int64_t m = p->m;
  const int k = p->k;
  if (p->dt == SL_F64) {
    if (k <= 64) return sl_ts_xm64((const double*)p->Y, m, k, k, p->Ri, k, p->Qb, k, SL_F64, s);
    if (p->big) return sl_ts_az(p->Y, m, k, k, p->Ri, k, p->Qb, k, SL_F64, s);
    return slb_gemm(SL_F64, false, false, m, k, k, 1.0, p->Y, k, p->Ri, k, 0.0, p->Qb, k, s);
  }
  k_cast2d<double, float><<<grid_of((int64_t)k * k), 256, 0, s>>>(p->Ri, k, k, k, (float*)p->Rf, k, nullptr);
  SL_LAUNCH_CHECK();
  if (k <= 64)
    return sl_tsk_f32_xm((const float*)p->Y, m, k, k, (const float*)p->Rf, k, (float*)p->Qb, k, nullptr, nullptr, s);
  if (p->big || p->dt == SL_BF16) return sl_ts_az(p->Y, m, k, k, p->Rf, k, p->Qb, k, SL_F32, s);
  return slb_gemm(SL_F32, false, false, m, k, k, 1.0, p->Y, k, p->Rf, k, 0.0, p->Qb, k, s);
}

// WG[i][j] (f64, n x k) = sum over the np slabs of Wt[i][j] + Wt[i][k + j]
// (f32, n x 2k each): the bf16 pass's A^T Q_hi and A^T Q_lo halves (per row
// chunk), summed in f64
__global__ void __launch_bounds__(256) k_sum_halves(const float* __restrict__ Wt, int np, int64_t n, int k,
                                                   double* __restrict__ WG) {
  const int64_t tot = n * k;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < tot; t += (int64_t)gridDim.x * 256) {
    const int64_t i = t / k;
    const int j = (int)(t - i * k);
    double acc = 0.0;
    for (int q = 0; q < np; ++q) {
      const float* w = Wt + (int64_t)q * n * 2 * k + i * 2 * k;
      acc += (double)w[j] + (double)w[k + j];
    }
    WG[t] = acc;
  }
}

// second half of pass i: Ry = R^{-1} of the (all-reduced) Y^T Y (pivot
// dropping), Q = Y Ry (orthonormal: the power iteration re-orthonormalises
// after every application of A, so the condition number never squares --
// reference nla/svd.hpp:71-149), W = A^T Q -> WG[0 : n k], and on the final
// pass G = Q^T Q (~ I: the core's second CholeskyQR step).  bf16 A: Q is
// split into bf16 hi / lo planes side by side (one m x 2k operand, so A is
// read once for both), and Q' = hi + lo is kept as the stored basis so W, G
// and U = Q' M all see the same rows.
int apply_t(GPlan* p, const void* A, bool final_pass, int i, hipStream_t s) {
  const int64_t m = p->m, n = p->n;
  const int k = p->k;
  (void)i;
  int rc = chol_inv(p, p->WG + n * k, p->Ri, p->st + 10, s);
  if (rc != SL_OK) return rc;
  if ((rc = q_from_y(p, s)) != SL_OK) return rc;
  if (p->big) {
    // W = A^T Q straight into WG (row-group slabs summed in f64)
    rc = sl_ts_atq(A, m, n, p->lda, p->Qb, k, p->WG, k, p->atqw, p->dt, s);
  } else if (p->dt == SL_BF16) {
    k_split_bf16<<<grid_of(m * k), 256, 0, s>>>((float*)p->Qb, m, k, (bf16_t*)p->Yh);
    SL_LAUNCH_CHECK();
    const bf16_t* Ab = (const bf16_t*)A;
    const bf16_t* Q2 = (const bf16_t*)p->Yh;
    float* out = (float*)p->Wt;
    int nparts = 1;
    if (p->np > 0) {
      // split K: np row chunks in one strided-batched launch (+ the remainder rows)
      const int64_t tot = n * 2 * k;
      out = (float*)p->parts;
      rc = slb_gemm_strided(SL_BF16, true, false, n, 2 * k, p->ch, 1.0, Ab, p->lda, p->ch * p->lda, Q2, 2 * k,
                            p->ch * 2 * k, 0.0, out, 2 * k, tot, p->np, s);
      if (rc != SL_OK) return rc;
      nparts = p->np;
      const int64_t r0 = p->ch * p->np;
      if (r0 < m) {
        rc = slb_gemm(SL_BF16, true, false, n, 2 * k, m - r0, 1.0, Ab + r0 * p->lda, p->lda, Q2 + r0 * 2 * k, 2 * k,
                      0.0, out + (int64_t)p->np * tot, 2 * k, s);
        if (rc != SL_OK) return rc;
        ++nparts;
      }
    } else {
      rc = slb_gemm(SL_BF16, true, false, n, 2 * k, m, 1.0, A, p->lda, p->Yh, 2 * k, 0.0, p->Wt, 2 * k, s);
      if (rc != SL_OK) return rc;
    }
    k_sum_halves<<<grid_of(n * k), 256, 0, s>>>(out, nparts, n, k, p->WG);
    SL_LAUNCH_CHECK();
  } else {
    // library A/B (g_gen_big = 0, k > 64): W = A^T Q as np row-chunk products
    // (one strided-batched launch fills the chip; a single K = m product runs
    // on a handful of workgroups), then one f64 sum of the partial slabs
    const size_t es = p->dt == SL_F64 ? 8 : 4;
    const int64_t tot = n * k;
    rc = slb_gemm_strided(p->dt, true, false, n, k, p->ch, 1.0, A, p->lda, p->ch * p->lda, p->Qb, k, p->ch * k, 0.0,
                          p->parts, k, tot, p->np, s);
    if (rc != SL_OK) return rc;
    const int64_t r0 = p->ch * p->np;
    int nparts = p->np;
    if (r0 < m) {
      rc = slb_gemm(p->dt, true, false, n, k, m - r0, 1.0, (const char*)A + r0 * p->lda * es, p->lda,
                    (const char*)p->Qb + r0 * k * es, k, 0.0, (char*)p->parts + (int64_t)p->np * tot * es, k, s);
      if (rc != SL_OK) return rc;
      ++nparts;
    }
    rc = dispatch_dt(p->dt, [&](auto* tag) {
      using T = std::remove_pointer_t<decltype(tag)>;
      k_sum_parts<T><<<grid_of(tot), 256, 0, s>>>((const T*)p->parts, nparts, tot, p->WG, nullptr);
      SL_LAUNCH_CHECK();
      return SL_OK;
    });
  }
  if (rc != SL_OK) return rc;
  if (!final_pass) return SL_OK;
  return gram(p, p->Qb, p->WG + n * k, s);
}

// the boundary between pass i - 1 and pass i: CholeskyQR of the (all-reduced) W
// H (k x k) = W^T W of the f64 n x k W: the hand-written matrix-core Grams
int gram_w64(GPlan* p, const double* W, double* H, hipStream_t s) {
  const int k = p->k;
  return k > 64 ? sl_ts_gram_w(W, SL_F64, p->n, k, k, H, k, p->g64w, s) : sl_ts_gram64(W, p->n, k, k, H, k, p->g64w, s);
}

int inter(GPlan* p, int i, hipStream_t s) {
  const int k = p->k;
  const int64_t n = p->n;
  int rc = gram_w64(p, p->WG, p->H, s);
  if (rc != SL_OK) return rc;
  rc = chol_inv(p, p->H, p->Ri, p->st + 4 + 2 * (i % 2), s);
  if (rc != SL_OK) return rc;
  // Z = W R^{-1} in A's dtype (bf16: through the f64 Zf)
  if (k <= 64 && p->dt != SL_BF16) return sl_ts_xm64(p->WG, n, k, k, p->Ri, k, p->Z, k, p->dt, s);
  if (p->big && p->dt == SL_F64) return sl_ts_az(p->WG, n, k, k, p->Ri, k, p->Z, k, SL_F64, s);
  rc = k <= 64 ? sl_ts_xm64(p->WG, n, k, k, p->Ri, k, p->Zf, k, SL_F64, s)
       : p->big || p->dt == SL_BF16 ? sl_ts_az(p->WG, n, k, k, p->Ri, k, p->Zf, k, SL_F64, s)
                                    : slb_gemm(SL_F64, false, false, n, k, k, 1.0, p->WG, k, p->Ri, k, 0.0, p->Zf, k, s);
  if (rc != SL_OK) return rc;
  return dispatch_dt(p->dt, [&](auto* tag) {
    using T = std::remove_pointer_t<decltype(tag)>;
    k_cast2d<double, T><<<grid_of(n * k), 256, 0, s>>>(p->Zf, k, n, k, (T*)p->Z, k, nullptr);
    SL_LAUNCH_CHECK();
    return SL_OK;
  });
}

// eigenvectors (rows of Vt, ascending eigenvalues D) -> eig = [Ub_r (k x r, descending); sqrt(max(D, 0))]
__global__ void __launch_bounds__(256) k_pack_syevd(const double* __restrict__ Vt, const double* __restrict__ D,
                                                    int k, int r, double* __restrict__ eig) {
  for (int e = threadIdx.x; e < k * r; e += 256) {
    const int i = e / r, c = e % r;
    eig[e] = Vt[(int64_t)(k - 1 - c) * k + i];
  }
  for (int c = threadIdx.x; c < r; c += 256) {
    const double l = D[k - 1 - c];
    eig[k * r + c] = sqrt(l > 0.0 ? l : 0.0);
  }
}

int gen_pack_syevd(const double* Vt, const double* D, int k, int r, double* eig, hipStream_t s) {
  k_pack_syevd<<<1, 256, 0, s>>>(Vt, D, k, r, eig);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// the core after the final pass: Rt^{-1}, C, top eigenpairs, M, N, s
int core(GPlan* p, hipStream_t s) {
  const int k = p->k, r = p->r;
  const int64_t n = p->n;
  const double* W = p->WG;
  const double* G = p->WG + n * k;
  int rc = gram_w64(p, W, p->H, s);   // H = W^T W
  if (rc != SL_OK) return rc;
  rc = chol_inv(p, G, p->Ri, p->st + 8, s);
  if (rc != SL_OK) return rc;
  // the k x k products on sl_ts_small (one workgroup to k = 64, 32 x 32 tiles past)
  rc = sl_ts_small(0, 0, k, k, k, p->H, k, p->Ri, k, p->T1, k, s);   // T = H Rti
  if (rc != SL_OK) return rc;
  rc = sl_ts_small(1, 0, k, k, k, p->Ri, k, p->T1, k, p->Cc, k, s);   // C = Rti^T T
  if (rc != SL_OK) return rc;
  if (k <= 64) {
    SL_HIP_CHECK(hipMemsetAsync(p->st + 1, 0, 8, s));   // st[1] flag, st[2] re-solve no-convergence
    rc = sl_sym_eig_tridiag(p->Cc, k, k, r, p->eig, 1, p->st + 1, s);
    if (rc != SL_OK) return rc;
    // re-solve by Jacobi only when the tridiagonal path flagged the core (device-side condition)
    rc = sl_sym_eig_topr_if(p->Cc, k, k, r, p->eig, 1, 40, p->st + 1, s);
    if (rc != SL_OK) return rc;
  } else {
    // rocSOLVER divide and conquer; eigenvectors in the rows of T1 (ascending)
    SL_HIP_CHECK(hipMemcpyAsync(p->T1, p->Cc, (size_t)k * k * 8, hipMemcpyDeviceToDevice, s));
    rc = slb_dsyevd(k, p->T1, k, p->eig + k * r + r, p->eig + k * r + r + k, p->st + 12, s);
    if (rc != SL_OK) return rc;
    rc = gen_pack_syevd(p->T1, p->eig + k * r + r, k, r, p->eig, s);
    if (rc != SL_OK) return rc;
  }
  // M = Rti Ub_r (k x r), N = M S^{-1}, s
  rc = sl_ts_small(0, 0, k, r, k, p->Ri, k, p->eig, r, p->M, r, s);
  if (rc != SL_OK) return rc;
  const int udt = p->dt == SL_BF16 ? SL_F32 : p->dt;
  rc = dispatch_dt(udt, [&](auto* tag) {
    using T = std::remove_pointer_t<decltype(tag)>;
    k_core_epi<T><<<1, 256, 0, s>>>(p->eig, k, r, p->M, p->N, (T*)p->Md, p->st);
    SL_LAUNCH_CHECK();
    return SL_OK;
  });
  if (rc != SL_OK) return rc;
  k_status_merge<<<1, 64, 0, s>>>(p->st);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

int nseg(const GPlan* p) { return 2 * p->q + 3; }

// segment i of the call: even 2 j = [the boundary before pass j] + Y = A Z +
// Y^T Y; odd 2 j + 1 = Q = Y R^{-1} + W = A^T Q (+ Q^T Q on the last pass);
// the last = the core.  After segment i < nseg - 1, several ranks sum the
// WG span reduce_span(i) (Y^T Y after an even segment, W (+ G) after an odd).
int seg(GPlan* p, const void* A, int i, hipStream_t s) {
  if (i < 0 || i >= nseg(p)) { sl_set_last_error("rsvd_gen: segment out of range"); return SL_ERR_INVALID; }
  if (i == nseg(p) - 1) return core(p, s);
  const int j = i / 2;
  if (i % 2) return apply_t(p, A, j == p->q, j, s);
  int rc;
  if (j == 0) {
    SL_HIP_CHECK(hipMemsetAsync(p->st, 0, 16 * sizeof(int), s));
    rc = make_z(p, s);
  } else {
    rc = inter(p, j, s);
  }
  if (rc != SL_OK) return rc;
  return apply_z(p, A, s);
}

void reduce_span(const GPlan* p, int i, int64_t* off, int64_t* cnt) {
  const int64_t nk = p->n * p->k, kk = (int64_t)p->k * p->k;
  if (i < 0 || i >= nseg(p) - 1) { *off = 0; *cnt = 0; return; }
  if (i % 2 == 0) { *off = nk; *cnt = kk; return; }
  *off = 0;
  *cnt = (i / 2 == p->q) ? nk + kk : nk;
}

}  // namespace

// A: m x n row shard (lda) of dtype dt (SL_F32 / SL_F64 / SL_BF16), k <= 128
// sketch columns, r <= k rank, q power iterations.  Allocates every device
// buffer of the call once.
SL_API int sl_rsvd_gen_create(int64_t m, int64_t n, int64_t lda, int k, int r, int q, int dt, void** out) {
  *out = nullptr;
  if (m < 1 || n < 1 || lda < n || k < 1 || k > 128 || r < 1 || r > k || q < 0 || k > n ||
      (dt != SL_F32 && dt != SL_F64 && dt != SL_BF16)) {
    sl_set_last_error("rsvd_gen: needs m, n >= 1, lda >= n, 1 <= r <= k <= min(n, 128), q >= 0, dtype f32/f64/bf16");
    return SL_ERR_UNSUPPORTED;
  }
  const bool hand = k <= 64 && dt != SL_BF16;
  if (!hand && (!slb_available() || (k > 64 && !slb_solver_available()))) {
    sl_set_last_error("rsvd_gen: rocBLAS / rocSOLVER not available");
    return SL_ERR_UNSUPPORTED;
  }
  GPlan* p = new (std::nothrow) GPlan();
  if (!p) return SL_ERR_GENERIC;
  p->m = m; p->n = n; p->lda = lda; p->k = k; p->r = r; p->q = q; p->dt = dt; p->hand = hand;
  p->big = dt != SL_BF16 && (hand || g_gen_big);
  const size_t es = esize(dt);
  const size_t ys = dt == SL_BF16 ? 4 : es;   // Y / Wt element size
  int64_t off = 0;
  const int64_t o_z = off;   off = align256(off + n * k * (int64_t)es);
  const int64_t o_y = off;   off = align256(off + m * k * (int64_t)ys);
  const int64_t o_yh = off;  off = align256(off + (dt == SL_BF16 ? m * 2 * k * 2 : 0));   // bf16: [hi lo] planes
  const int64_t o_w = off;   off = align256(off + n * (dt == SL_BF16 ? 2 * k : k) * (int64_t)ys);
  const int64_t o_qb = off;  off = align256(off + m * k * (int64_t)ys);
  const int64_t o_rf = off;  off = align256(off + (int64_t)k * k * 4);
  const int64_t o_wg = off;  off = align256(off + (n + k) * k * 8);
  const int64_t o_zf = off;  off = align256(off + n * k * 8);
  const int64_t o_h = off;   off = align256(off + (int64_t)k * k * 8);
  const int64_t o_ri = off;  off = align256(off + (int64_t)k * k * 8);
  const int64_t o_t1 = off;  off = align256(off + (int64_t)k * k * 8);
  const int64_t o_c = off;   off = align256(off + (int64_t)k * k * 8);
  const int64_t o_e = off;   off = align256(off + ((int64_t)k * r + r + 2 * k) * 8);
  const int64_t o_m = off;   off = align256(off + (int64_t)k * r * 8);
  const int64_t o_n = off;   off = align256(off + (int64_t)k * r * 8);
  const int64_t o_md = off;  off = align256(off + (int64_t)k * r * 8);
  const int64_t o_vf = off;  off = align256(off + n * r * 8);
  const int64_t o_gw = off;  off = align256(off + (k <= 64 ? sl_tsk_gram64_workspace(m, k) : 256));
  // f32 / f64 A: row-chunk partials of A^T Y (and of Y^T Y), <= 64 MB of slabs
  int np = 0;
  int64_t ch = 0;
  // (bf16 A: of A^T [Q_hi Q_lo], n x 2k f32 slabs, when g_bf16_split)
  const bool bsplit = dt == SL_BF16 && g_bf16_split;
  const int64_t slab_el = dt == SL_BF16 ? n * 2 * k : std::max<int64_t>(n * k, (int64_t)k * k);
  const int64_t slab_es = dt == SL_BF16 ? 4 : (int64_t)es;
  if ((dt != SL_BF16 && !p->big) || bsplit) {
    np = (int)std::max<int64_t>(1, std::min<int64_t>({128, (int64_t(64) << 20) / (slab_el * slab_es), m / 512}));
    ch = m / np;
  }
  const int64_t o_pt = off;  off = align256(off + (np ? (int64_t)(np + 1) * slab_el * slab_es : 0));
  const int64_t o_aw = off;  off = align256(off + (p->big ? sl_ts_atq_workspace(m, n, k, dt) : 0));
  const int64_t o_g6 = off;  off = align256(off + sl_ts_gram64_workspace(std::max(m, n), k));
  const int64_t o_st = off;  off = align256(off + 64 * 4);
  if (hipMalloc((void**)&p->base, (size_t)off) != hipSuccess) {
    delete p;
    sl_set_last_error("rsvd_gen: device allocation failed");
    return SL_ERR_HIP;
  }
  char* b = p->base;
  p->Z = b + o_z; p->Y = b + o_y; p->Yh = b + o_yh; p->Wt = b + o_w;
  p->Qb = b + o_qb; p->Rf = b + o_rf;
  p->WG = (double*)(b + o_wg); p->Zf = (double*)(b + o_zf); p->H = (double*)(b + o_h); p->Ri = (double*)(b + o_ri);
  p->T1 = (double*)(b + o_t1); p->Cc = (double*)(b + o_c); p->eig = (double*)(b + o_e); p->M = (double*)(b + o_m);
  p->N = (double*)(b + o_n); p->Md = b + o_md; p->Vf = (double*)(b + o_vf); p->gws = b + o_gw;
  p->st = (int*)(b + o_st);
  p->parts = b + o_pt;
  p->atqw = b + o_aw;
  p->g64w = b + o_g6;
  p->np = np;
  p->ch = ch;
  if (hipMemset(p->st, 0, 64 * 4) != hipSuccess) {
    (void)hipFree(p->base);
    delete p;
    return SL_ERR_HIP;
  }
  *out = p;
  return SL_OK;
}

SL_API void sl_rsvd_gen_set_big(int v) { g_gen_big = v ? 1 : 0; }
SL_API void sl_rsvd_gen_set_bf16_split(int v) { g_bf16_split = v ? 1 : 0; }

SL_API int sl_rsvd_gen_destroy(void* plan) {
  GPlan* p = (GPlan*)plan;
  if (!p) return SL_OK;
  (void)hipFree(p->base);
  delete p;
  return SL_OK;
}

// the sketch operator of the next call: FJLT (N Rademacher signs at baseD, k
// DCT frequencies at baseS, scale sqrt(n / k)), realised on the device
SL_API int sl_rsvd_gen_set_fjlt(void* plan, uint64_t seed, uint64_t baseD, uint64_t baseS, double scale) {
  GPlan* p = (GPlan*)plan;
  p->sk = 1; p->seed = seed; p->b0 = baseD; p->b1 = baseS; p->scale = scale;
  return SL_OK;
}

// dense operator (JLT: Normal, CT: Cauchy, ...): scale * dist(seed, base + i k + j)
SL_API int sl_rsvd_gen_set_dense(void* plan, int dist, uint64_t seed, uint64_t base, double p0, double p1,
                                 double scale) {
  GPlan* p = (GPlan*)plan;
  p->sk = 2; p->dist = dist; p->seed = seed; p->b0 = base; p->p0 = p0; p->p1 = p1; p->scale = scale;
  return SL_OK;
}

// explicit operator Z (n x k, row-major, A's dtype, device)
SL_API int sl_rsvd_gen_set_z(void* plan, const void* Z, void* stream) {
  GPlan* p = (GPlan*)plan;
  p->sk = 0;
  SL_HIP_CHECK(hipMemcpyAsync(p->Z, Z, (size_t)(p->n * p->k) * esize(p->dt), hipMemcpyDeviceToDevice,
                              (hipStream_t)stream));
  return SL_OK;
}

SL_API double* sl_rsvd_gen_reduce_buffer(void* plan) { return ((GPlan*)plan)->WG; }

// 1: every product of this plan runs on the hand-written kernels (f32 / f64
// A, k <= 64); 0: library GEMMs (bf16 A, or k > 64)
SL_API int sl_rsvd_gen_native(void* plan) { return ((GPlan*)plan)->hand ? 1 : 0; }

// Use caller-owned buffers for the [W; G] reduce buffer ((n + k) * k f64) and
// / or the status words (16 ints; [0] is the call's status), e.g. torch
// tensors the caller all-reduces / reads; null keeps the plan's own.
SL_API int sl_rsvd_gen_bind(void* plan, double* WG, int* status) {
  GPlan* p = (GPlan*)plan;
  if (WG) p->WG = WG;
  if (status) p->st = status;
  return SL_OK;
}
SL_API int* sl_rsvd_gen_status_ptr(void* plan) { return ((GPlan*)plan)->st; }

// segments of one call (2 q + 3) and the WG span (f64 elements) that several
// ranks sum after segment i (count 0: none)
SL_API int sl_rsvd_gen_num_segments(void* plan) { return nseg((GPlan*)plan); }
SL_API int sl_rsvd_gen_reduce_span(void* plan, int i, int64_t* off, int64_t* cnt) {
  reduce_span((GPlan*)plan, i, off, cnt);
  return SL_OK;
}

SL_API int sl_rsvd_gen_segment(void* plan, const void* A, int i, void* stream) {
  return seg((GPlan*)plan, A, i, (hipStream_t)stream);
}

// U (m x r, row stride ldu), s (r), V (n x r): f32 for f32 / bf16 A, f64 for f64 A
SL_API int sl_rsvd_gen_finish(void* plan, void* U, int64_t ldu, void* s_out, void* V, void* stream) {
  GPlan* p = (GPlan*)plan;
  hipStream_t s = (hipStream_t)stream;
  const int k = p->k, r = p->r;
  const int udt = p->dt == SL_BF16 ? SL_F32 : p->dt;
  if (k <= 64) {
    int rc = sl_ts_xm64(p->WG, p->n, k, k, p->N, r, V, r, udt, s);   // V = W N
    if (rc != SL_OK) return rc;
    rc = dispatch_dt(udt, [&](auto* tag) {
      using T = std::remove_pointer_t<decltype(tag)>;
      k_store_s<T><<<1, 256, 0, s>>>(p->eig + k * r, r, (T*)s_out);
      SL_LAUNCH_CHECK();
      return SL_OK;
    });
    if (rc != SL_OK) return rc;
    if (udt == SL_F64) return sl_ts_xm64((const double*)p->Qb, p->m, k, k, p->M, r, U, ldu, SL_F64, s);   // U = Q M
    return sl_tsk_f32_xm((const float*)p->Qb, p->m, k, k, (const float*)p->Md, r, (float*)U, ldu, nullptr, nullptr, s);
  }
  const bool own = p->big || p->dt == SL_BF16;   // hand-written past k = 64 (all but the library A/B)
  int rc = own ? sl_ts_az(p->WG, p->n, k, k, p->N, r, p->Vf, r, SL_F64, s)
                  : slb_gemm(SL_F64, false, false, p->n, r, k, 1.0, p->WG, k, p->N, r, 0.0, p->Vf, r, s);   // V = W N
  if (rc != SL_OK) return rc;
  rc = dispatch_dt(udt, [&](auto* tag) {
    using T = std::remove_pointer_t<decltype(tag)>;
    k_cast2d<double, T><<<grid_of(p->n * r), 256, 0, s>>>(p->Vf, r, p->n, r, (T*)V, r, nullptr);
    SL_LAUNCH_CHECK();
    k_store_s<T><<<1, 256, 0, s>>>(p->eig + k * r, r, (T*)s_out);
    SL_LAUNCH_CHECK();
    return SL_OK;
  });
  if (rc != SL_OK) return rc;
  if (own) return sl_ts_az(p->Qb, p->m, k, k, p->Md, r, U, ldu, udt, s);   // U = Q M
  return slb_gemm(udt, false, false, p->m, r, k, 1.0, p->Qb, k, p->Md, r, 0.0, U, ldu, s);
}

// single rank: every segment, then the finish
SL_API int sl_rsvd_gen_run(void* plan, const void* A, void* U, int64_t ldu, void* s, void* V, void* stream) {
  GPlan* p = (GPlan*)plan;
  for (int i = 0; i < nseg(p); ++i) {
    const int rc = seg(p, A, i, (hipStream_t)stream);
    if (rc != SL_OK) return rc;
  }
  return sl_rsvd_gen_finish(plan, U, ldu, s, V, stream);
}

// several ranks from C: the segments with a NativeComm (RCCL) sum of the
// [W; G] buffer after each pass
SL_API int sl_rsvd_gen_run_comm(void* plan, const void* A, void* comm, void* U, int64_t ldu, void* s, void* V,
                                void* stream) {
  GPlan* p = (GPlan*)plan;
  for (int i = 0; i < nseg(p); ++i) {
    int rc = seg(p, A, i, (hipStream_t)stream);
    if (rc != SL_OK) return rc;
    int64_t off, cnt;
    reduce_span(p, i, &off, &cnt);
    if (cnt && comm) {
      rc = sl_comm_all_reduce(comm, p->WG + off, p->WG + off, cnt, SL_F64, 0, stream);
      if (rc != SL_OK) return rc;
    }
  }
  return sl_rsvd_gen_finish(plan, U, ldu, s, V, stream);
}

// status bits of the last call (synchronises the stream)
SL_API int sl_rsvd_gen_status(void* plan, int* out, void* stream) {
  GPlan* p = (GPlan*)plan;
  SL_HIP_CHECK(hipMemcpyAsync(out, p->st, sizeof(int), hipMemcpyDeviceToHost, (hipStream_t)stream));
  SL_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
  return SL_OK;
}
