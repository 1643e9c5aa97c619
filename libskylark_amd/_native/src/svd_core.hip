// Small fp64 stages of the device randomized SVD (nla/svd.py, _DevicePlan),
// fused so that each stage is one or two launches inside the captured graph
// instead of 6-7 library/elementwise kernels of ~5 us each.
//
// Reference math: nla/svd.hpp:71-149 (ApproximateSVD: B = Q^T A, SVD of the
// small factor).  Here B^T = A^T Q = W Rt^{-1} with W = A^T Y (n x k, from the
// final streaming pass) and Rt the Cholesky factor of Y^T Y, and the right
// singular pairs of B come from the k x k Gram C = Vt^T Vt (Vt = W Rt^{-1}).
//
//   sl_svd_core:   Vt = W Rt^{-1} (n x k, f64) and C = Vt^T Vt, symmetric by
//                  construction (only a <= c is summed, mirrored), written
//                  with the breakdown status into the host staging vector
//                  [C (k*k) | status].  Row blocks of 16: Rt^{-1} and the W
//                  block in LDS, per-block C partials in a slab, reduced in a
//                  fixed slab order by a second kernel (one thread per entry)
//                  (deterministic, no float atomics).
//   sl_svd_finish: V = Vt Ub diag(1/s) (n x r, f32), M = Rt^{-1} Ub (k x r,
//                  f32; U = Y M is the caller's tall product) and s as f32.
#include "sl_common.hpp"

namespace {

constexpr int RB = 16;     // rows per block (more blocks: these kernels are latency bound)
constexpr int KMAX = 64;

// global -> LDS staging of n <= 256 * U doubles with every load issued before
// the first LDS store (a rolled copy loop waits on one global load at a time)
template <int U>
__device__ __forceinline__ void stage(double* __restrict__ dst, const double* __restrict__ src, int n, int t) {
  double v[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int e = t + 256 * u;
    v[u] = e < n ? src[e] : 0.0;
  }
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int e = t + 256 * u;
    if (e < n) dst[e] = v[u];
  }
}

// All dot products read LDS in unrolled loops (loads issued ahead of the
// dependent FMA chain) -- the first version, with rolled loops, spent ~30 us
// per kernel waiting on one LDS / global load at a time.
__global__ void __launch_bounds__(256)
k_svd_core_block(const double* __restrict__ W, int n, int k, int ldw, const double* __restrict__ Rti,
                 double* __restrict__ Vt, double* __restrict__ slabs) {
  __shared__ double sR[KMAX * KMAX];
  __shared__ double sW[RB * KMAX];
  __shared__ double sV[RB * KMAX];
  const int t = threadIdx.x;
  const int r0 = blockIdx.x * RB;
  const int rows = min(RB, n - r0);
  stage<KMAX * KMAX / 256>(sR, Rti, k * k, t);
  {
    double v[RB * KMAX / 256];
#pragma unroll
    for (int u = 0; u < RB * KMAX / 256; ++u) {
      const int e = t + 256 * u, i = e / k, j = e - i * k;
      v[u] = (e < RB * k && i < rows) ? W[(int64_t)(r0 + i) * ldw + j] : 0.0;
    }
#pragma unroll
    for (int u = 0; u < RB * KMAX / 256; ++u) {
      const int e = t + 256 * u;
      if (e < RB * k) sW[e] = v[u];
    }
  }
  __syncthreads();
  for (int e = t; e < RB * k; e += 256) {
    const int i = e / k, j = e - i * k;
    const double* w = sW + i * k;
    double v0 = 0.0, v1 = 0.0;
    int l = 0;
#pragma unroll 4
    for (; l + 1 <= j; l += 2) {   // Rt^{-1} upper triangular: l <= j
      v0 = fma(w[l], sR[l * k + j], v0);
      v1 = fma(w[l + 1], sR[(l + 1) * k + j], v1);
    }
    if (l == j) v0 = fma(w[l], sR[l * k + j], v0);
    const double v = v0 + v1;
    sV[e] = v;
    if (i < rows) Vt[(int64_t)(r0 + i) * k + j] = v;
  }
  __syncthreads();
  double* slab = slabs + (int64_t)blockIdx.x * k * k;
  for (int e = t; e < k * k; e += 256) {
    const int a = e / k, c = e - a * k;
    double s0 = 0.0, s1 = 0.0;
    if (a <= c) {
#pragma unroll
      for (int i = 0; i < RB; i += 2) {     // padded rows are zero
        s0 = fma(sV[i * k + a], sV[i * k + c], s0);
        s1 = fma(sV[(i + 1) * k + a], sV[(i + 1) * k + c], s1);
      }
    }
    slab[e] = s0 + s1;
  }
}

// one thread per entry a <= c, slabs summed in order (loads unrolled ahead)
__global__ void __launch_bounds__(256)
k_svd_core_reduce(const double* __restrict__ slabs, int nb, int k, const int* __restrict__ status,
                  double* __restrict__ host_src) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e == 0) host_src[k * k] = status ? (double)status[0] : 0.0;
  if (e >= k * k) return;
  const int a = e / k, c = e - a * k;
  if (a > c) return;
  const int64_t kk = (int64_t)k * k;
  double s = 0.0;
  int b = 0;
  for (; b + 8 <= nb; b += 8) {
    double x[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) x[u] = slabs[(b + u) * kk + e];
#pragma unroll
    for (int u = 0; u < 8; ++u) s += x[u];
  }
  for (; b < nb; ++b) s += slabs[b * kk + e];
  host_src[a * k + c] = s;
  host_src[c * k + a] = s;
}

__global__ void __launch_bounds__(256)
k_svd_finish(const double* __restrict__ Vt, int n, int k, const double* __restrict__ Rti,
             const double* __restrict__ small, int r, float* __restrict__ V, float* __restrict__ M,
             float* __restrict__ s32) {
  __shared__ double sU[KMAX * KMAX];
  __shared__ double sA[KMAX * KMAX];   // Vt row block (RB x k) or Rt^{-1} (k x k)
  __shared__ double sinv[KMAX];
  const int t = threadIdx.x;
  const double* Ub = small;          // k x r, row-major
  const double* s = small + k * r;   // r singular values
  stage<KMAX * KMAX / 256>(sU, Ub, k * r, t);
  if (t < r) sinv[t] = 1.0 / fmax(s[t], 1e-300);
  const int nb = (n + RB - 1) / RB;
  const bool last = (int)blockIdx.x == nb;
  const int r0 = blockIdx.x * RB;
  const int rows = last ? k : min(RB, n - r0);
  const double* src = last ? Rti : Vt + (int64_t)r0 * k;
  stage<KMAX * KMAX / 256>(sA, src, rows * k, t);
  __syncthreads();
  for (int e = t; e < rows * r; e += 256) {
    const int i = e / r, j = e - i * r;
    const double* a = sA + i * k;
    double v0 = 0.0, v1 = 0.0;
    int l = 0;
#pragma unroll 4
    for (; l + 2 <= k; l += 2) {
      v0 = fma(a[l], sU[l * r + j], v0);
      v1 = fma(a[l + 1], sU[(l + 1) * r + j], v1);
    }
    if (l < k) v0 = fma(a[l], sU[l * r + j], v0);
    const double v = v0 + v1;
    if (last) M[e] = (float)v;
    else V[(int64_t)(r0 + i) * r + j] = (float)(v * sinv[j]);
  }
  if (last)
    for (int j = t; j < r; j += 256) s32[j] = (float)s[j];
}

}  // namespace

// slabs: ceil(n / 16) * k * k doubles of workspace.
SL_API int sl_svd_core(const double* W, int n, int k, int ldw, const double* Rti, double* Vt, double* slabs,
                       double* host_src, const int* status, void* stream) {
  if (k < 1 || k > KMAX || n < 1) {
    sl_set_last_error("svd_core: 1 <= k <= 64, n >= 1");
    return SL_ERR_UNSUPPORTED;
  }
  hipStream_t s = (hipStream_t)stream;
  const int nb = (n + RB - 1) / RB;
  k_svd_core_block<<<nb, 256, 0, s>>>(W, n, k, ldw, Rti, Vt, slabs);
  k_svd_core_reduce<<<(k * k + 255) / 256, 256, 0, s>>>(slabs, nb, k, status, host_src);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

SL_API int sl_svd_finish(const double* Vt, int n, int k, const double* Rti, const double* small, int r, float* V,
                         float* M, float* s32, void* stream) {
  if (k < 1 || k > KMAX || r < 1 || r > k || n < 1) {
    sl_set_last_error("svd_finish: 1 <= r <= k <= 64, n >= 1");
    return SL_ERR_UNSUPPORTED;
  }
  const int nb = (n + RB - 1) / RB;
  k_svd_finish<<<nb + 1, 256, 0, (hipStream_t)stream>>>(Vt, n, k, Rti, small, r, V, M, s32);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

SL_API int sl_tsk_f32_xm(const float* Y, int64_t m, int k, int64_t ldy, const float* M, int k2, float* out,
                         int64_t ldo, double* G, void* ws, void* stream);

// The randSVD call's last two launches from one host call: V, M, s from the
// eigenpairs (sl_svd_finish), then U = Y M (m x r, sl_tsk_f32_xm) -- the
// host-side launch cost sits on the critical path between the eigensolve
// and the end of the call.
SL_API int sl_svd_finish_u(const double* Vt, int n, int k, const double* Rti, const double* small, int r, float* V,
                           float* M, float* s32, const float* Y, int64_t m, float* U, void* stream) {
  int rc = sl_svd_finish(Vt, n, k, Rti, small, r, V, M, s32, stream);
  if (rc != SL_OK) return rc;
  return sl_tsk_f32_xm(Y, m, k, k, M, r, U, r, nullptr, nullptr, stream);
}
