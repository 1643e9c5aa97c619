// Y = A X for a wide f32 operator and a short block X (k <= 4 columns): the
// CG / Chebyshev step of kernel ridge regression on a stored Gram (reference
// ml/krr.hpp:452-541 with algorithms/Krylov/CG.hpp:24-163: one K x product
// per iteration over an n x n Gram, 40 GB at n = 1e5), and any DenseOp whose
// rows are too wide for the one-pass normal kernel (ata_kernels.hip takes
// n <= 6144).  The library GEMV streams such a matrix at ~3.6 TB/s.
//
// gfx950 design: a 256-thread workgroup owns RB = 4 rows and walks their
// columns in float4 steps, U steps per iteration with every load of the
// iteration issued before the FMAs (4 RB + 4 k-row loads of 16 B per thread
// in flight); X arrives transposed (k x n, contiguous rows) so its float4
// loads are contiguous too, and is re-read from L2 by every workgroup (one x
// load serves RB rows).  Per row and column of X the 256 partial dots are
// reduced by a wave shuffle tree and across the 4 waves in LDS.
#include "sl_common.hpp"

namespace {

constexpr int NTG = 256;
constexpr int RB = 4;   // rows per workgroup
constexpr int U = 4;    // float4 steps per iteration

template <int K>
__global__ void __launch_bounds__(NTG)
k_gemv_rows(const float* __restrict__ A, int64_t m, int64_t n, int64_t lda, const float* __restrict__ Xt,
            float* __restrict__ Y, int64_t ldy) {
  __shared__ float red[NTG / 64][RB * K];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * RB;
  const float* rows[RB];
#pragma unroll
  for (int r = 0; r < RB; ++r) rows[r] = A + (r0 + r < m ? r0 + r : m - 1) * lda;
  float acc[RB][K];
#pragma unroll
  for (int r = 0; r < RB; ++r)
#pragma unroll
    for (int kk = 0; kk < K; ++kk) acc[r][kk] = 0.f;
  const int64_t n4 = n / 4;                 // float4 columns (n % 4 == 0)
  const int64_t step = (int64_t)NTG * U;
  for (int64_t c0 = tid; c0 < n4; c0 += step) {
    float4 a[U][RB], x[U][K];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t c = c0 + (int64_t)u * NTG;
      const int64_t cc = c < n4 ? c : n4 - 1;   // clamped: unconditional loads
#pragma unroll
      for (int r = 0; r < RB; ++r) a[u][r] = *(const float4*)(rows[r] + 4 * cc);
#pragma unroll
      for (int kk = 0; kk < K; ++kk) x[u][kk] = *(const float4*)(Xt + kk * n + 4 * cc);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      // steps past the row end re-read its last float4: their x counts zero
      // (a multiply after the load, no branch around it)
      const float ok = c0 + (int64_t)u * NTG < n4 ? 1.f : 0.f;
#pragma unroll
      for (int kk = 0; kk < K; ++kk) {
        const float4 xv = make_float4(ok * x[u][kk].x, ok * x[u][kk].y, ok * x[u][kk].z, ok * x[u][kk].w);
#pragma unroll
        for (int r = 0; r < RB; ++r) {
          float s = acc[r][kk];
          s = fmaf(a[u][r].x, xv.x, s);
          s = fmaf(a[u][r].y, xv.y, s);
          s = fmaf(a[u][r].z, xv.z, s);
          s = fmaf(a[u][r].w, xv.w, s);
          acc[r][kk] = s;
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < RB; ++r)
#pragma unroll
    for (int kk = 0; kk < K; ++kk) {
      float v = acc[r][kk];
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
      if (lane == 0) red[wave][r * K + kk] = v;
    }
  __syncthreads();
  if (tid < RB * K) {
    const int r = tid / K, kk = tid - r * K;
    float s = 0.f;
#pragma unroll
    for (int w = 0; w < NTG / 64; ++w) s += red[w][tid];
    if (r0 + r < m) Y[(r0 + r) * ldy + kk] = s;
  }
}

}  // namespace

// Y (m x k, row stride ldy) = A (m x n f32, lda) X, X given transposed as Xt
// (k x n, contiguous).  Needs k in {1, 2, 4}, n, lda multiples of 4, A and Xt
// 16-B aligned.
SL_API int sl_gemv_rows_f32(const float* A, int64_t m, int64_t n, int64_t lda, const float* Xt, int k, float* Y,
                            int64_t ldy, void* stream) {
  if (m <= 0) return SL_OK;
  if (n <= 0 || n % 4 || lda % 4 || ((uintptr_t)A & 15) || ((uintptr_t)Xt & 15) || !(k == 1 || k == 2 || k == 4)) {
    sl_set_last_error("gemv_rows_f32: needs n, lda multiples of 4, 16-B aligned A / Xt, k in {1, 2, 4}");
    return SL_ERR_INVALID;
  }
  const unsigned g = (unsigned)((m + RB - 1) / RB);
  hipStream_t s = (hipStream_t)stream;
  if (k == 1) k_gemv_rows<1><<<g, NTG, 0, s>>>(A, m, n, lda, Xt, Y, ldy);
  else if (k == 2) k_gemv_rows<2><<<g, NTG, 0, s>>>(A, m, n, lda, Xt, Y, ldy);
  else k_gemv_rows<4><<<g, NTG, 0, s>>>(A, m, n, lda, Xt, Y, ldy);
  SL_LAUNCH_CHECK();
  return SL_OK;
}
