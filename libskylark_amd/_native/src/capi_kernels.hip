// Small device kernels of the C API's interpreter-free paths (capi/
// native_device.hpp): host "Matrix" / "SparseMatrix" operands are staged to
// the GPU, and these fill the gaps between the library GEMMs and the sketch
// kernels:
//   sl_transpose        LDS-tiled out = in^T (f32 / f64): a column-major host
//                       matrix is the row-major transpose, so the tall /
//                       wide re-orientations of the NLA paths are one pass
//   sl_csr_to_dense     CSR (int32 indices, f64 values) scattered into a
//                       zeroed row-major dense buffer (duplicates summed)
//   sl_dft_cs           cos / sin tables C[k][t] = cos(2 pi (k t mod S) / S)
//                       (the angle index reduced exactly in 64-bit integers):
//                       the TensorSketch (PPT) DFTs as GEMMs on the matrix cores
//   sl_ppt_spectrum     prod_i (F_i + sqrt(c) h_i e^{-2 pi i k idx_i / S}) with
//                       the irfft weights w_k / S folded in
//   sl_symmetrize       full symmetric copy of one stored triangle
//   sl_dev_count        visible devices (0 on a GPU-less host)
#include "sl_common.hpp"

namespace {

template <typename T>
__global__ void __launch_bounds__(256) k_transpose(const T* __restrict__ in, int64_t rows, int64_t cols, int64_t ldi,
                                                   T* __restrict__ out, int64_t ldo) {
  __shared__ T tile[64][65];
  const int64_t r0 = (int64_t)blockIdx.y * 64, c0 = (int64_t)blockIdx.x * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;   // 64 x 4
  for (int y = ty; y < 64; y += 4) {
    const int64_t r = r0 + y, c = c0 + tx;
    if (r < rows && c < cols) tile[y][tx] = in[r * ldi + c];
  }
  __syncthreads();
  for (int y = ty; y < 64; y += 4) {
    const int64_t c = c0 + y, r = r0 + tx;   // out row c, column r
    if (r < rows && c < cols) out[c * ldo + r] = tile[tx][y];
  }
}

template <typename T>
__global__ void __launch_bounds__(256) k_csr_to_dense(const int* __restrict__ rowptr, const int* __restrict__ col,
                                                      const double* __restrict__ val, int64_t nrows,
                                                      T* __restrict__ out, int64_t ld) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= nrows) return;
  for (int64_t q = rowptr[r] + (threadIdx.x & 63); q < rowptr[r + 1]; q += 64)
    atomicAdd(&out[r * ld + col[q]], (T)val[q]);
}

template <typename T>
__global__ void __launch_bounds__(256) k_dft_cs(int64_t S, int64_t K, T* __restrict__ C, T* __restrict__ Sn) {
  const double w = 6.283185307179586476925 / (double)S;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < K * S; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = t / S, n = t - k * S;
    const double a = w * (double)((k * n) % S);
    C[t] = (T)cos(a);
    Sn[t] = (T)sin(a);
  }
}

// F: 2q planes (q cosine transforms C u_i, then q sine transforms S u_i, so
// DFT(u_i) = C u_i - i S u_i) of K x ncol entries at (k, c) -> k * sk + c * sc;
// P: 2 planes (real, imaginary), same layout
template <typename T>
__global__ void __launch_bounds__(256) k_ppt_spectrum(const T* __restrict__ F, int q, int64_t K, int64_t ncol,
                                                      int64_t sk, int64_t sc, int64_t plane, int64_t S,
                                                      const int64_t* __restrict__ hidx, const double* __restrict__ hval,
                                                      double csq, T* __restrict__ P) {
  const double w = 6.283185307179586476925 / (double)S;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < K * ncol; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = t / ncol, c = t - k * ncol, o = k * sk + c * sc;
    double pr = 1.0, pi = 0.0;
    for (int i = 0; i < q; ++i) {
      const double a = w * (double)((k * hidx[i]) % S);
      const double re = (double)F[i * plane + o] + csq * hval[i] * cos(a);
      const double im = -(double)F[(q + i) * plane + o] - csq * hval[i] * sin(a);
      const double nr = pr * re - pi * im;
      pi = pr * im + pi * re;
      pr = nr;
    }
    const double wk = (k == 0 || (S % 2 == 0 && k == S / 2)) ? 1.0 : 2.0;
    P[o] = (T)(pr * wk / (double)S);
    P[plane + o] = (T)(pi * wk / (double)S);
  }
}

template <typename T>
__global__ void __launch_bounds__(256) k_symmetrize(const T* __restrict__ A, int64_t n, int64_t lda, int lower,
                                                    T* __restrict__ out, int64_t ldo) {
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n * n; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t j = t / n, i = t - j * n;   // column-major (i, j)
    const bool mine = lower ? i >= j : i <= j;
    out[i + j * ldo] = mine ? A[i + j * lda] : A[j + i * lda];
  }
}

}  // namespace

SL_API int sl_transpose(const void* in, int dtype, int64_t rows, int64_t cols, int64_t ldi, void* out, int64_t ldo,
                        void* stream) {
  if (rows <= 0 || cols <= 0) return SL_OK;
  if ((cols + 63) / 64 > 0x7fffffff || (rows + 63) / 64 > 65535) {
    sl_set_last_error("transpose: too many row tiles");
    return SL_ERR_UNSUPPORTED;
  }
  dim3 grid((unsigned)((cols + 63) / 64), (unsigned)((rows + 63) / 64));
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SL_F64) k_transpose<double><<<grid, 256, 0, s>>>((const double*)in, rows, cols, ldi, (double*)out, ldo);
  else if (dtype == SL_F32) k_transpose<float><<<grid, 256, 0, s>>>((const float*)in, rows, cols, ldi, (float*)out, ldo);
  else { sl_set_last_error("transpose: f32 / f64"); return SL_ERR_UNSUPPORTED; }
  SL_LAUNCH_CHECK();
  return SL_OK;
}

SL_API int sl_csr_to_dense(const int* rowptr, const int* col, const double* val, int64_t nrows, void* out, int dtype,
                           int64_t ld, void* stream) {
  if (nrows <= 0) return SL_OK;
  const unsigned grid = (unsigned)((nrows + 3) / 4);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SL_F64) k_csr_to_dense<double><<<grid, 256, 0, s>>>(rowptr, col, val, nrows, (double*)out, ld);
  else if (dtype == SL_F32) k_csr_to_dense<float><<<grid, 256, 0, s>>>(rowptr, col, val, nrows, (float*)out, ld);
  else { sl_set_last_error("csr_to_dense: f32 / f64"); return SL_ERR_UNSUPPORTED; }
  SL_LAUNCH_CHECK();
  return SL_OK;
}

SL_API int sl_dft_cs(int64_t S, int64_t K, void* C, void* Sn, int dtype, void* stream) {
  if (S <= 0 || K <= 0) return SL_OK;
  const unsigned grid = sl_grid_for((size_t)(K * S), 256, 8192);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SL_F64) k_dft_cs<double><<<grid, 256, 0, s>>>(S, K, (double*)C, (double*)Sn);
  else if (dtype == SL_F32) k_dft_cs<float><<<grid, 256, 0, s>>>(S, K, (float*)C, (float*)Sn);
  else { sl_set_last_error("dft_cs: f32 / f64"); return SL_ERR_UNSUPPORTED; }
  SL_LAUNCH_CHECK();
  return SL_OK;
}

SL_API int sl_ppt_spectrum(const void* F, int q, int64_t K, int64_t ncol, int64_t sk, int64_t sc, int64_t plane,
                           int64_t S, const int64_t* hidx, const double* hval, double csq, void* P, int dtype,
                           void* stream) {
  if (K <= 0 || ncol <= 0) return SL_OK;
  const unsigned grid = sl_grid_for((size_t)(K * ncol), 256, 8192);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SL_F64)
    k_ppt_spectrum<double><<<grid, 256, 0, s>>>((const double*)F, q, K, ncol, sk, sc, plane, S, hidx, hval, csq,
                                                (double*)P);
  else if (dtype == SL_F32)
    k_ppt_spectrum<float><<<grid, 256, 0, s>>>((const float*)F, q, K, ncol, sk, sc, plane, S, hidx, hval, csq,
                                               (float*)P);
  else { sl_set_last_error("ppt_spectrum: f32 / f64"); return SL_ERR_UNSUPPORTED; }
  SL_LAUNCH_CHECK();
  return SL_OK;
}

SL_API int sl_symmetrize(const void* A, int dtype, int64_t n, int64_t lda, int lower, void* out, int64_t ldo,
                         void* stream) {
  if (n <= 0) return SL_OK;
  const unsigned grid = sl_grid_for((size_t)(n * n), 256, 8192);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SL_F64) k_symmetrize<double><<<grid, 256, 0, s>>>((const double*)A, n, lda, lower, (double*)out, ldo);
  else if (dtype == SL_F32) k_symmetrize<float><<<grid, 256, 0, s>>>((const float*)A, n, lda, lower, (float*)out, ldo);
  else { sl_set_last_error("symmetrize: f32 / f64"); return SL_ERR_UNSUPPORTED; }
  SL_LAUNCH_CHECK();
  return SL_OK;
}

SL_API int sl_dev_count(int* n) {
  *n = 0;
  if (hipGetDeviceCount(n) != hipSuccess) {
    (void)hipGetLastError();
    *n = 0;
  }
  return SL_OK;
}
