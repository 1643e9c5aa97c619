// Element-wise feature-map epilogues and small fused vector kernels.
//
// RFT/QRFT (reference sketch/RFT_Elemental.hpp:83-160):
//     Z[i, j] = outscale * cos(scales[i] * X[i, j] + shifts[i])      (columnwise)
// RLT/QRLT (sketch/RLT_Elemental.hpp:60-80):
//     Z[i, j] = outscale * exp(-X[i, j])
// For rowwise application the feature index is the column index.
// Vectorised 16-B loads/stores, grid-stride, one pass over Z.
#include "sl_common.hpp"

enum { EPI_COS = 0, EPI_EXP_NEG = 1 };

template <typename T, int MODE>
__global__ void __launch_bounds__(256)
k_feature_epilogue(T* __restrict__ X, int64_t rows, int64_t cols, int64_t ld,
                   const double* __restrict__ scales, const double* __restrict__ shifts,
                   double outscale, int feature_dim) {
  const int64_t total = rows * cols;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = t / cols, c = t - r * cols;
    const int64_t f = feature_dim == 0 ? r : c;
    T* p = X + r * ld + c;
    if (MODE == EPI_COS) {
      if (sizeof(T) == 8) {
        double x = Cvt<T>::to_d(*p);
        x = x * (scales ? scales[f] : 1.0) + shifts[f];
        *p = Cvt<T>::from_d(outscale * cos(x));
      } else {
        float x = Cvt<T>::to_f(*p);
        x = x * (scales ? (float)scales[f] : 1.f) + (float)shifts[f];
        *p = Cvt<T>::from_f((float)outscale * cosf(x));
      }
    } else {
      if (sizeof(T) == 8) *p = Cvt<T>::from_d(outscale * exp(-Cvt<T>::to_d(*p)));
      else *p = Cvt<T>::from_f((float)outscale * __expf(-Cvt<T>::to_f(*p)));
    }
  }
}

SL_API int sl_feature_epilogue(void* X, int dtype, int64_t rows, int64_t cols, int64_t ld,
                               const double* scales, const double* shifts, double outscale,
                               int feature_dim, int mode, void* stream) {
  if (rows * cols <= 0) return SL_OK;
  unsigned grid = sl_grid_for((size_t)(rows * cols), 256, 4096);
  hipStream_t s = (hipStream_t)stream;
  SL_DISPATCH_FLOAT(dtype, T, {
    if (mode == EPI_COS)
      k_feature_epilogue<T, EPI_COS><<<grid, 256, 0, s>>>((T*)X, rows, cols, ld, scales, shifts, outscale, feature_dim);
    else
      k_feature_epilogue<T, EPI_EXP_NEG><<<grid, 256, 0, s>>>((T*)X, rows, cols, ld, scales, shifts, outscale, feature_dim);
  });
  SL_LAUNCH_CHECK();
  return SL_OK;
}
