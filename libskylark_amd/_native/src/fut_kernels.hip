// Explicit sampled rows of the orthonormal DCT-II with a diagonal sign/scale:
//     W[j][i] = scale * d[i] * c(p_j) * cos(pi * p_j * (2 i + 1) / (2 N)),
//     c(0) = sqrt(1/N), c(p>0) = sqrt(2/N)
// i.e. the FJLT operator sqrt(N/S) P F D realised in ONE launch (reference
// sketch/FJLT_Elemental.hpp:144-171 applies it as D-scale, DCT, sampling).
// The angle index p (2i+1) is reduced exactly modulo 4N in 64-bit integers
// before the f64 cosine, so entries stay accurate for N up to 2^30.
// transpose = 1 writes the N x S layout (Z = W^T, the power-iteration operand).
#include "sl_common.hpp"

template <typename T>
__global__ void __launch_bounds__(256)
k_dct2_rows(const int64_t* __restrict__ rows, int64_t S, int64_t N, const double* __restrict__ d, double scale,
            T* __restrict__ out, int64_t ld, int transpose) {
  const int64_t total = S * N;
  const double c0 = sqrt(1.0 / (double)N), c1 = sqrt(2.0 / (double)N);
  const double w = 3.14159265358979323846 / (2.0 * (double)N);
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    int64_t j, i;
    if (transpose) { i = t / S; j = t - i * S; }   // out is N x S: consecutive threads walk j
    else { j = t / N; i = t - j * N; }
    const int64_t p = rows[j];
    const int64_t a = (p * (2 * i + 1)) % (4 * N);
    double v = cos(w * (double)a) * (p == 0 ? c0 : c1) * scale;
    if (d) v *= d[i];
    if (transpose) out[i * ld + j] = Cvt<T>::from_d(v);
    else out[j * ld + i] = Cvt<T>::from_d(v);
  }
}

SL_API int sl_dct2_rows(const int64_t* rows, int64_t S, int64_t N, const double* d, double scale, void* out,
                        int dtype, int64_t ld, int transpose, void* stream) {
  if (S <= 0 || N <= 0) return SL_OK;
  unsigned grid = sl_grid_for((size_t)(S * N), 256, 4096);
  hipStream_t s = (hipStream_t)stream;
  SL_DISPATCH_FLOAT(dtype, T, {
    k_dct2_rows<T><<<grid, 256, 0, s>>>(rows, S, N, d, scale, (T*)out, ld, transpose);
  });
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// The whole FJLT operator from the counter-based stream, with its stream
// coordinates read from DEVICE memory (prm = {seed, base_D, base_samples}):
//     W[j][i] = scale * D_i * dct_row(p_j)[i],
//     D_i = Rademacher(seed, base_D + i),  p_j = UniformInt[0, N-1](seed, base_S + j)
// (the draw layout of FJLT_data: N Rademacher signs, then S sample rows).
// Because nothing per-call is a kernel argument, the launch can live inside
// a replayed hipGraph: a new sketch only rewrites the 24-byte prm buffer.
#include "sl_rng.hpp"

template <typename T>
__global__ void __launch_bounds__(256)
k_fjlt_operator(const uint64_t* __restrict__ prm, int64_t S, int64_t N, double scale, T* __restrict__ out,
                int64_t ld, int transpose) {
  const uint64_t seed = prm[0], baseD = prm[1], baseS = prm[2];
  const int64_t total = S * N;
  const double c0 = sqrt(1.0 / (double)N), c1 = sqrt(2.0 / (double)N);
  const double w = 3.14159265358979323846 / (2.0 * (double)N);
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    int64_t j, i;
    if (transpose) { i = t / S; j = t - i * S; }
    else { j = t / N; i = t - j * N; }
    const int64_t p = sl::uniform_int(sl::stream_block(seed, baseS + (uint64_t)j).x, 0, N - 1);
    const double d = (sl::stream_block(seed, baseD + (uint64_t)i).x >> 63) ? 1.0 : -1.0;
    const int64_t a = (p * (2 * i + 1)) % (4 * N);
    const double v = cos(w * (double)a) * (p == 0 ? c0 : c1) * scale * d;
    if (transpose) out[i * ld + j] = Cvt<T>::from_d(v);
    else out[j * ld + i] = Cvt<T>::from_d(v);
  }
}

SL_API int sl_fjlt_operator(const uint64_t* prm, int64_t S, int64_t N, double scale, void* out, int dtype,
                            int64_t ld, int transpose, void* stream) {
  if (S <= 0 || N <= 0) return SL_OK;
  unsigned grid = sl_grid_for((size_t)(S * N), 256, 4096);
  hipStream_t s = (hipStream_t)stream;
  SL_DISPATCH_FLOAT(dtype, T, {
    k_fjlt_operator<T><<<grid, 256, 0, s>>>(prm, S, N, scale, (T*)out, ld, transpose);
  });
  SL_LAUNCH_CHECK();
  return SL_OK;
}
