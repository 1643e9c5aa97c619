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

// ---------------------------------------------------------------------------
// FJLT / RFUT DCT-II pipeline for large S (reference sketch/FJLT_Elemental.hpp
// :144-171, RFUT_Elemental.hpp:66-85, utility/fft/fftw_futs.h:50-108).
//   pre:  v = Makhoul reorder of (D x) along the transform axis, in one pass
//         (v[n] = d[2n] x[2n] for n < ceil(N/2), v[N-1-n] = d[2n+1] x[2n+1]),
//         written as f32 for rocFFT's real-to-complex transform;
//   post: only the S sampled frequencies k_s of the orthonormal DCT-II,
//         X_k = c_k Re(e^{-i pi k / 2N} V_k) with V_k = conj(V_{N-k}) past N/2,
//         times the sketch scale -- one gather of S rows/columns of the
//         half spectrum instead of the full transform + index_select.
// Layout: the transform runs along dim 0 (N x m, row-major) or dim 1 (m x N).

template <typename T>
__global__ void __launch_bounds__(256)
k_fjlt_pre(const T* __restrict__ x, int64_t N, int64_t m, int64_t ldx, int dim, const double* __restrict__ d,
           float* __restrict__ v, int64_t ldv) {
  const int64_t total = N * m;
  const int64_t half = (N + 1) / 2;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    int64_t n, c;
    if (dim == 0) { n = t / m; c = t - n * m; }   // consecutive threads along the row (coalesced)
    else { c = t / N; n = t - c * N; }
    const int64_t src = n < half ? 2 * n : 2 * (N - 1 - n) + 1;
    const float sgn = (float)d[src];
    if (dim == 0) v[n * ldv + c] = sgn * Cvt<T>::to_f(x[src * ldx + c]);
    else v[c * ldv + n] = sgn * Cvt<T>::to_f(x[c * ldx + src]);
  }
}

// dim 0 input (N x m) written TRANSPOSED (m x N) so that rocFFT runs
// contiguous transforms (a strided N = 1e6 transform over 1000 columns ran
// ~10x below the contiguous one): 64 x 64 tiles through LDS, coalesced on
// both sides.
template <typename T>
__global__ void __launch_bounds__(256)
k_fjlt_pre_t(const T* __restrict__ x, int64_t N, int64_t m, int64_t ldx, const double* __restrict__ d,
             float* __restrict__ vt, int64_t ldv) {
  __shared__ float tile[64][65];
  const int64_t half = (N + 1) / 2;
  const int64_t n0 = (int64_t)blockIdx.x * 64, c0 = (int64_t)blockIdx.y * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int64_t n = n0 + i, c = c0 + tx;
    float val = 0.f;
    if (n < N && c < m) {
      const int64_t src = n < half ? 2 * n : 2 * (N - 1 - n) + 1;
      val = (float)d[src] * Cvt<T>::to_f(x[src * ldx + c]);
    }
    tile[i][tx] = val;
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int64_t c = c0 + i, n = n0 + tx;
    if (c < m && n < N) vt[c * ldv + n] = tile[tx][i];
  }
}

// V: complex half spectrum (interleaved f32 pairs), (N/2+1) x m (vt = 0) or
// m x (N/2+1) (vt = 1), leading dimension ldV in complex elements; the output
// is S x m (ot = 0) or m x S (ot = 1).
__global__ void __launch_bounds__(256)
k_fjlt_post(const float2* __restrict__ V, int64_t N, int64_t m, int64_t ldV, int vt, int ot,
            const int64_t* __restrict__ samples, int64_t S, double scale, float* __restrict__ out, int64_t ldo) {
  const int64_t total = S * m;
  const double c0 = sqrt(1.0 / (double)N), c1 = sqrt(2.0 / (double)N);
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    int64_t s, c;
    if (ot == 0) { s = t / m; c = t - s * m; }
    else { c = t / S; s = t - c * S; }
    const int64_t k = samples[s];
    const bool mirror = 2 * k > N;
    const int64_t kk = mirror ? N - k : k;
    const float2 z = vt == 0 ? V[kk * ldV + c] : V[c * ldV + kk];
    const double re = z.x, im = mirror ? -(double)z.y : (double)z.y;
    // angle -pi k / 2N reduced exactly in integers (k < N)
    double sn, cs;
    sincospi(-(double)k / (2.0 * (double)N), &sn, &cs);
    const double val = (re * cs - im * sn) * (k == 0 ? c0 : c1) * scale;
    if (ot == 0) out[s * ldo + c] = (float)val;
    else out[c * ldo + s] = (float)val;
  }
}

// dim = 2: dim-0 input (N x m) written transposed (m x N, row stride ldv)
SL_API int sl_fjlt_pre(const void* x, int dtype, int64_t N, int64_t m, int64_t ldx, int dim, const double* d,
                       float* v, int64_t ldv, void* stream) {
  if (N <= 0 || m <= 0) return SL_OK;
  hipStream_t s = (hipStream_t)stream;
  if (dim == 2) {
    dim3 grid((unsigned)((N + 63) / 64), (unsigned)((m + 63) / 64));
    if (dtype == SL_F32) k_fjlt_pre_t<float><<<grid, 256, 0, s>>>((const float*)x, N, m, ldx, d, v, ldv);
    else if (dtype == SL_BF16) k_fjlt_pre_t<bf16_t><<<grid, 256, 0, s>>>((const bf16_t*)x, N, m, ldx, d, v, ldv);
    else { sl_set_last_error("fjlt_pre: f32 or bf16 input"); return SL_ERR_UNSUPPORTED; }
    SL_LAUNCH_CHECK();
    return SL_OK;
  }
  const unsigned grid = sl_grid_for((size_t)(N * m), 256, 8192);
  if (dtype == SL_F32) k_fjlt_pre<float><<<grid, 256, 0, s>>>((const float*)x, N, m, ldx, dim, d, v, ldv);
  else if (dtype == SL_BF16) k_fjlt_pre<bf16_t><<<grid, 256, 0, s>>>((const bf16_t*)x, N, m, ldx, dim, d, v, ldv);
  else { sl_set_last_error("fjlt_pre: f32 or bf16 input"); return SL_ERR_UNSUPPORTED; }
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// layout = vt + 2 * ot (see k_fjlt_post)
SL_API int sl_fjlt_post(const void* V, int64_t N, int64_t m, int64_t ldV, int layout, const int64_t* samples, int64_t S,
                        double scale, float* out, int64_t ldo, void* stream) {
  if (S <= 0 || m <= 0) return SL_OK;
  const unsigned grid = sl_grid_for((size_t)(S * m), 256, 8192);
  k_fjlt_post<<<grid, 256, 0, (hipStream_t)stream>>>((const float2*)V, N, m, ldV, layout & 1, (layout >> 1) & 1,
                                                       samples, S, scale, out, ldo);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// ---------------------------------------------------------------------------
// PPT / TensorSketch spectral product (reference sketch/PPT_Elemental.hpp
// :140-185).  F holds the q half spectra (q x (S/2+1) x m, complex f32) of the
// UNSCALED CountSketches C_i A; the reference adds sqrt(c) h_i e_{idx_i} to
// sqrt(gamma) C_i A before its FFT, which is folded in analytically here:
//     P[k][c] = prod_i ( sqrt(gamma) F_i[k][c] + sqrt(c) h_i w^(k idx_i) ),
//     w = exp(-2 pi i / S)
// -- one pass over the q spectra, no per-sketch scale / add / multiply passes.
__global__ void __launch_bounds__(256)
k_ppt_product(const float2* __restrict__ F, int q, int64_t K, int64_t m, int64_t S, const int64_t* __restrict__ idx,
              const double* __restrict__ hv, double sg, double sc, float2* __restrict__ P) {
  const int64_t total = K * m;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = t / m;
    float pr = 1.f, pi = 0.f;
    for (int i = 0; i < q; ++i) {
      const float2 z = F[(int64_t)i * total + t];
      // w^(k idx) with the exponent reduced mod S in integers (exact angle)
      const int64_t e = (k * idx[i]) % S;
      double sn, cs;
      sincospi(-2.0 * (double)e / (double)S, &sn, &cs);
      const float ar = (float)(sg * z.x + sc * hv[i] * cs), ai = (float)(sg * z.y + sc * hv[i] * sn);
      const float nr = pr * ar - pi * ai, ni = pr * ai + pi * ar;
      pr = nr;
      pi = ni;
    }
    P[t] = make_float2(pr, pi);
  }
}

SL_API int sl_ppt_product(const void* F, int q, int64_t K, int64_t m, int64_t S, const int64_t* idx, const double* hv,
                          double sg, double sc, void* P, void* stream) {
  if (K <= 0 || m <= 0) return SL_OK;
  const unsigned grid = sl_grid_for((size_t)(K * m), 256, 8192);
  k_ppt_product<<<grid, 256, 0, (hipStream_t)stream>>>((const float2*)F, q, K, m, S, idx, hv, sg, sc, (float2*)P);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// ------------------------------------------------------------------ WHT
// Orthonormal Walsh-Hadamard transform of V vectors of length N (power of
// two, N * V * 4 B <= 64 KB) per workgroup, entirely in LDS: one coalesced
// load of the tile, log2 N butterfly stages (each a pass of 256 threads over
// the N/2 pairs of every vector, one barrier per stage), the 1/sqrt(N) scale
// folded into the store.  Element e of vector v is x[v * vs + e * es]: dim 0
// of a row-major N x m matrix has es = ld, vs = 1 (V consecutive columns per
// workgroup -> 4V-byte contiguous row pieces), dim 1 has es = 1, vs = ld.
// Reference: the Spiral WHT of utility/fft/fftw_futs.h (WHT_t).
namespace {
template <typename T>
__global__ void __launch_bounds__(256) k_wht_lds(const T* __restrict__ x, T* __restrict__ y, int64_t nvec, int N,
                                                 int V, int64_t es, int64_t vs, int logn, float scale) {
  extern __shared__ __attribute__((aligned(16))) float tile[];   // [N][V], vector index fastest
  const int64_t v0 = (int64_t)blockIdx.x * V;
  const int vcount = (int)((nvec - v0) < V ? (nvec - v0) : V);
  const int tot = N * V;
  for (int t = threadIdx.x; t < tot; t += 256) {
    const int e = t / V, v = t - e * V;
    tile[t] = v < vcount ? (float)Cvt<T>::to_f(x[(v0 + v) * vs + (int64_t)e * es]) : 0.f;
  }
  __syncthreads();
  const int pairs = (N >> 1) * V;
  for (int s = 0; s < logn; ++s) {
    const int h = 1 << s;
    for (int t = threadIdx.x; t < pairs; t += 256) {
      const int pv = t / V, v = t - pv * V;                 // pair index within the vector
      const int i = ((pv >> s) << (s + 1)) + (pv & (h - 1));
      const float a = tile[i * V + v], b = tile[(i + h) * V + v];
      tile[i * V + v] = a + b;
      tile[(i + h) * V + v] = a - b;
    }
    __syncthreads();
  }
  for (int t = threadIdx.x; t < tot; t += 256) {
    const int e = t / V, v = t - e * V;
    if (v < vcount) y[(v0 + v) * vs + (int64_t)e * es] = Cvt<T>::from_f(tile[t] * scale);
  }
}
}  // namespace

// y = WHT(x) / sqrt(N) on nvec vectors (element stride es, vector stride vs);
// x and y may alias.  N a power of two, N <= 16384.
SL_API int sl_wht(const void* x, void* y, int dtype, int64_t nvec, int N, int64_t es, int64_t vs, void* stream) {
  if (nvec <= 0) return SL_OK;
  if (N < 1 || (N & (N - 1)) || N > 16384) {
    sl_set_last_error("wht: N must be a power of two <= 16384");
    return SL_ERR_UNSUPPORTED;
  }
  if (dtype != SL_F32 && dtype != SL_BF16) {
    sl_set_last_error("wht: f32 / bf16 (f64 stays on the host path)");
    return SL_ERR_UNSUPPORTED;
  }
  int logn = 0;
  while ((1 << logn) < N) ++logn;
  // vectors per workgroup: up to 16 (64-B row pieces for dim 0), LDS <= 64 KB
  int V = es == 1 ? 1 : 16;
  while (V > 1 && (int64_t)N * V * 4 > 65536) V >>= 1;
  const size_t lds = (size_t)N * V * 4;
  const unsigned grid = (unsigned)((nvec + V - 1) / V);
  const float scale = 1.0f / sqrtf((float)N);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SL_F32)
    k_wht_lds<float><<<grid, 256, lds, s>>>((const float*)x, (float*)y, nvec, N, V, es, vs, logn, scale);
  else
    k_wht_lds<bf16_t><<<grid, 256, lds, s>>>((const bf16_t*)x, (bf16_t*)y, nvec, N, V, es, vs, logn, scale);
  SL_LAUNCH_CHECK();
  return SL_OK;
}
