// Fused Fastfood random features for large N (reference sketch/FRFT_Elemental.hpp
// :72-160 FastRFT: per block  x -> Sm * F G Pi F (B * x)  with F the
// orthonormal DCT-II, then the cosine feature map of sketch/FRFT_data.hpp).
//
// One workgroup per (data row, Fastfood block): the whole row lives in LDS
// and every step of the block runs there -- the B sign flip, both DCT-IIs
// (Makhoul reorder + real-to-complex packing + an in-LDS Stockham FFT of
// M = N / 2 points, radix 16 with one radix-8/4/2 pass when log2 M is not a
// multiple of 4), the permutation Pi and the Gaussian scale G between them,
// the feature scale Sm and (optionally) the cosine epilogue
// outscale * cos(. + shift) -- and only the block's S features go back to
// HBM.  The previous GPU path ran two rocFFT pipelines per block (a pre
// pass, an R2C, a post gather each) with the whole m x N intermediate
// through HBM four times, plus torch scales and a concatenation.
//
// LDS: two padded complex buffers of M + M/16 points (one float2 of padding
// per 16 keeps the radix-16 pass's stride-16 stores off a single bank), 8.5 N
// bytes: N = 8192 -> 68 KB (two workgroups per CU), N = 16384 -> 136 KB.
// Twiddles come from small per-N tables in global memory (L2 resident):
// W_M^x, W_N^k (k <= M) and W_4N^k.
#include "sl_common.hpp"

namespace {

constexpr int FF_NT = 256;

__host__ __device__ __forceinline__ int padc(int i) { return i + (i >> 4); }
__device__ __forceinline__ float2 cmul(float2 a, float2 b) {
  return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ float2 cadd(float2 a, float2 b) { return make_float2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ float2 csub(float2 a, float2 b) { return make_float2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ float2 mul_mi(float2 a) { return make_float2(a.y, -a.x); }   // -i a

// forward DFTs in registers (X[k] = sum_n x[n] exp(-2 pi i n k / R))
__device__ __forceinline__ void dft4(float2& v0, float2& v1, float2& v2, float2& v3) {
  const float2 a0 = cadd(v0, v2), a1 = csub(v0, v2), b0 = cadd(v1, v3), b1 = mul_mi(csub(v1, v3));
  v0 = cadd(a0, b0);
  v2 = csub(a0, b0);
  v1 = cadd(a1, b1);
  v3 = csub(a1, b1);
}

template <int R>
__device__ __forceinline__ void dft(float2 (&v)[R]);

template <>
__device__ __forceinline__ void dft<2>(float2 (&v)[2]) {
  const float2 a = v[0], b = v[1];
  v[0] = cadd(a, b);
  v[1] = csub(a, b);
}
template <>
__device__ __forceinline__ void dft<4>(float2 (&v)[4]) { dft4(v[0], v[1], v[2], v[3]); }
template <>
__device__ __forceinline__ void dft<8>(float2 (&v)[8]) {
  // n = 2 n1 + n2, k = k1 + 4 k2
  float2 y0[4] = {v[0], v[2], v[4], v[6]}, y1[4] = {v[1], v[3], v[5], v[7]};
  dft4(y0[0], y0[1], y0[2], y0[3]);
  dft4(y1[0], y1[1], y1[2], y1[3]);
  const float h = 0.70710678118654752f;
  y1[1] = cmul(y1[1], make_float2(h, -h));
  y1[2] = mul_mi(y1[2]);
  y1[3] = cmul(y1[3], make_float2(-h, -h));
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1) {
    v[k1] = cadd(y0[k1], y1[k1]);
    v[k1 + 4] = csub(y0[k1], y1[k1]);
  }
}
template <>
__device__ __forceinline__ void dft<16>(float2 (&v)[16]) {
  // n = 4 n1 + n2, k = k1 + 4 k2: 4-point DFTs over n1, twiddle W16^(n2 k1),
  // 4-point DFTs over n2
  float2 y[4][4];
#pragma unroll
  for (int n2 = 0; n2 < 4; ++n2) {
    y[n2][0] = v[n2];
    y[n2][1] = v[4 + n2];
    y[n2][2] = v[8 + n2];
    y[n2][3] = v[12 + n2];
    dft4(y[n2][0], y[n2][1], y[n2][2], y[n2][3]);
  }
  const float c1 = 0.92387953251128676f, s1 = 0.38268343236508977f, h = 0.70710678118654752f;
  // W16^e = (cos 2 pi e / 16, -sin 2 pi e / 16), e = n2 k1
  y[1][1] = cmul(y[1][1], make_float2(c1, -s1));
  y[1][2] = cmul(y[1][2], make_float2(h, -h));
  y[1][3] = cmul(y[1][3], make_float2(s1, -c1));
  y[2][1] = cmul(y[2][1], make_float2(h, -h));
  y[2][2] = mul_mi(y[2][2]);
  y[2][3] = cmul(y[2][3], make_float2(-h, -h));
  y[3][1] = cmul(y[3][1], make_float2(s1, -c1));
  y[3][2] = cmul(y[3][2], make_float2(-h, -h));
  y[3][3] = cmul(y[3][3], make_float2(-c1, s1));
#pragma unroll
  for (int k1 = 0; k1 < 4; ++k1) {
    float2 a = y[0][k1], b = y[1][k1], c = y[2][k1], d = y[3][k1];
    dft4(a, b, c, d);
    v[k1] = a;
    v[k1 + 4] = b;
    v[k1 + 8] = c;
    v[k1 + 12] = d;
  }
}

// one Stockham pass (radix R, sub-transform length Ns so far): natural-order
// output after the last pass
template <int R>
__device__ __forceinline__ void fft_pass(const float2* in, float2* out, int M, int Ns, const float2* __restrict__ twM) {
  const int nbf = M / R;
  for (int j = threadIdx.x; j < nbf; j += FF_NT) {
    float2 v[R];
    const int jm = j & (Ns - 1);
#pragma unroll
    for (int r = 0; r < R; ++r) v[r] = in[padc(j + r * nbf)];
    if (Ns > 1) {
      const int step = jm * (M / (Ns * R));   // W_{Ns R}^{jm r} = W_M^{step r}
#pragma unroll
      for (int r = 1; r < R; ++r) v[r] = cmul(v[r], twM[(step * r) & (M - 1)]);
    }
    dft<R>(v);
    const int idxD = (j - jm) * R + jm;
#pragma unroll
    for (int r = 0; r < R; ++r) out[padc(idxD + r * Ns)] = v[r];
  }
}

// FFT of M = 2^p points from a (padded) into a or b; returns the buffer holding the result
__device__ __forceinline__ float2* fft_m(float2* a, float2* b, int M, int logm, const float2* __restrict__ twM) {
  int Ns = 1;
  float2* src = a;
  float2* dst = b;
  const int n16 = logm / 4, rem = logm % 4;
  for (int p = 0; p < n16; ++p) {
    fft_pass<16>(src, dst, M, Ns, twM);
    __syncthreads();
    Ns *= 16;
    float2* t = src; src = dst; dst = t;
  }
  if (rem) {
    if (rem == 1) fft_pass<2>(src, dst, M, Ns, twM);
    else if (rem == 2) fft_pass<4>(src, dst, M, Ns, twM);
    else fft_pass<8>(src, dst, M, Ns, twM);
    __syncthreads();
    float2* t = src; src = dst; dst = t;
  }
  return src;
}

// orthonormal DCT-II coefficient k (< N) from the packed half-length FFT Z
__device__ __forceinline__ float dct_coef(const float2* Z, int k, int N, int M, const float2* __restrict__ twN,
                                          const float2* __restrict__ tw4N, float c0, float c1) {
  const bool mir = k > M;
  const int kk = mir ? N - k : k;
  const float2 zk = Z[padc(kk & (M - 1))];
  const float2 zm = Z[padc((M - kk) & (M - 1))];
  const float2 zmc = make_float2(zm.x, -zm.y);
  const float2 e = make_float2(0.5f * (zk.x + zmc.x), 0.5f * (zk.y + zmc.y));
  const float2 o = mul_mi(make_float2(0.5f * (zk.x - zmc.x), 0.5f * (zk.y - zmc.y)));
  float2 vk = cadd(e, cmul(twN[kk], o));
  if (mir) vk.y = -vk.y;
  const float2 w = tw4N[k];
  return (w.x * vk.x - w.y * vk.y) * (k == 0 ? c0 : c1);
}

__device__ __forceinline__ int makhoul_src(int n, int N) { return n < N / 2 ? 2 * n : 2 * (N - 1 - n) + 1; }

__device__ __forceinline__ float to_f(float v) { return v; }
__device__ __forceinline__ float to_f(bf16_t v) { return bf16_to_f(v); }

template <typename TA>
__global__ void __launch_bounds__(FF_NT)
k_fastfood(const TA* __restrict__ A, int N, int64_t lda, int logm, const float* __restrict__ Bs,
           const int* __restrict__ perm, const float* __restrict__ G, const float* __restrict__ Sm,
           const float* __restrict__ shifts, float outscale, int epi, int S, int b0, int s_lo, int s_hi,
           const float2* __restrict__ twM, const float2* __restrict__ twN, const float2* __restrict__ tw4N,
           float* __restrict__ out, int64_t ldo) {
  extern __shared__ __attribute__((aligned(16))) float2 ffs[];
  const int M = N >> 1;
  const int PM = padc(M) + 1;
  float2* bufA = ffs;
  float2* bufB = ffs + PM;
  float* fB = (float*)bufB;   // real views (N floats fit: 2 PM > N)
  float* fA = (float*)bufA;
  const int64_t row = blockIdx.x;
  const int blk = b0 + (int)blockIdx.y;
  const float* Bb = Bs + (int64_t)blk * N;
  const int* Pb = perm + (int64_t)blk * N;
  const float* Gb = G + (int64_t)blk * N;
  const float c0 = sqrtf(1.0f / (float)N), c1 = sqrtf(2.0f / (float)N);
  // ---- row -> LDS (coalesced), B applied
  const TA* x = A + row * lda;
  for (int n = threadIdx.x; n < N; n += FF_NT) fB[n] = to_f(x[n]) * Bb[n];
  __syncthreads();
  // ---- Makhoul reorder + real-to-complex packing: z[j] = (u[src(2j)], u[src(2j+1)])
  for (int j = threadIdx.x; j < M; j += FF_NT)
    bufA[padc(j)] = make_float2(fB[makhoul_src(2 * j, N)], fB[makhoul_src(2 * j + 1, N)]);
  __syncthreads();
  float2* Z = fft_m(bufA, bufB, M, logm, twM);
  float* Xf = (float*)(Z == bufA ? bufB : bufA);   // the other buffer, as N reals
  // ---- first DCT-II: every coefficient (the permutation reads them all)
  for (int k = threadIdx.x; k < N; k += FF_NT) Xf[k] = dct_coef(Z, k, N, M, twN, tw4N, c0, c1);
  __syncthreads();
  // ---- y = G * X[perm], repacked for the second DCT-II into Z's buffer
  for (int j = threadIdx.x; j < M; j += FF_NT) {
    const int s0 = makhoul_src(2 * j, N), s1 = makhoul_src(2 * j + 1, N);
    Z[padc(j)] = make_float2(Xf[Pb[s0]] * Gb[s0], Xf[Pb[s1]] * Gb[s1]);
  }
  __syncthreads();
  float2* other = Z == bufA ? bufB : bufA;
  float2* Z2 = fft_m(Z, other, M, logm, twM);
  // ---- second DCT-II: this block's features only, scaled, (cosine epilogue)
  const int f_lo = max(blk * N, s_lo), f_hi = min(min((blk + 1) * N, S), s_hi);
  float* o = out + row * ldo;
  for (int s = f_lo + threadIdx.x; s < f_hi; s += FF_NT) {
    const int k = s - blk * N;
    float v = dct_coef(Z2, k, N, M, twN, tw4N, c0, c1) * Sm[s];
    if (epi) v = outscale * cosf(v + shifts[s]);
    o[s - s_lo] = v;
  }
  (void)fA;
}

__global__ void k_ff_tables(int N, float2* twM, float2* twN, float2* tw4N) {
  const int M = N >> 1;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < N; i += gridDim.x * blockDim.x) {
    double sn, cs;
    if (i < M) {
      sincospi(-2.0 * (double)i / (double)M, &sn, &cs);
      twM[i] = make_float2((float)cs, (float)sn);
    }
    if (i <= M) {
      sincospi(-2.0 * (double)i / (double)N, &sn, &cs);
      twN[i] = make_float2((float)cs, (float)sn);
    }
    sincospi(-(double)i / (2.0 * (double)N), &sn, &cs);
    tw4N[i] = make_float2((float)cs, (float)sn);
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    double sn, cs;
    sincospi(-2.0 * (double)M / (double)N, &sn, &cs);
    twN[M] = make_float2((float)cs, (float)sn);
  }
}

}  // namespace

// floats of the twiddle tables for block size N (a power of two, 2^10..2^14):
// W_M (M), W_N (M + 1), W_4N (N) complex
SL_API int64_t sl_fastfood_tables_size(int N) { return (int64_t)2 * ((N >> 1) + (N >> 1) + 1 + N); }

SL_API int sl_fastfood_tables(int N, float* tab, void* stream) {
  if (N < 1024 || N > 16384 || (N & (N - 1))) {
    sl_set_last_error("fastfood: N must be a power of two in [1024, 16384]");
    return SL_ERR_UNSUPPORTED;
  }
  const int M = N >> 1;
  float2* twM = (float2*)tab;
  float2* twN = twM + M;
  float2* tw4N = twN + M + 1;
  k_ff_tables<<<(N + 255) / 256, 256, 0, (hipStream_t)stream>>>(N, twM, twN, tw4N);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// Fastfood features of the m rows of A (m x N, lda; f32 or bf16), blocks
// b0 .. b1 - 1 of size N, features [s_lo, s_hi) of S into out (m x (s_hi -
// s_lo), ldo): out = Sm * (F G Pi F B x)[block] (epi = 0) or outscale *
// cos(that + shift) (epi = 1).  Bs / G: nb x N f32, perm: nb x N int32
// (indices into [0, N)), Sm / shifts: S f32; tab from sl_fastfood_tables.
SL_API int sl_fastfood_apply(const void* A, int dtype, int64_t m, int N, int64_t lda, const float* Bs, const int* perm,
                             const float* G, const float* Sm, const float* shifts, float outscale, int epi, int S,
                             int b0, int b1, int s_lo, int s_hi, const float* tab, float* out, int64_t ldo,
                             void* stream) {
  if (m <= 0 || b1 <= b0) return SL_OK;
  if (N < 1024 || N > 16384 || (N & (N - 1)) || lda < N || (dtype != SL_F32 && dtype != SL_BF16) ||
      m > 0x7fffffff || b1 - b0 > 65535) {
    sl_set_last_error("fastfood: N a power of two in [1024, 16384], f32 / bf16 rows");
    return SL_ERR_UNSUPPORTED;
  }
  const int M = N >> 1;
  int logm = 0;
  while ((1 << logm) < M) ++logm;
  const float2* twM = (const float2*)tab;
  const float2* twN = twM + M;
  const float2* tw4N = twN + M + 1;
  const size_t lds = (size_t)2 * (padc(M) + 1) * sizeof(float2);
  hipStream_t s = (hipStream_t)stream;
  const dim3 grid((unsigned)m, (unsigned)(b1 - b0));
  if (dtype == SL_F32) {
    SL_LDS_ATTR((k_fastfood<float>), lds);
    k_fastfood<float><<<grid, FF_NT, lds, s>>>((const float*)A, N, lda, logm, Bs, perm, G, Sm, shifts, outscale, epi,
                                               S, b0, s_lo, s_hi, twM, twN, tw4N, out, ldo);
  } else {
    SL_LDS_ATTR((k_fastfood<bf16_t>), lds);
    k_fastfood<bf16_t><<<grid, FF_NT, lds, s>>>((const bf16_t*)A, N, lda, logm, Bs, perm, G, Sm, shifts, outscale,
                                                epi, S, b0, s_lo, s_hi, twM, twN, tw4N, out, ldo);
  }
  SL_LAUNCH_CHECK();
  return SL_OK;
}
