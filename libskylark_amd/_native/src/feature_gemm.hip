// Fused dense-sketch / random-feature GEMM on bf16 MFMA (K1 + K6 of SURVEY §2.4).
//
//   Z[r, f] = outscale * epi( scale_f * sum_k A[r, k] * W[f, k] + shift_f )
//
// A (M x K, row-major, f32 or bf16) is the input (rows = examples for a
// rowwise apply, the transposed input for a columnwise one); W (Nf x K) is
// the realised sketching matrix of a dense transform (JLT / CT / SJLT) or
// the frequency matrix of a feature map (RFT / QRFT / RLT / QRLT), held as a
// bf16 hi + lo pair so that W_hi + W_lo equals the f32 realisation to
// ~2^-17.  epi = identity (linear sketches), cos (Fourier features,
// reference sketch/RFT_Elemental.hpp:83-160) or exp(-x) (Laplace features,
// sketch/RLT_Elemental.hpp:60-80).  The output is written row-major
// (Z[r*ldo + f]) or transposed (Z[f*ldo + r], columnwise apply).
//
// Reference counterpart: dense_transform_t realises S panel by panel and
// calls a BLAS GEMM, then RFT applies the cosine in a separate loop; here the
// GEMM and the nonlinearity are one launch, so the M x Nf product never
// round-trips through HBM before the epilogue.
//
// gfx950 design:
//   * 128 x 128 output tile per 256-thread workgroup (2 x 2 waves, each a
//     64 x 64 block = 4 x 4 v_mfma_f32_16x16x32_bf16 tiles), 64 KB of LDS so
//     two workgroups share a CU and hide each other's load latency;
//   * f32 A is split in-kernel into bf16 hi + lo while staging to LDS, and
//     the product is the 3-term sum  Ah*Wh + Al*Wh + Ah*Wl  (f32-class
//     accuracy at 3/16 of the bf16 MFMA cost instead of f32 MFMA's 1/16 rate);
//   * K slices of 32 are double-buffered in LDS (64-B rows: ds_read_b128 of
//     a 16-row x 32-k fragment touches 1 KB contiguous, conflict free) and
//     the global loads run two slices ahead in two register sets;
//   * MFMAs are issued term-major (16 independent accumulators between two
//     updates of the same one);
//   * XCD-aware tile order: W is split over the 8 XCDs (each XCD's slice of W
//     stays L2 resident while A streams past), see the kernel's mapping.
#include "sl_common.hpp"

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int BM = 128, BN = 128, BK = 32, NT = 256;

enum { EPI_NONE = 0, EPI_COS = 1, EPI_EXPNEG = 2 };

__device__ __forceinline__ uint32_t f2bf_bits(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7fffu + ((u >> 16) & 1u);
  return u >> 16;
}

// split 4 floats into packed bf16 hi (2 x u32) and lo (2 x u32)
__device__ __forceinline__ void split4(const float4 v, uint2& hi, uint2& lo) {
  uint32_t h0 = f2bf_bits(v.x), h1 = f2bf_bits(v.y), h2 = f2bf_bits(v.z), h3 = f2bf_bits(v.w);
  uint32_t l0 = f2bf_bits(v.x - __uint_as_float(h0 << 16));
  uint32_t l1 = f2bf_bits(v.y - __uint_as_float(h1 << 16));
  uint32_t l2 = f2bf_bits(v.z - __uint_as_float(h2 << 16));
  uint32_t l3 = f2bf_bits(v.w - __uint_as_float(h3 << 16));
  hi = make_uint2(h0 | (h1 << 16), h2 | (h3 << 16));
  lo = make_uint2(l0 | (l1 << 16), l2 | (l3 << 16));
}

template <typename OutT> __device__ __forceinline__ OutT cvt_out(float v);
template <> __device__ __forceinline__ float cvt_out<float>(float v) { return v; }
template <> __device__ __forceinline__ bf16_t cvt_out<bf16_t>(float v) { return (bf16_t)f2bf_bits(v); }

template <int EPI>
__device__ __forceinline__ float epilogue(float x, float sc, float sh, float outscale) {
  if constexpr (EPI == EPI_COS) {
    // cos via v_cos_f32, which takes revolutions: reduce to [0, 1) first
    float rev = (x * sc + sh) * 0.15915494309189535f;
    rev = rev - floorf(rev);
    return outscale * __builtin_amdgcn_cosf(rev);
  } else if constexpr (EPI == EPI_EXPNEG) {
    return outscale * __expf(-x);
  } else {
    return outscale * x;
  }
}

template <bool AF32, bool WLO, int EPI, bool OUT_T, typename OutT>
__global__ void __launch_bounds__(NT, 2)
k_feat_gemm(const void* __restrict__ Av, int64_t M, int64_t K, int64_t lda,
            const bf16_t* __restrict__ Whi, const bf16_t* __restrict__ Wlo, int64_t Nf, int64_t ldw,
            const float* __restrict__ scales, const float* __restrict__ shifts, float outscale,
            OutT* __restrict__ out, int64_t ldo, int ntm, int ntn, int per) {
  __shared__ __attribute__((aligned(16))) bf16_t sAh[2][BM * BK];
  __shared__ __attribute__((aligned(16))) bf16_t sAl[2][AF32 ? BM * BK : 8];
  __shared__ __attribute__((aligned(16))) bf16_t sWh[2][BN * BK];
  __shared__ __attribute__((aligned(16))) bf16_t sWl[2][WLO ? BN * BK : 8];

  // XCD-aware tile order (block b runs on XCD b % 8).  When the feature tiles
  // split evenly over the 8 XCDs, XCD x owns feature tiles
  // [x * ntn/8, (x+1) * ntn/8) for every row block, so its slice of W stays
  // resident in its own L2 and only A streams (once per XCD, via the MALL).
  // The XCD's feature tiles are strided (x, x+8, ...): a contiguous slice per
  // XCD made row-major output 5x slower (measured), strided spreads the writes.
  // Otherwise XCD x takes a contiguous run of tiles with the feature tile
  // fastest, so the workgroups sharing an A row block share that L2.
  const int b = blockIdx.x, xcd = b & 7, li = b >> 3;
  int tm, tn;
  if ((ntn & 7) == 0) {
    const int nx = ntn >> 3;
    if (li >= ntm * nx) return;
    tm = li / nx;
    tn = xcd + 8 * (li - tm * nx);     // strided: an XCD's output columns spread over the row
  } else {
    const int tile = xcd * per + li;
    if (tile >= ntm * ntn) return;
    tm = tile / ntn;
    tn = tile - tm * ntn;
  }
  const int64_t row0 = (int64_t)tm * BM;
  const int64_t col0 = (int64_t)tn * BN;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;          // 2 x 2 waves, 64 x 64 each
  const int nk = (int)((K + BK - 1) / BK);

  // ---- global -> register staging (two register sets: k-steps of each parity)
  // A f32: 128 rows x 32 k = 1024 float4 chunks, 4 per thread (row = c>>3, k = (c&7)*4)
  // A bf16: 512 chunks of 8 bf16, 2 per thread (row = c>>2, k = (c&3)*8)
  // W: 128 rows x 32 k bf16 = 512 chunks per plane, 2 per thread
  constexpr int ACH = AF32 ? 4 : 2;
  struct Regs { uint4 a[ACH]; uint4 wh[2]; uint4 wl[2]; };
  Regs R0, R1;

  auto load_global = [&](Regs& R, int kt) {
    const int64_t k0 = (int64_t)kt * BK;
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int c = tid + NT * i;
      int r, kk;
      if (AF32) { r = c >> 3; kk = (c & 7) * 4; } else { r = c >> 2; kk = (c & 3) * 8; }
      const int64_t gr = row0 + r, gk = k0 + kk;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (gr < M) {
        constexpr int W = AF32 ? 4 : 8;
        if (gk + W <= K) {
          if (AF32) v = *(const uint4*)((const float*)Av + gr * lda + gk);
          else v = *(const uint4*)((const bf16_t*)Av + gr * lda + gk);
        } else if (gk < K) {
          if (AF32) {
            const float* p = (const float*)Av + gr * lda;
            float t[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) t[e] = (gk + e < K) ? p[gk + e] : 0.f;
            v = make_uint4(__float_as_uint(t[0]), __float_as_uint(t[1]), __float_as_uint(t[2]), __float_as_uint(t[3]));
          } else {
            const bf16_t* p = (const bf16_t*)Av + gr * lda;
            uint32_t t[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) t[e] = (gk + e < K) ? p[gk + e] : 0u;
            v = make_uint4(t[0] | (t[1] << 16), t[2] | (t[3] << 16), t[4] | (t[5] << 16), t[6] | (t[7] << 16));
          }
        }
      }
      R.a[i] = v;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + NT * i;
      const int r = c >> 2, kk = (c & 3) * 8;
      const int64_t off = (col0 + r) * ldw + k0 + kk;
      R.wh[i] = *(const uint4*)(Whi + off);
      if (WLO) R.wl[i] = *(const uint4*)(Wlo + off);
    }
  };

  auto store_lds = [&](const Regs& R, int s) {
#pragma unroll
    for (int i = 0; i < ACH; ++i) {
      const int c = tid + NT * i;
      if (AF32) {
        const int r = c >> 3, kk = (c & 7) * 4;
        uint2 hi, lo;
        float4 f = make_float4(__uint_as_float(R.a[i].x), __uint_as_float(R.a[i].y),
                               __uint_as_float(R.a[i].z), __uint_as_float(R.a[i].w));
        split4(f, hi, lo);
        *(uint2*)&sAh[s][r * BK + kk] = hi;
        *(uint2*)&sAl[s][r * BK + kk] = lo;
      } else {
        const int r = c >> 2, kk = (c & 3) * 8;
        *(uint4*)&sAh[s][r * BK + kk] = R.a[i];
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int c = tid + NT * i;
      const int r = c >> 2, kk = (c & 3) * 8;
      *(uint4*)&sWh[s][r * BK + kk] = R.wh[i];
      if (WLO) *(uint4*)&sWl[s][r * BK + kk] = R.wl[i];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int frag_off = (lane & 15) * BK + (lane >> 4) * 8;
  auto compute = [&](int s) {
    bf16x8 ah[4], al[4], wh[4], wl[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const int o = (wc * 64 + cb * 16) * BK + frag_off;
      wh[cb] = *(const bf16x8*)&sWh[s][o];
      if (WLO) wl[cb] = *(const bf16x8*)&sWl[s][o];
    }
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) {
      const int o = (wr * 64 + rb * 16) * BK + frag_off;
      ah[rb] = *(const bf16x8*)&sAh[s][o];
      if (AF32) al[rb] = *(const bf16x8*)&sAl[s][o];
    }
    // term-major order: 16 independent MFMAs between dependent ones
#pragma unroll
    for (int rb = 0; rb < 4; ++rb)
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
        acc[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[rb], wh[cb], acc[rb][cb], 0, 0, 0);
    if (AF32) {
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
          acc[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[rb], wh[cb], acc[rb][cb], 0, 0, 0);
    }
    if (WLO) {
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
#pragma unroll
        for (int cb = 0; cb < 4; ++cb)
          acc[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[rb], wl[cb], acc[rb][cb], 0, 0, 0);
    }
  };

  // prologue: step 0 staged in LDS, step 1 in flight in R1
  load_global(R0, 0);
  if (nk > 1) load_global(R1, 1);
  store_lds(R0, 0);
  __syncthreads();

  // steady state, unrolled by two so the register set of each parity is static:
  //   issue loads of kt+2, compute kt, land kt+1 in LDS, barrier
  int kt = 0;
  for (; kt + 1 < nk; kt += 2) {
    if (kt + 2 < nk) load_global(R0, kt + 2);
    compute(0);
    store_lds(R1, 1);
    __syncthreads();
    if (kt + 3 < nk) load_global(R1, kt + 3);
    compute(1);
    if (kt + 2 < nk) store_lds(R0, 0);
    __syncthreads();
  }
  if (kt < nk) compute(0);

  // ---- epilogue: C[row][col], col = lane & 15, row = 4 * (lane >> 4) + reg
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    const int64_t f = col0 + wc * 64 + cb * 16 + (lane & 15);
    if (f >= Nf) continue;
    const float sc = scales ? scales[f] : 1.f;
    const float sh = shifts ? shifts[f] : 0.f;
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) {
      const int64_t r = row0 + wr * 64 + rb * 16 + 4 * (lane >> 4);
      float v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = epilogue<EPI>(acc[rb][cb][e], sc, sh, outscale);
      if (OUT_T) {
        OutT* p = out + f * ldo + r;
        if (r + 3 < M) {
          if constexpr (sizeof(OutT) == 4) {
            if ((((uintptr_t)p) & 15) == 0) { *(float4*)p = make_float4(v[0], v[1], v[2], v[3]); continue; }
          }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (r + e < M) p[e] = cvt_out<OutT>(v[e]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (r + e < M) out[(r + e) * ldo + f] = cvt_out<OutT>(v[e]);
      }
    }
  }
}

template <bool AF32, bool WLO, int EPI>
int launch_out(const void* A, int64_t M, int64_t K, int64_t lda, const bf16_t* Whi, const bf16_t* Wlo,
               int64_t Nf, int64_t ldw, const float* sc, const float* sh, float outscale, void* out,
               int out_dtype, int64_t ldo, int out_t, hipStream_t s) {
  const int ntm = (int)((M + BM - 1) / BM), ntn = (int)((Nf + BN - 1) / BN);
  const int T = ntm * ntn, per = (T + 7) / 8;
  const unsigned grid = (unsigned)(8 * per);
#define SL_FG_L(OT, TRANS) \
  k_feat_gemm<AF32, WLO, EPI, TRANS, OT><<<grid, NT, 0, s>>>(A, M, K, lda, Whi, Wlo, Nf, ldw, sc, sh, outscale, (OT*)out, ldo, ntm, ntn, per)
  if (out_dtype == SL_F32) { if (out_t) SL_FG_L(float, true); else SL_FG_L(float, false); }
  else if (out_dtype == SL_BF16) { if (out_t) SL_FG_L(bf16_t, true); else SL_FG_L(bf16_t, false); }
  else return SL_ERR_UNSUPPORTED;
#undef SL_FG_L
  SL_LAUNCH_CHECK();
  return SL_OK;
}

}  // namespace

// Host contract (checked here; the Python wrapper pads W):
//   * A: M x K row-major, row stride lda elements, 16-B aligned rows
//     (lda % 4 == 0 for f32, % 8 == 0 for bf16);
//   * Whi / Wlo: ceil(Nf/128)*128 rows x ldw bf16, ldw % 32 == 0, ldw >= K,
//     zero in the padding (Wlo may be null: 2-term / 1-term products);
//   * out: f32 or bf16, Z[r*ldo + f] (out_t = 0) or Z[f*ldo + r] (out_t = 1).
SL_API int sl_feature_gemm(const void* A, int a_dtype, int64_t M, int64_t K, int64_t lda,
                           const bf16_t* Whi, const bf16_t* Wlo, int64_t Nf, int64_t ldw,
                           const float* scales, const float* shifts, float outscale, int epi,
                           void* out, int out_dtype, int64_t ldo, int out_t, void* stream) {
  if (M <= 0 || Nf <= 0) return SL_OK;
  if (K <= 0 || ldw % BK != 0 || ldw < K) return SL_ERR_DIMENSION;
  const int align = a_dtype == SL_F32 ? 4 : 8;
  if (lda % align != 0 || ((uintptr_t)A & 15) != 0 || ((uintptr_t)Whi & 15) != 0) return SL_ERR_INVALID;
  if ((M + BM - 1) / BM * ((Nf + BN - 1) / BN) > (int64_t)0x7fffffff) return SL_ERR_DIMENSION;
  if (epi == EPI_COS && shifts == nullptr) return SL_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  const bool wlo = Wlo != nullptr;
#define SL_FG_E(AF, WL)                                                                              \
  switch (epi) {                                                                                     \
    case EPI_NONE: return launch_out<AF, WL, EPI_NONE>(A, M, K, lda, Whi, Wlo, Nf, ldw, scales, shifts, outscale, out, out_dtype, ldo, out_t, s); \
    case EPI_COS: return launch_out<AF, WL, EPI_COS>(A, M, K, lda, Whi, Wlo, Nf, ldw, scales, shifts, outscale, out, out_dtype, ldo, out_t, s); \
    case EPI_EXPNEG: return launch_out<AF, WL, EPI_EXPNEG>(A, M, K, lda, Whi, Wlo, Nf, ldw, scales, shifts, outscale, out, out_dtype, ldo, out_t, s); \
    default: return SL_ERR_INVALID;                                                                  \
  }
  if (a_dtype == SL_F32) { if (wlo) { SL_FG_E(true, true) } else { SL_FG_E(true, false) } }
  else if (a_dtype == SL_BF16) { if (wlo) { SL_FG_E(false, true) } else { SL_FG_E(false, false) } }
#undef SL_FG_E
  return SL_ERR_UNSUPPORTED;
}
