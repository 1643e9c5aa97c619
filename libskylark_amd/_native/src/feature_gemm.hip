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
//   * f32 A is split once into bf16 hi + lo planes by k_split_bf16 (doing
//     it while staging cost ~5 VALU instructions per MFMA and made the kernel
//     VALU bound: A is re-read by every feature tile), and the product is the
//     3-term sum  Ah*Wh + Al*Wh + Ah*Wl  (f32-class accuracy at 3/16 of the
//     bf16 MFMA cost instead of f32 MFMA's 1/16 rate);
//   * K slices of 32 are double-buffered in LDS (64-B rows: ds_read_b128 of
//     a 16-row x 32-k fragment touches 1 KB contiguous, conflict free) and
//     the global loads run two slices ahead in two register sets;
//   * MFMAs are issued term-major (16 independent accumulators between two
//     updates of the same one);
//   * XCD-aware tile order: W is split over the 8 XCDs (each XCD's slice of W
//     stays L2 resident while A streams past), see the kernel's mapping.
#include "sl_common.hpp"
#include <stdlib.h>

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int BM = 128, BN = 128, BK = 32, NT = 256;

enum { EPI_NONE = 0, EPI_COS = 1, EPI_EXPNEG = 2, EPI_GAUSS = 3, EPI_POLY = 4 };

// Staging planes are [row][32 k] bf16 (64-B rows), so rows r and r + 4 share
// LDS banks: with plain addressing every ds_read_b128 fragment read (lane =
// 16 rows x 4 k-chunks; gfx950 services b128 reads in lane groups
// {0-3,12-15,20-27}, ... -- MI355X_MICROARCH.md) was 2-way conflicted
// (PMC: SQ_LDS_BANK_CONFLICT 1.1e9 per launch at 1e6 x 512 -> 4096).  The
// 16-B k-chunk is XOR-ed with row bit 2 (found by exhaustive search over
// GF(2) row maps): conflict-free fragment reads, and the row-contiguous b128
// stores only permute chunks within a row.
__device__ __forceinline__ int lds_swz(int row, int kk) { return kk ^ (((row >> 1) & 2) << 3); }

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

// EPI_GAUSS: kernel Gram exp(-a |x_i - y_j|^2) = exp(2a x.y - a|y|^2 - a|x|^2)
// with sc = 2a, sh = -a|y_j|^2, rt = -a|x_i|^2 (exponent clamped at 0: the
// distance can round below zero); EPI_POLY: (a x.y + c)^q with sc = a, sh = c,
// p0 = q.  (Reference kernels: ml/kernels.hpp gram().)
template <int EPI>
__device__ __forceinline__ float epilogue(float x, float sc, float sh, float outscale, float rt = 0.f,
                                          float p0 = 0.f) {
  if constexpr (EPI == EPI_GAUSS) {
    return outscale * __expf(fminf(x * sc + sh + rt, 0.f));
  } else if constexpr (EPI == EPI_POLY) {
    return outscale * powf(x * sc + sh, p0);
  } else if constexpr (EPI == EPI_COS) {
    // cos via v_cos_f32, which takes revolutions: reduce to [0, 1) first
    // v_fract_f32: one instruction for the reduction to [0, 1)
    const float rev = __builtin_amdgcn_fractf((x * sc + sh) * 0.15915494309189535f);
    return outscale * __builtin_amdgcn_cosf(rev);
  } else if constexpr (EPI == EPI_EXPNEG) {
    return outscale * __expf(-x);
  } else {
    return outscale * x;
  }
}

template <bool ALO, bool WLO, int EPI, bool OUT_T, typename OutT>
__global__ void __launch_bounds__(NT, 2)
k_feat_gemm(const bf16_t* __restrict__ Ahi, const bf16_t* __restrict__ Alo, int64_t M, int64_t K, int64_t lda,
            const bf16_t* __restrict__ Whi, const bf16_t* __restrict__ Wlo, int64_t Nf, int64_t ldw,
            const float* __restrict__ scales, const float* __restrict__ shifts, float outscale,
            OutT* __restrict__ out, int64_t ldo, int ntm, int ntn, int per,
            const float* __restrict__ rowterm, float p0) {
  // one LDS array: the K-loop staging planes, reused by the epilogue to turn
  // the MFMA C fragments (4 rows x 1 column per lane) into row-contiguous
  // 16-B stores (the store tail is issue-bound: cdna_hip_programming.md T21)
  constexpr int PLANE = 2 * BM * BK;                           // bf16 elements, 2 stages
  constexpr int STAGE_ELEMS = PLANE * (2 + (ALO ? 1 : 0) + (WLO ? 1 : 0));
  constexpr int EPI_LD = 64 + 4;                               // f32 row stride of a wave's 64 x 64 block
  constexpr int EPI_ELEMS = 4 * 64 * EPI_LD * 2;               // as bf16 elements (4 waves, f32)
  constexpr int LDS_ELEMS = (OUT_T ? STAGE_ELEMS : (STAGE_ELEMS > EPI_ELEMS ? STAGE_ELEMS : EPI_ELEMS));
  __shared__ __attribute__((aligned(16))) bf16_t lds_all[LDS_ELEMS];
  bf16_t (*sAh)[BM * BK] = (bf16_t (*)[BM * BK])(lds_all);
  bf16_t (*sWh)[BN * BK] = (bf16_t (*)[BN * BK])(lds_all + PLANE);
  bf16_t (*sAl)[BM * BK] = (bf16_t (*)[BM * BK])(lds_all + 2 * PLANE);
  bf16_t (*sWl)[BN * BK] = (bf16_t (*)[BN * BK])(lds_all + (ALO ? 3 : 2) * PLANE);

  // XCD-aware tile order (block b runs on XCD b % 8).  When the feature tiles
  // split evenly over the 8 XCDs, XCD x owns ntn/8 of them for every row block,
  // so its slice of W stays resident in its own L2 and only A streams (once
  // per XCD, via the MALL).  The XCD's feature tiles are strided (x, x+8, ...)
  // so its output columns spread over the row.  Otherwise XCD x takes a
  // contiguous run of tiles with the feature tile fastest, so the workgroups
  // sharing an A row block share that L2.
  const int b = blockIdx.x, xcd = b & 7, li = b >> 3;
  int tm, tn;
  if ((ntn & 7) == 0) {
    const int nx = ntn >> 3;
    if (li >= ntm * nx) return;
    tm = li / nx;
    tn = xcd + 8 * (li - tm * nx);
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

  // ---- global -> register staging, two register sets (k-steps of each parity).
  // Every operand tile is 128 rows x 32 k bf16 = 512 chunks of 16 B, two per
  // thread (row = c >> 2, k = (c & 3) * 8).  The planes are zero padded to a
  // multiple of 32 columns by the host and rows past M are clamped (their
  // results are never stored), so the loop has no bounds checks and each
  // chunk is one 16-B load from a pointer fixed for the whole K loop.
  const bf16_t* pa[2];
  const bf16_t* pw[2];
  int soff[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int c = tid + NT * i;
    const int r = c >> 2, kk = (c & 3) * 8;
    int64_t gr = row0 + r;
    gr = gr < M ? gr : M - 1;
    pa[i] = Ahi + gr * lda + kk;
    pw[i] = Whi + (col0 + r) * ldw + kk;
    soff[i] = r * BK + lds_swz(r, kk);
  }
  const int64_t alo_off = ALO ? (Alo - Ahi) : 0;     // planes addressed from the hi pointers
  const int64_t wlo_off = WLO ? (Wlo - Whi) : 0;
  // register staging sets as plain local arrays driven by macros: passing a
  // struct of arrays by reference into lambdas made hipcc keep them in
  // scratch memory (every prefetch went through scratch_store / load)
  // (named scalars, not arrays: hipcc's alloca promotion gave up on the
  // 2 x 8 x uint4 staging arrays and kept them in scratch)
  uint4 r0ah0, r0ah1, r0al0, r0al1, r0wh0, r0wh1, r0wl0, r0wl1;
  uint4 r1ah0, r1ah1, r1al0, r1al1, r1wh0, r1wh1, r1wl0, r1wl1;
  const bf16_t* const pa0 = pa[0];
  const bf16_t* const pa1 = pa[1];
  const bf16_t* const pw0 = pw[0];
  const bf16_t* const pw1 = pw[1];
  const int so0 = soff[0], so1 = soff[1];
#define SL_FG_LOAD(P, KT)                                                     \
  {                                                                           \
    const int k0_ = (KT) * BK;                                                \
    P##ah0 = *(const uint4*)(pa0 + k0_);                                      \
    P##ah1 = *(const uint4*)(pa1 + k0_);                                      \
    if (ALO) { P##al0 = *(const uint4*)(pa0 + alo_off + k0_);                 \
               P##al1 = *(const uint4*)(pa1 + alo_off + k0_); }               \
    P##wh0 = *(const uint4*)(pw0 + k0_);                                      \
    P##wh1 = *(const uint4*)(pw1 + k0_);                                      \
    if (WLO) { P##wl0 = *(const uint4*)(pw0 + wlo_off + k0_);                 \
               P##wl1 = *(const uint4*)(pw1 + wlo_off + k0_); }               \
  }
#define SL_FG_STORE(P, S)                                                     \
  {                                                                           \
    *(uint4*)&sAh[S][so0] = P##ah0;                                           \
    *(uint4*)&sAh[S][so1] = P##ah1;                                           \
    if (ALO) { *(uint4*)&sAl[S][so0] = P##al0; *(uint4*)&sAl[S][so1] = P##al1; } \
    *(uint4*)&sWh[S][so0] = P##wh0;                                           \
    *(uint4*)&sWh[S][so1] = P##wh1;                                           \
    if (WLO) { *(uint4*)&sWl[S][so0] = P##wl0; *(uint4*)&sWl[S][so1] = P##wl1; } \
  }

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int frag_off = (lane & 15) * BK + lds_swz(lane & 15, (lane >> 4) * 8);
  // (a macro, not a lambda: a lambda capturing acc by reference demotes it to scratch)
#define SL_FG_COMPUTE(S)                                                                      \
  {                                                                                           \
    bf16x8 ah[4], al[4], wh[4], wl[4];                                                        \
    _Pragma("unroll") for (int cb = 0; cb < 4; ++cb) {                                       \
      const int o = (wc * 64 + cb * 16) * BK + frag_off;                                      \
      wh[cb] = *(const bf16x8*)&sWh[S][o];                                                    \
      if (WLO) wl[cb] = *(const bf16x8*)&sWl[S][o];                                           \
    }                                                                                         \
    _Pragma("unroll") for (int rb = 0; rb < 4; ++rb) {                                       \
      const int o = (wr * 64 + rb * 16) * BK + frag_off;                                      \
      ah[rb] = *(const bf16x8*)&sAh[S][o];                                                    \
      if (ALO) al[rb] = *(const bf16x8*)&sAl[S][o];                                           \
    }                                                                                         \
    /* term-major order: 16 independent MFMAs between dependent ones */                      \
    _Pragma("unroll") for (int rb = 0; rb < 4; ++rb)                                         \
      _Pragma("unroll") for (int cb = 0; cb < 4; ++cb)                                       \
        acc[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[rb], wh[cb], acc[rb][cb], 0, 0, 0); \
    if (ALO) {                                                                                \
      _Pragma("unroll") for (int rb = 0; rb < 4; ++rb)                                       \
        _Pragma("unroll") for (int cb = 0; cb < 4; ++cb)                                     \
          acc[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al[rb], wh[cb], acc[rb][cb], 0, 0, 0); \
    }                                                                                         \
    if (WLO) {                                                                                \
      _Pragma("unroll") for (int rb = 0; rb < 4; ++rb)                                       \
        _Pragma("unroll") for (int cb = 0; cb < 4; ++cb)                                     \
          acc[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[rb], wl[cb], acc[rb][cb], 0, 0, 0); \
    }                                                                                         \
  }

  // prologue: step 0 staged in LDS, step 1 in flight in set r1
  SL_FG_LOAD(r0, 0)
  if (nk > 1) SL_FG_LOAD(r1, 1)
  SL_FG_STORE(r0, 0)
  __syncthreads();

  // steady state, unrolled by two so the register set of each parity is static:
  //   issue loads of kt+2, compute kt, land kt+1 in LDS, barrier
  int kt = 0;
  for (; kt + 1 < nk; kt += 2) {
    if (kt + 2 < nk) SL_FG_LOAD(r0, kt + 2)
    SL_FG_COMPUTE(0)
    SL_FG_STORE(r1, 1)
    __syncthreads();
    if (kt + 3 < nk) SL_FG_LOAD(r1, kt + 3)
    SL_FG_COMPUTE(1)
    if (kt + 2 < nk) SL_FG_STORE(r0, 0)
    __syncthreads();
  }
  if (kt < nk) SL_FG_COMPUTE(0)
#undef SL_FG_COMPUTE
#undef SL_FG_LOAD
#undef SL_FG_STORE

  // ---- epilogue: C[row][col], col = lane & 15, row = 4 * (lane >> 4) + reg
  if constexpr (!OUT_T) {
    // stage the wave's 64 x 64 block (after the epilogue map) in LDS, then
    // store whole 16-B row pieces: 16 dwordx4 (f32) per lane instead of 64 dwords
    __syncthreads();                                   // every wave is done with the staging planes
    float* blk = (float*)lds_all + wave * 64 * EPI_LD;
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const int64_t f = col0 + wc * 64 + cb * 16 + (lane & 15);
      const float sc = (scales && f < Nf) ? scales[f] : 1.f;
      const float sh = (shifts && f < Nf) ? shifts[f] : 0.f;
#pragma unroll
      for (int rb = 0; rb < 4; ++rb)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float rt = 0.f;
          if constexpr (EPI == EPI_GAUSS) {
            const int64_t r = row0 + wr * 64 + rb * 16 + 4 * (lane >> 4) + e;
            rt = (rowterm && r < M) ? rowterm[r] : 0.f;
          }
          blk[(rb * 16 + 4 * (lane >> 4) + e) * EPI_LD + cb * 16 + (lane & 15)] =
              epilogue<EPI>(acc[rb][cb][e], sc, sh, outscale, rt, p0);
        }
    }
    __syncthreads();
    const int64_t rbase = row0 + wr * 64;
    const int64_t fbase = col0 + wc * 64;
    const bool fullc = fbase + 64 <= Nf && ((ldo & 3) == 0);
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int idx = it * 64 + lane;
      const int rr = idx >> 4, c4 = (idx & 15) * 4;
      const int64_t r = rbase + rr;
      if (r >= M) continue;
      const f32x4 v = *(const f32x4*)&blk[rr * EPI_LD + c4];
      OutT* p = out + r * ldo + fbase + c4;
      if (fullc) {
        if constexpr (sizeof(OutT) == 4) {
          *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
        } else {
          *(uint2*)p = make_uint2(f2bf_bits(v[0]) | (f2bf_bits(v[1]) << 16), f2bf_bits(v[2]) | (f2bf_bits(v[3]) << 16));
        }
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (fbase + c4 + e < Nf) p[e] = cvt_out<OutT>(v[e]);
      }
    }
  } else {
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
        for (int e = 0; e < 4; ++e) {
          float rt = 0.f;
          if constexpr (EPI == EPI_GAUSS) rt = (rowterm && r + e < M) ? rowterm[r + e] : 0.f;
          v[e] = epilogue<EPI>(acc[rb][cb][e], sc, sh, outscale, rt, p0);
        }
        OutT* p = out + f * ldo + r;
        if (r + 3 < M) {
          if constexpr (sizeof(OutT) == 4) {
            if ((((uintptr_t)p) & 15) == 0) { *(float4*)p = make_float4(v[0], v[1], v[2], v[3]); continue; }
          }
        }
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (r + e < M) p[e] = cvt_out<OutT>(v[e]);
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Large-tile variant for row-major output (the feature-map / dense-sketch hot
// path): 256 x 128 output tile per 512-thread workgroup (4 x 2 waves of
// 64 x 64, the same MFMA block per wave as k_feat_gemm), one workgroup per CU.
//   * operands move HBM/L2 -> LDS by LDS-DMA (global_load_lds_dwordx4, 1 KiB
//     per wave-instruction) into a 3-stage ring, two K-slices in flight while
//     the third is consumed: no register staging, ONE s_barrier per K-slice
//     (the waves consume each other's DMA'd rows, so the barrier both
//     publishes slice kt and retires slot kt-1 for the next DMA);
//   * the LDS image uses the same k-chunk ^ row-bit-2 swizzle as lds_swz,
//     applied through the DMA's SOURCE address (the DMA writes each wave-
//     instruction's 1 KiB contiguously);
//   * 256-row A tiles halve the A traffic per feature tile against 128 x 128,
//     and the XCD map is 2 (rows) x 4 (features): XCD (i, j) owns the feature
//     tiles of quarter j (W slice L2-resident) and the row tiles of parity i,
//     so A is fetched by 4 XCDs (not 8) and W by 2.
constexpr int L_BM = 256, L_BN = 128, L_NT = 512, L_NBUF = 3;

__device__ __forceinline__ void fg_glds16(const void* gsrc, unsigned lds_base) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_base)
      : "memory");
}

template <bool ALO, bool WLO, int EPI, typename OutT>
__global__ void __launch_bounds__(L_NT, 1)
k_feat_gemm_l(const bf16_t* __restrict__ Ahi, const bf16_t* __restrict__ Alo, int64_t M, int64_t K, int64_t lda,
              const bf16_t* __restrict__ Whi, const bf16_t* __restrict__ Wlo, int64_t Nf, int64_t ldw,
              const float* __restrict__ scales, const float* __restrict__ shifts, float outscale,
              OutT* __restrict__ out, int64_t ldo, int ntm, int ntn, const float* __restrict__ rowterm, float p0) {
  constexpr int APL = L_BM * BK;                        // bf16 elements per A plane per stage
  constexpr int WPL = L_BN * BK;
  constexpr int STAGE = APL * (ALO ? 2 : 1) + WPL * (WLO ? 2 : 1);
  constexpr int EPI_LD = 64 + 4;
  constexpr int EPI_ELEMS = 8 * 64 * EPI_LD * 2;        // 8 waves' 64 x 64 f32 blocks, as bf16 elements
  constexpr int LDS_ELEMS = (L_NBUF * STAGE > EPI_ELEMS) ? L_NBUF * STAGE : EPI_ELEMS;
  extern __shared__ __attribute__((aligned(16))) bf16_t lds_l[];
  static_assert(LDS_ELEMS * 2 <= 160 * 1024, "LDS budget");

  // ---- tile of this workgroup (XCD b % 8 = (i, j): row parity i, feature quarter j)
  const int b = blockIdx.x, xcd = b & 7, li = b >> 3;
  int tm, tn;
  {
    const int nq = ntn >> 2;                 // feature tiles per quarter (host guarantees ntn % 4 == 0)
    const int xi = xcd & 1, xj = xcd >> 1;
    const int mi = li / nq, nj = li - mi * nq;
    tm = 2 * mi + xi;
    tn = xj * nq + nj;
    if (tm >= ntm) return;
  }
  const int64_t row0 = (int64_t)tm * L_BM;
  const int64_t col0 = (int64_t)tn * L_BN;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;             // 4 x 2 waves, 64 x 64 each
  const int nk = (int)((K + BK - 1) / BK);

  // ---- DMA plan: a plane of R rows x 32 k is R/16 wave-instructions of 1 KiB
  // (16 rows x 64 B); lane l fills LDS row l/4, slot l%4 of its instruction's
  // block, i.e. fetches global k-chunk (l%4) ^ swizzle(row).
  const int drow = lane >> 2;                           // row within the 16-row block
  const int dchunk = (lane & 3) ^ ((drow >> 1) & 2);    // global k-chunk for this lane's LDS slot
  // A: 16 blocks per plane over 8 waves -> 2 per wave; W: 8 blocks -> 1 per wave
  const bf16_t* pa[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int blk = wave + 8 * i;
    int64_t gr = row0 + blk * 16 + drow;
    gr = gr < M ? gr : M - 1;
    pa[i] = Ahi + gr * lda + dchunk * 8;
  }
  const bf16_t* pw = Whi + (col0 + wave * 16 + drow) * ldw + dchunk * 8;
  const int64_t alo_off = ALO ? (Alo - Ahi) : 0;
  const int64_t wlo_off = WLO ? (Wlo - Whi) : 0;
  constexpr int NDMA = 2 * (ALO ? 2 : 1) + (WLO ? 2 : 1);   // DMA instructions per wave per stage

  auto lds_addr = [&](int elem) -> unsigned {
    return __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(__attribute__((address_space(3))) void*)(lds_l + elem));
  };
  auto issue = [&](int kt) {
    const int slot = kt % L_NBUF;
    const int base = slot * STAGE;
    const int64_t k0 = (int64_t)kt * BK;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int blk = wave + 8 * i;
      fg_glds16(pa[i] + k0, lds_addr(base + blk * 16 * BK));
      if constexpr (ALO) fg_glds16(pa[i] + alo_off + k0, lds_addr(base + APL + blk * 16 * BK));
    }
    const int wb = base + APL * (ALO ? 2 : 1);
    fg_glds16(pw + k0, lds_addr(wb + wave * 16 * BK));
    if constexpr (WLO) fg_glds16(pw + wlo_off + k0, lds_addr(wb + WPL + wave * 16 * BK));
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int frag_off = (lane & 15) * BK + lds_swz(lane & 15, (lane >> 4) * 8);

  issue(0);
  if (nk > 1) issue(1);
  for (int kt = 0; kt < nk; ++kt) {
    // own DMAs of slice kt landed (slice kt+1's may still be in flight) ...
    if (kt + 1 < nk) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NDMA) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // ... and every wave's: slice kt is readable, slot (kt-1)%3 is free
    __builtin_amdgcn_s_barrier();
    if (kt + 2 < nk) issue(kt + 2);
    const int base = (kt % L_NBUF) * STAGE;
    const bf16_t* sAh = lds_l + base;
    const bf16_t* sAl = lds_l + base + APL;
    const bf16_t* sWh = lds_l + base + APL * (ALO ? 2 : 1);
    const bf16_t* sWl = sWh + WPL;
    bf16x8 ah[4], al[4], wh[4], wl[4];
#pragma unroll
    for (int cb = 0; cb < 4; ++cb) {
      const int o = (wc * 64 + cb * 16) * BK + frag_off;
      wh[cb] = *(const bf16x8*)&sWh[o];
      if (WLO) wl[cb] = *(const bf16x8*)&sWl[o];
    }
#pragma unroll
    for (int rb = 0; rb < 4; ++rb) {
      const int o = (wr * 64 + rb * 16) * BK + frag_off;
      ah[rb] = *(const bf16x8*)&sAh[o];
      if (ALO) al[rb] = *(const bf16x8*)&sAl[o];
    }
#pragma unroll
    for (int rb = 0; rb < 4; ++rb)
#pragma unroll
      for (int cb = 0; cb < 4; ++cb)
        acc[rb][cb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[rb], wh[cb], acc[rb][cb], 0, 0, 0);
    if (ALO) {
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
  }

  // ---- epilogue: stage each wave's 64 x 64 block (after the map), then
  // row-contiguous 16-B stores
  __syncthreads();
  float* blkp = (float*)lds_l + wave * 64 * EPI_LD;
#pragma unroll
  for (int cb = 0; cb < 4; ++cb) {
    const int64_t f = col0 + wc * 64 + cb * 16 + (lane & 15);
    const float sc = (scales && f < Nf) ? scales[f] : 1.f;
    const float sh = (shifts && f < Nf) ? shifts[f] : 0.f;
#pragma unroll
    for (int rb = 0; rb < 4; ++rb)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float rt = 0.f;
        if constexpr (EPI == EPI_GAUSS) {
          const int64_t r = row0 + wr * 64 + rb * 16 + 4 * (lane >> 4) + e;
          rt = (rowterm && r < M) ? rowterm[r] : 0.f;
        }
        blkp[(rb * 16 + 4 * (lane >> 4) + e) * EPI_LD + cb * 16 + (lane & 15)] =
            epilogue<EPI>(acc[rb][cb][e], sc, sh, outscale, rt, p0);
      }
  }
  __syncthreads();
  const int64_t rbase = row0 + wr * 64;
  const int64_t fbase = col0 + wc * 64;
  const bool fullc = fbase + 64 <= Nf && ((ldo & 3) == 0);
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int idx = it * 64 + lane;
    const int rr = idx >> 4, c4 = (idx & 15) * 4;
    const int64_t r = rbase + rr;
    if (r >= M) continue;
    const f32x4 v = *(const f32x4*)&blkp[rr * EPI_LD + c4];
    OutT* p = out + r * ldo + fbase + c4;
    if (fullc) {
      if constexpr (sizeof(OutT) == 4) {
        *(float4*)p = make_float4(v[0], v[1], v[2], v[3]);
      } else {
        *(uint2*)p = make_uint2(f2bf_bits(v[0]) | (f2bf_bits(v[1]) << 16), f2bf_bits(v[2]) | (f2bf_bits(v[3]) << 16));
      }
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (fbase + c4 + e < Nf) p[e] = cvt_out<OutT>(v[e]);
    }
  }
}

template <bool ALO, bool WLO, int EPI, typename OutT>
int launch_large(const bf16_t* Ahi, const bf16_t* Alo, int64_t M, int64_t K, int64_t lda, const bf16_t* Whi,
                 const bf16_t* Wlo, int64_t Nf, int64_t ldw, const float* sc, const float* sh, float outscale,
                 OutT* out, int64_t ldo, hipStream_t s, const float* rt, float p0) {
  const int ntm = (int)((M + L_BM - 1) / L_BM), ntn = (int)((Nf + L_BN - 1) / L_BN);
  constexpr int APL = L_BM * BK, WPL = L_BN * BK;
  constexpr int STAGE = APL * (ALO ? 2 : 1) + WPL * (WLO ? 2 : 1);
  constexpr int EPI_ELEMS = 8 * 64 * (64 + 4) * 2;
  constexpr size_t LDS = (size_t)((L_NBUF * STAGE > EPI_ELEMS) ? L_NBUF * STAGE : EPI_ELEMS) * 2;
  auto kern = k_feat_gemm_l<ALO, WLO, EPI, OutT>;
  SL_LDS_ATTR(kern, (int)LDS);
  const unsigned grid = (unsigned)(8 * ((ntm + 1) / 2) * (ntn / 4));
  kern<<<grid, L_NT, LDS, s>>>(Ahi, Alo, M, K, lda, Whi, Wlo, Nf, ldw, sc, sh, outscale, out, ldo, ntm, ntn, rt, p0);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

template <bool ALO, bool WLO, int EPI>
int launch_out(const bf16_t* Ahi, const bf16_t* Alo, int64_t M, int64_t K, int64_t lda, const bf16_t* Whi,
               const bf16_t* Wlo, int64_t Nf, int64_t ldw, const float* sc, const float* sh, float outscale,
               void* out, int out_dtype, int64_t ldo, int out_t, hipStream_t s, const float* rt, float p0) {
  // large tiles: row-major output, the feature tiles split into 4 XCD quarters,
  // and W padded to whole 128-row tiles (the host pads to 128)
  if (!out_t && ((Nf + L_BN - 1) / L_BN) % 4 == 0 && M >= L_BM) {
    if (out_dtype == SL_F32)
      return launch_large<ALO, WLO, EPI, float>(Ahi, Alo, M, K, lda, Whi, Wlo, Nf, ldw, sc, sh, outscale,
                                                 (float*)out, ldo, s, rt, p0);
    if (out_dtype == SL_BF16)
      return launch_large<ALO, WLO, EPI, bf16_t>(Ahi, Alo, M, K, lda, Whi, Wlo, Nf, ldw, sc, sh, outscale,
                                                  (bf16_t*)out, ldo, s, rt, p0);
  }
  const int ntm = (int)((M + BM - 1) / BM), ntn = (int)((Nf + BN - 1) / BN);
  const int T = ntm * ntn, per = (T + 7) / 8;
  const unsigned grid = (unsigned)(8 * per);
#define SL_FG_L(OT, TRANS) \
  k_feat_gemm<ALO, WLO, EPI, TRANS, OT><<<grid, NT, 0, s>>>(Ahi, Alo, M, K, lda, Whi, Wlo, Nf, ldw, sc, sh, outscale, (OT*)out, ldo, ntm, ntn, per, rt, p0)
  if (out_dtype == SL_F32) { if (out_t) SL_FG_L(float, true); else SL_FG_L(float, false); }
  else if (out_dtype == SL_BF16) { if (out_t) SL_FG_L(bf16_t, true); else SL_FG_L(bf16_t, false); }
  else return SL_ERR_UNSUPPORTED;
#undef SL_FG_L
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// f32 rows -> bf16 hi + lo planes (hi = rne(x), lo = rne(x - hi)), zero padded
// to ldp columns: one streaming pass, so the GEMM's K loop carries no
// conversion VALU work (A is re-read once per feature tile).
__global__ void __launch_bounds__(256)
k_split_bf16(const float* __restrict__ A, int64_t M, int64_t K, int64_t lda, bf16_t* __restrict__ hi,
             bf16_t* __restrict__ lo, int64_t ldp, int64_t wpad) {
  const int64_t per_row = wpad / 4;
  const int64_t total = M * per_row;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t r = t / per_row, k = (t - r * per_row) * 4;
    float x[4];
    if (k + 4 <= K && (lda & 3) == 0) {
      const float4 v = *(const float4*)(A + r * lda + k);
      x[0] = v.x; x[1] = v.y; x[2] = v.z; x[3] = v.w;
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) x[e] = (k + e < K) ? A[r * lda + k + e] : 0.f;
    }
    uint32_t h[4], l[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      h[e] = (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)x[e]);
      const float res = x[e] - __uint_as_float(h[e] << 16);
      l[e] = (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)res);
    }
    *(uint2*)(hi + r * ldp + k) = make_uint2(h[0] | (h[1] << 16), h[2] | (h[3] << 16));
    *(uint2*)(lo + r * ldp + k) = make_uint2(l[0] | (l[1] << 16), l[2] | (l[3] << 16));
  }
}

}  // namespace

// Host contract (checked here; the Python wrapper pads the planes):
//   * A: M x K as bf16 planes Ahi (+ optional Alo), row stride lda elements,
//     lda % 32 == 0, zero in columns [K, lda) (sl_split_bf16 produces them);
//   * Whi / Wlo: ceil(Nf/128)*128 rows x ldw bf16, ldw % 32 == 0, ldw >= K,
//     zero in the padding (Wlo may be null);
//   * out: f32 or bf16, Z[r*ldo + f] (out_t = 0) or Z[f*ldo + r] (out_t = 1).
SL_API int sl_feature_gemm2(const bf16_t* Ahi, const bf16_t* Alo, int64_t M, int64_t K, int64_t lda,
                            const bf16_t* Whi, const bf16_t* Wlo, int64_t Nf, int64_t ldw,
                            const float* scales, const float* shifts, float outscale, int epi,
                            void* out, int out_dtype, int64_t ldo, int out_t, const float* rowterm, float p0,
                            void* stream) {
  if (M <= 0 || Nf <= 0) return SL_OK;
  if (K <= 0 || ldw % BK != 0 || ldw < K || lda % BK != 0 || lda < K) return SL_ERR_DIMENSION;
  if (((uintptr_t)Ahi & 15) || ((uintptr_t)Whi & 15) || (Alo && ((uintptr_t)Alo & 15)) ||
      (Wlo && ((uintptr_t)Wlo & 15)))
    return SL_ERR_INVALID;
  if ((M + BM - 1) / BM * ((Nf + BN - 1) / BN) > (int64_t)0x7fffffff) return SL_ERR_DIMENSION;
  if (epi == EPI_COS && shifts == nullptr) return SL_ERR_INVALID;
  hipStream_t s = (hipStream_t)stream;
  const bool alo = Alo != nullptr, wlo = Wlo != nullptr;
#define SL_FG_C(AL, WL, E) \
  return launch_out<AL, WL, E>(Ahi, Alo, M, K, lda, Whi, Wlo, Nf, ldw, scales, shifts, outscale, out, out_dtype, ldo, out_t, s, rowterm, p0)
#define SL_FG_E(AL, WL)                                  \
  switch (epi) {                                         \
    case EPI_NONE: SL_FG_C(AL, WL, EPI_NONE);            \
    case EPI_COS: SL_FG_C(AL, WL, EPI_COS);              \
    case EPI_EXPNEG: SL_FG_C(AL, WL, EPI_EXPNEG);        \
    case EPI_GAUSS: SL_FG_C(AL, WL, EPI_GAUSS);          \
    case EPI_POLY: SL_FG_C(AL, WL, EPI_POLY);            \
    default: return SL_ERR_INVALID;                      \
  }
  if (alo) { if (wlo) { SL_FG_E(true, true) } else { SL_FG_E(true, false) } }
  else { if (wlo) { SL_FG_E(false, true) } else { SL_FG_E(false, false) } }
#undef SL_FG_E
#undef SL_FG_C
  return SL_ERR_UNSUPPORTED;
}

SL_API int sl_feature_gemm(const bf16_t* Ahi, const bf16_t* Alo, int64_t M, int64_t K, int64_t lda,
                           const bf16_t* Whi, const bf16_t* Wlo, int64_t Nf, int64_t ldw,
                           const float* scales, const float* shifts, float outscale, int epi,
                           void* out, int out_dtype, int64_t ldo, int out_t, void* stream) {
  return sl_feature_gemm2(Ahi, Alo, M, K, lda, Whi, Wlo, Nf, ldw, scales, shifts, outscale, epi, out, out_dtype, ldo,
                          out_t, nullptr, 0.f, stream);
}

// hi / lo planes of width wpad (zero padded past K) with row stride ldp >= wpad
SL_API int sl_split_bf16_2(const float* A, int64_t M, int64_t K, int64_t lda, bf16_t* hi, bf16_t* lo, int64_t wpad,
                           int64_t ldp, void* stream) {
  if (M <= 0) return SL_OK;
  if (wpad % 4 != 0 || wpad < K || ldp < wpad || ldp % 4 != 0 || ((uintptr_t)hi & 7) || ((uintptr_t)lo & 7))
    return SL_ERR_INVALID;
  const unsigned grid = sl_grid_for((size_t)(M * (wpad / 4)), 256, 8192);
  k_split_bf16<<<grid, 256, 0, (hipStream_t)stream>>>(A, M, K, lda, hi, lo, ldp, wpad);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

SL_API int sl_split_bf16(const float* A, int64_t M, int64_t K, int64_t lda, bf16_t* hi, bf16_t* lo, int64_t ldp,
                         void* stream) {
  return sl_split_bf16_2(A, M, K, lda, hi, lo, ldp, ldp, stream);
}
