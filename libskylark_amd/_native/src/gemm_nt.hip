// Large bf16 NT GEMM on MFMA for the dense-sketch / random-feature hot path
// (K1 / K6 of SURVEY §2.4): C (M x N) = epi(A (M x K) B^T), A and B both
// K-contiguous bf16 (B is the realised sketch panel or the feature frequency
// matrix: reference sketch/dense_transform_data.hpp:79-152 realises S panel
// by panel and hands it to a BLAS GEMM; sketch/RFT_Elemental.hpp:83-160 then
// applies the cosine in a separate loop -- here it is the GEMM's epilogue).
//
// gfx950 design (one 256 x 256 output tile per 512-thread workgroup, one
// workgroup per CU):
//   * 8 waves as 2 (M) x 4 (N), each a 128 x 64 block = 8 x 4 accumulators
//     of v_mfma_f32_16x16x32_bf16 (128 VGPRs of C);
//   * K slices of 64 staged global -> LDS by LDS-DMA (global_load_lds_dwordx4,
//     1 KB = 8 rows x 128 B per wave instruction), two 64 KB stages: the DMA
//     of slice t + 1 is issued right after the barrier that opens slice t and
//     has the whole of slice t's 64 MFMAs per wave to land; one counted wait
//     and one raw s_barrier per slice (no __syncthreads: its fence would
//     drain the DMA early);
//   * LDS image [row][8 x 16-B chunks] with chunk ^= (row >> 1) & 7, set by
//     the per-lane SOURCE address of the DMA: every ds_read_b128 fragment
//     read is conflict-free under gfx950's b128 lane groups
//     ({0-3,12-15,20-27}, ...: MI355X_MICROARCH.md §LDS);
//   * XCD-aware grouped tile order: the 32 tiles an XCD runs at once form a
//     4 x 8 block of (row, column) tiles, so they share 4 A and 8 B panels
//     in that XCD's L2 as the K slices advance;
//   * epilogue straight from the C fragments: alpha * acc (optionally
//     += into C), or a feature / kernel map of t = scale_f acc + shift_f
//     (+ u_d): outscale * cos(t) (random Fourier features), exp(-acc)
//     (Laplacian / exp-semigroup features), exp(min(t + u_d, 0)) (Gaussian
//     kernel Gram: t = 2a x.y - a|y|^2, u = -a|x|^2), t^p (polynomial
//     kernel); the feature index f runs along the columns (rowwise maps,
//     C = X W^T) or, FROW, along the rows (columnwise maps, C = W X^T), the
//     data index d along the other side.  f32 or bf16 out.
//     (This kernel replaced feature_gemm.hip's 128 x 128 / 256 x 128 tiles
//     for every map: the f32-exact products go in as hi / lo terms
//     concatenated along K.)
// Rows / columns past M / N are clamped on load and never stored; K must be
// a multiple of 64 (callers zero-pad).
#include "sl_common.hpp"

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

constexpr int BM = 256, BN = 256, BK = 64, NT = 512;
constexpr int OPB = BM * BK * 2;        // bytes of one operand slice (32 KB)
constexpr int STAGE = 2 * OPB;          // A + B slice (64 KB)
constexpr int GM = 4;                   // tile rows per XCD group

enum { EPI_LINEAR = 0, EPI_COS = 1, EPI_EXPNEG = 2, EPI_GAUSS = 3, EPI_POLY = 4 };

// the map of one accumulator: s / t the feature's scale / shift, u the data
// point's term, a = alpha (outscale)
template <int EPI>
__device__ __forceinline__ float epi_map(float acc, float a, float s, float t, float u, float p0) {
  if constexpr (EPI == EPI_COS) {
    // v_cos_f32 takes revolutions: reduce to [0, 1) with v_fract_f32 first
    const float rev = __builtin_amdgcn_fractf((acc * s + t) * 0.15915494309189535f);
    return a * __builtin_amdgcn_cosf(rev);
  } else if constexpr (EPI == EPI_EXPNEG) {
    return a * __expf(-acc);
  } else if constexpr (EPI == EPI_GAUSS) {
    return a * __expf(fminf(acc * s + t + u, 0.f));   // the squared distance can round below 0
  } else if constexpr (EPI == EPI_POLY) {
    return a * powf(acc * s + t, p0);
  } else {
    return a * acc;
  }
}

__device__ __forceinline__ int swz(int r) { return (r >> 1) & 7; }

__device__ __forceinline__ void glds16(const void* g, char* lds_base) {
  __builtin_amdgcn_global_load_lds(g, (__attribute__((address_space(3))) void*)lds_base, 16, 0, 0);
}

template <typename OutT> __device__ __forceinline__ OutT cvt(float v);
template <> __device__ __forceinline__ float cvt<float>(float v) { return v; }
// hardware round-to-nearest-even (v_cvt_pk_bf16_f32): the software RNE of
// f_to_bf16 cost ~6 VALU per output element in the bf16-out epilogue
__device__ __forceinline__ uint32_t hw_bf16(float v) { return (uint16_t)__builtin_bit_cast(uint16_t, (__bf16)v); }
__device__ __forceinline__ uint32_t hw_bf16x2(float lo, float hi) {
  typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
  const bf16x2_t p = __builtin_convertvector((__attribute__((ext_vector_type(2))) float){lo, hi}, bf16x2_t);
  return __builtin_bit_cast(uint32_t, p);
}
template <> __device__ __forceinline__ bf16_t cvt<bf16_t>(float v) { return (bf16_t)hw_bf16(v); }
template <typename OutT> __device__ __forceinline__ float ld_out(const OutT* p);
template <> __device__ __forceinline__ float ld_out<float>(const float* p) { return *p; }
template <> __device__ __forceinline__ float ld_out<bf16_t>(const bf16_t* p) { return bf16_to_f(*p); }

template <int EPI, typename OutT, bool ACC, bool FROW>
__global__ void __launch_bounds__(NT, 1)
k_gemm_nt(const bf16_t* __restrict__ A, int64_t lda, const bf16_t* __restrict__ B, int64_t ldb, int M, int N, int K,
          OutT* __restrict__ C, int64_t ldc, float alpha, const float* __restrict__ scales,
          const float* __restrict__ shifts, const float* __restrict__ uterm, float p0, int ntm, int ntn, int per,
          int ntst) {
  __shared__ __attribute__((aligned(1024))) char lds[2 * STAGE];

  // ---- XCD-aware grouped tile order
  const int b = blockIdx.x, xcd = b & 7, li = b >> 3;
  const int id = xcd * per + li;
  if (id >= ntm * ntn) return;
  const int gsz = GM * ntn;
  const int g = id / gsz, gi = id - g * gsz;
  const int gm0 = g * GM;
  const int gh = min(GM, ntm - gm0);
  const int tm = gm0 + gi % gh, tn = gi / gh;
  const int row0 = tm * BM, col0 = tn * BN;

  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int wm = w >> 2, wn = w & 3;

  // ---- DMA sources: instruction i of wave w fills LDS rows (4w + i) * 8 + lane / 8,
  //      chunk slot lane % 8, with the global chunk (lane % 8) ^ swz(row)
  const bf16_t* ga[4];
  const bf16_t* gb[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int r = (4 * w + i) * 8 + (lane >> 3);
    const int c = (lane & 7) ^ swz(r);
    const int ar = min(row0 + r, M - 1), br = min(col0 + r, N - 1);
    ga[i] = A + (int64_t)ar * lda + c * 8;
    gb[i] = B + (int64_t)br * ldb + c * 8;
  }
  auto issue = [&](int kt, int st) {
    char* base = lds + st * STAGE + w * 4 * 1024;
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < 4; ++i) glds16(ga[i] + k0, base + i * 1024);
#pragma unroll
    for (int i = 0; i < 4; ++i) glds16(gb[i] + k0, base + OPB + i * 1024);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // fragment read offsets (bytes within an operand slice) for k-half kh:
  // row = base + (lane & 15), chunk = 4 kh + (lane >> 4)
  const int fr = lane & 15, fq = lane >> 4;
  const int nk = K / BK;
  auto read_frags = [&](int st, int kh, bf16x8 (&a)[8], bf16x8 (&bb)[4]) {
    const char* sA = lds + st * STAGE;
    const char* sB = sA + OPB;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = wm * 128 + i * 16 + fr;
      a[i] = *(const bf16x8*)(sA + r * 128 + (((4 * kh + fq) ^ swz(r)) << 4));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = wn * 64 + j * 16 + fr;
      bb[j] = *(const bf16x8*)(sB + r * 128 + (((4 * kh + fq) ^ swz(r)) << 4));
    }
  };
  auto mfmas = [&](const bf16x8 (&a)[8], const bf16x8 (&bb)[4]) {
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[i], bb[j], acc[i][j], 0, 0, 0);
  };
  // Per slice kt: the second K-half's fragments are read BEFORE the slice's
  // closing barrier but their 32 MFMAs run AFTER it, under the first
  // ds_reads of slice kt + 1, and the MFMA stretch runs at raised wave
  // priority.  The barrier still closes every read of stage kt & 1
  // (lgkmcnt(0) before it), which is all the DMA into that stage needs.
  // Same-box A/B (profiles/r4/gemm_nt_prio_ab.jsonl): 1160 / 1138 TF square
  // 8192^3 / LSRN panel against 1143 / 1119 for the plain loop; the deferral
  // alone (no priority) measured 1013 / 1115.  A ring of four K-half slots
  // (each half's DMA three phases ahead, one counted wait + barrier per K
  // half) lost: 938 / 1052 vs 1159 / 1158 TF (profiles/r5/gemm_nt_ring_ab.jsonl).
  // A persistent short-K form (next tile's slice 0 in flight during the
  // epilogue, +- a start stagger) measured no gain at K = 512 and lost at
  // K = 1024 (profiles/r5/gemm_nt_pers_ab.jsonl).
  bf16x8 a0[8], b0[4], a1[8], b1[4];
  issue(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_sched_barrier(0);
  for (int kt = 0; kt < nk; ++kt) {
    const int st = kt & 1;
    if (kt + 1 < nk) issue(kt + 1, st ^ 1);
    read_frags(st, 0, a0, b0);
    __builtin_amdgcn_s_setprio(1);
    if (kt > 0) mfmas(a1, b1);            // slice kt - 1, second half
    read_frags(st, 1, a1, b1);
    mfmas(a0, b0);
    __builtin_amdgcn_s_setprio(0);
    // slice kt + 1 landed (this wave's DMA), everyone done reading stage st
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  }
  if (nk > 0) mfmas(a1, b1);

  // ---- epilogue: lane holds C[4 fq + e][fr] of each 16 x 16 block.  The
  //      wave's 128 x 64 block goes out in four 32-row passes through a
  //      wave-private LDS patch (row stride 68 floats: the four fq row groups
  //      of one write land 16 banks apart), re-read as row-contiguous float4
  //      so every store instruction writes 4 rows x 256 B (f32) / 128 B (bf16).
  constexpr int EP_LD = 68;
  float* ep = (float*)lds + w * (32 * EP_LD);
  // per-column terms: the feature's scale / shift (rowwise maps) or the data
  // point's term (FROW)
  float csc[4], csh[4], cu[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = min(col0 + wn * 64 + j * 16 + fr, N - 1);
    csc[j] = 1.f;
    csh[j] = 0.f;
    cu[j] = 0.f;
    if constexpr (EPI != EPI_LINEAR) {
      if constexpr (FROW) {
        cu[j] = uterm ? uterm[col] : 0.f;
      } else {
        csc[j] = scales ? scales[col] : 1.f;
        csh[j] = shifts ? shifts[col] : 0.f;
      }
    }
  }
  const int rr = lane >> 4, cq = (lane & 15) * 4;     // read-back: row rr + 4 u, columns cq .. cq + 3
  const int gcol = col0 + wn * 64 + cq;
  const bool c_al = ((uintptr_t)C & 15) == 0 && (ldc & 3) == 0;   // every f32 row 16-B aligned
#pragma unroll
  for (int pss = 0; pss < 4; ++pss) {
#pragma unroll
    for (int ii = 0; ii < 2; ++ii) {
      const int i = 2 * pss + ii;
      // per-row terms of this fragment row group: the data point's term
      // (rowwise maps) or the feature's scale / shift (FROW)
      float rs[4], rt[4], ru[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int r = min(row0 + wm * 128 + i * 16 + 4 * fq + e, M - 1);
        rs[e] = 1.f;
        rt[e] = 0.f;
        ru[e] = 0.f;
        if constexpr (EPI != EPI_LINEAR) {
          if constexpr (FROW) {
            rs[e] = scales ? scales[r] : 1.f;
            rt[e] = shifts ? shifts[r] : 0.f;
          } else if constexpr (EPI == EPI_GAUSS) {
            ru[e] = uterm ? uterm[r] : 0.f;
          }
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float v = FROW ? epi_map<EPI>(acc[i][j][e], alpha, rs[e], rt[e], cu[j], p0)
                               : epi_map<EPI>(acc[i][j][e], alpha, csc[j], csh[j], ru[e], p0);
          ep[(ii * 16 + 4 * fq + e) * EP_LD + j * 16 + fr] = v;
        }
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // accumulate (f32 out, 16-B aligned rows): this pass's eight C reads issued
    // together from clamped addresses and pinned -- read inside the row /
    // column branches they compiled to one load-and-wait at a time
    f32x4 cpre[8];
    if constexpr (ACC && sizeof(OutT) == 4) {
      if (c_al) {
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int row = row0 + wm * 128 + pss * 32 + rr + 4 * u;
          cpre[u] = *(const f32x4*)((const float*)C + (int64_t)(row < M ? row : M - 1) * ldc + (gcol + 3 < N ? gcol : 0));
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) asm volatile("" : "+v"(cpre[u]));
      }
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int lr = rr + 4 * u;
      const int row = row0 + wm * 128 + pss * 32 + lr;
      const float4 v = *(const float4*)(ep + lr * EP_LD + cq);
      if (row < M) {
        OutT* p = C + (int64_t)row * ldc + gcol;
        if (gcol + 3 < N && (((uintptr_t)p) & (4 * sizeof(OutT) - 1)) == 0) {
          if constexpr (sizeof(OutT) == 4) {
            float4 o = v;
            if (ACC) {
              const f32x4 c = c_al ? cpre[u] : *(const f32x4*)p;
              o.x += c[0]; o.y += c[1]; o.z += c[2]; o.w += c[3];
            }
            if (ntst) __builtin_nontemporal_store(f32x4{o.x, o.y, o.z, o.w}, (f32x4*)p);
            else *(float4*)p = o;
          } else {
            float o[4] = {v.x, v.y, v.z, v.w};
            if (ACC) {
              const uint2 c = *(const uint2*)p;
              o[0] += bf16_to_f((bf16_t)(c.x & 0xffff)); o[1] += bf16_to_f((bf16_t)(c.x >> 16));
              o[2] += bf16_to_f((bf16_t)(c.y & 0xffff)); o[3] += bf16_to_f((bf16_t)(c.y >> 16));
            }
            const uint2 q = make_uint2(hw_bf16x2(o[0], o[1]), hw_bf16x2(o[2], o[3]));
            typedef __attribute__((ext_vector_type(2))) unsigned u32x2;
            if (ntst) __builtin_nontemporal_store(u32x2{q.x, q.y}, (u32x2*)p);
            else *(uint2*)p = q;
          }
        } else {
          const float o[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (gcol + q < N) {
              float x = o[q];
              if (ACC) x += ld_out<OutT>(p + q);
              p[q] = cvt<OutT>(x);
            }
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
}



// C written with non-temporal stores when it is large (>= 64 MiB) and K is
// short (<= 2048: the C write is then a large share of the traffic and would
// only evict the A / B panels the K loop re-reads from L2; 1e6 x 4096 x 512
// with the cos map: bf16 out 5.50 -> 5.03 ms, f32 out 5.99 -> 5.73 ms,
// profiles/r5/gemm_nt_epilogue_v2.jsonl).  A/B knob: -1 auto, 0 off, 1 on.
int g_nt_store = -1;

template <int EPI, typename OutT, bool ACC, bool FROW = false>
int launch(const void* A, int64_t lda, const void* B, int64_t ldb, int M, int N, int K, void* C, int64_t ldc,
           float alpha, const float* scales, const float* shifts, hipStream_t s, const float* uterm = nullptr,
           float p0 = 0.f) {
  const int ntm = (M + BM - 1) / BM, ntn = (N + BN - 1) / BN;
  const int tiles = ntm * ntn;
  const int per = (tiles + 7) / 8;
  const int nt = g_nt_store >= 0 ? g_nt_store
                                 : ((double)M * N * sizeof(OutT) >= 64.0 * (1 << 20) && K <= 2048 ? 1 : 0);
  k_gemm_nt<EPI, OutT, ACC, FROW><<<(unsigned)(per * 8), NT, 0, s>>>((const bf16_t*)A, lda, (const bf16_t*)B, ldb, M,
                                                                      N, K, (OutT*)C, ldc, alpha, scales, shifts,
                                                                      uterm, p0, ntm, ntn, per, nt);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// f32 rows -> bf16 hi + lo planes (hi = rne(x), lo = rne(x - hi)), zero padded
// to wpad columns, row stride ldp: one streaming pass, so the GEMM's K loop
// carries no conversion work (the X operand is re-read by every feature tile)
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

// Transposing bf16 hi / lo split of an f32 panel: X (w x m, ldx) ->
// Ht, Lt (m x wpad, ldt; Ht + Lt = X^T to ~2^-17, zero for k >= w), the
// K-contiguous B operand of a columnwise sketch panel product S_panel X.
// 64 (k) x 64 (column) tiles through LDS: coalesced row reads of X, one
// 128-B bf16 row piece per output row and plane.
// the 64 x 64 f32 tile X[k0 .., c0 ..] (zero outside w x m) into LDS: all 16
// loads of a thread issued unconditionally from clamped addresses, then
// zeroed (a `cond ? X[..] : 0` load compiled to one exec-masked branch per
// load, each waiting for its own)
__device__ __forceinline__ void load_tile_t(const float* __restrict__ X, int w, int m, int64_t ldx, int c0, int k0,
                                            float (&tile)[64][65]) {
  const int t = threadIdx.x;
  if (w > 0) {
    float v[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int e = t + 256 * i, k = k0 + (e >> 6), c = c0 + (e & 63);
      v[i] = X[(int64_t)(k < w ? k : w - 1) * ldx + (c < m ? c : m - 1)];
    }
#pragma unroll
    for (int i = 0; i < 16; ++i) asm volatile("" : "+v"(v[i]));
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int e = t + 256 * i, kk = e >> 6, cc = e & 63;
      tile[kk][cc] = (k0 + kk < w && c0 + cc < m) ? v[i] : 0.f;
    }
  } else {
    for (int e = t; e < 64 * 64; e += 256) tile[e >> 6][e & 63] = 0.f;
  }
  __syncthreads();
}

// bf16 pair (x0, x1) -> the packed hardware RNE word and the two rounded values
__device__ __forceinline__ uint32_t rne_pair(float x0, float x1, float* r0, float* r1) {
  const uint32_t p = hw_bf16x2(x0, x1);
  *r0 = bf16_to_f((bf16_t)(p & 0xffffu));
  *r1 = bf16_to_f((bf16_t)(p >> 16));
  return p;
}

__global__ void __launch_bounds__(256)
k_split_t(const float* __restrict__ X, int w, int m, int64_t ldx, bf16_t* __restrict__ Ht, bf16_t* __restrict__ Lt,
          int wpad, int64_t ldt) {
  __shared__ float tile[64][65];
  const int c0 = blockIdx.x * 64, k0 = blockIdx.y * 64;
  load_tile_t(X, w, m, ldx, c0, k0, tile);
  const int t = threadIdx.x;
  const int cc = t >> 2, q = t & 3;
  const int c = c0 + cc;
  if (c >= m || k0 + 16 * q >= wpad) return;
  // hi = rne(x), lo = rne(x - hi), two elements per hardware conversion
  uint32_t h[8], l[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const float x0 = tile[16 * q + 2 * u][cc], x1 = tile[16 * q + 2 * u + 1][cc];
    float h0, h1, d0, d1;
    h[u] = rne_pair(x0, x1, &h0, &h1);
    l[u] = rne_pair(x0 - h0, x1 - h1, &d0, &d1);
  }
  uint4* ph = (uint4*)(Ht + (int64_t)c * ldt + k0 + 16 * q);
  uint4* pl = (uint4*)(Lt + (int64_t)c * ldt + k0 + 16 * q);
  ph[0] = make_uint4(h[0], h[1], h[2], h[3]);
  ph[1] = make_uint4(h[4], h[5], h[6], h[7]);
  pl[0] = make_uint4(l[0], l[1], l[2], l[3]);
  pl[1] = make_uint4(l[4], l[5], l[6], l[7]);
}

// Exact three-plane split of an f32 panel, transposed, into the stacked
// layout of the split Gram (ml/krr.py _gram_split): X (w x m, ldx) -> S (m x
// 5 seg, row stride lds) with segments [L | H | M | H | L] of width seg
// (H = rne(x), M = rne(x - H), L = rne(x - H - M): H + M + L == x for normal
// f32), zero for k >= w.  Then [H M] [H M]^T + [H M H L] [L H M H]^T = X^T X
// up to the M L / L L terms, both products NT on windows of S.
__global__ void __launch_bounds__(256)
k_split3_t(const float* __restrict__ X, int w, int m, int64_t ldx, bf16_t* __restrict__ S, int seg, int64_t lds) {
  __shared__ float tile[64][65];
  const int c0 = blockIdx.x * 64, k0 = blockIdx.y * 64;
  load_tile_t(X, w, m, ldx, c0, k0, tile);
  const int t = threadIdx.x;
  const int cc = t >> 2, q = t & 3;
  const int c = c0 + cc;
  if (c >= m || k0 + 16 * q >= seg) return;
  uint32_t h[8], md[8], l[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    const float x0 = tile[16 * q + 2 * u][cc], x1 = tile[16 * q + 2 * u + 1][cc];
    float h0, h1, m0, m1, d0, d1;
    h[u] = rne_pair(x0, x1, &h0, &h1);
    const float r0 = x0 - h0, r1 = x1 - h1;
    md[u] = rne_pair(r0, r1, &m0, &m1);
    l[u] = rne_pair(r0 - m0, r1 - m1, &d0, &d1);
  }
  bf16_t* row = S + (int64_t)c * lds + k0 + 16 * q;
  auto put = [&](int sg, const uint32_t* v) {
    uint4* p = (uint4*)(row + (int64_t)sg * seg);
    p[0] = make_uint4(v[0], v[1], v[2], v[3]);
    p[1] = make_uint4(v[4], v[5], v[6], v[7]);
  };
  put(0, l);
  put(1, h);
  put(2, md);
  put(3, h);
  put(4, l);
}

}  // namespace

// S (m x 5 seg bf16, row stride lds; seg % 64 == 0, 16-B aligned rows) =
// [L | H | M | H | L] of the f32 panel X (w x m, ldx) transposed: see k_split3_t.
SL_API int sl_split3_bf16_t(const float* X, int w, int m, int64_t ldx, void* S, int seg, int64_t lds, void* stream) {
  if (w < 0 || m <= 0 || seg % 64 || seg < w || lds < 5 * (int64_t)seg || lds % 8) {
    sl_set_last_error("split3_bf16_t: needs seg % 64 == 0, seg >= w, lds >= 5 seg, lds % 8 == 0");
    return SL_ERR_INVALID;
  }
  dim3 grid((unsigned)((m + 63) / 64), (unsigned)(seg / 64));
  k_split3_t<<<grid, 256, 0, (hipStream_t)stream>>>(X, w, m, ldx, (bf16_t*)S, seg, lds);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// C (M x N, ldc) = alpha A B^T (+ C when accumulate) with A M x K, B N x K
// bf16 row-major (lda, ldb elements, 16-B aligned rows), K % 64 == 0.
// epi 1: C = alpha * cos(scales[n] * (A B^T) + shifts[n]).  out: SL_F32 / SL_BF16.
// A/B knob: non-temporal C stores, -1 auto (large C), 0 off, 1 on
SL_API void sl_gemm_nt_set_nt_store(int v) { g_nt_store = v < 0 ? -1 : (v ? 1 : 0); }

SL_API int sl_gemm_nt_bf16(const void* A, int64_t lda, const void* B, int64_t ldb, int M, int N, int K, void* C,
                           int64_t ldc, int out_dtype, int accumulate, int epi, float alpha, const float* scales,
                           const float* shifts, void* stream) {
  if (M <= 0 || N <= 0) return SL_OK;
  if (K <= 0 || K % BK || lda % 8 || ldb % 8 || lda < K || ldb < K || ldc < N) {
    sl_set_last_error("gemm_nt_bf16: needs K % 64 == 0, lda / ldb multiples of 8 and >= K, ldc >= N");
    return SL_ERR_INVALID;
  }
  if ((epi == EPI_COS && accumulate) || (epi != EPI_LINEAR && epi != EPI_COS)) {
    sl_set_last_error("gemm_nt_bf16: epilogue 0 (linear, optional accumulate) or 1 (cos)");
    return SL_ERR_INVALID;
  }
  hipStream_t s = (hipStream_t)stream;
  if (out_dtype == SL_F32) {
    if (epi == EPI_COS) return launch<EPI_COS, float, false>(A, lda, B, ldb, M, N, K, C, ldc, alpha, scales, shifts, s);
    if (accumulate) return launch<EPI_LINEAR, float, true>(A, lda, B, ldb, M, N, K, C, ldc, alpha, nullptr, nullptr, s);
    return launch<EPI_LINEAR, float, false>(A, lda, B, ldb, M, N, K, C, ldc, alpha, nullptr, nullptr, s);
  }
  if (out_dtype == SL_BF16) {
    if (epi == EPI_COS) return launch<EPI_COS, bf16_t, false>(A, lda, B, ldb, M, N, K, C, ldc, alpha, scales, shifts, s);
    if (accumulate) return launch<EPI_LINEAR, bf16_t, true>(A, lda, B, ldb, M, N, K, C, ldc, alpha, nullptr, nullptr, s);
    return launch<EPI_LINEAR, bf16_t, false>(A, lda, B, ldb, M, N, K, C, ldc, alpha, nullptr, nullptr, s);
  }
  sl_set_last_error("gemm_nt_bf16: f32 / bf16 output");
  return SL_ERR_UNSUPPORTED;
}

// C (M x N, ldc) = map(A B^T) (see epi_map): epi 0 linear (alpha A B^T), 1
// cos, 2 exp(-x), 3 Gaussian-kernel exp, 4 polynomial; scales / shifts per
// feature, uterm per data point, frow = features along C's rows.
SL_API int sl_gemm_nt_map(const void* A, int64_t lda, const void* B, int64_t ldb, int M, int N, int K, void* C,
                          int64_t ldc, int out_dtype, int epi, int frow, float alpha, const float* scales,
                          const float* shifts, const float* uterm, float p0, void* stream) {
  if (M <= 0 || N <= 0) return SL_OK;
  if (K <= 0 || K % BK || lda % 8 || ldb % 8 || lda < K || ldb < K || ldc < N) {
    sl_set_last_error("gemm_nt_map: needs K % 64 == 0, lda / ldb multiples of 8 and >= K, ldc >= N");
    return SL_ERR_INVALID;
  }
  if (epi < EPI_LINEAR || epi > EPI_POLY || (out_dtype != SL_F32 && out_dtype != SL_BF16)) {
    sl_set_last_error("gemm_nt_map: epilogue 0..4, f32 / bf16 output");
    return SL_ERR_INVALID;
  }
  hipStream_t s = (hipStream_t)stream;
#define SL_GM(E, T, FR) \
  return launch<E, T, false, FR>(A, lda, B, ldb, M, N, K, C, ldc, alpha, scales, shifts, s, uterm, p0)
#define SL_GM_T(E, FR)                                    \
  if (out_dtype == SL_F32) { SL_GM(E, float, FR); }       \
  else { SL_GM(E, bf16_t, FR); }
#define SL_GM_E(FR)                                       \
  switch (epi) {                                          \
    case EPI_LINEAR: SL_GM_T(EPI_LINEAR, FR)              \
    case EPI_COS: SL_GM_T(EPI_COS, FR)                    \
    case EPI_EXPNEG: SL_GM_T(EPI_EXPNEG, FR)              \
    case EPI_GAUSS: SL_GM_T(EPI_GAUSS, FR)                \
    default: SL_GM_T(EPI_POLY, FR)                        \
  }
  if (frow) { SL_GM_E(true) }
  else { SL_GM_E(false) }
#undef SL_GM_E
#undef SL_GM_T
#undef SL_GM
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

// Ht / Lt (m x wpad bf16, row stride ldt, wpad % 64 == 0, 16-B aligned rows)
// from the f32 panel X (w x m, ldx): see k_split_t.
SL_API int sl_split_bf16_t(const float* X, int w, int m, int64_t ldx, void* Ht, void* Lt, int wpad, int64_t ldt,
                           void* stream) {
  if (w < 0 || m <= 0 || wpad % 64 || wpad < w || ldt < wpad || ldt % 8) {
    sl_set_last_error("split_bf16_t: needs wpad % 64 == 0, wpad >= w, ldt >= wpad, ldt % 8 == 0");
    return SL_ERR_INVALID;
  }
  dim3 grid((unsigned)((m + 63) / 64), (unsigned)(wpad / 64));
  k_split_t<<<grid, 256, 0, (hipStream_t)stream>>>(X, w, m, ldx, (bf16_t*)Ht, (bf16_t*)Lt, wpad, ldt);
  SL_LAUNCH_CHECK();
  return SL_OK;
}
