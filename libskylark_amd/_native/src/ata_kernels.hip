// One-pass normal-equations product for tall f32 operators: W = A^T (A Y)
// (and optionally Y_out = A Y), A m x n row-major with n up to 6144, Y n x K
// with K in {1, 2, 4}.
//
// Reference hot loops: LSQR's A Z then A^T U (algorithms/Krylov/LSQR.hpp
// :113-248) and the Chebyshev semi-iteration's A^T R / A V pair
// (algorithms/Krylov/Chebyshev.hpp:18-85) each read A twice per iteration;
// both only need A^T A applied to a short block (the residual recurrences
// move to n-space, see algorithms/krylov.py), so one streaming read of A
// per iteration suffices -- half the HBM traffic of the Krylov phase of
// LSRN (1.25e6 x 5e3 f32 = 25 GB per GPU per read).
//
// gfx950 design: 256-thread workgroups, thread t owns the columns
// t, t + 256, ... (J per thread) and keeps its slice of Y and of the W
// accumulators in registers for the whole kernel; rows stream in blocks of
// BM = 4..16 (BM * n * 4 B >= ~64 KB in flight per workgroup; coalesced 4-B
// loads, 1 KB per wave-instruction), the BM x K dots are reduced across the
// workgroup (recursive-halving shuffles inside a wave, V - 1 shuffles for V
// values; LDS across the 4 waves), then every thread updates its W slice.  Several
// workgroups per CU hide the load latency; per-workgroup W partial slabs are
// summed by the shared slab-reduce kernel.
#include "sl_common.hpp"
#include <type_traits>

namespace {

constexpr int NT = 256;

// Sum of vals[0..V) over the 64 lanes of a wave by recursive halving: at each
// xor step a lane keeps half of its values (the lower or the upper half,
// chosen by its lane bit) and adds the partner's copy of that half, so the
// whole reduction costs V - 1 shuffles instead of 6 V.  On return vals[0] of
// lane l holds the wave total of value index l >> (6 - log2 V).
template <int CNT, int OFF, int V>
__device__ __forceinline__ void wave_rs_step(float (&vals)[V], int lane) {
  if constexpr (OFF >= 1) {
    if constexpr (CNT > 1) {
      constexpr int HALF = CNT / 2;
      const bool upper = (lane & OFF) != 0;
#pragma unroll
      for (int i = 0; i < HALF; ++i) {
        const float send = upper ? vals[i] : vals[i + HALF];
        const float keep = upper ? vals[i + HALF] : vals[i];
        vals[i] = keep + __shfl_xor(send, OFF, 64);
      }
      wave_rs_step<HALF, OFF / 2, V>(vals, lane);
    } else {
      vals[0] += __shfl_xor(vals[0], OFF, 64);
      wave_rs_step<1, OFF / 2, V>(vals, lane);
    }
  }
}

template <int V>
__device__ __forceinline__ void wave_reduce_scatter(float (&vals)[V], int lane) {
  wave_rs_step<V, 32, V>(vals, lane);
}

template <int V>
constexpr int log2c() { return V <= 1 ? 0 : 1 + log2c<V / 2>(); }

// DUAL: the W update uses a GIVEN long block D (W = A^T D) instead of A Y;
// with STORE_Y the pass still emits A Y (the BlockADMM pair {Z Wbar, Z^T d}).
// BM rows per iteration: enough bytes in flight per workgroup (BM * n * 4 >= ~64 KB).
// A element types: f32, or bf16 (a feature cache at half the bytes; the
// values are exact bf16 widened to f32, every product and sum in f32).  The
// prefetched rows stay in their storage type and widen at use: converting at
// load would make the compiler wait for the loads right there.
template <typename TA> __device__ __forceinline__ float widen(TA v);
template <> __device__ __forceinline__ float widen<float>(float v) { return v; }
template <> __device__ __forceinline__ float widen<bf16_t>(bf16_t v) { return bf16_to_f(v); }

// PAIR (bf16 with n, lda even): a thread owns adjacent column pairs
// (2 tid + 2 NT i, + 1), loaded as one 4-B word and kept packed until use --
// half the load instructions and prefetch registers of one column per lane.
// acc_y: Yout += A Y (callers summing several blocks' products).
template <typename TA, int J, int K, int BM, bool STORE_Y, bool DUAL, bool PAIR>
__global__ void __launch_bounds__(NT, 2)
k_ata_pass(const TA* __restrict__ A, int64_t m, int n, int64_t lda, const float* __restrict__ Y,
           float* __restrict__ Wslab, float* __restrict__ Yout, int64_t ldyo,
           const float* __restrict__ Dm, int64_t ldd_r, int64_t ldd_c, int acc_y) {
  static_assert(!PAIR || (sizeof(TA) == 2 && J % 2 == 0), "pairs: bf16, even J");
  auto colof = [&](int j) { return PAIR ? 2 * (threadIdx.x + NT * (j >> 1)) + (j & 1) : (int)threadIdx.x + NT * j; };
  constexpr int V = BM * K;
  static_assert(V <= 64 && (V & (V - 1)) == 0, "BM * K must be a power of two <= 64");
  constexpr int SH = 6 - log2c<V>();
  __shared__ float red[NT / 64][V];
  __shared__ __attribute__((aligned(16))) float yrow[V];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  constexpr bool NEED_DOT = !(DUAL && !STORE_Y);
  float yv[J][K], wacc[J][K];
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int c = colof(j);
#pragma unroll
    for (int kk = 0; kk < K; ++kk) {
      yv[j][kk] = (c < n && NEED_DOT) ? Y[(int64_t)c * K + kk] : 0.f;
      wacc[j][kk] = 0.f;
    }
  }
  const int64_t nblk = (m + BM - 1) / BM;
  // the next block's rows are loaded into a second register set while this
  // block's dots, cross-wave reduction and W update run (the loads of block
  // i + 1 stay in flight across block i's two barriers); only for J <= 4,
  // wider rows would spill the second set
  constexpr bool PF = J <= 4;
  // raw storage words: one element, or (PAIR) two packed bf16
  using RW = typename std::conditional<PAIR, uint32_t, TA>::type;
  constexpr int JW = PAIR ? J / 2 : J;
  RW an[PF ? BM : 1][JW];
  auto load_block = [&](int64_t blk_, RW (&dst)[BM][JW]) {
    const int64_t r0_ = blk_ * BM;
#pragma unroll
    for (int b = 0; b < BM; ++b) {
      const int64_t r = r0_ + b < m ? r0_ + b : m - 1;
      const TA* row = A + r * lda;
#pragma unroll
      for (int jw = 0; jw < JW; ++jw) {
        const int c = colof(PAIR ? 2 * jw : jw);
        if constexpr (PAIR) dst[b][jw] = (c < n && r0_ + b < m) ? *(const uint32_t*)(row + c) : 0u;
        else dst[b][jw] = (c < n && r0_ + b < m) ? row[c] : (TA)0;
      }
    }
  };
  auto widen_row = [&](const RW (&src)[JW], float (&dst)[J]) {
#pragma unroll
    for (int jw = 0; jw < JW; ++jw) {
      if constexpr (PAIR) {
        dst[2 * jw] = __uint_as_float(src[jw] << 16);
        dst[2 * jw + 1] = __uint_as_float(src[jw] & 0xffff0000u);
      } else {
        dst[jw] = widen<TA>(src[jw]);
      }
    }
  };
  if constexpr (PF)
    if ((int64_t)blockIdx.x < nblk) load_block(blockIdx.x, an);
  for (int64_t blk = blockIdx.x; blk < nblk; blk += gridDim.x) {
    const int64_t r0 = blk * BM;
    float a[BM][J];
    if constexpr (PF) {
#pragma unroll
      for (int b = 0; b < BM; ++b) widen_row(an[b], a[b]);
      if (blk + gridDim.x < nblk) load_block(blk + gridDim.x, an);
    } else {
      RW raw[BM][JW];
      load_block(blk, raw);
#pragma unroll
      for (int b = 0; b < BM; ++b) widen_row(raw[b], a[b]);
    }
    if (!NEED_DOT) {
      // W = A^T D: the D rows of this block straight from memory (tiny, cached)
      if (tid < V) {
        const int b = tid / K, kk = tid - (tid / K) * K;
        yrow[tid] = r0 + b < m ? Dm[(r0 + b) * ldd_r + kk * ldd_c] : 0.f;
      }
      __syncthreads();
    } else {
      float p[V];
#pragma unroll
      for (int b = 0; b < BM; ++b)
#pragma unroll
        for (int kk = 0; kk < K; ++kk) {
          float s = 0.f;
#pragma unroll
          for (int j = 0; j < J; ++j) s = fmaf(a[b][j], yv[j][kk], s);
          p[b * K + kk] = s;
        }
      wave_reduce_scatter<V>(p, lane);
      if ((lane & ((1 << SH) - 1)) == 0) red[wave][lane >> SH] = p[0];
      __syncthreads();
      if (tid < V) {
        float s = 0.f;
#pragma unroll
        for (int v = 0; v < NT / 64; ++v) s += red[v][tid];
        const int b = tid / K, kk = tid - (tid / K) * K;
        if (STORE_Y && r0 + b < m) {
          float* yo = Yout + (r0 + b) * ldyo + kk;
          *yo = acc_y ? *yo + s : s;
        }
        yrow[tid] = DUAL ? (r0 + b < m ? Dm[(r0 + b) * ldd_r + kk * ldd_c] : 0.f) : s;
      }
      __syncthreads();
    }
#pragma unroll
    for (int b = 0; b < BM; ++b) {
      float yr[K];
#pragma unroll
      for (int kk = 0; kk < K; ++kk) yr[kk] = yrow[b * K + kk];   // LDS broadcast
#pragma unroll
      for (int j = 0; j < J; ++j)
#pragma unroll
        for (int kk = 0; kk < K; ++kk) wacc[j][kk] = fmaf(a[b][j], yr[kk], wacc[j][kk]);
    }
    // with the dot path, the two barriers above already order this block's
    // yrow / red reads before the next block's writes; the D path needs one
    if (!NEED_DOT) __syncthreads();
  }
  float* ws = Wslab + (int64_t)blockIdx.x * n * K;
#pragma unroll
  for (int j = 0; j < J; ++j) {
    const int c = colof(j);
    if (c < n) {
#pragma unroll
      for (int kk = 0; kk < K; ++kk) ws[(int64_t)c * K + kk] = wacc[j][kk];
    }
  }
}

int ata_grid() {
  static int ncu = -1;
  if (ncu < 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      ncu = 256;
  }
  return 2 * ncu;
}

}  // namespace

int sl_slab_reduce_launch(const float* slab, int nslab, int64_t slab_stride, int ld_in, int rows, int cols,
                          float* out, int ld_out, hipStream_t s);

SL_API int64_t sl_ata_workspace(int64_t n, int k) { return (int64_t)ata_grid() * n * k * 4 + 256; }

namespace {
template <typename TA>
int ata_run(const TA* A, int64_t m, int64_t n, int64_t lda, const float* Y, int k, float* W, float* Yout,
            int64_t ldyo, const float* D, int64_t ldd_r, int64_t ldd_c, void* ws, void* stream, int acc_y = 0) {
  if (m <= 0 || n <= 0) return SL_OK;
  const int64_t Jn = (n + NT - 1) / NT;
  // register budget (no spills): J <= 8 any k, J <= 16 k <= 2, J <= 24 k == 1
  if (n > 6144 || !(k == 1 || k == 2 || k == 4) || (Jn > 8 && k == 4) || (Jn > 16 && k > 1)) {
    sl_set_last_error("ata_pass: needs n <= 6144, k in {1, 2, 4} (k <= 2 past n = 2048, k = 1 past 4096)");
    return SL_ERR_UNSUPPORTED;
  }
  hipStream_t s = (hipStream_t)stream;
  const int J = (int)((n + NT - 1) / NT);
  // rows per iteration: J = 4 -> 16, J = 8 -> 8, else 4 (>= 64 KB of A in flight per workgroup)
  const int bm = J <= 4 ? 16 : (J <= 8 ? 8 : 4);
  const int g = (int)std::min<int64_t>((int64_t)ata_grid(), (m + bm - 1) / bm);
  float* slab = (float*)ws;
  constexpr bool BF = sizeof(TA) == 2;
  const bool pair = BF && n % 2 == 0 && lda % 2 == 0 && ((uintptr_t)A & 3) == 0;
#define SL_ATA_GO(JJ, KK, SY, DU)                                                                                    \
  if (pair) k_ata_pass<TA, JJ, KK, (JJ <= 4 ? 16 : (JJ <= 8 ? 8 : 4)), SY, DU, BF><<<g, NT, 0, s>>>(A, m, (int)n, lda, Y, slab, Yout, ldyo, D, ldd_r, ldd_c, acc_y); \
  else k_ata_pass<TA, JJ, KK, (JJ <= 4 ? 16 : (JJ <= 8 ? 8 : 4)), SY, DU, false><<<g, NT, 0, s>>>(A, m, (int)n, lda, Y, slab, Yout, ldyo, D, ldd_r, ldd_c, acc_y);
#define SL_ATA(JJ, KK)                                                      \
  if (D) {                                                                  \
    if (Yout) { SL_ATA_GO(JJ, KK, true, true) } else { SL_ATA_GO(JJ, KK, false, true) } \
  } else {                                                                  \
    if (Yout) { SL_ATA_GO(JJ, KK, true, false) } else { SL_ATA_GO(JJ, KK, false, false) } \
  }
#define SL_ATA_K(JJ) \
  if (k == 1) { SL_ATA(JJ, 1) } else if (k == 2) { SL_ATA(JJ, 2) } else { SL_ATA(JJ, 4) }
  if (J <= 4) { SL_ATA_K(4) }
  else if (J <= 8) { SL_ATA_K(8) }
  else if (J <= 16) { if (k == 1) { SL_ATA(16, 1) } else { SL_ATA(16, 2) } }
  else { SL_ATA(24, 1) }
#undef SL_ATA_K
#undef SL_ATA
#undef SL_ATA_GO
  SL_LAUNCH_CHECK();
  return sl_slab_reduce_launch(slab, g, n * k, k, (int)n, k, W, k, s);
}
}  // namespace

// W (n x k, row-major) = A^T (A Y) -- or A^T D when D is non-null (D(r, c) at
// D[r * ldd_r + c * ldd_c]); Yout (m x k, ld ldyo) = A Y when non-null.
SL_API int sl_ata_pass2(const float* A, int64_t m, int64_t n, int64_t lda, const float* Y, int k, float* W,
                        float* Yout, int64_t ldyo, const float* D, int64_t ldd_r, int64_t ldd_c, void* ws,
                        void* stream) {
  return ata_run<float>(A, m, n, lda, Y, k, W, Yout, ldyo, D, ldd_r, ldd_c, ws, stream);
}

// the same with A stored as bf16 (SL_BF16) or f32 (SL_F32), selected by a_dt
// acc_y = 1: Yout += A Y (several blocks' products summed in place).
SL_API int sl_ata_pass3(const void* A, int a_dt, int64_t m, int64_t n, int64_t lda, const float* Y, int k, float* W,
                        float* Yout, int64_t ldyo, const float* D, int64_t ldd_r, int64_t ldd_c, void* ws,
                        void* stream, int acc_y) {
  if (a_dt == SL_BF16)
    return ata_run<bf16_t>((const bf16_t*)A, m, n, lda, Y, k, W, Yout, ldyo, D, ldd_r, ldd_c, ws, stream, acc_y);
  if (a_dt != SL_F32) { sl_set_last_error("ata_pass: A must be f32 or bf16"); return SL_ERR_UNSUPPORTED; }
  return ata_run<float>((const float*)A, m, n, lda, Y, k, W, Yout, ldyo, D, ldd_r, ldd_c, ws, stream, acc_y);
}

SL_API int sl_ata_pass(const float* A, int64_t m, int64_t n, int64_t lda, const float* Y, int k, float* W,
                       float* Yout, int64_t ldyo, void* ws, void* stream) {
  return sl_ata_pass2(A, m, n, lda, Y, k, W, Yout, ldyo, nullptr, 0, 0, ws, stream);
}
