// Software-pipelined fused tall-skinny pass (v2 of sl_tsk_fused_pass).
//
// Same contract as k_tsk_pass (tsk_kernels.hip): ONE read of a bf16 row
// shard A (m x n) gives W = A^T (A Z), optionally G = Y^T Y and Y = A Z.
// Reference hot loop: the two El::Gemm calls + QR Gram per power iteration
// (nla/svd.hpp:71-149).
//
// What changes against v1 (whose per-block chain was serial: wait -> y
// partials -> barrier -> reduce -> barrier -> prefetch -> W update):
//   * the LDS ring regions are private to each wave (a wave DMAs only its
//     own columns), so the next prefetch is issued at the TOP of the
//     iteration, before the wait: the in-flight depth stays at PD blocks
//     all the time instead of dipping while the chain runs;
//   * two-stage software pipeline: iteration b does step 1 (y partials) of
//     block b and steps 3/4 (W += A^T y, Gram, Y store) of block b-1, so the
//     two MFMA streams are independent and hide each other's LDS latency;
//   * every wave sums the 8 partials of y itself (redundant, 24 KB of LDS
//     reads per wave per block) instead of a reducer wave + second barrier:
//     with double-buffered partials (YPB = 2) one s_barrier per block;
//   * the A fragments of block b (step-1 rows and the transposed step-3
//     reads) are taken into registers in iteration b, so the ring slot is
//     free again at the top of iteration b+1 (ring depth = PD + 1);
//   * partials laid out [wave][lane-group g][col][4 rows]: each 16-lane
//     ds_read_b128 group touches 16 distinct 16-B bank groups (no conflicts);
//   * Y stores are unconditional per instruction (rows past m go to a dump
//     slot in the workspace), so the per-wave vmcnt bookkeeping is exact and
//     the final pass keeps its full prefetch depth.
#include "sl_common.hpp"
#include <stdlib.h>

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) double f64x4;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int WAVES = 8;
constexpr int THREADS = WAVES * 64;
constexpr int BM = 16;

__device__ __forceinline__ short bf16_bits(float f) { return __builtin_bit_cast(short, (__bf16)f); }
__device__ __forceinline__ float bf16_val(short h) { return (float)__builtin_bit_cast(__bf16, h); }

__device__ __forceinline__ void glds16(const void* gsrc, unsigned lds_base) {
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

__device__ __forceinline__ void glds16_nt(const void* gsrc, unsigned lds_base) {
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off nt\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(lds_base)
      : "memory");
}

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (clamped: a smaller count
// only waits longer, never too little)
#define SL_VMW(N) case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
__device__ __forceinline__ void wait_vm(int n) {
  switch (n < 24 ? n : 24) {
    SL_VMW(0) SL_VMW(1) SL_VMW(2) SL_VMW(3) SL_VMW(4) SL_VMW(5) SL_VMW(6) SL_VMW(7) SL_VMW(8)
    SL_VMW(9) SL_VMW(10) SL_VMW(11) SL_VMW(12) SL_VMW(13) SL_VMW(14) SL_VMW(15) SL_VMW(16)
    SL_VMW(17) SL_VMW(18) SL_VMW(19) SL_VMW(20) SL_VMW(21) SL_VMW(22) SL_VMW(23)
    default: asm volatile("s_waitcnt vmcnt(24)" ::: "memory"); break;
  }
}
#undef SL_VMW

template <int NW, int KT, int NBUF, int YPB>
struct Geo2 {
  static constexpr int ROWB = NW * 2;        // bytes per LDS row of a wave region
  static constexpr int NCH = NW / 8;         // 16-B chunks per row
  static constexpr int REGION = BM * ROWB;   // bytes per wave per ring slot
  static constexpr int LPB = REGION / 1024;  // LDS-DMA instructions per block per wave
  static constexpr int KP = KT * 16;
  static constexpr int ABYTES = NBUF * WAVES * REGION;
  static constexpr int YPW = 4 * KP * 4;     // floats of one wave's partial ([g][col][4])
  static constexpr int YP_BYTES = YPB * WAVES * YPW * 4;
  static constexpr int LDS = ABYTES + YP_BYTES;
  static constexpr int GTILES = KT * KT;
  static constexpr int GS = (GTILES + WAVES - 1) / WAVES;
  static constexpr int GT64 = KT * (KT + 1) / 2;
  static constexpr int GS64 = (GT64 + WAVES - 1) / WAVES;
  static constexpr int NSTORE = 4 * KT;      // Y store instructions per block (all waves)
};

template <int NW, int KT, bool DO_G, bool STORE_Y, bool HI_T, bool G64, int NBUF, int YPB, bool ST = false>
__global__ void __launch_bounds__(THREADS, 1)
k_tsk_pass2(const bf16_t* __restrict__ A, int64_t m, int n, int64_t lda,
            const bf16_t* __restrict__ Zt, int k,
            float* __restrict__ Wslab, float* __restrict__ Gslab,
            float* __restrict__ Y, int64_t ldy, float* __restrict__ ydump, int ab,
            unsigned long long* __restrict__ dbg) {
  using GG = Geo2<NW, KT, NBUF, YPB>;
  // diagnostic build only (ST): per-phase s_memtime sums, written to dbg
  unsigned long long st_acc[6] = {0, 0, 0, 0, 0, 0}, st_prev = 0;
#define SL_STAMP(I)                                                      \
  if constexpr (ST) {                                                    \
    const unsigned long long t_ = __builtin_amdgcn_s_memtime();          \
    if ((I) > 0 && my > 1) st_acc[(I) - 1] += t_ - st_prev;              \
    st_prev = t_;                                                        \
  }
  constexpr int PD = NBUF - 1;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* abuf = smem;
  float* yp = (float*)(smem + GG::ABYTES);

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g4 = lane >> 4, i16 = lane & 15;
  const int c0w = w * NW;
  const int64_t nblocks = (m + BM - 1) / BM;
  const int64_t b0 = blockIdx.x;
  const int64_t bstep = gridDim.x;
  const int64_t nloc = b0 < nblocks ? (nblocks - 1 - b0) / bstep + 1 : 0;
  // Y store instructions of this wave per block: pairs p = 4t + j with p % 8 == w
  const int sy = STORE_Y ? (GG::NSTORE - w + WAVES - 1) / WAVES : 0;

  // ---- Z fragments (B operand of step 1)
  bf16x8 zh[NW / 32][KT];
#pragma unroll
  for (int ks = 0; ks < NW / 32; ++ks)
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      const int col = 16 * t + i16;
      const int kk = c0w + 32 * ks + 8 * g4;
      bf16x8 v = {};
      if (col < k && kk + 8 <= n) v = *(const bf16x8*)(Zt + (int64_t)col * n + kk);
      zh[ks][t] = v;
    }
#pragma unroll
  for (int ks = 0; ks < NW / 32; ++ks)
#pragma unroll
    for (int t = 0; t < KT; ++t) asm volatile("" ::"v"(zh[ks][t]));

  f32x4 accW[NW / 16][KT];
#pragma unroll
  for (int a = 0; a < NW / 16; ++a)
#pragma unroll
    for (int t = 0; t < KT; ++t) accW[a][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 accG[G64 ? 1 : GG::GS];
  f64x4 accG64[G64 ? GG::GS64 : 1];
#pragma unroll
  for (int s = 0; s < (G64 ? 1 : GG::GS); ++s) accG[s] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < (G64 ? GG::GS64 : 1); ++s) accG64[s] = f64x4{0.0, 0.0, 0.0, 0.0};

  auto issue = [&](int64_t blk, int buf) {
    char* region = abuf + (buf * WAVES + w) * GG::REGION;
    const int64_t r0 = blk * BM;
#pragma unroll
    for (int i = 0; i < GG::LPB; ++i) {
      const int byte = i * 1024 + lane * 16;
      const int row = byte / GG::ROWB;
      const int slot = (byte % GG::ROWB) / 16;
      const int chunk = slot ^ (row & (GG::NCH - 1));
      int64_t grow = r0 + row;
      grow = grow < m ? grow : m - 1;
      int col = c0w + chunk * 8;
      col = col + 8 <= n ? col : n - 8;
      const bf16_t* src = A + grow * lda + col;
      const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_void*)(region + i * 1024));
      if (ab & 64) glds16_nt((const void*)src, dst);
      else glds16((const void*)src, dst);
    }
  };

#pragma unroll
  for (int p = 0; p < PD; ++p)
    if (p < nloc) issue(b0 + p * bstep, p);

  // tr fragments (step-3 A^T operand) of the previous block, held across the
  // barrier in registers; the phases below are fenced with sched_barrier so
  // hipcc keeps at most one group of LDS reads in flight (no spills)
  s16x4 atr[NW / 16];
#pragma unroll
  for (int c = 0; c < NW / 16; ++c) atr[c] = s16x4{0, 0, 0, 0};
  const int q = i16 >> 2, pp = i16 & 3;

  for (int64_t my = 0; my <= nloc; ++my) {
    const bool have_cur = my < nloc;
    const bool have_prev = my > 0;
    const int buf = (int)(my % NBUF);
    SL_STAMP(0)
    const char* region = abuf + (buf * WAVES + w) * GG::REGION;
    // ---- P0: prefetch PD blocks ahead, then wait for this block
    if (have_cur) {
      if (my + PD < nloc) issue(b0 + (my + PD) * bstep, (int)((my + PD) % NBUF));
      // ops issued after block my's loads: the loads of up to PD younger blocks
      // plus the Y stores of iterations max(my-PD,1) .. my-1
      const int64_t yl = nloc - 1 - my;
      const int younger = (int)(yl < PD ? yl : PD);
      const int64_t lo = my - PD > 1 ? my - PD : 1;
      const int nst = (int)((my - 1) - lo + 1 > 0 ? (my - 1) - lo + 1 : 0);
      wait_vm(younger * GG::LPB + nst * sy);
    }
    SL_STAMP(1)
    __builtin_amdgcn_sched_barrier(0);
    // ---- P1: step-1 row fragments of block my
    bf16x8 af[NW / 32];
    if (have_cur) {
#pragma unroll
      for (int ks = 0; ks < NW / 32; ++ks) {
        const int row = i16;
        const int chunk = g4 + 4 * ks;
        af[ks] = *(const bf16x8*)(region + row * GG::ROWB + (chunk ^ (row & (GG::NCH - 1))) * 16);
      }
    }
    // ---- P2: y(prev) = sum of the 8 wave partials (fixed order, every wave)
    f32x4 ys[KT];
    if (have_prev) {
      const float* ypb = yp + (int)((my - 1) % YPB) * (WAVES * GG::YPW);
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        f32x4 s = *(const f32x4*)&ypb[(g4 * GG::KP + 16 * t + i16) * 4];
#pragma unroll
        for (int v = 1; v < WAVES; ++v) s += *(const f32x4*)&ypb[v * GG::YPW + (g4 * GG::KP + 16 * t + i16) * 4];
        ys[t] = s;
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    if constexpr (ST) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    SL_STAMP(2)
    if constexpr (YPB == 1) {
      // every wave holds y(prev): the single partial buffer may be rewritten
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
    SL_STAMP(3)
    // ---- P3: steps 3/4 of block prev (registers only)
    if (have_prev) {
      const int64_t r0 = (b0 + (my - 1) * bstep) * BM;
      if (r0 + BM > m) {  // ragged last block: rows past m contribute nothing
#pragma unroll
        for (int t = 0; t < KT; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (r0 + 4 * g4 + j >= m) ys[t][j] = 0.f;
      }
      if constexpr (STORE_Y) {
#pragma unroll
        for (int p = 0; p < GG::NSTORE; ++p) {
          if ((p % WAVES) == w) {
            const int t = p / 4, j = p % 4;
            const int64_t r = r0 + 4 * g4 + j;
            const int col = 16 * t + i16;
            float* dst = (r < m && col < k) ? Y + r * ldy + col : ydump + lane;
            *dst = ys[t][j];
          }
        }
      }
      constexpr bool hi_only = HI_T;
      s16x4 yh[KT], ylo[KT];
#pragma unroll
      for (int t = 0; t < KT; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const short h = bf16_bits(ys[t][j]);
          yh[t][j] = h;
          ylo[t][j] = bf16_bits(ys[t][j] - bf16_val(h));
        }
      if (!(ab & 4)) {
        if constexpr (hi_only) {
#pragma unroll
          for (int ct = 0; ct < NW / 16; ++ct)
#pragma unroll
            for (int t = 0; t < KT; ++t)
              accW[ct][t] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(atr[ct], yh[t], accW[ct][t], 0, 0, 0);
        } else {
#pragma unroll
          for (int ct = 0; ct < NW / 16; ++ct)
#pragma unroll
            for (int t = 0; t < KT; ++t) {
              accW[ct][t] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(atr[ct], yh[t], accW[ct][t], 0, 0, 0);
              accW[ct][t] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(atr[ct], ylo[t], accW[ct][t], 0, 0, 0);
            }
        }
      }
      if constexpr (DO_G) {
        if constexpr (G64) {
          // upper tile tau = (t1, t2): rows taken as 4 g + u on both sides
          // (a consistent permutation of the block's rows: same Gram)
          int tau = 0;
#pragma unroll
          for (int t1 = 0; t1 < KT; ++t1)
#pragma unroll
            for (int t2 = t1; t2 < KT; ++t2, ++tau) {
              if ((tau % WAVES) == w) {
                const int s = tau / WAVES;
#pragma unroll
                for (int u = 0; u < 4; ++u)
                  accG64[s] = __builtin_amdgcn_mfma_f64_16x16x4f64((double)ys[t1][u], (double)ys[t2][u], accG64[s], 0, 0, 0);
              }
            }
        } else {
#pragma unroll
          for (int tau = 0; tau < GG::GTILES; ++tau) {
            if ((tau % WAVES) == w) {
              const int s = tau / WAVES, t1 = tau / KT, t2 = tau % KT;
              accG[s] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(yh[t1], yh[t2], accG[s], 0, 0, 0);
              accG[s] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(yh[t1], ylo[t2], accG[s], 0, 0, 0);
              accG[s] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(ylo[t1], yh[t2], accG[s], 0, 0, 0);
            }
          }
        }
      }
    }
    SL_STAMP(4)
    __builtin_amdgcn_sched_barrier(0);
    if (have_cur) {
      // ---- P4: transposed fragments of block my for the NEXT iteration's step 3
      const int row = 4 * g4 + q;
#pragma unroll
      for (int ct = 0; ct < NW / 16; ++ct) {
        const int chunk = 2 * ct + (pp >> 1);
        const char* addr = region + row * GG::ROWB + (chunk ^ (row & (GG::NCH - 1))) * 16 + (pp & 1) * 8;
        atr[ct] = __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4 __attribute__((address_space(3)))*)addr);
      }
      // ---- P5: step 1 of block my: partial y over this wave's columns
      f32x4 accY[KT];
#pragma unroll
      for (int t = 0; t < KT; ++t) accY[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < NW / 32; ++ks)
#pragma unroll
        for (int t = 0; t < KT; ++t) accY[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks], zh[ks][t], accY[t], 0, 0, 0);
      // ---- P6: publish the partial
      float* ypb = yp + (int)(my % YPB) * (WAVES * GG::YPW) + w * GG::YPW;
#pragma unroll
      for (int t = 0; t < KT; ++t) *(f32x4*)&ypb[(g4 * GG::KP + 16 * t + i16) * 4] = accY[t];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    SL_STAMP(5)
    __builtin_amdgcn_s_barrier();
    SL_STAMP(6)
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (ST) {
    if (lane == 0) {
      unsigned long long* d = dbg + ((int64_t)blockIdx.x * WAVES + w) * 8;
#pragma unroll
      for (int i = 0; i < 6; ++i) d[i] = st_acc[i];
      d[6] = (unsigned long long)nloc;
      d[7] = 0;
    }
  }
#undef SL_STAMP

  // ---- partial slabs (same layout as v1: W [WAVES*NW][KP], G [KP][KP])
  {
    float* ws = Wslab + (int64_t)blockIdx.x * (WAVES * NW) * GG::KP;
#pragma unroll
    for (int ct = 0; ct < NW / 16; ++ct)
#pragma unroll
      for (int t = 0; t < KT; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          ws[(c0w + 16 * ct + g4 * 4 + j) * GG::KP + 16 * t + i16] = accW[ct][t][j];
  }
  if constexpr (DO_G && G64) {
    double* gs = (double*)Gslab + (int64_t)blockIdx.x * GG::KP * GG::KP;
    int tau = 0;
#pragma unroll
    for (int t1 = 0; t1 < KT; ++t1)
#pragma unroll
      for (int t2 = t1; t2 < KT; ++t2, ++tau) {
        if ((tau % WAVES) == w) {
          const int s = tau / WAVES;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int i = 16 * t1 + g4 + 4 * r, j = 16 * t2 + i16;
            gs[i * GG::KP + j] = accG64[s][r];
            if (t1 != t2) gs[j * GG::KP + i] = accG64[s][r];
          }
        }
      }
  } else if constexpr (DO_G) {
    float* gs = Gslab + (int64_t)blockIdx.x * GG::KP * GG::KP;
#pragma unroll
    for (int s = 0; s < GG::GS; ++s) {
      const int tau = w + WAVES * s;
      if (tau < GG::GTILES) {
        const int t1 = tau / KT, t2 = tau % KT;
#pragma unroll
        for (int j = 0; j < 4; ++j) gs[(16 * t1 + g4 * 4 + j) * GG::KP + 16 * t2 + i16] = accG[s][j];
      }
    }
  }
}

int grid2_for(int64_t m) {
  static int ncu = -1;
  if (ncu < 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      ncu = 256;
  }
  int64_t nb = (m + BM - 1) / BM;
  return (int)(nb < ncu ? nb : ncu);
}

int g_v2_ypb = -1;   // 1 or 2 partial buffers (SL_TSK2_YPB), tuning
int g_v2_ab = 0;     // ablation / policy bits (64: nt loads, 32: W from y_hi, 4: skip W)

template <int NW, int KT, bool DO_G, bool STORE_Y, bool HI_T, bool G64, int NBUF, int YPB>
int launch2(const bf16_t* A, int64_t m, int n, int64_t lda, const bf16_t* Zt, int k, float* Wslab,
            float* Gslab, float* Y, int64_t ldy, float* ydump, hipStream_t s) {
  using GG = Geo2<NW, KT, NBUF, YPB>;
  static_assert(GG::LDS <= 160 * 1024, "LDS budget");
  auto kern = k_tsk_pass2<NW, KT, DO_G, STORE_Y, HI_T, G64, NBUF, YPB>;
  static bool attr = false;
  if (!attr) {
    SL_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, GG::LDS));
    attr = true;
  }
  kern<<<grid2_for(m), THREADS, GG::LDS, s>>>(A, m, n, lda, Zt, k, Wslab, Gslab, Y, ldy, ydump, g_v2_ab, nullptr);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// deepest ring that fits 160 KiB next to the partial buffers
template <int NW, int KT, int YPB>
struct Ring {
  static constexpr int v = Geo2<NW, KT, 5, YPB>::LDS <= 160 * 1024 ? 5
                         : Geo2<NW, KT, 4, YPB>::LDS <= 160 * 1024 ? 4
                         : Geo2<NW, KT, 3, YPB>::LDS <= 160 * 1024 ? 3 : 2;
};

template <int NW, int KT, bool DO_G, bool STORE_Y, bool HI_T, bool G64>
int launch2_cfg(const bf16_t* A, int64_t m, int n, int64_t lda, const bf16_t* Zt, int k, float* Wslab,
                float* Gslab, float* Y, int64_t ldy, float* ydump, hipStream_t s) {
  if (g_v2_ypb < 0) {
    const char* e = getenv("SL_TSK2_YPB");
    g_v2_ypb = e ? atoi(e) : 2;
  }
  if (g_v2_ypb == 1)
    return launch2<NW, KT, DO_G, STORE_Y, HI_T, G64, Ring<NW, KT, 1>::v, 1>(A, m, n, lda, Zt, k, Wslab, Gslab, Y, ldy, ydump, s);
  return launch2<NW, KT, DO_G, STORE_Y, HI_T, G64, Ring<NW, KT, 2>::v, 2>(A, m, n, lda, Zt, k, Wslab, Gslab, Y, ldy, ydump, s);
}

}  // namespace

int sl_slab_reduce_launch(const float* slab, int nslab, int64_t slab_stride, int ld_in, int rows, int cols,
                          float* out, int ld_out, hipStream_t s);
int sl_slab_reduce_launch_d2d(const double* slab, int nslab, int64_t slab_stride, int ld_in, int rows,
                              int cols, double* out, int ld_out, hipStream_t s);

SL_API int sl_tsk2_set_tuning(int ypb, int ab) {
  g_v2_ypb = ypb;
  g_v2_ab = ab;
  return SL_OK;
}

// Same contract and workspace as sl_tsk_fused_pass (k <= 48 here; the
// caller falls back to v1 for wider sketches).  The Y dump slot sits at the
// end of the workspace (sl_tsk_fused_workspace reserves 256 bytes there).
SL_API int sl_tsk2_fused_pass(const void* A, int64_t m, int64_t n, int64_t lda, const void* Zt, int k,
                              float* W, float* G, float* Y, int64_t ldy, void* ws, int64_t ws_bytes, int flags,
                              void* stream) {
  if (m <= 0) return SL_OK;
  if (n % 8 || lda % 8 || n > 1024 || k > 48 || k < 1 || n < 8) {
    sl_set_last_error("tsk2_fused_pass: needs n%8==0, lda%8==0, 8<=n<=1024, 1<=k<=48");
    return SL_ERR_UNSUPPORTED;
  }
  hipStream_t s = (hipStream_t)stream;
  const int KT = (k + 15) / 16;
  const int KP = KT * 16;
  const bool small = n <= 512;
  const int NWT = small ? 512 : 1024;
  const int g = grid2_for(m);
  float* Wslab = (float*)ws;
  float* Gslab = Wslab + (int64_t)g * NWT * KP;
  float* ydump = (float*)((char*)ws + ws_bytes - 256);
  const bf16_t* a = (const bf16_t*)A;
  const bf16_t* z = (const bf16_t*)Zt;
  const bool nogram = flags & 1;
  const bool hi = flags & 2;
  const bool g64 = (flags & 4) != 0;
  if (g64 && (nogram || hi || !Y)) {
    sl_set_last_error("tsk2_fused_pass: the f64 Gram (flag 4) needs Y and flags & 3 == 0");
    return SL_ERR_UNSUPPORTED;
  }
  int rc = SL_ERR_UNSUPPORTED;
  // variants: intermediate (no G, no Y, W from y_hi), final (Y + f64 G),
  // final without G, generic exact (G f32, optional Y)
#define SL_T2(NW, KTT)                                                                                           \
  rc = g64 ? launch2_cfg<NW, KTT, true, true, false, true>(a, m, (int)n, lda, z, k, Wslab, Gslab, Y, ldy, ydump, s) \
     : (!Y && nogram && hi) ? launch2_cfg<NW, KTT, false, false, true, false>(a, m, (int)n, lda, z, k, Wslab, Gslab, Y, ldy, ydump, s) \
     : (Y && nogram) ? launch2_cfg<NW, KTT, false, true, false, false>(a, m, (int)n, lda, z, k, Wslab, Gslab, Y, ldy, ydump, s) \
     : Y ? launch2_cfg<NW, KTT, true, true, false, false>(a, m, (int)n, lda, z, k, Wslab, Gslab, Y, ldy, ydump, s) \
         : launch2_cfg<NW, KTT, true, false, false, false>(a, m, (int)n, lda, z, k, Wslab, Gslab, Y, ldy, ydump, s)
  if (small) {
    switch (KT) { case 1: SL_T2(64, 1); break; case 2: SL_T2(64, 2); break; default: SL_T2(64, 3); }
  } else {
    switch (KT) { case 1: SL_T2(128, 1); break; case 2: SL_T2(128, 2); break; default: SL_T2(128, 3); }
  }
#undef SL_T2
  if (rc != SL_OK) return rc;
  rc = sl_slab_reduce_launch(Wslab, g, (int64_t)NWT * KP, KP, (int)n, k, W, k, s);
  if (rc != SL_OK || nogram) return rc;
  if (g64) return sl_slab_reduce_launch_d2d((const double*)Gslab, g, (int64_t)KP * KP, KP, k, k, (double*)G, k, s);
  return sl_slab_reduce_launch(Gslab, g, (int64_t)KP * KP, KP, k, k, G, k, s);
}

// Diagnostic: the intermediate (or final G64) pass of the headline shape with
// per-phase s_memtime sums per wave: dbg[(wg * 8 + wave) * 8 + i], i < 6 the
// phases (wait, partial sum, barrier-1, steps 3/4, step 1 + publish, barrier),
// 6 = blocks of this workgroup.  Not used by the library.
SL_API int sl_tsk2_stamp_pass(const void* A, int64_t m, int64_t n, int64_t lda, const void* Zt, int k, void* ws,
                              int64_t ws_bytes, float* Y, unsigned long long* dbg, int final_pass, int ypb,
                              void* stream) {
  if (n != 1000 && n != 1024) return SL_ERR_UNSUPPORTED;
  if (k > 48 || k <= 32) return SL_ERR_UNSUPPORTED;
  hipStream_t s = (hipStream_t)stream;
  const bf16_t* a = (const bf16_t*)A;
  const bf16_t* z = (const bf16_t*)Zt;
  float* Wslab = (float*)ws;
  const int g = grid2_for(m);
  float* Gslab = Wslab + (int64_t)g * 1024 * 48;
  float* ydump = (float*)((char*)ws + ws_bytes - 256);
#define SL_ST(DG, SY, HI, G6, YB)                                                                        \
  {                                                                                                      \
    using GG = Geo2<128, 3, Ring<128, 3, YB>::v, YB>;                                                      \
    auto kern = k_tsk_pass2<128, 3, DG, SY, HI, G6, Ring<128, 3, YB>::v, YB, true>;                       \
    SL_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, GG::LDS)); \
    kern<<<g, THREADS, GG::LDS, s>>>(a, m, (int)n, lda, z, k, Wslab, Gslab, Y, k, ydump, g_v2_ab, dbg);      \
  }
  if (final_pass) {
    if (ypb == 1) SL_ST(true, true, false, true, 1) else SL_ST(true, true, false, true, 2)
  } else {
    if (ypb == 1) SL_ST(false, false, true, false, 1) else SL_ST(false, false, true, false, 2)
  }
#undef SL_ST
  SL_LAUNCH_CHECK();
  return SL_OK;
}
