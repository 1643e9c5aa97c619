// Fused tall-skinny pass, v3: four 256-column waves per CU (one per SIMD).
//
// Same contract as sl_tsk_fused_pass (tsk_kernels.hip): ONE read of a bf16
// row shard A (m x n, n <= 1024) gives W = A^T (A Z) and optionally
// G = Y^T Y (f64) and Y = A Z.  Reference hot loop: the two El::Gemm calls +
// QR Gram per power iteration (nla/svd.hpp:71-149).
//
// Why this shape (measured with the s_memtime build of v2, see
// benchmarks/tsk_stamps.py and profiles/): with eight 128-column waves the
// pass is LDS-bound -- every wave must see y = sum of the 8 wave partials,
// ~190 KB of LDS reads per 32 KB row block -- and the final pass spends
// ~2.5 k cycles per block in v_mfma_f32_16x16x16_bf16, which runs at HALF
// the rate of the K = 32 form on gfx950.  So:
//   * 4 waves x 256 columns (one wave per SIMD, up to 512 VGPRs: Z slice 96,
//     W accumulators 192): y is the sum of only 4 partials, and every wave
//     sums them itself (48 KB of LDS reads per block, one s_barrier);
//   * step 3 (W += A^T y) is ONE v_mfma_f32_16x16x32_bf16 per 16 x 16 tile
//     with K = [16 rows of y_hi ; the same 16 rows of y_lo]: exact-f32
//     equivalent W (every pass) at the cost of the old hi-only K = 16 form.
//     Lanes 32-63 carry the lo half: each lane reads 4 rows of a transposed
//     A tile and of the y partials, v_permlane32_swap gives it the other 4;
//   * software pipeline: iteration b runs step 1 of block b and steps 3/4 of
//     block b-1, the LDS-DMA prefetch (private per-wave ring regions) is
//     issued at the top of the iteration, PD = 3 blocks (96 KB) in flight;
//   * the f64 Gram (final pass) from the f32 y on v_mfma_f64_16x16x4;
//   * Y stores exact per instruction (rows past m to a dump slot), so the
//     per-wave vmcnt accounting is exact.
#include "sl_common.hpp"
#include <stdlib.h>

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) double f64x4;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int WAVES = 4;
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
  switch (n < 40 ? n : 40) {
    SL_VMW(0) SL_VMW(1) SL_VMW(2) SL_VMW(3) SL_VMW(4) SL_VMW(5) SL_VMW(6) SL_VMW(7) SL_VMW(8)
    SL_VMW(9) SL_VMW(10) SL_VMW(11) SL_VMW(12) SL_VMW(13) SL_VMW(14) SL_VMW(15) SL_VMW(16)
    SL_VMW(17) SL_VMW(18) SL_VMW(19) SL_VMW(20) SL_VMW(21) SL_VMW(22) SL_VMW(23) SL_VMW(24)
    SL_VMW(25) SL_VMW(26) SL_VMW(27) SL_VMW(28) SL_VMW(29) SL_VMW(30) SL_VMW(31) SL_VMW(32)
    SL_VMW(33) SL_VMW(34) SL_VMW(35) SL_VMW(36) SL_VMW(37) SL_VMW(38) SL_VMW(39)
    default: asm volatile("s_waitcnt vmcnt(40)" ::: "memory"); break;
  }
}
#undef SL_VMW

// value of x held by lane (l ^ 32).  Inline asm on purpose: hipcc (ROCm 7.2)
// merged several __builtin_amdgcn_permlane32_swap(x, x) calls on DIFFERENT x
// into one swap (tsk3 .s: one v_permlane32_swap feeding four selects) -- the real
// cause was the element bit_cast below, the asm form is kept anyway.  The s_nop covers the VALU-write -> permlane hazard.
__device__ __forceinline__ unsigned partner32(unsigned x, bool low) {
  unsigned a = x, b = x;
  asm("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(a), "+v"(b));
  return low ? b : a;
}
__device__ __forceinline__ f32x4 partner32(f32x4 v, bool low) {
  f32x4 o;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
            // scalar copy first: clang's __builtin_bit_cast of an ext_vector ELEMENT
            // lvalue reads element 0 (ROCm 7.2), which silently broke this swap
            const float e = v[j];
            o[j] = __builtin_bit_cast(float, partner32(__builtin_bit_cast(unsigned, e), low));
          }
  return o;
}
__device__ __forceinline__ s16x4 partner32(s16x4 v, bool low) {
  typedef __attribute__((ext_vector_type(2))) unsigned u32x2;
  u32x2 u = __builtin_bit_cast(u32x2, v);
  u[0] = partner32(u[0], low);
  u[1] = partner32(u[1], low);
  return __builtin_bit_cast(s16x4, u);
}

template <int NW, int KT, int NBUF>
struct Geo3 {
  static constexpr int ROWB = NW * 2;        // bytes per LDS row of a wave region
  static constexpr int NCH = NW / 8;         // 16-B chunks per row
  static constexpr int REGION = BM * ROWB;   // bytes per wave per ring slot
  static constexpr int LPB = REGION / 1024;  // LDS-DMA instructions per block per wave
  static constexpr int KP = KT * 16;
  static constexpr int ABYTES = NBUF * WAVES * REGION;
  static constexpr int YPW = 4 * KP * 4;     // floats of one wave's partial: [row group g][col][4 rows]
  static constexpr int YP_BYTES = 2 * WAVES * YPW * 4;
  static constexpr int LDS = ABYTES + YP_BYTES;
  static constexpr int GT64 = KT * (KT + 1) / 2;
  static constexpr int GS64 = (GT64 + WAVES - 1) / WAVES;
};

template <int NW, int KT, bool DO_G, bool STORE_Y, int NBUF, int SWAP_GROUP = 4>
__global__ void __launch_bounds__(THREADS, 1)
k_tsk_pass3(const bf16_t* __restrict__ A, int64_t m, int n, int64_t lda,
            const bf16_t* __restrict__ Zt, int k,
            float* __restrict__ Wslab, float* __restrict__ Gslab,
            float* __restrict__ Y, int64_t ldy, float* __restrict__ ydump, int ab) {
  using GG = Geo3<NW, KT, NBUF>;
  constexpr int PD = NBUF - 1;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* abuf = smem;
  float* yp = (float*)(smem + GG::ABYTES);

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g4 = lane >> 4, i16 = lane & 15;
  const bool low = lane < 32;
  // this lane's 4-row group of a 16-row block in steps 3/4: rows rb .. rb+3,
  // rb = 8 (g & 1) + 4 (g >> 1); its partner lane (l ^ 32) holds rb ^ 4
  const int rgrp = 2 * (g4 & 1) + (g4 >> 1);
  const int rb = 4 * rgrp;
  const int c0w = w * NW;
  const int64_t nblocks = (m + BM - 1) / BM;
  const int64_t b0 = blockIdx.x;
  const int64_t bstep = gridDim.x;
  const int64_t nloc = b0 < nblocks ? (nblocks - 1 - b0) / bstep + 1 : 0;
  // Y stores per block of this wave: one per tile (rows rb + w)
  const int sy = STORE_Y ? KT : 0;

  // ---- Z fragments (B operand of step 1): Z[c0w + 32 ks + 8 g + j][16 t + i16]
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
  f64x4 accG64[GG::GS64];
#pragma unroll
  for (int s = 0; s < GG::GS64; ++s) accG64[s] = f64x4{0.0, 0.0, 0.0, 0.0};

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

  // transposed A fragments of the previous block (4 rows rb..rb+3 of each
  // 16-column tile), carried across the barrier in registers
  s16x4 atr[NW / 16];
#pragma unroll
  for (int c = 0; c < NW / 16; ++c) atr[c] = s16x4{0, 0, 0, 0};
  const int q = i16 >> 2, pp = i16 & 3;

  for (int64_t my = 0; my <= nloc; ++my) {
    const bool have_cur = my < nloc;
    const bool have_prev = my > 0;
    const int buf = (int)(my % NBUF);
    const char* region = abuf + (buf * WAVES + w) * GG::REGION;
    // ---- P0: prefetch PD blocks ahead, then wait for this block
    if (have_cur) {
      if (my + PD < nloc) issue(b0 + (my + PD) * bstep, (int)((my + PD) % NBUF));
      const int64_t yl = nloc - 1 - my;
      const int younger = (int)(yl < PD ? yl : PD);
      const int64_t lo = my - PD > 1 ? my - PD : 1;
      const int nst = (int)((my - 1) - lo + 1 > 0 ? (my - 1) - lo + 1 : 0);
      wait_vm(younger * GG::LPB + nst * sy);
    }
    __builtin_amdgcn_sched_barrier(0);
    // ---- P2: y(prev) rows rb..rb+3 = sum of the 4 wave partials (fixed order)
    f32x4 ys[KT];
    if (have_prev) {
      const float* ypb = yp + (int)((my - 1) & 1) * (WAVES * GG::YPW);
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        const int o = (rgrp * GG::KP + 16 * t + i16) * 4;
        f32x4 s = *(const f32x4*)&ypb[o];
#pragma unroll
        for (int v = 1; v < WAVES; ++v) s += *(const f32x4*)&ypb[v * GG::YPW + o];
        ys[t] = s;
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    // ---- P3: steps 3/4 of block prev (registers only)
    if (have_prev) {
      const int64_t r0 = (b0 + (my - 1) * bstep) * BM;
      if (r0 + BM > m) {  // ragged last block: rows past m contribute nothing
#pragma unroll
        for (int t = 0; t < KT; ++t)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (r0 + rb + j >= m) ys[t][j] = 0.f;
      }
      if constexpr (STORE_Y) {
#pragma unroll
        for (int t = 0; t < KT; ++t) {
          const int64_t r = r0 + rb + w;
          const int col = 16 * t + i16;
          float* dst = (r < m && col < k) ? Y + r * ldy + col : ydump + lane;
          *dst = ys[t][w];
        }
      }
      if constexpr (DO_G) {
        // upper tiles (t1, t2), tau % WAVES == w; rows rb + u on both sides
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
      }
      // B operand over K = [y_hi rows 0..15 ; y_lo rows 0..15]: lanes g < 2 hold
      // hi of rows 8g..8g+7, lanes g >= 2 lo of rows 8(g-2)..8(g-2)+7
      bf16x8 yb[KT];
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        const f32x4 other = partner32(ys[t], low);
        const f32x4 r03 = low ? ys[t] : other;   // rows 8(g&1) + 0..3
        const f32x4 r47 = low ? other : ys[t];   // rows 8(g&1) + 4..7
        s16x8 v;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const short h0 = bf16_bits(r03[j]), h1 = bf16_bits(r47[j]);
          v[j] = low ? h0 : bf16_bits(r03[j] - bf16_val(h0));
          v[4 + j] = low ? h1 : bf16_bits(r47[j] - bf16_val(h1));
        }
        yb[t] = __builtin_bit_cast(bf16x8, v);
      }
      if (!(ab & 4)) {
#pragma unroll
        for (int ct = 0; ct < NW / 16; ++ct) {
          const s16x4 other = partner32(atr[ct], low);
          s16x8 a8;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            a8[j] = low ? atr[ct][j] : other[j];
            a8[4 + j] = low ? other[j] : atr[ct][j];
          }
          const bf16x8 af8 = __builtin_bit_cast(bf16x8, a8);
#pragma unroll
          for (int t = 0; t < KT; ++t)
            accW[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af8, yb[t], accW[ct][t], 0, 0, 0);
          // bound the hoisting of the lane swaps (register pressure at KT = 3)
          if ((ct & (SWAP_GROUP - 1)) == SWAP_GROUP - 1) __builtin_amdgcn_sched_barrier(0);
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    if (have_cur) {
      // ---- P4: transposed fragments (rows rb..rb+3) of block my for the next iteration
      const int row = rb + q;
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
      // row fragments A[row i16][c0w + 32 ks + 8 g + j], read in groups of 4
      // k-steps (register pressure: the W accumulators fill half the file)
#pragma unroll
      for (int k0 = 0; k0 < NW / 32; k0 += 4) {
        bf16x8 af[4];
#pragma unroll
        for (int u = 0; u < 4 && k0 + u < NW / 32; ++u) {
          const int chunk = g4 + 4 * (k0 + u);
          af[u] = *(const bf16x8*)(region + i16 * GG::ROWB + (chunk ^ (i16 & (GG::NCH - 1))) * 16);
        }
#pragma unroll
        for (int u = 0; u < 4 && k0 + u < NW / 32; ++u)
#pragma unroll
          for (int t = 0; t < KT; ++t)
            accY[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[u], zh[k0 + u][t], accY[t], 0, 0, 0);
      }
      // ---- P6: publish the partial (C fragment: rows 4 g + j of col 16 t + i16)
      float* ypb = yp + (int)(my & 1) * (WAVES * GG::YPW) + w * GG::YPW;
#pragma unroll
      for (int t = 0; t < KT; ++t) *(f32x4*)&ypb[(g4 * GG::KP + 16 * t + i16) * 4] = accY[t];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // ---- partial slabs (same layout as v1: W [WAVES*NW][KP], G [KP][KP] f64)
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
  if constexpr (DO_G) {
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
  }
}

int grid3_for(int64_t m) {
  static int ncu = -1;
  if (ncu < 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      ncu = 256;
  }
  int64_t nb = (m + BM - 1) / BM;
  return (int)(nb < ncu ? nb : ncu);
}

int g_v3_ab = 0;  // tuning bits (64: nt loads, 4: skip the W update)

template <int NW, int KT>
struct Ring3 {
  static constexpr int v = Geo3<NW, KT, 5>::LDS <= 160 * 1024 ? 5
                         : Geo3<NW, KT, 4>::LDS <= 160 * 1024 ? 4
                         : Geo3<NW, KT, 3>::LDS <= 160 * 1024 ? 3 : 2;
};

template <int NW, int KT, bool DO_G, bool STORE_Y>
int launch3(const bf16_t* A, int64_t m, int n, int64_t lda, const bf16_t* Zt, int k, float* Wslab,
            float* Gslab, float* Y, int64_t ldy, float* ydump, hipStream_t s) {
  constexpr int NB = Ring3<NW, KT>::v;
  using GG = Geo3<NW, KT, NB>;
  static_assert(GG::LDS <= 160 * 1024, "LDS budget");
  auto kern = k_tsk_pass3<NW, KT, DO_G, STORE_Y, NB>;
  static bool attr = false;
  if (!attr) {
    SL_HIP_CHECK(hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, GG::LDS));
    attr = true;
  }
  kern<<<grid3_for(m), THREADS, GG::LDS, s>>>(A, m, n, lda, Zt, k, Wslab, Gslab, Y, ldy, ydump, g_v3_ab);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

}  // namespace

int sl_slab_reduce_launch(const float* slab, int nslab, int64_t slab_stride, int ld_in, int rows, int cols,
                          float* out, int ld_out, hipStream_t s);
int sl_slab_reduce_launch_d2d(const double* slab, int nslab, int64_t slab_stride, int ld_in, int rows,
                              int cols, double* out, int ld_out, hipStream_t s);

SL_API int sl_tsk3_set_tuning(int ab) {
  g_v3_ab = ab;
  return SL_OK;
}

// Same contract and workspace as sl_tsk_fused_pass, for k <= 48.  W is exact
// (f32-equivalent) in every mode; flag 1 skips G, flag 4 asks for the f64 G
// (needs Y); a Gram without flag 4 is also formed in f64.  Flag 2 (bf16 y
// for W) is accepted and ignored: the exact W costs the same here.  The Y
// dump slot is the last 256 bytes of the workspace.
SL_API int sl_tsk3_fused_pass(const void* A, int64_t m, int64_t n, int64_t lda, const void* Zt, int k,
                              float* W, void* G, float* Y, int64_t ldy, void* ws, int64_t ws_bytes, int flags,
                              void* stream) {
  if (m <= 0) return SL_OK;
  if (n % 8 || lda % 8 || n > 1024 || k > 48 || k < 1 || n < 8) {
    sl_set_last_error("tsk3_fused_pass: needs n%8==0, lda%8==0, 8<=n<=1024, 1<=k<=48");
    return SL_ERR_UNSUPPORTED;
  }
  hipStream_t s = (hipStream_t)stream;
  const int KT = (k + 15) / 16;
  const int KP = KT * 16;
  const bool small = n <= 512;
  const int NWT = small ? 512 : 1024;
  const int g = grid3_for(m);
  float* Wslab = (float*)ws;
  float* Gslab = Wslab + (int64_t)g * NWT * KP;
  float* ydump = (float*)((char*)ws + ws_bytes - 256);
  const bf16_t* a = (const bf16_t*)A;
  const bf16_t* z = (const bf16_t*)Zt;
  const bool dog = !(flags & 1);
  int rc = SL_ERR_UNSUPPORTED;
#define SL_T3(NW, KTT)                                                                                       \
  rc = (dog && Y) ? launch3<NW, KTT, true, true>(a, m, (int)n, lda, z, k, Wslab, Gslab, Y, ldy, ydump, s)     \
     : dog ? launch3<NW, KTT, true, false>(a, m, (int)n, lda, z, k, Wslab, Gslab, Y, ldy, ydump, s)            \
     : Y ? launch3<NW, KTT, false, true>(a, m, (int)n, lda, z, k, Wslab, Gslab, Y, ldy, ydump, s)              \
         : launch3<NW, KTT, false, false>(a, m, (int)n, lda, z, k, Wslab, Gslab, Y, ldy, ydump, s)
  if (small) {
    switch (KT) { case 1: SL_T3(128, 1); break; case 2: SL_T3(128, 2); break; default: SL_T3(128, 3); }
  } else {
    switch (KT) { case 1: SL_T3(256, 1); break; case 2: SL_T3(256, 2); break; default: SL_T3(256, 3); }
  }
#undef SL_T3
  if (rc != SL_OK) return rc;
  rc = sl_slab_reduce_launch(Wslab, g, (int64_t)NWT * KP, KP, (int)n, k, W, k, s);
  if (rc != SL_OK || !dog) return rc;
  return sl_slab_reduce_launch_d2d((const double*)Gslab, g, (int64_t)KP * KP, KP, k, k, (double*)G, k, s);
}
