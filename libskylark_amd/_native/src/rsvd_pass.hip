// Fused randSVD pass (the streaming core of nla/svd.hpp:71-149 and :278-317).
//
// ONE read of A (m x n bf16, row-major) produces, per workgroup,
//     y = A_blk Z           (16 x k per row block, never leaves the chip)
//     W_part += A_blk^T y   (n x k f32, held in registers for the whole kernel)
// plus, in the FINAL form, the stored Y = A Z (m x k f32) and the fp64 Gram
// Y^T Y.  W / G partials go to per-workgroup slabs that a second kernel
// (k_rsvd_reduce*) sums.
//
// gfx950 structure (one 512-thread workgroup per CU, persistent grid; the
// role split is described at k_rsvd_pass5):
//   * A arrives by LDS-DMA (global_load_lds_dwordx4, inline asm so the
//     compiler neither tracks nor drains it) into a ring of 16-row slots in a
//     swizzled image that both the row reads of step 1 and the transposed
//     reads (ds_read_b64_tr_b16) of step 3 hit conflict-free;
//   * completion is ordered by hand-counted s_waitcnt vmcnt(N), one workgroup
//     barrier per block;
//   * step 3 W += A^T (y_hi + y_lo) is one v_mfma_f32_16x16x32_bf16 per
//     16 x 16 W tile and block: K = 32 packs [8 rows of y_hi | the same 8
//     rows of y_lo], so W sees y to ~16 bits while A streams as bf16.
#include <algorithm>

#include "sl_common.hpp"

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) double f64x4;
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(3))) s16x4 lds_s16x4;


// LDS-DMA of 16 B per lane into LDS[lds_base + lane * 16], as inline asm so
// hipcc neither tracks it nor drains it with its own vmcnt(0) before later
// LDS reads; completion is ordered by the hand-counted waits below.
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

// same with a wave-uniform 64-bit base in SGPRs and a per-lane 32-bit byte
// offset (global_load_lds ... saddr form): no per-block address VALU.
// NT: the non-temporal policy (A is read once per pass: the stream alone
// runs at 7.0 TB/s with it against 6.35 without, benchmarks/probe/dma_stream.hip)
template <bool NT = false>
__device__ __forceinline__ void glds16s(unsigned voff, const void* sbase, unsigned lds_base) {
  unsigned keep;
  if constexpr (NT)
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %3\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, %2 nt\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(sbase), "s"(lds_base)
        : "memory");
  else
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %3\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, %2\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(voff), "s"(sbase), "s"(lds_base)
        : "memory");
}

// s_waitcnt vmcnt(n) for a run-time (wave-uniform) n
__device__ __forceinline__ void wait_vm(int n) {
  switch (n) {
#define SLW(N) case N: asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory"); break;
    SLW(0) SLW(1) SLW(2) SLW(3) SLW(4) SLW(5) SLW(6) SLW(7) SLW(8) SLW(9) SLW(10) SLW(11) SLW(12) SLW(13)
    SLW(14) SLW(15) SLW(16) SLW(17) SLW(18) SLW(19) SLW(20) SLW(21) SLW(22) SLW(23) SLW(24) SLW(25)
    SLW(26) SLW(27) SLW(28) SLW(29) SLW(30) SLW(31)
#undef SLW
    default: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
  }
}

// workgroup barrier over LDS: this wave's LDS ops complete, then s_barrier;
// the trailing compiler fence keeps later LDS reads from being hoisted above
// the barrier (the s_barrier builtin alone is not a memory fence to LLVM)
__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// swizzle of 16-B chunk slots by row (see tsk_kernels.hip: a GF(2) map that
// keeps the b128 row reads and the transposed reads conflict-free)
template <int NCH>
__device__ __forceinline__ int swz4(int row) {
  if constexpr (NCH == 16) return ((row << 1) & 15) ^ (((row >> 3) & 1) * 9);
  else return row & (NCH - 1);
}


// out[i][j] (i < rows, j < cols) = sum_s slab[s][i * cols + j], summed in f64.
// 128 consecutive elements per 512-thread workgroup (two per lane); wave v
// sums slabs v, v + 8, ... with four loads in flight; 8 partials through LDS.
template <typename IT, typename OT>
__device__ __forceinline__ void reduce_body(const IT* __restrict__ slab, int nslab, int64_t total, int cols,
                                            OT* __restrict__ out, int ldo, int blk, double (*part)[128]) {
  const int lane = threadIdx.x & 63, v = threadIdx.x >> 6;
  const int64_t e0 = (int64_t)blk * 128 + 2 * lane;
  double a0 = 0, a1 = 0, b0 = 0, b1 = 0;
  if (e0 + 1 < total) {
    int s = v;
    // eight slabs' loads in flight per wave (a round trip to the slabs is
    // ~0.5 us; two in flight left the reduce latency-bound)
    for (; s + 56 < nslab; s += 64) {
      IT x0[8], x1[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const IT* p = slab + (int64_t)(s + 8 * q) * total + e0;
        x0[q] = p[0];
        x1[q] = p[1];
      }
#pragma unroll
      for (int q = 0; q < 8; q += 2) {
        a0 += (double)x0[q]; a1 += (double)x1[q];
        b0 += (double)x0[q + 1]; b1 += (double)x1[q + 1];
      }
    }
    for (; s + 8 < nslab; s += 16) {
      const IT* p = slab + (int64_t)s * total + e0;
      const IT* q = p + 8 * total;
      a0 += (double)p[0]; a1 += (double)p[1];
      b0 += (double)q[0]; b1 += (double)q[1];
    }
    for (; s < nslab; s += 8) {
      const IT* p = slab + (int64_t)s * total + e0;
      a0 += (double)p[0]; a1 += (double)p[1];
    }
  } else if (e0 < total) {
    for (int s = v; s < nslab; s += 8) a0 += (double)slab[(int64_t)s * total + e0];
  }
  part[v][2 * lane] = a0 + b0;
  part[v][2 * lane + 1] = a1 + b1;
  __syncthreads();
  if (threadIdx.x < 128) {
    const int64_t e = (int64_t)blk * 128 + threadIdx.x;
    if (e < total) {
      double sum = 0;
#pragma unroll
      for (int u = 0; u < 8; ++u) sum += part[u][threadIdx.x];
      const int64_t i = e / cols, j = e - i * cols;
      out[i * ldo + j] = (OT)sum;
    }
  }
}

template <typename IT, typename OT>
__global__ void __launch_bounds__(512)
k_rsvd_reduce(const IT* __restrict__ slab, int nslab, int64_t total, int cols, OT* __restrict__ out, int ldo,
              int* __restrict__ zero_word) {
  __shared__ double part[8][128];
  if (zero_word && blockIdx.x == 0 && threadIdx.x == 0) *zero_word = 0;
  reduce_body<IT, OT>(slab, nslab, total, cols, out, ldo, blockIdx.x, part);
}

// the final pass's two sums in ONE launch: blocks [0, gw) the f32 W slabs
// into f64, the rest the fp64 Gram slabs
__global__ void __launch_bounds__(512)
k_rsvd_reduce_wg(const float* __restrict__ wslab, int64_t tw, int cols, double* __restrict__ wout, int ldw,
                 const double* __restrict__ gslab, int64_t tg, double* __restrict__ gout, int ldg, int nslab, int gw,
                 int* __restrict__ zero_word) {
  __shared__ double part[8][128];
  if (zero_word && blockIdx.x == 0 && threadIdx.x == 0) *zero_word = 0;
  if ((int)blockIdx.x < gw) reduce_body<float, double>(wslab, nslab, tw, cols, wout, ldw, blockIdx.x, part);
  else reduce_body<double, double>(gslab, nslab, tg, cols, gout, ldg, blockIdx.x - gw, part);
}

// ---------------------------------------------------------------- pass v5
// Role-split form of the fused pass:
//   * step 1 (y = A_blk Z) is owned by KT "y waves": wave t < KT computes the
//     whole 16 x 16 tile t of y over ALL n columns (its Z^T slice, 32 bf16
//     fragments, in registers), so y never needs a cross-wave sum (no
//     partial tiles, no reducer phase);
//   * step 3 (W += A^T (y_hi + y_lo)) is split over all 8 waves by 16-column
//     W tiles, sized so every SIMD pair (waves w and w + 4 share a SIMD) gets
//     about the same matrix-core work (the y waves take 0-2 W tiles);
//   * ONE barrier per block: the phase after barrier j runs step 3 of block j
//     (y(j) published before it) and, on the y waves, step 1 of block j + 1
//     into the other half of a double-buffered y image; the DMA of block
//     j + 1 is waited for by every wave (its own LDS-DMA, counted vmcnt)
//     before barrier j, so any wave may read any region;
//   * the ring keeps NBUF = 4 slots of 16 rows x 1024 columns: in phase j
//     slots j (step 3) and j + 1 (step 1) are read, j + 2 and j + 3 in flight.
// The two roles run separately instantiated loop bodies (the y waves hold
// 32 Z fragments and <= 2 W tiles, the W waves <= 12 W tiles), so the
// register allocation is the larger of the two, not their sum.
struct P5Tiles {
  int base[8];
  int cnt[8];
  int gown[8];   // Gram tiles: first tau owned and stride (FINAL), per wave
  int prio;      // s_setprio of the y waves (tuning knob, variant bits 6-7)
  int rev;       // walk the row blocks last-to-first (variant bit 8): consecutive
                 // passes alternate, so a pass starts on the rows the previous
                 // one read last (still in the MALL)
  int nt;        // LDS-DMA cache policy (variant bits 9-11): 0 default; 1 nt for
                 // every block; c >= 2 nt except each workgroup's last
                 // ntail = 8 (c - 1) blocks, which keep the default policy so
                 // the next pass (walking the other way) finds them in the MALL
  int ntail;
  int nty;       // FINAL: non-temporal stores of Y (variant bit 12)
  // EXT forms (sl_rsvd_pass_ext): the operand Zt holds [X_hi^T; X_lo^T]
  // (2 kx rows) and step 1 folds the two halves, y = A (X_hi + X_lo) in f32
  // (kx <= 8 real columns); EXT 2 also streams a given column-major D (m x
  // kx, column stride lddc) beside A and forms W = A^T D instead of A^T y
  int kx;
  const float* D;
  int64_t lddc;
};

#ifndef P1_PD
#define P1_PD 8   // step-1 A fragments in flight per y wave
#endif
#ifndef P3_PT
#define P3_PT 4   // step-3 W tiles' A^T fragments in flight per wave
#endif
constexpr int P5_NBUF = 4, P5_BM = 16, P5_ROWB = 256, P5_REGION = 4096, P5_LPB = 4, P5_T1 = 2, P5_T2 = 12,
              P5_GS = 2;

template <int KT>
constexpr int p5_y16p() { return 16 * KT * P5_BM * 2 + 16; }
template <int KT, bool FINAL, int EXT = 0>
constexpr int p5_lds() {
  return P5_NBUF * 8 * P5_REGION + 4 * p5_y16p<KT>() + (FINAL ? 2 * P5_BM * 16 * KT * 4 : 0) +
         (EXT == 2 ? P5_NBUF * P5_BM * 16 * 4 : 0);
}

template <int KT, bool FINAL, bool GRAM, bool YROLE, int TM, int KS, int EXT>
__device__ __forceinline__ void p5_body(const bf16_t* __restrict__ A, int64_t m, int n, int64_t lda,
                                        const bf16_t* __restrict__ Zt, int k, float* __restrict__ Wslab,
                                        double* __restrict__ Gslab, float* __restrict__ Y, int64_t ldy,
                                        float* __restrict__ scratch, const P5Tiles& pt, char* smem, const int w) {
  constexpr int KP = 16 * KT, BM = P5_BM, NBUF = P5_NBUF, ROWB = P5_ROWB, REGION = P5_REGION, LPB = P5_LPB;
  constexpr int Y16P = p5_y16p<KT>();
  char* ring = smem;
  char* y16b = smem + NBUF * 8 * REGION;                 // [2 buffers][hi | lo]
  float* yfb = (float*)(y16b + 4 * Y16P);                // FINAL: [2][BM * k] f32 rows of y'
  float* dsl = yfb + 2 * BM * KP;                        // EXT 2: [NBUF][16 columns][BM rows] of D
  const int kr = EXT ? pt.kx : k;                        // real columns of y / W / Y
  const int lane = threadIdx.x & 63;
  const int g4 = lane >> 4, i16 = lane & 15;
  const int64_t nblocks = (m + BM - 1) / BM;
  const int64_t b0 = blockIdx.x, bstep = gridDim.x;
  const int64_t nloc = b0 < nblocks ? (nblocks - 1 - b0) / bstep + 1 : 0;
  const bool rev = pt.rev != 0;
  auto row0 = [&](int64_t jb) -> int64_t {
    const int64_t b = b0 + jb * bstep;
    return (rev ? nblocks - 1 - b : b) * BM;
  };
  // step 1 runs KS (16 or 32) k-steps of 32 columns: regions past n were
  // zeroed (below) and Z is zero past n, so the extra products add exact zeros
  const bool dma_on = 128 * w < n;                        // this wave's 128-column region exists
  const int tbase = pt.base[w], tcnt = pt.cnt[w];
  if (!dma_on) {
    // never DMA'd: zero this region of every slot once (stale LDS could hold NaNs)
    for (int sl = 0; sl < NBUF; ++sl)
      for (int o = lane * 16; o < REGION; o += 1024) *(f32x4*)(ring + (sl * 8 + w) * REGION + o) = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  // ---- y waves: Z^T slice of tile t = w (B operand: lane holds Z[32 ks + 8 g4 + j][16 w + i16])
  bf16x8 zf[YROLE ? KS : 1];
  if constexpr (YROLE) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int col = 16 * w + i16, kk = 32 * ks + 8 * g4;
      bf16x8 v = {};
      if (col < k && kk + 8 <= n) v = *(const bf16x8*)(Zt + (int64_t)col * n + kk);
      zf[ks] = v;
    }
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) asm volatile("" ::"v"(zf[ks]));
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  f32x4 accW[TM > 0 ? TM : 1][KT];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int t = 0; t < KT; ++t) accW[a][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr bool G_ON = GRAM && !YROLE;
  f64x4 accG[G_ON ? P5_GS : 1];
  f32x4 gblk[G_ON ? P5_GS : 1];
#pragma unroll
  for (int s = 0; s < (G_ON ? P5_GS : 1); ++s) {
    accG[s] = f64x4{0.0, 0.0, 0.0, 0.0};
    gblk[s] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  constexpr int GT = KT * (KT + 1) / 2;
  const int gfirst = pt.gown[w] & 0xff, gstride = pt.gown[w] >> 8;   // Gram tiles gfirst, +gstride, ...
  bool gpend = false;
  auto gram_acc = [&]() {
    if constexpr (G_ON) {
      if (gpend) {
#pragma unroll
        for (int s = 0; s < P5_GS; ++s)
#pragma unroll
          for (int e = 0; e < 4; ++e) accG[s][e] += (double)gblk[s][e];
      }
    }
  };

  // LDS-DMA of this wave's region of row block blk into slot `slot` (swizzled image)
  unsigned voff[LPB];
#pragma unroll
  for (int i = 0; i < LPB; ++i) {
    const int byte = i * 1024 + lane * 16;
    const int row = byte / ROWB;
    const int sl = (byte % ROWB) / 16;
    const int chunk = sl ^ swz4<16>(row);
    int col = 128 * w + chunk * 8;
    col = col + 8 <= n ? col : n - 8;
    voff[i] = (unsigned)((row * lda + col) * 2);
  }
  // (vmcnt bookkeeping is analytic, see the main loop: no per-slot counters)
  auto issue = [&](int64_t blk) {
    if (!dma_on) return;
    const int slot = (int)(blk % NBUF);
    char* region = ring + (slot * 8 + w) * REGION;
    const int64_t r0 = row0(blk);
    if (r0 + BM <= m) {
      const bf16_t* base = A + r0 * lda;
      if (pt.nt && blk < nloc - pt.ntail) {
#pragma unroll
        for (int i = 0; i < LPB; ++i) {
          const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_void*)(region + i * 1024));
          glds16s<true>(voff[i], (const void*)base, dst);
        }
      } else {
#pragma unroll
        for (int i = 0; i < LPB; ++i) {
          const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_void*)(region + i * 1024));
          glds16s<false>(voff[i], (const void*)base, dst);
        }
      }
      if constexpr (EXT == 2) {
        // the block's D rows: lane l < 4 kx loads column l / 4, rows 4 (l % 4)
        // .. + 3 (16 B, column-major D) into dsl[slot][col][row]; m % 16 == 0
        // (the host checks), so every block is whole
        if (w == 0) {
          const int c = lane >> 2, rq = lane & 3;
          const float* src = pt.D + (c < kr ? (int64_t)c * pt.lddc + r0 + 4 * rq : 0);
          const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_void*)(dsl + slot * BM * 16));
          glds16((const void*)src, dst);
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < LPB; ++i) {
        const int byte = i * 1024 + lane * 16;
        const int row = byte / ROWB;
        int64_t grow = r0 + row;
        grow = grow < m ? grow : m - 1;
        const unsigned dst = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(lds_void*)(region + i * 1024));
        glds16((const void*)((const char*)(A + grow * lda) + (voff[i] - (unsigned)(row * lda * 2))), dst);
      }
    }
  };
  const int lpb = dma_on ? (EXT == 2 && w == 0 ? LPB + 1 : LPB) : 0;

  // ---- step 1 of block jb (y waves): tile w of y over all columns, published
  //      as the bf16 hi / lo B-fragment images (and, FINAL, the f32 rows of y')
  auto step1 = [&](int64_t jb) {
    if constexpr (YROLE) {
      const char* reg0 = ring + (int)(jb % NBUF) * 8 * REGION;
      const int sw = swz4<16>(i16);
      // The A fragments stream through a ring of P1_PD registers (that many
      // LDS reads in flight) and the K steps alternate between two
      // accumulators: written as one read -> MFMA chain, the compiler kept
      // two reads in flight and every MFMA waited on an LDS round trip.
      // Inter passes in the engine 361 -> 357 / 351 -> 338 us, the pass
      // alone 409 -> 385 us (profiles/r6/pass_prefetch_ab_*.txt).
      auto rd = [&](int ks) -> bf16x8 {
        const int chunk = ((ks & 3) << 2) + g4;
        return *(const bf16x8*)(reg0 + (ks >> 2) * REGION + i16 * ROWB + ((chunk ^ sw) << 4));
      };
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      if constexpr (FINAL) {
        // (the FINAL form, whose W waves also store Y and form the Gram,
        // keeps the compiler's order: the pinned ring below measured 20 us
        // slower per pass there)
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rd(ks), zf[ks], acc, 0, 0, 0);
      } else {
        constexpr int PD = P1_PD < KS ? P1_PD : KS;
        // its own scheduling region, ordered: PD reads, then (MFMA, read)
        // pairs, then the last PD MFMAs (left to itself the scheduler
        // re-serialised the reads to save registers)
        __builtin_amdgcn_sched_barrier(0);
        bf16x8 afr[PD];
#pragma unroll
        for (int u = 0; u < PD; ++u) afr[u] = rd(u);
        f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) {
          const bf16x8 af = afr[ks % PD];
          if (ks & 1) acc1 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, zf[ks], acc1, 0, 0, 0);
          else acc0 = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, zf[ks], acc0, 0, 0, 0);
          if (ks + PD < KS) afr[ks % PD] = rd(ks + PD);
        }
        __builtin_amdgcn_sched_group_barrier(0x100, PD, 0);
#pragma unroll
        for (int ks = 0; ks + PD < KS; ++ks) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x008, PD, 0);
        __builtin_amdgcn_sched_barrier(0);
        acc = acc0 + acc1;
      }
      const int64_t r0 = row0(jb);
      if (r0 + BM > m) {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (r0 + 4 * g4 + e >= m) acc[e] = 0.f;
      }
      f32x4 yfold = acc;
      if constexpr (EXT != 0) {
        // y = A X_hi + A X_lo: column c + kx of the tile is column c's low part
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float part = __shfl_down(acc[e], kr, 16);
          yfold[e] = i16 < kr ? acc[e] + part : 0.f;
        }
        acc = yfold;
        if constexpr (EXT == 2) {
          // step 3 takes D, not y: D's block rows from the slot DMA'd with A
          const float* dsp = dsl + (int)(jb % NBUF) * BM * 16;
#pragma unroll
          for (int e = 0; e < 4; ++e) acc[e] = i16 < kr ? dsp[i16 * 16 + 4 * g4 + e] : 0.f;
        }
      }
      // y = hi + lo as two bf16 planes, by integer round-to-nearest-even on
      // the f32 bits (f_to_bf16) and packed by hand: the __bf16-typed form
      // of this conversion was miscompiled in some instantiations (wrong
      // planes with a correct accumulator, profiles/r5 diagnostics)
      unsigned hb[4], lb[4];
      float yv[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        hb[e] = f_to_bf16(acc[e]);
        const float hv = __uint_as_float(hb[e] << 16);
        lb[e] = f_to_bf16(acc[e] - hv);
        yv[e] = hv + __uint_as_float(lb[e] << 16);
      }
      char* y16 = y16b + (int)(jb & 1) * 2 * Y16P;
      const int col = 16 * w + i16;
      *(uint2*)(y16 + col * 32 + g4 * 8) = make_uint2(hb[0] | (hb[1] << 16), hb[2] | (hb[3] << 16));
      *(uint2*)(y16 + Y16P + col * 32 + g4 * 8) = make_uint2(lb[0] | (lb[1] << 16), lb[2] | (lb[3] << 16));
      s16x4 hi, lo;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        hi[e] = (short)hb[e];
        lo[e] = (short)lb[e];
      }
      if constexpr (FINAL) {
        float* yf = yfb + (int)(jb & 1) * BM * KP;
        if (col < kr) {
#pragma unroll
          for (int e = 0; e < 4; ++e) yf[(4 * g4 + e) * kr + col] = EXT ? yfold[e] : yv[e];
        }
      }
    }
  };

  // ---- FINAL: this wave's share of block jb's stored Y (after the barrier that
  //      published it).  Store waves: the W waves 0.. of the W role, one
  //      instruction each (float4 rows when ldy == k, else 4-B elements).
  const bool vecY = FINAL && (kr % 4 == 0) && (ldy == kr);
  const int wy = YROLE ? -1 : w - KT;                 // index among the W waves
  const int nyv = (BM * kr + (vecY ? 255 : 63)) / (vecY ? 256 : 64);   // store instructions per block
  const int nst = (!FINAL || wy < 0 || wy >= nyv) ? 0 : (nyv - wy + (8 - KT) - 1) / (8 - KT);
  auto store_y = [&](int64_t jb) {
    if constexpr (FINAL && !YROLE) {
      const float* yf = yfb + (int)(jb & 1) * BM * KP;
      const int64_t r0 = row0(jb);
      for (int q = wy; q < nyv; q += 8 - KT) {
        if (vecY) {
          const int t = q * 64 + lane;
          const bool ok = t < BM * kr / 4 && r0 + (4 * t) / kr < m;
          f32x4 v = {0.f, 0.f, 0.f, 0.f};
          if (ok) v = *(const f32x4*)&yf[4 * t];
          float* dst = ok ? Y + r0 * ldy + 4 * t : scratch + 4 * lane;
          if (pt.nty) __builtin_nontemporal_store(v, (f32x4*)dst);
          else *(f32x4*)dst = v;
        } else {
          const int t = q * 64 + lane;
          const int row = t / kr, col = t - (t / kr) * kr;
          const bool ok = t < BM * kr && r0 + row < m;
          const float v = ok ? yf[t] : 0.f;
          float* dst = ok ? Y + (r0 + row) * ldy + col : scratch + lane;
          *dst = v;
        }
      }
    }
  };

  // ---- step 3 of block j: W tiles of this wave (+ FINAL Gram tiles of y')
  auto step3 = [&](int64_t j) {
    const char* slotp = ring + (int)(j % NBUF) * 8 * REGION;
    const char* y16 = y16b + (int)(j & 1) * 2 * Y16P;
    const int rb = 8 * (g4 >> 1);
    const char* yp = y16 + (g4 & 1) * Y16P + rb * 2;
    bf16x8 yfr[KT];
#pragma unroll
    for (int t = 0; t < KT; ++t) yfr[t] = *(const bf16x8*)(yp + (16 * t + i16) * 32);
    if constexpr (G_ON) {
      // this wave's Gram tiles tau = gfirst + s * gstride (slot s), operands
      // picked by selects; a wave owning none skips, a second slot past GT
      // multiplies a dummy pair that is never stored
#pragma unroll
      for (int sg = 0; sg < P5_GS; ++sg) {
        const int tau = gfirst + sg * gstride;
        if (gstride == 0 || tau >= GT) break;   // uniform: no dummy products
        const int t1 = tau < KT ? 0 : (tau < 2 * KT - 1 ? 1 : 2);
        const int t2 = t1 == 0 ? tau : (t1 == 1 ? tau - KT + 1 : 2);
        bf16x8 y1 = yfr[0], y2 = yfr[0];
#pragma unroll
        for (int t = 1; t < KT; ++t) {
          y1 = t1 == t ? yfr[t] : y1;
          y2 = t2 == t ? yfr[t] : y2;
        }
        const bf16x8 ysw = *(const bf16x8*)(y16 + ((g4 & 1) ^ 1) * Y16P + rb * 2 + (16 * t2 + i16) * 32);
        const f32x4 z4 = {0.f, 0.f, 0.f, 0.f};
        gblk[sg] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(y1, y2, z4, 0, 0, 0);
        gblk[sg] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(y1, ysw, gblk[sg], 0, 0, 0);
      }
      gpend = true;
    }
    (void)GT;
    const int q = i16 >> 2, p = i16 & 3;
    // the A^T fragment of W tile ct (two transposed LDS reads); a slot past
    // this wave's count re-reads its first tile into an accumulator that is
    // never stored (no branch in the MFMA stream)
    auto tile_rd = [&](int ct) -> bf16x8 {
      const int gt = tbase + (YROLE || ct < tcnt ? ct : 0);
      const char* region = slotp + (gt >> 3) * REGION;
      const int chunk = 2 * (gt & 7) + (p >> 1);
      const int ra = rb + q, rbb = rb + 4 + q;
      const char* aa = region + ra * ROWB + ((chunk ^ swz4<16>(ra)) << 4) + (p & 1) * 8;
      const char* ab2 = region + rbb * ROWB + ((chunk ^ swz4<16>(rbb)) << 4) + (p & 1) * 8;
      const s16x4 a4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)aa);
      const s16x4 b4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s16x4*)ab2);
      s16x8 a8;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        a8[u] = a4[u];
        a8[4 + u] = b4[u];
      }
      return __builtin_bit_cast(bf16x8, a8);
    };
    if constexpr (FINAL) {
#pragma unroll
      for (int ct = 0; ct < TM; ++ct) {
        const bf16x8 af8 = tile_rd(ct);
#pragma unroll
        for (int t = 0; t < KT; ++t) accW[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af8, yfr[t], accW[ct][t], 0, 0, 0);
      }
    } else if constexpr (TM > 0) {
      // P3_PT tiles' reads in flight, pinned like step 1's ring (the
      // scheduler's own order kept one or two tiles ahead)
      constexpr int PT = P3_PT < TM ? P3_PT : TM;
      __builtin_amdgcn_sched_barrier(0);
      bf16x8 tfr[PT];
#pragma unroll
      for (int u = 0; u < PT; ++u) tfr[u] = tile_rd(u);
#pragma unroll
      for (int ct = 0; ct < TM; ++ct) {
        const bf16x8 af8 = tfr[ct % PT];
#pragma unroll
        for (int t = 0; t < KT; ++t) accW[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af8, yfr[t], accW[ct][t], 0, 0, 0);
        if (ct + PT < TM) tfr[ct % PT] = tile_rd(ct + PT);
      }
      __builtin_amdgcn_sched_group_barrier(0x100, 2 * PT, 1);
#pragma unroll
      for (int ct = 0; ct + PT < TM; ++ct) {
        __builtin_amdgcn_sched_group_barrier(0x008, KT, 1);
        __builtin_amdgcn_sched_group_barrier(0x100, 2, 1);
      }
      __builtin_amdgcn_sched_group_barrier(0x008, KT * PT, 1);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  // ---- prologue: NBUF - 1 blocks in flight, block 0 landed everywhere, y(0)
#pragma unroll
  for (int b = 0; b < NBUF - 1; ++b)
    if (b < nloc) issue(b);
  // block 0 landed: younger are the DMAs of blocks 1 and 2
  if (nloc > 0) wait_vm(lpb * ((1 < nloc) + (2 < nloc)));
  lds_barrier();
  if (nloc > 0) step1(0);

  for (int64_t j = 0; j < nloc; ++j) {
    // block j + 1 landed (own DMA), then the phase barrier: y(j) published,
    // every wave past step 3 of block j - 1 (its slot is free again).  Issue
    // order of a phase p: DMA(p + 3), then the Y stores of block p, so the
    // ops younger than DMA(j + 1) are DMA(j + 2) and the stores of phases
    // max(0, j - 2) .. j - 1
    if (j + 1 < nloc) wait_vm(lpb * (j + 2 < nloc) + nst * (int)(j < 2 ? j : 2));
    lds_barrier();
    gram_acc();
    if (j + NBUF - 1 < nloc) issue(j + NBUF - 1);
    if constexpr (FINAL && !YROLE) store_y(j);
    if (j + 1 < nloc) step1(j + 1);
    step3(j);
  }
  gram_acc();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // ---- W partial slab [n][k]: this wave's tiles
  {
    float* ws = Wslab + (int64_t)blockIdx.x * n * kr;
#pragma unroll
    for (int ct = 0; ct < TM; ++ct)
      if (ct < tcnt) {
        const int gt = tbase + ct;
#pragma unroll
        for (int t = 0; t < KT; ++t)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int row = 16 * gt + 4 * g4 + e, col = 16 * t + i16;
            if (row < n && col < kr) ws[(int64_t)row * kr + col] = accW[ct][t][e];
          }
      }
  }
  if constexpr (G_ON) {
    double* gs = Gslab + (int64_t)blockIdx.x * k * k;
#pragma unroll
    for (int sg = 0; sg < P5_GS; ++sg) {
      const int tau = gfirst + sg * gstride;
      if (gstride == 0 || tau >= GT) break;
      const int t1 = tau < KT ? 0 : (tau < 2 * KT - 1 ? 1 : 2);
      const int t2 = t1 == 0 ? tau : (t1 == 1 ? tau - KT + 1 : 2);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int i = 16 * t1 + 4 * g4 + r, jj = 16 * t2 + i16;
        if (i < k && jj < k && (t1 != t2 || i <= jj)) {
          gs[i * k + jj] = accG[sg][r];
          if (i != jj) gs[jj * k + i] = accG[sg][r];
        }
      }
    }
  }
}

template <int KT, bool FINAL, bool GRAM, int KS, int EXT = 0>
__global__ void __launch_bounds__(512, 1)
k_rsvd_pass5(const bf16_t* __restrict__ A, int64_t m, int n, int64_t lda, const bf16_t* __restrict__ Zt, int k,
             float* __restrict__ Wslab, double* __restrict__ Gslab, float* __restrict__ Y, int64_t ldy,
             float* __restrict__ scratch, P5Tiles pt) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (w < KT) {
    // the y waves carry each phase's critical path (step 1 of the next block)
    if (pt.prio == 1) __builtin_amdgcn_s_setprio(1);
    else if (pt.prio >= 2) __builtin_amdgcn_s_setprio(2);
    // the y waves' W-tile count is a compile-time constant of their body
    const int yt = pt.cnt[0];
    if (yt == 0)
      p5_body<KT, FINAL, GRAM, true, 0, KS, EXT>(A, m, n, lda, Zt, k, Wslab, Gslab, Y, ldy, scratch, pt, smem, w);
    else if (yt == 1)
      p5_body<KT, FINAL, GRAM, true, 1, KS, EXT>(A, m, n, lda, Zt, k, Wslab, Gslab, Y, ldy, scratch, pt, smem, w);
    else
      p5_body<KT, FINAL, GRAM, true, 2, KS, EXT>(A, m, n, lda, Zt, k, Wslab, Gslab, Y, ldy, scratch, pt, smem, w);
  } else {
    p5_body<KT, FINAL, GRAM, false, P5_T2, KS, EXT>(A, m, n, lda, Zt, k, Wslab, Gslab, Y, ldy, scratch, pt, smem, w);
  }
}

// W-tile / Gram-tile ownership for (n, KT): the y waves (0 .. KT-1) take T1 <=
// 2 W tiles each, the W waves the rest in order; T1 minimises the largest
// per-SIMD-pair (w, w + 4) matrix-core load.  Gram tiles round-robin over the
// W waves.  Returns false when the tiles do not fit the register budget.
bool p5_tiles(int n, int KT, P5Tiles* pt) {
  const int nt16 = (n + 15) / 16, nks = (n + 31) / 32, nw = 8 - KT;
  int best = 1 << 30, bestT1 = -1;
  for (int T1 = 0; T1 <= P5_T1; ++T1) {
    const int rem = nt16 - KT * T1;
    if (rem < 0) break;
    const int T2 = (rem + nw - 1) / nw;
    if (T2 > P5_T2) continue;
    int cnt[8];
    int left = rem;
    for (int w = 0; w < 8; ++w) {
      if (w < KT) { cnt[w] = T1; continue; }
      cnt[w] = left < T2 ? left : T2;
      left -= cnt[w];
    }
    int worst = 0;
    for (int w = 0; w < 4; ++w) {
      auto load = [&](int v) { return (v < KT ? nks : 0) + KT * cnt[v]; };
      worst = std::max(worst, load(w) + load(w + 4));
    }
    if (worst < best) { best = worst; bestT1 = T1; }
  }
  if (bestT1 < 0) return false;
  const int rem = nt16 - KT * bestT1, T2 = (rem + nw - 1) / nw;
  int left = rem, base = 0;
  for (int w = 0; w < 8; ++w) {
    const int c = w < KT ? bestT1 : (left < T2 ? left : T2);
    if (w >= KT) left -= c;
    pt->base[w] = base;
    pt->cnt[w] = c;
    base += c;
  }
  const int GT = KT * (KT + 1) / 2;
  for (int w = 0; w < 8; ++w) {
    const int wi = w - KT;
    const bool own = wi >= 0 && wi < GT;
    pt->gown[w] = own ? (wi | (nw << 8)) : 0;
    if (own && (GT - wi + nw - 1) / nw > P5_GS) return false;
  }
  return true;
}

template <int KT, bool FINAL, bool GRAM>
int launch_pass5(const bf16_t* A, int64_t m, int n, int64_t lda, const bf16_t* Zt, int k, float* Wslab, double* Gslab,
                 float* Y, int64_t ldy, float* scratch, int grid, hipStream_t s, int variant) {
  P5Tiles pt{};
  pt.prio = (variant >> 6) & 3;
  pt.rev = (variant >> 8) & 1;
  {
    const int c = (variant >> 9) & 7;
    pt.nt = c != 0;
    pt.ntail = c >= 2 ? 8 * (c - 1) : 0;
  }
  pt.nty = (variant >> 12) & 1;
  if (!p5_tiles(n, KT, &pt)) {
    sl_set_last_error("rsvd_pass: no tile split for this n / k");
    return SL_ERR_UNSUPPORTED;
  }
  constexpr int LDS = p5_lds<KT, FINAL>();
  static_assert(LDS <= 160 * 1024, "LDS budget");
  if (n > 512) {
    SL_LDS_ATTR((k_rsvd_pass5<KT, FINAL, GRAM, 32>), LDS);
    k_rsvd_pass5<KT, FINAL, GRAM, 32><<<grid, 512, LDS, s>>>(A, m, n, lda, Zt, k, Wslab, Gslab, Y, ldy, scratch, pt);
  } else {
    SL_LDS_ATTR((k_rsvd_pass5<KT, FINAL, GRAM, 16>), LDS);
    k_rsvd_pass5<KT, FINAL, GRAM, 16><<<grid, 512, LDS, s>>>(A, m, n, lda, Zt, k, Wslab, Gslab, Y, ldy, scratch, pt);
  }
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// EXT forms (fixed KT = 1, FINAL with Y, no Gram): see P5Tiles::kx
template <int EXT>
int launch_pass5_ext(const bf16_t* A, int64_t m, int n, int64_t lda, const bf16_t* Zt2, int kx, float* Wslab,
                     float* Y, int64_t ldy, const float* D, int64_t lddc, float* scratch, int grid, hipStream_t s,
                     int variant) {
  P5Tiles pt{};
  pt.prio = (variant >> 6) & 3;
  pt.rev = (variant >> 8) & 1;
  pt.kx = kx;
  pt.D = D;
  pt.lddc = lddc;
  if (!p5_tiles(n, 1, &pt)) {
    sl_set_last_error("rsvd_pass_ext: no tile split for this n");
    return SL_ERR_UNSUPPORTED;
  }
  constexpr int LDS = p5_lds<1, true, EXT>();
  static_assert(LDS <= 160 * 1024, "LDS budget");
  if (n > 512) {
    SL_LDS_ATTR((k_rsvd_pass5<1, true, false, 32, EXT>), LDS);
    k_rsvd_pass5<1, true, false, 32, EXT><<<grid, 512, LDS, s>>>(A, m, n, lda, Zt2, 2 * kx, Wslab, nullptr, Y, ldy,
                                                                 scratch, pt);
  } else {
    SL_LDS_ATTR((k_rsvd_pass5<1, true, false, 16, EXT>), LDS);
    k_rsvd_pass5<1, true, false, 16, EXT><<<grid, 512, LDS, s>>>(A, m, n, lda, Zt2, 2 * kx, Wslab, nullptr, Y, ldy,
                                                                 scratch, pt);
  }
  SL_LAUNCH_CHECK();
  return SL_OK;
}

int cu_count() {
  static int ncu = -1;
  if (ncu < 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      ncu = 256;
  }
  return ncu;
}

}  // namespace

// grid of the pass for m rows (one workgroup per CU, at most one per block)
SL_API int sl_rsvd_pass_grid(int64_t m) {
  const int64_t nb = (m + 15) / 16;
  const int64_t c = cu_count();
  return (int)(nb < c ? (nb > 0 ? nb : 1) : c);
}

// bytes of slab workspace the pass needs: W slabs [grid][n][k] f32 and
// (final) G slabs [grid][k][k] f64, plus a 1 KiB scratch line
SL_API int64_t sl_rsvd_pass_workspace(int64_t m, int64_t n, int k) {
  const int64_t g = sl_rsvd_pass_grid(m);
  int64_t b = g * n * k * 4;
  b = (b + 255) & ~(int64_t)255;
  b += g * (int64_t)k * k * 8;
  b = (b + 255) & ~(int64_t)255;
  return b + 1024;
}

// One fused pass.  A: m x n bf16 (lda % 8 == 0, 16 <= n <= 1024, n % 8 == 0);
// Zt: k x n bf16 (1 <= k <= 48).  ws: sl_rsvd_pass_workspace bytes.
// final = 0: W slabs only.  final = 1: also Y (m x k f32, row stride ldy >=
// k; Y = y_hi + y_lo, the bf16 pair W is formed from) and the fp64 Gram slabs
// of that Y (exact bf16 products, f32 per 16-row block, f64 across blocks);
// final = 2: W slabs and Y only.  variant bits: 256 = walk the row blocks
// last-to-first, 64/128 = y-wave priority (tuning), bits 9-11 the LDS-DMA
// cache policy (P5Tiles::nt).
SL_API int sl_rsvd_pass(const void* A, int64_t m, int64_t n, int64_t lda, const void* Zt, int k, void* ws,
                        float* Y, int64_t ldy, int final_pass, int variant, void* stream) {
  if (m <= 0) return SL_OK;
  if (n % 8 || lda % 8 || n > 1024 || n < 16 || k < 1 || k > 48 || (final_pass && (!Y || ldy < k))) {
    sl_set_last_error("rsvd_pass: needs n % 8 == 0, lda % 8 == 0, 16 <= n <= 1024, 1 <= k <= 48 (and Y when final)");
    return SL_ERR_UNSUPPORTED;
  }
  hipStream_t s = (hipStream_t)stream;
  const int grid = sl_rsvd_pass_grid(m);
  char* base = (char*)ws;
  float* Wslab = (float*)base;
  int64_t off = ((int64_t)grid * n * k * 4 + 255) & ~(int64_t)255;
  double* Gslab = (double*)(base + off);
  off += (int64_t)grid * k * k * 8;
  off = (off + 255) & ~(int64_t)255;
  float* scratch = (float*)(base + off);
  const bf16_t* a = (const bf16_t*)A;
  const bf16_t* z = (const bf16_t*)Zt;
  const int KT = (k + 15) / 16;
#define SL_P5(KTT)                                                                                                 \
  return final_pass == 1 ? launch_pass5<KTT, true, true>(a, m, (int)n, lda, z, k, Wslab, Gslab, Y, ldy, scratch, grid, s, variant) \
       : final_pass == 2 ? launch_pass5<KTT, true, false>(a, m, (int)n, lda, z, k, Wslab, Gslab, Y, ldy, scratch, grid, s, variant) \
                         : launch_pass5<KTT, false, false>(a, m, (int)n, lda, z, k, Wslab, Gslab, Y, ldy, scratch, grid, s, variant)
  switch (KT) {
    case 1: SL_P5(1);
    case 2: SL_P5(2);
    default: SL_P5(3);
  }
#undef SL_P5
}

// One-read normal products on the fused pass for a bf16 A with few columns
// of X (BlockADMM's {Z Wbar, Z^T d} and {o = Z W, Z^T o} on its bf16 feature
// cache): Zt2 = [X_hi^T; X_lo^T] (2 kx x n bf16, the hi / lo planes of the
// f32 X, kx <= 8), Y (m x kx f32, row stride ldy) = A X (products of the
// bf16 A with both planes, f32 sums), and the W slabs (reduced by
// sl_rsvd_reduce_z with k = kx) = A^T y (D null) or A^T D (D given:
// column-major m x kx f32, column stride lddc % 4 == 0, 16-B aligned, m % 16
// == 0), the long operand entering the matrix cores as bf16 hi + lo (~2^-17
// relative).  ws: sl_rsvd_pass_workspace(m, n, kx).
SL_API int sl_rsvd_pass_ext(const void* A, int64_t m, int64_t n, int64_t lda, const void* Zt2, int kx, void* ws,
                            float* Y, int64_t ldy, const float* D, int64_t lddc, int variant, void* stream) {
  if (m <= 0) return SL_OK;
  if (n % 8 || lda % 8 || n > 1024 || n < 16 || kx < 1 || kx > 8 || !Y || ldy < kx ||
      (D && (m % 16 || lddc % 4 || ((uintptr_t)D & 15) || lddc < m))) {
    sl_set_last_error("rsvd_pass_ext: needs n % 8 == 0, lda % 8 == 0, 16 <= n <= 1024, 1 <= kx <= 8, Y; "
                      "D: m % 16 == 0, lddc % 4 == 0, 16-B aligned");
    return SL_ERR_UNSUPPORTED;
  }
  const int grid = sl_rsvd_pass_grid(m);
  char* base = (char*)ws;
  int64_t off = ((int64_t)grid * n * kx * 4 + 255) & ~(int64_t)255;
  off += (int64_t)grid * kx * kx * 8;
  off = (off + 255) & ~(int64_t)255;
  float* scratch = (float*)(base + off);
  const bf16_t* a = (const bf16_t*)A;
  const bf16_t* z = (const bf16_t*)Zt2;
  hipStream_t s = (hipStream_t)stream;
  return D ? launch_pass5_ext<2>(a, m, (int)n, lda, z, kx, (float*)base, Y, ldy, D, lddc, scratch, grid, s, variant)
           : launch_pass5_ext<1>(a, m, (int)n, lda, z, kx, (float*)base, Y, ldy, nullptr, 0, scratch, grid, s, variant);
}

// Sum the pass slabs: W (n x k, into Wout with row stride ldw; f64 when
// w_f64) and, when Gout is given, the fp64 Gram (k x k, row stride ldg).
// as sl_rsvd_reduce, and zero_word (if given) is set to 0 by the same launch
// (the engine clears the call's status word here instead of a memset node)
SL_API int sl_rsvd_reduce_z(const void* ws, int64_t m, int64_t n, int k, void* Wout, int w_f64, int ldw,
                            double* Gout, int ldg, int* zero_word, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int grid = sl_rsvd_pass_grid(m);
  const char* base = (const char*)ws;
  const int64_t tw = n * k;
  const unsigned gw = (unsigned)((tw + 127) / 128);
  if (Gout && w_f64) {
    const int64_t off = ((int64_t)grid * n * k * 4 + 255) & ~(int64_t)255;
    const int64_t tg = (int64_t)k * k;
    const unsigned gg = (unsigned)((tg + 127) / 128);
    k_rsvd_reduce_wg<<<gw + gg, 512, 0, s>>>((const float*)base, tw, k, (double*)Wout, ldw,
                                              (const double*)(base + off), tg, Gout, ldg, grid, (int)gw, zero_word);
    SL_LAUNCH_CHECK();
    return SL_OK;
  }
  if (w_f64)
    k_rsvd_reduce<float, double><<<gw, 512, 0, s>>>((const float*)base, grid, tw, k, (double*)Wout, ldw, zero_word);
  else
    k_rsvd_reduce<float, float><<<gw, 512, 0, s>>>((const float*)base, grid, tw, k, (float*)Wout, ldw, zero_word);
  SL_LAUNCH_CHECK();
  if (Gout) {
    const int64_t off = ((int64_t)grid * n * k * 4 + 255) & ~(int64_t)255;
    const int64_t tg = (int64_t)k * k;
    k_rsvd_reduce<double, double><<<(unsigned)((tg + 127) / 128), 512, 0, s>>>((const double*)(base + off), grid, tg,
                                                                               k, Gout, ldg, nullptr);
    SL_LAUNCH_CHECK();
  }
  return SL_OK;
}

SL_API int sl_rsvd_reduce(const void* ws, int64_t m, int64_t n, int k, void* Wout, int w_f64, int ldw,
                          double* Gout, int ldg, void* stream) {
  return sl_rsvd_reduce_z(ws, m, n, k, Wout, w_f64, ldw, Gout, ldg, nullptr, stream);
}
