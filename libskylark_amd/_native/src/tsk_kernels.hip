// Tall-skinny streaming kernels for the randomized SVD / power iteration.
//
//   sl_tsk_fused_pass:  ONE read of A (m x n bf16, row-major) produces
//        Y = A Z            (m x k, optional store, f32)
//        W = A^T Y          (n x k, f32)
//        G = Y^T Y          (k x k, f32)
//   sl_tsk_matmul:      Y = A Z  (Z given as bf16 hi + lo split, f32 out)
//
// Reference hot loops these replace: the two El::Gemm calls per power
// iteration plus the QR Gram (nla/svd.hpp:71-149, base/Gemm.hpp:84-103).
//
// gfx950 design (one workgroup of 8 waves per CU, persistent):
//   * the n columns are split over the 8 waves (NW = 64 or 128 columns
//     each); a wave keeps its slice of Z (bf16 MFMA B-fragments) and its
//     slice of W (f32 accumulators) in registers for the whole kernel;
//   * row blocks of BM = 16 rows stream HBM -> LDS by LDS-DMA
//     (global_load_lds_dwordx4, 1 KiB per wave-instruction), double
//     buffered, each wave fetching only its own columns; the LDS image is
//     XOR-swizzled through the SOURCE address (chunk ^ row) so both reads
//     below are (nearly) conflict-free:
//       - step 1  y_w = A_w Z_w  : ds_read_b128 row fragments,
//                                  v_mfma_f32_16x16x32_bf16
//       - step 2  y = sum_w y_w  : partials through LDS (2 barriers)
//       - step 3  W_w += A_w^T y : ds_read_b64_tr_b16 transposed fragments
//                                  of the SAME LDS image, y as bf16 hi+lo,
//                                  v_mfma_f32_16x16x16_bf16 (2 per tile)
//       - step 4  G += y^T y     : hi*hi + hi*lo + lo*hi, tiles spread
//                                  over the waves; or (G64) the upper
//                                  16x16 tiles in f64 from the reduced f32
//                                  y with v_mfma_f64_16x16x4_f64 — the fp64
//                                  Gram CholeskyQR needs, hidden in the
//                                  pass instead of a second read of Y;
//   * raw s_barrier + counted vmcnt (no __syncthreads, which would drain
//     the DMA queue), all LDS in one dynamic array;
//   * per-workgroup W/G partial slabs, summed in f64 by a second kernel.
#include "sl_common.hpp"
#include <stdlib.h>
#include <type_traits>

namespace {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) short s16x4;
typedef __attribute__((ext_vector_type(8))) short s16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) double f64x4;
typedef __attribute__((address_space(3))) void lds_void;

constexpr int WAVES = 8;
constexpr int THREADS = WAVES * 64;
constexpr int BM = 16;
constexpr int NBUF_DEFAULT = 2;   // LDS-DMA ring depth (the randSVD engine uses rsvd_pass.hip)
int g_flags = 0;   // per-call mode bits (8: no Gram, 32: y_hi only, 128: reverse, 256: b128 Y rows)

// hardware round-to-nearest-even (v_cvt_pk_bf16_f32), NaN-preserving, branch-free
__device__ __forceinline__ short bf16_bits(float f) { return __builtin_bit_cast(short, (__bf16)f); }
__device__ __forceinline__ float bf16_val(short h) { return (float)__builtin_bit_cast(__bf16, h); }

// LDS-DMA of 16 B per lane into LDS[lds_base + lane*16], issued as inline asm
// so hipcc does not insert its own (draining) vmcnt(0) before later LDS
// reads; completion is tracked by the hand-counted s_waitcnt vmcnt(N).
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

template <int NW, int KT, int NBUF, int YFB = 1>
struct Geo {
  static constexpr int ROWB = NW * 2;                 // bytes per LDS row of a wave region
  static constexpr int NCH = NW / 8;                  // 16-B chunks per row
  static constexpr int REGION = BM * ROWB;            // bytes per wave per buffer
  static constexpr int LPB = REGION / 1024;           // glds instructions per block per wave
  static constexpr int KP = KT * 16;
  static constexpr int ABYTES = NBUF * WAVES * REGION;
  // column stride of the y partials (f32): 16 rows + 4 pad, so the b128
  // partial stores (8-lane groups, banks mod 32) and the reducer's b128 reads
  // hit distinct banks (stride 16: 4-way / 8-way)
  static constexpr int YPS = BM + 4;
  // reduced y: 16 rows per column, no pad; the 16-B row quads are XOR-
  // swizzled by column (yswz) instead, which makes the reduction's b128 stores
  // and the step-3/4 b128 fragment reads conflict-free under the gfx950 lane
  // grouping (b128 reads: 4 groups of 16 lanes {0-3,12-15,20-27}, ...; b128
  // writes: 8 groups of 8, banks mod 32 -- MI355X_MICROARCH.md LDS table),
  // where the old 16+4 stride left both 2-way conflicted
  static constexpr int YFS = BM;
  static constexpr int YP_BYTES = WAVES * YPS * KP * 4;
  static constexpr int YF_BYTES = YFB * YFS * KP * 4;   // YFB = 2: double-buffered (PIPE)
  static constexpr int LDS = ABYTES + YP_BYTES + YF_BYTES;
  static constexpr int GTILES = KT * KT;
  static constexpr int GS = (GTILES + WAVES - 1) / WAVES;  // G tiles per wave
  static constexpr int GT64 = KT * (KT + 1) / 2;            // upper tiles (f64 Gram)
  static constexpr int GS64 = (GT64 + WAVES - 1) / WAVES;
};

// LDS chunk swizzle of A row `row` (16-B chunks; slot = chunk ^ swz(row)).
// For 16 chunks per row the linear map row -> [0,2,4,..,14, 9,11,..,7]
// (found by exhaustive search over GF(2) maps) keeps every read of the pass
// conflict-free: the step-1 ds_read_b128 fragments, and the step-3
// ds_read_b64_tr_b16 tiles of both the K = 16 (rows 0-7 / 8-15 per half-wave)
// and the K = 32 (rows {0-3, 8-11} / {4-7, 12-15}) forms -- with plain
// row & 15 the transposed reads were 2-way conflicted.
// float offset of row quad q (rows 4q..4q+3) of column col in the reduced-y buffer
template <int YFS>
__device__ __forceinline__ int yidx(int col, int q) { return col * YFS + 4 * (q ^ ((col >> 1) & 3)); }

template <int NCH>
__device__ __forceinline__ int swz(int row) {
  if constexpr (NCH == 16) return ((row << 1) & 15) ^ (((row >> 3) & 1) * 9);
  else return row & (NCH - 1);
}

template <int NW, int KT, bool DO_W, bool DO_G, bool STORE_Y, bool ZSPLIT, int NBUF, bool HI_T = false,
          bool G64 = false, int X = 0>
__global__ void __launch_bounds__(THREADS, 1)
k_tsk_pass(const bf16_t* __restrict__ A, int64_t m, int n, int64_t lda,
           const bf16_t* __restrict__ Zt, int k,  // Zt: (ZSPLIT ? 2k : k) x n, row-major
           float* __restrict__ Wslab, float* __restrict__ Gslab,
           float* __restrict__ Y, int64_t ldy, int ab) {
  using GG = Geo<NW, KT, NBUF, 1>;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* abuf = smem;
  float* yp = (float*)(smem + GG::ABYTES);
  float* yf = (float*)(smem + GG::ABYTES + GG::YP_BYTES);

  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c0w = w * NW;
  const int64_t nblocks = (m + BM - 1) / BM;
  const int64_t b0 = blockIdx.x;
  const int64_t bstep = gridDim.x;

  // ---- Z fragments (B operand of step 1): lane holds Z[c0w+32ks+8(l>>4)+j][16t+(l&15)]
  bf16x8 zh[NW / 32][KT];
  bf16x8 zl[ZSPLIT ? NW / 32 : 1][ZSPLIT ? KT : 1];
#pragma unroll
  for (int ks = 0; ks < NW / 32; ++ks)
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      const int col = 16 * t + (lane & 15);
      const int kk = c0w + 32 * ks + 8 * (lane >> 4);
      bf16x8 v = {};
      if (col < k && kk + 8 <= n) v = *(const bf16x8*)(Zt + (int64_t)col * n + kk);
      zh[ks][t] = v;
      if constexpr (ZSPLIT) {
        bf16x8 u = {};
        if (col < k && kk + 8 <= n) u = *(const bf16x8*)(Zt + (int64_t)(col + k) * n + kk);
        zl[ks][t] = u;
      }
    }

  // Consume the Z registers here so hipcc's vmcnt wait for these loads sits
  // before the loop (otherwise it lands on the first MFMA of every
  // iteration and drains the LDS-DMA prefetch queue).
#pragma unroll
  for (int ks = 0; ks < NW / 32; ++ks)
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      asm volatile("" ::"v"(zh[ks][t]));
      if constexpr (ZSPLIT) asm volatile("" ::"v"(zl[ks][t]));
    }

  f32x4 accW[DO_W ? NW / 16 : 1][DO_W ? KT : 1];
  if constexpr (DO_W) {
#pragma unroll
    for (int a = 0; a < NW / 16; ++a)
#pragma unroll
      for (int t = 0; t < KT; ++t) accW[a][t] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  f32x4 accG[G64 ? 1 : GG::GS];
  f64x4 accG64[G64 ? GG::GS64 : 1];
  if constexpr (G64) {
#pragma unroll
    for (int s = 0; s < GG::GS64; ++s) accG64[s] = f64x4{0.0, 0.0, 0.0, 0.0};
  } else {
#pragma unroll
    for (int s = 0; s < GG::GS; ++s) accG[s] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  // ab & 128: walk the row blocks last-to-first.  Alternate passes over the
  // same A run in opposite directions, so a pass starts on the rows its
  // predecessor read last -- still resident in the 256 MB Infinity Cache --
  // instead of on rows long evicted from it.
  const bool rev = (ab & 128) != 0;
  auto phys = [&](int64_t blk) { return rev ? nblocks - 1 - blk : blk; };

  // ---- LDS-DMA of one row block (this wave's columns) into buffer `buf`
  auto issue = [&](int64_t blk, int buf) {
    char* region = abuf + (buf * WAVES + w) * GG::REGION;
    const int64_t r0 = phys(blk) * BM;
#pragma unroll
    for (int i = 0; i < GG::LPB; ++i) {
      const int byte = i * 1024 + lane * 16;
      const int row = byte / GG::ROWB;
      const int slot = (byte % GG::ROWB) / 16;
      const int chunk = slot ^ swz<GG::NCH>(row);
      int64_t grow = r0 + row;
      grow = grow < m ? grow : m - 1;
      int col = c0w + chunk * 8;
      col = col + 8 <= n ? col : n - 8;
      const bf16_t* src = A + grow * lda + col;
      const unsigned dst = __builtin_amdgcn_readfirstlane(
          (unsigned)(uintptr_t)(lds_void*)(region + i * 1024));
      glds16((const void*)src, dst);
    }
  };

  constexpr bool PIPE = false;
  constexpr int PD = NBUF - 1;
  static_assert(PD >= 1, "ring too shallow");
  constexpr int YFSZ = GG::YFS * GG::KP;   // floats per reduced-y buffer
#pragma unroll
  for (int p = 0; p < PD; ++p)
    if (b0 + p * bstep < nblocks) issue(b0 + p * bstep, p);

  // blocks this workgroup owns (one 64-bit division, outside the loop)
  const int64_t nloc = b0 < nblocks ? (nblocks - 1 - b0) / bstep + 1 : 0;
  const int64_t niter = nloc + (PIPE && nloc > 0 ? 1 : 0);
  int64_t my = 0;  // local iteration index
  for (; my < niter; ++my) {
    const int64_t blk = b0 + my * bstep;
    const bool have = my < nloc;   // false only on PIPE's drain iteration
    const int buf = (int)(my % NBUF);
    // X: the ring slots are private to the wave, so the next prefetch goes out
    // at the top of the iteration (into the slot this wave finished with in the
    // previous one) and PD blocks stay in flight throughout
    if constexpr ((X & 1) != 0 || PIPE) {
      if (have && blk + PD * bstep < nblocks) issue(blk + PD * bstep, (int)((my + PD) % NBUF));
    }
    const char* region = abuf + (buf * WAVES + w) * GG::REGION;
    float* yfc = PIPE ? yf + (my & 1) * YFSZ : yf;
    const int g4 = lane >> 4, i16 = lane & 15;
    if (have) {
    // blocks issued after this one and still possibly in flight
    const int64_t rem = nloc - 1 - my;
    const int younger = ((X & 1) || PIPE) ? (int)(rem < PD ? rem : PD) : (int)(rem < PD - 1 ? rem : PD - 1);
    if (younger >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * GG::LPB) : "memory");
    else if (younger == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * GG::LPB) : "memory");
    else if (younger == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(GG::LPB) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    // ---- step 1: partial y over this wave's columns
    f32x4 accY[KT];
#pragma unroll
    for (int t = 0; t < KT; ++t) accY[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < NW / 32; ++ks) {
      const int row = lane & 15;
      const int chunk = (lane >> 4) + 4 * ks;
      const int slot = chunk ^ swz<GG::NCH>(row);
      const bf16x8 af = *(const bf16x8*)(region + row * GG::ROWB + slot * 16);
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        accY[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, zh[ks][t], accY[t], 0, 0, 0);
        if constexpr (ZSPLIT) accY[t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, zl[ks][t], accY[t], 0, 0, 0);
      }
    }
    // ---- step 2: cross-wave reduction of y through LDS.  Partials are stored
    //      column-major ([wave][col][16 rows]) so that every access is b128:
    //      a lane's C fragment is 4 consecutive rows of one column.
    {
#pragma unroll
    for (int t = 0; t < KT; ++t)
      *(f32x4*)&yp[((w * GG::KP) + 16 * t + i16) * GG::YPS + 4 * g4] = accY[t];
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    {
      constexpr int CPW = GG::KP / WAVES;  // columns reduced per wave
      const int64_t r0 = phys(blk) * BM;
      const bool full = r0 + BM <= m;        // wave-uniform: only the last block is ragged
      if (lane < CPW * 4) {
        const int col = w * CPW + (lane >> 2), rg = lane & 3;
        f32x4 sum = *(const f32x4*)&yp[col * GG::YPS + 4 * rg];
#pragma unroll
        for (int v = 1; v < WAVES; ++v) sum += *(const f32x4*)&yp[(v * GG::KP + col) * GG::YPS + 4 * rg];
        if (!full) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (r0 + 4 * rg + j >= m) sum[j] = 0.f;
        }
        *(f32x4*)&yfc[yidx<GG::YFS>(col, rg)] = sum;
        if constexpr (STORE_Y) {
          if (col < k && !(ab & 256)) {
            float* yrow = Y + (r0 + 4 * rg) * ldy + col;
            if (full) {
#pragma unroll
              for (int j = 0; j < 4; ++j) yrow[j * ldy] = sum[j];
            } else {
#pragma unroll
              for (int j = 0; j < 4; ++j)
                if (r0 + 4 * rg + j < m) yrow[j * ldy] = sum[j];
            }
          }
        }
      }
    }
    if constexpr (!PIPE) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if constexpr (STORE_Y) {
        if (ab & 256) {
          // Y rows as 16-B pieces (k % 4 == 0, 16-B aligned rows): thread t of
          // the workgroup stores columns 4 (t % (k/4)) .. +3 of row t / (k/4),
          // gathered from the reduced, column-major y in LDS -- 160 b128
          // stores per 16 x 40 block instead of 640 scattered dword stores
          const int tq = k >> 2;
          const int t = w * 64 + lane;
          const int64_t r0 = phys(blk) * BM;
          if (t < BM * tq) {
            const int row = t / tq, c4 = 4 * (t - row * tq);
            if (r0 + row < m) {
              f32x4 v;
#pragma unroll
              for (int e = 0; e < 4; ++e) v[e] = yfc[yidx<GG::YFS>(c4 + e, row >> 2) + (row & 3)];
              *(f32x4*)(Y + (r0 + row) * ldy + c4) = v;
            }
          }
        }
      }
    }
    }
    }  // have

    // prefetch PD blocks ahead into the buffer this wave consumed last iteration
    if constexpr ((X & 1) == 0 && !PIPE) {
      if (blk + PD * bstep < nblocks) issue(blk + PD * bstep, (int)((my + PD) % NBUF));
    }

    // ---- steps 3/4 on block `my` (or, PIPE, on block my - 1)
    if (!PIPE || my > 0) {
    const char* s3region = PIPE ? abuf + ((int)((my - 1) % NBUF) * WAVES + w) * GG::REGION : region;
    const float* s3yf = PIPE ? yf + ((my - 1) & 1) * YFSZ : yf;
    // y fragments with rows 4(l>>4)+j of column 16t+(l&15) (K=16 MFMA layout), hi/lo
    const bool hi_only = (ab & 32) != 0;
    const bool need_g = DO_G;
    s16x4 yh[KT], yl[KT];
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      const f32x4 v = *(const f32x4*)&s3yf[yidx<GG::YFS>(16 * t + i16, g4)];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const short h = bf16_bits(v[j]);
        yh[t][j] = h;
        yl[t][j] = bf16_bits(v[j] - bf16_val(h));
      }
    }
    if (DO_W) {
      const int q = i16 >> 2, p = i16 & 3;
      // ---- step 3: one transposed LDS read per 16-column tile of A,
      //      W += A^T y_hi (+ A^T y_lo).
      const int row = 4 * g4 + q;
      // hi_only is wave-uniform: one branch selects a whole unrolled copy
      // (a macro, not a lambda: capturing the accumulator arrays by reference
      // makes hipcc demote them to scratch)
#define SL_STEP3(HI)                                                                                  \
  _Pragma("unroll") for (int ct = 0; ct < NW / 16; ++ct) {                                           \
    const int chunk = 2 * ct + (p >> 1);                                                             \
    const char* addr = s3region + row * GG::ROWB + (chunk ^ swz<GG::NCH>(row)) * 16 + (p & 1) * 8;    \
    const s16x4 af = __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4 __attribute__((address_space(3)))*)addr); \
    _Pragma("unroll") for (int t = 0; t < KT; ++t) {                                                 \
      accW[ct][t] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(af, yh[t], accW[ct][t], 0, 0, 0);     \
      if (!(HI)) accW[ct][t] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(af, yl[t], accW[ct][t], 0, 0, 0); \
    }                                                                                                \
  }
      if constexpr ((X & 2) != 0) {
        // one v_mfma_f32_16x16x32_bf16 per tile over K = [16 rows of y_hi ; the
        // same 16 rows of y_lo] (the K = 16 form runs at half rate on gfx950):
        // lane group g holds rows 8 (g & 1) .. +7 -- of y_hi for g < 2, of y_lo
        // for g >= 2 -- read directly (two transposed A reads and two y reads
        // per lane; lane swaps measured far slower).  Exact W at hi-only cost.
        const bool low = lane < 32;
        const int r8 = 8 * (g4 & 1);
        bf16x8 yb[KT];
#pragma unroll
        for (int t = 0; t < KT; ++t) {
          const f32x4 va = *(const f32x4*)&s3yf[yidx<GG::YFS>(16 * t + i16, r8 >> 2)];
          const f32x4 vb = *(const f32x4*)&s3yf[yidx<GG::YFS>(16 * t + i16, (r8 >> 2) + 1)];
          s16x8 e;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const short ha = bf16_bits(va[j]), hb = bf16_bits(vb[j]);
            e[j] = low ? ha : bf16_bits(va[j] - bf16_val(ha));
            e[4 + j] = low ? hb : bf16_bits(vb[j] - bf16_val(hb));
          }
          yb[t] = __builtin_bit_cast(bf16x8, e);
        }
#pragma unroll
        for (int ct = 0; ct < NW / 16; ++ct) {
          const int chunk = 2 * ct + (p >> 1);
          const int ra = r8 + q, rbb = r8 + 4 + q;
          const char* aa = s3region + ra * GG::ROWB + (chunk ^ swz<GG::NCH>(ra)) * 16 + (p & 1) * 8;
          const char* ab2 = s3region + rbb * GG::ROWB + (chunk ^ swz<GG::NCH>(rbb)) * 16 + (p & 1) * 8;
          const s16x4 a4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4 __attribute__((address_space(3)))*)aa);
          const s16x4 b4 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((s16x4 __attribute__((address_space(3)))*)ab2);
          s16x8 a8;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            a8[j] = a4[j];
            a8[4 + j] = b4[j];
          }
          const bf16x8 af8 = __builtin_bit_cast(bf16x8, a8);
#pragma unroll
          for (int t = 0; t < KT; ++t)
            accW[ct][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af8, yb[t], accW[ct][t], 0, 0, 0);
        }
      } else if constexpr (HI_T) {
        SL_STEP3(true)
      } else {
        SL_STEP3(hi_only)
      }
#undef SL_STEP3
    }
    if constexpr (G64) {
      // ---- step 4 (f64): upper tile tau = w + 8 s is (t1, t2), t1 <= t2;
      //      K step u pairs lane group kk with row 4 kk + u:
      //      A[i][kk] = y[4kk+u][16 t1 + i], B[kk][j] = y[4kk+u][16 t2 + j]
      //      (lane: i = j = l & 15, kk = l >> 4), so a lane needs exactly the
      //      row quad kk of its two columns: two b128 reads per tile, then
      //      four K=4 steps (the 16 rows are summed in a different order)
      if (need_g) {
        int tau = 0;
#pragma unroll
        for (int t1 = 0; t1 < KT; ++t1)
#pragma unroll
          for (int t2 = t1; t2 < KT; ++t2, ++tau) {
            if ((tau % WAVES) == w) {
              const int s = tau / WAVES;
              const f32x4 qa = *(const f32x4*)&s3yf[yidx<GG::YFS>(16 * t1 + i16, g4)];
              const f32x4 qb = *(const f32x4*)&s3yf[yidx<GG::YFS>(16 * t2 + i16, g4)];
#pragma unroll
              for (int u = 0; u < BM / 4; ++u)
                accG64[s] = __builtin_amdgcn_mfma_f64_16x16x4f64((double)qa[u], (double)qb[u], accG64[s], 0, 0, 0);
            }
          }
      }
    } else if (need_g) {
      // ---- step 4: G tiles tau = w + 8 s (t1 = tau / KT, t2 = tau % KT):
      //      hi*hi + hi*lo + lo*hi
      // tile indices are compile-time; only the owner test (wave-uniform) is runtime
#pragma unroll
      for (int tau = 0; tau < GG::GTILES; ++tau) {
        if ((tau % WAVES) == w) {
          const int s = tau / WAVES, t1 = tau / KT, t2 = tau % KT;
          accG[s] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(yh[t1], yh[t2], accG[s], 0, 0, 0);
          accG[s] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(yh[t1], yl[t2], accG[s], 0, 0, 0);
          accG[s] = __builtin_amdgcn_mfma_f32_16x16x16bf16_1k(yl[t1], yh[t2], accG[s], 0, 0, 0);
        }
      }
    }
    }  // steps 3/4
    if constexpr (PIPE) {
      if (have) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // ---- partial slabs: W rows = A columns, layout [WAVES*NW][KP]
  if constexpr (DO_W) {
    float* ws = Wslab + (int64_t)blockIdx.x * (WAVES * NW) * GG::KP;
#pragma unroll
    for (int ct = 0; ct < NW / 16; ++ct)
#pragma unroll
      for (int t = 0; t < KT; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j)
          ws[(c0w + 16 * ct + (lane >> 4) * 4 + j) * GG::KP + 16 * t + (lane & 15)] = accW[ct][t][j];
  }
  if constexpr (DO_G && G64) {
    // f64 slab [KP][KP]: each upper tile and its mirror (D row = l>>4 + 4 r, col = l & 15)
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
            const int i = 16 * t1 + (lane >> 4) + 4 * r, j = 16 * t2 + (lane & 15);
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
        for (int j = 0; j < 4; ++j)
          gs[(16 * t1 + (lane >> 4) * 4 + j) * GG::KP + 16 * t2 + (lane & 15)] = accG[s][j];
      }
    }
  }
}

}  // namespace

// out[i][j] = sum_s slab[s][i][j]  (i < rows, j < cols <= 64) accumulated in f64.
// A 1024-thread workgroup owns 64 consecutive output elements; its 16 waves
// split the slabs (wave g sums slabs g, g+16, ...), each lane of a wave on
// consecutive elements of a slab row (coalesced), 4 slabs in flight per lane;
// the 16 partials are combined through LDS.  Enough parallelism both for
// the n x k W slabs and for the k x k Gram slabs.
template <typename IT, typename OT>
__global__ void __launch_bounds__(1024)
k_slab_reduce_rows(const IT* __restrict__ slab, int nslab, int64_t slab_stride, int ld_in,
                   int cols, OT* __restrict__ out, int ld_out, int rows) {
  __shared__ double part[16][64];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int64_t t = (int64_t)blockIdx.x * 64 + lane;
  const bool ok = t < (int64_t)rows * cols;
  double acc = 0.0;
  if (ok) {
    const int64_t i = t / cols, j = t - i * cols;
    const IT* p = slab + i * ld_in + j;
    double a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    int b = g;
    for (; b + 48 < nslab; b += 64) {
      a0 += p[(int64_t)b * slab_stride];
      a1 += p[(int64_t)(b + 16) * slab_stride];
      a2 += p[(int64_t)(b + 32) * slab_stride];
      a3 += p[(int64_t)(b + 48) * slab_stride];
    }
    for (; b < nslab; b += 16) a0 += p[(int64_t)b * slab_stride];
    acc = (a0 + a1) + (a2 + a3);
  }
  part[g][lane] = acc;
  __syncthreads();
  if (g == 0 && ok) {
    double s = 0.0;
#pragma unroll
    for (int v = 0; v < 16; ++v) s += part[v][lane];
    const int64_t i = t / cols, j = t - i * cols;
    out[i * ld_out + j] = (OT)s;
  }
}

int sl_slab_reduce_launch_d2d(const double* slab, int nslab, int64_t slab_stride, int ld_in, int rows,
                              int cols, double* out, int ld_out, hipStream_t s);
int sl_slab_reduce_launch(const float* slab, int nslab, int64_t slab_stride, int ld_in, int rows,
                          int cols, float* out, int ld_out, hipStream_t s) {
  if (rows <= 0 || cols <= 0) return SL_OK;
  const unsigned grid = (unsigned)(((int64_t)rows * cols + 63) / 64);
  k_slab_reduce_rows<float, float><<<grid, 1024, 0, s>>>(slab, nslab, slab_stride, ld_in, cols, out, ld_out, rows);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

int sl_slab_reduce_launch_f64(const float* slab, int nslab, int64_t slab_stride, int ld_in, int rows,
                              int cols, double* out, int ld_out, hipStream_t s) {
  if (rows <= 0 || cols <= 0) return SL_OK;
  const unsigned grid = (unsigned)(((int64_t)rows * cols + 63) / 64);
  k_slab_reduce_rows<float, double><<<grid, 1024, 0, s>>>(slab, nslab, slab_stride, ld_in, cols, out, ld_out, rows);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

int sl_slab_reduce_launch_d2d(const double* slab, int nslab, int64_t slab_stride, int ld_in, int rows,
                              int cols, double* out, int ld_out, hipStream_t s) {
  if (rows <= 0 || cols <= 0) return SL_OK;
  const unsigned grid = (unsigned)(((int64_t)rows * cols + 63) / 64);
  k_slab_reduce_rows<double, double><<<grid, 1024, 0, s>>>(slab, nslab, slab_stride, ld_in, cols, out, ld_out, rows);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

namespace {

int grid_for(int64_t m) {
  static int ncu = -1;
  if (ncu < 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      ncu = 256;
  }
  int64_t nb = (m + BM - 1) / BM;
  return (int)(nb < ncu ? nb : ncu);
}

template <int NW, int KT, bool DO_W, bool DO_G, bool STORE_Y, bool ZSPLIT, int NBUF, bool HI_T, bool G64, int X>
int launch_x(const bf16_t* A, int64_t m, int n, int64_t lda, const bf16_t* Zt, int k, float* Wslab,
           float* Gslab, float* Y, int64_t ldy, hipStream_t s) {
  using GG = Geo<NW, KT, NBUF, 1>;
  auto kern = k_tsk_pass<NW, KT, DO_W, DO_G, STORE_Y, ZSPLIT, NBUF, HI_T, G64, X>;
  SL_LDS_ATTR(kern, GG::LDS);
  kern<<<grid_for(m), THREADS, GG::LDS, s>>>(A, m, n, lda, Zt, k, Wslab, Gslab, Y, ldy, g_flags);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// X bit 0: the prefetch goes out at the top of the iteration; bit 1: the
// exact step 3 as one K = 32 MFMA per tile over [y_hi | y_lo] (needs the W
// update, a non-split Z and a non-hi-only pass).  2-deep LDS-DMA ring.
template <int NW, int KT, bool DO_W, bool DO_G, bool STORE_Y, bool ZSPLIT, bool HI_T = false, bool G64 = false>
int launch_nb(const bf16_t* A, int64_t m, int n, int64_t lda, const bf16_t* Zt, int k, float* Wslab,
              float* Gslab, float* Y, int64_t ldy, hipStream_t s) {
  constexpr int X = (DO_W && !ZSPLIT && KT <= 3 && !HI_T) ? 3 : 1;
  return launch_x<NW, KT, DO_W, DO_G, STORE_Y, ZSPLIT, NBUF_DEFAULT, HI_T, G64, X>(A, m, n, lda, Zt, k, Wslab, Gslab,
                                                                                   Y, ldy, s);
}

}  // namespace

// workspace bytes needed by sl_tsk_fused_pass
SL_API int64_t sl_tsk_fused_workspace(int64_t m, int64_t n, int k) {
  const int KP = ((k + 15) / 16) * 16;
  const int NWP = n <= 512 ? 512 : 1024;
  const int64_t g = 256;  // upper bound on the grid
  return g * (int64_t)NWP * KP * 4 + g * (int64_t)KP * KP * 8 + 256;  // G slab sized for f64
}

// flags: bit0 (1) skip the Gram G (G left untouched), bit1 (2) W from y_hi only
// (bf16-rounded y: for intermediate power iterations, whose W is only
// orthonormalised), bit2 (4) G in f64 (G is a double*; exact products of the
// f32 y accumulated in f64 — needs Y stored, i.e. the final pass).
// bit5 (32) walks the row blocks last-to-first (same results up to the
// summation order of the per-workgroup slabs; alternating passes then start
// on rows still held in the Infinity Cache).
// Default 0 = exact-f32-equivalent W and G.
SL_API int sl_tsk_fused_pass(const void* A, int64_t m, int64_t n, int64_t lda, const void* Zt, int k,
                             float* W, float* G, float* Y, int64_t ldy, void* ws, int flags, void* stream) {
  if (m <= 0) return SL_OK;
  if (n % 8 || lda % 8 || n > 1024 || k > 64 || k < 1 || n < 8) {
    sl_set_last_error("tsk_fused_pass: needs n%8==0, lda%8==0, 8<=n<=1024, 1<=k<=64");
    return SL_ERR_UNSUPPORTED;
  }
  hipStream_t s = (hipStream_t)stream;
  const int KT = (k + 15) / 16;
  const int KP = KT * 16;
  const bool small = n <= 512;
  const int NWT = small ? 512 : 1024;
  const int g = grid_for(m);
  float* Wslab = (float*)ws;
  float* Gslab = Wslab + (int64_t)g * NWT * KP;
  int rc = SL_ERR_UNSUPPORTED;
  const bf16_t* a = (const bf16_t*)A;
  const bf16_t* z = (const bf16_t*)Zt;
  g_flags = ((flags & 1) ? 8 : 0) | ((flags & 2) ? 32 : 0) | ((flags & 32) ? 128 : 0) |
            ((Y && (k & 3) == 0 && (ldy & 3) == 0 && ((uintptr_t)Y & 15) == 0) ? 256 : 0);
  // intermediate power-iteration passes (no Gram, bf16 y): compile-time specialisation
  const bool inter = (flags & 3) == 3 && !Y;
  // final pass whose Gram is taken separately (fp64 Gram of the stored Y)
  const bool nog = (flags & 3) == 1;
  const bool g64 = (flags & 4) && !(flags & 3) && Y;
  if ((flags & 4) && !g64) {
    sl_set_last_error("tsk_fused_pass: the f64 Gram (flag 4) needs Y and flags & 3 == 0");
    return SL_ERR_UNSUPPORTED;
  }
#define SL_TSK(NW, KTT)                                                                              \
  rc = g64 ? launch_nb<NW, KTT, true, true, true, false, false, true>(a, m, (int)n, lda, z, k, Wslab, Gslab, Y, ldy, s) \
     : (Y && nog) ? launch_nb<NW, KTT, true, false, true, false>(a, m, (int)n, lda, z, k, Wslab, Gslab, Y, ldy, s) \
     : Y ? launch_nb<NW, KTT, true, true, true, false>(a, m, (int)n, lda, z, k, Wslab, Gslab, Y, ldy, s) \
     : inter ? launch_nb<NW, KTT, true, false, false, false, true>(a, m, (int)n, lda, z, k, Wslab, Gslab, Y, ldy, s) \
         : launch_nb<NW, KTT, true, true, false, false>(a, m, (int)n, lda, z, k, Wslab, Gslab, Y, ldy, s)
  if (small) {
    switch (KT) { case 1: SL_TSK(64, 1); break; case 2: SL_TSK(64, 2); break; case 3: SL_TSK(64, 3); break; default: SL_TSK(64, 4); }
  } else {
    switch (KT) { case 1: SL_TSK(128, 1); break; case 2: SL_TSK(128, 2); break; case 3: SL_TSK(128, 3); break; default: SL_TSK(128, 4); }
  }
#undef SL_TSK
  g_flags = 0;
  if (rc != SL_OK) return rc;
  // flags & 16: W is an f64 output (reduced straight from the f32 slabs; the
  // randSVD final pass writes it into its [W; G] buffer with no extra cast/cat)
  rc = (flags & 16) ? sl_slab_reduce_launch_f64(Wslab, g, (int64_t)NWT * KP, KP, (int)n, k, (double*)W, k, s)
                    : sl_slab_reduce_launch(Wslab, g, (int64_t)NWT * KP, KP, (int)n, k, W, k, s);
  if (rc != SL_OK || (flags & 1)) return rc;
  if (g64) return sl_slab_reduce_launch_d2d((const double*)Gslab, g, (int64_t)KP * KP, KP, k, k, (double*)G, k, s);
  return sl_slab_reduce_launch(Gslab, g, (int64_t)KP * KP, KP, k, k, G, k, s);
}

// Y = A Z with Z given as [Z_hi; Z_lo] (2k x n, bf16, "Zt" layout), f32 out.
SL_API int sl_tsk_matmul(const void* A, int64_t m, int64_t n, int64_t lda, const void* Zt, int k,
                         float* Y, int64_t ldy, int zsplit, void* stream) {
  if (m <= 0) return SL_OK;
  if (n % 8 || lda % 8 || n > 1024 || k > 64 || k < 1 || n < 8) {
    sl_set_last_error("tsk_matmul: needs n%8==0, lda%8==0, 8<=n<=1024, 1<=k<=64");
    return SL_ERR_UNSUPPORTED;
  }
  hipStream_t s = (hipStream_t)stream;
  const int KT = (k + 15) / 16;
  const bf16_t* a = (const bf16_t*)A;
  const bf16_t* z = (const bf16_t*)Zt;
  int rc = SL_ERR_UNSUPPORTED;
#define SL_MM(NW, KTT)                                                                                      \
  rc = zsplit ? launch_nb<NW, KTT, false, false, true, true>(a, m, (int)n, lda, z, k, nullptr, nullptr, Y, ldy, s) \
              : launch_nb<NW, KTT, false, false, true, false>(a, m, (int)n, lda, z, k, nullptr, nullptr, Y, ldy, s)
  if (n <= 512) {
    switch (KT) { case 1: SL_MM(64, 1); break; case 2: SL_MM(64, 2); break; case 3: SL_MM(64, 3); break; default: SL_MM(64, 4); }
  } else {
    switch (KT) { case 1: SL_MM(128, 1); break; case 2: SL_MM(128, 2); break; case 3: SL_MM(128, 3); break; default: SL_MM(128, 4); }
  }
#undef SL_MM
  return rc;
}
