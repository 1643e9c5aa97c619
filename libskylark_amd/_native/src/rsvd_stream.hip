// Hand-written tall-skinny products of the general-precision randomized SVD
// (rsvd_general.hip, f32 / f64 A, k <= 64; reference nla/svd.hpp:71-149 and
// :222-318 ApproximateSVD<float / double>, whose power iteration applies A
// and A^T to an n x k / m x k block and re-orthonormalises after each):
//
//   sl_ts_az     Y (m x k) = A (m x n) Z (n x k)          one streaming read of A
//   sl_ts_atq    W (n x k, f64) = A^T Q (Q m x k)         one streaming read of A,
//                                                         per-row-group slabs + f64 sum
//                                                         (f32, 16 < k <= 128: k_ts_atq_bs)
//   sl_ts_xm64   out (rows x k2, f32 / f64) = X (rows x k, f64) M (k x k2, f64)
//   sl_ts_gram64 G (k x k, f64) = X^T X (X rows x k, f64)
//   sl_ts_gram_w G = X^T X for 64 < k <= 128 (X f32 / f64)
//   sl_ts_small  C = op(A) op(B), k x k operands, one workgroup (f64)
//
// Both big products run at A's own precision on the matrix cores
// (v_mfma_f32_16x16x4_f32: exact f32 products in a k-ordered fmaf chain;
// v_mfma_f64_16x16x4_f64) -- the reference's precision.  For f32 with 16 < k <= 48,
// Y = A Z uses an exact three-plane bf16 split of A and Z instead (six
// 16x16x32 bf16 MFMAs per group, f32 accumulation, dropped terms below 2^-24
// |a| |z|): the same error bound, and the product took 1168 -> 1032 us on a
// 1e6 x 1000 operand (profiles/r6/az_bf16_split_ab.txt).  At k = 40 (three 16-column tiles) a pass over a 1e6 x 1000 f32 A
// is 2 x 0.96e11 FLOP, i.e. 0.62 ms per product at the f32 matrix peak against
// 0.67 ms of HBM for the 4 GB read: the kernels are built so neither the
// matrix pipe nor the memory system waits on the other (software-pipelined
// global loads straight into the MFMA operand registers, no LDS staging of A).
//
// MFMA operand trick shared by both: a 16x16x4 MFMA sums over 4 values of
// its K index held by lane groups l >> 4; WHICH columns (rows) of A those are
// is free as long as both operands agree.  So a lane loads 16 contiguous
// bytes of one row of A (VW = 4 f32 / 2 f64 consecutive elements) and feeds
// element s of that vector to the s-th MFMA of the group: global loads stay
// 16-B per lane and 64-256 B contiguous per row, with no transposition.
#include "sl_common.hpp"

#include <type_traits>

int sl_slab_reduce_launch_f64(const float* slab, int nslab, int64_t slab_stride, int ld_in, int rows, int cols,
                              double* out, int ld_out, hipStream_t s);
int sl_slab_reduce_launch_d2d(const double* slab, int nslab, int64_t slab_stride, int ld_in, int rows, int cols,
                              double* out, int ld_out, hipStream_t s);

namespace {

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) double f64x4;
typedef __attribute__((ext_vector_type(2))) double f64x2;
typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;

// Exact three-plane bf16 split of f32 values (H = rne(x), M = rne(x - H),
// L = rne(x - H - M); H + M + L == x for normal f32), two values per
// hardware conversion; the packed words (element 2u in the low half of u).
__device__ __forceinline__ uint32_t bf2(float lo, float hi) {
  typedef __attribute__((ext_vector_type(2))) __bf16 b2;
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((__attribute__((ext_vector_type(2))) float){lo, hi}, b2));
}
__device__ __forceinline__ void split_pair(float x0, float x1, uint32_t& h, uint32_t& m, uint32_t& l) {
  h = bf2(x0, x1);
  const float r0 = x0 - __uint_as_float(h << 16), r1 = x1 - __uint_as_float(h & 0xffff0000u);
  m = bf2(r0, r1);
  l = bf2(r0 - __uint_as_float(m << 16), r1 - __uint_as_float(m & 0xffff0000u));
}

template <typename T>
struct Mf;
template <>
struct Mf<float> {
  using acc = f32x4;
  using vec = f32x4;
  static constexpr int VW = 4;
  static __device__ __forceinline__ acc mfma(float a, float b, acc c) {
    return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
  }
  // row of accumulator element r in lane l (f32 16x16 C/D map)
  static __device__ __forceinline__ int drow(int l, int r) { return 4 * (l >> 4) + r; }
};
template <>
struct Mf<double> {
  using acc = f64x4;
  using vec = f64x2;
  static constexpr int VW = 2;
  static __device__ __forceinline__ acc mfma(double a, double b, acc c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
  }
  // the f64 MFMA's own C/D map (not the f32 one)
  static __device__ __forceinline__ int drow(int l, int r) { return (l >> 4) + 4 * r; }
};

// Global loads as inline asm (the compiler neither tracks nor waits for
// them): the A^T Q loop keeps a ring of loads in flight across its loop
// back-edge, where the compiler's own wait insertion fell back to draining
// every load each iteration.  The matching waits are explicit (wait_ring).
template <typename V>
__device__ __forceinline__ V ld16(const void* p) {
  V v;
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ float2 ld8(const void* p) {
  float2 v;
  asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ float ld_el(const float* p) {
  float v;
  asm volatile("global_load_dword %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ double ld_el(const double* p) {
  double v;
  asm volatile("global_load_dwordx2 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
  return v;
}

// ------------------------------------------------------------------ Y = A Z
// 256-thread workgroups (two per CU), persistent over 128-row blocks; wave w
// owns rows 32 w .. 32 w + 31 of the block (RT = 2 row tiles) and all KT
// column tiles of y.  The n columns stream in groups of GW = 4 EPL columns
// (EPL = VL VW: VL = 2 adjacent 16-B loads per lane and row tile, so the 4
// lanes of a row cover one whole 128-B line per group -- single 16-B pieces
// per group left every line to two half-line fetches a group apart), 4
// groups per chunk; the chunk's Z rows sit in LDS as ready-made B fragments
// ([group][tile][lane] x EPL, VL ds_read_b128 per tile and group),
// double-buffered: chunk c + 1 is loaded into registers while chunk c
// computes and stored after it, one barrier per chunk.  A is prefetched PD =
// 2 groups ahead in a register ring (slot g % 2, static in the unrolled body).
// Work split: R = nrb / g - 1 interleaved rounds of whole row blocks
// (workgroup b takes blocks b, b + g, ...: the blocks in flight at a time
// stay within a window of ~g blocks of A -- contiguous per-workgroup ranges
// over the whole operand ran the f32 product 14% slower), then the last g ..
// 2g - 1 blocks stream-K style: their (block, chunk) pairs cut into g equal
// contiguous ranges, so every workgroup streams the same number of chunks
// (whole blocks only left 2e5-row f64 operands at 4 vs 3.05 blocks per
// workgroup: a 30% tail).  A tail block cut by a range boundary is finished
// by two workgroups, each adding its partial y with an atomic add (the block
// is zeroed first by k_az_zero_cut; two addends onto zero sum the same in
// either order, so the result stays deterministic: every tail range spans
// at least one whole block, so no block has a third contributor).
constexpr int AZ_VL = 2, AZ_NG = 4, AZ_PD = 2, AZ_BR = 128;
// KT <= 4: 256 threads, each wave two 16-row tiles (two workgroups per CU);
// KT = 5..8 (64 < k <= 128): 512 threads, one row tile per wave (the
// accumulators of eight column tiles, one workgroup per CU: the Z chunk
// buffers take KT x 16 KB of LDS) -- the same 128-row blocks either way
template <int KT> constexpr int az_nt() { return KT > 4 ? 512 : 256; }
template <int KT> constexpr int az_rt() { return KT > 4 ? 1 : 2; }

// BS (f32 only): A and Z enter the matrix cores as exact three-plane bf16
// splits, six v_mfma_f32_16x16x32_bf16 per 32-column group and tile (H H, H M,
// M H, M M, H L, L H; the dropped M L / L M / L L terms are below 2^-24 of
// |a| |z|) instead of eight v_mfma_f32_16x16x4_f32: 96 instead of 256 matrix
// cycles per group.  Z's B fragments sit in LDS as the three planes (48 B per
// lane and tile instead of 32).
template <typename T, int KT, bool BS = false>
constexpr int az_lds() { return 2 * AZ_NG * KT * 64 * (BS ? 48 : 16 * AZ_VL); }

// whole-block interleaved rounds before the stream-K tail (the tail keeps
// g .. 2g - 1 blocks; g <= nrb)
__host__ __device__ inline int64_t az_rounds(int64_t nrb, int64_t g) { return nrb >= 2 * g ? nrb / g - 1 : 0; }

template <typename T, int KT, bool VEC, bool BS>
__global__ void __launch_bounds__(az_nt<KT>(), KT > 4 ? 1 : 2)
k_ts_az(const T* __restrict__ A, int64_t m, int n, int64_t lda, const T* __restrict__ Z, int k, T* __restrict__ Y,
        int64_t ldy, int split, int P, int stepB) {
  using M = Mf<T>;
  using vec = typename M::vec;
  using acc_t = typename M::acc;
  constexpr int AZ_NT = az_nt<KT>(), AZ_RT = az_rt<KT>(), RW = 16 * AZ_RT;   // RW rows per wave
  constexpr int VW = M::VW, EPL = AZ_VL * VW, GW = 4 * EPL, CW = AZ_NG * GW, KP = 16 * KT;
  // Z of a chunk is loaded as (column vector of VW, k index) pairs: VW
  // coalesced scalar loads per pair, one 16-B LDS store (scalar stores at the
  // fragment layout's 32-B stride were 8-way bank conflicts: 9e7 conflict
  // cycles per f32 k = 40 launch, in front of the chunk barrier)
  constexpr int CQ = CW / VW;                         // column vectors per chunk
  constexpr int ZQ = (CQ * KP + AZ_NT - 1) / AZ_NT;   // pairs per thread per chunk
  constexpr int ZE = ZQ * VW;                          // Z loads per thread per chunk
  extern __shared__ __attribute__((aligned(16))) char smem[];
  T* zl = (T*)smem;                                    // [2][NG][KT][64][EPL]
  static_assert(!BS || (sizeof(T) == 4 && KT <= 4), "bf16 split: f32, k <= 64");
  constexpr int BUFB = AZ_NG * KT * 64 * 48;           // BS: bytes per Z buffer
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  // Row-alignment classes.  With P > 1, A's row pitch (stepB = lda * sizeof(T)
  // mod 128, a multiple of 32) is not a whole number of 128-B lines, so the row
  // starts cycle through P offsets.  Wave w takes only rows of class
  // cl = w % P and shifts its column groups back by osh lane groups of 32 B,
  // so every 128-B piece it loads is one whole cache line.  Loading each
  // piece straddling two lines capped the f32 1e6 x 1000 product at
  // ~4.2 TB/s (profiles/r6/az_row_alignment.log).  Z's fragments are read
  // with the same shift; the lane groups shifted past a group's start take
  // the previous group's fragments, and past a chunk's start the previous
  // chunk's, which stays resident in the other LDS buffer.  The columns before
  // 0 of chunk 0 meet zeroed operands.
  const int lp = P == 4 ? 2 : P == 2 ? 1 : 0;
  const int cl = w & (P - 1);
  const int osh = ((cl * stepB) & 127) >> 5;
  int rowb[AZ_RT];   // block-relative row of lane & 15 in tile rt; store rows: rowb - P (lane & 15) + P drow
#pragma unroll
  for (int rt = 0; rt < AZ_RT; ++rt) rowb[rt] = P * (16 * ((w >> lp) * AZ_RT + rt) + (lane & 15)) + cl;
  const int nchunk = (n + (P > 1 ? 3 * EPL : 0) + CW - 1) / CW;
  const int64_t nrb = (m + AZ_BR - 1) / AZ_BR;
  const int64_t G = gridDim.x;
  // split 0 (A/B only): whole blocks round-robin, no tail
  const int64_t R = split ? az_rounds(nrb, G) : (int64_t)blockIdx.x < nrb ? (nrb - 1 - blockIdx.x) / G + 1 : 0;
  const int64_t tail = split ? (nrb - R * G) * nchunk : 0;   // flat (block, chunk) pairs of the tail
  const int64_t FR = R * nchunk;                     // this workgroup's round chunks
  const int64_t F0 = R * G * nchunk + tail * blockIdx.x / G;   // its tail range [F0, F0 + FT)
  const int64_t FT = R * G * nchunk + tail * (blockIdx.x + 1) / G - F0;
  const int64_t nfc = FR + FT;
  if (nfc <= 0) return;
  // (row block j, chunk c) of flat chunk f + 1 from that of f, clamped at
  // the last one (no divisions in the loop: hipcc's 64-bit division expands
  // into out-of-line blocks)
  const int64_t jt0 = F0 / nchunk;
  const int ct0 = (int)(F0 - jt0 * nchunk);
  auto advance = [&](int64_t f, int64_t& j, int& c) {
    if (f + 1 >= nfc) return;
    if (f + 1 == FR) {
      j = jt0;
      c = ct0;
    } else if (++c == nchunk) {
      c = 0;
      j += f + 1 < FR ? G : 1;
    }
  };

  // Every global load of the loop is inline asm (ld16 / ld_el) with explicit
  // waits: the ring crosses the chunk loop's back-edge, where the compiler's
  // own wait insertion kept only a few loads in flight.  Loads return in
  // issue order, so waiting for "at most N outstanding" with N = the loads
  // issued after the one needed is exact (stores in between only make it
  // stricter).  Issue order per chunk: Z of the next chunk (ZE loads, always
  // issued, clamped), then per group g its MFMAs and the refill of its slot
  // g % PD with group g + PD (the first PD groups of the next chunk for the
  // last PD groups).  When group g is used, the loads issued after its
  // refill are the next PD - 1 refills, plus the chunk's Z loads for g < PD.
  static_assert(AZ_NG == 2 * AZ_PD, "slot arithmetic");
  constexpr int LPG = AZ_RT * AZ_VL * (VEC ? 1 : VW);
  constexpr int RWA = (AZ_PD - 1) * LPG + ZE < 63 ? (AZ_PD - 1) * LPG + ZE : 63;   // g < PD
  constexpr int RWB = (AZ_PD - 1) * LPG < 63 ? (AZ_PD - 1) * LPG : 63;             // g >= PD
  constexpr int ZW = AZ_NG * LPG < 63 ? AZ_NG * LPG : 63;   // loads after a Z chunk's at its LDS store
  T zr[ZQ][VW];
  auto zload = [&](int c) {
#pragma unroll
    for (int u = 0; u < ZQ; ++u) {
      const int qd = tid + AZ_NT * u;
      const int cq = qd / KP, jj = qd - cq * KP;
#pragma unroll
      for (int s = 0; s < VW; ++s) {
        int col = c * CW + cq * VW + s;
        col = col < n ? col : n - 1;
        zr[u][s] = ld_el(Z + (int64_t)col * k + (jj < k ? jj : k - 1));
      }
    }
  };
  auto zstore = [&](int buf, int c) {
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(ZW) : "memory");
#pragma unroll
    for (int u = 0; u < ZQ; ++u)
#pragma unroll
      for (int s = 0; s < VW; ++s) asm volatile("" : "+v"(zr[u][s]));
    T* zb = zl + buf * (AZ_NG * KT * 64 * EPL);
#pragma unroll
    for (int u = 0; u < ZQ; ++u) {
      const int qd = tid + AZ_NT * u;
      if (qd < CQ * KP) {
        const int cq = qd / KP, jj = qd - cq * KP;
        const int cc = cq * VW, q = cc / GW, wq = cc - q * GW, kk = wq / EPL, s0 = wq - kk * EPL;
        const int t = jj >> 4, j16 = jj & 15;
        vec v;
#pragma unroll
        for (int s = 0; s < VW; ++s) v[s] = (c * CW + cc + s < n && jj < k) ? zr[u][s] : (T)0;
        if constexpr (BS) {
          // planes H / M / L of the slot at +0 / +16 / +32 B, elements s0 .. s0 + 3
          uint32_t h[2], md[2], l[2];
          split_pair(v[0], v[1], h[0], md[0], l[0]);
          split_pair(v[2], v[3], h[1], md[1], l[1]);
          char* p = smem + buf * BUFB + ((q * KT + t) * 64 + kk * 16 + j16) * 48 + 2 * s0;
          *(uint2*)p = make_uint2(h[0], h[1]);
          *(uint2*)(p + 16) = make_uint2(md[0], md[1]);
          *(uint2*)(p + 32) = make_uint2(l[0], l[1]);
        } else {
          *(vec*)(zb + ((q * KT + t) * 64 + kk * 16 + j16) * EPL + s0) = v;
        }
      }
    }
  };

  // A group loads: rows clamped to m - 1 (never stored), columns past n
  // clamped to a valid position (their Z rows are zero), a flat chunk past
  // the end re-reads the last one (never used)
  vec ring[AZ_PD][AZ_RT][AZ_VL];
  // (columns before 0 -- shifted lane groups of chunk 0 -- read the previous
  // row's tail, or A[0] for row 0; their operands are zeroed at use)
  auto issue = [&](int64_t j, int c, int g, int slot) {
    const int64_t rb = j * AZ_BR;
    const int col0 = c * CW + g * GW + EPL * ((lane >> 4) - osh);
#pragma unroll
    for (int rt = 0; rt < AZ_RT; ++rt) {
      int64_t row = rb + rowb[rt];
      row = row < m ? row : m - 1;
      const int64_t base = row * lda;
#pragma unroll
      for (int vl = 0; vl < AZ_VL; ++vl) {
        const int col = col0 + VW * vl;
        if constexpr (VEC) {
          int64_t off = base + (col < n ? col : n - VW);
          off = off < 0 ? 0 : off;
          ring[slot][rt][vl] = ld16<vec>(A + off);
        } else {
          vec v;
#pragma unroll
          for (int e = 0; e < VW; ++e) {
            int64_t off = base + (col + e < n ? col + e : n - 1);
            off = off < 0 ? 0 : off;
            v[e] = ld_el(A + off);
          }
          ring[slot][rt][vl] = v;
        }
      }
    }
  };
  auto wait_slot = [&](int g) {
    const int slot = g % AZ_PD;
    if (g < AZ_PD) asm volatile("s_waitcnt vmcnt(%1)" : "+v"(ring[slot][0][0]) : "n"(RWA));
    else asm volatile("s_waitcnt vmcnt(%1)" : "+v"(ring[slot][0][0]) : "n"(RWB));
#pragma unroll
    for (int rt = 0; rt < AZ_RT; ++rt)
#pragma unroll
      for (int vl = 0; vl < AZ_VL; ++vl)
        if (rt + vl > 0) asm volatile("" : "+v"(ring[slot][rt][vl]));
  };

  acc_t acc[AZ_RT][KT];
#pragma unroll
  for (int rt = 0; rt < AZ_RT; ++rt)
#pragma unroll
    for (int t = 0; t < KT; ++t) acc[rt][t] = acc_t{};

  // prologue: chunk 0 of Z in buffer 0, groups 0 .. PD - 1 of flat chunk 0
  // in flight (issued before the chunk loop's first Z loads, as the
  // previous chunk's refills would be)
  int64_t jb = FR > 0 ? (int64_t)blockIdx.x : jt0;   // flat chunk fc
  int c = FR > 0 ? 0 : ct0;
  int64_t jn = jb;                                     // flat chunk fc + 1
  int cn = c;
  advance(0, jn, cn);
  const int c0 = c;
  zload(c0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  zstore(0, c0);
  if (P > 1 && c0 > 0 && nchunk > 1) {   // a range starting inside a block: chunk c0 - 1 for the shift
    zload(c0 - 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    zstore(1, c0 - 1);
  }
#pragma unroll
  for (int g = 0; g < AZ_PD; ++g) issue(jb, c, g, g);
  __syncthreads();

  // this lane's Z fragments: lane group (lane >> 4) - osh of the same group,
  // or (when negative) + 4 of the previous group
  const int kd = (lane >> 4) - osh;
  const bool zprev = kd < 0;
  const int lsrc = ((kd + 4) & 3) * 16 + (lane & 15);
  for (int64_t fc = 0; fc < nfc; ++fc) {
    const int buf = nchunk > 1 ? (int)(fc & 1) : 0;   // one chunk: Z never reloads
    zload(cn);   // always issued: the wait arithmetic counts it
    const T* zb = zl + buf * (AZ_NG * KT * 64 * EPL);
    // fragment group of this lane for group g: -1 = the previous chunk's last
    auto zgrp = [&](int g) { return zprev ? g - 1 : g; };
#pragma unroll
    for (int g = 0; g < AZ_NG; ++g) {
      wait_slot(g);
      const int slot = g % AZ_PD;
      // chunk 0's shifted lane groups of group 0 sit before column 0
      const bool zero = g == 0 && zprev && c == 0;
      if (g == 0 && c == 0 && osh > 0) {
#pragma unroll
        for (int rt = 0; rt < AZ_RT; ++rt)
#pragma unroll
          for (int vl = 0; vl < AZ_VL; ++vl) ring[slot][rt][vl] = zero ? vec{} : ring[slot][rt][vl];
      }
      const int gs = zgrp(g);
      const int zbuf = gs < 0 ? buf ^ 1 : buf;
      const int zg = gs < 0 ? AZ_NG - 1 : gs;
      if constexpr (BS) {
        // the lane's 8 columns (both 16-B pieces) are the K index of one
        // 16x16x32 MFMA; the slot's planes hold the same 8 columns of Z
        const char* zs = smem + zbuf * BUFB;
        bf16x8 zp[3][KT];
#pragma unroll
        for (int t = 0; t < KT; ++t)
#pragma unroll
          for (int pl = 0; pl < 3; ++pl) {
            bf16x8 v = *(const bf16x8*)(zs + ((zg * KT + t) * 64 + lsrc) * 48 + 16 * pl);
            asm volatile("" : "+v"(v));
            zp[pl][t] = zero ? bf16x8{} : v;
          }
#pragma unroll
        for (int rt = 0; rt < AZ_RT; ++rt) {
          uint32_t h[4], md[4], l[4];
#pragma unroll
          for (int u = 0; u < 4; ++u)
            split_pair(ring[slot][rt][u >> 1][2 * (u & 1)], ring[slot][rt][u >> 1][2 * (u & 1) + 1], h[u], md[u], l[u]);
          const bf16x8 ah = __builtin_bit_cast(bf16x8, make_uint4(h[0], h[1], h[2], h[3]));
          const bf16x8 am = __builtin_bit_cast(bf16x8, make_uint4(md[0], md[1], md[2], md[3]));
          const bf16x8 al = __builtin_bit_cast(bf16x8, make_uint4(l[0], l[1], l[2], l[3]));
#pragma unroll
          for (int t = 0; t < KT; ++t) {
            acc_t a = acc[rt][t];
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, zp[0][t], a, 0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, zp[2][t], a, 0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, zp[1][t], a, 0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, zp[0][t], a, 0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, zp[1][t], a, 0, 0, 0);
            acc[rt][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, zp[0][t], a, 0, 0, 0);
          }
        }
      } else {
#pragma unroll
        for (int vl = 0; vl < AZ_VL; ++vl) {
          vec zv[KT];
          const T* zsb = zl + zbuf * (AZ_NG * KT * 64 * EPL);
#pragma unroll
          for (int t = 0; t < KT; ++t) {
            vec v = *(const vec*)(zsb + ((zg * KT + t) * 64 + lsrc) * EPL + VW * vl);
            asm volatile("" : "+v"(v));
            zv[t] = zero ? vec{} : v;
          }
#pragma unroll
          for (int s = 0; s < VW; ++s)
#pragma unroll
            for (int rt = 0; rt < AZ_RT; ++rt)
#pragma unroll
              for (int t = 0; t < KT; ++t) acc[rt][t] = M::mfma(ring[slot][rt][vl][s], zv[t][s], acc[rt][t]);
        }
      }
      // refill this slot with group g + PD (of the next flat chunk past the end)
      __builtin_amdgcn_sched_barrier(0);
      if (g + AZ_PD < AZ_NG) issue(jb, c, g + AZ_PD, slot);
      else issue(jn, cn, g + AZ_PD - AZ_NG, slot);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (c == nchunk - 1 || fc == nfc - 1) {
      // this workgroup's part of the row block is complete: y out (added
      // atomically into a block cut by a range boundary), accumulators cleared
      const bool cut = fc >= FR && (jb * nchunk < F0 || (jb + 1) * nchunk > F0 + FT);
      const int64_t rb = jb * AZ_BR;
#pragma unroll
      for (int rt = 0; rt < AZ_RT; ++rt)
#pragma unroll
        for (int t = 0; t < KT; ++t) {
          const int col = 16 * t + (lane & 15);
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int64_t row = rb + rowb[rt] + P * (M::drow(lane, r) - (lane & 15));
            if (row < m && col < k) {
              if (cut) atomicAdd(Y + row * ldy + col, acc[rt][t][r]);
              else Y[row * ldy + col] = acc[rt][t][r];
            }
          }
          acc[rt][t] = acc_t{};
        }
    }
    zstore(buf ^ 1, cn);   // (one chunk: a scratch copy into the unused buffer)
    __syncthreads();
    if (P > 1 && fc + 1 == FR && cn > 0 && nchunk > 1) {
      // entering the stream-K range inside a block: its chunk cn - 1 into the
      // buffer just consumed (the next chunk's "previous"); once per workgroup
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      zload(cn - 1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      zstore(buf, cn - 1);
      __syncthreads();
    }
    jb = jn;
    c = cn;
    advance(fc + 1, jn, cn);
  }
  // the clamped refills past the end: landed, and kept live until then (an
  // asm load's register the compiler thinks dead could be reused in flight)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
  for (int g = 0; g < AZ_PD; ++g)
#pragma unroll
    for (int rt = 0; rt < AZ_RT; ++rt)
#pragma unroll
      for (int vl = 0; vl < AZ_VL; ++vl) asm volatile("" : "+v"(ring[g][rt][vl]));
}

// zero the row blocks of y that a range boundary of k_ts_az cuts (one
// workgroup per boundary b = 1 .. grid - 1)
template <typename T>
__global__ void __launch_bounds__(256)
k_az_zero_cut(T* __restrict__ Y, int64_t m, int k, int64_t ldy, int64_t nrb, int nchunk, int grid) {
  const int64_t R = az_rounds(nrb, grid);
  const int64_t tail = (nrb - R * grid) * nchunk;
  const int64_t F = R * grid * nchunk + tail * (blockIdx.x + 1) / grid;
  if (F % nchunk == 0) return;
  const int64_t r0 = F / nchunk * AZ_BR;
  for (int e = threadIdx.x; e < AZ_BR * k; e += 256) {
    const int64_t row = r0 + e / k;
    if (row < m) Y[row * ldy + e % k] = (T)0;
  }
}

// ---------------------------------------------------------------- W = A^T Q
// 512-thread workgroups: blockIdx.x = a column slice of CS = 8 x V x 16 VW
// columns (wave w: V vectors of 16 lanes x VW columns per row), blockIdx.y =
// a row group.  Per row quad the lane (kk = l >> 4, nn = l & 15) loads row
// r + kk, columns cb + VW nn .. + VW - 1 of each vector: element e of vector
// v is the A^T operand of W tile (v, e), whose 16 rows are the columns
// cb + VW nn + e (stride VW) -- so the loads are plain row segments and the
// W tiles come out column-interleaved (undone at the slab store).  Q's B
// fragments (Q[r + kk][16 t + nn]) load straight from global (the 8 waves of
// a workgroup read the same rows: L1 / L2 hits).  W accumulates over the
// whole row group in registers (A's precision), then one slab per row group.
// AV = vectors per wave and row: 2 (default: one workgroup per CU, > 128
// VGPRs) or 1 (half the columns per wave, two workgroups per CU; A/B knob)
constexpr int AT_NT = 512;
int g_atq_av = 2;
// ring depth: 8 row quads in flight, 4 at KT = 4 (register budget)
template <int KT, int AV>
constexpr int at_pd() { return AV == 1 ? (KT >= 4 ? 4 : 6) : (KT >= 4 ? 4 : 8); }

template <typename T, int KT, bool VEC, int AV>
__global__ void __launch_bounds__(AT_NT, AV == 1 && KT <= 4 ? 2 : 1)
k_ts_atq(const T* __restrict__ A, int64_t m, int n, int64_t lda, const T* __restrict__ Q, int k, int64_t rows_per,
         T* __restrict__ slab) {
  using M = Mf<T>;
  using vec = typename M::vec;
  using acc_t = typename M::acc;
  constexpr int VW = M::VW, WC = AV * 16 * VW, CS = 8 * WC, PD = at_pd<KT, AV>();
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kk = lane >> 4, nn = lane & 15;
  const int64_t rbeg = (int64_t)blockIdx.y * rows_per;
  int64_t rend = rbeg + rows_per;
  rend = rend < m ? rend : m;
  const int cbw = blockIdx.x * CS + w * WC;   // this wave's first column
  // waves of the last slice past n idle (wave-uniform)
  const int64_t nq = (rend > rbeg && cbw < n) ? (rend - rbeg + 3) / 4 : 0;

  acc_t acc[AV][VW][KT];
#pragma unroll
  for (int v = 0; v < AV; ++v)
#pragma unroll
    for (int e = 0; e < VW; ++e)
#pragma unroll
      for (int t = 0; t < KT; ++t) acc[v][e][t] = acc_t{};

  // loads branch-free (see k_ts_az): rows clamped into the group, columns
  // into [0, n); the Q fragment of a row past the group (or a k column past
  // k) is zeroed at USE time from a mask formed at issue time, so nothing
  // touches a loaded value before its turn in the MFMA stream
  vec ra[PD][AV];
  T rq[PD][KT];
  bool rok[PD];
  auto issue = [&](int64_t qi, int slot) {
    int64_t row = rbeg + 4 * qi + kk;
    rok[slot] = row < rend;
    row = row < rend ? row : rend - 1;
    const T* src = A + row * lda;
#pragma unroll
    for (int v = 0; v < AV; ++v) {
      const int col = cbw + v * 16 * VW + VW * nn;
      if constexpr (VEC) {
        ra[slot][v] = ld16<vec>(src + (col < n ? col : n - VW));
      } else {
        vec x;
#pragma unroll
        for (int e = 0; e < VW; ++e) x[e] = ld_el(src + (col + e < n ? col + e : n - 1));
        ra[slot][v] = x;
      }
    }
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      const int col = 16 * t + nn;
      rq[slot][t] = ld_el(Q + row * k + (col < k ? col : k - 1));
    }
  };
  // loads per slot; slot p is waited for with the PD - 1 later slots in flight
  constexpr int LPS = AV * (VEC ? 1 : VW) + KT;
  // (waiting for at most 63 when more are in flight is stricter, still exact-safe)
  constexpr int INFLIGHT = (PD - 1) * LPS < 63 ? (PD - 1) * LPS : 63;
  auto wait_ring = [&](int p) {
    asm volatile("s_waitcnt vmcnt(%1)" : "+v"(ra[p][0]) : "n"(INFLIGHT));
#pragma unroll
    for (int v = 1; v < AV; ++v) asm volatile("" : "+v"(ra[p][v]));
#pragma unroll
    for (int t = 0; t < KT; ++t) asm volatile("" : "+v"(rq[p][t]));
  };

  if (nq > 0) {
#pragma unroll
    for (int p = 0; p < PD; ++p) issue(p, p);
    for (int64_t q0 = 0; q0 < nq; q0 += PD) {
#pragma unroll
      for (int p = 0; p < PD; ++p) {
        wait_ring(p);
        // a quad past nq has rok false in every lane: its Q operand is zero
        T b[KT];
#pragma unroll
        for (int t = 0; t < KT; ++t) b[t] = (rok[p] && 16 * t + nn < k) ? rq[p][t] : (T)0;
#pragma unroll
        for (int v = 0; v < AV; ++v)
#pragma unroll
          for (int e = 0; e < VW; ++e)
#pragma unroll
            for (int t = 0; t < KT; ++t) acc[v][e][t] = M::mfma(ra[p][v][e], b[t], acc[v][e][t]);
        // slot p's MFMAs, then its refill (scheduling barriers keep the
        // order the vmcnt arithmetic assumes)
        __builtin_amdgcn_sched_barrier(0);
        issue(q0 + p + PD, p);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // the clamped refills past the end: landed, and kept live until then
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int p = 0; p < PD; ++p) {
#pragma unroll
      for (int v = 0; v < AV; ++v) asm volatile("" : "+v"(ra[p][v]));
#pragma unroll
      for (int t = 0; t < KT; ++t) asm volatile("" : "+v"(rq[p][t]));
    }
  }
  if (cbw >= n) return;
  // slab (row group y) [n][k]: tile (v, e) row i is column cbw + v 16 VW + VW i + e
  T* sb = slab + (int64_t)blockIdx.y * n * k;
#pragma unroll
  for (int v = 0; v < AV; ++v)
#pragma unroll
    for (int e = 0; e < VW; ++e)
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        const int kc = 16 * t + nn;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int i = M::drow(lane, r);
          const int col = cbw + v * 16 * VW + VW * i + e;
          if (col < n && kc < k) sb[(int64_t)col * k + kc] = acc[v][e][t][r];
        }
      }
}

// ----------------------------------------------- W = A^T Q, f32 on bf16 splits
// 512-thread workgroups as k_ts_atq; wave w owns 64 columns of the slice (16
// lanes x 4) and all rows of the row group.  Per 32-row step the lane (kk =
// l >> 4, nn = l & 15) loads rows r + 8 kk + j (j < 8), columns cbw + 4 nn ..
// + 3: element e of those 8 rows is the K = 32 A^T operand of W tile e, whose
// 16 rows are the columns cbw + 4 i + e; the Q operand is Q[r + 8 kk + j][16 t
// + nn].  Both enter the matrix cores as exact three-plane bf16 splits, six
// v_mfma_f32_16x16x32_bf16 per tile pair (the split form of k_ts_az), instead
// of eight v_mfma_f32_16x16x4_f32 per 32 rows: the f32 product at k = 40 was
// bound by the f32 matrix rate (profiles/r6/atq_bf16_split_ab.txt).
constexpr int ATB_PD = 2;

// EW = 4 columns per lane and row (k <= 64); EW = 2 for 64 < k <= 128 (six /
// eight Q tiles: the accumulators of four A tiles would not fit), 32-column
// windows, 8-B loads.
template <int KT, int EW = 4>
__global__ void __launch_bounds__(AT_NT, 1)
k_ts_atq_bs(const float* __restrict__ A, int64_t m, int n, int64_t lda, const float* __restrict__ Q, int k,
            int64_t rows_per, float* __restrict__ slab) {
  static_assert(EW == 4 || EW == 2, "EW");
  using ev = typename std::conditional<EW == 4, f32x4, float2>::type;
  constexpr int WC = 16 * EW, CS = 8 * WC;
  const int tid = threadIdx.x, lane = tid & 63, w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int kk = lane >> 4, nn = lane & 15;
  const int64_t rbeg = (int64_t)blockIdx.y * rows_per;
  int64_t rend = rbeg + rows_per;
  rend = rend < m ? rend : m;
  const int cbw = blockIdx.x * CS + w * WC;
  // every wave runs every step (the per-step barrier); waves past n discard
  const int64_t nq = rend > rbeg ? (rend - rbeg + 31) / 32 : 0;
  // Q's split is shared: per step each thread splits KT of the 32 x 16 KT Q
  // elements into the LDS B fragments [buf][plane][tile][lane][row] (the 8
  // waves all need the same ones; split in every wave, the kernel was
  // VALU-bound, profiles/r6/atq_pmc.txt)
  __shared__ __attribute__((aligned(16))) uint16_t qs[2][3][KT][64][8];
  f32x4 acc[EW][KT];
#pragma unroll
  for (int e = 0; e < EW; ++e)
#pragma unroll
    for (int t = 0; t < KT; ++t) acc[e][t] = f32x4{};
  // loads branch-free: rows clamped into the group (their Q operand zeroed at
  // use from the mask formed at issue), columns clamped into [0, n)
  ev ra[ATB_PD][8];
  float rq[ATB_PD][KT];
  int rok[ATB_PD];
  const int col = cbw + EW * nn;
  const int cc = col < n ? col : n - EW;
  auto issue = [&](int64_t qi, int slot) {
    const int64_t r0 = rbeg + 32 * qi + 8 * kk;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      int64_t row = r0 + j;
      row = row < rend ? row : rend - 1;
      if constexpr (EW == 4) ra[slot][j] = ld16<f32x4>(A + row * lda + cc);
      else ra[slot][j] = ld8(A + row * lda + cc);
    }
    int ok = 0;
#pragma unroll
    for (int u = 0; u < KT; ++u) {
      const int e = tid + AT_NT * u, qr = e / (16 * KT), qc = e - qr * (16 * KT);
      int64_t row = rbeg + 32 * qi + qr;
      ok |= (row < rend && qc < k ? 1 : 0) << u;
      row = row < rend ? row : rend - 1;
      rq[slot][u] = ld_el(Q + row * k + (qc < k ? qc : k - 1));
    }
    rok[slot] = ok;
  };
  constexpr int LPS = 8 + KT;
  constexpr int INFLIGHT = (ATB_PD - 1) * LPS < 63 ? (ATB_PD - 1) * LPS : 63;
  auto wait_ring = [&](int p) {
    asm volatile("s_waitcnt vmcnt(%1)" : "+v"(ra[p][0]) : "n"(INFLIGHT));
#pragma unroll
    for (int j = 1; j < 8; ++j) asm volatile("" : "+v"(ra[p][j]));
#pragma unroll
    for (int u = 0; u < KT; ++u) asm volatile("" : "+v"(rq[p][u]));
  };
  if (nq > 0) {
#pragma unroll
    for (int p = 0; p < ATB_PD; ++p) issue(p, p);
    for (int64_t q0 = 0; q0 < nq; q0 += ATB_PD) {
#pragma unroll
      for (int p = 0; p < ATB_PD; ++p) {
        wait_ring(p);
        const int b = p & 1;   // LDS buffer of this step (ATB_PD even: steps alternate)
#pragma unroll
        for (int u = 0; u < KT; ++u) {
          const int e = tid + AT_NT * u, qr = e / (16 * KT), qc = e - qr * (16 * KT);
          const float v = ((rok[p] >> u) & 1) ? rq[p][u] : 0.f;
          uint32_t h, md, l;
          split_pair(v, 0.f, h, md, l);
          uint16_t* d = &qs[b][0][qc >> 4][(qr >> 3) * 16 + (qc & 15)][qr & 7];
          d[0] = (uint16_t)h;
          d[KT * 64 * 8] = (uint16_t)md;
          d[2 * KT * 64 * 8] = (uint16_t)l;
        }
        __syncthreads();
        if constexpr (EW == 2) {
          // A planes of both tiles first, then Q's per tile (the register budget of eight tiles)
          bf16x8 ap[EW][3];
#pragma unroll
          for (int e = 0; e < EW; ++e) {
            uint32_t h[4], md[4], l[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) split_pair(ra[p][2 * u][e], ra[p][2 * u + 1][e], h[u], md[u], l[u]);
            ap[e][0] = __builtin_bit_cast(bf16x8, make_uint4(h[0], h[1], h[2], h[3]));
            ap[e][1] = __builtin_bit_cast(bf16x8, make_uint4(md[0], md[1], md[2], md[3]));
            ap[e][2] = __builtin_bit_cast(bf16x8, make_uint4(l[0], l[1], l[2], l[3]));
          }
#pragma unroll
          for (int t = 0; t < KT; ++t) {
            bf16x8 qt[3];
#pragma unroll
            for (int pl = 0; pl < 3; ++pl) qt[pl] = *(const bf16x8*)&qs[b][pl][t][lane][0];
#pragma unroll
            for (int e = 0; e < EW; ++e) {
              f32x4 a = acc[e][t];
              a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ap[e][2], qt[0], a, 0, 0, 0);
              a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ap[e][0], qt[2], a, 0, 0, 0);
              a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ap[e][1], qt[1], a, 0, 0, 0);
              a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ap[e][1], qt[0], a, 0, 0, 0);
              a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ap[e][0], qt[1], a, 0, 0, 0);
              acc[e][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ap[e][0], qt[0], a, 0, 0, 0);
            }
          }
        } else {
        bf16x8 qp[3][KT];
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
#pragma unroll
          for (int t = 0; t < KT; ++t) qp[pl][t] = *(const bf16x8*)&qs[b][pl][t][lane][0];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          uint32_t h[4], md[4], l[4];
#pragma unroll
          for (int u = 0; u < 4; ++u) split_pair(ra[p][2 * u][e], ra[p][2 * u + 1][e], h[u], md[u], l[u]);
          const bf16x8 ah = __builtin_bit_cast(bf16x8, make_uint4(h[0], h[1], h[2], h[3]));
          const bf16x8 am = __builtin_bit_cast(bf16x8, make_uint4(md[0], md[1], md[2], md[3]));
          const bf16x8 al = __builtin_bit_cast(bf16x8, make_uint4(l[0], l[1], l[2], l[3]));
#pragma unroll
          for (int t = 0; t < KT; ++t) {
            f32x4 a = acc[e][t];
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, qp[0][t], a, 0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, qp[2][t], a, 0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, qp[1][t], a, 0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, qp[0][t], a, 0, 0, 0);
            a = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, qp[1][t], a, 0, 0, 0);
            acc[e][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, qp[0][t], a, 0, 0, 0);
          }
        }
        }
        __builtin_amdgcn_sched_barrier(0);
        issue(q0 + p + ATB_PD, p);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    // the clamped refills past the end: landed, and kept live until then
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int p = 0; p < ATB_PD; ++p) {
#pragma unroll
      for (int j = 0; j < 8; ++j) asm volatile("" : "+v"(ra[p][j]));
#pragma unroll
      for (int u = 0; u < KT; ++u) asm volatile("" : "+v"(rq[p][u]));
    }
  }
  if (cbw >= n) return;
  // slab (row group y) [n][k]: tile e row i (D row 4 (l >> 4) + r) is column cbw + EW i + e
  float* sb = slab + (int64_t)blockIdx.y * n * k;
#pragma unroll
  for (int e = 0; e < EW; ++e)
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      const int kc = 16 * t + nn;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int cw = cbw + EW * (4 * kk + r) + e;
        if (cw < n && kc < k) sb[(int64_t)cw * k + kc] = acc[e][t][r];
      }
    }
}

// ------------------------------------------------------- small f64 helpers
// out (rows x k2, TO, ldo) = X (rows x k, f64, ldx) M (k x k2, f64): 64-row
// tiles staged in LDS (coalesced), thread (row = t & 63, column group t >> 6)
// forms columns cg, cg + 4, ...; the tile goes back through LDS so the
// stores are row-contiguous.
template <typename TO>
__global__ void __launch_bounds__(256) k_ts_xm64(const double* __restrict__ X, int64_t rows, int k, int64_t ldx,
                                                 const double* __restrict__ Mm, int k2, TO* __restrict__ out,
                                                 int64_t ldo) {
  __shared__ double ms[64 * 64];
  __shared__ double xs[64 * 65];
  for (int e = threadIdx.x; e < k * k2; e += 256) ms[e] = Mm[e];
  const int tid = threadIdx.x, row = tid & 63, cg = tid >> 6;
  for (int64_t r0 = (int64_t)blockIdx.x * 64; r0 < rows; r0 += (int64_t)gridDim.x * 64) {
    __syncthreads();
    for (int e = tid; e < 64 * k; e += 256) {
      const int rr = e / k, c = e - rr * k;
      xs[rr * 65 + c] = r0 + rr < rows ? X[(r0 + rr) * ldx + c] : 0.0;
    }
    __syncthreads();
    double acc[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = 0.0;
    for (int l = 0; l < k; ++l) {
      const double x = xs[row * 65 + l];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const int c = cg + 4 * j;
        if (c < k2) acc[j] = fma(x, ms[l * k2 + c], acc[j]);
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int c = cg + 4 * j;
      if (c < k2) xs[row * 65 + c] = acc[j];
    }
    __syncthreads();
    for (int e = tid; e < 64 * k2; e += 256) {
      const int rr = e / k2, c = e - rr * k2;
      if (r0 + rr < rows) out[(r0 + rr) * ldo + c] = (TO)xs[rr * 65 + c];
    }
  }
}

// per-workgroup slab (k x k f64) of X^T X over its rows: 64-row tiles in
// LDS, thread t owns entries t, t + 256, ... of the upper triangle
__global__ void __launch_bounds__(256) k_ts_gram64(const double* __restrict__ X, int64_t rows, int k, int64_t ldx,
                                                   double* __restrict__ slab) {
  __shared__ double xs[64 * 65];
  const int tid = threadIdx.x;
  const int ntri = k * (k + 1) / 2;
  int pi[9], pj[9];
  double acc[9];
#pragma unroll
  for (int u = 0; u < 9; ++u) {
    int e = tid + 256 * u, i = 0;
    if (e < ntri) {
      while (e >= k - i) { e -= k - i; ++i; }
      pi[u] = i;
      pj[u] = i + e;
    } else {
      pi[u] = pj[u] = 0;
    }
    acc[u] = 0.0;
  }
  for (int64_t r0 = (int64_t)blockIdx.x * 64; r0 < rows; r0 += (int64_t)gridDim.x * 64) {
    __syncthreads();
    for (int e = tid; e < 64 * k; e += 256) {
      const int rr = e / k, c = e - rr * k;
      xs[rr * 65 + c] = r0 + rr < rows ? X[(r0 + rr) * ldx + c] : 0.0;
    }
    __syncthreads();
    for (int rr = 0; rr < 64; ++rr) {
#pragma unroll
      for (int u = 0; u < 9; ++u) acc[u] = fma(xs[rr * 65 + pi[u]], xs[rr * 65 + pj[u]], acc[u]);
    }
  }
  double* sb = slab + (int64_t)blockIdx.x * k * k;
#pragma unroll
  for (int u = 0; u < 9; ++u) {
    if (tid + 256 * u < ntri) {
      sb[pi[u] * k + pj[u]] = acc[u];
      sb[pj[u] * k + pi[u]] = acc[u];
    }
  }
}

// The same two helpers on the f64 matrix cores (v_mfma_f64_16x16x4f64), for
// even k / ldx with X 16-B aligned (k_ts_xm64 / k_ts_gram64 above serve the
// rest).  The LDS-tile VALU forms ran at ~0.7-1.3 TB/s (95 / 101 us on the
// 2e5 x 40 iterate of the f64 engine, ten Grams and seven X M per call).
//
// X M: a wave owns 16-row tiles (strided over the grid, two per iteration so
// ten 16-B loads per lane are in flight); lane (kg = l >> 4, r = l & 15) loads
// X[r][8 s + 2 kg .. + 1] for every 8-column step s and feeds element e to
// the MFMA whose K index 8 s + 2 kg + e its M fragment (held in registers
// for the whole kernel) agrees on.  Out tiles leave as 128-B row segments.
template <typename TO, int KT2>
__global__ void __launch_bounds__(256) k_ts_xm64m(const double* __restrict__ X, int64_t rows, int k, int64_t ldx,
                                                  const double* __restrict__ Mm, int k2, TO* __restrict__ out,
                                                  int64_t ldo) {
  constexpr int KS = 8;   // 8-column steps (k <= 64)
  const int lane = threadIdx.x & 63, kg = lane >> 4, r16 = lane & 15;
  const int ks = (k + 7) >> 3;
  double bm[KS][2][KT2];
#pragma unroll
  for (int st = 0; st < KS; ++st)
#pragma unroll
    for (int e = 0; e < 2; ++e)
#pragma unroll
      for (int tj = 0; tj < KT2; ++tj) {
        const int kr = 8 * st + 2 * kg + e, c = 16 * tj + r16;
        bm[st][e][tj] = (kr < k && c < k2) ? Mm[kr * k2 + c] : 0.0;
      }
  const int64_t ntile = (rows + 15) >> 4;
  const int64_t nw = (int64_t)gridDim.x * 4;
  for (int64_t t0 = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); t0 < ntile; t0 += 2 * nw) {
    f64x2 xv[2][KS];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int64_t t = t0 + u * nw;
      int64_t row = 16 * t + r16;
      row = row < rows ? row : rows - 1;   // clamped (never stored)
      const double* src = X + row * ldx;
      // unconditional loads from clamped columns, pinned by an empty asm
      // (else the compiler sinks each into an exec-masked branch with its
      // own vmcnt(0)), zeroed after
#pragma unroll
      for (int st = 0; st < KS; ++st) {
        const int c = 8 * st + 2 * kg;
        xv[u][st] = *(const f64x2*)(src + (c < k ? c : 0));
      }
    }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int st = 0; st < KS; ++st) {
        asm volatile("" : "+v"(xv[u][st]));
        const int c = 8 * st + 2 * kg;
        if (!(st < ks && c < k)) xv[u][st] = f64x2{0.0, 0.0};
      }
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int64_t t = t0 + u * nw;
      if (t >= ntile) break;
      f64x4 acc[KT2];
#pragma unroll
      for (int tj = 0; tj < KT2; ++tj) acc[tj] = f64x4{};
#pragma unroll
      for (int st = 0; st < KS; ++st) {
        if (st >= ks) break;
#pragma unroll
        for (int e = 0; e < 2; ++e)
#pragma unroll
          for (int tj = 0; tj < KT2; ++tj)
            acc[tj] = __builtin_amdgcn_mfma_f64_16x16x4f64(xv[u][st][e], bm[st][e][tj], acc[tj], 0, 0, 0);
      }
#pragma unroll
      for (int tj = 0; tj < KT2; ++tj) {
        const int c = 16 * tj + r16;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t row = 16 * t + Mf<double>::drow(lane, r);
          if (row < rows && c < k2) out[row * ldo + c] = (TO)acc[tj][r];
        }
      }
    }
  }
}

// X^T X: a wave owns a contiguous range of 4-row K-steps (rows 4 q + kg,
// columns 16 t + r16 per lane: the A and B fragments of every tile come from
// the same KT loaded values), upper-triangle tiles only, four steps of
// loads in flight; the four waves' tiles are summed in LDS and the slab is
// written from the upper triangle (exactly symmetric).
template <int KT>
__global__ void __launch_bounds__(256) k_ts_gram64m(const double* __restrict__ X, int64_t rows, int k, int64_t ldx,
                                                    double* __restrict__ slab) {
  constexpr int KP = 16 * KT, U = 4;
  __shared__ double red[KP][KP + 1];
  const int lane = threadIdx.x & 63, kg = lane >> 4, r16 = lane & 15, w = threadIdx.x >> 6;
  f64x4 acc[KT][KT];
#pragma unroll
  for (int a = 0; a < KT; ++a)
#pragma unroll
    for (int b = 0; b < KT; ++b) acc[a][b] = f64x4{};
  const int64_t nq = (rows + 3) >> 2;
  const int64_t nw = (int64_t)gridDim.x * 4;
  const int64_t wid = (int64_t)blockIdx.x * 4 + w;
  const int64_t q0 = nq * wid / nw, q1 = nq * (wid + 1) / nw;
  for (int64_t q = q0; q < q1; q += U) {
    double xv[U][KT];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t row = 4 * (q + u) + kg;
      const bool rok = q + u < q1 && row < rows;
      const double* src = X + (row < rows ? row : rows - 1) * ldx;
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        const int c = 16 * t + r16;
        xv[u][t] = src[c < k ? c : k - 1];   // unconditional, pinned below (see k_ts_xm64m)
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t row = 4 * (q + u) + kg;
      const bool rok = q + u < q1 && row < rows;
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        asm volatile("" : "+v"(xv[u][t]));
        if (!(rok && 16 * t + r16 < k)) xv[u][t] = 0.0;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int a = 0; a < KT; ++a)
#pragma unroll
        for (int b = a; b < KT; ++b) acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(xv[u][a], xv[u][b], acc[a][b], 0, 0, 0);
  }
  for (int ww = 0; ww < 4; ++ww) {
    if (w == ww) {
#pragma unroll
      for (int a = 0; a < KT; ++a)
#pragma unroll
        for (int b = a; b < KT; ++b)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int i = 16 * a + Mf<double>::drow(lane, r), j = 16 * b + r16;
            red[i][j] = ww == 0 ? acc[a][b][r] : red[i][j] + acc[a][b][r];
          }
    }
    __syncthreads();
  }
  double* sb = slab + (int64_t)blockIdx.x * k * k;
  for (int e = threadIdx.x; e < k * k; e += 256) {
    const int i = e / k, j = e - i * k;
    sb[e] = i <= j ? red[i][j] : red[j][i];
  }
}

// X^T X for 64 < k <= 128 (f32 or f64 X, f64 products and sums): the 36
// upper 16 x 16 tile pairs of the 8 x 8 tile grid are dealt round-robin to
// the four waves (9 accumulators each, 72 VGPRs: all 36 on one wave would
// need 288), and the four waves of a workgroup walk the SAME rows -- wave w
// loads all 8 column tiles of each 4-row step (the other waves' loads of the
// same lines hit L1 / L2) and keeps only its own pairs.  Each workgroup owns
// a contiguous row range and writes its k x k slab directly (the pairs are
// disjoint: no LDS reduction), mirrored from the upper tiles.
__host__ __device__ constexpr int gw_pa(int p) { int a = 0; while (p >= 8 - a) { p -= 8 - a; ++a; } return a; }
__host__ __device__ constexpr int gw_pb(int p) { int a = 0; while (p >= 8 - a) { p -= 8 - a; ++a; } return a + p; }

// the nine MFMAs of wave W on one 4-row step, pair indices folded at compile
// time (constexpr locals: in an unrolled loop the pair functions were left as
// run-time scalar loops with a dynamic register index before every MFMA)
template <int W, int E>
__device__ __forceinline__ void gw_mma(f64x4 (&acc)[9], const double (&xv)[8]) {
  if constexpr (E < 9) {
    constexpr int a = gw_pa(W + 4 * E), b = gw_pb(W + 4 * E);
    acc[E] = __builtin_amdgcn_mfma_f64_16x16x4f64(xv[a], xv[b], acc[E], 0, 0, 0);
    gw_mma<W, E + 1>(acc, xv);
  }
}
template <int W, int E>
__device__ __forceinline__ void gw_store(const f64x4 (&acc)[9], double* sb, int k, int lane, int r16) {
  if constexpr (E < 9) {
    constexpr int a = gw_pa(W + 4 * E), b = gw_pb(W + 4 * E);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = 16 * a + Mf<double>::drow(lane, r), j = 16 * b + r16;
      if (i < k && j < k) {
        sb[(int64_t)i * k + j] = acc[E][r];
        if (a != b) sb[(int64_t)j * k + i] = acc[E][r];
      }
    }
    gw_store<W, E + 1>(acc, sb, k, lane, r16);
  }
}

template <typename T, int W>
__device__ __forceinline__ void gram_w_body(const T* __restrict__ X, int64_t rows, int k, int64_t ldx,
                                            double* __restrict__ slab) {
  // U 4-row steps per load group; f32 X keeps its raw words in the ping-pong
  // buffers (half the registers of f64), so it prefetches deeper
  constexpr int KT = 8, NP = 9, U = sizeof(T) == 4 ? 8 : 4;
  const int lane = threadIdx.x & 63, kg = lane >> 4, r16 = lane & 15;
  f64x4 acc[NP];
#pragma unroll
  for (int e = 0; e < NP; ++e) acc[e] = f64x4{};
  const int64_t nq = (rows + 3) >> 2;
  const int64_t q0 = nq * blockIdx.x / gridDim.x, q1 = nq * (blockIdx.x + 1) / gridDim.x;
  // software-pipelined: the next U steps' loads are in flight while this U's
  // MFMAs run (a load-then-compute loop waited out the memory latency every
  // iteration: 2.5 ms for a 1e6 x 128 f32 Gram).  Unconditional loads from
  // clamped addresses (a conditional load became an exec-masked branch with a
  // vmcnt(0)); the widening and the zero-select happen at the MFMA, so nothing
  // waits on a group's loads before the previous group's MFMAs have issued
  auto load = [&](int64_t q, T (&raw)[U][KT]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t row = 4 * (q + u) + kg;
      const T* src = X + (row < rows ? row : rows - 1) * ldx;
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        const int c = 16 * t + r16;
        raw[u][t] = src[c < k ? c : k - 1];
      }
    }
  };
  auto mma = [&](int64_t q, const T (&raw)[U][KT]) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t row = 4 * (q + u) + kg;
      const bool rok = q + u < q1 && row < rows;
      double xv[KT];
#pragma unroll
      for (int t = 0; t < KT; ++t) xv[t] = (rok && 16 * t + r16 < k) ? (double)raw[u][t] : 0.0;
      gw_mma<W, 0>(acc, xv);
    }
  };
  T xa[U][KT], xb[U][KT];
  if (q0 < q1) load(q0, xa);
  for (int64_t q = q0; q < q1; q += 2 * U) {
    if (q + U < q1) load(q + U, xb);
    mma(q, xa);
    if (q + U >= q1) break;
    if (q + 2 * U < q1) load(q + 2 * U, xa);
    mma(q + U, xb);
  }
  gw_store<W, 0>(acc, slab + (int64_t)blockIdx.x * k * k, k, lane, r16);
}

template <typename T>
__global__ void __launch_bounds__(256) k_ts_gram_w(const T* __restrict__ X, int64_t rows, int k, int64_t ldx,
                                                   double* __restrict__ slab) {
  switch (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) {
    case 0: gram_w_body<T, 0>(X, rows, k, ldx, slab); break;
    case 1: gram_w_body<T, 1>(X, rows, k, ldx, slab); break;
    case 2: gram_w_body<T, 2>(X, rows, k, ldx, slab); break;
    default: gram_w_body<T, 3>(X, rows, k, ldx, slab); break;
  }
}

// C (mr x nc, ldc) = op(A) op(B), op(A) mr x kd, op(B) kd x nc, row-major f64,
// one workgroup (k x k sizes of the core): both operands staged in LDS first
// when they fit (coalesced reads; the strided global form took ~36 us)
__global__ void __launch_bounds__(256) k_ts_small(int ta, int tb, int mr, int nc, int kd, const double* __restrict__ A,
                                                  int lda, const double* __restrict__ B, int ldb,
                                                  double* __restrict__ C, int ldc) {
  __shared__ double as[64 * 65], bs[64 * 65];
  {
    // as[i][l] = op(A)[i][l], bs[j][l] = op(B)[l][j] (pitch 65: conflict-free rows)
    for (int e = threadIdx.x; e < mr * kd; e += 256) {
      if (ta) {   // A is kd x mr: as[i][l] = A[l][i]
        const int l = e / mr, i = e - l * mr;
        as[i * 65 + l] = A[l * lda + i];
      } else {
        const int i = e / kd, l = e - i * kd;
        as[i * 65 + l] = A[i * lda + l];
      }
    }
    for (int e = threadIdx.x; e < kd * nc; e += 256) {
      if (tb) {
        const int j = e / kd, l = e - j * kd;
        bs[j * 65 + l] = B[j * ldb + l];
      } else {
        const int l = e / nc, j = e - l * nc;
        bs[j * 65 + l] = B[l * ldb + j];
      }
    }
    __syncthreads();
    for (int e = threadIdx.x; e < mr * nc; e += 256) {
      const int i = e / nc, j = e - i * nc;
      double s = 0.0;
      for (int l = 0; l < kd; ++l) s = fma(as[i * 65 + l], bs[j * 65 + l], s);
      C[i * ldc + j] = s;
    }
  }
}

// the same product past 64 (the 64 < k <= 128 core): one 32 x 32 tile of C
// per workgroup, kd in 32-wide chunks through LDS (coalesced along the
// contiguous index of each operand), four outputs per thread
__global__ void __launch_bounds__(256) k_ts_small_tiled(int ta, int tb, int mr, int nc, int kd,
                                                        const double* __restrict__ A, int lda,
                                                        const double* __restrict__ B, int ldb,
                                                        double* __restrict__ C, int ldc) {
  __shared__ double as[32][33], bs[32][33];   // as[i][l] = op(A)[i0 + i][l0 + l], bs[j][l] = op(B)[l0 + l][j0 + j]
  const int i0 = blockIdx.y * 32, j0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  double acc[4] = {0.0, 0.0, 0.0, 0.0};
  for (int l0 = 0; l0 < kd; l0 += 32) {
    for (int e = threadIdx.x; e < 32 * 32; e += 256) {
      const int hi = e >> 5, lo = e & 31;
      // op(A): ta -> A is kd x mr (contiguous along i), else mr x kd (along l)
      const int ai = ta ? lo : hi, al = ta ? hi : lo;
      const int gi = i0 + ai, gl = l0 + al;
      as[ai][al] = (gi < mr && gl < kd) ? (ta ? A[(int64_t)gl * lda + gi] : A[(int64_t)gi * lda + gl]) : 0.0;
      // op(B): tb -> B is nc x kd (contiguous along l), else kd x nc (along j)
      const int bj = tb ? hi : lo, bl = tb ? lo : hi;
      const int gj = j0 + bj, gm = l0 + bl;
      bs[bj][bl] = (gj < nc && gm < kd) ? (tb ? B[(int64_t)gj * ldb + gm] : B[(int64_t)gm * ldb + gj]) : 0.0;
    }
    __syncthreads();
#pragma unroll 8
    for (int l = 0; l < 32; ++l) {
      const double bv = bs[tx][l];
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] = fma(as[ty + 8 * u][l], bv, acc[u]);
    }
    __syncthreads();
  }
  const int j = j0 + tx;
  if (j < nc) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int i = i0 + ty + 8 * u;
      if (i < mr) C[(int64_t)i * ldc + j] = acc[u];
    }
  }
}

int ncu() {
  static int c = -1;
  if (c < 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      c = 256;
  }
  return c;
}

// 16-B loads: A 16-B aligned, lda and n multiples of the vector width (a
// vector then never straddles the end of a row)
template <typename T>
bool vec_ok(const T* A, int64_t lda, int64_t n) {
  const int64_t vw = 16 / (int64_t)sizeof(T);
  return ((uintptr_t)A % 16) == 0 && lda % vw == 0 && n % vw == 0;
}

int g_az_split = 1;
int g_az_align = 1;   // row-alignment classes in Y = A Z (0: A/B)
int g_az_bf16 = 1;   // f32, 16 < k <= 48: the exact-split bf16 form of Y = A Z (0: f32 MFMA, A/B)

template <typename T, int KT, bool BS>
int launch_az_(const T* A, int64_t m, int n, int64_t lda, const T* Z, int k, T* Y, int64_t ldy, hipStream_t s) {
  constexpr int LDS = az_lds<T, KT, BS>();
  constexpr int EPL = AZ_VL * Mf<T>::VW, CW = AZ_NG * 4 * EPL;
  // row pitch not a whole number of 128-B lines (but of 32-B lane groups),
  // A line-aligned: the kernel's alignment classes (P = 2 or 4 row offsets)
  int P = 1, stepB = 0;
  if (g_az_align && ((uintptr_t)A % 128) == 0) {
    const int64_t sb = (lda * (int64_t)sizeof(T)) & 127;
    if (sb != 0 && sb % 32 == 0) {
      P = sb == 64 ? 2 : 4;
      stepB = (int)sb;
    }
  }
  const int64_t nrb = (m + AZ_BR - 1) / AZ_BR;
  const int nchunk = (n + (P > 1 ? 3 * EPL : 0) + CW - 1) / CW;
  // g <= nrb: every stream-K range spans at least one whole row block
  const int64_t res = (KT > 4 ? 1 : 2) * (int64_t)ncu();   // resident workgroups
  const int64_t g = nrb < res ? nrb : res;
  if (g > 1 && g_az_split) {
    k_az_zero_cut<T><<<(unsigned)(g - 1), 256, 0, s>>>(Y, m, k, ldy, nrb, nchunk, (int)g);
    SL_LAUNCH_CHECK();
  }
  if (vec_ok(A, lda, n)) {
    SL_LDS_ATTR((k_ts_az<T, KT, true, BS>), LDS);
    k_ts_az<T, KT, true, BS><<<(unsigned)g, az_nt<KT>(), LDS, s>>>(A, m, n, lda, Z, k, Y, ldy, g_az_split, P, stepB);
  } else {
    SL_LDS_ATTR((k_ts_az<T, KT, false, BS>), LDS);
    k_ts_az<T, KT, false, BS><<<(unsigned)g, az_nt<KT>(), LDS, s>>>(A, m, n, lda, Z, k, Y, ldy, g_az_split, P, stepB);
  }
  SL_LAUNCH_CHECK();
  return SL_OK;
}

template <typename T, int KT>
int launch_az(const T* A, int64_t m, int n, int64_t lda, const T* Z, int k, T* Y, int64_t ldy, hipStream_t s) {
  // the split form's Z planes (48 B per slot) keep two workgroups per CU in
  // LDS up to three column tiles; one column tile (k <= 16) streams faster
  // on the f32 form (720 vs 759 us at k = 16, profiles/r6/az_align_ab.txt)
  if constexpr (sizeof(T) == 4 && KT >= 2 && KT <= 3)
    if (g_az_bf16) return launch_az_<T, KT, true>(A, m, n, lda, Z, k, Y, ldy, s);
  return launch_az_<T, KT, false>(A, m, n, lda, Z, k, Y, ldy, s);
}

// vectors per wave and row: the knob for k <= 64; one (with one 512-thread
// workgroup per CU, > 128 VGPRs of accumulators) for 64 < k <= 128
int atq_av(int k) { return k > 64 ? 1 : g_atq_av; }

int g_atq_bf16 = 1;   // f32, 16 < k <= 128: k_ts_atq_bs (0: f32 MFMA, A/B)
bool atq_bs(int k) { return g_atq_bf16 && k > 16; }
int atq_bs_cs(int k) { return k > 64 ? 256 : 512; }   // slice width of k_ts_atq_bs (EW = 2 / 4)

// row groups of the A^T Q product: ~2 workgroups per CU over all slices
// (bs: the split-form kernel's 512-column slices)
template <typename T>
void atq_geometry(int64_t m, int n, int k, int* slices, int* groups, int64_t* rows_per, bool bs = false) {
  const int CS = bs ? atq_bs_cs(k) : 8 * atq_av(k) * 16 * (16 / (int)sizeof(T));
  *slices = (n + CS - 1) / CS;
  // AV = 2: one 512-thread workgroup per CU is resident (k_ts_atq needs >
  // 128 VGPRs): slices x groups <= 2 x CUs is two full rounds (rounding the
  // group count up left a third round of a few workgroups: f64 n = 5000
  // ran 520 workgroups, ~50% over); AV = 1: two resident, one round
  int64_t g = 2 * (int64_t)ncu() / *slices;
  const int64_t maxg = (m + 63) / 64;   // at least 64 rows per group
  if (g > maxg) g = maxg;
  if (g < 1) g = 1;
  int64_t rp = (m + g - 1) / g;
  rp = (rp + 3) & ~(int64_t)3;
  *groups = (int)((m + rp - 1) / rp);
  *rows_per = rp;
}

template <typename T, int KT>
int launch_atq(const T* A, int64_t m, int n, int64_t lda, const T* Q, int k, T* slab, int slices, int groups,
               int64_t rp, hipStream_t s) {
  const dim3 grid((unsigned)slices, (unsigned)groups);
  const bool v = vec_ok(A, lda, n);
  if constexpr (KT > 4) {
    if (v) k_ts_atq<T, KT, true, 1><<<grid, AT_NT, 0, s>>>(A, m, n, lda, Q, k, rp, slab);
    else k_ts_atq<T, KT, false, 1><<<grid, AT_NT, 0, s>>>(A, m, n, lda, Q, k, rp, slab);
  } else if (atq_av(k) == 1) {
    if (v) k_ts_atq<T, KT, true, 1><<<grid, AT_NT, 0, s>>>(A, m, n, lda, Q, k, rp, slab);
    else k_ts_atq<T, KT, false, 1><<<grid, AT_NT, 0, s>>>(A, m, n, lda, Q, k, rp, slab);
  } else {
    if (v) k_ts_atq<T, KT, true, 2><<<grid, AT_NT, 0, s>>>(A, m, n, lda, Q, k, rp, slab);
    else k_ts_atq<T, KT, false, 2><<<grid, AT_NT, 0, s>>>(A, m, n, lda, Q, k, rp, slab);
  }
  SL_LAUNCH_CHECK();
  return SL_OK;
}

template <typename T>
int az_dispatch(const T* A, int64_t m, int n, int64_t lda, const T* Z, int k, T* Y, int64_t ldy, hipStream_t s) {
  switch ((k + 15) / 16) {
    case 1: return launch_az<T, 1>(A, m, n, lda, Z, k, Y, ldy, s);
    case 2: return launch_az<T, 2>(A, m, n, lda, Z, k, Y, ldy, s);
    case 3: return launch_az<T, 3>(A, m, n, lda, Z, k, Y, ldy, s);
    case 4: return launch_az<T, 4>(A, m, n, lda, Z, k, Y, ldy, s);
    // 64 < k <= 128: six or eight column tiles (seven spilled f32 registers)
    case 5: case 6: return launch_az<T, 6>(A, m, n, lda, Z, k, Y, ldy, s);
    default: return launch_az<T, 8>(A, m, n, lda, Z, k, Y, ldy, s);
  }
}

template <typename T>
int atq_dispatch(const T* A, int64_t m, int n, int64_t lda, const T* Q, int k, T* slab, int slices, int groups,
                 int64_t rp, hipStream_t s) {
  switch ((k + 15) / 16) {
    case 1: return launch_atq<T, 1>(A, m, n, lda, Q, k, slab, slices, groups, rp, s);
    case 2: return launch_atq<T, 2>(A, m, n, lda, Q, k, slab, slices, groups, rp, s);
    case 3: return launch_atq<T, 3>(A, m, n, lda, Q, k, slab, slices, groups, rp, s);
    case 4: return launch_atq<T, 4>(A, m, n, lda, Q, k, slab, slices, groups, rp, s);
    case 5: case 6: return launch_atq<T, 6>(A, m, n, lda, Q, k, slab, slices, groups, rp, s);
    default: return launch_atq<T, 8>(A, m, n, lda, Q, k, slab, slices, groups, rp, s);
  }
}

int gram_grid(int64_t rows) {
  const int64_t g = (rows + 255) / 256;
  const int64_t cap = 2 * (int64_t)ncu();
  return (int)(g < 1 ? 1 : (g > cap ? cap : g));
}

}  // namespace

// Y (m x k, row stride ldy) = A (m x n, lda) Z (n x k, row-major); dt SL_F32 / SL_F64, 1 <= k <= 128
SL_API int sl_ts_az(const void* A, int64_t m, int64_t n, int64_t lda, const void* Z, int k, void* Y, int64_t ldy,
                    int dt, void* stream) {
  if (m <= 0) return SL_OK;
  if (k < 1 || k > 128 || n < 1 || n > (int64_t)1 << 30 || lda < n || ldy < k || (dt != SL_F32 && dt != SL_F64)) {
    sl_set_last_error("ts_az: needs 1 <= k <= 128, lda >= n, ldy >= k, f32 / f64");
    return SL_ERR_UNSUPPORTED;
  }
  hipStream_t s = (hipStream_t)stream;
  if (dt == SL_F32) return az_dispatch<float>((const float*)A, m, (int)n, lda, (const float*)Z, k, (float*)Y, ldy, s);
  return az_dispatch<double>((const double*)A, m, (int)n, lda, (const double*)Z, k, (double*)Y, ldy, s);
}

// A/B knob: vectors per wave and row of A^T Q (1 or 2; plans size their
// workspace with sl_ts_atq_workspace after setting it)
SL_API void sl_ts_set_atq_av(int v) { g_atq_av = v == 1 ? 1 : 2; }

// A/B knob: 1 (default) whole-block rounds + stream-K tail, 0 whole blocks round-robin
SL_API void sl_ts_set_az_split(int v) { g_az_split = v ? 1 : 0; }
SL_API void sl_ts_set_az_bf16(int v) { g_az_bf16 = v ? 1 : 0; }
SL_API void sl_ts_set_az_align(int v) { g_az_align = v ? 1 : 0; }
SL_API void sl_ts_set_atq_bf16(int v) { g_atq_bf16 = v ? 1 : 0; }

// bytes of slab workspace sl_ts_atq needs
SL_API int64_t sl_ts_atq_workspace(int64_t m, int64_t n, int k, int dt) {
  int slices = 0, groups = 0;
  int64_t rp = 0;
  if (dt == SL_F64) {
    atq_geometry<double>(m, (int)n, k, &slices, &groups, &rp);
  } else {
    // either f32 kernel may run (the split form needs 16-B loads): the larger
    atq_geometry<float>(m, (int)n, k, &slices, &groups, &rp);
    int s2 = 0, g2 = 0;
    atq_geometry<float>(m, (int)n, k, &s2, &g2, &rp, true);
    groups = g2 > groups ? g2 : groups;
  }
  return (int64_t)groups * n * k * (dt == SL_F64 ? 8 : 4) + 256;
}

// W (n x k f64, row stride ldw) = A^T Q, A m x n (lda), Q m x k (row-major, A's dtype)
SL_API int sl_ts_atq(const void* A, int64_t m, int64_t n, int64_t lda, const void* Q, int k, double* W, int ldw,
                     void* ws, int dt, void* stream) {
  if (k < 1 || k > 128 || n < 1 || n > (int64_t)1 << 30 || lda < n || ldw < k || (dt != SL_F32 && dt != SL_F64)) {
    sl_set_last_error("ts_atq: needs 1 <= k <= 128, lda >= n, ldw >= k, f32 / f64");
    return SL_ERR_UNSUPPORTED;
  }
  hipStream_t s = (hipStream_t)stream;
  if (m <= 0) return hipMemset2DAsync(W, (size_t)ldw * 8, 0, (size_t)k * 8, (size_t)n, s) == hipSuccess ? SL_OK : SL_ERR_HIP;
  int slices = 0, groups = 0;
  int64_t rp = 0;
  int rc;
  if (dt == SL_F32) {
    const bool bs = atq_bs(k) && vec_ok((const float*)A, lda, n);
    atq_geometry<float>(m, (int)n, k, &slices, &groups, &rp, bs);
    if (bs) {
      const dim3 grid((unsigned)slices, (unsigned)groups);
      if (k > 96) k_ts_atq_bs<8, 2><<<grid, AT_NT, 0, s>>>((const float*)A, m, (int)n, lda, (const float*)Q, k, rp, (float*)ws);
      else if (k > 64) k_ts_atq_bs<6, 2><<<grid, AT_NT, 0, s>>>((const float*)A, m, (int)n, lda, (const float*)Q, k, rp, (float*)ws);
      else if (k > 48) k_ts_atq_bs<4><<<grid, AT_NT, 0, s>>>((const float*)A, m, (int)n, lda, (const float*)Q, k, rp, (float*)ws);
      else if (k > 32) k_ts_atq_bs<3><<<grid, AT_NT, 0, s>>>((const float*)A, m, (int)n, lda, (const float*)Q, k, rp, (float*)ws);
      else k_ts_atq_bs<2><<<grid, AT_NT, 0, s>>>((const float*)A, m, (int)n, lda, (const float*)Q, k, rp, (float*)ws);
      SL_LAUNCH_CHECK();
      rc = SL_OK;
    } else {
      rc = atq_dispatch<float>((const float*)A, m, (int)n, lda, (const float*)Q, k, (float*)ws, slices, groups, rp, s);
    }
    if (rc != SL_OK) return rc;
    return sl_slab_reduce_launch_f64((const float*)ws, groups, n * k, k, (int)n, k, W, ldw, s);
  }
  atq_geometry<double>(m, (int)n, k, &slices, &groups, &rp);
  rc = atq_dispatch<double>((const double*)A, m, (int)n, lda, (const double*)Q, k, (double*)ws, slices, groups, rp, s);
  if (rc != SL_OK) return rc;
  return sl_slab_reduce_launch_d2d((const double*)ws, groups, n * k, k, (int)n, k, W, ldw, s);
}

// out (rows x k2, ldo; out_dt SL_F32 / SL_F64) = X (rows x k f64, ldx) M (k x k2 f64, row-major), k, k2 <= 64
SL_API int sl_ts_xm64(const double* X, int64_t rows, int k, int64_t ldx, const double* Mm, int k2, void* out,
                      int64_t ldo, int out_dt, void* stream) {
  if (rows <= 0) return SL_OK;
  if (k < 1 || k > 64 || k2 < 1 || k2 > 64 || ldx < k || ldo < k2 || (out_dt != SL_F32 && out_dt != SL_F64)) {
    sl_set_last_error("ts_xm64: needs 1 <= k, k2 <= 64");
    return SL_ERR_UNSUPPORTED;
  }
  hipStream_t s = (hipStream_t)stream;
  if (k % 2 == 0 && ldx % 2 == 0 && ((uintptr_t)X & 15) == 0) {
    // matrix-core form: 16-row tiles, two per wave and iteration
    const int64_t t8 = ((rows + 15) / 16 + 7) / 8;
    const unsigned g = (unsigned)(t8 < 2 * (int64_t)ncu() ? t8 : 2 * (int64_t)ncu());
#define SL_XM(TO, KT2) k_ts_xm64m<TO, KT2><<<g, 256, 0, s>>>(X, rows, k, ldx, Mm, k2, (TO*)out, ldo)
#define SL_XM2(TO) switch ((k2 + 15) / 16) { case 1: SL_XM(TO, 1); break; case 2: SL_XM(TO, 2); break; \
                                             case 3: SL_XM(TO, 3); break; default: SL_XM(TO, 4); break; }
    if (out_dt == SL_F32) { SL_XM2(float) }
    else { SL_XM2(double) }
#undef SL_XM2
#undef SL_XM
    SL_LAUNCH_CHECK();
    return SL_OK;
  }
  const int64_t tiles = (rows + 63) / 64;
  const unsigned g = (unsigned)(tiles < 4 * (int64_t)ncu() ? tiles : 4 * (int64_t)ncu());
  if (out_dt == SL_F32) k_ts_xm64<float><<<g, 256, 0, s>>>(X, rows, k, ldx, Mm, k2, (float*)out, ldo);
  else k_ts_xm64<double><<<g, 256, 0, s>>>(X, rows, k, ldx, Mm, k2, (double*)out, ldo);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

SL_API int64_t sl_ts_gram64_workspace(int64_t rows, int k) { return (int64_t)gram_grid(rows) * k * k * 8 + 256; }

// G (k x k f64, ldg) = X^T X, X rows x k f64 (ldx), k <= 64 (ws: sl_ts_gram64_workspace bytes)
SL_API int sl_ts_gram64(const double* X, int64_t rows, int k, int64_t ldx, double* G, int ldg, void* ws,
                        void* stream) {
  if (k < 1 || k > 64 || ldx < k || ldg < k) {
    sl_set_last_error("ts_gram64: needs 1 <= k <= 64");
    return SL_ERR_UNSUPPORTED;
  }
  hipStream_t s = (hipStream_t)stream;
  if (rows <= 0) return hipMemset2DAsync(G, (size_t)ldg * 8, 0, (size_t)k * 8, (size_t)k, s) == hipSuccess ? SL_OK : SL_ERR_HIP;
  const int g = gram_grid(rows);
  switch ((k + 15) / 16) {
    case 1: k_ts_gram64m<1><<<g, 256, 0, s>>>(X, rows, k, ldx, (double*)ws); break;
    case 2: k_ts_gram64m<2><<<g, 256, 0, s>>>(X, rows, k, ldx, (double*)ws); break;
    case 3: k_ts_gram64m<3><<<g, 256, 0, s>>>(X, rows, k, ldx, (double*)ws); break;
    default: k_ts_gram64m<4><<<g, 256, 0, s>>>(X, rows, k, ldx, (double*)ws); break;
  }
  SL_LAUNCH_CHECK();
  return sl_slab_reduce_launch_d2d((const double*)ws, g, (int64_t)k * k, k, k, k, G, ldg, s);
}

// G (k x k f64, ldg) = X^T X for 64 < k <= 128, X rows x k f32 (dt SL_F32) or
// f64 (ldx); ws: sl_ts_gram64_workspace bytes
SL_API int sl_ts_gram_w(const void* X, int dt, int64_t rows, int k, int64_t ldx, double* G, int ldg, void* ws,
                        void* stream) {
  if (k < 1 || k > 128 || ldx < k || ldg < k || (dt != SL_F32 && dt != SL_F64)) {
    sl_set_last_error("ts_gram_w: needs 1 <= k <= 128, f32 / f64");
    return SL_ERR_UNSUPPORTED;
  }
  hipStream_t s = (hipStream_t)stream;
  if (rows <= 0) return hipMemset2DAsync(G, (size_t)ldg * 8, 0, (size_t)k * 8, (size_t)k, s) == hipSuccess ? SL_OK : SL_ERR_HIP;
  const int g = gram_grid(rows);
  if (dt == SL_F64) k_ts_gram_w<double><<<g, 256, 0, s>>>((const double*)X, rows, k, ldx, (double*)ws);
  else k_ts_gram_w<float><<<g, 256, 0, s>>>((const float*)X, rows, k, ldx, (double*)ws);
  SL_LAUNCH_CHECK();
  return sl_slab_reduce_launch_d2d((const double*)ws, g, (int64_t)k * k, k, k, k, G, ldg, s);
}

// C (mr x nc, ldc) = op(A) op(B) (row-major f64; ta / tb: transpose), one workgroup
SL_API int sl_ts_small(int ta, int tb, int mr, int nc, int kd, const double* A, int lda, const double* B, int ldb,
                       double* C, int ldc, void* stream) {
  if (mr < 1 || nc < 1 || kd < 1) {
    sl_set_last_error("ts_small: needs positive sizes");
    return SL_ERR_DIMENSION;
  }
  if (mr <= 64 && nc <= 64 && kd <= 64) {
    k_ts_small<<<1, 256, 0, (hipStream_t)stream>>>(ta, tb, mr, nc, kd, A, lda, B, ldb, C, ldc);
  } else {
    const dim3 grid((unsigned)((nc + 31) / 32), (unsigned)((mr + 31) / 32));
    k_ts_small_tiled<<<grid, 256, 0, (hipStream_t)stream>>>(ta, tb, mr, nc, kd, A, lda, B, ldb, C, ldc);
  }
  SL_LAUNCH_CHECK();
  return SL_OK;
}
