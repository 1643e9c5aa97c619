// Latency-oriented small dense linear algebra for ONE workgroup on gfx950:
// the k x k (k <= 64) algebra of the randomized SVD's pass boundaries
// (reference nla/svd.hpp:71-149 re-orthonormalisation, :278-317 the core SVD
// of the k x k Rayleigh-Ritz matrix), where every microsecond is on the
// critical path of the call.
//
// Design rules (MI355X: one wave issues an f64 FMA every ~4-8 cycles, a DS
// read returns in ~50 cycles, an 8-wave s_barrier costs ~100+):
//   * the sequential k-step factorisations run in ONE wave with the matrix
//     in registers (lane = row or column, register index = the other index,
//     every step unrolled at a compile-time K so register indices are
//     static): no workgroup barrier inside the chain, only wave-local LDS
//     broadcasts and DPP reductions;
//   * the embarrassingly parallel phases (bisection per eigenvalue, the
//     back-transformation per eigenvector) spread over all waves.
//
//   wave_chol_inv<K>   X = R^{-1} of G = R^T R: in-place LDL^T elimination of
//                      [G | I] with lane c holding column c of whichever half
//                      is live (T column c until pivot c, then L^{-1} column c)
//   wg_chol_inv<K,NW>  the same X with the elimination's rows split over NW
//                      waves (one barrier per step)
//   wave_tridiag<K>    Householder tridiagonalisation T = Q^T C Q (lane = row)
//   sym_top_eig<K>     top-nt eigenvalues of T by multisection on a
//                      division-free Sturm count, eigenvectors of T by the
//                      twisted factorisation, MGS inside close clusters, and
//                      the back-transformation Q x (16 lanes per vector)
#pragma once
#include "sl_common.hpp"


// prefetch distances (steps) of the LDS-broadcast operands of the Sturm
// count and the twisted factorisation (A/B knobs of benchmarks/probe: 4 to
// 16 steps, and readlane broadcasts instead of LDS, all within 1% -- the
// phases are f64 VALU issue-bound on one wave per eigenvalue group,
// profiles/r5/eig_stamps_v2.jsonl)
#ifndef SLW_STURM_PF
#define SLW_STURM_PF 4
#endif
#ifndef SLW_TWIST_PF
#define SLW_TWIST_PF 4
#endif

namespace slw {

// ------------------------------------------------------------ wave helpers
template <int CTRL>
__device__ __forceinline__ double dpp(double x) {
  // every pattern used here is a full permutation (no invalid source lane):
  // mov_dpp needs no initialised destination
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(x), CTRL, 0xF, 0xF, true);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(x), CTRL, 0xF, 0xF, true);
  return __hiloint2double(hi, lo);
}

// value of x in lane l (l wave-uniform)
__device__ __forceinline__ double lane_d(double x, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(x), l),
                          __builtin_amdgcn_readlane(__double2loint(x), l));
}

// sum over each DPP row of 16 lanes, result in every lane of the row
__device__ __forceinline__ double row16_sum(double x) {
  x += dpp<0xB1>(x);    // quad_perm [1,0,3,2]
  x += dpp<0x4E>(x);    // quad_perm [2,3,0,1]
  x += dpp<0x141>(x);   // row_half_mirror
  x += dpp<0x140>(x);   // row_mirror
  return x;
}

__device__ __forceinline__ double wave_sum(double x) {
  x = row16_sum(x);
  return (lane_d(x, 0) + lane_d(x, 16)) + (lane_d(x, 32) + lane_d(x, 48));
}

__device__ __forceinline__ double wave_max(double x) {
  x = fmax(x, dpp<0xB1>(x));
  x = fmax(x, dpp<0x4E>(x));
  x = fmax(x, dpp<0x141>(x));
  x = fmax(x, dpp<0x140>(x));
  return fmax(fmax(lane_d(x, 0), lane_d(x, 16)), fmax(lane_d(x, 32), lane_d(x, 48)));
}

__device__ __forceinline__ double wave_min(double x) {
  x = fmin(x, dpp<0xB1>(x));
  x = fmin(x, dpp<0x4E>(x));
  x = fmin(x, dpp<0x141>(x));
  x = fmin(x, dpp<0x140>(x));
  return fmin(fmin(lane_d(x, 0), lane_d(x, 16)), fmin(lane_d(x, 32), lane_d(x, 48)));
}

// LDS written by this wave is visible to this wave's later reads (and the
// compiler may not move LDS accesses across it)
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// f64 reciprocal / reciprocal square root: hardware estimate + two Newton steps
__device__ __forceinline__ double rcp64(double d) {
  double r = __builtin_amdgcn_rcp(d);
  r = r * fma(-d, r, 2.0);
  r = r * fma(-d, r, 2.0);
  return r;
}
__device__ __forceinline__ double rsq64(double d) {
  double r = __builtin_amdgcn_rsq(d);
  r = r * fma(-0.5 * d * r, r, 1.5);
  r = r * fma(-0.5 * d * r, r, 1.5);
  return r;
}

// ------------------------------------------------------ Cholesky inverse
// X = R^{-1} (upper, k x k) of G = R^T R, by ONE wave (all 64 lanes call it).
// LDL^T elimination of the augmented [G | I] by columns, in place: lane c
// keeps column c of the live half in registers -- the trailing G column
// until pivot c, then column c of L^{-1} (L^{-1}[j][c] = 0 for c > j and
// G[.][c] is dead for c <= j, so one array serves both).  The multiplier of
// row i at pivot j is G[j][i] / d_j, held by lane i itself (the trailing
// block is symmetric), so a step is: readlane the pivot, every lane
// publishes its multiplier to LDS, one broadcast read, one FMA per live
// entry, and the pivot lane (exec-masked) switches its column to
// (0 .. 1, -f_{j+1} .. -f_{K-1}).  X[c][i] = L^{-1}[i][c] d_i^{-1/2}.  A pivot
// at or below 1e-13 max_i G_ii drops its direction (column and row of X
// zero) and sets bit 1 of *st.  G / X: LDS or global (ldg, ldx); fsh: >= 192
// doubles of 16-B aligned LDS.  k <= K <= 64; the padding is the identity.
template <int K>
__device__ __forceinline__ void wave_chol_inv(const double* G, int ldg, double* X, int ldx, int k, double* fsh,
                                              int* st) {
  static_assert(K % 2 == 0 && K <= 64, "K");
  const int c = threadIdx.x & 63;
  double A[K];
#pragma unroll
  for (int i = 0; i < K; ++i) A[i] = (i < k && c < k) ? G[i * ldg + c] : (i == c ? 1.0 : 0.0);
  const double thr = 1e-13 * wave_max(c < k ? fabs(G[c * ldg + c]) : 0.0);
  double* rsh = fsh + 128;   // d_j^{-1/2}
  int bad = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const double d = lane_d(A[j], j);
    const bool ok = (d > thr && d == d) || j >= k;
    bad |= !ok;
    const double r = ok ? rcp64(d) : 0.0;
    if (c == 0) rsh[j] = ok ? d : 0.0;      // d_j^{-1/2} formed after the loop (off the pivot chain)
    if (j + 1 < K) {
      double* fb_ = fsh + (j & 1) * 64;   // double-buffered: no second sync per step
      fb_[c] = A[j] * r;    // multiplier of row c (valid for c > j)
      wave_lds_sync();
      const double aj = A[j];
      // the pivot lane switches its column to (0 .. 1, -f_{j+1} .. -f_{K-1})
      // by a select on the same loaded multipliers (a divergent second pass
      // over them re-read every multiplier with the other lanes masked off)
      const bool piv = c == j;
#pragma unroll
      for (int i = (j + 1) & ~1; i < K; i += 2) {
        const double2 f = *(const double2*)(fb_ + i);
        if (i > j) A[i] = piv ? -f.x : fma(-f.x, aj, A[i]);
        A[i + 1] = piv ? -f.y : fma(-f.y, aj, A[i + 1]);
      }
    }
    if (c == j) A[j] = 1.0;
  }
  if (bad && c == 0) atomicOr(st, 1);
  wave_lds_sync();
  if (c < K) {
    const double dj = rsh[c];
    rsh[c] = dj > 0.0 ? rsq64(dj) : 0.0;
  }
  wave_lds_sync();
  if (c < k) {
#pragma unroll
    for (int i = 0; i < K; i += 2) {
      const double2 rr = *(const double2*)(rsh + i);
      if (i < k) X[c * ldx + i] = i >= c ? A[i] * rr.x : 0.0;
      if (i + 1 < k) X[c * ldx + i + 1] = i + 1 >= c ? A[i + 1] * rr.y : 0.0;
    }
  }
}

// The same X = R^{-1} with the rows of the elimination split over NW waves of
// the workgroup (every thread of the workgroup calls it; waves >= NW only
// meet the barriers).  Row i of [G | I] lives in wave i % NW, register
// i / NW, lane = column (the live-half trick as above: lane c holds column
// c of G's part until pivot c, then column c of L^{-1}).  Step j: the owner
// of row j publishes it to LDS (double-buffered, ONE workgroup barrier per
// step), every wave reads the pivot d_j and its lane's entry of row j, and
// updates its own rows below j with f_i = M[i][j] / d_j taken by readlane
// from lane j of the same row -- K / NW FMAs per lane and step instead of
// K - j on one wave (the one-wave form is issue-bound: time ~ K^2,
// profiles/r5/chol_wave_variants.md).  fsh >= 192 doubles of LDS.
template <int K, int NW>
__device__ __forceinline__ void wg_chol_inv(const double* G, int ldg, double* X, int ldx, int k, double* fsh,
                                            int* st) {
  static_assert(K % NW == 0 && K <= 64, "K");
  constexpr int R = K / NW;
  const int tid = threadIdx.x, c = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool act = w < NW;
  double* rowbuf = fsh;        // [2][64]
  double* dsh = fsh + 128;     // d_i (0: dropped)
  double M[R];
#pragma unroll
  for (int q = 0; q < R; ++q) {
    const int i = q * NW + w;
    M[q] = !act ? 0.0 : ((i < k && c < k) ? G[i * ldg + c] : (i == c ? 1.0 : 0.0));
  }
  const double thr = 1e-13 * wave_max(c < k ? fabs(G[c * ldg + c]) : 0.0);
  int bad = 0;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const int wj = j % NW, qj = j / NW;
    double* rb = rowbuf + (j & 1) * 64;
    if (w == wj) rb[c] = M[qj];
    __syncthreads();
    const double rj = rb[c];
    const double d = rb[j];
    const bool ok = (d > thr && d == d) || j >= k;
    bad |= !ok;
    const double r = ok ? rcp64(d) : 0.0;
    if (w == wj && c == 0) dsh[j] = ok ? d : 0.0;
    if (act) {
#pragma unroll
      for (int q = 0; q < R; ++q) {
        const int i = q * NW + w;
        if (i > j) {
          const double fi = lane_d(M[q], j) * r;
          M[q] = c == j ? -fi : fma(-fi, rj, M[q]);
        } else {
          M[q] = c == j ? (i == j ? 1.0 : 0.0) : M[q];
        }
      }
    }
  }
  if (bad && tid == 0) atomicOr(st, 1);
  __syncthreads();
  if (act && c < k) {
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int i = q * NW + w;
      if (i < k) {
        const double di = dsh[i];
        const double rs = di > 0.0 ? rsq64(di) : 0.0;
        X[c * ldx + i] = i >= c ? M[q] * rs : 0.0;
      }
    }
  }
}

// The same X with the elimination taken B pivots per step (B = 2 or 4): the
// owners of rows j .. j + B - 1 publish them (one barrier per block of
// pivots instead of one per pivot); every lane runs the block's own
// elimination on its column (the B x B pivot block's scalars -- pivots d and
// multipliers f -- are formed redundantly by every lane from broadcast
// reads), and each row i below the block takes all B updates at once: its
// multipliers m_t come from its block-column entries, read by symmetry of
// the trailing matrix as the published rows' entries at column i (broadcast
// LDS reads instead of cross-lane moves), m_t = (G[j+t][i] - sum_{s<t} m_s
// r'_s[j+t]) / d_t, then M[i][c] -= sum_t m_t r'_t[c] with the block's
// columns switching to their L^{-1} entries exactly as B single steps would
// leave them.  Pivot dropping as above.  K % B == 0, K % NW == 0; fsh >=
// 2 * B * 64 + 64 doubles of LDS (double-buffered pivot rows + d).  Every
// thread of the workgroup calls it (waves >= NW only meet the barriers).
// k = 40: 14.1 us (one pivot per step, 4 waves) -> see profiles/r6/chol_*.
template <int K, int NW, int B>
__device__ __forceinline__ void wg_chol_invB(const double* G, int ldg, double* X, int ldx, int k, double* fsh,
                                             int* st) {
  static_assert(K % NW == 0 && K % B == 0 && K <= 64 && (B == 2 || B == 4), "K");
  constexpr int R = K / NW;
  const int tid = threadIdx.x, c = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const bool act = w < NW;
  double* rowbuf = fsh;             // [2][B][64]
  double* dsh = fsh + 2 * B * 64;   // d_i (0: dropped)
  double M[R];
#pragma unroll
  for (int q = 0; q < R; ++q) {
    const int i = q * NW + w;
    M[q] = !act ? 0.0 : ((i < k && c < k) ? G[i * ldg + c] : (i == c ? 1.0 : 0.0));
  }
  const double thr = 1e-13 * wave_max(c < k ? fabs(G[c * ldg + c]) : 0.0);
  int bad = 0;
#pragma unroll
  for (int j = 0; j < K; j += B) {
    double* rb = rowbuf + ((j / B) & 1) * B * 64;
#pragma unroll
    for (int t = 0; t < B; ++t)
      if (w == (j + t) % NW) rb[t * 64 + c] = M[(j + t) / NW];
    __syncthreads();
    // the block rows at this lane's column, and the B x B pivot block
    double rl[B], pb[B][B];
#pragma unroll
    for (int t = 0; t < B; ++t) {
      rl[t] = rb[t * 64 + c];
#pragma unroll
      for (int u = 0; u < B; ++u) pb[t][u] = rb[t * 64 + j + u];
    }
    // the block's elimination: pivots d_t, multipliers f[u][t] (u > t); pb
    // and rl updated in place (pb[u][v], v > t: row u's trailing entries)
    double rc[B], f[B][B];
#pragma unroll
    for (int t = 0; t < B; ++t) {
      const double d = pb[t][t];
      const bool ok = (d > thr && d == d) || j + t >= k;
      bad |= !ok;
      rc[t] = ok ? rcp64(d) : 0.0;
      if (tid == 0) dsh[j + t] = ok ? d : 0.0;
#pragma unroll
      for (int u = t + 1; u < B; ++u) {
        f[u][t] = pb[u][t] * rc[t];
#pragma unroll
        for (int v = t + 1; v < B; ++v) pb[u][v] = fma(-f[u][t], pb[t][v], pb[u][v]);
        rl[u] = c == j + t ? -f[u][t] : fma(-f[u][t], rl[t], rl[u]);
      }
    }
    if (act) {
#pragma unroll
      for (int q = 0; q < R; ++q) {
        const int i = q * NW + w;   // wave-uniform
        if (i >= j + B) {
          // multipliers from the block rows' entries at column i (symmetry)
          double a[B], m[B];
#pragma unroll
          for (int t = 0; t < B; ++t) a[t] = rb[t * 64 + i];
#pragma unroll
          for (int t = 0; t < B; ++t) {
            m[t] = a[t] * rc[t];
#pragma unroll
            for (int v = t + 1; v < B; ++v) a[v] = fma(-m[t], pb[t][v], a[v]);
          }
          double x = M[q];
#pragma unroll
          for (int t = 0; t < B; ++t) x = c == j + t ? -m[t] : fma(-m[t], rl[t], x);
          M[q] = x;
        } else if (i >= j) {
          // a block row: its eliminated row, 1 on its pivot, 0 right of it in the block
          const int u = i - j;
          double x = rl[0];
#pragma unroll
          for (int t = 1; t < B; ++t) x = u == t ? rl[t] : x;
          M[q] = c == i ? 1.0 : ((c > i && c < j + B) ? 0.0 : x);
        } else {
          M[q] = (c >= j && c < j + B) ? 0.0 : M[q];
        }
      }
    }
  }
  if (bad && tid == 0) atomicOr(st, 1);
  __syncthreads();
  if (act && c < k) {
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int i = q * NW + w;
      if (i < k) {
        const double di = dsh[i];
        const double rs = di > 0.0 ? rsq64(di) : 0.0;
        X[c * ldx + i] = i >= c ? M[q] * rs : 0.0;
      }
    }
  }
}

// The B-pivot elimination for 64 < k <= 128: a row of [G | I] spans TWO
// waves (thread column c = tid & 127) and the rows cycle over the NG =
// blockDim / 128 row groups (row i in group i % NG, register i / NG).
// Everything else -- the block rows published to LDS once per B pivots, the
// pivot block formed redundantly by every thread, the multipliers of row i
// read by symmetry from the published rows at column i (one broadcast LDS
// read per block row), pivot dropping -- is wg_chol_invB's.  NG % B == 0 so
// the B block rows sit in B different groups.  fsh >= 2 * B * 128 + 136
// doubles of 16-B aligned LDS.  Every thread of the (NG * 128)-thread
// workgroup calls it.  The general randSVD engine's CholeskyQR at k = 65 ..
// 128 (eigen-whitening on rocSOLVER syevd before: ~2.4 ms per factor).
template <int K, int NG, int B>
__device__ __forceinline__ void wg_chol_invW(const double* G, int ldg, double* X, int ldx, int k, double* fsh,
                                             int* st) {
  static_assert(K % NG == 0 && K % B == 0 && K <= 128 && NG % B == 0 && (B == 2 || B == 4), "K");
  constexpr int R = K / NG, CW = 128;
  const int tid = threadIdx.x, c = tid & (CW - 1);
  const int g = __builtin_amdgcn_readfirstlane(tid >> 7);
  double* rowbuf = fsh;              // [2][B][128]
  double* dsh = fsh + 2 * B * CW;    // d_i (0: dropped)
  double* red = dsh + CW;            // max G_ii
  double M[R];
#pragma unroll
  for (int q = 0; q < R; ++q) {
    const int i = q * NG + g;
    M[q] = (i < k && c < k) ? G[i * ldg + c] : (i == c ? 1.0 : 0.0);
  }
  if (tid < 64) {
    const double a = tid < k ? fabs(G[tid * ldg + tid]) : 0.0;
    const double b = tid + 64 < k ? fabs(G[(tid + 64) * ldg + tid + 64]) : 0.0;
    const double mx = wave_max(fmax(a, b));
    if (tid == 0) red[0] = mx;
  }
  __syncthreads();
  const double thr = 1e-13 * red[0];
  int bad = 0;
#pragma unroll 1
  for (int j = 0; j < K; j += B) {
    double* rb = rowbuf + ((j / B) & 1) * B * CW;
#pragma unroll
    for (int t = 0; t < B; ++t)
      if (g == (j + t) % NG) {
        // (j + t) / NG is this group's register of row j + t; R is small and
        // the index is wave-uniform, so a select chain keeps M in registers
        const int qj = (j + t) / NG;
        double v = M[0];
#pragma unroll
        for (int q = 1; q < R; ++q) v = q == qj ? M[q] : v;
        rb[t * CW + c] = v;
      }
    __syncthreads();
    double rl[B], pb[B][B];
#pragma unroll
    for (int t = 0; t < B; ++t) {
      rl[t] = rb[t * CW + c];
#pragma unroll
      for (int u = 0; u < B; ++u) pb[t][u] = rb[t * CW + j + u];
    }
    double rc[B], f[B][B];
#pragma unroll
    for (int t = 0; t < B; ++t) {
      const double d = pb[t][t];
      const bool ok = (d > thr && d == d) || j + t >= k;
      bad |= !ok;
      rc[t] = ok ? rcp64(d) : 0.0;
      if (tid == 0) dsh[j + t] = ok ? d : 0.0;
#pragma unroll
      for (int u = t + 1; u < B; ++u) {
        f[u][t] = pb[u][t] * rc[t];
#pragma unroll
        for (int v = t + 1; v < B; ++v) pb[u][v] = fma(-f[u][t], pb[t][v], pb[u][v]);
        rl[u] = c == j + t ? -f[u][t] : fma(-f[u][t], rl[t], rl[u]);
      }
    }
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int i = q * NG + g;   // wave-uniform
      if (i >= j + B) {
        double a[B], m[B];
#pragma unroll
        for (int t = 0; t < B; ++t) a[t] = rb[t * CW + i];
#pragma unroll
        for (int t = 0; t < B; ++t) {
          m[t] = a[t] * rc[t];
#pragma unroll
          for (int v = t + 1; v < B; ++v) a[v] = fma(-m[t], pb[t][v], a[v]);
        }
        double x = M[q];
#pragma unroll
        for (int t = 0; t < B; ++t) x = c == j + t ? -m[t] : fma(-m[t], rl[t], x);
        M[q] = x;
      } else if (i >= j) {
        const int u = i - j;
        double x = rl[0];
#pragma unroll
        for (int t = 1; t < B; ++t) x = u == t ? rl[t] : x;
        M[q] = c == i ? 1.0 : ((c > i && c < j + B) ? 0.0 : x);
      } else {
        M[q] = (c >= j && c < j + B) ? 0.0 : M[q];
      }
    }
  }
  if (bad && tid == 0) atomicOr(st, 1);
  __syncthreads();
  if (c < k) {
#pragma unroll
    for (int q = 0; q < R; ++q) {
      const int i = q * NG + g;
      if (i < k) {
        const double di = dsh[i];
        const double rs = di > 0.0 ? rsq64(di) : 0.0;
        X[c * ldx + i] = i >= c ? M[q] * rs : 0.0;
      }
    }
  }
}

// ------------------------------------------------- tridiagonalisation
// T = Q^T C Q, Q = H_0 H_1 ... H_{K-3}, H_j = I - 2 v_j v_j^T, by ONE wave:
// lane i keeps row i of the trailing matrix in registers.  Step j: ||x||
// of column j below the diagonal (DPP sum), v, p = A v (broadcast v through
// LDS), K_j = v^T p (DPP sum), w = 2 (p - K_j v), A -= v w^T + w v^T.
// Output: dd[0..K-1], ee[0..K-2] (ee[j] = T[j+1][j]), refl[i * ldr + j] =
// (v_j)_i (zero for i <= j).  The k x k input C (ldc) is padded to K with
// -beta on the diagonal (beta > ||C||_2), so the padding's eigenvalues sit
// below every eigenvalue of C and the top ones are C's.
template <int K, int J>
__device__ __forceinline__ void tri_step(double (&arow)[K], int i, double* vsh, double* wsh, double* refl, int ldr,
                                         double* dd, double* ee) {
  constexpr int c0 = (J + 1) & ~1;
  // ||x||^2 of column J below the diagonal and its first entry, from the
  // column itself (lane i > J holds x_i): the rank-2 updates keep the
  // register matrix symmetric only to rounding, and a norm taken from row J
  // while v is built from column J left H non-orthogonal by eps ||A|| / ||x||
  // (backward errors of 1e-12 on graded trailing blocks)
  const double xi = (i > J) ? arow[J] : 0.0;
  const double s2 = wave_sum(xi * xi);
  const double x0 = lane_d(arow[J], J + 1);
  const double sig2 = s2 - x0 * x0;
  const bool refl_on = sig2 > 1e-300;
  // sqrt(s2) as s2 / sqrt(s2) on the rsq estimate + Newton (shorter chain
  // than the library sqrt's denormal-scaling sequence; s2 > 1e-300 here)
  const double rs = rsq64(refl_on ? s2 : 1.0);
  const double alpha = refl_on ? (x0 >= 0.0 ? -s2 * rs : s2 * rs) : x0;
  const double rn = refl_on ? rsq64(2.0 * (s2 - alpha * x0)) : 0.0;
  const double vi = (i > J) ? (xi - (i == J + 1 ? alpha : 0.0)) * rn : 0.0;
  if (i == J) { dd[J] = arow[J]; ee[J] = alpha; }
  if (i < K) {
    vsh[i] = vi;
    refl[i * ldr + J] = vi;
  }
  wave_lds_sync();
  // p = A v, v streamed from LDS in pairs (entry J, when the first pair
  // starts there, has v_J = 0)
  double p0 = 0.0, p1 = 0.0, p2 = 0.0, p3 = 0.0;
#pragma unroll
  for (int c = c0; c < K; c += 4) {
    const double2 t = *(const double2*)(vsh + c);
    p0 = fma(arow[c], t.x, p0);
    p1 = fma(arow[c + 1], t.y, p1);
    if (c + 2 < K) {
      const double2 u = *(const double2*)(vsh + c + 2);
      p2 = fma(arow[c + 2], u.x, p2);
      p3 = fma(arow[c + 3], u.y, p3);
    }
    // (K >= 48: a compiler barrier per 16 entries keeps the streamed reads
    // from all being hoisted ahead -- that spilled the K = 48 / 64 rows)
    if constexpr (K >= 48)
      if (((c - c0) & 15) == 12) asm volatile("" ::: "memory");
  }
  const double p = (p0 + p1) + (p2 + p3);
  const double Kd = wave_sum(vi * p);
  const double wi = (i > J) ? 2.0 * (p - Kd * vi) : 0.0;
  if (i < K) wsh[i] = wi;
  wave_lds_sync();
  // A -= v w^T + w v^T on the trailing columns (v, w streamed again)
#pragma unroll
  for (int c = c0; c < K; c += 2) {
    const double2 tv = *(const double2*)(vsh + c);
    const double2 tw = *(const double2*)(wsh + c);
    arow[c] = fma(-vi, tw.x, fma(-wi, tv.x, arow[c]));
    arow[c + 1] = fma(-vi, tw.y, fma(-wi, tv.y, arow[c + 1]));
    if constexpr (K >= 48)
      if (((c - c0) & 15) == 14) asm volatile("" ::: "memory");
  }
}

// vsh / wsh: 2 x K doubles each (alternate steps use alternate halves, so a
// step's writes never meet the previous step's reads)
template <int K, int J>
__device__ __forceinline__ void tri_steps(double (&arow)[K], int i, double* vsh, double* wsh, double* refl, int ldr,
                                          double* dd, double* ee) {
  if constexpr (J + 2 < K) {
    tri_step<K, J>(arow, i, vsh + (J & 1) * K, wsh + (J & 1) * K, refl, ldr, dd, ee);
    tri_steps<K, J + 1>(arow, i, vsh, wsh, refl, ldr, dd, ee);
  }
}

// returns ||T||-scale (max |Gershgorin bound|) in every lane; *bad |= non-finite input
template <int K>
__device__ __forceinline__ void wave_tridiag(const double* C, int ldc, int k, double* refl, int ldr, double* dd,
                                             double* ee, double* vsh, double* wsh, int* bad) {
  const int i = threadIdx.x & 63;
  double arow[K];
  double f2 = 0.0;
  int nf = 0;
#pragma unroll
  for (int c = 0; c < K; ++c) {
    const double v = (i < k && c < k) ? C[i * ldc + c] : 0.0;
    nf |= !(fabs(v) <= 1.7e308);
    f2 = fma(v, v, f2);
    arow[c] = v;
  }
  if (nf) atomicOr(bad, 1);
  const double beta = 1.0625 * sqrt(wave_sum(f2)) + 1e-300;   // > ||C||_F >= -lambda_min
#pragma unroll
  for (int c = 0; c < K; ++c)
    if (c >= k && c == i) arow[c] = -beta;
  tri_steps<K, 0>(arow, i, vsh, wsh, refl, ldr, dd, ee);
  // the last 2 x 2 block
  if (i == K - 2) dd[K - 2] = arow[K - 2];
  if (i == K - 1) {
    dd[K - 1] = arow[K - 1];
    ee[K - 2] = arow[K - 2];
    ee[K - 1] = 0.0;
  }
  wave_lds_sync();
}

// The same T by FOUR waves: wave w keeps columns [w K/4, (w + 1) K/4) of
// the trailing matrix (lane = row).  Step J: the wave owning column J forms
// v (norm by DPP sum, as above) and publishes it; barrier; every wave forms
// its columns' share of p = A v; barrier; every wave sums the four shares,
// K_J = v^T p (DPP sum), w = 2 (p - K_J v), and updates its own columns
// (w_c by readlane).  Two barriers per step against the single wave's two
// LDS round trips, and a quarter of the step's FMAs per wave.  Columns
// already reduced take the (zero) updates of v_c = w_c = 0 instead of a
// branch.  vsh: >= 128 doubles, psh: >= 256 doubles (LDS).  Every thread of
// the workgroup calls it (waves >= 4 only meet the barriers).
template <int K, int J>
__device__ __forceinline__ void wtri_steps(double (&acol)[K / 4], int i, int w, double* vsh, double* psh,
                                           double* refl, int ldr, double* dd, double* ee) {
  if constexpr (J + 2 < K) {
    constexpr int CW = K / 4, OW = J / CW, LC = J % CW;
    const bool act = w < 4;
    double* vb = vsh + (J & 1) * 64;
    if (w == OW) {
      const double xi = (i > J) ? acol[LC] : 0.0;
      const double s2 = wave_sum(xi * xi);
      const double x0 = lane_d(acol[LC], J + 1);
      const double sig2 = s2 - x0 * x0;
      const bool refl_on = sig2 > 1e-300;
      const double rs = rsq64(refl_on ? s2 : 1.0);
      const double alpha = refl_on ? (x0 >= 0.0 ? -s2 * rs : s2 * rs) : x0;
      const double rn = refl_on ? rsq64(2.0 * (s2 - alpha * x0)) : 0.0;
      const double vi = (i > J) ? (xi - (i == J + 1 ? alpha : 0.0)) * rn : 0.0;
      if (i == J) { dd[J] = acol[LC]; ee[J] = alpha; }
      vb[i] = i < K ? vi : 0.0;
      if (i < K) refl[i * ldr + J] = vi;
    }
    __syncthreads();
    double vi = 0.0;
    if (act) {
      vi = vb[i];
      double p0 = 0.0, p1 = 0.0;
#pragma unroll
      for (int l = 0; l < CW; l += 2) {
        p0 = fma(acol[l], vb[w * CW + l], p0);
        if (l + 1 < CW) p1 = fma(acol[l + 1], vb[w * CW + l + 1], p1);
      }
      psh[w * 64 + i] = p0 + p1;
    }
    __syncthreads();
    if (act) {
      const double p = (psh[i] + psh[64 + i]) + (psh[128 + i] + psh[192 + i]);
      const double Kd = wave_sum(vi * p);
      const double wi = (i > J) ? 2.0 * (p - Kd * vi) : 0.0;
#pragma unroll
      for (int l = 0; l < CW; ++l) {
        const int c = w * CW + l;
        acol[l] = fma(-vi, lane_d(wi, c), fma(-wi, vb[c], acol[l]));
      }
    }
    wtri_steps<K, J + 1>(acol, i, w, vsh, psh, refl, ldr, dd, ee);
  }
}

template <int K>
__device__ __forceinline__ void wg_tridiag(const double* C, int ldc, int k, double* refl, int ldr, double* dd,
                                           double* ee, double* vsh, double* psh, int* bad) {
  static_assert(K % 4 == 0 && K <= 64, "K");
  constexpr int CW = K / 4;
  const int i = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool act = w < 4;
  double acol[CW];
  double f2 = 0.0;
  int nf = 0;
#pragma unroll
  for (int l = 0; l < CW; ++l) {
    const int c = w * CW + l;
    const double v = (act && i < k && c < k) ? C[i * ldc + c] : 0.0;
    nf |= !(fabs(v) <= 1.7e308);
    f2 = fma(v, v, f2);
    acol[l] = v;
  }
  if (act) {
    f2 = wave_sum(f2);
    if (i == 0) psh[w] = f2;
    if (nf) atomicOr(bad, 1);
  }
  if (threadIdx.x < 128) vsh[threadIdx.x] = 0.0;
  __syncthreads();
  const double beta = 1.0625 * sqrt((psh[0] + psh[1]) + (psh[2] + psh[3])) + 1e-300;   // > ||C||_F
  __syncthreads();
#pragma unroll
  for (int l = 0; l < CW; ++l) {
    const int c = w * CW + l;
    if (act && c >= k && c == i) acol[l] = -beta;
  }
  wtri_steps<K, 0>(acol, i, w, vsh, psh, refl, ldr, dd, ee);
  // the last 2 x 2 block
  constexpr int W2 = (K - 2) / CW, L2 = (K - 2) % CW, W1 = (K - 1) / CW, L1 = (K - 1) % CW;
  if (w == W2 && i == K - 2) dd[K - 2] = acol[L2];
  if (w == W2 && i == K - 1) ee[K - 2] = acol[L2];
  if (w == W1 && i == K - 1) {
    dd[K - 1] = acol[L1];
    ee[K - 1] = 0.0;
  }
  __syncthreads();
}

// ------------------------------------------- symmetric tridiagonal eigen
// Sturm counts of eigenvalues of T below P points at once, division-free:
// the characteristic polynomials p_i(x) (p_{i+1} = (d_i - x) p_i - e_{i-1}^2
// p_{i-1}); a sign change between p_i and p_{i+1} is a negative LDL^T pivot.
// T is pre-scaled to ||T|| ~ 1 and p is re-normalised every 8 steps
// (exponent only), so nothing over- or underflows.  One FMA of latency per
// step and point; the P chains interleave.  (An exactly zero p_i -- measure
// zero -- counts as positive, i.e. the count of a point a rounding error
// away.)
template <int K, int P>
__device__ __forceinline__ void sturm_counts(const double2* de2, const double (&x)[P], int (&cnt)[P]) {
  // (d_i, e_{i-1}^2) broadcast from LDS, fetched PF steps ahead into a
  // register ring (a full register copy of T per lane -- 4 K VGPRs, the same
  // values in every lane -- spilled the K >= 48 solvers)
  constexpr int PF = SLW_STURM_PF < K ? SLW_STURM_PF : K;
  double2 ring[PF];
#pragma unroll
  for (int q = 0; q < PF; ++q)
    if (q < K) ring[q] = de2[q];
  double p[P], pp[P];
  {
    const double2 t0 = ring[0];
    if (PF < K) ring[0] = de2[PF];
#pragma unroll
    for (int q = 0; q < P; ++q) {
      pp[q] = 1.0;
      p[q] = t0.x - x[q];
      cnt[q] = p[q] < 0.0;
    }
  }
#pragma unroll
  for (int i = 1; i < K; ++i) {
    const double2 t = ring[i % PF];
    if (i + PF < K) ring[i % PF] = de2[i + PF];
    asm volatile("" ::: "memory");
#pragma unroll
    for (int q = 0; q < P; ++q) {
      const double pn = fma(t.x - x[q], p[q], -t.y * pp[q]);
      cnt[q] += (pn < 0.0) != (p[q] < 0.0);
      pp[q] = p[q];
      p[q] = pn;
    }
    if ((i & 7) == 7) {
#pragma unroll
      for (int q = 0; q < P; ++q) {
        const int ex = __builtin_amdgcn_frexp_exp(p[q]);
        p[q] = __builtin_amdgcn_ldexp(p[q], -ex);
        pp[q] = __builtin_amdgcn_ldexp(pp[q], -ex);
      }
    }
  }
}

__device__ __forceinline__ double rcp64n(double d) {   // estimate + one Newton step
  const double r = __builtin_amdgcn_rcp(d);
  return r * fma(-d, r, 2.0);
}

// Eigenvector of the (scaled) tridiagonal T for the eigenvalue l by the
// twisted factorisation T - l I = N_r D_r N_r^T, one lane per vector:
// backward pivots D-_i and forward pivots D+_i, the twist r = argmin
// |gamma_i|, then z by the two one-term recurrences.  zdm receives z
// (unnormalised), zdp / zrd are scratch; the return value is 1 / ||z||.
// The d / e operands (LDS broadcasts) are fetched PF steps ahead into a
// register ring, with a compiler barrier per step: the pivot chain never
// waits on an LDS round trip, and the loads are not all hoisted to the top
// (which spilled the unrolled K = 40 chain to scratch).
template <int K>
__device__ __forceinline__ void twisted_vec(const double* dd, const double* ee, double l, double* zdm, double* zdp,
                                            double* zrd, int* rt_out) {
  constexpr int PF = SLW_TWIST_PF < K - 1 ? SLW_TWIST_PF : K - 1;
  const double pivmin = 1e-290;
  double dm = dd[K - 1] - l;
  if (fabs(dm) < pivmin) dm = -pivmin;
  zdm[K - 1] = dm;
  double dp = dd[0] - l;
  if (fabs(dp) < pivmin) dp = -pivmin;
  zdp[0] = dp;
  // ring slot q holds the operands of step s_ = q (mod PF)
  double rb_e[PF], rb_d[PF], rf_e[PF], rf_d[PF];
#pragma unroll
  for (int q = 0; q < PF; ++q)
    if (q < K - 1) {
      rb_e[q] = ee[K - 2 - q];
      rb_d[q] = dd[K - 2 - q];
      rf_e[q] = ee[q];
      rf_d[q] = dd[q + 1];
    }
#pragma unroll
  for (int s_ = 0; s_ < K - 1; ++s_) {
    const int ib = K - 2 - s_, jf = s_ + 1, q = s_ % PF;
    const double eb = rb_e[q], db = rb_d[q], ef = rf_e[q], df = rf_d[q];
    if (s_ + PF < K - 1) {
      rb_e[q] = ee[ib - PF];
      rb_d[q] = dd[ib - PF];
      rf_e[q] = ee[jf - 1 + PF];
      rf_d[q] = dd[jf + PF];
    }
    asm volatile("" ::: "memory");
    const double rdm = rcp64n(dm);        // 1 / D-_{ib+1}
    zrd[ib + 1] = -eb * rdm;
    dm = (db - l) - (eb * eb) * rdm;
    if (fabs(dm) < pivmin) dm = -pivmin;
    zdm[ib] = dm;
    const double rdp = rcp64n(dp);        // 1 / D+_{jf-1}
    dp = (df - l) - (ef * ef) * rdp;
    if (fabs(dp) < pivmin) dp = -pivmin;
    zdp[jf] = dp;
  }
  // the twist: argmin |gamma_i|, gamma_i = D+_i + D-_i - (d_i - l)
  int rt = 0;
  double best = 1e300;
#pragma unroll
  for (int i = 0; i < K; ++i) {
    const double gm = fabs(zdp[i] + zdm[i] - (dd[i] - l));
    if (gm < best) { best = gm; rt = i; }
    if ((i & 7) == 7) asm volatile("" ::: "memory");
  }
  // above the twist: z_i = -(e_i / D+_i) z_{i+1} (the reciprocals formed
  // again here, off the z chain), into zdp; below: z_i = ratio_i z_{i-1},
  // into zrd.  Branch-free: every lane runs both full recurrences with z
  // held at 1 outside its range (a masked branch per entry cost more than
  // the arithmetic); the caller picks zdp / 1 / zrd by the twist (*rt_out).
  double z = 1.0;
#pragma unroll
  for (int i = K - 2; i >= 0; --i) {
    const double f = -(ee[i] * rcp64n(zdp[i]));
    z = i < rt ? f * z : 1.0;
    zdp[i] = z;
    if ((i & 7) == 0) asm volatile("" ::: "memory");
  }
  z = 1.0;
  asm volatile("" ::: "memory");
#pragma unroll
  for (int i = 1; i < K; ++i) {
    const double rd = zrd[i];           // loaded unconditionally: a load inside the select
    z = i > rt ? rd * z : 1.0;          // became a branch with an LDS round trip per entry
    zrd[i] = z;
    if ((i & 7) == 7) asm volatile("" ::: "memory");
  }
  *rt_out = rt;
}

// Eigenpairs of the symmetric K x K matrix given by its tridiagonal form
// (dd, ee) and reflectors (refl): the nt largest eigenvalues, descending,
// in lam[0..nt-1] and the eigenvectors of the ORIGINAL matrix (Q x) for the
// first nv <= 64 of them in X[i * ldx + t] (rows i < kx <= K).  Every thread of the
// workgroup (NT threads, NT % 64 == 0) calls it; dd / ee are overwritten
// (scaled).  Scratch: sc >= 3 nv (K + 1) doubles of LDS.  *st bit 1: numerically repeated eigenvalues among the
// wanted ones, a vector that fails the residual check or non-finite values --
// the caller should fall back to a robust solver.
template <int K, int NT>
__device__ __forceinline__ void sym_top_eig(double* dd, double* ee, const double* refl, int ldr, int nt, int nv,
                                            double* lam, double* X, int ldx, int kx, double* sc, int* st) {
  const int tid = threadIdx.x, lane = tid & 63;
  __shared__ double s_scale;
  __shared__ int s_clus;
  __shared__ double2 de2[K];
  // ---- scale to ||T|| ~ 1 (Gershgorin radius)
  if (tid < 64) {
    const int i = lane;
    double g = 0.0;
    if (i < K) g = fabs(dd[i]) + fabs(ee[i]) + (i > 0 ? fabs(ee[i - 1]) : 0.0);
    g = wave_max(g);
    if (lane == 0) { s_scale = g > 0.0 ? g : 1.0; s_clus = 0; }
  }
  __syncthreads();
  const double tn = s_scale, itn = 1.0 / tn;
  if (tid < K) {
    const double em = tid > 0 ? ee[tid - 1] * itn : 0.0;
    de2[tid] = double2{dd[tid] * itn, em * em};
  }
  __syncthreads();
  // ---- multisection: 8 lanes (a DPP half-row) per eigenvalue, one point
  //      per lane (bracket / 9 per round).  The Sturm count is issue-bound
  //      (~9 VALU per point and step): 16 lanes x 2 points put 21 wanted
  //      eigenvalues on 5.25 waves, two waves on some SIMD, for 5 bits per
  //      round; 8 x 1 fits them on 3 waves (one per SIMD) for 3.2 bits per
  //      round at a quarter of the issue per round (measured 58k -> see
  //      profiles/r4).  T streamed from LDS.
  constexpr double eps = 2.220446049250313e-16;
  constexpr int LPE = 8;
  // eigenvalues closer than CLUS (scaled: ||T|| = 1) are orthogonalised
  // against each other; farther apart the twisted vectors are orthogonal to
  // ~eps / gap < 1e-11 on their own
  constexpr double CLUS = 1e-4;
  const int row = tid / LPE, g = tid % LPE;
  constexpr int ROWS = NT / LPE;
  static_assert(NT % 256 == 0, "NT: whole groups of four waves");
  // eigenvalue of this row: consecutive t go to consecutive SIMDs (wave w
  // runs on SIMD w % 4), so the nt active rows fill one wave per SIMD first
  const int wv_ = row >> 3, tmap = (((wv_ >> 2) << 3) + (row & 7)) * 4 + (wv_ & 3);
  {
    for (int t0 = 0; t0 < nt; t0 += ROWS) {
      const int t = t0 + tmap;
      const bool act = t < nt;
      const int idx = K - 1 - t;   // ascending index of this row's eigenvalue
      double lo = -1.0 - 4.0 * eps, hi = 1.0 + 4.0 * eps;
      for (int it = 0; it < 96; ++it) {
        // absolute accuracy 2 eps ||T|| (||T|| = 1 after the scaling): what the
        // backward-stable reduction determines; resolving tiny eigenvalues to
        // full relative precision cost ~20 more bits
        const bool conv = !act || (hi - lo) <= 4.0 * eps;
        if (__builtin_amdgcn_ballot_w64(!conv) == 0) break;
        double x[1];
        int c[1];
        x[0] = lo + (hi - lo) * (double)(g + 1) * (1.0 / (LPE + 1));
        sturm_counts<K, 1>(de2, x, c);
        // fewer than idx + 1 eigenvalues below x: x is a lower bound
        double nlo = c[0] <= idx ? fmax(lo, x[0]) : lo;
        double nhi = c[0] <= idx ? hi : fmin(hi, x[0]);
        nlo = fmax(nlo, dpp<0xB1>(nlo));
        nhi = fmin(nhi, dpp<0xB1>(nhi));
        nlo = fmax(nlo, dpp<0x4E>(nlo));
        nhi = fmin(nhi, dpp<0x4E>(nhi));
        nlo = fmax(nlo, dpp<0x141>(nlo));
        nhi = fmin(nhi, dpp<0x141>(nhi));
        if (act && !conv) { lo = nlo; hi = nhi; }
      }
      if (act && g == 0) lam[t] = 0.5 * (lo + hi);   // scaled
    }
  }
  __syncthreads();
  // ---- eigenvectors of T: one lane per vector (twisted factorisation of
  //      the scaled T - l I).  Per lane t: zdm = sc[t * LZ + i] holds the
  //      backward pivots D-_i (later the vector), zdp the forward pivots, zrd
  //      the ratios -e_{i-1} / D-_i below the twist; the reciprocals of the
  //      forward pivots stay in registers.  The backward and forward chains
  //      run interleaved in one loop; d / e come from LDS (broadcast reads).
  constexpr int LZ = K + 1;   // sc[t * LZ + i]: vector t, component i
  if (tid < K) {
    dd[tid] *= itn;
    ee[tid] *= itn;
  }
  __syncthreads();
  // vector t on wave t % 4, lane t / 4: the per-vector chains (f64 VALU
  // issue-bound) spread over the four SIMDs instead of one wave
  const int tv = (tid >> 6) < 4 ? (tid & 63) * 4 + (tid >> 6) : nv;
  if (tv < nv) {
    const int t = tv;
    const double l = lam[t];
    const double gap = fmin(t > 0 ? lam[t - 1] - l : 1e300, t + 1 < nt ? l - lam[t + 1] : 1e300);
    if (!(gap > 1e-13)) atomicOr(st, 1);       // numerically repeated (~ bisection accuracy): the caller falls back
    if (gap < CLUS) atomicOr(&s_clus, 1);
    int rt;
    twisted_vec<K>(dd, ee, l, sc + t * LZ, sc + (nv + t) * LZ, sc + (2 * nv + t) * LZ, &rt);
    // the normalised vector into sc[t * LZ + .] (its own lane's scratch):
    // the pieces gathered and squared from LDS, then scaled (the norm summed
    // inside the z recurrences held all of z live and spilled it)
    asm volatile("" ::: "memory");
    const double* za = sc + (nv + t) * LZ;
    const double* zb = sc + (2 * nv + t) * LZ;
    double n0 = 0.0, n1 = 0.0;
#pragma unroll
    for (int i = 0; i < K; i += 2) {
      const double xa0 = za[i], xb0 = zb[i], xa1 = za[i + 1], xb1 = zb[i + 1];
      const double a0 = i < rt ? xa0 : (i > rt ? xb0 : 1.0);
      const double a1 = i + 1 < rt ? xa1 : (i + 1 > rt ? xb1 : 1.0);
      sc[t * LZ + i] = a0;
      sc[t * LZ + i + 1] = a1;
      n0 = fma(a0, a0, n0);
      n1 = fma(a1, a1, n1);
      if ((i & 7) == 6) asm volatile("" ::: "memory");
    }
    const double s = rsq64(n0 + n1);
    if (!(s > 0.0) || !(s < 1e300)) atomicOr(st, 1);
    asm volatile("" ::: "memory");
#pragma unroll
    for (int i = 0; i < K; ++i) {
      sc[t * LZ + i] *= s;
      if ((i & 7) == 7) asm volatile("" ::: "memory");
    }
  }
  __syncthreads();
  // ---- MGS inside close clusters (rare): wave 0, lane = component.  Two
  //      passes ("twice is enough"): inside a tight cluster the twisted
  //      vectors can be nearly parallel, and one pass then leaves a small
  //      remainder that is not orthogonal to the others.  A vector that
  //      vanishes under both passes flags the core (Jacobi re-solve).
  if (s_clus && tid < 64) {
    const int i = lane;
    for (int t = 1; t < nv; ++t) {
      double xc = i < K ? sc[t * LZ + i] : 0.0;
      bool touched = false;
      for (int pass = 0; pass < 2; ++pass) {
        for (int u = 0; u < t; ++u) {
          if (lam[u] - lam[t] >= CLUS) continue;
          const double dt = wave_sum(i < K ? sc[u * LZ + i] * xc : 0.0);
          xc -= dt * (i < K ? sc[u * LZ + i] : 0.0);
          touched = true;
        }
        if (!touched) break;
      }
      if (touched) {
        const double n2 = wave_sum(xc * xc);
        if (!(n2 > 1e-24) && lane == 0) atomicOr(st, 1);
        if (i < K) sc[t * LZ + i] = xc * rsq64(n2);
      }
      wave_lds_sync();
    }
  }
  __syncthreads();
  // ---- residual check of every vector against T (scaled), one lane per
  //      vector, spread over the SIMDs as above
  if (tv < nv) {
    const int t = tv;
    const double l = lam[t];
    double r2 = 0.0;
#pragma unroll
    for (int i = 0; i < K; ++i) {
      double tx = (dd[i] - l) * sc[t * LZ + i];
      if (i > 0) tx = fma(ee[i - 1], sc[t * LZ + i - 1], tx);
      if (i + 1 < K) tx = fma(ee[i], sc[t * LZ + i + 1], tx);
      r2 = fma(tx, tx, r2);
    }
    if (!(r2 <= 1e-22)) atomicOr(st, 1);
  }
  // ---- back-transform x <- H_0 ... H_{K-3} x: 16 lanes (a DPP row) per vector
  {
    constexpr int U = (K + 15) / 16;
    const int v = tid >> 4, q = tid & 15;
    for (int vb = 0; vb < nv; vb += NT / 16) {
      const int vv_ = vb + v;
      const bool act = vv_ < nv;
      double x[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = q + 16 * u;
        x[u] = (act && i < K) ? sc[vv_ * (K + 1) + i] : 0.0;
      }
#pragma unroll 2
      for (int j = K - 3; j >= 0; --j) {
        double h[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int i = q + 16 * u;
          h[u] = i < K ? refl[i * ldr + j] : 0.0;
        }
        double part = 0.0;
#pragma unroll
        for (int u = 0; u < U; ++u) part = fma(h[u], x[u], part);
        part = 2.0 * row16_sum(part);
#pragma unroll
        for (int u = 0; u < U; ++u) x[u] = fma(-part, h[u], x[u]);
      }
      if (act) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int i = q + 16 * u;
          if (i < kx) X[i * ldx + vv_] = x[u];
        }
      }
    }
  }
  __syncthreads();
  // eigenvalues back to the matrix's scale
  for (int t = tid; t < nt; t += NT) lam[t] *= tn;
  __syncthreads();
}

}  // namespace slw
