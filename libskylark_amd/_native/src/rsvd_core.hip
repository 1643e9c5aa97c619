// Device-resident small linear algebra of the randomized SVD
// (reference nla/svd.hpp:71-149 PowerIteration's re-orthonormalisation and
// :278-317 ApproximateSVD's El::SVD of the k x k core), so the whole call runs
// on the GPU with no host round trip.
//
//   k_boundary<INTER>  at each boundary between two power passes: the pass's
//                      W slabs summed (f64), H = W^T W, Cholesky H = R^T R with
//                      pivot dropping, R^{-1}, and the next pass operand
//                      Z^T = (W R^{-1})^T in bf16.  ("orth(W)": CholeskyQR.)
//   k_boundary<FINAL>  after the final pass: the same sums (+ the fp64 Gram of
//                      Y), H = W^T W (W = A^T Y), the Cholesky Y^T Y = Rt^T Rt,
//                      Rt^{-1}, the symmetric core C = Rt^{-T} H Rt^{-1} =
//                      Ub S^2 Ub^T, its top eigenpairs, the small factors
//                      M = Rt^{-1} Ub_r (U = Y M) and N = M S^{-1}, and V = W N.
//
// Structure: the n rows of W are split over n / 16 workgroups; each sums its
// rows, forms their partial Gram (f64) and publishes it with an agent-scope
// release and a ticket counter; the LAST arriving workgroup (agent-scope
// acquire) sums the partials and runs the k x k algebra alone in LDS (k <= 48)
// while the others wait on a generation word, then every workgroup forms its
// rows of Z^T / V.  One launch per boundary (see k_boundary).
//
// The k x k algebra is latency-bound, so it runs on ONE wave with the matrix
// in registers (sl_wave_la.hpp): the Cholesky inverse as an in-place LDL^T
// elimination of [G | I], the core eigenproblem as Householder
// tridiagonalisation + multisection (division-free Sturm counts) + twisted
// factorisation + a DPP back-transform over all waves.  Every call solves
// its core from scratch; cyclic Jacobi (jacobi() below) is kept as the
// fallback for numerically repeated eigenvalues.
#include <string>

#include "sl_common.hpp"
#include "sl_rng.hpp"
#include "sl_wave_la.hpp"

#include <map>
#include <mutex>

namespace {

constexpr int NT = 512;      // threads per workgroup of the small-LA kernels
constexpr int KMAX = 64;
constexpr int RED = KMAX + 16;   // doubles of small scratch (max diag, D^{-1/2})
// dynamic LDS of the small-LA kernels: four k x k f64 buffers, RED doubles, int flags / order
constexpr size_t GRAM_LA_LDS = (size_t)(4 * KMAX * (KMAX + 1) + RED) * sizeof(double) + (4 + KMAX + 1) * sizeof(int);


enum : int { ST_PIVOT = 1, ST_NONFINITE = 2, ST_NOCONV = 4, ST_RANK = 8, ST_TIMEOUT = 16 };

// C = A^T B (transa) or A B for k x k LDS matrices (row stride ld) on f64
// MFMA: 16 x 16 output tiles over the 8 waves, K in steps of 4
// (v_mfma_f64_16x16x4_f64: lane l holds A[l & 15][l >> 4], B[l >> 4][l & 15];
// C/D col = l & 15, row = (l >> 4) + 4 r).  Out-of-range rows / k read 0.
// (The 512-thread FMA loop this replaces took ~6.5 us per k = 40 product.)
typedef __attribute__((ext_vector_type(4))) double f64x4;
__device__ void small_gemm(const double* A, const double* B, double* C, int k, int ld, bool transa) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int nt = (k + 15) >> 4;
  const int fr = lane & 15, fq = lane >> 4;
  for (int t = w; t < nt * nt; t += NT / 64) {
    const int ti = t / nt, tj = t - ti * nt;
    const int row = ti * 16 + fr, col = tj * 16 + fr;
    f64x4 acc = {0.0, 0.0, 0.0, 0.0};
    for (int k0 = 0; k0 < k; k0 += 4) {
      const int kk = k0 + fq;
      const double a = (row < k && kk < k) ? (transa ? A[kk * ld + row] : A[row * ld + kk]) : 0.0;
      const double b = (col < k && kk < k) ? B[kk * ld + col] : 0.0;
      acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int orow = ti * 16 + fq + 4 * r;
      if (orow < k && col < k) C[orow * ld + col] = acc[r];
    }
  }
}

// ---------------------------------------------------------------- Jacobi
struct Rot { double c, s, t; bool rot; };

// rotation zeroing a_pq of the (p, q) plane (J = [[c, s], [-s, c]]).
// big: this pair was still coupled above 1e-6 relative before the rotation
// and above the roundoff floor of the matrix (noise2 = (1e-14 max|a_ii|)^2:
// rotations of other pairs keep re-seeding off-diagonals at eps * |A|, which
// a purely relative test on tiny eigenvalues would chase for many sweeps).
__device__ __forceinline__ Rot jrot(double app, double aqq, double apq, double noise2, bool* big) {
  Rot r{1.0, 0.0, 0.0, false};
  const double pq2 = apq * apq, dd = fabs(app * aqq);
  *big = pq2 > 1e-12 * dd && pq2 > noise2;
  if (!(pq2 > 2.5e-32 * dd) || apq == 0.0) return r;
  const double d = aqq - app;
  // f32 estimate of the tangent of the smaller angle (t^2 + 2 tau t - 1 = 0)
  float t0;
  if (fabs(apq) < 1e-30 * fabs(d)) {
    t0 = (float)(apq / d);
  } else {
    const float tau = (float)d * __builtin_amdgcn_rcpf(2.f * (float)apq);
    t0 = fabsf(tau) > 1e8f ? 0.5f * __builtin_amdgcn_rcpf(tau)
                           : copysignf(__builtin_amdgcn_rcpf(fabsf(tau) + __builtin_amdgcn_sqrtf(fmaf(tau, tau, 1.f))), tau);
  }
  // one f64 Newton step on g(t) = apq t^2 + d t - apq
  double t = (double)t0;
  const double g = fma(apq * t, t, fma(d, t, -apq));
  const double gp = fma(2.0 * apq, t, d);
  t -= (double)__builtin_amdgcn_rcpf((float)gp) * g;
  // c = 1 / sqrt(1 + t^2): f32 rsqrt + one f64 Newton step
  const double u = fma(t, t, 1.0);
  double c = (double)__builtin_amdgcn_rsqf((float)u);
  c = c * fma(-0.5 * u * c, c, 1.5);
  r.c = c;
  r.s = t * c;
  r.t = t;
  r.rot = true;
  return r;
}

__device__ __forceinline__ int player(int pos, int rd, int kp) { return pos == 0 ? 0 : 1 + (pos - 1 + rd) % (kp - 1); }

// Eigen-decomposition of the symmetric kp x kp matrix in A (ld), V <- eigenvectors
// (columns), in place.  Per round: (1) the hp rotations, one thread each,
// into an LDS table; barrier; (2) waves 4-7 apply them to the upper 2 x 2
// blocks of A (and mirror), waves 0-3 to the rows of V (lane = row);
// barrier.  The pair schedule of every round is tabulated once.
__device__ double* jacobi(double* A, double* B, double* V, int kp, int ld, int max_sweeps, int* flags, int* st,
                          bool v_given = false) {
  (void)B;
  __shared__ unsigned short btab[KMAX / 2 * (KMAX / 2 + 1) / 2];
  __shared__ unsigned short rtab[(KMAX - 1) * (KMAX / 2)];
  __shared__ double rot_c[KMAX / 2], rot_s[KMAX / 2], rot_t[KMAX / 2];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int hp = kp / 2;
  const int nA = hp * (hp + 1) / 2;
  if (!v_given) {
    for (int e = tid; e < kp * ld; e += NT) {
      const int i = e / ld, c = e - i * ld;
      V[e] = (i == c) ? 1.0 : 0.0;
    }
  }
  if (tid < 3) flags[tid] = 0;
  for (int b = tid; b < nA; b += NT) {
    int t = b, bi = 0;
    while (t >= hp - bi) { t -= hp - bi; ++bi; }
    btab[b] = (unsigned short)(bi | ((bi + t) << 8));
  }
  for (int e = tid; e < (kp - 1) * hp; e += NT) {
    const int rd = e / hp, i = e - rd * hp;
    (void)0;
    int p = player(i, rd, kp), q = player(kp - 1 - i, rd, kp);
    if (p > q) { const int x = p; p = q; q = x; }
    rtab[e] = (unsigned short)(p | (q << 8));
  }
  if (tid < 64) {
    double v = tid < kp ? fabs(A[tid * ld + tid]) : 0.0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    if (tid == 0) rot_c[0] = v;
  }
  __syncthreads();
  const double amax = rot_c[0];
  const double noise2 = (1e-14 * amax) * (1e-14 * amax);
  __syncthreads();
  // this thread's first A block (held in registers)
  int b0i = 0, b0j = 0;
  if (tid >= 256 && tid - 256 < nA) { b0i = btab[tid - 256] & 255; b0j = btab[tid - 256] >> 8; }
  int sweep = 0;
  bool conv = false;
  for (; sweep < max_sweeps; ++sweep) {
    int* flag = flags + sweep % 3;
    if (tid == 0) flags[(sweep + 1) % 3] = 0;
    for (int rd = 0; rd < kp - 1; ++rd) {
      const unsigned short* rt = rtab + rd * hp;
      // (1) rotations of the round's pairs
      if (tid < hp) {
        const int p = rt[tid] & 255, q = rt[tid] >> 8;
        bool big;
        const Rot R = jrot(A[p * ld + p], A[q * ld + q], A[p * ld + q], noise2, &big);
        if (big) *flag = 1;
        rot_c[tid] = R.c;
        rot_s[tid] = R.s;
        rot_t[tid] = R.rot ? R.t : 0.0;
      }
      __syncthreads();
      // (2) apply: waves 4-7 the blocks of A, waves 0-3 the rows of V
      if (wid >= 4) {
#pragma unroll 1
        for (int b = tid - 256, u = 0; b < nA; b += NT - 256, ++u) {
          const int bi = u == 0 ? b0i : (btab[b] & 255), bj = u == 0 ? b0j : (btab[b] >> 8);
          const int pi = rt[bi] & 255, qi = rt[bi] >> 8;
          if (bi == bj) {
            const double t = rot_t[bi];
            const double apq = A[pi * ld + qi];
            A[pi * ld + pi] -= t * apq;
            A[qi * ld + qi] += t * apq;
            if (t != 0.0) { A[pi * ld + qi] = 0.0; A[qi * ld + pi] = 0.0; }
          } else {
            const int pj = rt[bj] & 255, qj = rt[bj] >> 8;
            const double ci = rot_c[bi], si = rot_s[bi], cj = rot_c[bj], sj = rot_s[bj];
            const double x00 = A[pi * ld + pj], x01 = A[pi * ld + qj], x10 = A[qi * ld + pj], x11 = A[qi * ld + qj];
            // Y = X R_j, X' = R_i^T Y
            const double y00 = cj * x00 - sj * x01, y01 = sj * x00 + cj * x01;
            const double y10 = cj * x10 - sj * x11, y11 = sj * x10 + cj * x11;
            const double z00 = ci * y00 - si * y10, z01 = ci * y01 - si * y11;
            const double z10 = si * y00 + ci * y10, z11 = si * y01 + ci * y11;
            A[pi * ld + pj] = z00; A[pi * ld + qj] = z01; A[qi * ld + pj] = z10; A[qi * ld + qj] = z11;
            A[pj * ld + pi] = z00; A[qj * ld + pi] = z01; A[pj * ld + qi] = z10; A[qj * ld + qi] = z11;
          }
        }
      } else if (lane < kp) {
        // V <- V J: row `lane`, pairs wid, wid + 4, ... (loads first, then
        // the rotations: no dependent LDS round trips inside the loop)
        double* vr = V + lane * ld;
        constexpr int JU = KMAX / 2 / 4;
        int pp[JU], qq[JU];
        double vp[JU], vq[JU];
#pragma unroll
        for (int u = 0; u < JU; ++u) {
          const int j = wid + 4 * u;
          const unsigned short pq = j < hp ? rt[j] : (unsigned short)0;
          pp[u] = pq & 255;
          qq[u] = pq >> 8;
        }
#pragma unroll
        for (int u = 0; u < JU; ++u) {
          vp[u] = vr[pp[u]];
          vq[u] = vr[qq[u]];
        }
#pragma unroll
        for (int u = 0; u < JU; ++u) {
          const int j = wid + 4 * u;
          if (j < hp && rot_t[j] != 0.0) {
            const double c = rot_c[j], sn = rot_s[j];
            vr[pp[u]] = c * vp[u] - sn * vq[u];
            vr[qq[u]] = sn * vp[u] + c * vq[u];
          }
        }
      }
      __syncthreads();
    }
    if (!*flag) { conv = true; ++sweep; break; }
  }
  if (!conv && tid == 0) *st |= ST_NOCONV;
  if (tid == 0) flags[3] = sweep;
  __syncthreads();
  return A;
}

// ---------------------------------------------------------------- final core
// After the final pass (H = W^T W in b0, Rti = Rt^{-1} of Y^T Y = Rt^T Rt in
// b3, row stride ld = k + 1): C = Rti^T H Rti = Ub S^2 Ub^T, its top r + 1
// eigenvalues and top r eigenvectors (Householder tridiagonalisation on one
// wave, multisection + twisted factorisation + back-transform on all waves,
// sl_wave_la.hpp), s, M = Rti Ub_r (f32) and N = M S^{-1} (f64).  Every call
// solves its core from scratch.  If the tridiagonal path reports
// numerically repeated wanted eigenvalues or a vector that fails its
// residual check, the core is re-solved by cyclic Jacobi (robust to
// clusters, rare).  Run by ONE workgroup.  status_or: OR the call's status
// bits into *status (0: store them -- the call's first writer).
struct CoreLds {
  __attribute__((aligned(16))) double dd[KMAX], ee[KMAX], lam[KMAX], vsh[2 * KMAX], wsh[2 * KMAX], fsh[9 * 64];
  int bad, fb;
};

template <int K>
__device__ __forceinline__ void final_core(double* b0, double* b1, double* b2, double* b3, int* flags, int* order, CoreLds& cs,
                           double* Cbak, int k, int r, float* __restrict__ M, double* __restrict__ N,
                           double* __restrict__ s_out, int* __restrict__ status, int* mirror, int* st_sh_p,
                           int status_or) {
  int& st_sh = *st_sh_p;
  const int tid = threadIdx.x;
  const int ld = k + 1;
  constexpr int SO = 16;
  (void)SO;
  // C = Rti^T H Rti:  T = H Rti -> b1, C = Rti^T T -> b2
  small_gemm(b0, b3, b1, k, ld, false);
  __syncthreads();
  small_gemm(b3, b1, b2, k, ld, true);
  __syncthreads();
  // symmetrise into b0 (+ a global copy for the rare fallback)
  for (int e = tid; e < k * k; e += NT) {
    const int i = e / k, c = e - i * k;
    const double v = 0.5 * (b2[i * ld + c] + b2[c * ld + i]);
    b0[i * ld + c] = v;
    Cbak[e] = v;
  }
  if (tid == 0) { cs.bad = 0; cs.fb = 0; }
  __syncthreads();
  // tridiagonalise (wave 0; reflectors into b2, ld K + 1)
  const int nt = r < k ? r + 1 : k;
  if (tid < 64) slw::wave_tridiag<K>(b0, ld, k, b2, K + 1, cs.dd, cs.ee, cs.vsh, cs.wsh, &cs.bad);
  __syncthreads();
  // top nt eigenvalues, top r eigenvectors of C into b1 (ld), scratch b0
  slw::sym_top_eig<K, NT>(cs.dd, cs.ee, b2, K + 1, nt, r, cs.lam, b1, ld, k, b0, &cs.fb);
  if (cs.fb | cs.bad) {
    // robust path: Jacobi on the saved core (C in b2, V in b1, ld)
    const int kp = k + (k & 1);
    for (int e = tid; e < kp * kp; e += NT) {
      const int i = e / kp, c = e - i * kp;
      b2[i * ld + c] = (i < k && c < k) ? Cbak[i * k + c] : 0.0;
    }
    __syncthreads();
    double* Af = jacobi(b2, b0, b1, kp, ld, 40, flags, st_sh_p);
    for (int i = tid; i < k; i += NT) {
      const double li = Af[i * ld + i];
      int rk = 0;
      for (int j = 0; j < k; ++j) {
        const double lj = Af[j * ld + j];
        rk += (lj > li) || (lj == li && j < i);
      }
      order[rk] = i;
    }
    __syncthreads();
    // eigenvectors in descending order into b0 (ld), eigenvalues into lam
    for (int e = tid; e < k * r; e += NT) {
      const int i = e / r, c = e - i * r;
      b0[i * ld + c] = b1[i * ld + order[c]];
    }
    for (int c = tid; c < nt; c += NT) cs.lam[c] = Af[order[c] * ld + order[c]];
    __syncthreads();
    for (int e = tid; e < k * r; e += NT) {
      const int i = e / r, c = e - i * r;
      b1[i * ld + c] = b0[i * ld + c];
    }
    if (tid == 0 && cs.bad) st_sh |= ST_NONFINITE;
    __syncthreads();
  }
  // ---- s, M = Rti Ub_r (f32), N = M S^{-1} (f64)
  for (int c = tid; c < r; c += NT) {
    const double lam = cs.lam[c];
    s_out[c] = lam > 0.0 ? sqrt(lam) : 0.0;
    if (!(lam > 0.0)) atomicOr(st_sh_p, ST_RANK);
    if (!(lam == lam)) atomicOr(st_sh_p, ST_NONFINITE);
  }
  __syncthreads();
  for (int e = tid; e < k * r; e += NT) {
    const int i = e / r, c = e - i * r;
    double a = 0.0;
    for (int l = i; l < k; ++l) a += b3[i * ld + l] * b1[l * ld + c];
    M[e] = (float)a;
    const double lam = cs.lam[c];
    N[e] = lam > 0.0 ? a * slw::rsq64(lam) : 0.0;
  }
  if (tid == 0) {
    int all = st_sh;
    if (status_or) all |= atomicOr(status, st_sh);
    else __hip_atomic_store(status, st_sh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // the call's final status word, straight to host-mapped memory (no D2H copy)
    if (mirror) __hip_atomic_store(mirror, all, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// ---------------------------------------------------------------- fused boundary
// ONE launch at each pass boundary, after the (full-chip) slab reduce and, on
// several ranks, the all-reduce of [W; G]; it replaces the Gram / small-LA
// kernel, the Z^T kernel and (after the last pass) the V = W N kernel:
//   1. workgroup b loads its BR rows of W (one batch of loads) into LDS
//   2. the packed upper partial Gram of its rows -> global, then a ticket
//   3. the last arriving workgroup sums the partials (16-B loads, a batch in
//      flight), runs the k x k algebra (INTER: Cholesky inverse with its rows over 4 waves;
//      FINAL: final_core) and bumps the generation word (agent-scope release)
//   4. every workgroup (the others spin on the generation word meanwhile; the
//      <= BMAX workgroups are co-resident on the 256 CUs) forms its rows of
//      the next pass operand Z^T = (W R^{-1})^T (INTER) or of V = W N (FINAL)
//      from the W rows it still holds in LDS.
// Graph replays: the last arriver resets the ticket; the generation only
// grows (a waiter compares with the value it read before arriving).
// (Summing the 256 pass slabs inside this kernel was measured: 63 workgroups
// pulling 655 KB each of 2.5 KB pieces took 58 us, against 9 us for the
// full-chip reduce kernel, so the reduce stays a launch of its own.)
constexpr int BR = 16;     // rows of W per workgroup
constexpr int BMAX = 64;   // workgroups (n <= 1024)
constexpr int BK = 48;     // largest k of the pass
constexpr int WLD = KMAX + 1;   // LDS row stride of the W rows (odd: rows on distinct banks)

struct BndArgs {
  int n, k, r;
  int nbr;                // workgroups holding rows (FINAL: one more, the Y^T Y Cholesky worker)
  double* rti;            // FINAL: the worker's Rt^{-1} (k x k) and status word
  double* cbak;           // FINAL: k x k copy of the core (fallback)
  double* WG;             // [W (n x k); Gy (k x k)] f64
  double* part;           // BMAX packed partial Grams, stride ldp doubles
  int ldp;
  unsigned* sync;         // [0] ticket, [16] generation, [32] finished FINAL workers, [33] consumed
  int* status;
  int status_or;
  double* Rinv;           // INTER: k x k
  bf16_t* Zt;             // INTER: k x n
  float* M;               // FINAL: k x r, N (k x r), s64 (r)
  double* N;
  double* s64;
  int* mirror;
  float* V;               // FINAL: n x r (null: no V), s32 (r)
  float* s32;
  float* const* optr;     // {U, s, V} read at run time when set (graph replays)
  uint64_t bound;         // spin bound (100 MHz ticks)
  int missing;            // test knob: arrivals expected beyond the grid (0 in production)
};

// dynamic LDS: four k x k f64 buffers + small scratch (GRAM_LA_LDS), then the BR x KMAX rows of W
constexpr size_t BND_WR_OFF = (GRAM_LA_LDS + 15) / 16 * 2;   // in doubles
constexpr size_t BND_LDS = BND_WR_OFF * sizeof(double) + (size_t)BR * WLD * sizeof(double);

template <bool FINAL, int K>
__global__ void __launch_bounds__(NT) k_boundary(BndArgs a) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int n = a.n, k = a.k, nb = a.nbr;
  const int ld = k + 1;
  const int mat = KMAX * (KMAX + 1);
  double* b0 = sm;
  double* b1 = sm + mat;
  double* b2 = sm + 2 * mat;
  double* b3 = sm + 3 * mat;
  double* red = sm + 4 * mat;
  int* iscr = (int*)(red + RED);
  int* flags = iscr;
  int* order = iscr + 4;
  double* Wr = sm + BND_WR_OFF;   // BR x WLD rows of W
  __shared__ int st_sh;
  __shared__ int is_last;
  __shared__ unsigned gen0;
  __shared__ CoreLds cls;
  if (FINAL && (int)blockIdx.x == nb) {
    // the Y^T Y worker: Rt^{-1} of the reduced Gram (independent of W) while
    // the row workgroups form and sum H, published as a finished-worker count
    if (tid == 0) st_sh = 0;
    // G staged into LDS with coalesced loads (all in flight), the elimination
    // on LDS operands, X back with coalesced stores: the wave's per-lane
    // strided global reads / writes cost ~10 us on this critical path
    {
      const double* Gg = a.WG + (int64_t)n * k;
      constexpr int UB = BK * BK / NT + 1;
      double v[UB];
#pragma unroll
      for (int u = 0; u < UB; ++u) {
        const int e = tid + NT * u;
        v[u] = Gg[e < k * k ? e : 0];
      }
#pragma unroll
      for (int u = 0; u < UB; ++u) {
        const int e = tid + NT * u;
        if (e < k * k) {
          const int i = e / k, c = e - i * k;
          b0[i * ld + c] = v[u];
        }
      }
    }
    __syncthreads();
    slw::wg_chol_invB<K, 4, 4>(b0, ld, b2, ld, k, cls.fsh, &st_sh);   // 4 pivots per step, rows over 4 waves
    __syncthreads();
    for (int e = tid; e < k * k; e += NT) {
      const int i = e / k, c = e - i * k;
      a.rti[e] = b2[i * ld + c];
    }
    if (tid == 0) ((int*)(a.rti + k * k))[0] = st_sh;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      // publish: a monotone count of finished workers (sync[32]); the last
      // arriver consumes one per launch (sync[33]), so a late worker of a
      // timed-out launch can never satisfy a later launch's wait
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_fetch_add(&a.sync[32], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  const int r0 = blockIdx.x * BR;
  const int nr = min(BR, n - r0);
  const int E = nr * k;   // a multiple of 8 (n % 8 == 0)

  // ---- 1. this workgroup's rows of W (E <= BR * BK = 768: two loads per
  //      thread, both issued before the LDS stores, clamped addresses)
  {
    constexpr int UE = BR * BK / NT + 1;
    double v[UE];
#pragma unroll
    for (int u = 0; u < UE; ++u) {
      const int e = tid + NT * u;
      v[u] = a.WG[(int64_t)r0 * k + (e < E ? e : 0)];
    }
#pragma unroll
    for (int u = 0; u < UE; ++u) {
      const int e = tid + NT * u;
      if (e < E) {
        const int row = e / k, col = e - row * k;
        Wr[row * WLD + col] = v[u];
      }
    }
  }
  __syncthreads();
  // ---- 2. packed upper partial Gram of the rows: thread (gq, cq) owns (gq + 8u, cq)
  {
    const int gq = wv, cq = lane;
    double acc[KMAX / 8];
#pragma unroll
    for (int u = 0; u < KMAX / 8; ++u) acc[u] = 0.0;
    if (cq < k) {
      for (int row = 0; row < nr; ++row) {
        const double x = Wr[row * WLD + cq];
#pragma unroll
        for (int u = 0; u < KMAX / 8; ++u) acc[u] += Wr[row * WLD + gq + 8 * u] * x;
      }
      double* myp = a.part + (int64_t)blockIdx.x * a.ldp;
#pragma unroll
      for (int u = 0; u < KMAX / 8; ++u) {
        const int i = gq + 8 * u;
        if (i <= cq) myp[i * k - (i * (i - 1)) / 2 + (cq - i)] = acc[u];
      }
    }
  }

  // ---- 3. ticket: every wave's stores complete, then ONE agent-scope release
  //      (a fence per wave would write the L2 back once per wave)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    gen0 = __hip_atomic_load(&a.sync[16], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    const unsigned t = __hip_atomic_fetch_add(&a.sync[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    is_last = t == (unsigned)(nb + a.missing) - 1;
    if (is_last) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    st_sh = 0;
  }
  __syncthreads();
  if (is_last) {
    // sum of the nb packed partials, two entries per thread and load
    const int npair = a.ldp >> 1;
    double* Hp = b1;
    for (int p = tid; p < npair; p += NT) {
      const double2* src = (const double2*)a.part + p;
      double2 s2 = {0.0, 0.0};
      for (int g0 = 0; g0 < nb; g0 += 32) {
        // clamped addresses, all 32 loads in flight, out-of-range ones zeroed
        double2 v[32];
#pragma unroll
        for (int q = 0; q < 32; ++q) v[q] = src[(int64_t)min(g0 + q, nb - 1) * npair];
#pragma unroll
        for (int q = 0; q < 32; ++q)
          if (g0 + q >= nb) v[q] = double2{0.0, 0.0};
#pragma unroll
        for (int q = 0; q < 32; ++q) {
          s2.x += v[q].x;
          s2.y += v[q].y;
        }
      }
      Hp[2 * p] = s2.x;
      Hp[2 * p + 1] = s2.y;
    }
    __syncthreads();
    for (int e = tid; e < k * k; e += NT) {
      const int i = e / k, c = e - i * k;
      const int lo = min(i, c), hi = max(i, c);
      b0[i * ld + c] = Hp[lo * k - (lo * (lo - 1)) / 2 + (hi - lo)];
    }
    __syncthreads();
    if (tid == 0) a.sync[0] = 0u;   // ready for the next launch
    if (!FINAL) {
      slw::wg_chol_invB<K, 4, 4>(b0, ld, b2, ld, k, cls.fsh, &st_sh);   // 4 pivots per step, rows over 4 waves
      __syncthreads();
      for (int e = tid; e < k * k; e += NT) {
        const int i = e / k, c = e - i * k;
        const double v = b2[i * ld + c];
        if (!(fabs(v) < 1e300)) atomicOr(&st_sh, ST_NONFINITE);
        a.Rinv[e] = v;
      }
      __syncthreads();
      if (tid == 0) {
        if (a.status_or) atomicOr(a.status, st_sh);
        else __hip_atomic_store(a.status, st_sh, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    } else {
      // the worker's Rt^{-1}: bounded wait until the finished-worker count
      // passes the consumed count, then consume one (also after a timeout:
      // the late worker's publish is then already accounted for)
      if (tid == 0) {
        const unsigned want = __hip_atomic_load(&a.sync[33], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
        const uint64_t t0 = wall_clock64();
        while ((int)(__hip_atomic_load(&a.sync[32], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - want) < 0) {
          __builtin_amdgcn_s_sleep(1);
          if (wall_clock64() - t0 > a.bound) {
            st_sh |= ST_TIMEOUT;
            break;
          }
        }
        __hip_atomic_store(&a.sync[33], want, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        st_sh |= ((const int*)(a.rti + k * k))[0];
      }
      __syncthreads();
      {
        constexpr int UB = BK * BK / NT + 1;
        double v[UB];
#pragma unroll
        for (int u = 0; u < UB; ++u) {
          const int e = tid + NT * u;
          v[u] = a.rti[e < k * k ? e : 0];
        }
#pragma unroll
        for (int u = 0; u < UB; ++u) {
          const int e = tid + NT * u;
          if (e < k * k) {
            const int i = e / k, c = e - i * k;
            b3[i * ld + c] = v[u];
          }
        }
      }
      __syncthreads();
      final_core<K>(b0, b1, b2, b3, flags, order, cls, a.cbak, k, a.r, a.M, a.N, a.s64, a.status, a.mirror, &st_sh,
                    a.status_or);
    }
    // release the waiters
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      __hip_atomic_fetch_add(&a.sync[16], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  } else {
    if (tid == 0) {
      // bounded wait (never reached on a sane run: the last arriver has no
      // further dependency); a timeout flags the call instead of hanging
      const uint64_t t0 = wall_clock64();
      while (__hip_atomic_load(&a.sync[16], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gen0) {
        __builtin_amdgcn_s_sleep(2);
        if (wall_clock64() - t0 > a.bound) {
          atomicOr(a.status, ST_TIMEOUT);
          if (a.mirror) __hip_atomic_store(a.mirror, ST_TIMEOUT, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          break;
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    }
    __syncthreads();
  }

  // ---- 4. rows of Z^T = (W Rinv)^T (INTER) or V = W N (FINAL)
  float* V = FINAL ? (a.optr ? a.optr[2] : a.V) : nullptr;
  if (FINAL) {
    float* s32 = a.optr ? a.optr[1] : a.s32;
    if (blockIdx.x == 0 && s32 && tid < a.r) s32[tid] = (float)a.s64[tid];
    if (!V) return;
  }
  const int nc = FINAL ? a.r : k;
  const double* Bsrc = FINAL ? a.N : a.Rinv;
  double* Bs = b3;
  {
    // k * nc <= 48 * 48: five loads per thread in flight, then the stores
    constexpr int UB = BK * BK / NT + 1;
    double v[UB];
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int e = tid + NT * u;
      v[u] = Bsrc[e < k * nc ? e : 0];
    }
#pragma unroll
    for (int u = 0; u < UB; ++u) {
      const int e = tid + NT * u;
      if (e < k * nc) Bs[e] = v[u];
    }
  }
  __syncthreads();
  const int row = tid & (BR - 1);
  if (row < nr) {
    for (int c = tid / BR; c < nc; c += NT / BR) {
      double s0 = 0.0, s1 = 0.0;
      int l = 0;
      for (; l + 1 < k; l += 2) {
        s0 += Wr[row * WLD + l] * Bs[l * nc + c];
        s1 += Wr[row * WLD + l + 1] * Bs[(l + 1) * nc + c];
      }
      if (l < k) s0 += Wr[row * WLD + l] * Bs[l * nc + c];
      const double v = s0 + s1;
      if (FINAL) V[(int64_t)(r0 + row) * nc + c] = (float)v;
      else a.Zt[(int64_t)c * n + r0 + row] = f_to_bf16((float)v);
    }
  }
}

// Out (rows of W, k x nc) = W (n x k f64) B (k x nc f64, row-major), a 32-row
// slab of W and all of B staged in LDS with coalesced loads; thread
// (row = t & 31, column group t >> 5) forms columns cg, cg + 8, ... of its row.
template <typename Store>
__device__ __forceinline__ void rows_times_small(const double* __restrict__ W, int n, int k, int ldw,
                                                 const double* __restrict__ B, int nc, Store store) {
  __shared__ double Ws[32][KMAX + 1];
  __shared__ double Bs[KMAX][KMAX];
  const int t = threadIdx.x, row = t & 31, cg = t >> 5;
  const int i0 = blockIdx.x * 32;
  const int nr = min(32, n - i0);
  // every staging load of the thread issued before the first LDS store, from
  // clamped addresses (a rolled load -> store loop waits on one load at a time)
  constexpr int UB = KMAX * KMAX / 256, UW = 32 * KMAX / 256;
  double vb[UB], vw[UW];
#pragma unroll
  for (int u = 0; u < UB; ++u) {
    const int e = t + 256 * u;
    vb[u] = B[e < k * nc ? e : 0];
  }
#pragma unroll
  for (int u = 0; u < UW; ++u) {
    const int e = t + 256 * u;
    const int rr = e / k;
    vw[u] = W[e < nr * k ? (int64_t)(i0 + rr) * ldw + (e - rr * k) : (int64_t)i0 * ldw];
  }
#pragma unroll
  for (int u = 0; u < UB; ++u) {
    const int e = t + 256 * u;
    if (e < k * nc) {
      const int l = e / nc;
      Bs[l][e - l * nc] = vb[u];
    }
  }
#pragma unroll
  for (int u = 0; u < UW; ++u) {
    const int e = t + 256 * u;
    if (e < nr * k) {
      const int rr = e / k;
      Ws[rr][e - rr * k] = vw[u];
    }
  }
  __syncthreads();
  if (row >= nr) return;
  double acc[KMAX / 8];
#pragma unroll
  for (int u = 0; u < KMAX / 8; ++u) acc[u] = 0.0;
  for (int l = 0; l < k; ++l) {
    const double w = Ws[row][l];
#pragma unroll
    for (int u = 0; u < KMAX / 8; ++u) acc[u] += w * Bs[l][(cg + 8 * u) & (KMAX - 1)];
  }
#pragma unroll
  for (int u = 0; u < KMAX / 8; ++u) {
    const int c = cg + 8 * u;
    if (c < nc) store(i0 + row, c, acc[u]);
  }
}

// V (n x r f32) = W (n x k f64) N (k x r f64); s32 = s64 (r)
__global__ void __launch_bounds__(256)
k_make_v(const double* __restrict__ W, int n, int k, int ldw, const double* __restrict__ N, int r, float* __restrict__ V,
         const double* __restrict__ s64, float* __restrict__ s32, float* const* __restrict__ optr) {
  // optr: {U, s, V} read at run time (the graph-captured finish)
  if (optr) {
    s32 = optr[1];
    V = optr[2];
  }
  if (s32 && blockIdx.x == 0 && threadIdx.x < r) s32[threadIdx.x] = (float)s64[threadIdx.x];
  rows_times_small(W, n, k, ldw, N, r, [&](int i, int c, double v) { V[(int64_t)i * r + c] = (float)v; });
}

// FJLT operator of the rowwise sketch A Omega^T, as the pass operand Z^T
// (k x n bf16): Z^T[j][i] = scale * d_i * c_{p_j} cos(pi p_j (2 i + 1) / 2n)
// with d the n Rademacher signs at stream offset baseD and p_j the k sampled
// DCT-II frequencies at baseS (reference FJLT_data.hpp:79-86, sketch/fjlt.py)
__global__ void __launch_bounds__(256)
k_fjlt_zt(uint64_t seed, uint64_t baseD, uint64_t baseS, double scale, int k, int n, bf16_t* __restrict__ Zt,
          float** tab, float* ta, float* tb, float* tc) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  // the engine's {U, s, V} pointer table for this call (no launch of its own)
  if (tab && t < 3) tab[t] = t == 0 ? ta : (t == 1 ? tb : tc);
  if (t >= (int64_t)n * k) return;
  const int j = (int)(t / n), i = (int)(t - (int64_t)j * n);
  const int64_t p = sl::uniform_int(sl::stream_block(seed, baseS + (uint64_t)j).x, 0, n - 1);
  const double d = (sl::stream_block(seed, baseD + (uint64_t)i).x >> 63) ? 1.0 : -1.0;
  const int64_t a = (p * (2 * (int64_t)i + 1)) % (4 * (int64_t)n);
  const double w = 3.14159265358979323846 / (2.0 * (double)n);
  const double c0 = sqrt(1.0 / (double)n), c1 = sqrt(2.0 / (double)n);
  Zt[t] = f_to_bf16((float)(cos(w * (double)a) * (p == 0 ? c0 : c1) * scale * d));
}

// bf16(f32(x)): the realised f64 sketch operator as the pass operand, rounded
// exactly as the Python path's tensor casts (f64 -> f32 -> bf16, both RNE)
__global__ void __launch_bounds__(256) k_f64_to_bf16(const double* __restrict__ x, int64_t count, bf16_t* __restrict__ y) {
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t < count) y[t] = f_to_bf16((float)x[t]);
}

size_t gram_la_lds() { return GRAM_LA_LDS; }

}  // namespace

// ------------------------------------------------------------------ C ABI
SL_API int sl_rsvd_make_v(const double* W, int n, int k, int ldw, const double* N, int r, float* V, const double* s64,
                          float* s32, void* stream) {
  if (k < 1 || k > KMAX || r > k) { sl_set_last_error("rsvd_make_v: 1 <= r <= k <= 64"); return SL_ERR_UNSUPPORTED; }
  k_make_v<<<(unsigned)((n + 31) / 32), 256, 0, (hipStream_t)stream>>>(W, n, k, ldw, N, r, V, s64, s32, nullptr);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// V and s from optr[2] / optr[1] at run time (a graph node replayed into a
// new caller buffer each call; sl_rsvd_set_ptrs writes the table)
SL_API int sl_rsvd_make_v_ind(const double* W, int n, int k, int ldw, const double* N, int r, const double* s64,
                              float* const* optr, void* stream) {
  if (k < 1 || k > KMAX || r > k) { sl_set_last_error("rsvd_make_v: 1 <= r <= k <= 64"); return SL_ERR_UNSUPPORTED; }
  k_make_v<<<(unsigned)((n + 31) / 32), 256, 0, (hipStream_t)stream>>>(W, n, k, ldw, N, r, nullptr, s64, nullptr,
                                                                       optr);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

namespace {
__global__ void k_set_ptrs(float** tab, float* a, float* b, float* c) {
  if (threadIdx.x == 0) tab[0] = a;
  if (threadIdx.x == 1) tab[1] = b;
  if (threadIdx.x == 2) tab[2] = c;
}
}  // namespace

// tab[0..2] = {a, b, c} in stream order (one vector-store kernel)
SL_API int sl_rsvd_set_ptrs(float** tab, float* a, float* b, float* c, void* stream) {
  k_set_ptrs<<<1, 64, 0, (hipStream_t)stream>>>(tab, a, b, c);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// tab (optional): {a, b, c} written by the same launch (the engine's pointer table)
SL_API int sl_rsvd_fjlt_zt_tab(uint64_t seed, uint64_t baseD, uint64_t baseS, double scale, int k, int n, void* Zt,
                               float** tab, float* a, float* b, float* c, void* stream) {
  const int64_t tot = (int64_t)n * k;
  k_fjlt_zt<<<(unsigned)((tot + 255) / 256), 256, 0, (hipStream_t)stream>>>(seed, baseD, baseS, scale, k, n,
                                                                            (bf16_t*)Zt, tab, a, b, c);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

SL_API int sl_rsvd_fjlt_zt(uint64_t seed, uint64_t baseD, uint64_t baseS, double scale, int k, int n, void* Zt,
                           void* stream) {
  return sl_rsvd_fjlt_zt_tab(seed, baseD, baseS, scale, k, n, Zt, nullptr, nullptr, nullptr, nullptr, stream);
}

// Standalone symmetric eigensolver on the device (same Jacobi), for tests:
// C (k x k f64) -> w (k, descending) and V (k x k, columns).  One workgroup.
namespace {
__global__ void __launch_bounds__(NT)
k_sym_eig_jacobi2(const double* __restrict__ C, int k, double* __restrict__ w, double* __restrict__ Vout,
                  int* __restrict__ status, int max_sweeps) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int tid = threadIdx.x;
  const int ld = k + 1, mat = KMAX * (KMAX + 1);
  double *b0 = sm, *b1 = sm + mat, *b2 = sm + 2 * mat;
  double* red = sm + 4 * mat;
  int* iscr = (int*)(red + RED);
  int* flags = iscr;
  int* order = iscr + 4;
  __shared__ int st_sh;
  if (tid == 0) st_sh = 0;
  const int kp = k + (k & 1);
  for (int e = tid; e < kp * kp; e += NT) {
    const int i = e / kp, c = e - i * kp;
    b2[i * ld + c] = (i < k && c < k) ? 0.5 * (C[i * k + c] + C[c * k + i]) : 0.0;
  }
  __syncthreads();
  double* Af = jacobi(b2, b0, b1, kp, ld, max_sweeps, flags, &st_sh);
  for (int i = tid; i < k; i += NT) {
    const double li = Af[i * ld + i];
    int rk = 0;
    for (int j = 0; j < k; ++j) {
      const double lj = Af[j * ld + j];
      rk += (lj > li) || (lj == li && j < i);
    }
    order[rk] = i;
  }
  __syncthreads();
  for (int e = tid; e < k * k; e += NT) {
    const int i = e / k, c = e - i * k;
    Vout[e] = b1[i * ld + order[c]];
  }
  for (int c = tid; c < k; c += NT) w[c] = Af[order[c] * ld + order[c]];
  if (tid == 0) { status[0] = st_sh; status[1] = flags[3]; }
}
}  // namespace

SL_API int sl_sym_eig_jacobi2(const double* C, int k, double* w, double* V, int* status, int max_sweeps, void* stream) {
  if (k < 1 || k > KMAX) { sl_set_last_error("sym_eig_jacobi2: 1 <= k <= 64"); return SL_ERR_UNSUPPORTED; }
  SL_LDS_ATTR(k_sym_eig_jacobi2, (int)gram_la_lds());
  k_sym_eig_jacobi2<<<1, NT, gram_la_lds(), (hipStream_t)stream>>>(C, k, w, V, status, max_sweeps > 0 ? max_sweeps : 40);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

SL_API int sl_rsvd_zt_from_f64(const double* src, int64_t count, void* Zt, void* stream) {
  if (count <= 0) return SL_OK;
  k_f64_to_bf16<<<(unsigned)((count + 255) / 256), 256, 0, (hipStream_t)stream>>>(src, count, (bf16_t*)Zt);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// ------------------------------------------------------------ fused boundary

// Test-only fault injection per boundary workspace: `missing` arrivals the
// kernel waits for beyond its grid (so no workgroup is last and every wait
// times out) and the spin bound in 100 MHz ticks (0: the 2 s default).
namespace {
struct BndFault { int missing = 0; uint64_t bound = 0; };
std::mutex g_fault_mu;
std::map<const void*, BndFault> g_faults;
BndFault bnd_fault(const void* bws) {
  std::lock_guard<std::mutex> g(g_fault_mu);
  auto it = g_faults.find(bws);
  return it == g_faults.end() ? BndFault{} : it->second;
}
}  // namespace

SL_API int sl_rsvd_bnd_set_fault(const void* bws, int missing, uint64_t bound_ticks) {
  std::lock_guard<std::mutex> g(g_fault_mu);
  if (missing == 0 && bound_ticks == 0) g_faults.erase(bws);
  else g_faults[bws] = BndFault{missing, bound_ticks};
  return SL_OK;
}

// workspace of sl_rsvd_boundary: sync words (256 B, zeroed once; the kernel
// leaves the ticket zero and only advances the generation and worker counts)
// + BMAX partial Grams + the worker's Rt^{-1} and status + the core's copy
SL_API int64_t sl_rsvd_bnd_workspace(int k) {
  const int64_t ldp = ((int64_t)k * (k + 1) / 2 + 1) & ~(int64_t)1;
  return 256 + (int64_t)BMAX * ldp * 8 + (int64_t)k * k * 8 + 256 + (int64_t)k * k * 8;
}

namespace {
template <int K>
int launch_bnd(bool fin, unsigned nb, const BndArgs& a, hipStream_t s) {
  if (fin) {
    SL_LDS_ATTR((k_boundary<true, K>), (int)BND_LDS);
    k_boundary<true, K><<<nb + 1, NT, BND_LDS, s>>>(a);   // + the Y^T Y worker
  } else {
    SL_LDS_ATTR((k_boundary<false, K>), (int)BND_LDS);
    k_boundary<false, K><<<nb, NT, BND_LDS, s>>>(a);
  }
  SL_LAUNCH_CHECK();
  return SL_OK;
}
}  // namespace

namespace {
template <int K>
int bnd_capacity(int* cap) {
  int per_cu_f = 0, per_cu_i = 0, dev = 0, cus = 0;
  SL_LDS_ATTR((k_boundary<true, K>), (int)BND_LDS);
  SL_LDS_ATTR((k_boundary<false, K>), (int)BND_LDS);
  SL_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu_f, k_boundary<true, K>, NT, BND_LDS));
  SL_HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu_i, k_boundary<false, K>, NT, BND_LDS));
  SL_HIP_CHECK(hipGetDevice(&dev));
  SL_HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  *cap = std::min(per_cu_f, per_cu_i) * cus;
  return SL_OK;
}
}  // namespace

// Co-residency of the pass-boundary grid: k_boundary's workgroups wait on
// each other (a generation word), so every one of them must be resident at
// once.  The plan checks at creation that the device holds the whole grid
// (the FINAL launch has the most workgroups) with nothing else running; a
// concurrent kernel that still starves one of them is caught by the bounded
// wait (status bit 16, raised on that call).  *ok = 1 when it fits.
SL_API int sl_rsvd_bnd_coresident(int n, int k, int* ok) {
  *ok = 0;
  if (k < 1 || k > BK || n < 16 || n > BMAX * BR) {
    sl_set_last_error("rsvd_boundary: needs 1 <= k <= 48, 16 <= n <= 1024");
    return SL_ERR_UNSUPPORTED;
  }
  int cap = 0;
  const int rc = k <= 16 ? bnd_capacity<16>(&cap) : k <= 32 ? bnd_capacity<32>(&cap)
               : k <= 40 ? bnd_capacity<40>(&cap) : bnd_capacity<48>(&cap);
  if (rc != SL_OK) return rc;
  const int need = (n + BR - 1) / BR + 1;
  *ok = cap >= need ? 1 : 0;
  if (!*ok)
    sl_set_last_error(("rsvd_boundary: " + std::to_string(need) + " workgroups must be co-resident, the device holds " +
                       std::to_string(cap)).c_str());
  return SL_OK;
}

// One pass boundary on the reduced (and, on several ranks, all-reduced)
// [W (n x k); Gy (k x k)] f64 buffer WG.
// final_ = 0: Rinv and Z^T (bf16, k x n) for the next pass.  final_ = 1: the
// core (s64, M, N, status, mirror) and, when V or optr is given, V = W N
// (n x r f32) and s (f32).  status_or = 0 stores the status bits (the call's
// first writer), 1 ORs them.
SL_API int sl_rsvd_boundary(int final_, int n, int k, int r, double* WG, void* bws, int* status, int status_or,
                            double* Rinv, void* Zt, float* M, double* N, double* s64, int* mirror, float* V,
                            float* s32, float* const* optr, void* stream) {
  if (k < 1 || k > BK || n < 16 || n > BMAX * BR || n % 8 || (final_ && (r < 1 || r > k))) {
    sl_set_last_error("rsvd_boundary: needs 1 <= k <= 48, 16 <= n <= 1024, n % 8 == 0, 1 <= r <= k");
    return SL_ERR_UNSUPPORTED;
  }
  BndArgs a{};
  a.n = n; a.k = k; a.r = r;
  a.WG = WG;
  a.sync = (unsigned*)bws;
  a.part = (double*)((char*)bws + 256);
  a.ldp = (int)(((int64_t)k * (k + 1) / 2 + 1) & ~(int64_t)1);
  a.rti = a.part + (int64_t)BMAX * a.ldp;
  a.cbak = a.rti + (int64_t)k * k + 32;
  a.status = status;
  a.status_or = status_or;
  a.Rinv = Rinv;
  a.Zt = (bf16_t*)Zt;
  a.M = M; a.N = N; a.s64 = s64;
  a.mirror = mirror;
  a.V = V; a.s32 = s32; a.optr = optr;
  {
    // fault-injection knobs live in the plan (host side), keyed by workspace
    const BndFault f = bnd_fault(bws);
    a.missing = f.missing;
    a.bound = f.bound ? f.bound : 200000000ull;   // 2 s of the 100 MHz clock
  }
  const unsigned nb = (unsigned)((n + BR - 1) / BR);
  a.nbr = (int)nb;
  hipStream_t s = (hipStream_t)stream;
  if (!final_ && (!Rinv || !Zt)) { sl_set_last_error("rsvd_boundary: Rinv and Zt required"); return SL_ERR_INVALID; }
  const bool fin = final_ != 0;
  if (k <= 16) return launch_bnd<16>(fin, nb, a, s);
  if (k <= 32) return launch_bnd<32>(fin, nb, a, s);
  if (k <= 40) return launch_bnd<40>(fin, nb, a, s);
  return launch_bnd<48>(fin, nb, a, s);
}
