// Device symmetric eigensolver for the small k x k (k <= 64) f64 matrices of
// the randomized SVD's final step (replaces the host LAPACK call of the
// reference's El::SVD / El::HermitianEig on the k x k core, nla/svd.hpp:281,384).
//
// Two-sided cyclic Jacobi with the round-robin (tournament) ordering: each
// round applies k/2 disjoint rotations at once, k-1 rounds make a sweep, and
// sweeps repeat until the off-diagonal mass is below (eps * ||diag||)^2.
// Jacobi gives eigenvalues of an SPD matrix to high RELATIVE accuracy, so the
// small singular values sqrt(lambda) keep their digits.
//
// Each round is one data-parallel phase over the (k/2)^2 independent 2 x 2
// blocks X <- R_i^T X R_j (plus V's rows), with the k/2 rotation parameters
// computed first: two barriers per round (A ping-pongs between two LDS
// copies, so the block phase reads one and writes the other).
// A sweep with no rotation above roundoff ends the iteration.
// One 256-thread workgroup holds A and V in LDS; the output is the top-r
// eigenpairs in descending order, packed as the randSVD plan expects:
//     out[i * r + c] = V[i][order[c]]   (k x r)
//     out[k * r + c] = sqrt(max(lambda_order[c], 0)) if want_sqrt else lambda
// so no host round trip is needed between the Gram and the final products.
#include "sl_common.hpp"

namespace {

constexpr int KMAX = 64;
constexpr int NT = 256;

__global__ void __launch_bounds__(NT)
k_sym_eig_jacobi(const double* __restrict__ Cin, int k, int ldc, int r, double* __restrict__ out,
                 int want_sqrt, int max_sweeps, int* __restrict__ sweeps_out) {
  __shared__ double AB[2][KMAX][KMAX + 1];   // ping-pong copies of A
  __shared__ double V[KMAX][KMAX + 1];
  __shared__ double cs[KMAX / 2], sn[KMAX / 2];
  __shared__ int pp[KMAX / 2], qq[KMAX / 2];
  __shared__ int rotated;
  const int tid = threadIdx.x;
  const int kp = (k + 1) & ~1;  // even number of players (a padded index is an isolated 0 row)
  const int half = kp / 2;

  for (int t = tid; t < kp * kp; t += NT) {
    const int i = t / kp, j = t - i * kp;
    double v = 0.0;
    if (i < k && j < k) v = 0.5 * (Cin[i * ldc + j] + Cin[j * ldc + i]);
    AB[0][i][j] = v;
    V[i][j] = (i == j) ? 1.0 : 0.0;
  }
  __syncthreads();

  int cur = 0, sweep = 0;
  for (; sweep < max_sweeps; ++sweep) {
    if (tid == 0) rotated = 0;
    for (int round = 0; round < kp - 1; ++round) {
      double (*A)[KMAX + 1] = AB[cur];
      double (*B)[KMAX + 1] = AB[cur ^ 1];
      // rotations of the round's kp/2 disjoint pairs (circle method:
      // position 0 fixed, positions 1..kp-1 rotate)
      if (tid < half) {
        auto player = [&](int pos) { return pos == 0 ? 0 : 1 + (pos - 1 + round) % (kp - 1); };
        int p = player(tid), q = player(kp - 1 - tid);
        if (p > q) { int t = p; p = q; q = t; }
        const double apq = A[p][q], app = A[p][p], aqq = A[q][q];
        double c = 1.0, s = 0.0;
        // skip rotations at the roundoff level of the 2 x 2 block (then a
        // sweep without any rotation ends the iteration)
        if (fabs(apq) > 1e-13 * sqrt(fabs(app * aqq))) {
          const double theta = (aqq - app) / (2.0 * apq);
          const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
          c = 1.0 / sqrt(t * t + 1.0);
          s = t * c;
          rotated = 1;
        }
        cs[tid] = c; sn[tid] = s; pp[tid] = p; qq[tid] = q;
      }
      __syncthreads();
      // B = J^T A J as independent 2 x 2 blocks (pair i rows, pair j columns):
      //   X <- R_i^T X R_j,  R = [[c, s], [-s, c]] on (p, q);  V <- V J by rows.
      const int nb = half * half, nv = kp * half;
      for (int t = tid; t < nb; t += NT) {
        const int i = t / half, j = t - i * half;
        const int pi = pp[i], qi = qq[i], pj = pp[j], qj = qq[j];
        const double ci = cs[i], si = sn[i], cj = cs[j], sj = sn[j];
        const double x00 = A[pi][pj], x01 = A[pi][qj], x10 = A[qi][pj], x11 = A[qi][qj];
        const double t00 = ci * x00 - si * x10, t01 = ci * x01 - si * x11;
        const double t10 = si * x00 + ci * x10, t11 = si * x01 + ci * x11;
        const bool zero = (i == j) && si != 0.0;   // the pivot itself: exactly 0
        B[pi][pj] = cj * t00 - sj * t01;
        B[pi][qj] = zero ? 0.0 : sj * t00 + cj * t01;
        B[qi][pj] = zero ? 0.0 : cj * t10 - sj * t11;
        B[qi][qj] = sj * t10 + cj * t11;
      }
      for (int t = tid; t < nv; t += NT) {
        const int a = t / half, j = t - a * half;
        const int pj = pp[j], qj = qq[j];
        const double cj = cs[j], sj = sn[j];
        const double vp = V[a][pj], vq = V[a][qj];
        V[a][pj] = cj * vp - sj * vq;
        V[a][qj] = sj * vp + cj * vq;
      }
      __syncthreads();
      cur ^= 1;
    }
    if (!rotated) break;
    __syncthreads();
  }
  double (*A)[KMAX + 1] = AB[cur];

  // descending order by rank counting (ties by index), top r
  __shared__ int order[KMAX];
  if (tid < k) {
    const double li = A[tid][tid];
    int rank = 0;
    for (int j = 0; j < k; ++j) {
      const double lj = A[j][j];
      rank += (lj > li) || (lj == li && j < tid);
    }
    order[rank] = tid;
  }
  __syncthreads();
  for (int t = tid; t < k * r; t += NT) {
    const int i = t / r, c = t - i * r;
    out[t] = V[i][order[c]];
  }
  if (tid < r) {
    const double l = A[order[tid]][order[tid]];
    out[k * r + tid] = want_sqrt ? sqrt(l > 0.0 ? l : 0.0) : l;
  }
  if (tid == 0 && sweeps_out) *sweeps_out = sweep;
}

// ---------------------------------------------------------------------------
// Tridiagonal path (the randSVD default, k <= 64, r <= 32): the k x k core's
// top-r eigenpairs in one launch of one workgroup, ~20x fewer dependent
// steps than Jacobi sweeps, so the randomized SVD runs start to finish on
// the device (no host LAPACK round trip between its two halves).
//   1. Householder tridiagonalisation T = Q^T C Q (wave 0, lane = row; the
//      reflectors stay in C's lower triangle), one wave => no barriers.
//   2. Eigenvalues of T by multisection on Sturm counts: the 256 threads are
//      split over the r + 1 largest eigenvalues, G points per interval per
//      round, to absolute accuracy ~eps ||T|| (LAPACK dstebz's default).
//   3. Eigenvectors of T by the twisted factorisation at each eigenvalue
//      (one lane per vector): backward UDU^T and forward LDL^T pivots, twist
//      at min |gamma|, then two recurrences out from the twist.  Vectors in a
//      close cluster (relative gap < 1e-3) are re-orthogonalised by MGS; a gap
//      under 1e-14 ||T||, a tridiagonal residual above 1e-11 ||T||,
//      non-finite data or a vanishing r-th eigenvalue set status bit 1 and the caller re-runs that call through host LAPACK.
//   4. Back-transform Q x (4 lanes per vector, shuffles only).
// Output as k_sym_eig_jacobi: out[i * r + c] = V[i][c] descending, then
// sqrt(max(lambda, 0)) (or lambda) in out[k * r + c].
constexpr int TRK = 64, TRV = 32;

// DPP lane permutations of a double (two 32-bit moves); CTRL is a dpp_ctrl code
template <int CTRL>
__device__ __forceinline__ double dppd(double x) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), CTRL, 0xF, 0xF, false);
  return __hiloint2double(hi, lo);
}

__device__ __forceinline__ double lane_d(double x, int l) {
  return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(x), l),
                          __builtin_amdgcn_readlane(__double2loint(x), l));
}

// all-lanes reductions of a full wave: quad butterflies, half-row and row
// mirrors by DPP (no LDS round trips), then the four row results by readlane
__device__ __forceinline__ double wave_sum_d(double x) {
  x += dppd<0xB1>(x);
  x += dppd<0x4E>(x);
  x += dppd<0x141>(x);
  x += dppd<0x140>(x);
  return (lane_d(x, 0) + lane_d(x, 16)) + (lane_d(x, 32) + lane_d(x, 48));
}

__device__ __forceinline__ double wave_min_d(double x) {
  x = fmin(x, dppd<0xB1>(x));
  x = fmin(x, dppd<0x4E>(x));
  x = fmin(x, dppd<0x141>(x));
  x = fmin(x, dppd<0x140>(x));
  return fmin(fmin(lane_d(x, 0), lane_d(x, 16)), fmin(lane_d(x, 32), lane_d(x, 48)));
}

__device__ __forceinline__ double wave_max_d(double x) {
  x = fmax(x, dppd<0xB1>(x));
  x = fmax(x, dppd<0x4E>(x));
  x = fmax(x, dppd<0x141>(x));
  x = fmax(x, dppd<0x140>(x));
  return fmax(fmax(lane_d(x, 0), lane_d(x, 16)), fmax(lane_d(x, 32), lane_d(x, 48)));
}

__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// One Householder step j of the register-resident tridiagonalisation (wave 0,
// lane i holds row i): reflector from column j, p = A v, w = p - (v.p) v,
// A -= 2 (v w^T + w v^T) on the trailing columns only.
template <int K, int J>
__device__ __forceinline__ void tri_step(double (&arow)[K], int i, double safmin, double* vsh, double* wsh,
                                         double (*refl)[K + 1], double* dd, double* ee) {
  constexpr int c0 = (J + 1) & ~1;               // first active column, 16-B aligned
  double xi = arow[J];
  const double ajj = xi;                         // lane J: its diagonal (final now)
  xi = (i > J) ? xi : 0.0;
  const double s2 = wave_sum_d(xi * xi);
  const double x0 = lane_d(xi, J + 1);
  double vi = 0.0, alpha = x0;
  if (s2 - x0 * x0 > safmin * 4.0) {
    alpha = x0 >= 0.0 ? -sqrt(s2) : sqrt(s2);
    const double vn = sqrt(2.0 * (s2 - alpha * x0));
    vi = (xi - (i == J + 1 ? alpha : 0.0)) / vn;
    vi = (i > J) ? vi : 0.0;
  }
  if (i == J) { dd[J] = ajj; ee[J] = alpha; }
  if (i < K) {
    vsh[i] = vi;
    refl[i][J] = vi;
  }
  wave_lds_sync();
  // the whole broadcast vector in registers first (one LDS round trip per
  // vector, not one per pair of elements)
  double vv[K];
#pragma unroll
  for (int c = c0; c < K; c += 2) {
    const double2 t = *(const double2*)(vsh + c);
    vv[c] = t.x;
    vv[c + 1] = t.y;
  }
  double p0 = 0.0, p1 = 0.0;
#pragma unroll
  for (int c = c0; c < K; c += 2) {
    p0 = fma(arow[c], vv[c], p0);
    p1 = fma(arow[c + 1], vv[c + 1], p1);
  }
  const double p = (i > J) ? p0 + p1 : 0.0;
  const double Kd = wave_sum_d(vi * p);
  const double wi = (i > J) ? p - Kd * vi : 0.0;
  if (i < K) wsh[i] = wi;
  wave_lds_sync();
  double ww[K];
#pragma unroll
  for (int c = c0; c < K; c += 2) {
    const double2 t = *(const double2*)(wsh + c);
    ww[c] = t.x;
    ww[c + 1] = t.y;
  }
  const double v2 = 2.0 * vi, w2 = 2.0 * wi;
#pragma unroll
  for (int c = c0; c < K; ++c) arow[c] = fma(-v2, ww[c], fma(-w2, vv[c], arow[c]));
  wave_lds_sync();   // vsh / wsh are rewritten next step
}

template <int K, int J>
__device__ __forceinline__ void tri_steps(double (&arow)[K], int i, int k, double safmin, double* vsh, double* wsh,
                                          double (*refl)[K + 1], double* dd, double* ee) {
  if constexpr (J + 2 < K) {
    if (J + 2 < k) {
      tri_step<K, J>(arow, i, safmin, vsh, wsh, refl, dd, ee);
      tri_steps<K, J + 1>(arow, i, k, safmin, vsh, wsh, refl, dd, ee);
    }
  }
}

template <int K, bool ST>
__global__ void __launch_bounds__(NT)
k_sym_eig_tridiag(const double* __restrict__ Cin, int k, int ldc, int r, double* __restrict__ out, int want_sqrt,
                  int* __restrict__ status, long long* __restrict__ stamps) {
  __shared__ double refl[K][K + 1];     // Householder vectors (column j = step j)
  __shared__ __attribute__((aligned(16))) double vsh[K], wsh[K];
  __shared__ double dd[K], ee[K], e2[K];
  __shared__ double lam[K];
  __shared__ double T1[K][TRV + 1];     // per-vector pivots, then the vector itself
  __shared__ double bnd[2];
  __shared__ int bad_s, clus_s;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const double eps = 2.220446049250313e-16, safmin = 2.2250738585072014e-308;
  if constexpr (ST) { if (tid == 0) stamps[0] = clock64(); }
  if (tid == 0) { bad_s = 0; clus_s = 0; }
  __syncthreads();

  // ---- 1. tridiagonalisation (wave 0, lane i keeps row i in registers) -----
  if (wid == 0) {
    const int i = lane;
    double arow[K];
    int nf = 0;
#pragma unroll
    for (int c = 0; c < K; ++c) {
      double v = 0.0;
      if (i < k && c < k) v = 0.5 * (Cin[i * ldc + c] + Cin[c * ldc + i]);
      nf |= !isfinite(v);
      arow[c] = v;
    }
    if (nf) bad_s = 1;
    // steps instantiated per compile-time j (template recursion, a uniform
    // exit at k): the column j and the active range c >= j + 1 are static
    // register indices, so arow stays in registers and each step only touches
    // the trailing columns
    tri_steps<K, 0>(arow, i, k, safmin, vsh, wsh, refl, dd, ee);
    // the last two diagonal entries and the last off-diagonal one
    double dl = 0.0, el = 0.0;
#pragma unroll
    for (int c = 0; c < K; ++c) {
      if (c == i) dl = arow[c];
      if (c == k - 2) el = arow[c];
    }
    if (k >= 2 && i == k - 2) dd[k - 2] = dl;
    if (i == k - 1) { dd[k - 1] = dl; ee[k - 1] = 0.0; if (k >= 2) ee[k - 2] = el; }
    if (k == 1 && i == 0) dd[0] = dl;
    wave_lds_sync();
    if (i < k) e2[i] = ee[i] * ee[i];
    double glo = dd[0], ghi = dd[0];
    if (i < k) {
      const double rad = fabs(ee[i]) + (i > 0 ? fabs(ee[i - 1]) : 0.0);
      glo = dd[i] - rad;
      ghi = dd[i] + rad;
    }
    glo = wave_min_d(glo);
    ghi = wave_max_d(ghi);
    if (i == 0) {
      const double tn = fmax(fabs(glo), fabs(ghi));
      bnd[0] = glo - 2.0 * eps * tn - 4.0 * safmin;
      bnd[1] = ghi + 2.0 * eps * tn + 4.0 * safmin;
    }
  }
  __syncthreads();
  if constexpr (ST) { if (tid == 0) stamps[1] = clock64(); }

  // ---- 2. multisection for the nt largest eigenvalues ----------------------
  const int nt = r < k ? r + 1 : k;
  double pivmin = 1.0;
  for (int i = 0; i + 1 < k; ++i) pivmin = fmax(pivmin, e2[i]);
  pivmin *= safmin;
  const double tnorm = fmax(fabs(bnd[0]), fabs(bnd[1]));
  const double atol = 2.0 * eps * tnorm + 2.0 * pivmin;
  // One small lane group per wanted eigenvalue (8 lanes, 4 when more than 32
  // are wanted), groups never straddle a wave: each round every lane takes
  // one multisection point, and the group's new bracket is a 3-step DPP
  // max / min over its lanes -- no LDS, no workgroup barrier; the waves run
  // their rounds independently until all of their brackets are converged.
  const int GL = nt <= NT / 8 ? 8 : 4;
  const int tg = tid / GL, g = tid - tg * GL;
  const bool act = tg < nt;
  const int idx = k - 1 - tg;        // ascending index of this group's eigenvalue
  // T in registers for the whole multisection (the Sturm recurrence is one
  // dependent chain; LDS reads inside it exposed their latency every step)
  double dR[K], e2R[K];
#pragma unroll
  for (int i = 0; i < K; ++i) {
    dR[i] = i < k ? dd[i] : 0.0;
    e2R[i] = (i + 1 < k) ? e2[i] : 0.0;
  }
  const double gfrac = 1.0 / (double)(GL + 1);
  double lo = bnd[0], hi = bnd[1];
  for (int round = 0; round < 80; ++round) {
    const bool conv = !act || (hi - lo) <= fmax(atol, 2.0 * eps * fmax(fabs(lo), fabs(hi)));
    if (__all(conv)) break;
    if (act) {
      const double x = lo + (hi - lo) * (double)(g + 1) * gfrac;
      double q = dR[0] - x;
      if (fabs(q) < pivmin) q = -pivmin;
      int c = q < 0.0;
#pragma unroll
      for (int i = 1; i < K; ++i) {
        if (i < k) {
          // e2 / q by v_rcp_f64 + one Newton step (~full precision; only
          // the sign of q enters the count)
          double y = __builtin_amdgcn_rcp(q);
          y = fma(fma(-q, y, 1.0), y, y);
          q = (dR[i] - x) - e2R[i - 1] * y;
          if (fabs(q) < pivmin) q = -pivmin;
          c += q < 0.0;
        }
      }
      // fewer than idx + 1 eigenvalues below x: x is a lower bound
      double nlo = c <= idx ? x : lo, nhi = c <= idx ? hi : x;
      nlo = fmax(nlo, dppd<0xB1>(nlo));
      nhi = fmin(nhi, dppd<0xB1>(nhi));
      nlo = fmax(nlo, dppd<0x4E>(nlo));
      nhi = fmin(nhi, dppd<0x4E>(nhi));
      if (GL == 8) {
        nlo = fmax(nlo, dppd<0x141>(nlo));
        nhi = fmin(nhi, dppd<0x141>(nhi));
      }
      lo = nlo;
      hi = nhi;
    }
  }
  if (act && g == 0) lam[tg] = 0.5 * (lo + hi);
  __syncthreads();
  if constexpr (ST) { if (tid == 0) stamps[2] = clock64(); }

  // ---- 3. twisted-factorisation eigenvectors (wave 0, lane = vector) -------
  const double gtol = 1e-3 * tnorm;
  if (wid == 0) {
    const int v = lane;
    if (v < r) {
      const double l = lam[v];
      const double gap = fmin(v > 0 ? lam[v - 1] - l : 1e300, v + 1 < nt ? l - lam[v + 1] : 1e300);
      if (!(gap > 1e-14 * tnorm)) atomicOr(&bad_s, 1);   // numerically repeated
      if (gap < gtol) atomicOr(&clus_s, 1);
      // backward pivots D-_i (slot i)
      double dm = dd[k - 1] - l;
      if (fabs(dm) < pivmin) dm = -pivmin;
      T1[k - 1][v] = dm;
      for (int i = k - 2; i >= 0; --i) {
        dm = (dd[i] - l) - e2[i] / dm;
        if (fabs(dm) < pivmin) dm = -pivmin;
        T1[i][v] = dm;
      }
      // forward pivots D+_i and the twist gamma_i = D+_i + D-_i - (d_i - l)
      double dp = dd[0] - l;
      if (fabs(dp) < pivmin) dp = -pivmin;
      int rt = 0;
      double best = fabs(T1[0][v]);
      for (int i = 1; i < k; ++i) {
        dp = (dd[i] - l) - e2[i - 1] / dp;
        if (fabs(dp) < pivmin) dp = -pivmin;
        const double gm = fabs(dp + T1[i][v] - (dd[i] - l));
        if (gm < best) { best = gm; rt = i; }
      }
      // D+_i below the twist (slots 0..rt-1), then the two recurrences
      dp = dd[0] - l;
      if (fabs(dp) < pivmin) dp = -pivmin;
      for (int i = 0; i < rt; ++i) {
        T1[i][v] = dp;
        dp = (dd[i + 1] - l) - e2[i] / dp;
        if (fabs(dp) < pivmin) dp = -pivmin;
      }
      double x = 1.0, nrm = 1.0;
      for (int i = rt - 1; i >= 0; --i) {
        x = -(ee[i] / T1[i][v]) * x;
        T1[i][v] = x;
        nrm = fma(x, x, nrm);
      }
      T1[rt][v] = 1.0;
      x = 1.0;
      for (int i = rt; i + 1 < k; ++i) {
        x = -(ee[i] / T1[i + 1][v]) * x;
        T1[i + 1][v] = x;
        nrm = fma(x, x, nrm);
      }
      const double sc = 1.0 / sqrt(nrm);
      if (!isfinite(sc) || !(sc > 0.0)) atomicOr(&bad_s, 1);
      for (int i = 0; i < k; ++i) T1[i][v] *= sc;
    }
    wave_lds_sync();
    if (clus_s) {
      // MGS inside close clusters (lane = component)
      const int i = lane;
      for (int c = 1; c < r; ++c) {
        double xc = i < k ? T1[i][c] : 0.0;
        bool touched = false;
        for (int u = 0; u < c; ++u) {
          if (lam[u] - lam[c] >= gtol) continue;
          const double dt = wave_sum_d(i < k ? T1[i][u] * xc : 0.0);
          if (i < k) xc -= dt * T1[i][u];
          touched = true;
        }
        if (touched) {
          const double n2 = wave_sum_d(xc * xc);
          if (i < k) T1[i][c] = xc / sqrt(n2);
        }
        wave_lds_sync();
      }
    }
    // safety net: every vector must be an eigenvector of T to ~eps ||T||
    if (lane < r) {
      const double l = lam[lane];
      double r2 = 0.0;
      for (int i = 0; i < k; ++i) {
        double tx = dd[i] * T1[i][lane];
        if (i > 0) tx += ee[i - 1] * T1[i - 1][lane];
        if (i + 1 < k) tx += ee[i] * T1[i + 1][lane];
        const double d = tx - l * T1[i][lane];
        r2 = fma(d, d, r2);
      }
      if (!(sqrt(r2) <= 1e-11 * tnorm + 1e-300)) atomicOr(&bad_s, 1);
    }
  }
  __syncthreads();
  if constexpr (ST) { if (tid == 0) stamps[3] = clock64(); }

  // ---- 4. back-transform x <- H_0 ... H_{k-3} x (4 lanes per vector) --------
  {
    const int v = tid >> 2, q = tid & 3;
    if (v < r) {
      double xv[K / 4];
#pragma unroll
      for (int u = 0; u < K / 4; ++u) {
        const int i = q + 4 * u;
        xv[u] = i < k ? T1[i][v] : 0.0;
      }
      for (int j = k - 3; j >= 0; --j) {
        double part = 0.0;
#pragma unroll
        for (int u = 0; u < K / 4; ++u) part = fma(refl[q + 4 * u][j], xv[u], part);
        part += dppd<0xB1>(part);
        part += dppd<0x4E>(part);
#pragma unroll
        for (int u = 0; u < K / 4; ++u) xv[u] -= 2.0 * part * refl[q + 4 * u][j];
      }
#pragma unroll
      for (int u = 0; u < K / 4; ++u) {
        const int i = q + 4 * u;
        if (i < k) T1[i][v] = xv[u];
      }
    }
  }
  __syncthreads();
  if constexpr (ST) { if (tid == 0) stamps[4] = clock64(); }
  for (int t = tid; t < k * r; t += NT) {
    const int i = t / r, c = t - i * r;
    out[t] = T1[i][c];
  }
  if (tid < r) {
    const double l = lam[tid];
    out[k * r + tid] = want_sqrt ? sqrt(l > 0.0 ? l : 0.0) : l;
  }
  if (tid == 0) {
    // with want_sqrt (singular values of a Gram) a vanishing r-th eigenvalue
    // means fewer than r resolvable directions: the host path decides
    const int bad = bad_s || (want_sqrt && !(lam[r - 1] > 1e-30 * fmax(lam[0], 1e-300)));
    if (bad && status) atomicOr(status, 1);
  }
}

template <bool ST>
int launch_tridiag(const double* C, int k, int ldc, int r, double* out, int want_sqrt, int* status,
                   long long* stamps, hipStream_t s) {
  if (k <= 16)
    k_sym_eig_tridiag<16, ST><<<1, NT, 0, s>>>(C, k, ldc, r, out, want_sqrt, status, stamps);
  else if (k <= 32)
    k_sym_eig_tridiag<32, ST><<<1, NT, 0, s>>>(C, k, ldc, r, out, want_sqrt, status, stamps);
  else if (k <= 48)
    k_sym_eig_tridiag<48, ST><<<1, NT, 0, s>>>(C, k, ldc, r, out, want_sqrt, status, stamps);
  else
    k_sym_eig_tridiag<64, ST><<<1, NT, 0, s>>>(C, k, ldc, r, out, want_sqrt, status, stamps);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

}  // namespace

// Top-r eigenpairs by the tridiagonal path (k <= 64, r <= 32); status bit 1 =
// the caller should redo this matrix on the host (see the kernel comment).
SL_API int sl_sym_eig_tridiag(const double* C, int k, int ldc, int r, double* out, int want_sqrt, int* status,
                              void* stream) {
  if (k <= 0 || k > TRK || r <= 0 || r > k || r > TRV || ldc < k) return SL_ERR_DIMENSION;
  return launch_tridiag<false>(C, k, ldc, r, out, want_sqrt, status, nullptr, (hipStream_t)stream);
}

// diagnostic: shader-clock stamps at the phase boundaries (5 x int64)
SL_API int sl_sym_eig_tridiag_stamps(const double* C, int k, int ldc, int r, double* out, int* status,
                                     long long* stamps, void* stream) {
  if (k <= 0 || k > TRK || r <= 0 || r > k || r > TRV || ldc < k) return SL_ERR_DIMENSION;
  return launch_tridiag<true>(C, k, ldc, r, out, 0, status, stamps, (hipStream_t)stream);
}

SL_API int sl_sym_eig_topr(const double* C, int k, int ldc, int r, double* out, int want_sqrt,
                           int max_sweeps, int* sweeps_out, void* stream) {
  if (k <= 0 || k > KMAX || r <= 0 || r > k || ldc < k) return SL_ERR_DIMENSION;
  k_sym_eig_jacobi<<<1, NT, 0, (hipStream_t)stream>>>(C, k, ldc, r, out, want_sqrt,
                                                       max_sweeps > 0 ? max_sweeps : 30, sweeps_out);
  SL_LAUNCH_CHECK();
  return SL_OK;
}
