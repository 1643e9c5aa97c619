// PROBE (not part of the library): phase stamps (s_memtime) of the core
// eigensolver sl_wave_la.hpp::sym_top_eig at K = 40, one workgroup of 512.
// Built by benchmarks/probe/build.sh into libprobe.so; driven by
// benchmarks/probe/eig_stamps.py.
#include "sl_wave_la.hpp"
namespace slw {
template <int K, int NT>
__device__ __forceinline__ void sym_top_eig_st(double* dd, double* ee, const double* refl, int ldr, int nt, int nv,
                                            double* lam, double* X, int ldx, int kx, double* sc, int* st, long long* ts) {
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
  __syncthreads(); if (threadIdx.x == 0) ts[1] = __builtin_amdgcn_s_memtime();
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
  __syncthreads(); if (threadIdx.x == 0) ts[2] = __builtin_amdgcn_s_memtime();
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
  if (tid < nv) {
    const int t = tid;
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
  __syncthreads(); if (threadIdx.x == 0) ts[3] = __builtin_amdgcn_s_memtime();
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
  __syncthreads(); if (threadIdx.x == 0) ts[4] = __builtin_amdgcn_s_memtime();
  // ---- residual check of every vector against T (scaled), lane = vector
  if (tid < nv) {
    const int t = tid;
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
  __syncthreads(); if (threadIdx.x == 0) ts[5] = __builtin_amdgcn_s_memtime();
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
  __syncthreads(); if (threadIdx.x == 0) ts[6] = __builtin_amdgcn_s_memtime();
  // eigenvalues back to the matrix's scale
  for (int t = tid; t < nt; t += NT) lam[t] *= tn;
  __syncthreads();
}

}  // namespace slw

namespace {
constexpr int NT = 512;
__global__ void __launch_bounds__(NT) k_probe(const double* C, int k, int r, double* out, long long* ts) {
  __shared__ __attribute__((aligned(16))) double b0[64 * 65], b1[64 * 65], b2[64 * 65];
  __shared__ __attribute__((aligned(16))) double dd[64], ee[64], lam[64], vsh[128], wsh[128];
  __shared__ int bad, fb;
  const int tid = threadIdx.x, ld = k + 1;
  for (int e = tid; e < k * k; e += NT) b0[(e / k) * ld + e % k] = C[e];
  if (tid == 0) { bad = 0; fb = 0; }
  __syncthreads();
  if (tid == 0) ts[0] = __builtin_amdgcn_s_memtime();
  if (tid < 64) slw::wave_tridiag<40>(b0, ld, k, b2, 41, dd, ee, vsh, wsh, &bad);
  __syncthreads();
  if (tid == 0) ts[7] = __builtin_amdgcn_s_memtime();
  slw::sym_top_eig_st<40, NT>(dd, ee, b2, 41, r + 1, r, lam, b1, ld, k, b0, &fb, ts);
  __syncthreads();
  if (tid == 0) ts[8] = __builtin_amdgcn_s_memtime();
  for (int c = tid; c < r; c += NT) out[c] = lam[c];
  for (int e = tid; e < k * r; e += NT) out[r + e] = b1[(e / r) * ld + e % r];
  if (tid == 0) ts[9] = fb | (bad << 1);
}
}  // namespace

extern "C" int probe_eig(const double* C, int k, int r, double* out, long long* ts, void* s) {
  k_probe<<<1, NT, 0, (hipStream_t)s>>>(C, k, r, out, ts);
  return hipGetLastError() == hipSuccess ? 0 : 1;
}
