// Device-resident small linear algebra of the randomized SVD
// (reference nla/svd.hpp:71-149 PowerIteration's re-orthonormalisation and
// :278-317 ApproximateSVD's El::SVD of the k x k core), so the whole call runs
// on the GPU with no host round trip.
//
//   k_gram_la<INTER>  between two power passes: H = W^T W of the reduced
//                     W (n x k, f64), Cholesky H = R^T R with pivot dropping,
//                     R^{-1}; k_make_zt then forms the next pass operand
//                     Z^T = (W R^{-1})^T in bf16.  ("orth(W)": CholeskyQR.)
//   k_gram_la<FINAL>  after the final pass: H = W^T W (W = A^T Y), the
//                     Cholesky Y^T Y = Rt^T Rt of the pass's fp64 Gram, Rt^{-1},
//                     the symmetric core C = Rt^{-T} H Rt^{-1} = Ub S^2 Ub^T,
//                     a cyclic Jacobi eigensolve of C, and the small factors
//                     M = Rt^{-1} Ub_r (U = Y M) and N = M S^{-1} (V = W N).
//
// Structure: the n rows of W are split over NG workgroups, each forms the
// partial Gram of its rows (f64) and publishes it with an agent-scope release
// and a ticket counter; the LAST arriving workgroup (agent-scope acquire)
// sums the partials and runs the k x k algebra alone in LDS (k <= 64).
//
// Jacobi: round-robin (circle) ordering, k/2 disjoint rotations per round,
// ONE workgroup barrier per round (A ping-pongs between two LDS copies, every
// thread derives the rotations it needs from the old copy).  A rotation's
// tangent comes from an f32 estimate refined by one f64 Newton step on
// a_pq t^2 + (a_qq - a_pp) t - a_pq = 0 (no f64 division), its cosine from an
// f32 rsqrt refined in f64: f64-accurate rotations at f32 latency.  Sweeps
// stop once every pair's |a_pq| / sqrt|a_pp a_qq| was below 1e-8 before its
// rotation (the quadratic convergence of that sweep leaves ~1e-16).
#include "sl_common.hpp"
#include "sl_rng.hpp"

namespace {

constexpr int NT = 512;      // threads per workgroup of the small-LA kernels
constexpr int KMAX = 64;

enum : int { ST_PIVOT = 1, ST_NONFINITE = 2, ST_NOCONV = 4, ST_RANK = 8 };

// ---------------------------------------------------------------- Cholesky
// In LDS: G (k x ld) symmetric (upper triangle read) -> R (upper, k x ld,
// lower part zeroed).  A pivot at or below 1e-13 * max diag drops that
// direction (its row of R is zero) and sets ST_PIVOT.  One barrier per step:
// every thread scales the pivot row entries it needs itself.
__device__ void chol_upper(const double* G, double* R, double* T, int k, int ld, int* st, double* red) {
  const int tid = threadIdx.x;
  for (int e = tid; e < k * ld; e += NT) T[e] = G[e];
  if (tid == 0) {
    double mx = 0.0;
    for (int i = 0; i < k; ++i) mx = fmax(mx, fabs(G[i * ld + i]));
    red[0] = mx;
  }
  __syncthreads();
  const double thr = 1e-13 * red[0];
  for (int j = 0; j < k; ++j) {
    const double d = T[j * ld + j];
    const bool ok = d > thr && d == d;
    const double rs = ok ? 1.0 / sqrt(d) : 0.0;
    // row j of R
    for (int l = tid; l < k; l += NT) R[j * ld + l] = l < j ? 0.0 : T[j * ld + l] * rs;
    // trailing update of the upper triangle (reads only row j of T)
    if (ok) {
      const double rd = 1.0 / d;
      for (int e = tid; e < k * k; e += NT) {
        const int i = e / k, l = e - i * k;
        if (i > j && l >= i) T[i * ld + l] -= T[j * ld + i] * T[j * ld + l] * rd;
      }
    } else if (tid == 0) {
      *st |= ST_PIVOT;
    }
    __syncthreads();
  }
}

// X = R^{-1} for upper-triangular R (zero rows stay zero): eliminate column i
// of R from the identity, i = k-1 .. 0; two barriers per step.
__device__ void tri_inv_upper(const double* R, double* X, int k, int ld) {
  const int tid = threadIdx.x;
  for (int e = tid; e < k * ld; e += NT) {
    const int i = e / ld, c = e - i * ld;
    X[e] = (i == c && c < k) ? 1.0 : 0.0;
  }
  __syncthreads();
  for (int i = k - 1; i >= 0; --i) {
    const double rii = R[i * ld + i];
    const double ri = rii != 0.0 ? 1.0 / rii : 0.0;
    // X[i][*] /= R[i][i]  (row i of X only has entries at c >= i)
    for (int c = tid; c < k; c += NT) X[i * ld + c] *= ri;
    __syncthreads();
    // rows p < i:  X[p][c] -= R[p][i] X[i][c]
    for (int e = tid; e < i * k; e += NT) {
      const int p = e / k, c = e - p * k;
      if (c >= i) X[p * ld + c] -= R[p * ld + i] * X[i * ld + c];
    }
    __syncthreads();
  }
}

// C = A^T B (transa) or A B for k x k LDS matrices, four outputs per thread
__device__ void small_gemm(const double* A, const double* B, double* C, int k, int ld, bool transa) {
  const int tid = threadIdx.x;
  const int nq = (k + 3) / 4;
  for (int e = tid; e < k * nq; e += NT) {
    const int i = e / nq, c0 = 4 * (e - i * nq);
    double a0 = 0, a1 = 0, a2 = 0, a3 = 0;
    for (int l = 0; l < k; ++l) {
      const double a = transa ? A[l * ld + i] : A[i * ld + l];
      const double* b = B + l * ld + c0;
      a0 += a * b[0];
      if (c0 + 1 < k) a1 += a * b[1];
      if (c0 + 2 < k) a2 += a * b[2];
      if (c0 + 3 < k) a3 += a * b[3];
    }
    C[i * ld + c0] = a0;
    if (c0 + 1 < k) C[i * ld + c0 + 1] = a1;
    if (c0 + 2 < k) C[i * ld + c0 + 2] = a2;
    if (c0 + 3 < k) C[i * ld + c0 + 3] = a3;
  }
}

// ---------------------------------------------------------------- Jacobi
struct Rot { double c, s, t; bool rot; };

// rotation zeroing a_pq of the (p, q) plane (J = [[c, s], [-s, c]]).
// big: this pair was still coupled above 1e-6 relative before the rotation.
__device__ __forceinline__ Rot jrot(double app, double aqq, double apq, bool* big) {
  Rot r{1.0, 0.0, 0.0, false};
  const double pq2 = apq * apq, dd = fabs(app * aqq);
  *big = pq2 > 1e-12 * dd;
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
__device__ double* jacobi(double* A, double* B, double* V, int kp, int ld, int max_sweeps, int* flags, int* st) {
  (void)B;
  __shared__ unsigned short btab[KMAX / 2 * (KMAX / 2 + 1) / 2];
  __shared__ unsigned short rtab[(KMAX - 1) * (KMAX / 2)];
  __shared__ double rot_c[KMAX / 2], rot_s[KMAX / 2], rot_t[KMAX / 2];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int hp = kp / 2;
  const int nA = hp * (hp + 1) / 2;
  for (int e = tid; e < kp * ld; e += NT) {
    const int i = e / ld, c = e - i * ld;
    V[e] = (i == c) ? 1.0 : 0.0;
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
        const Rot R = jrot(A[p * ld + p], A[q * ld + q], A[p * ld + q], &big);
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
      } else {
        // V <- V J: item e = (row v, pair j), e = tid, tid + 256, ...
#pragma unroll 1
        for (int e = tid; e < kp * hp; e += 256) {
          const int v = e / hp, j = e - v * hp;
          const unsigned short pq = rt[j];
          const double t = rot_t[j], c = rot_c[j], sn = rot_s[j];
          const int p = pq & 255, q = pq >> 8;
          double* vr = V + v * ld;
          const double vp = vr[p], vq = vr[q];
          if (t != 0.0) {
            vr[p] = c * vp - sn * vq;
            vr[q] = sn * vp + c * vq;
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

// ---------------------------------------------------------------- kernel
template <bool FINAL>
__global__ void __launch_bounds__(NT)
k_gram_la(const double* __restrict__ W, int n, int k, int ldw, double* __restrict__ part,
          unsigned* __restrict__ counter, const double* __restrict__ Gy, int r, double* __restrict__ Rinv,
          float* __restrict__ M, double* __restrict__ N, double* __restrict__ s_out, int* __restrict__ status,
          int max_sweeps) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  const int tid = threadIdx.x;
  const int ld = k + 1;
  const int mat = KMAX * (KMAX + 1);
  double* b0 = sm;
  double* b1 = sm + mat;
  double* b2 = sm + 2 * mat;
  double* b3 = sm + 3 * mat;
  double* red = sm + 4 * mat;           // small scratch (16 doubles)
  int* iscr = (int*)(red + 16);         // flags[4], order[KMAX], is_last
  int* flags = iscr;
  int* order = iscr + 4;
  int* is_last = iscr + 4 + KMAX;
  __shared__ int st_sh;

  // ---- partial Gram of this workgroup's rows (upper triangle, f64)
  const int ng = gridDim.x;
  const int ch = (n + ng - 1) / ng;
  const int r0 = blockIdx.x * ch, r1 = min(n, r0 + ch);
  const int nr = r1 > r0 ? r1 - r0 : 0;
  double* chunk = b0;   // nr x k (row stride k)
  for (int e = tid; e < nr * k; e += NT) {
    const int i = e / k, c = e - i * k;
    chunk[e] = W[(int64_t)(r0 + i) * ldw + c];
  }
  __syncthreads();
  double* myp = part + (int64_t)blockIdx.x * k * k;
  for (int e = tid; e < k * k; e += NT) {
    const int i = e / k, c = e - i * k;
    if (c < i) continue;
    double a = 0.0;
    for (int row = 0; row < nr; ++row) a += chunk[row * k + i] * chunk[row * k + c];
    myp[e] = a;
  }
  // ---- publish, count, last arriver continues (release / acquire, agent scope)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned t = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    *is_last = (t == (unsigned)ng - 1);
    if (*is_last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    st_sh = 0;
  }
  __syncthreads();
  if (!*is_last) return;

  // ---- H = sum of the partials (symmetric, f64) -> b0
  for (int e = tid; e < k * k; e += NT) {
    const int i = e / k, c = e - i * k;
    if (c < i) continue;
    double a = 0.0;
    for (int g = 0; g < ng; ++g) a += part[(int64_t)g * k * k + e];
    b0[i * ld + c] = a;
    b0[c * ld + i] = a;
  }
  if (tid == 0) *counter = 0u;   // ready for the next launch (graph replays)
  __syncthreads();
  if (!FINAL) {
    // ---- INTER: H = R^T R, X = R^{-1} (f64, k x k) -> Rinv
    chol_upper(b0, b1, b2, k, ld, &st_sh, red);
    tri_inv_upper(b1, b2, k, ld);
    for (int e = tid; e < k * k; e += NT) {
      const int i = e / k, c = e - i * k;
      const double v = b2[i * ld + c];
      if (!(fabs(v) < 1e300)) atomicOr(&st_sh, ST_NONFINITE);
      Rinv[e] = v;
    }
    __syncthreads();
    if (tid == 0) atomicOr(status, st_sh);
    return;
  }
  // ---- FINAL: Y^T Y = Rt^T Rt (b1 <- Gy, Rt -> b2), Rti -> b3
  for (int e = tid; e < k * k; e += NT) {
    const int i = e / k, c = e - i * k;
    b1[i * ld + c] = Gy[e];
  }
  __syncthreads();
  chol_upper(b1, b2, b3, k, ld, &st_sh, red);   // b3 scratch
  tri_inv_upper(b2, b3, k, ld);                 // Rti in b3
  // C = Rti^T H Rti:  T = H Rti -> b1, C = Rti^T T -> b2
  small_gemm(b0, b3, b1, k, ld, false);
  __syncthreads();
  small_gemm(b3, b1, b2, k, ld, true);
  __syncthreads();
  // symmetrise, pad to an even order with an isolated zero row / column
  const int kp = k + (k & 1);
  for (int e = tid; e < kp * kp; e += NT) {
    const int i = e / kp, c = e - i * kp;
    double v = 0.0;
    if (i < k && c < k) v = 0.5 * (b2[i * ld + c] + b2[c * ld + i]);
    b0[i * ld + c] = v;
  }
  __syncthreads();
  for (int e = tid; e < kp * kp; e += NT) {
    const int i = e / kp, c = e - i * kp;
    b2[i * ld + c] = b0[i * ld + c];
  }
  __syncthreads();
  // Jacobi on b2 (ping-pong b0), V in b1
  double* Af = jacobi(b2, b0, b1, kp, ld, max_sweeps, flags, &st_sh);
  // ---- descending order of the k eigenvalues (rank by comparison)
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
  // ---- s, M = Rti Ub_r (f32), N = M S^{-1} (f64)
  for (int c = tid; c < r; c += NT) {
    const double lam = Af[order[c] * ld + order[c]];
    s_out[c] = lam > 0.0 ? sqrt(lam) : 0.0;
    if (!(lam > 0.0)) atomicOr(&st_sh, ST_RANK);
    if (!(lam == lam)) atomicOr(&st_sh, ST_NONFINITE);
  }
  __syncthreads();
  for (int e = tid; e < k * r; e += NT) {
    const int i = e / r, c = e - i * r;
    const int oc = order[c];
    double a = 0.0;
    for (int l = i; l < k; ++l) a += b3[i * ld + l] * b1[l * ld + oc];
    M[e] = (float)a;
    const double lam = Af[oc * ld + oc];
    N[e] = lam > 0.0 ? a / sqrt(lam) : 0.0;
  }
  if (tid == 0) atomicOr(status, st_sh);
}

// Z^T (k x n bf16) = (W R^{-1})^T, R^{-1} upper triangular (k x k f64)
__global__ void __launch_bounds__(256)
k_make_zt(const double* __restrict__ W, int n, int k, int ldw, const double* __restrict__ Rinv, bf16_t* __restrict__ Zt) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)n * k) return;
  const int c = (int)(t / n), i = (int)(t - (int64_t)c * n);
  double a = 0.0;
  for (int l = 0; l <= c; ++l) a += W[(int64_t)i * ldw + l] * Rinv[l * k + c];
  Zt[(int64_t)c * n + i] = f_to_bf16((float)a);
}

// V (n x r f32) = W (n x k f64) N (k x r f64); s32 = s64 (r)
__global__ void __launch_bounds__(256)
k_make_v(const double* __restrict__ W, int n, int k, int ldw, const double* __restrict__ N, int r, float* __restrict__ V,
         const double* __restrict__ s64, float* __restrict__ s32) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (s32 && t < r) s32[t] = (float)s64[t];
  if (t >= (int64_t)n * r) return;
  const int i = (int)(t / r), c = (int)(t - (int64_t)i * r);
  double a = 0.0;
  for (int l = 0; l < k; ++l) a += W[(int64_t)i * ldw + l] * N[l * r + c];
  V[t] = (float)a;
}

// FJLT operator of the rowwise sketch A Omega^T, as the pass operand Z^T
// (k x n bf16): Z^T[j][i] = scale * d_i * c_{p_j} cos(pi p_j (2 i + 1) / 2n)
// with d the n Rademacher signs at stream offset baseD and p_j the k sampled
// DCT-II frequencies at baseS (reference FJLT_data.hpp:79-86, sketch/fjlt.py)
__global__ void __launch_bounds__(256)
k_fjlt_zt(uint64_t seed, uint64_t baseD, uint64_t baseS, double scale, int k, int n, bf16_t* __restrict__ Zt) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)n * k) return;
  const int j = (int)(t / n), i = (int)(t - (int64_t)j * n);
  const int64_t p = sl::uniform_int(sl::stream_block(seed, baseS + (uint64_t)j).x, 0, n - 1);
  const double d = (sl::stream_block(seed, baseD + (uint64_t)i).x >> 63) ? 1.0 : -1.0;
  const int64_t a = (p * (2 * (int64_t)i + 1)) % (4 * (int64_t)n);
  const double w = 3.14159265358979323846 / (2.0 * (double)n);
  const double c0 = sqrt(1.0 / (double)n), c1 = sqrt(2.0 / (double)n);
  Zt[t] = f_to_bf16((float)(cos(w * (double)a) * (p == 0 ? c0 : c1) * scale * d));
}

size_t gram_la_lds() { return (size_t)(4 * KMAX * (KMAX + 1) + 16) * sizeof(double) + (4 + KMAX + 1) * sizeof(int); }

}  // namespace

// ------------------------------------------------------------------ C ABI
constexpr int SL_GRAM_NG = 16;   // workgroups of the partial-Gram phase

SL_API int64_t sl_rsvd_gram_workspace(int k) { return (int64_t)SL_GRAM_NG * k * k * 8 + 256; }

// Between two passes: Rinv (k x k f64) of the Cholesky factor of W^T W.
// ws: sl_rsvd_gram_workspace(k) bytes, its first 4 bytes a zeroed counter
// (the kernel leaves it zero again).
SL_API int sl_rsvd_inter_la(const double* W, int n, int k, int ldw, void* ws, double* Rinv, int* status, void* stream) {
  if (k < 1 || k > KMAX || n < 1 || (int64_t)((n + SL_GRAM_NG - 1) / SL_GRAM_NG) * k > 4 * KMAX * (KMAX + 1)) {
    sl_set_last_error("rsvd_inter_la: 1 <= k <= 64 and n * k <= 266240");
    return SL_ERR_UNSUPPORTED;
  }
  hipStream_t s = (hipStream_t)stream;
  static bool attr = false;
  if (!attr) {
    SL_HIP_CHECK(hipFuncSetAttribute((const void*)k_gram_la<false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)gram_la_lds()));
    attr = true;
  }
  unsigned* counter = (unsigned*)ws;
  double* part = (double*)((char*)ws + 256);
  const int ng = n < SL_GRAM_NG ? n : SL_GRAM_NG;
  k_gram_la<false><<<ng, NT, gram_la_lds(), s>>>(W, n, k, ldw, part, counter, nullptr, 0, Rinv, nullptr, nullptr,
                                                nullptr, status, 0);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// Z^T = (W Rinv)^T as bf16 (k x n)
SL_API int sl_rsvd_make_zt(const double* W, int n, int k, int ldw, const double* Rinv, void* Zt, void* stream) {
  const int64_t tot = (int64_t)n * k;
  k_make_zt<<<(unsigned)((tot + 255) / 256), 256, 0, (hipStream_t)stream>>>(W, n, k, ldw, Rinv, (bf16_t*)Zt);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// After the final pass: s (r), M (k x r f32), N (k x r f64) from W (n x k
// f64) and the fp64 Gram of Y (k x k).
SL_API int sl_rsvd_final_la(const double* W, int n, int k, int ldw, const double* Gy, int r, void* ws, float* M,
                            double* N, double* s, int* status, int max_sweeps, void* stream) {
  if (k < 1 || k > KMAX || r < 1 || r > k || (int64_t)((n + SL_GRAM_NG - 1) / SL_GRAM_NG) * k > 4 * KMAX * (KMAX + 1)) {
    sl_set_last_error("rsvd_final_la: 1 <= r <= k <= 64 and n * k <= 266240");
    return SL_ERR_UNSUPPORTED;
  }
  hipStream_t st = (hipStream_t)stream;
  static bool attr = false;
  if (!attr) {
    SL_HIP_CHECK(hipFuncSetAttribute((const void*)k_gram_la<true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)gram_la_lds()));
    attr = true;
  }
  unsigned* counter = (unsigned*)ws;
  double* part = (double*)((char*)ws + 256);
  const int ng = n < SL_GRAM_NG ? n : SL_GRAM_NG;
  k_gram_la<true><<<ng, NT, gram_la_lds(), st>>>(W, n, k, ldw, part, counter, Gy, r, nullptr, M, N, s, status,
                                                max_sweeps > 0 ? max_sweeps : 40);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

SL_API int sl_rsvd_make_v(const double* W, int n, int k, int ldw, const double* N, int r, float* V, const double* s64,
                          float* s32, void* stream) {
  const int64_t tot = (int64_t)n * r;
  k_make_v<<<(unsigned)((tot + 255) / 256), 256, 0, (hipStream_t)stream>>>(W, n, k, ldw, N, r, V, s64, s32);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

SL_API int sl_rsvd_fjlt_zt(uint64_t seed, uint64_t baseD, uint64_t baseS, double scale, int k, int n, void* Zt,
                           void* stream) {
  const int64_t tot = (int64_t)n * k;
  k_fjlt_zt<<<(unsigned)((tot + 255) / 256), 256, 0, (hipStream_t)stream>>>(seed, baseD, baseS, scale, k, n,
                                                                            (bf16_t*)Zt);
  SL_LAUNCH_CHECK();
  return SL_OK;
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
  int* iscr = (int*)(red + 16);
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
  static bool attr = false;
  if (!attr) {
    SL_HIP_CHECK(hipFuncSetAttribute((const void*)k_sym_eig_jacobi2, hipFuncAttributeMaxDynamicSharedMemorySize,
                                     (int)gram_la_lds()));
    attr = true;
  }
  k_sym_eig_jacobi2<<<1, NT, gram_la_lds(), (hipStream_t)stream>>>(C, k, w, V, status, max_sweeps > 0 ? max_sweeps : 40);
  SL_LAUNCH_CHECK();
  return SL_OK;
}
