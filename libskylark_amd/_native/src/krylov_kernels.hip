// Fused vector kernels for the Krylov solvers (LSQR / CG / Chebyshev) on
// tall-skinny blocks: all k right-hand sides advance together and every
// per-column scalar stays in device memory.
//
// Reference loops: algorithms/Krylov/LSQR.hpp:113-248 (steps 1-12 per
// iteration, each an Elemental Axpy / Scale / ColumnNrm2 over the block),
// base/inner.hpp:22-170 (ColumnNrm2 / ColumnDot with their all-reduces).
//
//   sl_colred       : per-column sum of x^2 (mode 0) or x*y (mode 1), f64
//                     accumulation, two launches (block partials, one-block
//                     finish) -- the column norms / dots of K9;
//   sl_axpby_colred : Y = a .* X + b .* Y (per-column device scalars) and the
//                     new Y's column sums of squares in the same pass;
//   sl_lsqr_step    : LSQR steps 4-12 in two launches: the Givens rotation
//                     (recomputed per lane from the device scalars), the X / W
//                     updates and |W| in one streaming pass, then one block
//                     that advances every scalar recurrence (norm / condition /
//                     stagnation / |x| estimates) and writes the stop flags.
//
// Layout of a tall-skinny block: m x k row-major with leading dimension ld.
// Thread (tx, ty) of a 256-thread workgroup owns column tx (KP = k rounded up
// to a power of two <= 64 threads per row) and rows ty, ty + 256 / KP, ...:
// consecutive lanes read consecutive columns of a row (coalesced).
#include "sl_common.hpp"
#include <math.h>

namespace {

constexpr int NT = 256;
constexpr int MAXPART = 1024;   // partial blocks per reduction

template <typename T> __device__ __forceinline__ double ld_d(const T* p) { return (double)Cvt<T>::to_d(*p); }

int kp_of(int k) {
  int kp = 1;
  while (kp < k) kp <<= 1;
  return kp;
}

unsigned part_blocks(int64_t m, int kp) {
  const int64_t rows_per_block = (NT / kp) * 8;   // ~8 rows per thread per block
  int64_t g = (m + rows_per_block - 1) / rows_per_block;
  if (g < 1) g = 1;
  if (g > MAXPART) g = MAXPART;
  return (unsigned)g;
}

// reduce the NT per-thread values of column tx over ty -> part[blockIdx.x * k + tx]
template <int KP>
__device__ __forceinline__ void block_col_reduce(double v, double* sh, double* part, int k) {
  const int tid = threadIdx.x, tx = tid % KP;
  sh[tid] = v;
  __syncthreads();
  for (int s = NT / 2; s >= KP; s >>= 1) {
    if (tid < s) sh[tid] += sh[tid + s];
    __syncthreads();
  }
  if (tid < KP && tx < k) part[(int64_t)blockIdx.x * k + tx] = sh[tid];
}

template <typename T, int KP, int MODE>
__global__ void __launch_bounds__(NT) k_colred(const T* __restrict__ X, int64_t ldx, const T* __restrict__ Yv,
                                               int64_t ldy, int64_t m, int k, double* __restrict__ part) {
  __shared__ double sh[NT];
  const int tx = threadIdx.x % KP, ty = threadIdx.x / KP;
  constexpr int RS = NT / KP;
  double acc = 0.0;
  if (tx < k) {
    for (int64_t r = (int64_t)blockIdx.x * RS + ty; r < m; r += (int64_t)gridDim.x * RS) {
      const double x = ld_d(X + r * ldx + tx);
      acc += MODE == 0 ? x * x : x * ld_d(Yv + r * ldy + tx);
    }
  }
  block_col_reduce<KP>(acc, sh, part, k);
}

// out[c] = sum_b part[b][c] (f64), optionally its square root; one block
__global__ void __launch_bounds__(NT) k_colred_finish(const double* __restrict__ part, int nb, int k,
                                                      double* __restrict__ out, int do_sqrt) {
  __shared__ double sh[NT];
  for (int c = 0; c < k; ++c) {
    double s = 0.0;
    for (int b = threadIdx.x; b < nb; b += NT) s += part[(int64_t)b * k + c];
    sh[threadIdx.x] = s;
    __syncthreads();
    for (int w = NT / 2; w > 0; w >>= 1) {
      if (threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
      __syncthreads();
    }
    if (threadIdx.x == 0) out[c] = do_sqrt ? sqrt(sh[0]) : sh[0];
    __syncthreads();
  }
}

// LSQR scalar-state rows (see the enum below): finish a column-norm reduction
// straight into the state.  mode 1: beta = |U| (and step 2's |A| estimate,
// which needs the previous alpha); mode 2: alpha = |V|.
__global__ void __launch_bounds__(NT) k_finish_state(const double* __restrict__ part, int nb, int k,
                                                     double* __restrict__ st, int mode);

// Y = (sa a .* X + sb b .* Y) ./ d  (a, b, d: device per-column f64 scalars;
// null a = 1, null b = 0, null d = 1; sa, sb = +-1), then (RED) the sums of
// squares of the new Y per column
template <typename T, int KP, bool RED>
__global__ void __launch_bounds__(NT) k_axpby_colred(const T* __restrict__ X, int64_t ldx, T* __restrict__ Yv,
                                                     int64_t ldy, int64_t m, int k, const double* __restrict__ a,
                                                     double sa, const double* __restrict__ b, double sb,
                                                     const double* __restrict__ d, double* __restrict__ part) {
  __shared__ double sh[NT];
  const int tx = threadIdx.x % KP, ty = threadIdx.x / KP;
  constexpr int RS = NT / KP;
  double acc = 0.0;
  if (tx < k) {
    const double dv = d ? d[tx] : 1.0;
    const double inv = dv != 0.0 ? 1.0 / dv : 0.0;
    const double av = sa * (a ? a[tx] : 1.0) * inv, bv = b ? sb * b[tx] * inv : 0.0;
    for (int64_t r = (int64_t)blockIdx.x * RS + ty; r < m; r += (int64_t)gridDim.x * RS) {
      T* y = Yv + r * ldy + tx;
      const double v = av * ld_d(X + r * ldx + tx) + (b ? bv * ld_d(y) : 0.0);
      const T vt = Cvt<T>::from_d(v);
      *y = vt;
      if (RED) {
        const double vr = Cvt<T>::to_d(vt);
        acc += vr * vr;
      }
    }
  }
  if (RED) block_col_reduce<KP>(acc, sh, part, k);
}

// Y .*= s (per column, device scalars; s = 1 / nrm when inv)
template <typename T, int KP>
__global__ void __launch_bounds__(NT) k_colscale(T* __restrict__ Yv, int64_t ldy, int64_t m, int k,
                                                 const double* __restrict__ s, int inv) {
  const int tx = threadIdx.x % KP, ty = threadIdx.x / KP;
  constexpr int RS = NT / KP;
  if (tx >= k) return;
  double sv = s[tx];
  if (inv) sv = sv > 0.0 ? 1.0 / sv : 0.0;
  for (int64_t r = (int64_t)blockIdx.x * RS + ty; r < m; r += (int64_t)gridDim.x * RS) {
    T* y = Yv + r * ldy + tx;
    *y = Cvt<T>::from_d(sv * ld_d(y));
  }
}

// ---------------------------------------------------------------- LSQR
// Scalar state (f64, each row k long), indices into st[NS][k]:
enum { S_ALPHA, S_BETA, S_RHOBAR, S_PHIBAR, S_NRMA, S_SQD, S_CNDA, S_NRMX, S_SQX, S_CS2, S_SN2, S_ZZ,
       S_NRMAR0, S_STAG, S_RHO, S_PHI, S_THETA, S_NRMAR, S_NS };

// Givens rotation of step 4, per column, from the state before the step
struct Givens {
  double rho, cs, sn, theta, rhobar, phi, phibar;
};
__device__ __forceinline__ Givens givens(const double* st, int k, int c) {
  Givens g;
  const double rhobar = st[S_RHOBAR * k + c], beta = st[S_BETA * k + c], alpha = st[S_ALPHA * k + c];
  const double phibar = st[S_PHIBAR * k + c];
  g.rho = sqrt(rhobar * rhobar + beta * beta);
  g.cs = rhobar / g.rho;
  g.sn = beta / g.rho;
  g.theta = g.sn * alpha;
  g.rhobar = -g.cs * alpha;
  g.phi = g.cs * phibar;
  g.phibar = g.sn * phibar;
  return g;
}

// step 5: X += (phi / rho) W ; W = Z - (theta / rho) W ; partial |W|^2
template <typename T, int KP>
__global__ void __launch_bounds__(NT) k_lsqr_xw(T* __restrict__ X, int64_t ldx, T* __restrict__ W, int64_t ldw,
                                                const T* __restrict__ Z, int64_t ldz, int64_t n, int k,
                                                const double* __restrict__ st, double* __restrict__ part) {
  __shared__ double sh[NT];
  const int tx = threadIdx.x % KP, ty = threadIdx.x / KP;
  constexpr int RS = NT / KP;
  double acc = 0.0;
  if (tx < k) {
    const Givens g = givens(st, k, tx);
    const double fx = g.phi / g.rho, fw = g.theta / g.rho;
    for (int64_t r = (int64_t)blockIdx.x * RS + ty; r < n; r += (int64_t)gridDim.x * RS) {
      T* x = X + r * ldx + tx;
      T* w = W + r * ldw + tx;
      const double wv = ld_d(w);
      *x = Cvt<T>::from_d(ld_d(x) + fx * wv);
      const T wn = Cvt<T>::from_d(ld_d(Z + r * ldz + tx) - fw * wv);
      *w = wn;
      const double wr = Cvt<T>::to_d(wn);
      acc += wr * wr;
    }
  }
  block_col_reduce<KP>(acc, sh, part, k);
}

// steps 4, 6-12 on the scalars (one block, thread c = column c); flags[c] bits:
// 1 S1 (|A^T r| small), 2 S2, 4 S3 (ill-conditioned), 8 stagnation
__global__ void __launch_bounds__(NT) k_lsqr_scalars(const double* __restrict__ part, int nb, int k,
                                                     double* __restrict__ st, int* __restrict__ flags,
                                                     double tol, double eps, int max_stag) {
  __shared__ double nw2[64];
  // |W|^2 per column from the partials (columns k <= 64)
  for (int c = 0; c < k; ++c) {
    __shared__ double sh[NT];
    double s = 0.0;
    for (int b = threadIdx.x; b < nb; b += NT) s += part[(int64_t)b * k + c];
    sh[threadIdx.x] = s;
    __syncthreads();
    for (int w = NT / 2; w > 0; w >>= 1) {
      if (threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
      __syncthreads();
    }
    if (threadIdx.x == 0) nw2[c] = sh[0];
    __syncthreads();
  }
  const int c = threadIdx.x;
  if (c >= k) return;
  const Givens g = givens(st, k, c);
  const double alpha = st[S_ALPHA * k + c];
  const double nrm_w = sqrt(nw2[c]);
  // 6-7. residual estimates
  const double nrm_r = g.phibar;
  const double nrm_ar = fabs(g.phibar * alpha * g.cs);
  const double nrm_a = st[S_NRMA * k + c];
  int f = 0;
  if (nrm_ar < tol * st[S_NRMAR0 * k + c]) f |= 1;
  if (nrm_ar < eps * nrm_a * nrm_r) f |= 2;
  // 9. condition estimate
  const double sqd = st[S_SQD * k + c] + (nrm_w * nrm_w) / (g.rho * g.rho);
  const double cnd = nrm_a * sqrt(sqd);
  if (cnd > 1.0 / eps) f |= 4;
  // 11. stagnation
  const double nrm_x = st[S_NRMX * k + c];
  double stag = st[S_STAG * k + c];
  stag = (fabs(g.phi / g.rho) * nrm_w < eps * nrm_x) ? stag + 1.0 : 0.0;
  if (stag >= max_stag) f |= 8;
  // 12. |x| estimate
  const double delta = st[S_SN2 * k + c] * g.rho;
  const double gambar = -st[S_CS2 * k + c] * g.rho;
  const double rhs = g.phi - delta * st[S_ZZ * k + c];
  const double zbar = rhs / gambar;
  const double sqx = st[S_SQX * k + c];
  st[S_NRMX * k + c] = sqrt(sqx + zbar * zbar);
  const double gamma = sqrt(gambar * gambar + g.theta * g.theta);
  st[S_CS2 * k + c] = gambar / gamma;
  st[S_SN2 * k + c] = g.theta / gamma;
  const double zz = rhs / gamma;
  st[S_ZZ * k + c] = zz;
  st[S_SQX * k + c] = sqx + zz * zz;
  st[S_SQD * k + c] = sqd;
  st[S_CNDA * k + c] = cnd;
  st[S_STAG * k + c] = stag;
  st[S_RHOBAR * k + c] = g.rhobar;
  st[S_PHIBAR * k + c] = g.phibar;
  st[S_RHO * k + c] = g.rho;
  st[S_PHI * k + c] = g.phi;
  st[S_THETA * k + c] = g.theta;
  st[S_NRMAR * k + c] = nrm_ar;
  flags[c] = f;
}

__global__ void __launch_bounds__(NT) k_finish_state(const double* __restrict__ part, int nb, int k,
                                                     double* __restrict__ st, int mode) {
  __shared__ double sh[NT];
  for (int c = 0; c < k; ++c) {
    double s = 0.0;
    for (int b = threadIdx.x; b < nb; b += NT) s += part[(int64_t)b * k + c];
    sh[threadIdx.x] = s;
    __syncthreads();
    for (int w = NT / 2; w > 0; w >>= 1) {
      if (threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      const double nrm = sqrt(sh[0]);
      if (mode == 1) {
        const double na = st[S_NRMA * k + c], al = st[S_ALPHA * k + c];
        st[S_NRMA * k + c] = sqrt(na * na + al * al + sh[0]);
        st[S_BETA * k + c] = nrm;
      } else {
        st[S_ALPHA * k + c] = nrm;
      }
    }
    __syncthreads();
  }
}

// Y = M X for a row-major M (nr x nc) and a thin X (nc x K, K <= 8): one wave
// per output row, lanes stride the row with 16-B loads, X rows from L2 (the
// preconditioner GEMVs of LSQR / Chebyshev: hipBLASLt ran 1000 x 1000 at
// ~85 GB/s here).
template <typename T, int K, int VEC>
__global__ void __launch_bounds__(NT) k_rows_gemm(const T* __restrict__ M, int64_t ldm, int64_t nr, int64_t nc,
                                                  const T* __restrict__ X, int64_t ldx, T* __restrict__ Yo,
                                                  int64_t ldy) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * (NT / 64) + (threadIdx.x >> 6);
  if (r >= nr) return;
  const T* row = M + r * ldm;
  double acc[K];
#pragma unroll
  for (int j = 0; j < K; ++j) acc[j] = 0.0;
  const bool vec = (ldm % VEC) == 0 && ((uintptr_t)M % (VEC * sizeof(T))) == 0;
  const int64_t ncv = vec ? (nc / VEC) * VEC : 0;
  for (int64_t c = (int64_t)lane * VEC; c < ncv; c += 64 * VEC) {
    T mv[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) mv[v] = row[c + v];
#pragma unroll
    for (int v = 0; v < VEC; ++v)
#pragma unroll
      for (int j = 0; j < K; ++j) acc[j] += (double)mv[v] * (double)X[(c + v) * ldx + j];
  }
  for (int64_t c = ncv + lane; c < nc; c += 64)
#pragma unroll
    for (int j = 0; j < K; ++j) acc[j] += (double)row[c] * (double)X[c * ldx + j];
#pragma unroll
  for (int j = 0; j < K; ++j) {
    double v = acc[j];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
    acc[j] = v;
  }
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < K; ++j) Yo[r * ldy + j] = (T)acc[j];
  }
}


// ---------------------------------------------------------------- CG / FCG
// Device-resident (flexible) CG (reference algorithms/Krylov/CG.hpp:24-163,
// FlexibleCG.hpp:23-153): per-column scalars in st[C_NS][k], every column
// reduction finished by the LAST block of its own pass (agent-scope release,
// ticket counter, acquire), so an unpreconditioned CG iteration is 3 launches
// of its own plus the operator product:
//   k_cg_p   P = Z + beta P (CG) / Z - beta P (FCG)
//   k_cg_dot P . Q -> alpha = rho / pq   |  R . Z -> rho, beta  |  FCG dots
//   k_cg_xr  X += alpha P, R -= alpha Q, |R|^2 -> rho, beta (unpreconditioned),
//            convergence flags |R| < tol |B|
enum { C_RHO, C_RHO0, C_ALPHA, C_BETA, C_PQ, C_RR, C_NRMB, C_NS };

// After each block wrote part[b * k + c] (threads ty == 0): the last block to
// arrive reduces them; returns true there, with the column total in `tot` on
// threads tid < KP.  The counter is left at zero for the next launch.
template <int KP>
__device__ __forceinline__ bool last_block_total(const double* part, int k, unsigned* counter, double* sh,
                                                 double& tot) {
  __shared__ int last_sh;
  __threadfence();
  __syncthreads();
  if (threadIdx.x == 0) last_sh = atomicAdd(counter, 1u) == gridDim.x - 1;
  __syncthreads();
  if (!last_sh) return false;
  __threadfence();
  const int tx = threadIdx.x % KP, ty = threadIdx.x / KP;
  constexpr int RS = NT / KP;
  double v = 0.0;
  if (tx < k)
    for (int b = ty; b < (int)gridDim.x; b += RS) v += __hip_atomic_load(part + (int64_t)b * k + tx, __ATOMIC_RELAXED,
                                                                         __HIP_MEMORY_SCOPE_AGENT);
  sh[threadIdx.x] = v;
  __syncthreads();
  for (int st = NT / 2; st >= KP; st >>= 1) {
    if ((int)threadIdx.x < st) sh[threadIdx.x] += sh[threadIdx.x + st];
    __syncthreads();
  }
  tot = sh[threadIdx.x % KP];
  if (threadIdx.x == 0) *counter = 0u;
  return true;
}

// per-column dot(s) with a last-block epilogue on the CG state:
//   MODE 0 (CG)        alpha = rho / (X . Y)
//   MODE 1 (CG, M)     rho0 = rho, rho = X . Y, beta = rho / rho0 (0 first)
//   MODE 2 (FCG)       beta = (X . Y) / pq
//   MODE 3 (FCG)       pq = X . Y, alpha = (X . Y2) / pq
template <typename T, int KP, int MODE>
__global__ void __launch_bounds__(NT) k_cg_dot(const T* __restrict__ X, int64_t ldx, const T* __restrict__ Yv,
                                              int64_t ldy, const T* __restrict__ Y2, int64_t ldy2, int64_t m, int k,
                                              double* __restrict__ part, double* __restrict__ part2,
                                              unsigned* __restrict__ counter, double* __restrict__ st) {
  __shared__ double sh[NT];
  const int tx = threadIdx.x % KP, ty = threadIdx.x / KP;
  constexpr int RS = NT / KP;
  double a1 = 0.0, a2 = 0.0;
  if (tx < k) {
    for (int64_t r = (int64_t)blockIdx.x * RS + ty; r < m; r += (int64_t)gridDim.x * RS) {
      const double x = ld_d(X + r * ldx + tx);
      a1 += x * ld_d(Yv + r * ldy + tx);
      if (MODE == 3) a2 += x * ld_d(Y2 + r * ldy2 + tx);
    }
  }
  block_col_reduce<KP>(a1, sh, part, k);
  if (MODE == 3) {
    __syncthreads();
    block_col_reduce<KP>(a2, sh, part2, k);
  }
  double t1, t2 = 0.0;
  if (!last_block_total<KP>(part, k, counter, sh, t1)) return;
  if (MODE == 3) {
    // second total: the ticket is spent, reduce part2 directly
    const int ty2 = threadIdx.x / KP;
    double v = 0.0;
    if (tx < k)
      for (int b = ty2; b < (int)gridDim.x; b += RS)
        v += __hip_atomic_load(part2 + (int64_t)b * k + tx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    sh[threadIdx.x] = v;
    __syncthreads();
    for (int s2 = NT / 2; s2 >= KP; s2 >>= 1) {
      if ((int)threadIdx.x < s2) sh[threadIdx.x] += sh[threadIdx.x + s2];
      __syncthreads();
    }
    t2 = sh[threadIdx.x % KP];
  }
  const int c = threadIdx.x;
  if (c >= k) return;
  if (MODE == 0) {
    st[C_ALPHA * k + c] = t1 != 0.0 ? st[C_RHO * k + c] / t1 : 0.0;
  } else if (MODE == 1) {
    const double rho0 = st[C_RHO * k + c];
    st[C_RHO0 * k + c] = rho0;
    st[C_RHO * k + c] = t1;
    st[C_BETA * k + c] = rho0 != 0.0 ? t1 / rho0 : 0.0;
  } else if (MODE == 2) {
    const double pq = st[C_PQ * k + c];
    st[C_BETA * k + c] = pq != 0.0 ? t1 / pq : 0.0;
  } else {
    st[C_PQ * k + c] = t1;
    st[C_ALPHA * k + c] = t1 != 0.0 ? t2 / t1 : 0.0;
  }
}

// P = Z + sb * beta .* P
template <typename T, int KP>
__global__ void __launch_bounds__(NT) k_cg_p(const T* __restrict__ Z, int64_t ldz, T* __restrict__ P, int64_t ldp,
                                            int64_t m, int k, const double* __restrict__ st, double sb) {
  const int tx = threadIdx.x % KP, ty = threadIdx.x / KP;
  constexpr int RS = NT / KP;
  if (tx >= k) return;
  const double b = sb * st[C_BETA * k + tx];
  for (int64_t r = (int64_t)blockIdx.x * RS + ty; r < m; r += (int64_t)gridDim.x * RS) {
    T* p = P + r * ldp + tx;
    *p = Cvt<T>::from_d(ld_d(Z + r * ldz + tx) + b * ld_d(p));
  }
}

// X += alpha P, R -= alpha Q, |R|^2 -> rr, flags; IDP: rho0 = rho, rho = rr, beta
template <typename T, int KP, bool IDP>
__global__ void __launch_bounds__(NT) k_cg_xr(T* __restrict__ X, int64_t ldx, const T* __restrict__ P, int64_t ldp,
                                             T* __restrict__ R, int64_t ldr, const T* __restrict__ Q, int64_t ldq,
                                             int64_t m, int k, double* __restrict__ part,
                                             unsigned* __restrict__ counter, double* __restrict__ st,
                                             int* __restrict__ flags, double tol) {
  __shared__ double sh[NT];
  const int tx = threadIdx.x % KP, ty = threadIdx.x / KP;
  constexpr int RS = NT / KP;
  double acc = 0.0;
  if (tx < k) {
    const double al = st[C_ALPHA * k + tx];
    for (int64_t r = (int64_t)blockIdx.x * RS + ty; r < m; r += (int64_t)gridDim.x * RS) {
      T* x = X + r * ldx + tx;
      *x = Cvt<T>::from_d(ld_d(x) + al * ld_d(P + r * ldp + tx));
      T* rr = R + r * ldr + tx;
      const T nv = Cvt<T>::from_d(ld_d(rr) - al * ld_d(Q + r * ldq + tx));
      *rr = nv;
      const double vd = Cvt<T>::to_d(nv);
      acc += vd * vd;
    }
  }
  block_col_reduce<KP>(acc, sh, part, k);
  double tot;
  if (!last_block_total<KP>(part, k, counter, sh, tot)) return;
  const int c = threadIdx.x;
  if (c >= k) return;
  st[C_RR * k + c] = tot;
  flags[c] = sqrt(tot) < tol * st[C_NRMB * k + c] ? 1 : 0;
  if (IDP) {
    const double rho0 = st[C_RHO * k + c];
    st[C_RHO0 * k + c] = rho0;
    st[C_RHO * k + c] = tot;
    st[C_BETA * k + c] = rho0 != 0.0 ? tot / rho0 : 0.0;
  }
}

}  // namespace

// Y (nr x k) = M (nr x nc, row-major, ld ldm) X (nc x k, ld ldx), k <= 8, f32/f64
SL_API int sl_rows_gemm(const void* M, int64_t ldm, int64_t nr, int64_t nc, const void* X, int64_t ldx, int k,
                        void* Y, int64_t ldy, int dtype, void* stream) {
  if (nr <= 0) return SL_OK;
  if (k < 1 || k > 8 || (dtype != SL_F32 && dtype != SL_F64)) {
    sl_set_last_error("rows_gemm: f32/f64, 1 <= k <= 8");
    return SL_ERR_UNSUPPORTED;
  }
  hipStream_t s = (hipStream_t)stream;
  const unsigned g = (unsigned)((nr + NT / 64 - 1) / (NT / 64));
#define SL_RG(TT, KK) k_rows_gemm<TT, KK, 16 / sizeof(TT)><<<g, NT, 0, s>>>((const TT*)M, ldm, nr, nc, (const TT*)X, ldx, (TT*)Y, ldy)
#define SL_RG_K(TT) switch (k) { case 1: SL_RG(TT, 1); break; case 2: SL_RG(TT, 2); break; \
    case 3: SL_RG(TT, 3); break; case 4: SL_RG(TT, 4); break; case 5: SL_RG(TT, 5); break; \
    case 6: SL_RG(TT, 6); break; case 7: SL_RG(TT, 7); break; default: SL_RG(TT, 8); }
  if (dtype == SL_F32) { SL_RG_K(float) } else { SL_RG_K(double) }
#undef SL_RG_K
#undef SL_RG
  SL_LAUNCH_CHECK();
  return SL_OK;
}

#define SL_KP_DISPATCH(KPV, ...)                                               \
  switch (KPV) {                                                               \
    case 1: { constexpr int KP = 1; __VA_ARGS__; break; }                      \
    case 2: { constexpr int KP = 2; __VA_ARGS__; break; }                      \
    case 4: { constexpr int KP = 4; __VA_ARGS__; break; }                      \
    case 8: { constexpr int KP = 8; __VA_ARGS__; break; }                      \
    case 16: { constexpr int KP = 16; __VA_ARGS__; break; }                    \
    case 32: { constexpr int KP = 32; __VA_ARGS__; break; }                    \
    default: { constexpr int KP = 64; __VA_ARGS__; break; }                    \
  }

// workspace: MAXPART * k doubles
SL_API int64_t sl_krylov_ws_bytes(int k) { return (int64_t)MAXPART * (k > 0 ? k : 1) * 8; }

// out[c] = sum_r X[r,c]^2 (mode 0) or X[r,c] * Y[r,c] (mode 1); sqrt if do_sqrt (mode 0)
SL_API int sl_colred(const void* X, int64_t ldx, const void* Y, int64_t ldy, int64_t m, int k, int dtype, int mode,
                     double* out, int do_sqrt, void* ws, void* stream) {
  if (k < 1 || k > 64) { sl_set_last_error("colred: 1 <= k <= 64"); return SL_ERR_UNSUPPORTED; }
  hipStream_t s = (hipStream_t)stream;
  const int kp = kp_of(k);
  const unsigned g = m > 0 ? part_blocks(m, kp) : 1;
  double* part = (double*)ws;
  if (m > 0) {
    SL_DISPATCH_FLOAT(dtype, T, {
      SL_KP_DISPATCH(kp, {
        if (mode == 0) k_colred<T, KP, 0><<<g, NT, 0, s>>>((const T*)X, ldx, nullptr, 0, m, k, part);
        else k_colred<T, KP, 1><<<g, NT, 0, s>>>((const T*)X, ldx, (const T*)Y, ldy, m, k, part);
      })
    });
  } else {
    SL_HIP_CHECK(hipMemsetAsync(part, 0, (size_t)k * 8, s));
  }
  k_colred_finish<<<1, NT, 0, s>>>(part, (int)g, k, out, do_sqrt);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// Y = (sa a .* X + sb b .* Y) ./ d, then per red_mode: 0 nothing, 1 out[c] =
// sum of squares of the new Y, 2 / 3 LSQR state st (beta + |A| estimate /
// alpha) set from |Y| (single-rank: the distributed caller uses mode 1, an
// all-reduce, then sl_lsqr_setstate)
SL_API int sl_axpby_red(const void* X, int64_t ldx, void* Y, int64_t ldy, int64_t m, int k, int dtype,
                        const double* a, double sa, const double* b, double sb, const double* d, int red_mode,
                        double* out, double* st, void* ws, void* stream) {
  if (k < 1 || k > 64) { sl_set_last_error("axpby_red: 1 <= k <= 64"); return SL_ERR_UNSUPPORTED; }
  hipStream_t s = (hipStream_t)stream;
  const int kp = kp_of(k);
  const unsigned g = m > 0 ? part_blocks(m, kp) : 1;
  double* part = (double*)ws;
  if (m > 0) {
    SL_DISPATCH_FLOAT(dtype, T, {
      SL_KP_DISPATCH(kp, {
        if (red_mode) k_axpby_colred<T, KP, true><<<g, NT, 0, s>>>((const T*)X, ldx, (T*)Y, ldy, m, k, a, sa, b, sb, d, part);
        else k_axpby_colred<T, KP, false><<<g, NT, 0, s>>>((const T*)X, ldx, (T*)Y, ldy, m, k, a, sa, b, sb, d, part);
      })
    });
  } else if (red_mode) {
    SL_HIP_CHECK(hipMemsetAsync(part, 0, (size_t)k * 8, s));
  }
  if (red_mode == 1) k_colred_finish<<<1, NT, 0, s>>>(part, (int)g, k, out, 0);
  else if (red_mode >= 2) k_finish_state<<<1, NT, 0, s>>>(part, (int)g, k, st, red_mode - 1);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// LSQR state from all-reduced sums of squares (mode 1 beta, 2 alpha)
SL_API int sl_lsqr_setstate(const double* sums, int k, double* st, int mode, void* stream) {
  k_finish_state<<<1, NT, 0, (hipStream_t)stream>>>(sums, 1, k, st, mode);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// Y[:, c] *= s[c]  (or / s[c] when inv; 0 where s[c] == 0)
SL_API int sl_colscale(void* Y, int64_t ldy, int64_t m, int k, int dtype, const double* sc, int inv, void* stream) {
  if (m <= 0) return SL_OK;
  if (k < 1 || k > 64) { sl_set_last_error("colscale: 1 <= k <= 64"); return SL_ERR_UNSUPPORTED; }
  hipStream_t s = (hipStream_t)stream;
  const int kp = kp_of(k);
  const unsigned g = part_blocks(m, kp);
  SL_DISPATCH_FLOAT(dtype, T, { SL_KP_DISPATCH(kp, k_colscale<T, KP><<<g, NT, 0, s>>>((T*)Y, ldy, m, k, sc, inv)) });
  SL_LAUNCH_CHECK();
  return SL_OK;
}

SL_API int sl_lsqr_nstate() { return S_NS; }

// LSQR steps 4-12 (Givens, X/W update, |W|, scalar recurrences, stop flags)
SL_API int sl_lsqr_step(void* X, int64_t ldx, void* W, int64_t ldw, const void* Z, int64_t ldz, int64_t n, int k,
                        int dtype, double* st, int* flags, double tol, double eps, int max_stag, void* ws,
                        void* stream) {
  if (k < 1 || k > 64) { sl_set_last_error("lsqr_step: 1 <= k <= 64"); return SL_ERR_UNSUPPORTED; }
  hipStream_t s = (hipStream_t)stream;
  const int kp = kp_of(k);
  const unsigned g = n > 0 ? part_blocks(n, kp) : 1;
  double* part = (double*)ws;
  if (n > 0) {
    SL_DISPATCH_FLOAT(dtype, T, {
      SL_KP_DISPATCH(kp, k_lsqr_xw<T, KP><<<g, NT, 0, s>>>((T*)X, ldx, (T*)W, ldw, (const T*)Z, ldz, n, k, st, part))
    });
  } else {
    SL_HIP_CHECK(hipMemsetAsync(part, 0, (size_t)k * 8, s));
  }
  k_lsqr_scalars<<<1, NT, 0, s>>>(part, (int)g, k, st, flags, tol, eps, max_stag);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// ---------------------------------------------------------------- CG / FCG
SL_API int sl_cg_nstate() { return C_NS; }

// grid of the CG passes: at most one block per CU-ish (the last block reduces
// every block's partial, so fewer, fatter blocks keep that tail short)
static unsigned cg_blocks(int64_t m, int kp) {
  unsigned g = part_blocks(m, kp);
  return g > 256 ? 256 : g;
}

// dots with the CG state epilogue (mode: 0 alpha = rho / X.Y; 1 rho, beta from
// X.Y; 2 FCG beta = X.Y / pq; 3 FCG pq = X.Y, alpha = X.Y2 / pq).  ws: 2 x
// sl_krylov_ws_bytes; counter: a zeroed unsigned the kernel leaves zeroed.
SL_API int sl_cg_dot(const void* X, int64_t ldx, const void* Y, int64_t ldy, const void* Y2, int64_t ldy2, int64_t m,
                     int k, int dtype, int mode, double* st, void* ws, unsigned* counter, void* stream) {
  if (k < 1 || k > 64 || m < 1 || mode < 0 || mode > 3) { sl_set_last_error("cg_dot: 1 <= k <= 64, m >= 1"); return SL_ERR_UNSUPPORTED; }
  hipStream_t s = (hipStream_t)stream;
  const int kp = kp_of(k);
  const unsigned g = cg_blocks(m, kp);
  double* part = (double*)ws;
  double* part2 = part + (int64_t)MAXPART * k;
  SL_DISPATCH_FLOAT(dtype, T, {
    SL_KP_DISPATCH(kp, {
      const T* x = (const T*)X; const T* y = (const T*)Y; const T* y2 = (const T*)Y2;
      switch (mode) {
        case 0: k_cg_dot<T, KP, 0><<<g, NT, 0, s>>>(x, ldx, y, ldy, y2, ldy2, m, k, part, part2, counter, st); break;
        case 1: k_cg_dot<T, KP, 1><<<g, NT, 0, s>>>(x, ldx, y, ldy, y2, ldy2, m, k, part, part2, counter, st); break;
        case 2: k_cg_dot<T, KP, 2><<<g, NT, 0, s>>>(x, ldx, y, ldy, y2, ldy2, m, k, part, part2, counter, st); break;
        default: k_cg_dot<T, KP, 3><<<g, NT, 0, s>>>(x, ldx, y, ldy, y2, ldy2, m, k, part, part2, counter, st); break;
      }
    })
  });
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// P = Z + sb * beta .* P
SL_API int sl_cg_p(const void* Z, int64_t ldz, void* P, int64_t ldp, int64_t m, int k, int dtype, const double* st,
                   double sb, void* stream) {
  if (m <= 0) return SL_OK;
  if (k < 1 || k > 64) { sl_set_last_error("cg_p: 1 <= k <= 64"); return SL_ERR_UNSUPPORTED; }
  hipStream_t s = (hipStream_t)stream;
  const int kp = kp_of(k);
  const unsigned g = part_blocks(m, kp);
  SL_DISPATCH_FLOAT(dtype, T, {
    SL_KP_DISPATCH(kp, k_cg_p<T, KP><<<g, NT, 0, s>>>((const T*)Z, ldz, (T*)P, ldp, m, k, st, sb))
  });
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// X += alpha P, R -= alpha Q, |R|^2, flags (|R| < tol |B|); idp: also rho, beta
SL_API int sl_cg_xr(void* X, int64_t ldx, const void* P, int64_t ldp, void* R, int64_t ldr, const void* Q, int64_t ldq,
                    int64_t m, int k, int dtype, int idp, double* st, int* flags, double tol, void* ws,
                    unsigned* counter, void* stream) {
  if (k < 1 || k > 64 || m < 1) { sl_set_last_error("cg_xr: 1 <= k <= 64, m >= 1"); return SL_ERR_UNSUPPORTED; }
  hipStream_t s = (hipStream_t)stream;
  const int kp = kp_of(k);
  const unsigned g = cg_blocks(m, kp);
  double* part = (double*)ws;
  SL_DISPATCH_FLOAT(dtype, T, {
    SL_KP_DISPATCH(kp, {
      if (idp) k_cg_xr<T, KP, true><<<g, NT, 0, s>>>((T*)X, ldx, (const T*)P, ldp, (T*)R, ldr, (const T*)Q, ldq, m, k, part, counter, st, flags, tol);
      else k_cg_xr<T, KP, false><<<g, NT, 0, s>>>((T*)X, ldx, (const T*)P, ldp, (T*)R, ldr, (const T*)Q, ldq, m, k, part, counter, st, flags, tol);
    })
  });
  SL_LAUNCH_CHECK();
  return SL_OK;
}
