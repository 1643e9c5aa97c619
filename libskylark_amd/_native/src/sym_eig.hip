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
#include "sl_wave_la.hpp"

namespace {

constexpr int KMAX = 64;
constexpr int NT = 256;

__global__ void __launch_bounds__(NT)
k_sym_eig_jacobi(const double* __restrict__ Cin, int k, int ldc, int r, double* __restrict__ out,
                 int want_sqrt, int max_sweeps, int* __restrict__ sweeps_out, const int* __restrict__ flag,
                 int* __restrict__ noconv = nullptr) {
  __shared__ double AB[2][KMAX][KMAX + 1];   // ping-pong copies of A
  __shared__ double V[KMAX][KMAX + 1];
  __shared__ double cs[KMAX / 2], sn[KMAX / 2];
  __shared__ int pp[KMAX / 2], qq[KMAX / 2];
  __shared__ int rotated;
  const int tid = threadIdx.x;
  if (flag && *flag == 0) return;   // conditional re-solve: only when the caller's solver flagged the matrix
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
  // conditional re-solve: report a Jacobi run that used every sweep and was
  // still rotating (the caller maps it to its "no convergence" status bit)
  if (tid == 0 && noconv && sweep >= max_sweeps) *noconv = 1;
}

// ---------------------------------------------------------------------------
// Tridiagonal path (k <= 64, r <= 64): the k x k matrix's top-r eigenpairs in
// one launch of one workgroup (sl_wave_la.hpp: Householder tridiagonalisation
// on one wave with the matrix in registers, multisection on a division-free
// Sturm count over all waves, twisted-factorisation eigenvectors, MGS inside
// close clusters, a DPP back-transform).  Status bit 1: the result must be
// recomputed by a robust solver (numerically repeated wanted eigenvalues, a
// vector failing its residual check, non-finite data or -- with want_sqrt --
// a vanishing r-th eigenvalue).  Output as k_sym_eig_jacobi:
// out[i * r + c] = V[i][c] descending, then sqrt(max(lambda, 0)) (or lambda)
// in out[k * r + c].
// tridiagonalisation: 1 = four waves (wg_tridiag), 0 = one wave, -1 = by size
// (default: four waves only at k > 48, where they win -- 128 vs 146 us at
// k = 64; one wave is 1-4 us faster below, profiles/r6/tridiag_four_wave_ab.jsonl)
int g_tri_host = -1;
template <int K>
__global__ void __launch_bounds__(512) k_sym_eig_wave_impl(const double* __restrict__ C, int k, int ldc, int r,
                                                           double* __restrict__ out, int want_sqrt,
                                                           int* __restrict__ status, int g_tri_variant) {
  __shared__ double refl[K * (K + 1)];
  __shared__ double sc[3 * 64 * (K + 1)];
  __shared__ __attribute__((aligned(16))) double dd[K], ee[K], lam[K], vsh[128], wsh[256];
  __shared__ int bad, fb;
  const int tid = threadIdx.x;
  if (tid == 0) { bad = 0; fb = 0; }
  __syncthreads();
  if (g_tri_variant) {
    slw::wg_tridiag<K>(C, ldc, k, refl, K + 1, dd, ee, vsh, wsh, &bad);
  } else {
    if (tid < 64) slw::wave_tridiag<K>(C, ldc, k, refl, K + 1, dd, ee, vsh, wsh, &bad);
    __syncthreads();
  }
  const int nt = r < k ? r + 1 : k;
  slw::sym_top_eig<K, 512>(dd, ee, refl, K + 1, nt, r, lam, out, r, k, sc, &fb);
  if (tid < r) {
    const double l = lam[tid];
    out[k * r + tid] = want_sqrt ? sqrt(l > 0.0 ? l : 0.0) : l;
  }
  if (tid == 0) {
    const bool vanish = want_sqrt && !(lam[r - 1] > 1e-30 * fmax(lam[0], 1e-300));
    if ((bad || fb || vanish) && status) atomicOr(status, 1);
  }
}

}  // namespace

// Top-r eigenpairs by the tridiagonal path (k <= 64, r <= k); status bit 1 =
// the caller should redo this matrix with a robust solver (see the kernel).
SL_API int sl_sym_eig_tridiag(const double* C, int k, int ldc, int r, double* out, int want_sqrt, int* status,
                              void* stream) {
  if (k <= 0 || k > 64 || r <= 0 || r > k || ldc < k) return SL_ERR_DIMENSION;
  hipStream_t s = (hipStream_t)stream;
  const int tv = g_tri_host < 0 ? (k > 48) : g_tri_host;
  if (k <= 16) k_sym_eig_wave_impl<16><<<1, 512, 0, s>>>(C, k, ldc, r, out, want_sqrt, status, tv);
  else if (k <= 32) k_sym_eig_wave_impl<32><<<1, 512, 0, s>>>(C, k, ldc, r, out, want_sqrt, status, tv);
  else if (k <= 40) k_sym_eig_wave_impl<40><<<1, 512, 0, s>>>(C, k, ldc, r, out, want_sqrt, status, tv);
  else if (k <= 48) k_sym_eig_wave_impl<48><<<1, 512, 0, s>>>(C, k, ldc, r, out, want_sqrt, status, tv);
  else k_sym_eig_wave_impl<64><<<1, 512, 0, s>>>(C, k, ldc, r, out, want_sqrt, status, tv);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

SL_API void sl_sym_eig_set_tri_variant(int v) { g_tri_host = v; }

SL_API int sl_sym_eig_topr(const double* C, int k, int ldc, int r, double* out, int want_sqrt,
                           int max_sweeps, int* sweeps_out, void* stream) {
  if (k <= 0 || k > KMAX || r <= 0 || r > k || ldc < k) return SL_ERR_DIMENSION;
  k_sym_eig_jacobi<<<1, NT, 0, (hipStream_t)stream>>>(C, k, ldc, r, out, want_sqrt,
                                                       max_sweeps > 0 ? max_sweeps : 30, sweeps_out, nullptr);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// the same, run only when *flag (device) is non-zero: the robust re-solve of a
// matrix the tridiagonal path flagged, decided on the device (no host sync)
SL_API int sl_sym_eig_topr_if(const double* C, int k, int ldc, int r, double* out, int want_sqrt, int max_sweeps,
                              const int* flag, void* stream) {
  if (k <= 0 || k > KMAX || r <= 0 || r > k || ldc < k) return SL_ERR_DIMENSION;
  // flag[1]: set when the re-solve itself ran out of sweeps
  k_sym_eig_jacobi<<<1, NT, 0, (hipStream_t)stream>>>(C, k, ldc, r, out, want_sqrt,
                                                       max_sweeps > 0 ? max_sweeps : 30, nullptr, flag,
                                                       const_cast<int*>(flag) + 1);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

