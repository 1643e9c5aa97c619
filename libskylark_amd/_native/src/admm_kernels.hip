// BlockADMM per-iteration element-wise work on the k x n output block, fused
// (reference ml/BlockADMM.hpp:400-498, losses algorithms/regression/loss.hpp:26-446).
//
// Per iteration the solver runs, over the k x n_i matrices O, Obar, nu, del_o:
//   pre : Obar -= nu ; O = prox_loss(Obar, lambda, Y) ; dsum = del_o + (P + 1) nu
//   post: s = O - sum_j o_j ; del_o = s ; Obar = O - s / (P + 1) ; nu += O - Obar ;
//         loss = sum L(sum_j Z_j Wbar_j, Y)
// -- a dozen torch element-wise launches, each a full pass over k x n_i.
// Here: one thread per example (column) and one launch each; the block
// sums sum_j o_j and sum_j Z_j Wbar_j arrive as the n x kp outputs the
// one-pass block kernels accumulate (ata_kernels.hip), which post zeroes
// for the next iteration.  The loss partials are per-workgroup f64 sums.
// Losses: 0 squared, 1 LAD, 2 hinge (+-1 targets), 3 multinomial logistic
// (targets +-1 one-vs-rest coding, label = the +1 row; per-example Newton
// with backtracking, as algorithms/loss.py).
#include "sl_common.hpp"

namespace {

constexpr int NTA = 256;
constexpr int KMAXA = 16;

enum { L_SQUARED = 0, L_LAD = 1, L_HINGE = 2, L_LOGISTIC = 3 };

__device__ __forceinline__ float lse(const float* z, int k) {
  float mx = z[0];
  for (int c = 1; c < k; ++c) mx = fmaxf(mx, z[c]);
  float s = 0.f;
  for (int c = 0; c < k; ++c) s += __expf(z[c] - mx);
  return mx + __logf(s);
}

__device__ __forceinline__ int label_of(const float* t, int k) {
  int y = 0;
  for (int c = 1; c < k; ++c)
    if (t[c] > t[y]) y = c;
  return y;
}

// argmin_z lam (lse(z) - z_y) + |z - x|^2 / 2, Newton with backtracking
__device__ void logistic_prox(const float* x, int y, float lam, int k, float* z) {
  float p[KMAXA], g[KMAXA], st[KMAXA], zn[KMAXA];
  for (int c = 0; c < k; ++c) z[c] = x[c];
  auto obj = [&](const float* v) {
    float q = 0.f;
    for (int c = 0; c < k; ++c) q += 0.5f * (v[c] - x[c]) * (v[c] - x[c]);
    return lam * (lse(v, k) - v[y]) + q;
  };
  for (int it = 0; it < 30; ++it) {
    const float l = lse(z, k);
    float gmax = 0.f, spu = 0.f, spw = 0.f;
    for (int c = 0; c < k; ++c) {
      p[c] = __expf(z[c] - l);
      g[c] = lam * (p[c] - (c == y ? 1.f : 0.f)) + (z[c] - x[c]);
      gmax = fmaxf(gmax, fabsf(g[c]));
      const float dv = 1.f + lam * p[c];
      spu += p[c] * (g[c] / dv);
      spw += p[c] * (p[c] / dv);
    }
    if (gmax < 1e-10f) break;
    // Hessian I + lam (diag p - p p^T): Sherman-Morrison
    const float coef = lam * spu / (1.f - lam * spw);
    float gs = 0.f;
    for (int c = 0; c < k; ++c) {
      const float dv = 1.f + lam * p[c];
      st[c] = g[c] / dv + coef * (p[c] / dv);
      gs += g[c] * st[c];
    }
    const float f0 = obj(z);
    float t = 1.f;
    for (int bt = 0; bt < 20; ++bt) {
      for (int c = 0; c < k; ++c) zn[c] = z[c] - t * st[c];
      if (obj(zn) <= f0 - 1e-4f * t * gs) break;
      t *= 0.5f;
    }
    for (int c = 0; c < k; ++c) z[c] -= t * st[c];
  }
}

__global__ void __launch_bounds__(NTA)
k_admm_pre(int loss, int k, int64_t n, float* __restrict__ Obar, const float* __restrict__ nu,
           const float* __restrict__ del_o, const float* __restrict__ Yt, float lam, float P1,
           float* __restrict__ O, float* __restrict__ Dp) {
  const int64_t j = (int64_t)blockIdx.x * NTA + threadIdx.x;
  if (j >= n) return;
  float x[KMAXA], t[KMAXA], z[KMAXA];
  for (int c = 0; c < k; ++c) {
    const int64_t e = c * n + j;
    const float v = nu[e];
    x[c] = Obar[e] - v;
    Obar[e] = x[c];
    t[c] = Yt[e];
    Dp[e] = del_o[e] + P1 * v;
  }
  if (loss == L_LOGISTIC) {
    logistic_prox(x, label_of(t, k), lam, k, z);
  } else {
    for (int c = 0; c < k; ++c) {
      if (loss == L_SQUARED) {
        z[c] = (x[c] + lam * t[c]) / (1.f + lam);
      } else if (loss == L_LAD) {
        const float d = x[c] - t[c];
        z[c] = t[c] + copysignf(fmaxf(fabsf(d) - lam, 0.f), d) * (d != 0.f ? 1.f : 0.f);
      } else {   // hinge: prox of max(0, 1 - t z)
        const float tx = t[c] * x[c];
        z[c] = tx >= 1.f ? x[c] : (tx <= 1.f - lam ? x[c] + lam * t[c] : t[c]);
      }
    }
  }
  for (int c = 0; c < k; ++c) O[c * n + j] = z[c];
}

__global__ void __launch_bounds__(NTA)
k_admm_post(int loss, int k, int kp, int64_t n, const float* __restrict__ O, float* __restrict__ zo,
            float* __restrict__ zw, const float* __restrict__ Yt, float P1, float* __restrict__ Obar,
            float* __restrict__ nu, float* __restrict__ del_o, double* __restrict__ partial) {
  __shared__ double red[NTA / 64];
  const int64_t j = (int64_t)blockIdx.x * NTA + threadIdx.x;
  double lv = 0.0;
  if (j < n) {
    float w[KMAXA], t[KMAXA];
    for (int c = 0; c < k; ++c) {
      const int64_t e = c * n + j;
      const float o = O[e];
      const float s = o - zo[j * kp + c];
      del_o[e] = s;
      const float ob = o - s / P1;
      Obar[e] = ob;
      nu[e] += o - ob;
      w[c] = zw[j * kp + c];
      t[c] = Yt[e];
    }
    for (int c = 0; c < kp; ++c) {   // ready for the next iteration's accumulation
      zo[j * kp + c] = 0.f;
      zw[j * kp + c] = 0.f;
    }
    if (loss == L_LOGISTIC) {
      lv = (double)(lse(w, k) - w[label_of(t, k)]);
    } else {
      for (int c = 0; c < k; ++c) {
        const float d = w[c] - t[c];
        lv += loss == L_SQUARED ? 0.5 * (double)d * d
              : loss == L_LAD   ? (double)fabsf(d)
                                : (double)fmaxf(1.f - t[c] * w[c], 0.f);
      }
    }
  }
  for (int off = 32; off > 0; off >>= 1) lv += __shfl_down(lv, off);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = lv;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int i = 0; i < NTA / 64; ++i) s += red[i];
    partial[blockIdx.x] = s;
  }
}

}  // namespace

SL_API int64_t sl_admm_partials(int64_t n) { return (n + NTA - 1) / NTA; }

// pre: Obar -= nu; O = prox(Obar); Dp[0:k] = del_o + P1 nu   (k x n row-major, Dp rows stride n)
SL_API int sl_admm_pre(int loss, int k, int64_t n, float* Obar, const float* nu, const float* del_o, const float* Yt,
                       double lam, double P1, float* O, float* Dp, void* stream) {
  if (k < 1 || k > KMAXA || loss < 0 || loss > 3) {
    sl_set_last_error("admm_pre: 1 <= k <= 16, loss in 0..3");
    return SL_ERR_INVALID;
  }
  if (n <= 0) return SL_OK;
  k_admm_pre<<<(unsigned)((n + NTA - 1) / NTA), NTA, 0, (hipStream_t)stream>>>(loss, k, n, Obar, nu, del_o, Yt,
                                                                              (float)lam, (float)P1, O, Dp);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// post: s = O - zo^T; del_o = s; Obar = O - s / P1; nu += O - Obar; zo, zw (n x kp) zeroed;
// partial[b] = the loss of zw^T against Yt over workgroup b's examples
SL_API int sl_admm_post(int loss, int k, int kp, int64_t n, const float* O, float* zo, float* zw, const float* Yt,
                        double P1, float* Obar, float* nu, float* del_o, double* partial, void* stream) {
  if (k < 1 || k > KMAXA || kp < k || loss < 0 || loss > 3) {
    sl_set_last_error("admm_post: 1 <= k <= kp, k <= 16, loss in 0..3");
    return SL_ERR_INVALID;
  }
  if (n <= 0) return SL_OK;
  k_admm_post<<<(unsigned)((n + NTA - 1) / NTA), NTA, 0, (hipStream_t)stream>>>(loss, k, kp, n, O, zo, zw, Yt,
                                                                               (float)P1, Obar, nu, del_o, partial);
  SL_LAUNCH_CHECK();
  return SL_OK;
}
