// Stand-alone probe: phase timing (s_memtime) of single-wave k x k Cholesky +
// inverse variants, to find where the time goes.  Build:
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 chol_probe.hip -o chol_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); return 1; } } while (0)

__device__ __forceinline__ long long now() { return __builtin_amdgcn_s_memtime(); }

// variant A: row per lane in registers, LDS broadcast of the pivot column, bulk reads
template <int K>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1)))
chol_bulk(const double* G, int k, double* Rinv, long long* ts) {
  __shared__ double colv[64];
  const int i = threadIdx.x;
  long long t0 = now();
  double a[K];
#pragma unroll
  for (int c = 0; c < K; ++c) a[c] = (i < k && c < k) ? G[i * k + c] : (i == c ? 1.0 : 0.0);
  __builtin_amdgcn_s_waitcnt(0);
  long long t1 = now();
#pragma unroll
  for (int j = 0; j < K; ++j) {
    colv[i] = a[j];
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    const double d = colv[j];
    const double piv = __builtin_sqrt(d);
    const double inv = 1.0 / piv;
    const double lij = (i == j) ? piv : a[j] * inv;
    if (i >= j) a[j] = lij;
    colv[i] = lij;
    double cv[K];
#pragma unroll
    for (int c = j + 1; c < K; ++c) cv[c] = colv[c];
#pragma unroll
    for (int c = j + 1; c < K; ++c)
      if (i > j) a[c] -= lij * cv[c];
  }
  long long t2 = now();
  if (i < k)
    for (int c = 0; c < k; ++c) Rinv[i * k + c] = a[c < K ? c : 0];
  long long t3 = now();
  if (i == 0) { ts[0] = t1 - t0; ts[1] = t2 - t1; ts[2] = t3 - t2; }
}

// variant A2: bulk-lds with rsqrt + 2 Newton steps instead of IEEE sqrt and divide
__device__ __forceinline__ double rsqrt_nr(double d) {
  double y = __builtin_amdgcn_rsq(d);
  y = y * (1.5 - 0.5 * d * y * y);
  y = y * (1.5 - 0.5 * d * y * y);
  return y;
}
template <int K>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1)))
chol_bulk_rsq(const double* G, int k, double* Rinv, long long* ts) {
  __shared__ double colv[64];
  const int i = threadIdx.x;
  long long t0 = now();
  double a[K];
#pragma unroll
  for (int c = 0; c < K; ++c) a[c] = (i < k && c < k) ? G[i * k + c] : (i == c ? 1.0 : 0.0);
  __builtin_amdgcn_s_waitcnt(0);
  long long t1 = now();
#pragma unroll
  for (int j = 0; j < K; ++j) {
    colv[i] = a[j];
    __builtin_amdgcn_s_waitcnt(0xc07f);
    const double d = colv[j];
    const double inv = rsqrt_nr(d);
    const double lij = (i == j) ? d * inv : a[j] * inv;
    if (i >= j) a[j] = lij;
    colv[i] = lij;
    double cv[K];
#pragma unroll
    for (int c = j + 1; c < K; ++c) cv[c] = colv[c];
#pragma unroll
    for (int c = j + 1; c < K; ++c)
      if (i > j) a[c] -= lij * cv[c];
  }
  long long t2 = now();
  if (i < k)
    for (int c = 0; c < k; ++c) Rinv[i * k + c] = a[c < K ? c : 0];
  long long t3 = now();
  if (i == 0) { ts[0] = t1 - t0; ts[1] = t2 - t1; ts[2] = t3 - t2; }
}

// variant D: only the broadcast + FMA part (pivot fixed to 1)
template <int K>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1)))
chol_nopiv(const double* G, int k, double* Rinv, long long* ts) {
  __shared__ double colv[64];
  const int i = threadIdx.x;
  double a[K];
#pragma unroll
  for (int c = 0; c < K; ++c) a[c] = (i < k && c < k) ? G[i * k + c] : (i == c ? 1.0 : 0.0);
  __builtin_amdgcn_s_waitcnt(0);
  long long t1 = now();
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const double lij = a[j] * 0.01;
    colv[i] = lij;
    double cv[K];
#pragma unroll
    for (int c = j + 1; c < K; ++c) cv[c] = colv[c];
#pragma unroll
    for (int c = j + 1; c < K; ++c)
      if (i > j) a[c] -= lij * cv[c];
  }
  long long t2 = now();
  if (i < k)
    for (int c = 0; c < k; ++c) Rinv[i * k + c] = a[c < K ? c : 0];
  if (i == 0) { ts[0] = 0; ts[1] = t2 - t1; ts[2] = 0; }
}

// variant B: same with readlane broadcasts
__device__ __forceinline__ double bcast(double v, int src) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = __builtin_amdgcn_readlane((unsigned)u, src);
  const unsigned hi = __builtin_amdgcn_readlane((unsigned)(u >> 32), src);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}
template <int K>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(1, 1)))
chol_rl(const double* G, int k, double* Rinv, long long* ts) {
  const int i = threadIdx.x;
  long long t0 = now();
  double a[K];
#pragma unroll
  for (int c = 0; c < K; ++c) a[c] = (i < k && c < k) ? G[i * k + c] : (i == c ? 1.0 : 0.0);
  __builtin_amdgcn_s_waitcnt(0);
  long long t1 = now();
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const double d = bcast(a[j], j);
    const double piv = __builtin_sqrt(d);
    const double inv = 1.0 / piv;
    const double lij = (i == j) ? piv : a[j] * inv;
    if (i >= j) a[j] = lij;
#pragma unroll
    for (int c = j + 1; c < K; ++c) {
      const double lcj = bcast(lij, c);
      if (i > j) a[c] -= lij * lcj;
    }
  }
  long long t2 = now();
  if (i < k)
    for (int c = 0; c < k; ++c) Rinv[i * k + c] = a[c < K ? c : 0];
  long long t3 = now();
  if (i == 0) { ts[0] = t1 - t0; ts[1] = t2 - t1; ts[2] = t3 - t2; }
}

// variant C: only sqrt/div chain (lower bound of the serial pivots)
template <int K>
__global__ void __launch_bounds__(64) chol_pivots(const double* G, int k, double* Rinv, long long* ts) {
  const int i = threadIdx.x;
  double x = G[i];
  long long t1 = now();
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const double piv = __builtin_sqrt(x);
    x = x / piv + 1.0;
  }
  long long t2 = now();
  Rinv[i] = x;
  if (i == 0) { ts[0] = 0; ts[1] = t2 - t1; ts[2] = 0; }
}

template <typename F>
int run(const char* name, F kern, const double* dG, int k, double* dR, long long* dts) {
  long long h[3];
  float best = 1e9;
  for (int r = 0; r < 20; ++r) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    kern<<<1, 64>>>(dG, k, dR, dts);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    if (ms < best) best = ms;
    hipEventDestroy(e0); hipEventDestroy(e1);
  }
  CK(hipMemcpy(h, dts, sizeof(h), hipMemcpyDeviceToHost));
  // s_memtime runs at 100 MHz on MI300/MI355 (10 ns ticks)
  printf("%-14s k=%d event %.1f us | load %lld  chol %lld  store %lld ticks\n", name, k, best * 1e3, h[0], h[1], h[2]);
  return 0;
}

int main() {
  const int k = 40;
  std::vector<double> G(k * k, 0.0);
  for (int i = 0; i < k; ++i) {
    for (int j = 0; j < k; ++j) G[i * k + j] = 1.0 / (1.0 + std::abs(i - j));
    G[i * k + i] += k;
  }
  double *dG, *dR; long long* dts;
  CK(hipMalloc(&dG, k * k * 8)); CK(hipMalloc(&dR, 64 * 64 * 8)); CK(hipMalloc(&dts, 64));
  CK(hipMemcpy(dG, G.data(), k * k * 8, hipMemcpyHostToDevice));
  run("bulk-lds<48>", chol_bulk<48>, dG, k, dR, dts);
  run("readlane<48>", chol_rl<48>, dG, k, dR, dts);
  run("bulk-rsq<48>", chol_bulk_rsq<48>, dG, k, dR, dts);
  run("nopiv<48>", chol_nopiv<48>, dG, k, dR, dts);
  run("bulk-lds<16>", chol_bulk<16>, dG, 16, dR, dts);
  run("readlane<16>", chol_rl<16>, dG, 16, dR, dts);
  return 0;
}
