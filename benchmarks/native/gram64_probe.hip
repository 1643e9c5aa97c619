// Stand-alone probe: where does the fp64 Gram (G = Y^T Y, Y m x 40 f32) spend
// its time?  Ablations of the k_gram64 structure: full, loads only, f64 MFMA
// only, and grid / unroll variants.  Build:
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 gram64_probe.hip -o gram64_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s\n", hipGetErrorString(e)); return 1; } } while (0)

typedef __attribute__((ext_vector_type(4))) double d4v;

// MODE 0 full, 1 loads only (VALU sum), 2 MFMA only (register operands)
template <int KT, int UNR, int MODE>
__global__ void __launch_bounds__(256)
gram(const float* __restrict__ Y, long m, int k, long ldy, double* __restrict__ out) {
  constexpr int NT = KT * (KT + 1) / 2;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int q = lane >> 4, c = lane & 15;
  d4v acc[NT];
#pragma unroll
  for (int p = 0; p < NT; ++p) acc[p] = d4v{0.0, 0.0, 0.0, 0.0};
  double vs = 0.0;
  const long step = (long)gridDim.x * 4 * 4 * UNR;
  for (long r0 = ((long)blockIdx.x * 4 + w) * 4 * UNR; r0 < m; r0 += step) {
    float v[UNR][KT];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const long r = r0 + 4 * u + q;
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        const int col = 16 * t + c;
        if constexpr (MODE == 2) v[u][t] = (float)(r0 + u + t) * 1e-9f;
        else v[u][t] = (r < m && col < k) ? Y[r * ldy + col] : 0.f;
      }
    }
    if constexpr (MODE == 1) {
#pragma unroll
      for (int u = 0; u < UNR; ++u)
#pragma unroll
        for (int t = 0; t < KT; ++t) vs += (double)v[u][t];
    } else {
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        int p = 0;
#pragma unroll
        for (int a = 0; a < KT; ++a)
#pragma unroll
          for (int b = a; b < KT; ++b, ++p)
            acc[p] = __builtin_amdgcn_mfma_f64_16x16x4f64((double)v[u][a], (double)v[u][b], acc[p], 0, 0, 0);
      }
    }
  }
  double s = vs;
#pragma unroll
  for (int p = 0; p < NT; ++p) s += acc[p][0] + acc[p][1] + acc[p][2] + acc[p][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

// Pipelined: contiguous 32-row chunks (k % 8 == 0, ldy == k), float4 loads of
// chunk i+1 in flight while chunk i goes registers -> wave-private LDS tile
// (pitch LD = 16 mod 32: conflict-free MFMA-layout ds_read_b32) -> f64 MFMA.
template <int KT>
__global__ void __launch_bounds__(256)
gram_pipe(const float* __restrict__ Y, long m, int k, long ldy, double* __restrict__ out) {
  constexpr int NT = KT * (KT + 1) / 2;
  constexpr int LD = (KT & 1) ? 16 * KT : 16 * KT + 16;
  constexpr int NLMAX = 8;  // k / 8 float4 per lane per chunk (k <= 64)
  __shared__ float tile[4][32 * LD];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int q = lane >> 4, c = lane & 15;
  float* T = tile[w];
  const int nl = k >> 3;
  int loff[NLMAX], lrow[NLMAX];
#pragma unroll
  for (int j = 0; j < NLMAX; ++j) {
    const int e = 4 * (64 * j + lane);
    lrow[j] = e / k;
    loff[j] = lrow[j] * LD + (e - lrow[j] * k);
  }
  d4v acc[NT];
#pragma unroll
  for (int p = 0; p < NT; ++p) acc[p] = d4v{0.0, 0.0, 0.0, 0.0};
  const long step = (long)gridDim.x * 4 * 32;
  long r0 = ((long)blockIdx.x * 4 + w) * 32;
  float4 nx[NLMAX];
  auto load = [&](long rb) {
#pragma unroll
    for (int j = 0; j < NLMAX; ++j)
      if (j < nl) nx[j] = (rb + lrow[j] < m) ? *(const float4*)(Y + rb * k + 4 * (64 * j + lane)) : float4{0, 0, 0, 0};
  };
  if (r0 < m) load(r0);
  for (; r0 < m; r0 += step) {
#pragma unroll
    for (int j = 0; j < NLMAX; ++j)
      if (j < nl) *(float4*)(T + loff[j]) = nx[j];
    if (r0 + step < m) load(r0 + step);
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      double v[KT];
#pragma unroll
      for (int t = 0; t < KT; ++t) v[t] = (16 * t + c < k) ? (double)T[(4 * u + q) * LD + 16 * t + c] : 0.0;
      int p = 0;
#pragma unroll
      for (int a = 0; a < KT; ++a)
#pragma unroll
        for (int b = a; b < KT; ++b, ++p) acc[p] = __builtin_amdgcn_mfma_f64_16x16x4f64(v[a], v[b], acc[p], 0, 0, 0);
    }
  }
  double s = 0.0;
#pragma unroll
  for (int p = 0; p < NT; ++p) s += acc[p][0] + acc[p][1] + acc[p][2] + acc[p][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int KT>
float run_pipe(const float* Y, long m, int k, double* out, int grid, int reps) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  gram_pipe<KT><<<grid, 256>>>(Y, m, k, k, out);
  hipEventRecord(e0);
  for (int i = 0; i < reps; ++i) gram_pipe<KT><<<grid, 256>>>(Y, m, k, k, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e3f / reps;
}

template <int KT, int UNR, int MODE>
float run(const float* Y, long m, int k, double* out, int grid, int reps) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  gram<KT, UNR, MODE><<<grid, 256>>>(Y, m, k, k, out);
  hipEventRecord(e0);
  for (int i = 0; i < reps; ++i) gram<KT, UNR, MODE><<<grid, 256>>>(Y, m, k, k, out);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  return ms * 1e3f / reps;
}

int main() {
  const long m = 1000000;
  const int k = 40;
  float* Y;
  double* out;
  CK(hipMalloc(&Y, m * k * 4));
  CK(hipMalloc(&out, 8192 * 256 * 8));
  CK(hipMemset(Y, 0, m * k * 4));
  const int grids[] = {256, 512, 1024, 2048};
  for (int g : grids) printf("grid %4d  pipelined %7.1f us\n", g, run_pipe<3>(Y, m, k, out, g, 20));
  for (int g : grids) {
    printf("grid %4d  full u8 %7.1f  u4 %7.1f  u16 %7.1f | loads u8 %7.1f | mfma u8 %7.1f us\n", g,
           run<3, 8, 0>(Y, m, k, out, g, 20), run<3, 4, 0>(Y, m, k, out, g, 20), run<3, 16, 0>(Y, m, k, out, g, 20),
           run<3, 8, 1>(Y, m, k, out, g, 20), run<3, 8, 2>(Y, m, k, out, g, 20));
  }
  CK(hipDeviceSynchronize());
  return 0;
}
