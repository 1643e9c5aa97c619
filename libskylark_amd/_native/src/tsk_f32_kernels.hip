// f32 tall-skinny helpers for the final randSVD basis (CholeskyQR2 + U):
//
//   sl_tsk_f32_xm:  Q = Y M  (Y: m x k f32, M: k x k2 f32, k, k2 <= 64)
//                   optionally stores Q and/or accumulates G = Q^T Q (f64 out)
//                   with M == NULL meaning Q = Y (a plain Gram pass).
//
// Y is only m x k floats (a few % of A's bytes) so these passes are cheap as
// long as they stream: one workgroup of 256 threads per 64-row chunk,
// persistent grid, Y chunk transposed into LDS, 4x4 register blocks for both
// the small GEMM and the Gram (16 FMAs per two ds_read_b128), per-workgroup
// Gram slabs summed by k_slab_reduce_rows in f64.  hipBLASLt's choice for
// these (k x 1e6) x (1e6 x k) shapes was ~40x slower (profiles/).
#include "sl_common.hpp"

int sl_slab_reduce_launch_f64(const float* slab, int nslab, int64_t slab_stride, int ld_in, int rows,
                              int cols, double* out, int ld_out, hipStream_t s);

namespace {

constexpr int CH = 64;  // rows per chunk
constexpr int KMAX = 64;

typedef __attribute__((ext_vector_type(4))) float f4;

__global__ void __launch_bounds__(256)
k_f32_xm(const float* __restrict__ Y, int64_t m, int k, int64_t ldy, const float* __restrict__ M,
         int k2, float* __restrict__ out, int64_t ldo, float* __restrict__ Gslab) {
  __shared__ __attribute__((aligned(16))) float Yt[KMAX][CH];      // transposed chunk
  __shared__ __attribute__((aligned(16))) float Ms[KMAX][KMAX];
  __shared__ __attribute__((aligned(16))) float Qs[CH][KMAX + 4];  // +4: b128-aligned, fewer conflicts
  const int t = threadIdx.x;
  const int rg = t >> 4, cg = t & 15;  // 4x4 block coordinates
  const bool ident = (M == nullptr);
  const int kq = ident ? k : k2;
  if (!ident) {
    for (int e = t; e < KMAX * KMAX; e += 256) {
      const int i = e / KMAX, j = e % KMAX;
      Ms[i][j] = (i < k && j < k2) ? M[i * k2 + j] : 0.f;
    }
  }
  float g[4][4] = {};
  const int64_t nchunks = (m + CH - 1) / CH;
  for (int64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const int64_t r0 = c * CH;
    __syncthreads();
    for (int e = t; e < CH * KMAX; e += 256) {
      const int row = e / KMAX, col = e % KMAX;
      float v = 0.f;
      if (col < k && r0 + row < m) v = Y[(r0 + row) * ldy + col];
      Yt[col][row] = v;
    }
    __syncthreads();
    // ---- Q block (rows 4rg.., cols 4cg..)
    float q[4][4] = {};
    if (ident) {
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) q[a][b] = Yt[4 * cg + b][4 * rg + a];
    } else {
      for (int i = 0; i < k; ++i) {
        const f4 y = *(const f4*)&Yt[i][4 * rg];
        const f4 mm = *(const f4*)&Ms[i][4 * cg];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 4; ++b) q[a][b] += y[a] * mm[b];
      }
    }
#pragma unroll
    for (int a = 0; a < 4; ++a) *(f4*)&Qs[4 * rg + a][4 * cg] = f4{q[a][0], q[a][1], q[a][2], q[a][3]};
    if (out) {
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const int64_t r = r0 + 4 * rg + a;
        if (r < m)
#pragma unroll
          for (int b = 0; b < 4; ++b)
            if (4 * cg + b < kq) out[r * ldo + 4 * cg + b] = q[a][b];
      }
    }
    if (Gslab) {
      __syncthreads();
      // ---- G block (rows 4rg.. of Q^T, cols 4cg..) over the chunk's rows
      for (int r = 0; r < CH; ++r) {
        const f4 x = *(const f4*)&Qs[r][4 * rg];
        const f4 z = *(const f4*)&Qs[r][4 * cg];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
          for (int b = 0; b < 4; ++b) g[a][b] += x[a] * z[b];
      }
    }
  }
  if (Gslab) {
    float* gs = Gslab + (int64_t)blockIdx.x * KMAX * KMAX;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 4; ++b) gs[(4 * rg + a) * KMAX + 4 * cg + b] = g[a][b];
  }
}

}  // namespace

SL_API int64_t sl_tsk_f32_workspace(int64_t m) {
  int64_t nch = (m + CH - 1) / CH;
  int64_t g = nch < 1024 ? nch : 1024;
  return g * KMAX * KMAX * 4 + 256;
}

SL_API int sl_tsk_f32_xm(const float* Y, int64_t m, int k, int64_t ldy, const float* M, int k2,
                         float* out, int64_t ldo, double* G, void* ws, void* stream) {
  if (m <= 0) return SL_OK;
  if (k < 1 || k > KMAX || (M && (k2 < 1 || k2 > KMAX))) {
    sl_set_last_error("tsk_f32_xm: needs 1 <= k, k2 <= 64");
    return SL_ERR_UNSUPPORTED;
  }
  hipStream_t s = (hipStream_t)stream;
  const int64_t nch = (m + CH - 1) / CH;
  const int g = (int)(nch < 1024 ? nch : 1024);
  float* slab = G ? (float*)ws : nullptr;
  k_f32_xm<<<g, 256, 0, s>>>(Y, m, k, ldy, M, k2, out, ldo, slab);
  SL_LAUNCH_CHECK();
  if (G) {
    const int kq = M ? k2 : k;
    return sl_slab_reduce_launch_f64(slab, g, (int64_t)KMAX * KMAX, KMAX, kq, kq, G, kq, s);
  }
  return SL_OK;
}
