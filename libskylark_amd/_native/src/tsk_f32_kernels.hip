// f32 tall-skinny helpers for the final randSVD basis (CholeskyQR2 + U):
//
//   sl_tsk_f32_xm:  Q = Y M  (Y: m x k f32, M: k x k2 f32, k, k2 <= 64)
//                   optionally stores Q and/or accumulates G = Q^T Q (f64 out)
//                   with M == NULL meaning Q = Y (a plain Gram pass).
//
// Exact-f32 products on the matrix cores (v_mfma_f32_32x32x2_f32 is a k-ordered
// fmaf chain, no reduced-precision shortcut).  One wave owns 32 rows at a time:
//   * Q tile (32 rows x 32 cols) = sum over k-pairs of mfma(Y[r, 2s+h], M[2s+h, c])
//     with M kept in registers for the whole kernel;
//   * the Q tile's ACCUMULATOR registers are directly the K = 2 operands of
//     the Gram MFMA: register `reg` of lane (h, c) holds row 4h + (reg&3) +
//     8(reg>>2), col c — both operands of mfma(Qa[reg], Qb[reg]) pair the same
//     two rows, so 16 MFMAs add the 32 rows' outer products with no LDS and
//     no shuffles;
//   * per-workgroup Gram slabs (waves summed through LDS), reduced in f64.
// hipBLASLt's choice for these (k x 1e6) x (1e6 x k) shapes was ~40x slower.
#include "sl_common.hpp"

int sl_slab_reduce_launch_f64(const float* slab, int nslab, int64_t slab_stride, int ld_in, int rows,
                              int cols, double* out, int ld_out, hipStream_t s);
int sl_slab_reduce_launch_d2d(const double* slab, int nslab, int64_t slab_stride, int ld_in, int rows,
                              int cols, double* out, int ld_out, hipStream_t s);

namespace {

typedef __attribute__((ext_vector_type(16))) float f16v;
constexpr int KMAX = 64;
constexpr int WPB = 4;  // waves per block

__device__ __forceinline__ int crow(int reg, int h) { return (reg & 3) + 8 * (reg >> 2) + 4 * h; }

template <int KT2, bool IDENT, bool STORE, bool GRAM>
__global__ void __launch_bounds__(256)
k_f32_mfma(const float* __restrict__ Y, int64_t m, int k, int64_t ldy, const float* __restrict__ M,
           int k2, float* __restrict__ out, int64_t ldo, float* __restrict__ Gslab) {
  __shared__ float gred[1][KT2 * 32][KT2 * 32 + 1];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  const int h = lane >> 5, c = lane & 31;
  const int kq = IDENT ? k : k2;

  // M fragments: B operand of step s: M[2s + h][32 ct + c]
  float mreg[IDENT ? 1 : KMAX / 2][KT2];
  if constexpr (!IDENT) {
#pragma unroll
    for (int s = 0; s < KMAX / 2; ++s)
#pragma unroll
      for (int ct = 0; ct < KT2; ++ct) {
        const int r = 2 * s + h, col = 32 * ct + c;
        mreg[s][ct] = (r < k && col < k2) ? M[r * k2 + col] : 0.f;
      }
  }
  f16v g[KT2][KT2];
#pragma unroll
  for (int a = 0; a < KT2; ++a)
#pragma unroll
    for (int b = 0; b < KT2; ++b) g[a][b] = f16v{};

  const int64_t ngroups = (m + 31) / 32;
  for (int64_t gi = (int64_t)blockIdx.x * WPB + w; gi < ngroups; gi += (int64_t)gridDim.x * WPB) {
    const int64_t r0 = gi * 32;
    f16v q[KT2];
    if constexpr (IDENT) {
#pragma unroll
      for (int ct = 0; ct < KT2; ++ct)
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
          const int64_t r = r0 + crow(reg, h);
          const int col = 32 * ct + c;
          q[ct][reg] = (r < m && col < k) ? Y[r * ldy + col] : 0.f;
        }
    } else {
#pragma unroll
      for (int ct = 0; ct < KT2; ++ct) q[ct] = f16v{};
      const int64_t r = r0 + c;
      const float* yr = Y + (r < m ? r : 0) * ldy;
      const bool rv = r < m;
#pragma unroll
      for (int s = 0; s < KMAX / 2; ++s) {
        if (2 * s >= k) break;
        const int col = 2 * s + h;
        const float a = (rv && col < k) ? yr[col] : 0.f;
#pragma unroll
        for (int ct = 0; ct < KT2; ++ct)
          q[ct] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, mreg[s][ct], q[ct], 0, 0, 0);
      }
    }
    if constexpr (STORE) {
#pragma unroll
      for (int ct = 0; ct < KT2; ++ct)
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
          const int64_t r = r0 + crow(reg, h);
          const int col = 32 * ct + c;
          if (r < m && col < kq) out[r * ldo + col] = q[ct][reg];
        }
    }
    if constexpr (GRAM) {
#pragma unroll
      for (int a = 0; a < KT2; ++a)
#pragma unroll
        for (int b = a; b < KT2; ++b)
#pragma unroll
          for (int reg = 0; reg < 16; ++reg)
            g[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(q[a][reg], q[b][reg], g[a][b], 0, 0, 0);
    }
  }
  if constexpr (GRAM) {
    // wave 0..3 partial tiles -> LDS -> one slab per workgroup (KMAX x KMAX)
    for (int v = 0; v < WPB; ++v) {
      if (w == v) {
#pragma unroll
        for (int a = 0; a < KT2; ++a)
#pragma unroll
          for (int b = 0; b < KT2; ++b)
#pragma unroll
            for (int reg = 0; reg < 16; ++reg) {
              const int i = 32 * a + crow(reg, h), j = 32 * b + c;
              const float val = (b >= a) ? g[a][b][reg] : 0.f;
              if (v == 0) gred[0][i][j] = val;
              else gred[0][i][j] += val;
            }
      }
      __syncthreads();
    }
    float* gs = Gslab + (int64_t)blockIdx.x * KMAX * KMAX;
    for (int e = threadIdx.x; e < KT2 * 32 * KT2 * 32; e += 256) {
      const int i = e / (KT2 * 32), j = e % (KT2 * 32);
      // symmetrise: upper tiles were accumulated, mirror into the lower part
      const float val = (j / 32 >= i / 32) ? gred[0][i][j] : gred[0][j][i];
      gs[i * KMAX + j] = val;
    }
  }
}

// G = Y^T Y in fp64 from f32 Y (k <= 64) on the f64 matrix cores
// (v_mfma_f64_16x16x4f64).  Lane l of a wave loads Y[r + (l>>4)][16 t + (l&15)]:
// that register is at once the A operand (G rows of tile t) and the B operand
// (G columns of tile t) of the 16x16x4 MFMA, so the upper-triangle tile pairs
// (a <= b) accumulate G with no data movement; 8 four-row chunks per wave
// iteration keep 8*KT loads in flight.  Products and sums are fp64 (f32 -> f64
// is exact), so G carries fp64 accuracy and one fp64 CholeskyQR of Y is as
// orthogonal as CholeskyQR2 with an f32 second Gram, at a third of the work.
// Per-workgroup k x k f64 slabs (the 4 waves summed through LDS), then a
// deterministic slab reduction.
typedef __attribute__((ext_vector_type(4))) double d4v;
constexpr int G64_UNR = 8;
constexpr int G64_GRID_MAX = 512;

template <int KT>
__global__ void __launch_bounds__(256)
k_gram64(const float* __restrict__ Y, int64_t m, int k, int64_t ldy, double* __restrict__ slab) {
  constexpr int KP = 16 * KT, NT = KT * (KT + 1) / 2;
  __shared__ double red[KP][KP + 1];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int q = lane >> 4, c = lane & 15;
  d4v acc[NT];
#pragma unroll
  for (int p = 0; p < NT; ++p) acc[p] = d4v{0.0, 0.0, 0.0, 0.0};
  const int64_t step = (int64_t)gridDim.x * WPB * 4 * G64_UNR;
  for (int64_t r0 = ((int64_t)blockIdx.x * WPB + w) * 4 * G64_UNR; r0 < m; r0 += step) {
    float v[G64_UNR][KT];
#pragma unroll
    for (int u = 0; u < G64_UNR; ++u) {
      const int64_t r = r0 + 4 * u + q;
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        const int col = 16 * t + c;
        v[u][t] = (r < m && col < k) ? Y[r * ldy + col] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < G64_UNR; ++u) {
      int p = 0;
#pragma unroll
      for (int a = 0; a < KT; ++a)
#pragma unroll
        for (int b = a; b < KT; ++b, ++p)
          acc[p] = __builtin_amdgcn_mfma_f64_16x16x4f64((double)v[u][a], (double)v[u][b], acc[p], 0, 0, 0);
    }
  }
  // C/D layout of the f64 16x16x4 form: col = lane & 15, row = (lane >> 4) + 4 reg
  for (int vw = 0; vw < WPB; ++vw) {
    if (w == vw) {
      int p = 0;
#pragma unroll
      for (int a = 0; a < KT; ++a)
#pragma unroll
        for (int b = a; b < KT; ++b, ++p)
#pragma unroll
          for (int reg = 0; reg < 4; ++reg) {
            const int i = 16 * a + q + 4 * reg, j = 16 * b + c;
            if (vw == 0) red[i][j] = acc[p][reg];
            else red[i][j] += acc[p][reg];
          }
    }
    __syncthreads();
  }
  double* gs = slab + (int64_t)blockIdx.x * k * k;
  for (int e = threadIdx.x; e < k * k; e += 256) {
    const int i = e / k, j = e - (e / k) * k;
    gs[e] = ((i >> 4) <= (j >> 4)) ? red[i][j] : red[j][i];  // mirror the lower tiles
  }
}

// Contiguous fast path (ldy == k, k % 8 == 0): each wave streams 32-row chunks
// (32 k contiguous floats) with float4 loads; chunk i+1 is in flight while
// chunk i goes registers -> a wave-private LDS tile (row pitch LD = 16 mod 32,
// so the MFMA-layout ds_read_b32 are bank-conflict free) -> f64 MFMAs.  The
// strided kernel above serialises its 4-byte loads with the MFMAs (loads
// 50 us + MFMA 51 us -> 118 us at m = 1e6, k = 40); this one overlaps them
// (60 us; benchmarks/native/gram64_probe.hip).
template <int KT>
__global__ void __launch_bounds__(256)
k_gram64_pipe(const float* __restrict__ Y, int64_t m, int k, double* __restrict__ slab) {
  constexpr int KP = 16 * KT, NT = KT * (KT + 1) / 2;
  constexpr int LD = (KT & 1) ? 16 * KT : 16 * KT + 16;
  constexpr int NLMAX = 2 * KT;  // k / 8 float4 per lane per chunk
  __shared__ float tile[WPB][32 * LD];
  __shared__ double red[KP][KP + 1];
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
  const int64_t step = (int64_t)gridDim.x * WPB * 32;
  int64_t r0 = ((int64_t)blockIdx.x * WPB + w) * 32;
  float4 nx[NLMAX];
  // unconditional loads (rows past m read row 0, zeroed after the load): a
  // per-element "load or zero" branch makes hipcc wait vmcnt(0) inside the
  // loop, which serialised the prefetch of the next chunk with this chunk's
  // MFMAs
  auto load = [&](int64_t rb) {
#pragma unroll
    for (int j = 0; j < NLMAX; ++j) {
      // every slot loads (slots past k / 8 read Y[0..3]: no branch, so no
      // conservative vmcnt(0) at the join points)
      const bool in = j < nl && rb + lrow[j] < m;
      const float4 v = *(const float4*)(Y + (in ? rb * k + 4 * (64 * j + lane) : 0));
      nx[j] = in ? v : float4{0.f, 0.f, 0.f, 0.f};
    }
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
  for (int vw = 0; vw < WPB; ++vw) {
    if (w == vw) {
      int p = 0;
#pragma unroll
      for (int a = 0; a < KT; ++a)
#pragma unroll
        for (int b = a; b < KT; ++b, ++p)
#pragma unroll
          for (int reg = 0; reg < 4; ++reg) {
            const int i = 16 * a + q + 4 * reg, j = 16 * b + c;
            if (vw == 0) red[i][j] = acc[p][reg];
            else red[i][j] += acc[p][reg];
          }
    }
    __syncthreads();
  }
  double* gs = slab + (int64_t)blockIdx.x * k * k;
  for (int e = threadIdx.x; e < k * k; e += 256) {
    const int i = e / k, j = e - (e / k) * k;
    gs[e] = ((i >> 4) <= (j >> 4)) ? red[i][j] : red[j][i];
  }
}

// Q = Y M, stored (no Gram), contiguous fast path (ldy == k, k % 8 == 0,
// ldo == k2): the U = Y (R^{-1} U_B) pass of randSVD.  Each wave streams 32-row
// chunks with float4 loads (next chunk in flight), stages them in a
// wave-private LDS tile of odd pitch k + 1 (row-per-lane A reads of the
// 32x32x2 f32 MFMA are then bank-conflict free), multiplies with M held in
// registers, and writes the 32 x k2 result back through LDS as coalesced
// float4 rows — the strided kernel above reads and writes one float per lane
// per instruction.
template <int KT2>
__global__ void __launch_bounds__(256)
k_xm_pipe(const float* __restrict__ Y, int64_t m, int k, const float* __restrict__ M, int k2,
          float* __restrict__ out, float* const* __restrict__ optr) {
  // optr: the output pointer read from device memory (a graph node whose
  // destination changes every replay)
  if (optr) out = optr[0];
  // wave tiles sized by k / k2 (dynamic LDS: xm_pipe_lds): 32 x (k + 1) in,
  // 32 x k2 out -- 31 KB per block at k = 40, k2 = 20, five blocks per CU
  extern __shared__ __attribute__((aligned(16))) float xsm[];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int h = lane >> 5, c = lane & 31;
  float* Ti = xsm + w * 32 * (k + 1);
  float* To = xsm + WPB * 32 * (k + 1) + w * 32 * k2;
  const int lda = k + 1;
  float mreg[KMAX / 2][KT2];
#pragma unroll
  for (int s = 0; s < KMAX / 2; ++s)
#pragma unroll
    for (int ct = 0; ct < KT2; ++ct) {
      const int r = 2 * s + h, col = 32 * ct + c;
      mreg[s][ct] = (r < k && col < k2) ? M[r * k2 + col] : 0.f;
    }
  // consume M here so hipcc's wait for its loads sits before the loop (else
  // the loop's first MFMA carries a vmcnt(0) that also drains the prefetch)
#pragma unroll
  for (int s = 0; s < KMAX / 2; ++s)
#pragma unroll
    for (int ct = 0; ct < KT2; ++ct) asm volatile("" ::"v"(mreg[s][ct]));
  constexpr int NLMAX = KMAX / 8;
  const int nl = k >> 3;
  int loff[NLMAX], lrow[NLMAX];
#pragma unroll
  for (int j = 0; j < NLMAX; ++j) {
    const int e = 4 * (64 * j + lane);
    lrow[j] = e / k;
    loff[j] = lrow[j] * lda + (e - lrow[j] * k);
  }
  const int64_t step = (int64_t)gridDim.x * WPB * 32;
  int64_t r0 = ((int64_t)blockIdx.x * WPB + w) * 32;
  float4 nx[NLMAX];
  // unconditional loads (rows past m read row 0, zeroed after the load): a
  // per-element "load or zero" branch makes hipcc wait vmcnt(0) inside the
  // loop, which serialised the prefetch of the next chunk with this chunk's
  // MFMAs
  auto load = [&](int64_t rb) {
#pragma unroll
    for (int j = 0; j < NLMAX; ++j) {
      // every slot loads (slots past k / 8 read Y[0..3]: no branch, so no
      // conservative vmcnt(0) at the join points)
      const bool in = j < nl && rb + lrow[j] < m;
      const float4 v = *(const float4*)(Y + (in ? rb * k + 4 * (64 * j + lane) : 0));
      nx[j] = in ? v : float4{0.f, 0.f, 0.f, 0.f};
    }
  };
  if (r0 < m) load(r0);
  for (; r0 < m; r0 += step) {
#pragma unroll
    for (int j = 0; j < NLMAX; ++j)
      if (j < nl) {
        float* d = Ti + loff[j];
        d[0] = nx[j].x;
        d[1] = nx[j].y;
        d[2] = nx[j].z;
        d[3] = nx[j].w;
      }
    if (r0 + step < m) load(r0 + step);
    f16v q[KT2];
#pragma unroll
    for (int ct = 0; ct < KT2; ++ct) q[ct] = f16v{};
#pragma unroll
    for (int s = 0; s < KMAX / 2; ++s) {
      if (2 * s >= k) break;
      const float a = Ti[c * lda + 2 * s + h];
#pragma unroll
      for (int ct = 0; ct < KT2; ++ct) q[ct] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, mreg[s][ct], q[ct], 0, 0, 0);
    }
#pragma unroll
    for (int ct = 0; ct < KT2; ++ct)
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int col = 32 * ct + c;
        if (col < k2) To[crow(reg, h) * k2 + col] = q[ct][reg];
      }
    const int64_t left = m - r0;
    float* o = out + r0 * k2;
    if (left >= 32) {
      for (int e4 = lane; e4 < 8 * k2; e4 += 64) *(float4*)(o + 4 * e4) = *(const float4*)(To + 4 * e4);
    } else {
      for (int e = lane; e < (int)left * k2; e += 64) o[e] = To[e];
    }
  }
}

// Q^T = (Y M)^T as bf16 (k2 x m, row stride ldo): the CholeskyQR step between
// randSVD power passes writes the next pass's operand directly in the fused
// pass's "Zt" layout (one launch instead of Q store + bf16 cast + transpose).
// Small m (the n x k iterate): M staged in LDS, one output per thread, r
// fastest so the bf16 stores coalesce.
__global__ void __launch_bounds__(256)
k_xm_bf16t(const float* __restrict__ Y, int64_t m, int k, int64_t ldy, const float* __restrict__ M, int k2,
           bf16_t* __restrict__ out, int64_t ldo) {
  __shared__ float ms[KMAX * KMAX];
  for (int e = threadIdx.x; e < k * k2; e += 256) ms[e] = M[e];
  __syncthreads();
  const int64_t total = m * k2;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int c = (int)(t / m);
    const int64_t r = t - (int64_t)c * m;
    const float* y = Y + r * ldy;
    float acc = 0.f;
    for (int j = 0; j < k; ++j) acc = fmaf(y[j], ms[j * k2 + c], acc);
    out[(int64_t)c * ldo + r] = f_to_bf16(acc);
  }
}

constexpr int XM_PIPE_GRID_MAX = 2048;
size_t xm_pipe_lds(int k, int k2) {
  const size_t b = (size_t)WPB * 32 * ((k + 1) + k2) * sizeof(float);
  if (b > 64 * 1024) {   // k, k2 near 64: past the default dynamic-LDS cap (per device)
    (void)sl_lds_attr((const void*)k_xm_pipe<1>, 96 * 1024);
    (void)sl_lds_attr((const void*)k_xm_pipe<2>, 96 * 1024);
  }
  return b;
}

constexpr int G64_PIPE_GRID_MAX = 1024;

int gram64_pipe_grid(int64_t m) {
  const int64_t g = (m + WPB * 32 - 1) / (WPB * 32);
  return (int)(g < G64_PIPE_GRID_MAX ? (g < 1 ? 1 : g) : G64_PIPE_GRID_MAX);
}

int gram64_grid(int64_t m) {
  const int64_t rows_per_block = (int64_t)WPB * 4 * G64_UNR;
  const int64_t g = (m + rows_per_block - 1) / rows_per_block;
  return (int)(g < G64_GRID_MAX ? (g < 1 ? 1 : g) : G64_GRID_MAX);
}

int grid_for(int64_t m) {
  const int64_t ng = (m + 31) / 32;
  int64_t g = (ng + WPB - 1) / WPB;
  return (int)(g < 512 ? (g < 1 ? 1 : g) : 512);
}

}  // namespace

SL_API int64_t sl_tsk_f32_workspace(int64_t m) { return (int64_t)grid_for(m) * KMAX * KMAX * 4 + 256; }

SL_API int64_t sl_tsk_gram64_workspace(int64_t m, int k) {
  const int g = gram64_grid(m) > gram64_pipe_grid(m) ? gram64_grid(m) : gram64_pipe_grid(m);
  return (int64_t)g * k * k * 8 + 256;
}

// G (k x k, f64) = Y^T Y with Y m x k f32 (row stride ldy); ws >= sl_tsk_gram64_workspace bytes.
SL_API int sl_tsk_gram64(const float* Y, int64_t m, int k, int64_t ldy, double* G, void* ws, void* stream) {
  if (k < 1 || k > KMAX) {
    sl_set_last_error("tsk_gram64: needs 1 <= k <= 64");
    return SL_ERR_UNSUPPORTED;
  }
  hipStream_t s = (hipStream_t)stream;
  if (m <= 0) return hipMemsetAsync(G, 0, (size_t)k * k * 8, s) == hipSuccess ? SL_OK : SL_ERR_HIP;
  double* slab = (double*)ws;
  if (ldy == k && k % 8 == 0) {
    const int g = gram64_pipe_grid(m);
    switch ((k + 15) / 16) {
      case 1: k_gram64_pipe<1><<<g, 256, 0, s>>>(Y, m, k, slab); break;
      case 2: k_gram64_pipe<2><<<g, 256, 0, s>>>(Y, m, k, slab); break;
      case 3: k_gram64_pipe<3><<<g, 256, 0, s>>>(Y, m, k, slab); break;
      default: k_gram64_pipe<4><<<g, 256, 0, s>>>(Y, m, k, slab); break;
    }
    SL_LAUNCH_CHECK();
    return sl_slab_reduce_launch_d2d(slab, g, (int64_t)k * k, k, k, k, G, k, s);
  }
  const int g = gram64_grid(m);
  switch ((k + 15) / 16) {
    case 1: k_gram64<1><<<g, 256, 0, s>>>(Y, m, k, ldy, slab); break;
    case 2: k_gram64<2><<<g, 256, 0, s>>>(Y, m, k, ldy, slab); break;
    case 3: k_gram64<3><<<g, 256, 0, s>>>(Y, m, k, ldy, slab); break;
    default: k_gram64<4><<<g, 256, 0, s>>>(Y, m, k, ldy, slab); break;
  }
  SL_LAUNCH_CHECK();
  return sl_slab_reduce_launch_d2d(slab, g, (int64_t)k * k, k, k, k, G, k, s);
}

// U = Y M with U read from optr[0] at run time (contiguous: ldy == k, k % 8
// == 0, U rows of k2 floats, U 16-byte aligned -- the caller checks U).
SL_API int sl_tsk_f32_xm_ind(const float* Y, int64_t m, int k, const float* M, int k2, float* const* optr,
                             void* stream) {
  if (m <= 0) return SL_OK;
  if (k < 8 || k > KMAX || k % 8 || k2 < 1 || k2 > KMAX || ((uintptr_t)Y & 15)) {
    sl_set_last_error("tsk_f32_xm_ind: needs 8 <= k <= 64, k % 8 == 0, 1 <= k2 <= 64, Y 16-byte aligned");
    return SL_ERR_UNSUPPORTED;
  }
  int64_t gx = (m + WPB * 32 - 1) / (WPB * 32);
  if (gx > XM_PIPE_GRID_MAX) gx = XM_PIPE_GRID_MAX;
  const size_t lds = xm_pipe_lds(k, k2);
  if (k2 > 32) k_xm_pipe<2><<<(int)gx, 256, lds, (hipStream_t)stream>>>(Y, m, k, M, k2, nullptr, optr);
  else k_xm_pipe<1><<<(int)gx, 256, lds, (hipStream_t)stream>>>(Y, m, k, M, k2, nullptr, optr);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

SL_API int sl_tsk_f32_xm(const float* Y, int64_t m, int k, int64_t ldy, const float* M, int k2,
                         float* out, int64_t ldo, double* G, void* ws, void* stream) {
  if (m <= 0) return SL_OK;
  if (k < 1 || k > KMAX || (M && (k2 < 1 || k2 > KMAX))) {
    sl_set_last_error("tsk_f32_xm: needs 1 <= k, k2 <= 64");
    return SL_ERR_UNSUPPORTED;
  }
  hipStream_t s = (hipStream_t)stream;
  const int g = grid_for(m);
  float* slab = G ? (float*)ws : nullptr;
  const int kq = M ? k2 : k;
  const bool two = kq > 32;
  const bool store = out != nullptr && M != nullptr;
#define SL_F(KT2, ID, ST, GR) k_f32_mfma<KT2, ID, ST, GR><<<g, 256, 0, s>>>(Y, m, k, ldy, M, k2, out, ldo, slab)
#define SL_F2(ID, ST, GR) { if (two) SL_F(2, ID, ST, GR); else SL_F(1, ID, ST, GR); }
  if (M && store && !G && ldy == k && k % 8 == 0 && ldo == k2 && ((uintptr_t)Y & 15) == 0 &&
      ((uintptr_t)out & 15) == 0) {
    int64_t gx = (m + WPB * 32 - 1) / (WPB * 32);
    if (gx > XM_PIPE_GRID_MAX) gx = XM_PIPE_GRID_MAX;
    const size_t lds = xm_pipe_lds(k, k2);
    if (two) k_xm_pipe<2><<<(int)gx, 256, lds, s>>>(Y, m, k, M, k2, out, nullptr);
    else k_xm_pipe<1><<<(int)gx, 256, lds, s>>>(Y, m, k, M, k2, out, nullptr);
    SL_LAUNCH_CHECK();
    return SL_OK;
  }
  if (!M) {
    if (!G) return SL_OK;
    SL_F2(true, false, true);
  } else if (store && G) SL_F2(false, true, true)
  else if (store) SL_F2(false, true, false)
  else if (G) SL_F2(false, false, true)
  else return SL_OK;
#undef SL_F2
#undef SL_F
  SL_LAUNCH_CHECK();
  if (G) return sl_slab_reduce_launch_f64(slab, g, (int64_t)KMAX * KMAX, KMAX, kq, kq, G, kq, s);
  return SL_OK;
}

// outT (k2 x m bf16, row stride ldo) = (Y M)^T, Y m x k f32 (row stride ldy), M k x k2 f32.
SL_API int sl_tsk_f32_xm_bf16t(const float* Y, int64_t m, int k, int64_t ldy, const float* M, int k2, void* outT,
                               int64_t ldo, void* stream) {
  if (m <= 0) return SL_OK;
  if (k < 1 || k > KMAX || k2 < 1 || k2 > KMAX || ldo < m) {
    sl_set_last_error("tsk_f32_xm_bf16t: needs 1 <= k, k2 <= 64 and ldo >= m");
    return SL_ERR_UNSUPPORTED;
  }
  const unsigned grid = sl_grid_for((size_t)(m * k2), 256, 2048);
  k_xm_bf16t<<<grid, 256, 0, (hipStream_t)stream>>>(Y, m, k, ldy, M, k2, (bf16_t*)outT, ldo);
  SL_LAUNCH_CHECK();
  return SL_OK;
}
