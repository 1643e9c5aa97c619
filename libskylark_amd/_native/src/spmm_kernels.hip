// CSR sparse x thin dense products (Krylov / randSVD operators on sparse A).
//
// Reference: base/Gemm.hpp:212-494 and base/Symm.hpp:86-158 (sparse x dense
// GEMM over Elemental / CombBLAS), used by LSQR / CG / ApproximateSVD on
// sparse inputs.  Y = A X with A m x n CSR and X n x k (k <= 64, row-major):
// G lanes per CSR row (G ~ average row length, a power of two), each lane
// walks its share of the row's nonzeros and gathers the K-wide rows of X
// (L2-resident for the thin blocks the solvers use), the G partial sums are
// combined with xor shuffles inside the group, and the group's lanes store
// the K results of the row.  Column blocks of 16 go through one launch each.
// A^T X runs the same kernel on the CSR of A^T (built once per operator).
#include "sl_common.hpp"

namespace {

constexpr int NT = 256;

template <typename IT, typename VT, int G, int K>
__global__ void __launch_bounds__(NT) k_csr_spmm(const int64_t* __restrict__ rowptr, const IT* __restrict__ col,
                                                 const VT* __restrict__ vals, int64_t nrows,
                                                 const VT* __restrict__ X, int64_t ldx, VT* __restrict__ Y,
                                                 int64_t ldy, int kk) {
  const int64_t gtid = (int64_t)blockIdx.x * NT + threadIdx.x;
  const int gl = threadIdx.x % G;
  const int64_t ngroups = (int64_t)gridDim.x * (NT / G);
  for (int64_t row = gtid / G; row < nrows; row += ngroups) {
    VT acc[K];
#pragma unroll
    for (int j = 0; j < K; ++j) acc[j] = (VT)0;
    const int64_t q1 = rowptr[row + 1];
    for (int64_t q = rowptr[row] + gl; q < q1; q += G) {
      const int64_t c = (int64_t)col[q];
      const VT v = vals[q];
      const VT* xr = X + c * ldx;
#pragma unroll
      for (int j = 0; j < K; ++j)
        if (j < kk) acc[j] += v * xr[j];
    }
#pragma unroll
    for (int j = 0; j < K; ++j) {
#pragma unroll
      for (int off = G / 2; off >= 1; off >>= 1) acc[j] += __shfl_xor(acc[j], off, G);
    }
    // lane gl stores columns gl, gl + G, ...
#pragma unroll
    for (int j = 0; j < K; ++j)
      if (j % G == gl && j < kk) Y[row * ldy + j] = acc[j];
  }
}

}  // namespace

// Y (nrows x k) = A X for CSR A (int64 rowptr, int32/int64 col, f32/f64 values).
SL_API int sl_csr_spmm(const int64_t* rowptr, const void* col, int idx32, const void* vals, int vdtype, int64_t nrows,
                       const void* X, int64_t ldx, int k, void* Y, int64_t ldy, int group, void* stream) {
  if (nrows <= 0 || k <= 0) return SL_OK;
  if (vdtype != SL_F32 && vdtype != SL_F64) { sl_set_last_error("csr_spmm: f32/f64 values"); return SL_ERR_UNSUPPORTED; }
  hipStream_t s = (hipStream_t)stream;
  const int G = group >= 64 ? 64 : group >= 16 ? 16 : group >= 4 ? 4 : 1;
  int64_t blocks = (nrows * G + NT - 1) / NT;
  if (blocks > 65536) blocks = 65536;
  const size_t esz = vdtype == SL_F64 ? 8 : 4;
  for (int c0 = 0; c0 < k; c0 += 16) {
    const int kk = k - c0 < 16 ? k - c0 : 16;
    const char* Xc = (const char*)X + (size_t)c0 * esz;
    char* Yc = (char*)Y + (size_t)c0 * esz;
#define SL_SP(IT, VT, GG, KK) k_csr_spmm<IT, VT, GG, KK><<<(unsigned)blocks, NT, 0, s>>>(rowptr, (const IT*)col, (const VT*)vals, nrows, (const VT*)Xc, ldx, (VT*)Yc, ldy, kk)
#define SL_SP_K(IT, VT, GG) \
    if (kk <= 1) SL_SP(IT, VT, GG, 1); else if (kk <= 2) SL_SP(IT, VT, GG, 2); else if (kk <= 4) SL_SP(IT, VT, GG, 4); \
    else if (kk <= 8) SL_SP(IT, VT, GG, 8); else SL_SP(IT, VT, GG, 16);
#define SL_SP_G(IT, VT) \
    switch (G) { case 1: { SL_SP_K(IT, VT, 1) } break; case 4: { SL_SP_K(IT, VT, 4) } break; \
                 case 16: { SL_SP_K(IT, VT, 16) } break; default: { SL_SP_K(IT, VT, 64) } }
    if (vdtype == SL_F32) {
      if (idx32) { SL_SP_G(int32_t, float) } else { SL_SP_G(int64_t, float) }
    } else {
      if (idx32) { SL_SP_G(int32_t, double) } else { SL_SP_G(int64_t, double) }
    }
#undef SL_SP_G
#undef SL_SP_K
#undef SL_SP
  }
  SL_LAUNCH_CHECK();
  return SL_OK;
}
