// Dense sketch of a CSR operand (reference sketch/dense_transform_Mixed.hpp:
// 19-101, the sparse-input branch of dense_transform_t): Y = A S^T for the
// S x N random matrix S realised lazily, panel by panel of its N columns.
//
// A panel P holds the realised sketch columns [c0, c1) as rows (P[c - c0][:]
// = S[:, c], so each is one contiguous, stream-ordered run of S samples --
// base + c S + i, the reference's column-major realisation) and stays
// L2 / Infinity-Cache resident while this kernel consumes it.  Mapping: one
// group of LPR lanes per CSR row; lane l of the group owns output columns
// l, l + LPR, ... (U of them, in registers); the group walks the row's
// nonzeros that fall in [c0, c1) (sorted column indices: one binary search
// for the first), and every nonzero is one coalesced LPR-wide sweep over the
// panel row of its column.  Four nonzeros are in flight per step.  The row's
// result is stored once per panel (or added to the previous panels' sum).
//
// Rowwise sketch (A S^T, A m x N): this kernel on A.  Columnwise (S A,
// A N x m): this kernel on the CSR of A^T, then one transpose of the small
// m x S result.
#include "sl_common.hpp"

namespace {

constexpr int NT = 256;

template <typename T, typename IT, int LPR, int U>
__global__ void __launch_bounds__(NT)
k_csr_panel(const int64_t* __restrict__ rowptr, const IT* __restrict__ col, const T* __restrict__ vals,
            int64_t nrows, int64_t c0, int64_t c1, int restrict_cols, const T* __restrict__ P, int64_t ldp, int S,
            T* __restrict__ Y, int64_t ldy, int accumulate) {
  const int gl = threadIdx.x % LPR;
  const int64_t ngroups = (int64_t)gridDim.x * (NT / LPR);
  for (int64_t row = ((int64_t)blockIdx.x * NT + threadIdx.x) / LPR; row < nrows; row += ngroups) {
    int64_t q = rowptr[row];
    const int64_t q1 = rowptr[row + 1];
    if (restrict_cols) {
      // first nonzero with col >= c0
      int64_t lo = q, hi = q1;
      while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if ((int64_t)col[mid] < c0) lo = mid + 1; else hi = mid;
      }
      q = lo;
    }
    T acc[U];
#pragma unroll
    for (int u = 0; u < U; ++u) acc[u] = (T)0;
    bool done = false;
    for (; q + 4 <= q1 && !done; q += 4) {
      int64_t c[4];
      T v[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        c[e] = (int64_t)col[q + e];
        v[e] = vals[q + e];
      }
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (c[e] >= c1) { v[e] = (T)0; c[e] = c0; done = true; }
      // every panel load issued unconditionally (clamped column, then zeroed):
      // `j < S ? pr[j] : 0` compiled to one exec-masked branch per load, each
      // waiting for its own load (same-box A/B: rowwise 10.5 -> 10.15 ms,
      // profiles/r6/csr_panel_loads_ab.jsonl; eight nonzeros per step with a
      // masked tail measured slower, 11.6 ms -- the panel gathers, ~1 KB per
      // nonzero from the Infinity Cache, are the bound, not load latency)
      T p[4][U];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const T* pr = P + (c[e] - c0) * ldp;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int j = gl + LPR * u;
          p[e][u] = pr[j < S ? j : 0];
        }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int u = 0; u < U; ++u) asm volatile("" : "+v"(p[e][u]));
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int u = 0; u < U; ++u)
          if (gl + LPR * u >= S) p[e][u] = (T)0;
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int u = 0; u < U; ++u) acc[u] += v[e] * p[e][u];
    }
    for (; q < q1 && !done; ++q) {
      const int64_t c = (int64_t)col[q];
      if (c >= c1) break;
      const T v = vals[q];
      const T* pr = P + (c - c0) * ldp;
      T p1[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int j = gl + LPR * u;
        p1[u] = pr[j < S ? j : 0];
      }
#pragma unroll
      for (int u = 0; u < U; ++u) asm volatile("" : "+v"(p1[u]));
#pragma unroll
      for (int u = 0; u < U; ++u)
        if (gl + LPR * u < S) acc[u] += v * p1[u];
    }
    T* yr = Y + row * ldy;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int j = gl + LPR * u;
      if (j < S) yr[j] = accumulate ? yr[j] + acc[u] : acc[u];
    }
  }
}

template <typename T, typename IT>
int launch(const int64_t* rowptr, const void* col, const void* vals, int64_t nrows, int64_t c0, int64_t c1,
           int restrict_cols, const void* P, int64_t ldp, int S, void* Y, int64_t ldy, int accumulate,
           hipStream_t s) {
  // lanes per row: the narrowest group whose 8 register columns cover S
  const int LPR = S > 256 ? 64 : S > 128 ? 64 : S > 64 ? 32 : S > 32 ? 16 : 8;
  int64_t blocks = (nrows * LPR + NT - 1) / NT;
  if (blocks > 131072) blocks = 131072;
  const IT* ci = (const IT*)col;
  const T* v = (const T*)vals;
  const T* p = (const T*)P;
  T* y = (T*)Y;
#define SL_CP(L, UU) \
  k_csr_panel<T, IT, L, UU><<<(unsigned)blocks, NT, 0, s>>>(rowptr, ci, v, nrows, c0, c1, restrict_cols, p, ldp, S, y, \
                                                            ldy, accumulate)
  if (S > 256) SL_CP(64, 8);
  else if (S > 128) SL_CP(64, 4);
  else if (LPR == 32) SL_CP(32, 4);
  else if (LPR == 16) SL_CP(16, 4);
  else SL_CP(8, 4);
#undef SL_CP
  SL_LAUNCH_CHECK();
  return SL_OK;
}

}  // namespace

// Y (nrows x S, ldy) (+)= A[:, c0:c1) P with A CSR (int64 rowptr, sorted
// int32 / int64 column indices, f32 / f64 values) and P the (c1 - c0) x S
// realised panel (row stride ldp, values dtype).  restrict_cols = 0 asserts
// every column index of A lies in [c0, c1) (one panel covers A).  S <= 512.
SL_API int sl_csr_sketch_panel(const int64_t* rowptr, const void* col, int idx32, const void* vals, int vdtype,
                               int64_t nrows, int64_t c0, int64_t c1, int restrict_cols, const void* P, int64_t ldp,
                               int S, void* Y, int64_t ldy, int accumulate, void* stream) {
  if (nrows <= 0) return SL_OK;
  if (S < 1 || S > 512 || ldp < S || ldy < S || c1 <= c0) {
    sl_set_last_error("csr_sketch_panel: needs 1 <= S <= 512, ldp >= S, ldy >= S, c1 > c0");
    return SL_ERR_INVALID;
  }
  hipStream_t s = (hipStream_t)stream;
  if (vdtype == SL_F32) {
    return idx32 ? launch<float, int32_t>(rowptr, col, vals, nrows, c0, c1, restrict_cols, P, ldp, S, Y, ldy,
                                          accumulate, s)
                 : launch<float, int64_t>(rowptr, col, vals, nrows, c0, c1, restrict_cols, P, ldp, S, Y, ldy,
                                          accumulate, s);
  }
  if (vdtype == SL_F64) {
    return idx32 ? launch<double, int32_t>(rowptr, col, vals, nrows, c0, c1, restrict_cols, P, ldp, S, Y, ldy,
                                           accumulate, s)
                 : launch<double, int64_t>(rowptr, col, vals, nrows, c0, c1, restrict_cols, P, ldp, S, Y, ldy,
                                           accumulate, s);
  }
  sl_set_last_error("csr_sketch_panel: f32 / f64 values");
  return SL_ERR_UNSUPPORTED;
}
