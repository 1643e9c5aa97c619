// CountSketch-family kernels (CWT / MMT / WZT): hash_transform_t.
//
// Reference: sketch/hash_transform_Elemental.hpp:83-130 (dense),
// :201-260 (CSC -> dense), sketch/hash_transform_local_sparse.hpp:88-223.
// Columnwise:  SA[h[r], :] += v[r] * A[r, :]     (A: N x m)
// Rowwise:     SA[:, h[c]] += v[c] * A[:, c]     (A: m x N)
//
// gfx950 design.  The sketch data (h, v) is static, so the host builds ONCE
// per sketch a bucket permutation (rows sorted by h; `perm`, `bptr`) and the
// kernels become gathers + segmented reductions instead of scattered float
// atomics into HBM (which run at ~1.3 TB/s at best and ~0.08 TB/s with one
// lane per row, MI355X_MICROARCH.md "Global float atomics"):
//   * dense columnwise: one workgroup per (bucket, 256*VEC column slice);
//     every thread owns VEC output columns in registers and streams the
//     bucket's rows (coalesced 16-B loads) -> deterministic, no atomics;
//   * dense rowwise: the input row is staged in LDS by coalesced loads, each
//     thread produces whole output buckets by gathering from LDS;
//   * CSR columnwise: one workgroup per (bucket, column chunk), the chunk
//     accumulated in LDS with ds_add_f32 / ds_add_f64 (value dtype), then one
//     coalesced store.
#include "sl_common.hpp"
#include <stdlib.h>
#include <type_traits>

// pval[p] = val[perm[p]] (bucket-ordered signs, built once per sketch): the
// bucket's row indices and weights are read coalesced, and the row loads of
// U rows are issued before any of them is consumed (U x fewer dependent
// latency rounds than one row at a time).
template <typename T, typename OT, int VEC, int U>
__global__ void __launch_bounds__(256)
k_hash_dense_col(const T* __restrict__ A, int64_t lda, int64_t m, const int64_t* __restrict__ perm,
                 const int64_t* __restrict__ bptr, const double* __restrict__ pval,
                 OT* __restrict__ out, int64_t ldo, int64_t row_offset, int accumulate) {
  const int64_t b = blockIdx.y;
  const int64_t c0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * VEC;
  float acc[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) acc[j] = 0.f;
  const int64_t p0 = bptr[b], p1 = bptr[b + 1];
  if (c0 < m) {
    const bool full = c0 + VEC <= m;
    int64_t p = p0;
    if (full) {
      for (; p + U <= p1; p += U) {
        float x[U][VEC], w[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const T* row = A + (perm[p + u] - row_offset) * lda + c0;   // wave-uniform row
          w[u] = (float)pval[p + u];
#pragma unroll
          for (int j = 0; j < VEC; ++j) x[u][j] = Cvt<T>::to_f(row[j]);
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int j = 0; j < VEC; ++j) acc[j] += w[u] * x[u][j];
      }
    }
    for (; p < p1; ++p) {
      const T* row = A + (perm[p] - row_offset) * lda + c0;
      const float w = (float)pval[p];
      for (int j = 0; j < VEC && c0 + j < m; ++j) acc[j] += w * Cvt<T>::to_f(row[j]);
    }
    OT* o = out + b * ldo + c0;
    for (int j = 0; j < VEC && c0 + j < m; ++j)
      o[j] = accumulate ? Cvt<OT>::from_f(Cvt<OT>::to_f(o[j]) + acc[j]) : Cvt<OT>::from_f(acc[j]);
  }
}

// double-precision variant: exact fp64 accumulation
template <int VEC>
__global__ void __launch_bounds__(256)
k_hash_dense_col_f64(const double* __restrict__ A, int64_t lda, int64_t m,
                     const int64_t* __restrict__ perm, const int64_t* __restrict__ bptr,
                     const double* __restrict__ val, double* __restrict__ out, int64_t ldo,
                     int64_t row_offset, int accumulate) {
  const int64_t b = blockIdx.y;
  const int64_t c0 = ((int64_t)blockIdx.x * 256 + threadIdx.x) * VEC;
  double acc[VEC];
#pragma unroll
  for (int j = 0; j < VEC; ++j) acc[j] = 0.0;
  const int64_t p0 = bptr[b], p1 = bptr[b + 1];
  if (c0 < m) {
    for (int64_t p = p0; p < p1; ++p) {
      const int64_t r = perm[p];
      const double w = val[p];
      const double* row = A + (r - row_offset) * lda + c0;
      for (int j = 0; j < VEC && c0 + j < m; ++j) acc[j] += w * row[j];
    }
    double* o = out + b * ldo + c0;
    for (int j = 0; j < VEC && c0 + j < m; ++j) o[j] = accumulate ? o[j] + acc[j] : acc[j];
  }
}

SL_API int sl_hash_dense_colwise(const void* A, int dtype, int64_t lda, int64_t m,
                                 const int64_t* perm, const int64_t* bptr, const double* val,
                                 int64_t S, void* out, int out_dtype, int64_t ldo,
                                 int64_t row_offset, int accumulate, void* stream) {
  if (S <= 0 || m <= 0) return SL_OK;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == SL_F64) {
    if (out_dtype != SL_F64) { sl_set_last_error("f64 input needs f64 output"); return SL_ERR_UNSUPPORTED; }
    constexpr int VEC = 2;
    dim3 grid((unsigned)((m + 256 * VEC - 1) / (256 * VEC)), (unsigned)S);
    k_hash_dense_col_f64<VEC><<<grid, 256, 0, s>>>((const double*)A, lda, m, perm, bptr, val,
                                                    (double*)out, ldo, row_offset, accumulate);
    SL_LAUNCH_CHECK();
    return SL_OK;
  }
  constexpr int VEC = 4;
  dim3 grid((unsigned)((m + 256 * VEC - 1) / (256 * VEC)), (unsigned)S);
#define SL_HC(TI, TO) k_hash_dense_col<TI, TO, VEC, 4><<<grid, 256, 0, s>>>((const TI*)A, lda, m, perm, bptr, val, (TO*)out, ldo, row_offset, accumulate)
  if (dtype == SL_F32 && out_dtype == SL_F32) SL_HC(float, float);
  else if (dtype == SL_BF16 && out_dtype == SL_F32) SL_HC(bf16_t, float);
  else if (dtype == SL_BF16 && out_dtype == SL_BF16) SL_HC(bf16_t, bf16_t);
  else if (dtype == SL_F32 && out_dtype == SL_BF16) SL_HC(float, bf16_t);
  else { sl_set_last_error("hash colwise: dtype combination"); return SL_ERR_UNSUPPORTED; }
#undef SL_HC
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// ---------------------------------------------------------------- rowwise
// One workgroup per input row: row -> LDS (coalesced), then thread t produces
// buckets t, t+256, ... by gathering the bucket members from LDS.
template <typename T, typename AT, typename OT>
__global__ void __launch_bounds__(256)
k_hash_dense_row(const T* __restrict__ A, int64_t lda, int64_t ncols, const int64_t* __restrict__ perm,
                 const int64_t* __restrict__ bptr, const double* __restrict__ val, int64_t S,
                 OT* __restrict__ out, int64_t ldo, int64_t col_offset, int accumulate) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  AT* row = (AT*)smem;
  const int64_t r = blockIdx.x;
  const T* a = A + r * lda;
  for (int64_t c = threadIdx.x; c < ncols; c += 256) row[c] = (AT)Cvt<T>::to_d(a[c]);
  __syncthreads();
  for (int64_t b = threadIdx.x; b < S; b += 256) {
    AT acc = 0;
    for (int64_t p = bptr[b]; p < bptr[b + 1]; ++p) {
      const int64_t c = perm[p];
      acc += (AT)val[c] * row[c - col_offset];
    }
    OT* o = out + r * ldo + b;
    if (accumulate) *o = Cvt<OT>::from_d(Cvt<OT>::to_d(*o) + (double)acc);
    else *o = Cvt<OT>::from_d((double)acc);
  }
}

SL_API int sl_hash_dense_rowwise(const void* A, int dtype, int64_t lda, int64_t rows,
                                 int64_t ncols, const int64_t* perm, const int64_t* bptr,
                                 const double* val, int64_t S, void* out, int out_dtype,
                                 int64_t ldo, int64_t col_offset, int accumulate, void* stream) {
  if (rows <= 0 || S <= 0) return SL_OK;
  hipStream_t s = (hipStream_t)stream;
  size_t esz = dtype == SL_F64 ? 8 : 4;
  size_t lds = (size_t)ncols * esz;
  if (lds > 160 * 1024) { sl_set_last_error("hash rowwise: row too long for LDS"); return SL_ERR_UNSUPPORTED; }
  if (dtype == SL_F64 && out_dtype == SL_F64)
    k_hash_dense_row<double, double, double><<<(unsigned)rows, 256, lds, s>>>((const double*)A, lda, ncols, perm, bptr, val, S, (double*)out, ldo, col_offset, accumulate);
  else if (dtype == SL_F32 && out_dtype == SL_F32)
    k_hash_dense_row<float, float, float><<<(unsigned)rows, 256, lds, s>>>((const float*)A, lda, ncols, perm, bptr, val, S, (float*)out, ldo, col_offset, accumulate);
  else if (dtype == SL_BF16 && out_dtype == SL_F32)
    k_hash_dense_row<bf16_t, float, float><<<(unsigned)rows, 256, lds, s>>>((const bf16_t*)A, lda, ncols, perm, bptr, val, S, (float*)out, ldo, col_offset, accumulate);
  else if (dtype == SL_BF16 && out_dtype == SL_BF16)
    k_hash_dense_row<bf16_t, float, bf16_t><<<(unsigned)rows, 256, lds, s>>>((const bf16_t*)A, lda, ncols, perm, bptr, val, S, (bf16_t*)out, ldo, col_offset, accumulate);
  else { sl_set_last_error("hash rowwise: dtype combination"); return SL_ERR_UNSUPPORTED; }
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// ------------------------------------------------------------ CSR columnwise
// A: CSR (rowptr, col, vals) holding global rows [row_offset, row_offset+nrows).
// Workgroup = (bucket b, column chunk [c0, c0+CW)); lanes are split in groups
// of G lanes per CSR row (G ~ average row length, a power of two), and each
// group keeps U rows in flight (their perm / rowptr loads issued together).
// The workgroup owns its output cells: plain stores, no zero-fill.
//
// DET (deterministic mode): the chunk is accumulated in int64 fixed point
// (ds_add_u64 is associative, so the result does not depend on the order the
// lanes arrive in) with the per-bucket scale 2^62 / (R_b * max|v| * max|w|):
// one row contributes at most one entry to a column, so no cell can overflow,
// and the quantum is 2^-62 of that bound (~2^-50 relative for 4k-row
// buckets, finer than f32 and close to f64 rounding).
template <typename IT, typename VT, int G, int U, bool DET>
__global__ void __launch_bounds__(512)
k_hash_csr_col(const int64_t* __restrict__ rowptr, const IT* __restrict__ col,
               const VT* __restrict__ vals, const int64_t* __restrict__ perm,
               const int64_t* __restrict__ bptr, const VT* __restrict__ pval,
               VT* __restrict__ out, int64_t ldo, int64_t m, int64_t CW,
               int64_t row_offset, const double* __restrict__ vmax, double wmax) {
  typedef typename std::conditional<DET, unsigned long long, VT>::type AT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  AT* acc = (AT*)smem;
  const int64_t b = blockIdx.y;
  const int64_t c0 = (int64_t)blockIdx.x * CW;
  const int64_t cw = (c0 + CW <= m) ? CW : (m - c0);
  for (int64_t c = threadIdx.x; c < cw; c += blockDim.x) acc[c] = (AT)0;
  __syncthreads();
  const int groups = blockDim.x / G;
  const int gid = threadIdx.x / G, gl = threadIdx.x % G;
  const bool chunked = cw != m;
  const int64_t p0 = bptr[b], p1 = bptr[b + 1];
  double sc = 0.0;
  if (DET) {
    const double bound = (double)(p1 - p0) * vmax[0] * wmax;
    sc = bound > 0.0 ? 0x1p62 / bound : 0.0;
  }
  for (int64_t p = p0 + gid; p < p1; p += (int64_t)groups * U) {
    int64_t rs[U], re[U];
    VT w[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t pp = p + (int64_t)u * groups;
      rs[u] = re[u] = 0;
      w[u] = (VT)0;
      if (pp < p1) {
        const int64_t lr = perm[pp] - row_offset;
        w[u] = pval[pp];
        rs[u] = rowptr[lr];
        re[u] = rowptr[lr + 1];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      for (int64_t q = rs[u] + gl; q < re[u]; q += G) {
        const int64_t c = (int64_t)col[q] - c0;
        if (!chunked || (c >= 0 && c < cw)) {
          if (DET) atomicAdd(&acc[c], (unsigned long long)__double2ll_rn((double)(w[u] * vals[q]) * sc));
          else atomicAdd(&acc[c], w[u] * vals[q]);
        }
      }
    }
  }
  __syncthreads();
  for (int64_t c = threadIdx.x; c < cw; c += blockDim.x) {
    if (DET) out[b * ldo + c0 + c] = sc > 0.0 ? (VT)((double)(long long)acc[c] / sc) : (VT)0;
    else out[b * ldo + c0 + c] = (VT)acc[c];
  }
}

SL_API int sl_hash_csr_colwise2(const int64_t* rowptr, const void* col, int idx32, const void* vals,
                                int vdtype, const int64_t* perm, const int64_t* bptr,
                                const void* pval, int64_t S, int64_t m, void* out, int64_t ldo,
                                int64_t row_offset, int group, int deterministic, const double* vmax,
                                double wmax, void* stream) {
  if (S <= 0 || m <= 0) return SL_OK;
  hipStream_t s = (hipStream_t)stream;
  const int64_t esz = (vdtype == SL_F64 || deterministic) ? 8 : 4;
  const int64_t cwmax = (128 * 1024) / esz;  // 128 KB of LDS at most
  int64_t CW = m < cwmax ? m : cwmax;
  dim3 grid((unsigned)((m + CW - 1) / CW), (unsigned)S);
  size_t lds = (size_t)CW * esz;
#define SL_CSR_U(IT, VT, G, DET, U) k_hash_csr_col<IT, VT, G, U, DET><<<grid, 512, lds, s>>>(rowptr, (const IT*)col, (const VT*)vals, perm, bptr, (const VT*)pval, (VT*)out, ldo, m, CW, row_offset, vmax, wmax)
#define SL_CSR(IT, VT, G, DET) SL_CSR_U(IT, VT, G, DET, 8)   /* 8 rows in flight per lane group */
#define SL_CSR_G(IT, VT, DET)                              \
  switch (group) {                                         \
    case 1: SL_CSR(IT, VT, 1, DET); break;                 \
    case 4: SL_CSR(IT, VT, 4, DET); break;                 \
    case 16: SL_CSR(IT, VT, 16, DET); break;               \
    default: SL_CSR(IT, VT, 64, DET); break;               \
  }
#define SL_CSR_D(IT, VT) if (deterministic) { SL_CSR_G(IT, VT, true) } else { SL_CSR_G(IT, VT, false) }
  if (vdtype == SL_F32) {
    if (idx32) { SL_CSR_D(int32_t, float) } else { SL_CSR_D(int64_t, float) }
  } else if (vdtype == SL_F64) {
    if (idx32) { SL_CSR_D(int32_t, double) } else { SL_CSR_D(int64_t, double) }
  } else { sl_set_last_error("hash csr: value dtype"); return SL_ERR_UNSUPPORTED; }
#undef SL_CSR_D
#undef SL_CSR_G
#undef SL_CSR
#undef SL_CSR_U
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// ------------------------------------------------------------- CSR rowwise
// out[r, h[c]] += v[c] * A[r, c]: G lanes per CSR row, f32/f64 atomics into the
// row of `out` (rows are disjoint between groups, so contention is per row).
// G = 1: the lane owns its output row and adds in CSR order with plain
// read-modify-writes -- no atomics, deterministic (short rows, and the
// deterministic mode).
template <typename IT, typename VT, int G>
__global__ void __launch_bounds__(256)
k_hash_csr_row(const int64_t* __restrict__ rowptr, const IT* __restrict__ col,
               const VT* __restrict__ vals, int64_t rows, const int64_t* __restrict__ h,
               const double* __restrict__ hval, VT* __restrict__ out, int64_t ldo,
               int64_t col_offset) {
  const int64_t gid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / G;
  const int gl = threadIdx.x % G;
  if (gid >= rows) return;
  for (int64_t q = rowptr[gid] + gl; q < rowptr[gid + 1]; q += G) {
    const int64_t c = (int64_t)col[q] + col_offset;
    if (G == 1) out[gid * ldo + h[c]] += (VT)hval[c] * vals[q];
    else atomicAdd(&out[gid * ldo + h[c]], (VT)hval[c] * vals[q]);
  }
}

SL_API int sl_hash_csr_rowwise(const int64_t* rowptr, const void* col, int idx32, const void* vals,
                               int vdtype, int64_t rows, const int64_t* h, const double* hval,
                               void* out, int64_t ldo, int64_t col_offset, int group,
                               void* stream) {
  if (rows <= 0) return SL_OK;
  hipStream_t s = (hipStream_t)stream;
#define SL_CR(IT, VT, G) k_hash_csr_row<IT, VT, G><<<(unsigned)((rows * G + 255) / 256), 256, 0, s>>>(rowptr, (const IT*)col, (const VT*)vals, rows, h, hval, (VT*)out, ldo, col_offset)
#define SL_CR_G(IT, VT)                                   \
  switch (group) {                                        \
    case 1: SL_CR(IT, VT, 1); break;                      \
    case 4: SL_CR(IT, VT, 4); break;                      \
    case 16: SL_CR(IT, VT, 16); break;                    \
    default: SL_CR(IT, VT, 64); break;                    \
  }
  if (vdtype == SL_F32) {
    if (idx32) { SL_CR_G(int32_t, float) } else { SL_CR_G(int64_t, float) }
  } else if (vdtype == SL_F64) {
    if (idx32) { SL_CR_G(int32_t, double) } else { SL_CR_G(int64_t, double) }
  } else { sl_set_last_error("hash csr rowwise: value dtype"); return SL_ERR_UNSUPPORTED; }
#undef SL_CR_G
#undef SL_CR
  SL_LAUNCH_CHECK();
  return SL_OK;
}
