// CountSketch (CWT / MMT / WZT) of a CSR matrix into a CSR result.
//
// Reference: sketch/hash_transform_local_sparse.hpp:88-223 (CSC -> CSC: every
// (bucket, column) pair the hashing touches becomes one output entry, the
// duplicates summed).  The generic tensor route (COO -> coalesce sort of all
// nnz -> CSR) costs two global radix sorts of the nnz (35-40 ms for 1e8 nnz on
// MI355X); these kernels avoid any global sort:
//
//   * rowwise (out = A S^T, nrows x S): the duplicates of an output row come
//     only from the same input row, so one THREAD owns one CSR row: its
//     (bucket, value) pairs go to registers, a compile-time bitonic network
//     of L = 8/16/32 elements sorts them by bucket (all indices static -> no
//     scratch), equal buckets are summed.  Pass 0 writes the per-row output
//     counts, an exclusive scan gives crow, pass 1 recomputes and stores.
//   * columnwise (out = S A, S x ncols): duplicates come from all rows of a
//     bucket, so the result is accumulated densely (the bucketed LDS kernel
//     of hash_kernels.hip, no global atomics), touched cells are marked in a
//     byte map (explicit / cancelled zeros stay entries, as in the
//     reference), and one wave per output row compacts its row with
//     ballot + mbcnt prefix counts (count pass, scan, fill pass).
#include "sl_common.hpp"

namespace {

template <typename IT, typename VT, typename OT, int L, bool FILL>
__global__ void __launch_bounds__(256)
k_cwt_rw_sparse(const int64_t* __restrict__ rowptr, const IT* __restrict__ col, const VT* __restrict__ vals,
                int64_t nrows, const int64_t* __restrict__ h, const double* __restrict__ hval,
                int64_t col_offset, int64_t* __restrict__ cnt_or_crow, int64_t* __restrict__ ocol,
                OT* __restrict__ oval) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (r >= nrows) return;
  const int64_t p0 = rowptr[r];
  const int n = (int)(rowptr[r + 1] - p0);
  uint32_t key[L];
  OT v[L];
#pragma unroll
  for (int j = 0; j < L; ++j) {
    key[j] = 0xFFFFFFFFu;
    v[j] = (OT)0;
  }
  if (n > 0) {
    // every load of the row issued unconditionally (entries past n re-read
    // entry n - 1) and pinned by an empty asm, then masked: per-entry
    // conditional loads compiled to exec-masked branches, each with its own
    // vmcnt(0), so the dependent col -> h / hval gathers ran one at a time
    int64_t cj[L];
    VT vj[L];
#pragma unroll
    for (int j = 0; j < L; ++j) {
      const int64_t q = p0 + (j < n ? j : n - 1);
      cj[j] = (int64_t)col[q] + col_offset;
      vj[j] = vals[q];
    }
#pragma unroll
    for (int j = 0; j < L; ++j) asm volatile("" : "+v"(cj[j]), "+v"(vj[j]));
    int64_t hj[L];
    double hv[L];
#pragma unroll
    for (int j = 0; j < L; ++j) {
      hj[j] = h[cj[j]];
      hv[j] = hval[cj[j]];
    }
#pragma unroll
    for (int j = 0; j < L; ++j) {
      asm volatile("" : "+v"(hj[j]), "+v"(hv[j]));
      if (j < n) {
        key[j] = (uint32_t)hj[j];
        v[j] = (OT)vj[j] * (OT)hv[j];
      }
    }
  }
#pragma unroll
  for (int k = 2; k <= L; k <<= 1) {
#pragma unroll
    for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
      for (int i = 0; i < L; ++i) {
        const int l = i ^ j;
        if (l > i) {
          const bool up = (i & k) == 0;
          const bool sw = up ? (key[i] > key[l]) : (key[i] < key[l]);
          const uint32_t ka = key[i], kb = key[l];
          const OT va = v[i], vb = v[l];
          key[i] = sw ? kb : ka;
          key[l] = sw ? ka : kb;
          v[i] = sw ? vb : va;
          v[l] = sw ? va : vb;
        }
      }
    }
  }
  if (!FILL) {
    int64_t cnt = 0;
#pragma unroll
    for (int i = 0; i < L; ++i)
      cnt += (key[i] != 0xFFFFFFFFu) && (i == 0 || key[i] != key[i - 1]);
    cnt_or_crow[r] = cnt;
    return;
  }
  int64_t pos = cnt_or_crow[r];
  OT acc = v[0];
  uint32_t ck = key[0];
#pragma unroll
  for (int i = 1; i < L; ++i) {
    if (key[i] != 0xFFFFFFFFu) {
      if (key[i] == ck) {
        acc += v[i];
      } else {
        ocol[pos] = ck;
        oval[pos] = acc;
        ++pos;
        ck = key[i];
        acc = v[i];
      }
    }
  }
  if (n > 0) {
    ocol[pos] = ck;
    oval[pos] = acc;
  }
}

// touched-cell map of the columnwise result: occ[h[r] * ncols + c] = 1
template <typename IT>
__global__ void __launch_bounds__(256)
k_cwt_col_mark(const int64_t* __restrict__ rowptr, const IT* __restrict__ col, int64_t nrows,
               const int64_t* __restrict__ h, int64_t row_offset, uint8_t* __restrict__ occ, int64_t ncols) {
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < nrows; r += (int64_t)gridDim.x * 256) {
    uint8_t* o = occ + h[r + row_offset] * ncols;
    for (int64_t q = rowptr[r]; q < rowptr[r + 1]; ++q) o[col[q]] = 1;
  }
}

__device__ __forceinline__ int lanes_below(uint64_t mask) {
  return __builtin_amdgcn_mbcnt_hi((uint32_t)(mask >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mask, 0));
}

// one wave per dense row: count (FILL = false) or compact (FILL = true)
template <typename DT, typename OT, bool FILL>
__global__ void __launch_bounds__(256)
k_dense_compact(const DT* __restrict__ dense, int64_t ldd, const uint8_t* __restrict__ occ, int64_t rows,
                int64_t cols, int64_t* __restrict__ cnt_or_crow, int64_t* __restrict__ ocol, OT* __restrict__ oval) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const uint8_t* o = occ + row * cols;
  int64_t pos = FILL ? cnt_or_crow[row] : 0;
  for (int64_t base = 0; base < cols; base += 64) {
    const int64_t c = base + lane;
    const bool on = c < cols && o[c] != 0;
    const uint64_t mask = __ballot(on);
    if (FILL && on) {
      const int64_t q = pos + lanes_below(mask);
      ocol[q] = c;
      oval[q] = (OT)dense[row * ldd + c];
    }
    pos += __popcll(mask);
  }
  if (!FILL && lane == 0) cnt_or_crow[row] = pos;
}

}  // namespace

// Rowwise CSR -> CSR.  pass 0: cnt[r] = distinct buckets of row r; pass 1:
// crow (exclusive scan of cnt, length nrows + 1) given, writes ocol / oval.
// maxlen = longest row (<= 32); values f32 (-> f32) or f64 (-> f64).
SL_API int sl_cwt_csr_rowwise_sparse(const int64_t* rowptr, const void* col, int idx32, const void* vals,
                                     int vdtype, int64_t nrows, int maxlen, const int64_t* h, const double* hval,
                                     int64_t col_offset, int pass, int64_t* cnt_or_crow, int64_t* ocol,
                                     void* oval, void* stream) {
  if (nrows <= 0) return SL_OK;
  if (maxlen > 32) {
    sl_set_last_error("cwt rowwise sparse: rows longer than 32 entries");
    return SL_ERR_UNSUPPORTED;
  }
  hipStream_t s = (hipStream_t)stream;
  const unsigned grid = (unsigned)((nrows + 255) / 256);
#define SL_RW(IT, VT, OT, L)                                                                                      \
  do {                                                                                                             \
    if (pass == 0)                                                                                                 \
      k_cwt_rw_sparse<IT, VT, OT, L, false><<<grid, 256, 0, s>>>(rowptr, (const IT*)col, (const VT*)vals, nrows, \
                                                                 h, hval, col_offset, cnt_or_crow, ocol,          \
                                                                 (OT*)oval);                                      \
    else                                                                                                           \
      k_cwt_rw_sparse<IT, VT, OT, L, true><<<grid, 256, 0, s>>>(rowptr, (const IT*)col, (const VT*)vals, nrows,  \
                                                                h, hval, col_offset, cnt_or_crow, ocol,           \
                                                                (OT*)oval);                                       \
  } while (0)
#define SL_RW_L(IT, VT, OT)              \
  if (maxlen <= 8) SL_RW(IT, VT, OT, 8); \
  else if (maxlen <= 16) SL_RW(IT, VT, OT, 16); \
  else SL_RW(IT, VT, OT, 32);
  if (vdtype == SL_F32) {
    if (idx32) { SL_RW_L(int32_t, float, float) } else { SL_RW_L(int64_t, float, float) }
  } else if (vdtype == SL_F64) {
    if (idx32) { SL_RW_L(int32_t, double, double) } else { SL_RW_L(int64_t, double, double) }
  } else {
    sl_set_last_error("cwt rowwise sparse: value dtype");
    return SL_ERR_UNSUPPORTED;
  }
#undef SL_RW_L
#undef SL_RW
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// occ[h[r + row_offset] * ncols + col] = 1 for every stored entry of the CSR rows.
SL_API int sl_cwt_csr_colwise_mark(const int64_t* rowptr, const void* col, int idx32, int64_t nrows,
                                   const int64_t* h, int64_t row_offset, uint8_t* occ, int64_t ncols, void* stream) {
  if (nrows <= 0) return SL_OK;
  hipStream_t s = (hipStream_t)stream;
  int64_t blocks = (nrows + 255) / 256;
  if (blocks > 65536) blocks = 65536;
  if (idx32)
    k_cwt_col_mark<int32_t><<<(unsigned)blocks, 256, 0, s>>>(rowptr, (const int32_t*)col, nrows, h, row_offset, occ,
                                                             ncols);
  else
    k_cwt_col_mark<int64_t><<<(unsigned)blocks, 256, 0, s>>>(rowptr, (const int64_t*)col, nrows, h, row_offset, occ,
                                                             ncols);
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// Dense (rows x cols, f32 or f64, leading dim ldd) + byte map -> CSR.  pass 0
// writes per-row counts; pass 1 takes crow and writes ocol / oval (odtype).
SL_API int sl_dense_occ_compact(const void* dense, int ddtype, int64_t ldd, const uint8_t* occ, int64_t rows,
                                int64_t cols, int pass, int64_t* cnt_or_crow, int64_t* ocol, void* oval, int odtype,
                                void* stream) {
  if (rows <= 0) return SL_OK;
  hipStream_t s = (hipStream_t)stream;
  const unsigned grid = (unsigned)((rows + 3) / 4);
#define SL_DC(DT, OT)                                                                                     \
  do {                                                                                                    \
    if (pass == 0)                                                                                        \
      k_dense_compact<DT, OT, false><<<grid, 256, 0, s>>>((const DT*)dense, ldd, occ, rows, cols, cnt_or_crow, \
                                                           ocol, (OT*)oval);                              \
    else                                                                                                  \
      k_dense_compact<DT, OT, true><<<grid, 256, 0, s>>>((const DT*)dense, ldd, occ, rows, cols, cnt_or_crow,  \
                                                          ocol, (OT*)oval);                               \
  } while (0)
  if (ddtype == SL_F32 && odtype == SL_F32) SL_DC(float, float);
  else if (ddtype == SL_F32 && odtype == SL_F64) SL_DC(float, double);
  else if (ddtype == SL_F64 && odtype == SL_F64) SL_DC(double, double);
  else {
    sl_set_last_error("dense_occ_compact: dtype pair");
    return SL_ERR_UNSUPPORTED;
  }
#undef SL_DC
  SL_LAUNCH_CHECK();
  return SL_OK;
}
