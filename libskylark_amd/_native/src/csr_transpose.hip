// CSR transpose on the device (the CSC of A as the CSR of A^T): the operand
// layout change in front of every columnwise sparse sketch / A^T X product
// (reference: the CombBLAS / Elemental transposes behind
// sketch/dense_transform_Mixed.hpp and base/Gemm.hpp's sparse branches).
//
// One stable LSD radix sort of (column, nonzero position) pairs over only the
// bits the column count needs (hipCUB / rocPRIM onesweep; 14 bits for 1e4
// columns = two digit passes), then one gather of the row indices and values
// through the sorted positions, and the column pointers by a binary search of
// the sorted keys per column.  Stability keeps the row indices ascending
// within every column.  torch's COO coalesce route sorts 64-bit linear keys
// (~41 ms at 1e8 nonzeros).
#include <hipcub/hipcub.hpp>

#include "sl_common.hpp"

namespace {

constexpr int NT = 256;

// one wave per row (lanes stride its nonzeros): coalesced for long and short rows
template <typename IT>
__global__ void __launch_bounds__(NT)
k_expand(const int64_t* __restrict__ rowptr, const IT* __restrict__ col, int64_t nrows, int* __restrict__ key,
         int* __restrict__ pos, int* __restrict__ row_of) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * (NT / 64);
  for (int64_t r = (int64_t)blockIdx.x * (NT / 64) + (threadIdx.x >> 6); r < nrows; r += nw) {
    const int64_t q1 = rowptr[r + 1];
    for (int64_t q = rowptr[r] + lane; q < q1; q += 64) {
      key[q] = (int)col[q];
      pos[q] = (int)q;
      row_of[q] = (int)r;
    }
  }
}

template <typename VT>
__global__ void __launch_bounds__(NT)
k_gather(const int* __restrict__ spos, const int* __restrict__ row_of, const VT* __restrict__ vals, int64_t nnz,
         int* __restrict__ orow, VT* __restrict__ oval) {
  const int64_t t = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (t >= nnz) return;
  const int p = spos[t];
  orow[t] = row_of[p];
  oval[t] = vals[p];
}

// colptr[c] = first sorted position with key >= c, c in [0, ncols]
__global__ void __launch_bounds__(NT)
k_colptr(const int* __restrict__ skey, int64_t nnz, int64_t ncols, int64_t* __restrict__ colptr) {
  const int64_t c = (int64_t)blockIdx.x * NT + threadIdx.x;
  if (c > ncols) return;
  int64_t lo = 0, hi = nnz;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if ((int64_t)skey[mid] < c) lo = mid + 1; else hi = mid;
  }
  colptr[c] = lo;
}

int bits_for(int64_t n) {
  int b = 1;
  while ((int64_t(1) << b) < n) ++b;
  return b;
}

}  // namespace

// Workspace bytes for sl_csr_transpose (nnz < 2^31, ncols < 2^31).
SL_API int64_t sl_csr_transpose_workspace(int64_t nnz, int64_t ncols) {
  size_t tmp = 0;
  if (hipcub::DeviceRadixSort::SortPairs(nullptr, tmp, (int*)nullptr, (int*)nullptr, (int*)nullptr, (int*)nullptr,
                                         (int)nnz, 0, bits_for(ncols + 1)) != hipSuccess)
    return -1;
  return (int64_t)(5 * ((nnz * 4 + 255) & ~int64_t(255))) + (int64_t)tmp + 256;
}

// A (nrows x ncols CSR: int64 rowptr, int32 / int64 col, f32 / f64 vals) ->
// A^T (ncols x nrows CSR: int64 colptr (ncols + 1), int32 row indices, vals).
SL_API int sl_csr_transpose(const int64_t* rowptr, const void* col, int idx32, const void* vals, int vdtype,
                            int64_t nrows, int64_t ncols, int64_t nnz, int64_t* colptr, int* orow, void* oval,
                            void* ws, int64_t ws_bytes, void* stream) {
  if (nnz < 0 || nnz >= (int64_t(1) << 31) || nrows >= (int64_t(1) << 31) || ncols >= (int64_t(1) << 31)) {
    sl_set_last_error("csr_transpose: needs nnz, nrows, ncols < 2^31");
    return SL_ERR_UNSUPPORTED;
  }
  if (vdtype != SL_F32 && vdtype != SL_F64) { sl_set_last_error("csr_transpose: f32 / f64 values"); return SL_ERR_UNSUPPORTED; }
  hipStream_t s = (hipStream_t)stream;
  const int64_t seg = (nnz * 4 + 255) & ~int64_t(255);
  char* base = (char*)(((uintptr_t)ws + 255) & ~(uintptr_t)255);
  int* key = (int*)base;
  int* key2 = (int*)(base + seg);
  int* pos = (int*)(base + 2 * seg);
  int* pos2 = (int*)(base + 3 * seg);
  int* row_of = (int*)(base + 4 * seg);
  void* tmp = base + 5 * seg;
  size_t tmp_bytes = (size_t)(ws_bytes - 5 * seg - 256);
  if (ws_bytes < 5 * seg + 256) { sl_set_last_error("csr_transpose: workspace too small"); return SL_ERR_INVALID; }
  if (nnz > 0) {
    int64_t gr64 = (nrows + NT / 64 - 1) / (NT / 64);
    const unsigned gr = (unsigned)(gr64 > 65536 ? 65536 : gr64);
    if (idx32) k_expand<int32_t><<<gr, NT, 0, s>>>(rowptr, (const int32_t*)col, nrows, key, pos, row_of);
    else k_expand<int64_t><<<gr, NT, 0, s>>>(rowptr, (const int64_t*)col, nrows, key, pos, row_of);
    SL_LAUNCH_CHECK();
    SL_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, key, key2, pos, pos2, (int)nnz, 0,
                                                    bits_for(ncols + 1), s));
    const unsigned gn = (unsigned)((nnz + NT - 1) / NT);
    if (vdtype == SL_F32)
      k_gather<float><<<gn, NT, 0, s>>>(pos2, row_of, (const float*)vals, nnz, orow, (float*)oval);
    else
      k_gather<double><<<gn, NT, 0, s>>>(pos2, row_of, (const double*)vals, nnz, orow, (double*)oval);
    SL_LAUNCH_CHECK();
  }
  k_colptr<<<(unsigned)((ncols + 1 + NT - 1) / NT), NT, 0, s>>>(key2, nnz, ncols, colptr);
  SL_LAUNCH_CHECK();
  return SL_OK;
}
