// Asynchronous randomized Gauss-Seidel (AsyRGS) on the GPU.
//
// Reference: algorithms/asynch/AsyRGS.hpp:12-57 (jstep / jstep1 under
// `#pragma omp atomic`, racy by design, IPDPS'14 analysis) and :82-236
// (sweeps * n random coordinates per synchronisation, drawn from the context
// stream with uniform_int(0, n-1)).
//
// gfx950 mapping: one wavefront per coordinate update.  Lanes split the
// coordinate's CSR row (= column, A symmetric) for the dot product A_i . X,
// reduce with cross-lane shuffles, then every right-hand side r < k receives
// x[i, r] += (b[i, r] - A_i . X[:, r]) / A_ii through a device-scope f64
// atomicAdd (global_atomic_add_f64) — the same lock-free semantics as the
// reference's OpenMP atomics, with the GPU's much higher concurrency.  The
// coordinate of step j is uniform_int(Threefry(seed, base + j), 0, n - 1):
// identical coordinate sequence on every run for a given context.
#include "sl_common.hpp"
#include "sl_rng.hpp"

template <typename IT, typename VT>
__global__ void __launch_bounds__(256)
k_asyrgs(const int64_t* __restrict__ rowptr, const IT* __restrict__ col, const VT* __restrict__ val, int64_t n,
         const double* __restrict__ B, double* __restrict__ X, int k, uint64_t seed, uint64_t base,
         int64_t nsteps) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = ((int64_t)gridDim.x * blockDim.x) >> 6;
  for (int64_t s = wave; s < nsteps; s += nwaves) {
    const sl::u64x2 rb = sl::stream_block(seed, base + (uint64_t)s);
    const int64_t i = sl::uniform_int(rb.x, 0, n - 1);
    const int64_t p0 = rowptr[i], p1 = rowptr[i + 1];
    if (p0 == p1) continue;
    for (int r0 = 0; r0 < k; r0 += 4) {
      double acc[4] = {0.0, 0.0, 0.0, 0.0};
      double dg = 0.0;
      for (int64_t p = p0 + lane; p < p1; p += 64) {
        const int64_t c = (int64_t)col[p];
        const double v = (double)val[p];
        if (c == i) dg = v;
#pragma unroll
        for (int q = 0; q < 4; ++q)
          if (r0 + q < k) acc[q] += v * __hip_atomic_load(&X[c * k + r0 + q], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
#pragma unroll
      for (int off = 32; off > 0; off >>= 1) {
        dg += __shfl_xor(dg, off);
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[q] += __shfl_xor(acc[q], off);
      }
      if (dg == 0.0) dg = 1.0;  // reference: diag defaults to 1 when absent
      if (lane < 4 && r0 + lane < k) {
        double a = acc[0];
        if (lane == 1) a = acc[1];
        if (lane == 2) a = acc[2];
        if (lane == 3) a = acc[3];
        const int r = r0 + lane;
        atomicAdd(&X[i * k + r], (B[i * k + r] - a) / dg);
      }
    }
  }
}

SL_API int sl_asyrgs(const int64_t* rowptr, const void* col, int idx32, const void* val, int vdtype, int64_t n,
                     const double* B, double* X, int k, uint64_t seed, uint64_t base, int64_t nsteps, void* stream) {
  if (nsteps <= 0 || n <= 0) return SL_OK;
  hipStream_t s = (hipStream_t)stream;
  // Concurrency bounds the staleness (delay) of the asynchronous updates: the
  // IPDPS'14 analysis needs the number of in-flight updates to stay well
  // below n, and two waves hitting the same coordinate double-apply its
  // correction.  Allow ~n/64 concurrent waves (4 per block), at most 8192
  // (enough to fill 256 CUs for large systems).
  int64_t waves = n / 64;
  if (waves < 1) waves = 1;
  if (waves > 8192) waves = 8192;
  if (waves > nsteps) waves = nsteps;
  unsigned grid = (unsigned)((waves + 3) / 4);
#define SL_A(IT, VT) k_asyrgs<IT, VT><<<grid, 256, 0, s>>>(rowptr, (const IT*)col, (const VT*)val, n, B, X, k, seed, base, nsteps)
  if (vdtype == SL_F64) {
    if (idx32) SL_A(int32_t, double); else SL_A(int64_t, double);
  } else if (vdtype == SL_F32) {
    if (idx32) SL_A(int32_t, float); else SL_A(int64_t, float);
  } else {
    sl_set_last_error("asyrgs: value dtype");
    return SL_ERR_UNSUPPORTED;
  }
#undef SL_A
  SL_LAUNCH_CHECK();
  return SL_OK;
}

// Host (CPU plumbing) version: sequential Gauss-Seidel with the same
// coordinate sequence (the asynchronous interleaving is the only difference).
SL_API int sl_asyrgs_host(const int64_t* rowptr, const int64_t* col, const double* val, int64_t n,
                          const double* B, double* X, int k, uint64_t seed, uint64_t base, int64_t nsteps) {
  for (int64_t s = 0; s < nsteps; ++s) {
    const sl::u64x2 rb = sl::stream_block(seed, base + (uint64_t)s);
    const int64_t i = sl::uniform_int(rb.x, 0, n - 1);
    if (rowptr[i] == rowptr[i + 1]) continue;
    for (int r = 0; r < k; ++r) {
      double dg = 1.0, v = B[i * k + r];
      for (int64_t p = rowptr[i]; p < rowptr[i + 1]; ++p) {
        if (col[p] == i) dg = val[p];
        v -= val[p] * X[col[p] * k + r];
      }
      X[i * k + r] += v / dg;
    }
  }
  return SL_OK;
}
