// One-shot all-reduce for SMALL operands over peer-mapped device memory
// (the k-scalar / (n+k) x k reductions of LSQR, CG, CondEst
// and the randSVD passes, reference sites base/inner.hpp:22,84,170 and
// nla/svd.hpp).  A ring all-reduce over point-to-point xGMI takes 2(p-1)
// latency-bound steps; here every rank pushes its whole operand ONCE into a
// slot of every peer's receive buffer (one xGMI hop, all links in parallel),
// raises a per-(rank, block) flag there, waits for the p-1 flags of its own
// buffer and sums the p slots IN RANK ORDER -- every rank computes the same
// bits, no reduction tree, one kernel (graph-capturable: the generation
// counter lives on the device).
//
// Buffer (one per rank, exported by IPC, uncached fine-grained memory):
//   data  [2 sets][p ranks][cap bytes]   double-buffered by generation parity
//   flags [2 sets][p ranks][GMAX blocks] uint64 generation stamps
// Reuse is safe with two sets: a rank at generation g+2 has seen every
// peer's generation-(g+1) flag, and a peer raises that flag only after its
// generation-g kernel (the last reader of set g&1) has finished.
//
// Every wait is bounded (wall clock): a peer that never arrives sets *err
// and the kernel exits instead of spinning forever.
#include <cstring>

#include "sl_common.hpp"

namespace {

constexpr int OS_NT = 256;
constexpr int OS_GMAX = 64;     // blocks per call (chunks of the operand)
constexpr int OS_PMAX = 16;     // ranks

struct OsLayout {
  int64_t cap;     // bytes per slot
  int p;
  __host__ __device__ int64_t data_bytes() const { return 2 * (int64_t)p * cap; }
  __host__ __device__ int64_t total() const { return data_bytes() + 2 * (int64_t)p * OS_GMAX * 8; }
  __host__ __device__ char* slot(char* base, int set, int src) const { return base + ((int64_t)set * p + src) * cap; }
  __host__ __device__ uint64_t* flag(char* base, int set, int src, int blk) const {
    return (uint64_t*)(base + data_bytes()) + ((int64_t)set * p + src) * OS_GMAX + blk;
  }
};

template <typename T>
__global__ void __launch_bounds__(OS_NT)
k_oneshot_allreduce(T* __restrict__ x, int64_t n, int rank, int p, const uint64_t* __restrict__ bases,
                    int64_t cap, uint64_t* __restrict__ gen, unsigned* __restrict__ done, int* __restrict__ err,
                    unsigned long long timeout_ticks) {
  const OsLayout L{cap, p};
  const uint64_t g = gen[0] + 1;
  const int set = (int)(g & 1);
  const int blk = blockIdx.x, nblk = gridDim.x;
  const int64_t chunk = (n + nblk - 1) / nblk;
  const int64_t lo = (int64_t)blk * chunk;
  const int64_t hi = lo + chunk < n ? lo + chunk : n;
  const int t = threadIdx.x;
  __shared__ int timed_out;
  if (t == 0) timed_out = 0;
  // 1. push this rank's chunk into slot [set][rank] of every peer
  for (int q = 0; q < p; ++q) {
    if (q == rank) continue;
    T* dst = (T*)L.slot((char*)bases[q], set, rank);
    for (int64_t i = lo + t; i < hi; i += OS_NT) dst[i] = x[i];
  }
  __threadfence_system();
  __syncthreads();
  // 2. raise this block's flag in every peer's buffer
  if (t < p && t != rank)
    __hip_atomic_store(L.flag((char*)bases[t], set, rank, blk), g, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  // 3. wait for every peer's flag for this block in the local buffer (bounded)
  if (t < p && t != rank) {
    uint64_t* f = L.flag((char*)bases[rank], set, t, blk);
    const unsigned long long t0 = wall_clock64();
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != g) {
      if (wall_clock64() - t0 > timeout_ticks) {
        timed_out = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  if (timed_out) {
    // never a silent partial sum: the operand is poisoned (NaN) on this rank
    // and the error word set; Comm.check_collectives() raises on it
    if (t == 0) atomicOr(err, 1);
    for (int64_t i = lo + t; i < hi; i += OS_NT) x[i] = (T)NAN;
  } else {
    // 4. sum the p contributions in rank order (identical bits on every rank)
    for (int64_t i = lo + t; i < hi; i += OS_NT) {
      T acc = (T)0;
      for (int q = 0; q < p; ++q) {
        const T v = (q == rank) ? x[i]
                                : __hip_atomic_load((T*)L.slot((char*)bases[rank], set, q) + i, __ATOMIC_RELAXED,
                                                    __HIP_MEMORY_SCOPE_SYSTEM);
        acc += v;
      }
      x[i] = acc;
    }
  }
  // 5. the last block to finish advances the device-side generation
  __syncthreads();
  if (t == 0) {
    __threadfence();
    const unsigned prev = atomicAdd(done, 1u);
    if (prev == (unsigned)nblk - 1) {
      done[0] = 0;
      gen[0] = g;
    }
  }
}

}  // namespace

SL_API int64_t sl_oneshot_buffer_bytes(int64_t cap, int p) { return OsLayout{cap, p}.total(); }

// Allocate this rank's receive buffer (uncached device memory, zeroed) and
// export its IPC handle (64 bytes into handle_out).  Returns SL_ERR_HIP when
// the memory cannot be exported -- the caller then stays on RCCL.
SL_API int sl_oneshot_alloc(int64_t cap, int p, void** buf_out, void* handle_out) {
  if (p < 2 || p > OS_PMAX || cap <= 0 || cap % 16) {
    sl_set_last_error("oneshot_alloc: 2 <= p <= 16, cap > 0, cap % 16 == 0");
    return SL_ERR_UNSUPPORTED;
  }
  const int64_t bytes = OsLayout{cap, p}.total();
  void* b = nullptr;
  if (hipExtMallocWithFlags(&b, (size_t)bytes, hipDeviceMallocUncached) != hipSuccess) {
    sl_set_last_error("oneshot_alloc: hipExtMallocWithFlags(uncached) failed");
    return SL_ERR_HIP;
  }
  if (hipMemset(b, 0, (size_t)bytes) != hipSuccess ||
      hipIpcGetMemHandle((hipIpcMemHandle_t*)handle_out, b) != hipSuccess) {
    (void)hipFree(b);
    sl_set_last_error("oneshot_alloc: IPC export of the receive buffer failed");
    return SL_ERR_HIP;
  }
  *buf_out = b;
  return SL_OK;
}

SL_API int sl_oneshot_open(const void* handle, void** peer_out) {
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  if (hipIpcOpenMemHandle(peer_out, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) {
    sl_set_last_error("oneshot_open: hipIpcOpenMemHandle failed");
    return SL_ERR_HIP;
  }
  return SL_OK;
}

SL_API int sl_oneshot_close(void* peer) { return hipIpcCloseMemHandle(peer) == hipSuccess ? SL_OK : SL_ERR_HIP; }

SL_API int sl_oneshot_free(void* buf) { return hipFree(buf) == hipSuccess ? SL_OK : SL_ERR_HIP; }

SL_API int sl_oneshot_handle_bytes() { return (int)sizeof(hipIpcMemHandle_t); }

// x (n elements, f32 / f64, device) <- sum over the p ranks.  bases: device
// array of the p receive-buffer addresses as mapped in THIS process (own
// buffer at index rank).  state: device uint64[2] = {generation, done count}.
SL_API int sl_oneshot_allreduce(void* x, int64_t n, int dtype, int rank, int p, const uint64_t* bases, int64_t cap,
                                uint64_t* state, int* err, double timeout_s, void* stream) {
  if (n <= 0) return SL_OK;
  const int64_t es = dtype == SL_F64 ? 8 : 4;
  if ((dtype != SL_F32 && dtype != SL_F64) || n * es > cap || p < 2 || p > OS_PMAX || rank < 0 || rank >= p) {
    sl_set_last_error("oneshot_allreduce: f32/f64, n * elem <= cap, 2 <= p <= 16");
    return SL_ERR_UNSUPPORTED;
  }
  int64_t blocks = (n + 4 * OS_NT - 1) / (4 * OS_NT);
  if (blocks > OS_GMAX) blocks = OS_GMAX;
  if (blocks < 1) blocks = 1;
  const unsigned long long ticks = (unsigned long long)(timeout_s * 1e8);   // wall_clock64: 100 MHz
  hipStream_t s = (hipStream_t)stream;
  uint64_t* gen = state;
  unsigned* done = (unsigned*)(state + 1);
  if (dtype == SL_F64)
    k_oneshot_allreduce<double><<<(int)blocks, OS_NT, 0, s>>>((double*)x, n, rank, p, bases, cap, gen, done, err, ticks);
  else
    k_oneshot_allreduce<float><<<(int)blocks, OS_NT, 0, s>>>((float*)x, n, rank, p, bases, cap, gen, done, err, ticks);
  SL_LAUNCH_CHECK();
  return SL_OK;
}
