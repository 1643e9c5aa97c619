// Randomized SVD engine: the whole device-resident ApproximateSVD call of a
// row-distributed bf16 A (reference nla/svd.hpp:222-318 with the power
// iteration of :71-149), driven from C++ with no Python and no host round trip.
//
// One call = q + 2 segments on a HIP stream:
//   seg 0        pass 0 over A (Z = the sketch operator) + slab reduction
//   seg 1 .. q   CholeskyQR of the previous W (last-arriver Gram + Cholesky
//                + R^{-1}), Z^T = (W R^{-1})^T, pass i, slab reduction
//                (pass q is the FINAL form: Y stored, fp64 Gram of Y)
//   seg q + 1    fp64 core: Cholesky of Y^T Y, C = Rt^{-T} W^T W Rt^{-1},
//                its top eigenpairs (tridiagonal eigensolver, from scratch
//                every call), M = Rt^{-1} Ub_r, N = M S^{-1}, s
// then the finish (U = Y M, V = W N, s) into the caller's buffers.
//
// Single rank: the segments and the finish are captured ONCE as a hipGraph
// (per A pointer) and replayed; the sketch operator is a plain launch (its
// arguments carry the per-call sketch counters) and the finish writes the
// caller's fresh U / s / V through a device pointer table that one tiny
// kernel fills in front of the replay.  Several ranks: after every reducing segment the
// [W; G] buffer is summed over the ranks, either by the caller (Python:
// torch.distributed / one-shot IPC between sl_rsvd_segment calls) or, from
// C, by a NativeComm RCCL communicator (sl_rsvd_run_comm) -- no interpreter.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <new>

#include "sl_common.hpp"

// kernels of rsvd_pass.hip / rsvd_core.hip / tsk_f32_kernels.hip / native_comm.cpp
SL_API int sl_rsvd_pass_grid(int64_t m);
SL_API int64_t sl_rsvd_pass_workspace(int64_t m, int64_t n, int k);
SL_API int sl_rsvd_pass(const void* A, int64_t m, int64_t n, int64_t lda, const void* Zt, int k, void* ws, float* Y,
                        int64_t ldy, int final_pass, int variant, void* stream);
SL_API int sl_rsvd_reduce_z(const void* ws, int64_t m, int64_t n, int k, void* Wout, int w_f64, int ldw,
                            double* Gout, int ldg, int* zero_word, void* stream);
SL_API int sl_rsvd_make_v(const double* W, int n, int k, int ldw, const double* N, int r, float* V, const double* s64,
                          float* s32, void* stream);
SL_API int sl_rsvd_make_v_ind(const double* W, int n, int k, int ldw, const double* N, int r, const double* s64,
                              float* const* optr, void* stream);
SL_API int sl_rsvd_set_ptrs(float** tab, float* a, float* b, float* c, void* stream);
SL_API int64_t sl_rsvd_bnd_workspace(int k);
SL_API int sl_rsvd_bnd_coresident(int n, int k, int* ok);
SL_API int sl_rsvd_bnd_set_fault(const void* bws, int missing, uint64_t bound_ticks);
SL_API int sl_rsvd_boundary(int final_, int n, int k, int r, double* WG, void* bws, int* status, int status_or,
                            double* Rinv, void* Zt, float* M, double* N, double* s64, int* mirror, float* V,
                            float* s32, float* const* optr, void* stream);
SL_API int sl_tsk_f32_xm_ind(const float* Y, int64_t m, int k, const float* M, int k2, float* const* optr,
                             void* stream);
SL_API int sl_rsvd_fjlt_zt_tab(uint64_t seed, uint64_t baseD, uint64_t baseS, double scale, int k, int n, void* Zt,
                               float** tab, float* a, float* b, float* c, void* stream);
SL_API int sl_rsvd_fjlt_zt(uint64_t seed, uint64_t baseD, uint64_t baseS, double scale, int k, int n, void* Zt,
                           void* stream);
SL_API int sl_tsk_f32_xm(const float* Y, int64_t m, int k, int64_t ldy, const float* M, int k2, float* out,
                         int64_t ldo, double* G, void* ws, void* stream);
SL_API int sl_rsvd_zt_from_f64(const double* src, int64_t count, void* Zt, void* stream);
SL_API int sl_fill_random(void* out, int dtype, int dist, uint64_t seed, uint64_t base, int64_t rows, int64_t cols,
                          int64_t sr, int64_t sc, int64_t r0, int64_t c0, int64_t ir, int64_t ic, double p0, double p1,
                          double scale, int precise, void* stream);
SL_API int sl_comm_all_reduce(void* comm, const void* send, void* recv, int64_t count, int dtype, int op,
                              void* stream);

namespace {

struct Plan {
  int64_t m = 0, n = 0, lda = 0;
  int k = 0, r = 0, q = 0;
  // device buffers (one allocation, carved)
  char* base = nullptr;
  void* pass_ws = nullptr;
  uint16_t* Zt = nullptr;   // k x n bf16
  double* WG = nullptr;     // [W (n x k) ; G (k x k)] f64: the reduced pass outputs
  float* Y = nullptr;       // m x k f32
  void* bnd_ws = nullptr;   // fused boundary: sync words + partial Grams (zeroed once)
  float* last_ptrs[3] = {nullptr, nullptr, nullptr};   // optr contents written last (and on which stream)
  hipStream_t last_ptrs_stream = nullptr;
  // FJLT operator set for the next call but not yet launched: the run launches
  // it together with the pointer-table write (one small kernel, not two)
  bool fjlt_pending = false;
  uint64_t fj_seed = 0, fj_baseD = 0, fj_baseS = 0;
  double fj_scale = 0.0;
  double* Rinv = nullptr;   // k x k
  float* M = nullptr;       // k x r
  double* N = nullptr;      // k x r
  double* s64 = nullptr;    // r
  float** optr = nullptr;   // {U, s, V} of the current call (the graph's finish reads them)
  int* status = nullptr;
  int* mirror_host = nullptr;   // host-mapped copy of the status word, written by the final kernel
  int* mirror_dev = nullptr;
  // graphs of the segments (single rank), valid for graph_A: [0] segments
  // only, [1] segments + the finish writing through optr
  hipGraph_t graph[2] = {nullptr, nullptr};
  hipGraphExec_t exec[2] = {nullptr, nullptr};
  const void* graph_A = nullptr;
  hipStream_t cap_stream = nullptr;   // capture happens here (never the legacy null stream)
  hipEvent_t cap_ev = nullptr;
};

int64_t align256(int64_t b) { return (b + 255) & ~(int64_t)255; }

// LDS-DMA cache policy of the passes (sl_rsvd_pass variant bits 9-11; env
// SL_PASS_NT overrides, for A/B runs)
int pass_nt_code() {
  static int c = -1;
  if (c < 0) {
    const char* e = std::getenv("SL_PASS_NT");
    c = e ? (std::atoi(e) & 7) : 0;
  }
  return c;
}

// the same policy for the FINAL pass alone (env SL_PASS_NT_FINAL, A/B): its
// A reads not allocated in the MALL, so the Y it writes may stay there for U = Y M
int pass_nt_final_code() {
  static int c = -1;
  if (c < 0) {
    const char* e = std::getenv("SL_PASS_NT_FINAL");
    c = e ? (std::atoi(e) & 7) : -1;
    if (c < 0) c = 8;   // unset: the all-pass policy
  }
  return c == 8 ? pass_nt_code() : c;
}

// launch a deferred FJLT operator (and, with tab, the pointer-table write)
int flush_fjlt(Plan* p, hipStream_t s, float** tab = nullptr, float* a = nullptr, float* b = nullptr,
               float* c = nullptr) {
  if (!p->fjlt_pending) return SL_OK;
  p->fjlt_pending = false;
  return sl_rsvd_fjlt_zt_tab(p->fj_seed, p->fj_baseD, p->fj_baseS, p->fj_scale, p->k, (int)p->n, p->Zt, tab, a, b,
                             c, s);
}

// Segment i: [the boundary after pass i - 1] + pass i + its slab reduce
// into [W; G] (between segments several ranks all-reduce [W; G]).  The
// boundary is ONE launch (k_boundary): CholeskyQR of W and the next pass
// operand, or after the last pass (segment q + 1, the boundary alone) the
// fp64 core and, when V / s32 / optr are given, V = W N and s.
int seg(Plan* p, const void* A, int i, hipStream_t s, float* V = nullptr, float* s32 = nullptr,
        float* const* optr = nullptr) {
  const bool final_pass = i == p->q;
  if (i > p->q + 1 || i < 0) { sl_set_last_error("rsvd: segment out of range"); return SL_ERR_INVALID; }
  int rc = SL_OK;
  if (i > 0) {
    const int fin = i == p->q + 1 ? 1 : 0;
    rc = sl_rsvd_boundary(fin, (int)p->n, p->k, p->r, p->WG, p->bnd_ws, p->status, 1, p->Rinv, p->Zt, p->M, p->N,
                          p->s64, p->mirror_dev, V, s32, optr, s);
    if (rc != SL_OK || fin) return rc;
  }
  // the final pass stores Y and forms its fp64 Gram in-pass (bf16 hi / lo
  // products on the fragments the W update already holds); one reduce sums
  // the W and Gram slabs into [W; G]
  // odd passes walk the row blocks backwards: each pass starts on the rows
  // the previous one read last, which are still in the MALL
  rc = sl_rsvd_pass(A, p->m, p->n, p->lda, p->Zt, p->k, p->pass_ws, final_pass ? p->Y : nullptr, p->k,
                    final_pass ? 1 : 0, ((i & 1) ? 256 : 0) | ((final_pass ? pass_nt_final_code() : pass_nt_code()) << 9),
                    s);
  if (rc != SL_OK) return rc;
  // the first reduce of the call also clears the status word (no memset node)
  return sl_rsvd_reduce_z(p->pass_ws, p->m, p->n, p->k, p->WG, 1, p->k, final_pass ? p->WG + p->n * p->k : nullptr,
                          p->k, i == 0 ? p->status : nullptr, s);
}

void drop_graph(Plan* p) {
  for (int v = 0; v < 2; ++v) {
    if (p->exec[v]) (void)hipGraphExecDestroy(p->exec[v]);
    if (p->graph[v]) (void)hipGraphDestroy(p->graph[v]);
    p->exec[v] = nullptr;
    p->graph[v] = nullptr;
  }
  p->graph_A = nullptr;
}

// the finish through the pointer table (inside the graph: no graph -> stream
// gap before it, no per-call launches)
// (V and s were written by the final boundary through the same table)
int finish_ind(Plan* p, hipStream_t s) {
  return sl_tsk_f32_xm_ind(p->Y, p->m, p->k, p->M, p->r, p->optr, s);
}

// capture every segment (+ the indirect finish) once on the plan's own stream
int capture(Plan* p, const void* A, int with_finish, hipStream_t st) {
  if (!p->cap_stream) {
    SL_HIP_CHECK(hipStreamCreateWithFlags(&p->cap_stream, hipStreamNonBlocking));
    SL_HIP_CHECK(hipEventCreateWithFlags(&p->cap_ev, hipEventDisableTiming));
  }
  // the capture stream starts after everything queued on the caller's
  // stream (nothing is enqueued on it while it captures)
  SL_HIP_CHECK(hipEventRecord(p->cap_ev, st));
  SL_HIP_CHECK(hipStreamWaitEvent(p->cap_stream, p->cap_ev, 0));
  SL_HIP_CHECK(hipStreamSynchronize(p->cap_stream));
  hipStream_t cst = p->cap_stream;
  SL_HIP_CHECK(hipStreamBeginCapture(cst, hipStreamCaptureModeThreadLocal));
  int rc = SL_OK;
  for (int i = 0; i <= p->q + 1 && rc == SL_OK; ++i)
    rc = seg(p, A, i, cst, nullptr, nullptr, with_finish ? p->optr : nullptr);
  if (rc == SL_OK && with_finish) rc = finish_ind(p, cst);
  hipGraph_t g = nullptr;
  const hipError_t e = hipStreamEndCapture(cst, &g);
  if (rc != SL_OK || e != hipSuccess) {
    if (g) (void)hipGraphDestroy(g);
    if (rc == SL_OK) { sl_set_last_error(hipGetErrorString(e)); rc = SL_ERR_HIP; }
    return rc;
  }
  hipGraphExec_t ex = nullptr;
  if (hipGraphInstantiate(&ex, g, nullptr, nullptr, 0) != hipSuccess) {
    (void)hipGraphDestroy(g);
    sl_set_last_error("rsvd_run: graph instantiate failed");
    return SL_ERR_HIP;
  }
  p->graph[with_finish] = g;
  p->exec[with_finish] = ex;
  p->graph_A = A;
  return SL_OK;
}

}  // namespace

// A: m x n bf16 row shard (lda), k = sketch width (<= 48), r = rank (<= k),
// q = power iterations.  Allocates every device buffer of the call once.
SL_API int sl_rsvd_plan_create(int64_t m, int64_t n, int64_t lda, int k, int r, int q, void** out) {
  *out = nullptr;
  if (m < 1 || n < 16 || n > 1024 || n % 8 || lda % 8 || k < 1 || k > 48 || r < 1 || r > k || q < 0) {
    sl_set_last_error("rsvd_plan: needs m >= 1, 16 <= n <= 1024, n % 8 == 0, lda % 8 == 0, 1 <= r <= k <= 48, q >= 0");
    return SL_ERR_UNSUPPORTED;
  }
  {
    // the boundary grid spins on itself: refuse a plan whose grid cannot be co-resident
    int ok = 0;
    const int rc = sl_rsvd_bnd_coresident((int)n, k, &ok);
    if (rc != SL_OK) return rc;
    if (!ok) return SL_ERR_UNSUPPORTED;
  }
  Plan* p = new (std::nothrow) Plan();
  if (!p) return SL_ERR_GENERIC;
  p->m = m; p->n = n; p->lda = lda; p->k = k; p->r = r; p->q = q;
  int64_t off = 0;
  const int64_t o_pass = off; off = align256(off + sl_rsvd_pass_workspace(m, n, k));
  const int64_t o_zt = off;   off = align256(off + n * k * 2);
  const int64_t o_wg = off;   off = align256(off + (n + k) * k * 8);
  const int64_t o_y = off;    off = align256(off + m * k * 4);
  const int64_t o_bnd = off;  off = align256(off + sl_rsvd_bnd_workspace(k));
  const int64_t o_ri = off;   off = align256(off + (int64_t)k * k * 8);
  const int64_t o_m = off;    off = align256(off + (int64_t)k * r * 4);
  const int64_t o_n = off;    off = align256(off + (int64_t)k * r * 8);
  const int64_t o_s = off;    off = align256(off + (int64_t)r * 8);
  const int64_t o_st = off;   off = align256(off + 16);
  const int64_t o_op = off;   off = align256(off + 4 * (int64_t)sizeof(float*));
  if (hipMalloc((void**)&p->base, (size_t)off) != hipSuccess) {
    delete p;
    sl_set_last_error("rsvd_plan: device allocation failed");
    return SL_ERR_HIP;
  }
  p->pass_ws = p->base + o_pass;
  p->Zt = (uint16_t*)(p->base + o_zt);
  p->WG = (double*)(p->base + o_wg);
  p->Y = (float*)(p->base + o_y);
  p->bnd_ws = p->base + o_bnd;
  p->Rinv = (double*)(p->base + o_ri);
  p->M = (float*)(p->base + o_m);
  p->N = (double*)(p->base + o_n);
  p->s64 = (double*)(p->base + o_s);
  p->status = (int*)(p->base + o_st);
  p->optr = (float**)(p->base + o_op);
  if (hipMemset(p->bnd_ws, 0, (size_t)sl_rsvd_bnd_workspace(k)) != hipSuccess ||
      hipMemset(p->status, 0, 16) != hipSuccess) {
    (void)hipFree(p->base);
    delete p;
    sl_set_last_error("rsvd_plan: memset failed");
    return SL_ERR_HIP;
  }
  if (hipHostMalloc((void**)&p->mirror_host, 64, hipHostMallocMapped) == hipSuccess) {
    *p->mirror_host = 0;
    if (hipHostGetDevicePointer((void**)&p->mirror_dev, p->mirror_host, 0) != hipSuccess) {
      (void)hipHostFree(p->mirror_host);
      p->mirror_host = p->mirror_dev = nullptr;
    }
  }
  *out = p;
  return SL_OK;
}

SL_API int sl_rsvd_plan_destroy(void* plan) {
  Plan* p = (Plan*)plan;
  if (!p) return SL_OK;
  drop_graph(p);
  (void)sl_rsvd_bnd_set_fault(p->bnd_ws, 0, 0);
  if (p->cap_ev) (void)hipEventDestroy(p->cap_ev);
  if (p->cap_stream) (void)hipStreamDestroy(p->cap_stream);
  if (p->mirror_host) (void)hipHostFree(p->mirror_host);
  (void)hipFree(p->base);
  delete p;
  return SL_OK;
}

// Use caller-owned buffers for the [W; G] reduce buffer ((n + k) * k f64)
// and / or the status word (e.g. torch tensors the caller all-reduces / reads);
// null keeps the plan's own.
SL_API int sl_rsvd_plan_bind(void* plan, double* WG, int* status) {
  Plan* p = (Plan*)plan;
  drop_graph(p);
  if (WG) p->WG = WG;
  if (status) p->status = status;
  return SL_OK;
}

// Test-only fault injection: the boundary kernels wait for `missing` arrivals
// beyond their grid (no workgroup is ever last, every wait times out and sets
// status bit 16) with a spin bound of `bound_ticks` of the 100 MHz clock
// (0: 2 s).  A plan that has timed out is not reusable (its sync words are
// left mid-protocol): destroy it.
SL_API int sl_rsvd_plan_set_fault(void* plan, int missing, uint64_t bound_ticks) {
  Plan* p = (Plan*)plan;
  drop_graph(p);   // launch arguments are baked into a captured graph
  return sl_rsvd_bnd_set_fault(p->bnd_ws, missing, bound_ticks);
}

// Sketch operator of the call: the FJLT of reference FJLT_data (N Rademacher
// signs at baseD, k DCT frequencies at baseS, scale sqrt(n / k)) realised as
// the pass's bf16 Z^T.
// (deferred: launched by the next run / first segment, in that call's stream order)
SL_API int sl_rsvd_set_fjlt(void* plan, uint64_t seed, uint64_t baseD, uint64_t baseS, double scale, void* stream) {
  (void)stream;
  Plan* p = (Plan*)plan;
  p->fjlt_pending = true;
  p->fj_seed = seed; p->fj_baseD = baseD; p->fj_baseS = baseS; p->fj_scale = scale;
  return SL_OK;
}

// Dense sketch operator (JLT: Normal, CT: Cauchy, ...) of the call: the k x n
// matrix scale * dist(seed, base + j k + i) (reference dense_transform_data
// column-major stream) realised in f64 on the device (in the W buffer, free
// until the first reduce), then rounded f64 -> f32 -> bf16 into Z^T.
SL_API int sl_rsvd_set_dense(void* plan, int dist, uint64_t seed, uint64_t base, double p0, double p1, double scale,
                             void* stream) {
  Plan* p = (Plan*)plan;
  p->fjlt_pending = false;
  int rc = sl_fill_random(p->WG, SL_F64, dist, seed, base, p->k, p->n, p->n, 1, 0, 0, 1, p->k, p0, p1, scale, 1,
                          stream);
  if (rc != SL_OK) return rc;
  return sl_rsvd_zt_from_f64(p->WG, p->n * p->k, p->Zt, stream);
}

// Sketch operator given explicitly (k x n bf16, device).
SL_API int sl_rsvd_set_zt(void* plan, const void* Zt, void* stream) {
  Plan* p = (Plan*)plan;
  p->fjlt_pending = false;
  SL_HIP_CHECK(hipMemcpyAsync(p->Zt, Zt, (size_t)(p->n * p->k * 2), hipMemcpyDeviceToDevice, (hipStream_t)stream));
  return SL_OK;
}

// launch a deferred sketch operator now (callers that replay their own
// captured segments flush before the replay)
SL_API int sl_rsvd_flush(void* plan, void* stream) { return flush_fjlt((Plan*)plan, (hipStream_t)stream); }

SL_API int sl_rsvd_segment(void* plan, const void* A, int i, void* stream) {
  if (i == 0) {
    const int rc = flush_fjlt((Plan*)plan, (hipStream_t)stream);
    if (rc != SL_OK) return rc;
  }
  return seg((Plan*)plan, A, i, (hipStream_t)stream);
}

// the [W (n x k) ; G (k x k)] f64 buffer every reducing segment leaves for
// the cross-rank sum ((n + k) * k doubles after segment q, n * k before)
SL_API double* sl_rsvd_reduce_buffer(void* plan) { return ((Plan*)plan)->WG; }
SL_API float* sl_rsvd_y(void* plan) { return ((Plan*)plan)->Y; }

// U (m x r, row stride ldu), s (r), V (n x r) f32 from the core's factors
SL_API int sl_rsvd_finish(void* plan, float* U, int64_t ldu, float* s, float* V, void* stream) {
  Plan* p = (Plan*)plan;
  int rc = sl_rsvd_make_v(p->WG, (int)p->n, p->k, p->k, p->N, p->r, V, p->s64, s, stream);
  if (rc != SL_OK) return rc;
  return sl_tsk_f32_xm(p->Y, p->m, p->k, p->k, p->M, p->r, U, ldu, nullptr, nullptr, stream);
}

// Single-rank call: every segment (one graph replay when use_graph) then the
// finish.  The sketch operator must have been set for this call.
SL_API int sl_rsvd_run(void* plan, const void* A, int use_graph, float* U, int64_t ldu, float* s, float* V,
                       void* stream) {
  Plan* p = (Plan*)plan;
  hipStream_t st = (hipStream_t)stream;
  if (!use_graph) {
    int rc0 = flush_fjlt(p, st);
    if (rc0 != SL_OK) return rc0;
    for (int i = 0; i <= p->q + 1; ++i) {
      const int rc = seg(p, A, i, st, V, s, nullptr);
      if (rc != SL_OK) return rc;
    }
    if (!V) return sl_rsvd_finish(plan, U, ldu, s, V, stream);
    return sl_tsk_f32_xm(p->Y, p->m, p->k, p->k, p->M, p->r, U, ldu, nullptr, nullptr, stream);
  }
  if (p->graph_A != A) drop_graph(p);
  // the finish joins the graph when its streaming kernel can take this U
  // (contiguous rows, 16-byte aligned) -- else a plain launch after it
  const int fin = (p->k % 8 == 0 && ldu == p->r && ((uintptr_t)U & 15) == 0 && V != nullptr) ? 1 : 0;
  // the table already holds U / s / V when the last call on this stream
  // wrote the same ones (a caching allocator hands them back); else the
  // deferred FJLT launch writes it, or a one-thread kernel
  const bool need_tab = fin && !(p->last_ptrs[0] == U && p->last_ptrs[1] == s && p->last_ptrs[2] == V &&
                                 p->last_ptrs_stream == st);
  if (need_tab && p->fjlt_pending) {
    const int rc = flush_fjlt(p, st, p->optr, U, s, V);
    if (rc != SL_OK) return rc;
  } else {
    const int rc = flush_fjlt(p, st);
    if (rc != SL_OK) return rc;
    if (need_tab) {
      const int rc2 = sl_rsvd_set_ptrs(p->optr, U, s, V, st);
      if (rc2 != SL_OK) return rc2;
    }
  }
  if (need_tab) {
    p->last_ptrs[0] = U; p->last_ptrs[1] = s; p->last_ptrs[2] = V;
    p->last_ptrs_stream = st;
  }
  if (!p->exec[fin]) {
    const int rc = capture(p, A, fin, st);
    if (rc != SL_OK) return rc;
  }
  if (fin) {
    SL_HIP_CHECK(hipGraphLaunch(p->exec[1], st));
    return SL_OK;
  }
  SL_HIP_CHECK(hipGraphLaunch(p->exec[0], st));
  return sl_rsvd_finish(plan, U, ldu, s, V, stream);
}

// Several ranks from C: the segments with a NativeComm (RCCL) sum of the
// [W; G] buffer after each pass -- the interpreter-free distributed call.
SL_API int sl_rsvd_run_comm(void* plan, const void* A, void* comm, float* U, int64_t ldu, float* s, float* V,
                            void* stream) {
  Plan* p = (Plan*)plan;
  const int rc0 = flush_fjlt(p, (hipStream_t)stream);
  if (rc0 != SL_OK) return rc0;
  for (int i = 0; i <= p->q + 1; ++i) {
    int rc = seg(p, A, i, (hipStream_t)stream);
    if (rc != SL_OK) return rc;
    if (i <= p->q && comm) {
      const int64_t cnt = (i == p->q ? p->n + p->k : p->n) * p->k;
      rc = sl_comm_all_reduce(comm, p->WG, p->WG, cnt, SL_F64, 0, stream);
      if (rc != SL_OK) return rc;
    }
  }
  return sl_rsvd_finish(plan, U, ldu, s, V, stream);
}

// Status bits of the last call (1 pivot dropped, 2 non-finite, 4 Jacobi not
// converged, 8 fewer than r positive eigenvalues); synchronises the stream.
SL_API int sl_rsvd_status(void* plan, int* out, void* stream) {
  Plan* p = (Plan*)plan;
  SL_HIP_CHECK(hipMemcpyAsync(out, p->status, sizeof(int), hipMemcpyDeviceToHost, (hipStream_t)stream));
  SL_HIP_CHECK(hipStreamSynchronize((hipStream_t)stream));
  return SL_OK;
}

// host pointer of the status word's mirror (written by the final kernel of
// every call; valid once the call has completed), or null if unavailable
SL_API int* sl_rsvd_status_mirror(void* plan) { return ((Plan*)plan)->mirror_host; }

// device pointer of the status word (for asynchronous checks)
SL_API int* sl_rsvd_status_ptr(void* plan) { return ((Plan*)plan)->status; }
