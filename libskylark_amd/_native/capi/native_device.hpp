// Interpreter-free device path of the C API: "DeviceMatrix" operands (GPU
// buffers, row-major with a leading dimension) go straight from the sl_* entry
// points into the HIP library (libskylark_hip.so, resolved next to this
// library) -- no CPython, no torch.  Reference dispatch being matched:
// capi/csketch.cpp:614-680 (sketch application), capi/cnla.cpp:15-84
// (ApproximateSVD), capi/ckernel.cpp:34-128 (kernel Gram).
//
//   sketch apply   JLT / CT: S panels realised by the Threefry kernel from the
//                  sketch's stream (same entries as the runtime), GEMM on
//                  rocBLAS; FJLT: the explicit sqrt(N/S) P F D operator
//                  (sl_fjlt_operator) then one GEMM; CWT / MMT / WZT: the
//                  bucketed hash kernels (sl_hash_dense_colwise / _rowwise)
//   randSVD        the C++ engine (rsvd_engine.cpp: fused passes, device
//                  CholeskyQR and Jacobi core, hipGraph replay) on bf16 A;
//                  the sketch operator drawn from the context's stream exactly
//                  as the runtime draws it (JLT/CT dense, FJLT, CWT)
//   kernel Gram    rocBLAS X Y^T + the native epilogue (sl_gram_map:
//                  Gaussian, polynomial, Matern) or the fused pairwise kernel
//                  (sl_pairwise_map_strided: Laplacian, exp-semigroup);
//                  points given as rows or columns without a transpose copy
// Every call runs on the default stream and returns after the device work.
#pragma once

#include <dlfcn.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "native_sketch.hpp"

namespace sldev {

enum { F32 = 0, F64 = 1, BF16 = 2 };

struct DevMat {
  void* data;
  int dtype;
  int64_t m, n, ld;   // row-major: element (i, j) at data[i * ld + j]
};

inline size_t esize(int dt) { return dt == F64 ? 8 : dt == F32 ? 4 : 2; }

// ------------------------------------------------------------ symbol table
struct Lib {
  bool loaded = false;
  std::string err;
  void* h = nullptr;
  void* rb = nullptr;
  const char* (*last_error)() = nullptr;
  int (*dev_malloc)(int64_t, void**) = nullptr;
  int (*dev_free)(void*) = nullptr;
  int (*dev_memcpy)(void*, const void*, int64_t, int, void*) = nullptr;
  int (*dev_memset)(void*, int, int64_t, void*) = nullptr;
  int (*dev_sync)(void*) = nullptr;
  int (*fill_random)(void*, int, int, uint64_t, uint64_t, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t,
                     int64_t, int64_t, double, double, double, int, void*) = nullptr;
  int (*fjlt_operator)(const uint64_t*, int64_t, int64_t, double, void*, int, int64_t, int, void*) = nullptr;
  int (*hash_colwise)(const void*, int, int64_t, int64_t, const int64_t*, const int64_t*, const double*, int64_t,
                      void*, int, int64_t, int64_t, int, void*) = nullptr;
  int (*hash_rowwise)(const void*, int, int64_t, int64_t, int64_t, const int64_t*, const int64_t*, const double*,
                      int64_t, void*, int, int64_t, int64_t, int, void*) = nullptr;
  int (*pairwise)(const void*, int64_t, int64_t, const void*, int64_t, int64_t, void*, int64_t, int, int64_t, int64_t,
                  int64_t, int, double, void*) = nullptr;
  int (*sqnorms)(const void*, int, int64_t, int64_t, int64_t, int64_t, void*, void*) = nullptr;
  int (*gram_map)(void*, int, int64_t, int64_t, int64_t, const void*, const void*, int, double, double, double,
                  void*) = nullptr;
  int (*plan_create)(int64_t, int64_t, int64_t, int, int, int, void**) = nullptr;
  int (*plan_destroy)(void*) = nullptr;
  int (*set_dense)(void*, int, uint64_t, uint64_t, double, double, double, void*) = nullptr;
  int (*set_fjlt)(void*, uint64_t, uint64_t, uint64_t, double, void*) = nullptr;
  int (*set_zt)(void*, const void*, void*) = nullptr;
  int (*run)(void*, const void*, int, float*, int64_t, float*, float*, void*) = nullptr;
  int (*status)(void*, int*, void*) = nullptr;
  int (*run_comm)(void*, const void*, void*, float*, int64_t, float*, float*, void*) = nullptr;
  int (*comm_id_bytes)() = nullptr;
  int (*comm_unique_id)(void*) = nullptr;
  int (*comm_init)(const void*, int, int, void**) = nullptr;
  int (*comm_destroy)(void*) = nullptr;
  int (*set_device)(int) = nullptr;
  // rocBLAS (plain library GEMMs)
  void* rb_handle = nullptr;
  int (*rb_dgemm)(void*, int, int, int, int, int, const double*, const double*, int, const double*, int,
                  const double*, double*, int) = nullptr;
  int (*rb_sgemm)(void*, int, int, int, int, int, const float*, const float*, int, const float*, int, const float*,
                  float*, int) = nullptr;
};

template <typename F>
inline bool bind(void* h, const char* name, F& f, std::string& err) {
  f = reinterpret_cast<F>(dlsym(h, name));
  if (!f) err = std::string("missing symbol ") + name;
  return f != nullptr;
}

// directory of this library (the HIP library sits next to it)
inline std::string self_dir() {
  Dl_info info;
  if (dladdr((void*)&self_dir, &info) && info.dli_fname) {
    std::string p(info.dli_fname);
    const auto k = p.find_last_of('/');
    if (k != std::string::npos) return p.substr(0, k);
  }
  return ".";
}

inline Lib& lib() {
  static Lib L;
  static std::once_flag once;
  std::call_once(once, [] {
    const std::string path = self_dir() + "/libskylark_hip.so";
    L.h = dlopen(path.c_str(), RTLD_NOW | RTLD_GLOBAL);
    if (!L.h) {
      L.err = std::string("cannot load ") + path + ": " + dlerror();
      return;
    }
    bool ok = bind(L.h, "sl_last_error", L.last_error, L.err) && bind(L.h, "sl_dev_malloc", L.dev_malloc, L.err) &&
              bind(L.h, "sl_dev_free", L.dev_free, L.err) && bind(L.h, "sl_dev_memcpy", L.dev_memcpy, L.err) &&
              bind(L.h, "sl_dev_memset", L.dev_memset, L.err) && bind(L.h, "sl_dev_sync", L.dev_sync, L.err) &&
              bind(L.h, "sl_fill_random", L.fill_random, L.err) &&
              bind(L.h, "sl_fjlt_operator", L.fjlt_operator, L.err) &&
              bind(L.h, "sl_hash_dense_colwise", L.hash_colwise, L.err) &&
              bind(L.h, "sl_hash_dense_rowwise", L.hash_rowwise, L.err) &&
              bind(L.h, "sl_pairwise_map_strided", L.pairwise, L.err) &&
              bind(L.h, "sl_point_sqnorms", L.sqnorms, L.err) && bind(L.h, "sl_gram_map", L.gram_map, L.err) &&
              bind(L.h, "sl_rsvd_plan_create", L.plan_create, L.err) &&
              bind(L.h, "sl_rsvd_plan_destroy", L.plan_destroy, L.err) &&
              bind(L.h, "sl_rsvd_set_dense", L.set_dense, L.err) && bind(L.h, "sl_rsvd_set_fjlt", L.set_fjlt, L.err) &&
              bind(L.h, "sl_rsvd_set_zt", L.set_zt, L.err) && bind(L.h, "sl_rsvd_run", L.run, L.err) &&
              bind(L.h, "sl_rsvd_status", L.status, L.err) && bind(L.h, "sl_rsvd_run_comm", L.run_comm, L.err) &&
              bind(L.h, "sl_comm_unique_id_bytes", L.comm_id_bytes, L.err) &&
              bind(L.h, "sl_comm_unique_id", L.comm_unique_id, L.err) &&
              bind(L.h, "sl_comm_init", L.comm_init, L.err) && bind(L.h, "sl_comm_destroy", L.comm_destroy, L.err) &&
              bind(L.h, "sl_dev_set_device", L.set_device, L.err);
    if (!ok) return;
    L.rb = dlopen("librocblas.so", RTLD_NOW | RTLD_LOCAL);
    if (!L.rb) L.rb = dlopen("/opt/rocm/lib/librocblas.so", RTLD_NOW | RTLD_LOCAL);
    if (!L.rb) {
      L.err = "cannot load librocblas.so";
      return;
    }
    int (*create)(void**) = nullptr;
    if (!bind(L.rb, "rocblas_create_handle", create, L.err) || !bind(L.rb, "rocblas_dgemm", L.rb_dgemm, L.err) ||
        !bind(L.rb, "rocblas_sgemm", L.rb_sgemm, L.err))
      return;
    if (create(&L.rb_handle) != 0) {
      L.err = "rocblas_create_handle failed";
      return;
    }
    L.loaded = true;
  });
  return L;
}

// error text of the last failed call of this path
inline std::string& error() {
  static std::string e;
  return e;
}

inline int fail(int code, const std::string& msg) {
  error() = msg;
  return code;
}

inline int check(int rc, const char* what) {
  if (rc == 0) return 0;
  Lib& L = lib();
  return fail(rc, std::string(what) + ": " + (L.last_error ? L.last_error() : "native error"));
}

#define SLDEV_TRY(expr, what)             \
  do {                                    \
    const int _rc = sldev::check((expr), what); \
    if (_rc) return _rc;                  \
  } while (0)

// device scratch freed at scope exit
struct Buf {
  void* p = nullptr;
  explicit Buf(int64_t bytes) { lib().dev_malloc(bytes, &p); }
  ~Buf() { if (p) lib().dev_free(p); }
  Buf(const Buf&) = delete;
  Buf& operator=(const Buf&) = delete;
};

// Row-major C (M x N, ldc) = alpha op(A) op(B) + beta C on rocBLAS (column-major:
// the row-major product is the column-major C^T = op(B)^T op(A)^T).
inline int gemm_rm(int dt, bool ta, bool tb, int64_t M, int64_t N, int64_t K, const void* A, int64_t lda,
                   const void* B, int64_t ldb, double beta, void* C, int64_t ldc) {
  Lib& L = lib();
  const int opA = ta ? 112 : 111, opB = tb ? 112 : 111;
  int rc;
  if (dt == F64) {
    const double al = 1.0, be = beta;
    rc = L.rb_dgemm(L.rb_handle, opB, opA, (int)N, (int)M, (int)K, &al, (const double*)B, (int)ldb,
                    (const double*)A, (int)lda, &be, (double*)C, (int)ldc);
  } else {
    const float al = 1.f, be = (float)beta;
    rc = L.rb_sgemm(L.rb_handle, opB, opA, (int)N, (int)M, (int)K, &al, (const float*)B, (int)ldb, (const float*)A,
                    (int)lda, &be, (float*)C, (int)ldc);
  }
  return rc == 0 ? 0 : fail(106, "rocBLAS gemm failed (status " + std::to_string(rc) + ")");
}

// ---------------------------------------------------------------- sketches
inline bool device_sketch_type(const std::string& t) {
  return t == "JLT" || t == "CT" || t == "FJLT" || t == "CWT" || t == "MMT" || t == "WZT";
}

// SA = S A (dim 0: A is N x n, SA is S x n) or A S^T (dim 1: A is m x N, SA is m x S)
inline int apply_sketch(const slnat::Sketch& s, const DevMat& A, const DevMat& SA, int dim) {
  Lib& L = lib();
  if (!L.loaded) return fail(106, "device C API: " + L.err);
  if (!device_sketch_type(s.type)) return fail(103, "sketch " + s.type + " has no device C path");
  if ((A.dtype != F32 && A.dtype != F64) || SA.dtype != A.dtype)
    return fail(103, "device sketch: A and SA must both be f32 or both f64");
  const int64_t sk_in = dim == 0 ? A.m : A.n;   // the sketched dimension (N)
  const int64_t other = dim == 0 ? A.n : A.m;
  if (sk_in != s.N || (dim == 0 ? (SA.m != s.S || SA.n != other) : (SA.m != other || SA.n != s.S)))
    return fail(104, "device sketch: dimension mismatch");
  const int dt = A.dtype;
  const size_t es = esize(dt);
  void* st = nullptr;
  if (s.type == "JLT" || s.type == "CT") {
    // S panels of b columns (<= 2^24 entries), accumulated into SA
    const int64_t b = std::max<int64_t>(1, std::min<int64_t>(s.N, (int64_t(1) << 24) / std::max<int64_t>(s.S, 1)));
    Buf P(s.S * b * (int64_t)es);
    if (!P.p) return fail(101, "device sketch: allocation failed");
    for (int64_t k0 = 0; k0 < s.N; k0 += b) {
      const int64_t kb = std::min(b, s.N - k0);
      SLDEV_TRY(L.fill_random(P.p, dt, s.dist, s.seed, s.ctr0, s.S, kb, kb, 1, 0, k0, 1, s.S, 0.0, 0.0, s.scale,
                              dt == F64 ? 1 : 0, st),
                "sketch panel");
      const double beta = k0 == 0 ? 0.0 : 1.0;
      int rc;
      if (dim == 0)
        rc = gemm_rm(dt, false, false, s.S, other, kb, P.p, kb, (const char*)A.data + k0 * A.ld * es, A.ld, beta,
                     SA.data, SA.ld);
      else
        rc = gemm_rm(dt, false, true, other, s.S, kb, (const char*)A.data + k0 * es, A.ld, P.p, kb, beta, SA.data,
                     SA.ld);
      if (rc) return rc;
    }
    return check(L.dev_sync(st), "sync");
  }
  if (s.type == "FJLT") {
    if (s.S * s.N > (int64_t(1) << 28)) return fail(103, "device FJLT: S x N operator too large for the explicit path");
    // FJLT_data draws: N Rademacher signs, then S frequencies
    const uint64_t prm_h[3] = {s.seed, s.ctr0, s.ctr0 + (uint64_t)s.N};
    Buf prm(sizeof prm_h), F(s.S * s.N * (int64_t)es);
    if (!prm.p || !F.p) return fail(101, "device FJLT: allocation failed");
    SLDEV_TRY(L.dev_memcpy(prm.p, prm_h, sizeof prm_h, 0, st), "copy");
    SLDEV_TRY(L.fjlt_operator((const uint64_t*)prm.p, s.S, s.N, std::sqrt((double)s.N / (double)s.S), F.p, dt, s.N, 0,
                              st),
              "fjlt operator");
    const int rc = dim == 0 ? gemm_rm(dt, false, false, s.S, other, s.N, F.p, s.N, A.data, A.ld, 0.0, SA.data, SA.ld)
                            : gemm_rm(dt, false, true, other, s.S, s.N, A.data, A.ld, F.p, s.N, 0.0, SA.data, SA.ld);
    if (rc) return rc;
    return check(L.dev_sync(st), "sync");
  }
  // hash sketches: bucket order of the N inputs (stable), bucket pointers
  std::vector<int64_t> perm((size_t)s.N), bptr((size_t)s.S + 1, 0);
  for (int64_t j = 0; j < s.N; ++j) ++bptr[(size_t)s.idx[(size_t)j] + 1];
  for (int64_t b = 0; b < s.S; ++b) bptr[(size_t)b + 1] += bptr[(size_t)b];
  {
    std::vector<int64_t> fill(bptr.begin(), bptr.end() - 1);
    for (int64_t j = 0; j < s.N; ++j) perm[(size_t)fill[(size_t)s.idx[(size_t)j]]++] = j;
  }
  std::vector<double> vals((size_t)s.N);
  for (int64_t j = 0; j < s.N; ++j) vals[(size_t)j] = dim == 0 ? s.val[(size_t)perm[(size_t)j]] : s.val[(size_t)j];
  Buf dperm(s.N * 8), dbptr((s.S + 1) * 8), dval(s.N * 8);
  if (!dperm.p || !dbptr.p || !dval.p) return fail(101, "device hash sketch: allocation failed");
  SLDEV_TRY(L.dev_memcpy(dperm.p, perm.data(), s.N * 8, 0, st), "copy");
  SLDEV_TRY(L.dev_memcpy(dbptr.p, bptr.data(), (s.S + 1) * 8, 0, st), "copy");
  SLDEV_TRY(L.dev_memcpy(dval.p, vals.data(), s.N * 8, 0, st), "copy");
  for (int64_t i = 0; i < SA.m; ++i)
    SLDEV_TRY(L.dev_memset((char*)SA.data + i * SA.ld * es, 0, SA.n * (int64_t)es, st), "memset");
  if (dim == 0) {
    SLDEV_TRY(L.hash_colwise(A.data, dt, A.ld, other, (const int64_t*)dperm.p, (const int64_t*)dbptr.p,
                             (const double*)dval.p, s.S, SA.data, dt, SA.ld, 0, 1, st),
              "hash colwise");
  } else {
    SLDEV_TRY(L.hash_rowwise(A.data, dt, A.ld, other, s.N, (const int64_t*)dperm.p, (const int64_t*)dbptr.p,
                             (const double*)dval.p, s.S, SA.data, dt, SA.ld, 0, 1, st),
              "hash rowwise");
  }
  return check(L.dev_sync(st), "sync");
}

// ---------------------------------------------------------------- randSVD
struct SvdParams {
  int ratio = 2, additive = 0, iters = 0;
  std::string sketch = "JLT";
};

inline SvdParams parse_svd_params(const char* js) {
  SvdParams p;
  if (!js || !*js) return p;
  double v;
  if (slnat::get_number(js, "oversampling_ratio", v)) p.ratio = (int)v;
  if (slnat::get_number(js, "oversampling_additive", v)) p.additive = (int)v;
  if (slnat::get_number(js, "num_iterations", v)) p.iters = (int)v;
  std::string sk;
  if (slnat::get_string(js, "sketch", sk)) {
    for (auto& c : sk) c = (char)toupper(c);
    p.sketch = sk;
  }
  return p;
}

// a few engine plans (device buffers + the captured graph) kept across calls
struct PlanKey {
  const void* A;
  int64_t m, n, ld;
  int k, r, q;
  bool operator==(const PlanKey& o) const {
    return A == o.A && m == o.m && n == o.n && ld == o.ld && k == o.k && r == o.r && q == o.q;
  }
};

struct PlanCache {
  std::vector<std::pair<PlanKey, void*>> v;
  int calls_since_create = 0;
  ~PlanCache() {
    // process exit: the runtime may already be torn down, leak deliberately
  }
};

inline PlanCache& plans() {
  static PlanCache c;
  return c;
}

inline void drop_rsvd_plan(void* plan) {
  auto& v = plans().v;
  for (size_t i = 0; i < v.size(); ++i)
    if (v[i].second == plan) {
      lib().plan_destroy(plan);
      v.erase(v.begin() + (long)i);
      return;
    }
}

// U (m x rank f32), S (rank f32, any 1-column / 1-row shape), V (n x rank f32)
// of bf16 A (m x n, m >= n).  ctr: the context counter (advanced by the
// sketch's draws exactly as the runtime advances it).  comm (a NativeComm
// RCCL communicator, sl_device_comm_create): A is this rank's row shard of a
// row-distributed matrix (every rank the same n), U its rows of the left
// factor, S and V replicated; the [W; G] pass sums are all-reduced over RCCL
// between the engine's segments (sl_rsvd_run_comm).
inline int approximate_svd(const DevMat& A, const DevMat& U, const DevMat& Sv, const DevMat& V, int rank,
                           const char* params, uint64_t seed, uint64_t& ctr, void* comm = nullptr) {
  Lib& L = lib();
  if (!L.loaded) return fail(106, "device C API: " + L.err);
  if (A.dtype != BF16) return fail(103, "device approximate_svd: A must be bf16");
  if (U.dtype != F32 || Sv.dtype != F32 || V.dtype != F32) return fail(103, "device approximate_svd: U, S, V are f32");
  const int64_t m = A.m, n = A.n;
  if (m < n && !comm) return fail(103, "device approximate_svd: needs a tall A (m >= n); pass A^T and swap U / V");
  if (rank < 1 || rank > n) return fail(109, "device approximate_svd: bad rank");
  const SvdParams p = parse_svd_params(params);
  const int k = (int)std::max<int64_t>(rank, std::min<int64_t>(n, (int64_t)p.ratio * rank + p.additive));
  if (U.m != m || U.n != rank || V.m != n || V.n != rank || V.ld != rank || Sv.m * Sv.n != rank)
    return fail(104, "device approximate_svd: output shapes");
  if (n % 8 || n < 16 || n > 1024 || A.ld % 8 || k > 48)
    return fail(103, "device approximate_svd: engine covers 16 <= n <= 1024, n % 8 == 0, lda % 8 == 0, k <= 48");
  const int q = std::max(0, p.iters);
  const PlanKey key{A.data, m, n, A.ld, k, rank, q};
  void* plan = nullptr;
  bool fresh = false;
  for (auto& e : plans().v)
    if (e.first == key) plan = e.second;
  if (!plan) {
    if (plans().v.size() >= 4) {
      L.plan_destroy(plans().v.front().second);
      plans().v.erase(plans().v.begin());
    }
    SLDEV_TRY(L.plan_create(m, n, A.ld, k, rank, q, &plan), "rsvd plan");
    plans().v.push_back({key, plan});
    fresh = true;
  }
  void* st = nullptr;
  const uint64_t base = ctr;
  if (p.sketch == "JLT" || p.sketch == "CT") {
    const bool jlt = p.sketch == "JLT";
    SLDEV_TRY(L.set_dense(plan, jlt ? sl::DIST_NORMAL : sl::DIST_CAUCHY, seed, base, 0.0, 0.0,
                          jlt ? std::sqrt(1.0 / k) : 1.0 / k, st),
              "sketch operator");
    ctr = base + (uint64_t)(n * k);
  } else if (p.sketch == "FJLT") {
    SLDEV_TRY(L.set_fjlt(plan, seed, base, base + (uint64_t)n, std::sqrt((double)n / k), st), "sketch operator");
    ctr = base + (uint64_t)(n + k);
  } else if (p.sketch == "CWT") {
    slnat::Sketch s;
    s.type = "CWT";
    s.N = n;
    s.S = k;
    s.seed = seed;
    s.ctr0 = base;
    ctr = slnat::build(s);
    // Z^T (k x n) = the CountSketch matrix, bf16
    std::vector<uint16_t> zt((size_t)(n * k), 0);
    for (int64_t j = 0; j < n; ++j) {
      const float f = (float)s.val[(size_t)j];
      uint32_t u;
      memcpy(&u, &f, 4);
      u += 0x7fffu + ((u >> 16) & 1u);
      zt[(size_t)(s.idx[(size_t)j] * n + j)] = (uint16_t)(u >> 16);
    }
    Buf d(n * k * 2);
    if (!d.p) return fail(101, "device approximate_svd: allocation failed");
    SLDEV_TRY(L.dev_memcpy(d.p, zt.data(), n * k * 2, 0, st), "copy");
    SLDEV_TRY(L.set_zt(plan, d.p, st), "sketch operator");
    SLDEV_TRY(L.dev_sync(st), "sync");
  } else {
    return fail(109, "device approximate_svd: sketch must be JLT, CT, FJLT or CWT");
  }
  if (comm) {
    SLDEV_TRY(L.run_comm(plan, A.data, comm, (float*)U.data, U.ld, (float*)Sv.data, (float*)V.data, st),
              "rsvd run (RCCL)");
  } else {
    // first call on a plan runs eagerly; later calls replay its graph
    SLDEV_TRY(L.run(plan, A.data, fresh ? 0 : 1, (float*)U.data, U.ld, (float*)Sv.data, (float*)V.data, st),
              "rsvd run");
  }
  int status = 0;
  SLDEV_TRY(L.status(plan, &status, st), "rsvd status");
  if (status & 16) {
    // a pass-boundary wait timed out: the outputs are invalid and the plan's
    // sync words are mid-protocol -- drop it so the next call builds a fresh one
    drop_rsvd_plan(plan);
    return fail(106, "device approximate_svd: a pass-boundary kernel timed out (status 16); outputs invalid");
  }
  if (status & 2) return fail(108, "device approximate_svd: non-finite values in A");
  return 0;
}

// -------------------------------------------------------------- kernel Gram
enum KType { K_NONE = -1, K_LINEAR = 0, K_GAUSSIAN, K_POLYNOMIAL, K_LAPLACIAN, K_EXPSEMIGROUP, K_MATERN };

struct Kern {
  int type = K_NONE;
  int N = 0;
  double p[3] = {0, 0, 0};   // gaussian/laplacian: sigma; expsemigroup: beta; polynomial: q, c, gamma; matern: nu, l
};

inline int kernel_type_of(const char* t) {
  std::string s(t);
  for (auto& c : s) c = (char)tolower(c);
  if (s == "linear") return K_LINEAR;
  if (s == "gaussian") return K_GAUSSIAN;
  if (s == "polynomial") return K_POLYNOMIAL;
  if (s == "laplacian") return K_LAPLACIAN;
  if (s == "expsemigroup") return K_EXPSEMIGROUP;
  if (s == "matern") return K_MATERN;
  return K_NONE;
}

// K[i, j] = k(x_i, y_j).  dir 1: points are the columns of the operand
// (reference default), 2: rows.
inline int kernel_gram(const Kern& kk, int dirX, int dirY, const DevMat& X, const DevMat& Y, const DevMat& K) {
  Lib& L = lib();
  if (!L.loaded) return fail(106, "device C API: " + L.err);
  const int dt = X.dtype;
  if ((dt != F32 && dt != F64) || Y.dtype != dt || K.dtype != dt)
    return fail(103, "device kernel_gram: X, Y, K must share dtype f32 or f64");
  const bool xr = dirX == 2, yr = dirY == 2;
  const int64_t mx = xr ? X.m : X.n, dx = xr ? X.n : X.m;
  const int64_t ny = yr ? Y.m : Y.n, dy = yr ? Y.n : Y.m;
  if (dx != dy || dx != kk.N) return fail(104, "device kernel_gram: point dimension mismatch");
  if (K.m != mx || K.n != ny) return fail(104, "device kernel_gram: K must be (#X points) x (#Y points)");
  // point stride / coordinate stride of each operand
  const int64_t xsp = xr ? X.ld : 1, xsd = xr ? 1 : X.ld;
  const int64_t ysp = yr ? Y.ld : 1, ysd = yr ? 1 : Y.ld;
  void* st = nullptr;
  if (kk.type == K_LAPLACIAN || kk.type == K_EXPSEMIGROUP) {
    const int mode = kk.type == K_LAPLACIAN ? 0 : 1;
    const double scale = kk.type == K_LAPLACIAN ? 1.0 / kk.p[0] : kk.p[0];
    SLDEV_TRY(L.pairwise(X.data, xsp, xsd, Y.data, ysp, ysd, K.data, K.ld, dt, mx, ny, dx, mode, scale, st),
              "pairwise kernel");
    return check(L.dev_sync(st), "sync");
  }
  if (kk.type == K_NONE) return fail(111, "device kernel_gram: unknown kernel");
  // G = X_p Y_p^T on rocBLAS (X_p = X for row points, X^T for column points)
  int rc = gemm_rm(dt, !xr, yr, mx, ny, dx, X.data, X.ld, Y.data, Y.ld, 0.0, K.data, K.ld);
  if (rc) return rc;
  if (kk.type == K_LINEAR) return check(L.dev_sync(st), "sync");
  const size_t es = esize(dt);
  Buf xn(mx * (int64_t)es), yn(ny * (int64_t)es);
  if (!xn.p || !yn.p) return fail(101, "device kernel_gram: allocation failed");
  int kind;
  double a = 0, c = 0, q = 1;
  if (kk.type == K_GAUSSIAN) {
    kind = 0;
    a = 1.0 / (2.0 * kk.p[0] * kk.p[0]);
  } else if (kk.type == K_POLYNOMIAL) {
    kind = 1;
    q = kk.p[0];
    c = kk.p[1];
    a = kk.p[2];
  } else {
    const double nu = kk.p[0];
    if (nu == 0.5) kind = 3;
    else if (nu == 1.5) kind = 4;
    else if (nu == 2.5) kind = 5;
    else return fail(103, "device kernel_gram: Matern nu must be 0.5, 1.5 or 2.5");
    a = 1.0 / kk.p[1];
  }
  if (kind != 1) {
    SLDEV_TRY(L.sqnorms(X.data, dt, mx, dx, xsp, xsd, xn.p, st), "point norms");
    SLDEV_TRY(L.sqnorms(Y.data, dt, ny, dy, ysp, ysd, yn.p, st), "point norms");
  }
  SLDEV_TRY(L.gram_map(K.data, dt, mx, ny, K.ld, xn.p, yn.p, kind, a, c, q, st), "kernel map");
  return check(L.dev_sync(st), "sync");
}

}  // namespace sldev
