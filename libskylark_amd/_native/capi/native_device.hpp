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
#include <cstdlib>
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
  int (*comm_all_reduce)(void*, const void*, void*, int64_t, int, int, void*) = nullptr;
  int (*comm_rank_size)(void*, int*, int*) = nullptr;
  int (*dev_memcpy2d)(void*, int64_t, const void*, int64_t, int64_t, int64_t, int, void*) = nullptr;
  int (*set_device)(int) = nullptr;
  int (*dev_count)(int*) = nullptr;
  int (*dct2_rows)(const int64_t*, int64_t, int64_t, const double*, double, void*, int, int64_t, int, void*) = nullptr;
  int (*feature_epi)(void*, int, int64_t, int64_t, int64_t, const double*, const double*, double, int, int,
                     void*) = nullptr;
  int (*transpose)(const void*, int, int64_t, int64_t, int64_t, void*, int64_t, void*) = nullptr;
  int (*csr_to_dense)(const int*, const int*, const double*, int64_t, void*, int, int64_t, void*) = nullptr;
  int (*dft_cs)(int64_t, int64_t, void*, void*, int, void*) = nullptr;
  int (*ppt_spectrum)(const void*, int, int64_t, int64_t, int64_t, int64_t, int64_t, int64_t, const int64_t*,
                      const double*, double, void*, int, void*) = nullptr;
  int (*hash_csr_col)(const int64_t*, const void*, int, const void*, int, const int64_t*, const int64_t*, const void*,
                      int64_t, int64_t, void*, int64_t, int64_t, int, int, const double*, double, void*) = nullptr;
  int (*hash_csr_row)(const int64_t*, const void*, int, const void*, int, int64_t, const int64_t*, const double*, void*,
                      int64_t, int64_t, int, void*) = nullptr;
  // general-precision randSVD engine (rsvd_general.hip)
  int (*gen_create)(int64_t, int64_t, int64_t, int, int, int, int, void**) = nullptr;
  int (*gen_destroy)(void*) = nullptr;
  int (*gen_set_fjlt)(void*, uint64_t, uint64_t, uint64_t, double) = nullptr;
  int (*gen_set_dense)(void*, int, uint64_t, uint64_t, double, double, double) = nullptr;
  int (*gen_set_z)(void*, const void*, void*) = nullptr;
  int (*gen_run)(void*, const void*, void*, int64_t, void*, void*, void*) = nullptr;
  int (*gen_status)(void*, int*, void*) = nullptr;
  int (*gen_run_comm)(void*, const void*, void*, void*, int64_t, void*, void*, void*) = nullptr;
  // host-operand NLA drivers (nla_native.hip) and the LIBSVM reader (libsvm_io.cpp)
  int (*sym_rsvd)(const double*, int64_t, int64_t, int, int, int, int, int, uint64_t, uint64_t, double*, int64_t,
                  double*, void*) = nullptr;
  int (*sym_rsvd_comm)(const double*, int64_t, int64_t, int64_t, int64_t, int, int, int, int, int, uint64_t, uint64_t,
                       double*, int64_t, double*, void*, void*) = nullptr;
  int (*blendenpik)(const double*, int64_t, int64_t, int64_t, const double*, int, int64_t, double*, int64_t, uint64_t,
                    uint64_t*, double, int, int*, void*) = nullptr;
  int (*blendenpik_comm)(const double*, int64_t, int64_t, int64_t, const double*, int, int64_t, double*, int64_t,
                         int64_t, int64_t, void*, uint64_t, uint64_t*, double, int, int*, void*) = nullptr;
  int (*libsvm_scan)(const char*, int64_t, int, int64_t*, int64_t*, int64_t*, int*) = nullptr;
  int (*libsvm_fill)(const char*, const int64_t*, const int64_t*, int, int64_t, double*, int64_t*, int64_t*,
                     double*) = nullptr;
  // rocBLAS (plain library GEMMs)
  void* rb_handle = nullptr;   // created on first use (needs a device)
  int (*rb_create)(void**) = nullptr;
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
              bind(L.h, "sl_comm_all_reduce", L.comm_all_reduce, L.err) &&
              bind(L.h, "sl_comm_rank_size", L.comm_rank_size, L.err) &&
              bind(L.h, "sl_dev_memcpy2d", L.dev_memcpy2d, L.err) &&
              bind(L.h, "sl_dev_set_device", L.set_device, L.err) && bind(L.h, "sl_dev_count", L.dev_count, L.err) &&
              bind(L.h, "sl_dct2_rows", L.dct2_rows, L.err) && bind(L.h, "sl_feature_epilogue", L.feature_epi, L.err) &&
              bind(L.h, "sl_transpose", L.transpose, L.err) && bind(L.h, "sl_csr_to_dense", L.csr_to_dense, L.err) &&
              bind(L.h, "sl_dft_cs", L.dft_cs, L.err) && bind(L.h, "sl_ppt_spectrum", L.ppt_spectrum, L.err) &&
              bind(L.h, "sl_hash_csr_colwise2", L.hash_csr_col, L.err) &&
              bind(L.h, "sl_hash_csr_rowwise", L.hash_csr_row, L.err) &&
              bind(L.h, "sl_rsvd_gen_create", L.gen_create, L.err) &&
              bind(L.h, "sl_rsvd_gen_destroy", L.gen_destroy, L.err) &&
              bind(L.h, "sl_rsvd_gen_set_fjlt", L.gen_set_fjlt, L.err) &&
              bind(L.h, "sl_rsvd_gen_set_dense", L.gen_set_dense, L.err) &&
              bind(L.h, "sl_rsvd_gen_set_z", L.gen_set_z, L.err) && bind(L.h, "sl_rsvd_gen_run", L.gen_run, L.err) &&
              bind(L.h, "sl_rsvd_gen_status", L.gen_status, L.err) &&
              bind(L.h, "sl_rsvd_gen_run_comm", L.gen_run_comm, L.err) &&
              bind(L.h, "sl_nat_sym_rsvd", L.sym_rsvd, L.err) &&
              bind(L.h, "sl_nat_sym_rsvd_comm", L.sym_rsvd_comm, L.err) && bind(L.h, "sl_nat_blendenpik", L.blendenpik, L.err) &&
              bind(L.h, "sl_nat_blendenpik_comm", L.blendenpik_comm, L.err) &&
              bind(L.h, "sl_libsvm_scan", L.libsvm_scan, L.err) && bind(L.h, "sl_libsvm_fill", L.libsvm_fill, L.err);
    if (!ok) return;
    L.rb = dlopen("librocblas.so", RTLD_NOW | RTLD_LOCAL);
    if (!L.rb) L.rb = dlopen("/opt/rocm/lib/librocblas.so", RTLD_NOW | RTLD_LOCAL);
    if (!L.rb) {
      L.err = "cannot load librocblas.so";
      return;
    }
    if (!bind(L.rb, "rocblas_create_handle", L.rb_create, L.err) || !bind(L.rb, "rocblas_dgemm", L.rb_dgemm, L.err) ||
        !bind(L.rb, "rocblas_sgemm", L.rb_sgemm, L.err))
      return;
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
                   const void* B, int64_t ldb, double beta, void* C, int64_t ldc, double alpha = 1.0) {
  Lib& L = lib();
  if (!L.rb_handle && L.rb_create(&L.rb_handle) != 0) {
    L.rb_handle = nullptr;
    return fail(106, "rocblas_create_handle failed");
  }
  const int opA = ta ? 112 : 111, opB = tb ? 112 : 111;
  int rc;
  if (dt == F64) {
    const double al = alpha, be = beta;
    rc = L.rb_dgemm(L.rb_handle, opB, opA, (int)N, (int)M, (int)K, &al, (const double*)B, (int)ldb,
                    (const double*)A, (int)lda, &be, (double*)C, (int)ldc);
  } else {
    const float al = (float)alpha, be = (float)beta;
    rc = L.rb_sgemm(L.rb_handle, opB, opA, (int)N, (int)M, (int)K, &al, (const float*)B, (int)ldb, (const float*)A,
                    (int)lda, &be, (float*)C, (int)ldc);
  }
  return rc == 0 ? 0 : fail(106, "rocBLAS gemm failed (status " + std::to_string(rc) + ")");
}

// ---------------------------------------------------------------- sketches
inline bool device_present() {
  Lib& L = lib();
  if (!L.loaded) return false;
  const char* e = getenv("SL_CAPI_HOST");   // force the host path (tests compare both)
  if (e && *e && *e != '0') return false;
  static int n = -1;
  if (n < 0) {
    int c = 0;
    L.dev_count(&c);
    n = c;
  }
  return n > 0;
}

// host vector -> device (freed with the Buf)
template <typename T>
inline int upload(Buf& b, const std::vector<T>& v) {
  if (!b.p) return fail(101, "device C API: allocation failed");
  if (v.empty()) return 0;
  return check(lib().dev_memcpy(b.p, v.data(), (int64_t)(v.size() * sizeof(T)), 0, nullptr), "copy");
}

// host f64 values as a device buffer of dtype dt
inline int upload_as(Buf& b, const double* v, int64_t n, int dt) {
  if (!b.p) return fail(101, "device C API: allocation failed");
  if (dt == F64) return check(lib().dev_memcpy(b.p, v, n * 8, 0, nullptr), "copy");
  std::vector<float> f((size_t)n);
  for (int64_t i = 0; i < n; ++i) f[(size_t)i] = (float)v[i];
  return check(lib().dev_memcpy(b.p, f.data(), n * 4, 0, nullptr), "copy");
}

inline int zero(const DevMat& M) {
  const size_t es = esize(M.dtype);
  if (M.ld == M.n) return check(lib().dev_memset(M.data, 0, M.m * M.n * (int64_t)es, nullptr), "memset");
  for (int64_t i = 0; i < M.m; ++i)
    SLDEV_TRY(lib().dev_memset((char*)M.data + i * M.ld * es, 0, M.n * (int64_t)es, nullptr), "memset");
  return 0;
}

// bucket structure of the hash kernels: perm (inputs sorted by bucket),
// bptr (S + 1), and the values in bucket order (pval) and input order (val)
struct HashDev {
  Buf perm, bptr, pval, val, idx;
  HashDev(int64_t N, int64_t S) : perm(N * 8), bptr((S + 1) * 8), pval(N * 8), val(N * 8), idx(N * 8) {}
};

inline int hash_upload(HashDev& H, const std::vector<int64_t>& idx, const std::vector<double>& val, int64_t S,
                       double mul = 1.0) {
  const int64_t N = (int64_t)idx.size();
  std::vector<int64_t> perm((size_t)N), bptr((size_t)S + 1, 0);
  for (int64_t j = 0; j < N; ++j) ++bptr[(size_t)idx[(size_t)j] + 1];
  for (int64_t b = 0; b < S; ++b) bptr[(size_t)b + 1] += bptr[(size_t)b];
  {
    std::vector<int64_t> fill(bptr.begin(), bptr.end() - 1);
    for (int64_t j = 0; j < N; ++j) perm[(size_t)fill[(size_t)idx[(size_t)j]]++] = j;
  }
  std::vector<double> pv((size_t)N), v((size_t)N);
  for (int64_t j = 0; j < N; ++j) {
    pv[(size_t)j] = mul * val[(size_t)perm[(size_t)j]];
    v[(size_t)j] = mul * val[(size_t)j];
  }
  int rc;
  if ((rc = upload(H.perm, perm)) || (rc = upload(H.bptr, bptr)) || (rc = upload(H.pval, pv)) || (rc = upload(H.val, v)) ||
      (rc = upload(H.idx, idx)))
    return rc;
  return 0;
}

// SA (= or +=) bucket sums of A along dim (rowwise needs the row in LDS)
inline int hash_apply(const HashDev& H, int64_t N, int64_t S, const DevMat& A, const DevMat& SA, int dim, int acc) {
  Lib& L = lib();
  if (dim == 0)
    return check(L.hash_colwise(A.data, A.dtype, A.ld, A.n, (const int64_t*)H.perm.p, (const int64_t*)H.bptr.p,
                                (const double*)H.pval.p, S, SA.data, SA.dtype, SA.ld, 0, acc, nullptr),
                 "hash colwise");
  return check(L.hash_rowwise(A.data, A.dtype, A.ld, A.m, N, (const int64_t*)H.perm.p, (const int64_t*)H.bptr.p,
                              (const double*)H.val.p, S, SA.data, SA.dtype, SA.ld, 0, acc, nullptr),
               "hash rowwise");
}

inline bool rowwise_fits(int64_t N, int dt) { return N * (int64_t)esize(dt) <= 160 * 1024; }

inline int apply_linear(const slnat::Sketch& s, const DevMat& A, const DevMat& SA, int dim, int64_t off);

// dim-1 application through dim 0 on the transposes (rows longer than LDS)
inline int apply_by_transpose(const slnat::Sketch& s, const DevMat& A, const DevMat& SA, int64_t off) {
  Lib& L = lib();
  const int dt = A.dtype;
  const size_t es = esize(dt);
  Buf At(A.n * A.m * (int64_t)es), T(s.S * A.m * (int64_t)es);
  if (!At.p || !T.p) return fail(101, "device sketch: allocation failed");
  SLDEV_TRY(L.transpose(A.data, dt, A.m, A.n, A.ld, At.p, A.m, nullptr), "transpose");
  const int rc = apply_linear(s, DevMat{At.p, dt, A.n, A.m, A.m}, DevMat{T.p, dt, s.S, A.m, A.m}, 0, off);
  if (rc) return rc;
  return check(L.transpose(T.p, dt, s.S, A.m, A.m, SA.data, SA.ld, nullptr), "transpose");
}

// sketch kinds whose operator mixes the whole sketched dimension non-linearly
// or through a structured transform with no column-range form here: their
// distributed application gathers the operand first
inline bool needs_whole(const slnat::Sketch& s) { return s.kind == slnat::K_FASTFOOD || s.kind == slnat::K_PPT; }

inline int epilogue_dev(const slnat::Sketch& s, const DevMat& SA, int dim) {
  if (s.epi == slnat::EPI_NONE) return 0;
  Buf sc(s.scales.empty() ? 8 : (int64_t)s.scales.size() * 8), sh(s.shifts.empty() ? 8 : (int64_t)s.shifts.size() * 8);
  int rc;
  if ((rc = upload(sc, s.scales)) || (rc = upload(sh, s.shifts))) return rc;
  return check(lib().feature_epi(SA.data, SA.dtype, SA.m, SA.n, SA.ld, s.scales.empty() ? nullptr : (const double*)sc.p,
                                 s.shifts.empty() ? nullptr : (const double*)sh.p, s.outscale, dim, s.epi, nullptr),
               "feature epilogue");
}

// The linear part of the sketch (no feature epilogue, no final sync) on the
// operator's sketched-dimension range [off, off + cnt), cnt = A's extent along
// dim: dim 0 SA (S x other) = S[:, off : off + cnt] A, dim 1 SA (other x S) =
// A S[:, off : off + cnt]^T.  off = 0, cnt = N is the whole application; a
// distributed operand's shard passes its global offset and the ranks' partial
// results sum to the whole (needs_whole kinds take off = 0, cnt = N only).
inline int apply_linear(const slnat::Sketch& s, const DevMat& A, const DevMat& SA, int dim, int64_t off) {
  Lib& L = lib();
  const int dt = A.dtype;
  const size_t es = esize(dt);
  const int64_t cnt = dim == 0 ? A.m : A.n;
  const int64_t other = dim == 0 ? A.n : A.m;
  const int64_t N = s.N, S = s.S;
  void* st = nullptr;
  using namespace slnat;
  if (off < 0 || off + cnt > N || (needs_whole(s) && (off != 0 || cnt != N)))
    return fail(104, "device sketch: operator column range");
  if (other == 0) return 0;
  if (cnt == 0) return zero(SA) ? 106 : 0;
  if (dim == 1 && (s.kind == K_HASH || s.kind == K_SAMPLE || s.kind == K_PPT) && !rowwise_fits(cnt, dt))
    return apply_by_transpose(s, A, SA, off);
  // operator columns k0.. (global) against rows k0 - off.. of A (dim 0) / columns (dim 1)
  auto acc_panel = [&](const void* P, bool p_rowmajor_sxk, int64_t k0, int64_t kb, double beta) -> int {
    // P: S x kb row-major (ld kb) if p_rowmajor_sxk, else kb x S row-major (ld S)
    const int64_t a0 = k0 - off;
    if (dim == 0)
      return gemm_rm(dt, !p_rowmajor_sxk, false, S, other, kb, P, p_rowmajor_sxk ? kb : S,
                     (const char*)A.data + a0 * A.ld * es, A.ld, beta, SA.data, SA.ld);
    return gemm_rm(dt, false, p_rowmajor_sxk, other, S, kb, (const char*)A.data + a0 * es, A.ld, P,
                   p_rowmajor_sxk ? kb : S, beta, SA.data, SA.ld);
  };
  if (s.kind == K_DENSE || s.kind == K_QMC) {
    const int64_t b = std::max<int64_t>(1, std::min<int64_t>(cnt, (int64_t(1) << 24) / std::max<int64_t>(S, 1)));
    Buf P(S * b * (int64_t)es);
    if (!P.p) return fail(101, "device sketch: allocation failed");
    std::vector<double> hp;
    for (int64_t k0 = off; k0 < off + cnt; k0 += b) {
      const int64_t kb = std::min(b, off + cnt - k0);
      if (s.kind == K_DENSE) {
        SLDEV_TRY(L.fill_random(P.p, dt, s.dist, s.seed, s.wbase, S, kb, kb, 1, 0, k0, 1, S, s.p0, 0.0, s.scale,
                                dt == F64 ? 1 : 0, st),
                  "sketch panel");
      } else {
        hp.resize((size_t)(S * kb));
        realise_cols(s, k0, kb, hp.data());   // column-major S x kb = row-major kb x S
        const int rc = upload_as(P, hp.data(), S * kb, dt);
        if (rc) return rc;
      }
      const int rc = acc_panel(P.p, s.kind == K_DENSE, k0, kb, k0 == off ? 0.0 : 1.0);
      if (rc) return rc;
    }
  } else if (s.kind == K_FJLT) {
    Buf dsamp(S * 8), dD(N * 8);
    int rc;
    if ((rc = upload(dsamp, s.samples)) || (rc = upload(dD, s.dsign))) return rc;
    const int64_t pb = std::max<int64_t>(1, std::min<int64_t>(S, (int64_t(1) << 25) / N));
    Buf W(pb * N * (int64_t)es);
    if (!W.p) return fail(101, "device FJLT: allocation failed");
    for (int64_t j0 = 0; j0 < S; j0 += pb) {
      const int64_t nb = std::min(pb, S - j0);
      SLDEV_TRY(L.dct2_rows((const int64_t*)dsamp.p + j0, nb, N, (const double*)dD.p, s.scale, W.p, dt, N, 0, st),
                "fjlt rows");
      // the operator's rows j0.. over all N columns; the shard's range is columns off..
      const char* Wo = (const char*)W.p + off * (int64_t)es;
      rc = dim == 0 ? gemm_rm(dt, false, false, nb, other, cnt, Wo, N, A.data, A.ld, 0.0,
                              (char*)SA.data + j0 * SA.ld * es, SA.ld)
                    : gemm_rm(dt, false, true, other, nb, cnt, A.data, A.ld, Wo, N, 0.0, (char*)SA.data + j0 * es,
                              SA.ld);
      if (rc) return rc;
    }
  } else if (s.kind == K_FASTFOOD) {
    // block b: SA[rows s..e] = F[0:e-s] diag(G_b) (F[perm_b] diag(B_b) A)
    const int64_t NB = N;
    std::vector<int64_t> iota((size_t)NB);
    for (int64_t i = 0; i < NB; ++i) iota[(size_t)i] = i;
    Buf drows(NB * 8), dperm(s.nb * NB * 8), dB(s.nb * NB * 8), dG(s.nb * NB * 8), A2(NB * N * (int64_t)es),
        A1(NB * N * (int64_t)es), T(NB * other * (int64_t)es);
    int rc;
    if ((rc = upload(drows, iota)) || (rc = upload(dperm, s.perms)) || (rc = upload(dB, s.fB)) || (rc = upload(dG, s.fG)))
      return rc;
    if (!A2.p || !A1.p || !T.p) return fail(101, "device Fastfood: allocation failed");
    for (int64_t b = 0; b < s.nb; ++b) {
      const int64_t r0 = b * NB, r1 = std::min(S, r0 + NB), nr = r1 - r0;
      SLDEV_TRY(L.dct2_rows((const int64_t*)dperm.p + b * NB, NB, N, (const double*)dB.p + b * NB, 1.0, A2.p, dt, N, 0,
                            st),
                "fastfood F P B");
      SLDEV_TRY(L.dct2_rows((const int64_t*)drows.p, nr, N, (const double*)dG.p + b * NB, 1.0, A1.p, dt, N, 0, st),
                "fastfood F G");
      if (dim == 0) {
        if ((rc = gemm_rm(dt, false, false, NB, other, N, A2.p, N, A.data, A.ld, 0.0, T.p, other))) return rc;
        if ((rc = gemm_rm(dt, false, false, nr, other, NB, A1.p, N, T.p, other, 0.0, (char*)SA.data + r0 * SA.ld * es,
                          SA.ld)))
          return rc;
      } else {
        if ((rc = gemm_rm(dt, false, true, other, NB, N, A.data, A.ld, A2.p, N, 0.0, T.p, NB))) return rc;
        if ((rc = gemm_rm(dt, false, true, other, nr, NB, T.p, NB, A1.p, N, 0.0, (char*)SA.data + r0 * es, SA.ld)))
          return rc;
      }
    }
  } else if (s.kind == K_HASH || s.kind == K_SAMPLE) {
    if (s.kind == K_HASH) {
      HashDev H(cnt, S);
      const std::vector<int64_t> idx(s.idx.begin() + off, s.idx.begin() + off + cnt);
      const std::vector<double> val(s.val.begin() + off, s.val.begin() + off + cnt);
      const int rc = hash_upload(H, idx, val, S);
      if (rc) return rc;
      if (hash_apply(H, cnt, S, A, SA, dim, 0)) return 106;
    } else {
      // output i = input samples[i]: the bucket structure of a gather (a
      // shard's buckets hold the samples inside its range, the rest are empty)
      std::vector<int64_t> bptr((size_t)S + 1, 0), perm;
      for (int64_t i = 0; i < S; ++i) {
        const int64_t j = s.samples[(size_t)i] - off;
        const bool in = j >= 0 && j < cnt;
        if (in) perm.push_back(j);
        bptr[(size_t)i + 1] = bptr[(size_t)i] + (in ? 1 : 0);
      }
      if (perm.empty()) return zero(SA) ? 106 : 0;
      std::vector<double> ones((size_t)std::max(cnt, S), 1.0);
      Buf dperm((int64_t)perm.size() * 8), dbptr((S + 1) * 8), dones((int64_t)ones.size() * 8);
      int rc;
      if ((rc = upload(dperm, perm)) || (rc = upload(dbptr, bptr)) || (rc = upload(dones, ones))) return rc;
      const Buf& perm_ = dperm;
      if (dim == 0)
        SLDEV_TRY(L.hash_colwise(A.data, dt, A.ld, A.n, (const int64_t*)perm_.p, (const int64_t*)dbptr.p,
                                 (const double*)dones.p, S, SA.data, dt, SA.ld, 0, 0, st),
                  "gather rows");
      else
        SLDEV_TRY(L.hash_rowwise(A.data, dt, A.ld, A.m, cnt, (const int64_t*)perm_.p, (const int64_t*)dbptr.p,
                                 (const double*)dones.p, S, SA.data, dt, SA.ld, 0, 0, st),
                  "gather columns");
    }
  } else {   // PPT: q CountSketches, DFTs as GEMMs, spectrum product, inverse DFT
    const int64_t q = s.q, K = S / 2 + 1;
    if (q == 0) return zero(SA) ? 106 : check(L.dev_sync(st), "sync");
    const int64_t plane = K * other;
    Buf U(S * other * (int64_t)es), F(2 * q * plane * (int64_t)es), P(2 * plane * (int64_t)es), Cm(K * S * (int64_t)es),
        Sm(K * S * (int64_t)es), hidx(q * 8), hval(q * 8);
    if (!U.p || !F.p || !P.p || !Cm.p || !Sm.p) return fail(101, "device PPT: allocation failed");
    int rc;
    if ((rc = upload(hidx, s.hidx)) || (rc = upload(hval, s.hval))) return rc;
    SLDEV_TRY(L.dft_cs(S, K, Cm.p, Sm.p, dt, st), "dft tables");
    const double sg = std::sqrt(s.gamma);
    for (int64_t i = 0; i < q; ++i) {
      HashDev H(N, S);
      std::vector<int64_t> idx(s.pidx.begin() + i * N, s.pidx.begin() + (i + 1) * N);
      std::vector<double> val(s.pval.begin() + i * N, s.pval.begin() + (i + 1) * N);
      if ((rc = hash_upload(H, idx, val, S, sg))) return rc;
      const DevMat Ui = dim == 0 ? DevMat{U.p, dt, S, other, other} : DevMat{U.p, dt, other, S, S};
      if (hash_apply(H, N, S, A, Ui, dim, 0)) return 106;
      char* Fr = (char*)F.p + i * plane * (int64_t)es;
      char* Fi = (char*)F.p + (q + i) * plane * (int64_t)es;
      if (dim == 0) {   // K x other = (K x S)(S x other)
        if ((rc = gemm_rm(dt, false, false, K, other, S, Cm.p, S, U.p, other, 0.0, Fr, other))) return rc;
        if ((rc = gemm_rm(dt, false, false, K, other, S, Sm.p, S, U.p, other, 0.0, Fi, other))) return rc;
      } else {          // other x K = (other x S)(S x K)
        if ((rc = gemm_rm(dt, false, true, other, K, S, U.p, S, Cm.p, S, 0.0, Fr, K))) return rc;
        if ((rc = gemm_rm(dt, false, true, other, K, S, U.p, S, Sm.p, S, 0.0, Fi, K))) return rc;
      }
    }
    const int64_t sk = dim == 0 ? other : 1, sc = dim == 0 ? 1 : K;
    SLDEV_TRY(L.ppt_spectrum(F.p, (int)q, K, other, sk, sc, plane, S, (const int64_t*)hidx.p, (const double*)hval.p,
                             std::sqrt(s.c), P.p, dt, st),
              "ppt spectrum");
    const char* Pr = (const char*)P.p;
    const char* Pi = (const char*)P.p + plane * (int64_t)es;
    if (dim == 0) {   // S x other = C^T Pr - Sn^T Pi
      if ((rc = gemm_rm(dt, true, false, S, other, K, Cm.p, S, Pr, other, 0.0, SA.data, SA.ld))) return rc;
      if ((rc = gemm_rm(dt, true, false, S, other, K, Sm.p, S, Pi, other, 1.0, SA.data, SA.ld, -1.0))) return rc;
    } else {          // other x S = Pr C - Pi Sn
      if ((rc = gemm_rm(dt, false, false, other, S, K, Pr, K, Cm.p, S, 0.0, SA.data, SA.ld))) return rc;
      if ((rc = gemm_rm(dt, false, false, other, S, K, Pi, K, Sm.p, S, 1.0, SA.data, SA.ld, -1.0))) return rc;
    }
  }
  return 0;
}

// SA = S A (dim 0: A is N x n, SA is S x n) or A S^T (dim 1: A is m x N, SA
// is m x S), row-major device operands of one dtype (f32 / f64): every
// sketch type of native_sketch.hpp.
inline int apply_sketch(const slnat::Sketch& s, const DevMat& A, const DevMat& SA, int dim) {
  Lib& L = lib();
  if (!L.loaded) return fail(106, "device C API: " + L.err);
  if ((A.dtype != F32 && A.dtype != F64) || SA.dtype != A.dtype)
    return fail(103, "device sketch: A and SA must both be f32 or both f64");
  const int64_t sk_in = dim == 0 ? A.m : A.n;   // the sketched dimension (N)
  const int64_t other = dim == 0 ? A.n : A.m;
  if (sk_in != s.N || (dim == 0 ? (SA.m != s.S || SA.n != other) : (SA.m != other || SA.n != s.S)))
    return fail(104, "device sketch: dimension mismatch");
  if (other == 0) return 0;
  int rc = apply_linear(s, A, SA, dim, 0);
  if (rc) return rc;
  if ((rc = epilogue_dev(s, SA, dim))) return rc;
  return check(L.dev_sync(nullptr), "sync");
}

// ------------------------------------------ distributed (DistMatrix) operands
// The reference's DistMatrix type names over a device communicator
// (sl_device_comm_create, or a caller's all-reduce via sl_comm_from_allreduce;
// null = one rank): each rank passes its shard of the global m x n matrix in
// the runtime's layouts (parallel/distmatrix.py -- contiguous balanced blocks):
//   LY_ROWS  DistMatrix_VC_STAR / _VR_STAR   rows [b, e) of block_of(m)
//   LY_COLS  DistMatrix_STAR_VC / _STAR_VR   columns [b, e) of block_of(n)
//   LY_STAR  SharedMatrix ([*,*])            the whole matrix on every rank
//   LY_ROOT  RootMatrix ([CIRC,CIRC])        the whole matrix on rank 0
// Only all-reduce is used (the one collective a caller's communicator has).
enum { LY_STAR = 0, LY_ROWS = 1, LY_COLS = 2, LY_ROOT = 3 };

struct DistMat {
  void* data;        // this rank's shard, row-major (ld)
  int dtype;
  int64_t m, n, ld;  // GLOBAL shape; the shard's shape follows from the layout
  void* comm;
};

inline void block_of(int64_t n, int p, int r, int64_t* b, int64_t* e) {
  const int64_t q = n / p, rem = n % p;
  *b = r * q + std::min<int64_t>(r, rem);
  *e = *b + q + (r < rem ? 1 : 0);
}

inline int comm_rank_size(void* comm, int* rank, int* size) {
  if (!comm) {
    *rank = 0;
    *size = 1;
    return 0;
  }
  return check(lib().comm_rank_size(comm, rank, size), "communicator");
}

// shard offset (r0, c0) and shape of a global m x n matrix in layout ly
inline void shard_of(int ly, int64_t m, int64_t n, int rank, int size, int64_t* r0, int64_t* c0, int64_t* lm,
                     int64_t* ln) {
  int64_t b = 0, e = 0;
  *r0 = 0;
  *c0 = 0;
  *lm = m;
  *ln = n;
  if (ly == LY_ROWS) {
    block_of(m, size, rank, &b, &e);
    *r0 = b;
    *lm = e - b;
  } else if (ly == LY_COLS) {
    block_of(n, size, rank, &b, &e);
    *c0 = b;
    *ln = e - b;
  } else if (ly == LY_ROOT && rank != 0) {
    *lm = 0;
    *ln = 0;
  }
}

// in-place sum over the ranks
inline int all_reduce(void* comm, int size, void* buf, int64_t count, int dt) {
  if (!comm || size == 1 || count == 0) return 0;
  SLDEV_TRY(lib().dev_sync(nullptr), "sync");
  SLDEV_TRY(lib().comm_all_reduce(comm, buf, buf, count, dt, 0, nullptr), "all-reduce");
  return check(lib().dev_sync(nullptr), "sync");
}

// rows x cols block: src at (sr, sc) -> dst at (dr, dc)
inline int copy_block(const DevMat& src, int64_t sr, int64_t sc, const DevMat& dst, int64_t dr, int64_t dc, int64_t rows,
                      int64_t cols) {
  if (rows <= 0 || cols <= 0) return 0;
  const int64_t es = (int64_t)esize(src.dtype);
  return check(lib().dev_memcpy2d((char*)dst.data + (dr * dst.ld + dc) * es, dst.ld * es,
                                  (const char*)src.data + (sr * src.ld + sc) * es, src.ld * es, cols * es, rows, 2,
                                  nullptr),
               "copy");
}

// the global matrix on every rank: each shard embedded in zeros, summed
inline int replicate(const DevMat& local, int64_t r0, int64_t c0, int64_t m, int64_t n, void* comm, int size, Buf& out,
                     DevMat* whole) {
  const int dt = local.dtype;
  if (!out.p && m * n > 0) return fail(101, "device sketch: allocation failed");
  *whole = DevMat{out.p, dt, m, n, n};
  if (m * n == 0) return 0;
  SLDEV_TRY(lib().dev_memset(out.p, 0, m * n * (int64_t)esize(dt), nullptr), "memset");
  int rc = copy_block(local, 0, 0, *whole, r0, c0, local.m, local.n);
  if (rc) return rc;
  return all_reduce(comm, size, out.p, m * n, dt);
}

// SA = S A (dim 0) or A S^T (dim 1) with A and SA distributed (layouts in_ly /
// out_ly).  The sketched dimension split over the ranks ([VC,*] columnwise,
// [*,VC] rowwise): every rank applies its column range of the operator to its
// shard and the partial sketches are summed (the random features' cosine
// after the sum); the other dimension split: the shards sketch locally, no
// communication; Fastfood / PPT gather the operand first.  Reference
// sketch/*_Elemental.hpp (the [VC,*] / [*,VR] specialisations).
inline int apply_sketch_dist(const slnat::Sketch& s, int in_ly, const DistMat& A, int out_ly, const DistMat& SA,
                             int dim) {
  Lib& L = lib();
  if (!L.loaded) return fail(106, "device C API: " + L.err);
  const int dt = A.dtype;
  if ((dt != F32 && dt != F64) || SA.dtype != dt) return fail(103, "distributed sketch: A and SA f32 or f64 alike");
  if (A.comm != SA.comm) return fail(109, "distributed sketch: A and SA on different communicators");
  int rank = 0, size = 1;
  int rc = comm_rank_size(A.comm, &rank, &size);
  if (rc) return rc;
  const int64_t om = dim == 0 ? s.S : A.m, on = dim == 0 ? A.n : s.S;
  if ((dim == 0 ? A.m : A.n) != s.N || SA.m != om || SA.n != on)
    return fail(104, "distributed sketch: dimension mismatch");
  int64_t ar0, ac0, alm, aln, or0, oc0, olm, oln;
  shard_of(in_ly, A.m, A.n, rank, size, &ar0, &ac0, &alm, &aln);
  shard_of(out_ly, om, on, rank, size, &or0, &oc0, &olm, &oln);
  const DevMat Al{A.data, dt, alm, aln, A.ld}, SAl{SA.data, dt, olm, oln, SA.ld};
  const bool split_sk = (in_ly == LY_ROWS && dim == 0) || (in_ly == LY_COLS && dim == 1);
  const bool split_other = (in_ly == LY_ROWS && dim == 1) || (in_ly == LY_COLS && dim == 0);
  if (split_other && out_ly == in_ly) return apply_sketch(s, Al, SAl, dim);   // local rows / columns
  // else: the whole result T (om x on) on every rank, then this rank's part of it
  const size_t es = esize(dt);
  Buf Tb(std::max<int64_t>(1, om * on) * (int64_t)es);
  if (!Tb.p) return fail(101, "distributed sketch: allocation failed");
  const DevMat T{Tb.p, dt, om, on, on};
  if (split_sk && !needs_whole(s)) {
    rc = apply_linear(s, Al, T, dim, dim == 0 ? ar0 : ac0);   // this shard's range of the operator
    if (!rc) rc = all_reduce(A.comm, size, T.data, om * on, dt);
    if (!rc) rc = epilogue_dev(s, T, dim);
  } else if (split_other) {
    // the local sketch rows / columns, gathered into T
    int64_t tr0, tc0, tlm, tln;
    shard_of(in_ly, om, on, rank, size, &tr0, &tc0, &tlm, &tln);
    Buf Rb(std::max<int64_t>(1, tlm * tln) * (int64_t)es);
    const DevMat R{Rb.p, dt, tlm, tln, tln};
    rc = tlm * tln > 0 ? apply_sketch(s, Al, R, dim) : 0;
    if (!rc) {
      SLDEV_TRY(L.dev_memset(T.data, 0, om * on * (int64_t)es, nullptr), "memset");
      rc = copy_block(R, 0, 0, T, tr0, tc0, tlm, tln);
    }
    if (!rc) rc = all_reduce(A.comm, size, T.data, om * on, dt);
  } else {
    // [*,*] / [CIRC,CIRC] inputs, or a kind that needs the whole operand
    DevMat W = Al;
    Buf Wb(in_ly == LY_STAR ? 0 : std::max<int64_t>(1, A.m * A.n) * (int64_t)es);
    if (in_ly != LY_STAR) rc = replicate(Al, ar0, ac0, A.m, A.n, A.comm, size, Wb, &W);
    if (!rc) rc = apply_sketch(s, W, T, dim);
  }
  if (rc) return rc;
  rc = copy_block(T, or0, oc0, SAl, 0, 0, olm, oln);
  if (rc) return rc;
  return check(L.dev_sync(nullptr), "sync");
}

// CSR on the device (rowptr int64, col int32, val f64): rows x cols.
struct DevCsr {
  const int64_t* rowptr;
  const int* col;
  const double* val;
  int64_t rows, cols, nnz;
  const int* rowptr32;   // the same row pointers as int32 (densify kernel)
};

// SA (f64 row-major) = sketch of the CSR matrix along dim; hash sketches run
// on the CSR directly, the rest on its dense form
inline int apply_sketch_csr(const slnat::Sketch& s, const DevCsr& A, const DevMat& SA, int dim) {
  Lib& L = lib();
  using namespace slnat;
  const int64_t sk_in = dim == 0 ? A.rows : A.cols, other = dim == 0 ? A.cols : A.rows;
  if (sk_in != s.N || (dim == 0 ? (SA.m != s.S || SA.n != other) : (SA.m != other || SA.n != s.S)))
    return fail(104, "device sketch: dimension mismatch");
  if (s.kind == K_HASH && SA.dtype == F64) {
    HashDev H(s.N, s.S);
    int rc = hash_upload(H, s.idx, s.val, s.S);
    if (rc) return rc;
    if (zero(SA)) return 106;
    const int64_t avg = A.rows ? A.nnz / A.rows : 0;
    if (dim == 0) {
      const int group = avg >= 48 ? 64 : avg >= 12 ? 16 : avg >= 3 ? 4 : 1;
      SLDEV_TRY(L.hash_csr_col(A.rowptr, A.col, 1, A.val, F64, (const int64_t*)H.perm.p, (const int64_t*)H.bptr.p,
                               H.pval.p, s.S, A.cols, SA.data, SA.ld, 0, group, 0, nullptr, 0.0, nullptr),
                "hash csr colwise");
    } else {
      SLDEV_TRY(L.hash_csr_row(A.rowptr, A.col, 1, A.val, F64, A.rows, (const int64_t*)H.idx.p, (const double*)H.val.p,
                               SA.data, SA.ld, 0, 1, nullptr),
                "hash csr rowwise");
    }
    return check(L.dev_sync(nullptr), "sync");
  }
  Buf D(A.rows * A.cols * 8);
  if (!D.p) return fail(101, "device sketch: allocation failed (dense form of the sparse input)");
  SLDEV_TRY(L.dev_memset(D.p, 0, A.rows * A.cols * 8, nullptr), "memset");
  SLDEV_TRY(L.csr_to_dense(A.rowptr32, A.col, A.val, A.rows, D.p, F64, A.cols, nullptr), "densify");
  return apply_sketch(s, DevMat{D.p, F64, A.rows, A.cols, A.cols}, SA, dim);
}

// ------------------------------------------- host operands staged to the GPU
// A "Matrix" (column-major m x n) is the row-major n x m A^T on the device, so
// sketching dim d of A is sketching dim 1 - d of that view, and the row-major
// result is the column-major SA: no transposes, one copy each way.
inline int apply_host_dense(const slnat::Sketch& s, const double* A, int64_t m, int64_t n, double* SA, int64_t sm,
                            int64_t sn, int dim) {
  Lib& L = lib();
  if (dim == 0 ? (m != s.N || sm != s.S || sn != n) : (n != s.N || sn != s.S || sm != m))
    return fail(104, "sl_apply_sketch_transform: dimension mismatch");
  Buf dA(std::max<int64_t>(1, m * n) * 8), dS(std::max<int64_t>(1, sm * sn) * 8);
  if (!dA.p || !dS.p) return fail(101, "device sketch: allocation failed");
  SLDEV_TRY(L.dev_memcpy(dA.p, A, m * n * 8, 0, nullptr), "copy");
  const int rc = apply_sketch(s, DevMat{dA.p, F64, n, m, m}, DevMat{dS.p, F64, sn, sm, sm}, 1 - dim);
  if (rc) return rc;
  SLDEV_TRY(L.dev_memcpy(SA, dS.p, sm * sn * 8, 1, nullptr), "copy");
  return check(L.dev_sync(nullptr), "sync");
}

// A "SparseMatrix" (CSC of m x n) is the CSR of the n x m A^T
inline int apply_host_csc(const slnat::Sketch& s, const int* indptr, const int* ind, const double* val, int64_t nnz,
                          int64_t m, int64_t n, double* SA, int64_t sm, int64_t sn, int dim) {
  Lib& L = lib();
  if (dim == 0 ? (m != s.N || sm != s.S || sn != n) : (n != s.N || sn != s.S || sm != m))
    return fail(104, "sl_apply_sketch_transform: dimension mismatch");
  std::vector<int64_t> rp64((size_t)n + 1);
  for (int64_t j = 0; j <= n; ++j) rp64[(size_t)j] = indptr[j];
  Buf drp(rp64.size() * 8), drp32((n + 1) * 4), dcol(std::max<int64_t>(1, nnz) * 4), dval(std::max<int64_t>(1, nnz) * 8),
      dS(std::max<int64_t>(1, sm * sn) * 8);
  int rc = upload(drp, rp64);
  if (rc) return rc;
  if (!drp32.p || !dcol.p || !dval.p || !dS.p) return fail(101, "device sketch: allocation failed");
  SLDEV_TRY(L.dev_memcpy(drp32.p, indptr, (n + 1) * 4, 0, nullptr), "copy");
  if (nnz) {
    SLDEV_TRY(L.dev_memcpy(dcol.p, ind, nnz * 4, 0, nullptr), "copy");
    SLDEV_TRY(L.dev_memcpy(dval.p, val, nnz * 8, 0, nullptr), "copy");
  }
  const DevCsr C{(const int64_t*)drp.p, (const int*)dcol.p, (const double*)dval.p, n, m, nnz, (const int*)drp32.p};
  rc = apply_sketch_csr(s, C, DevMat{dS.p, F64, sn, sm, sm}, 1 - dim);
  if (rc) return rc;
  SLDEV_TRY(L.dev_memcpy(SA, dS.p, sm * sn * 8, 1, nullptr), "copy");
  return check(L.dev_sync(nullptr), "sync");
}

// ---------------------------------------------------------------- randSVD
struct SvdParams {
  int ratio = 2, additive = 0, iters = 0;
  bool skip_qr = false;
  std::string sketch = "JLT";
};

inline SvdParams parse_svd_params(const char* js) {
  SvdParams p;
  if (!js || !*js) return p;
  double v;
  if (slnat::get_number(js, "oversampling_ratio", v)) p.ratio = (int)v;
  if (slnat::get_number(js, "oversampling_additive", v)) p.additive = (int)v;
  if (slnat::get_number(js, "num_iterations", v)) p.iters = (int)v;
  slnat::get_bool(js, "skip_qr", p.skip_qr);
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
// of bf16 A (m x n, m >= n) on the fused engine (16 <= n <= 1024, k <= 48;
// otherwise, and for f32 / f64 A, the general engine: approximate_svd_gen).
// ctr: the context counter (advanced by the sketch's draws exactly as the
// runtime advances it).  comm (a NativeComm
// RCCL communicator, sl_device_comm_create): A is this rank's row shard of a
// row-distributed matrix (every rank the same n), U its rows of the left
// factor, S and V replicated; the [W; G] pass sums are all-reduced over RCCL
// between the engine's segments (sl_rsvd_run_comm).
// f32 / f64 A on the general engine (rsvd_general.hip: hand-written products
// for k <= 128): U (m x rank), S (rank) and V (n x rank) in A's dtype; comm:
// A is this rank's row shard, the [W; G] spans all-reduced per segment
// (sl_rsvd_gen_run_comm).  Same operator streams as the runtime.
inline int approximate_svd_gen(const DevMat& A, const DevMat& U, const DevMat& Sv, const DevMat& V, int rank,
                               const char* params, uint64_t seed, uint64_t& ctr, void* comm) {
  Lib& L = lib();
  const int dt = A.dtype;
  const int udt = dt == BF16 ? F32 : dt;
  if (U.dtype != udt || Sv.dtype != udt || V.dtype != udt)
    return fail(103, "device approximate_svd: U, S, V in A's dtype (f32 for bf16 A)");
  const int64_t m = A.m, n = A.n;
  if (m < n && !comm) return fail(103, "device approximate_svd: needs a tall A (m >= n); pass A^T and swap U / V");
  if (rank < 1 || rank > n) return fail(109, "device approximate_svd: bad rank");
  const SvdParams p = parse_svd_params(params);
  const int k = (int)std::max<int64_t>(rank, std::min<int64_t>(n, (int64_t)p.ratio * rank + p.additive));
  if (k > 128) return fail(103, "device approximate_svd: the general engine covers k <= 128");
  if (U.m != m || U.n != rank || V.m != n || V.n != rank || V.ld != rank || Sv.m * Sv.n != rank)
    return fail(104, "device approximate_svd: output shapes");
  if (p.sketch != "JLT" && p.sketch != "CT" && p.sketch != "FJLT" && p.sketch != "CWT")
    return fail(109, "device approximate_svd: sketch must be JLT, CT, FJLT or CWT");
  const int q = std::max(0, p.iters);
  void* plan = nullptr;
  SLDEV_TRY(L.gen_create(m, n, A.ld, k, rank, q, dt, &plan), "rsvd plan");
  struct Guard {
    void* p;
    ~Guard() { lib().gen_destroy(p); }
  } guard{plan};
  const uint64_t base = ctr;
  if (p.sketch == "JLT" || p.sketch == "CT") {
    const bool jlt = p.sketch == "JLT";
    SLDEV_TRY(L.gen_set_dense(plan, jlt ? sl::DIST_NORMAL : sl::DIST_CAUCHY, seed, base, 0.0, 0.0,
                              jlt ? std::sqrt(1.0 / k) : 1.0 / k),
              "sketch operator");
    ctr = base + (uint64_t)(n * k);
  } else if (p.sketch == "FJLT") {
    SLDEV_TRY(L.gen_set_fjlt(plan, seed, base, base + (uint64_t)n, std::sqrt((double)n / k)), "sketch operator");
    ctr = base + (uint64_t)(n + k);
  } else {
    slnat::Sketch cw;
    cw.type = "CWT";
    cw.N = n;
    cw.S = k;
    cw.seed = seed;
    cw.ctr0 = base;
    ctr = slnat::build(cw);
    std::vector<double> z((size_t)(n * k), 0.0);   // Z = Omega^T (n x k)
    for (int64_t j = 0; j < n; ++j) z[(size_t)(j * k + cw.idx[(size_t)j])] = cw.val[(size_t)j];
    Buf dz(n * k * (int64_t)esize(dt));
    const int rc = upload_as(dz, z.data(), n * k, dt);
    if (rc) return rc;
    SLDEV_TRY(L.gen_set_z(plan, dz.p, nullptr), "sketch operator");
    SLDEV_TRY(L.dev_sync(nullptr), "sync");
  }
  if (comm)
    SLDEV_TRY(L.gen_run_comm(plan, A.data, comm, U.data, U.ld, Sv.data, V.data, nullptr), "rsvd run (comm)");
  else
    SLDEV_TRY(L.gen_run(plan, A.data, U.data, U.ld, Sv.data, V.data, nullptr), "rsvd run");
  int status = 0;
  SLDEV_TRY(L.gen_status(plan, &status, nullptr), "rsvd status");
  if (status & 2) return fail(108, "device approximate_svd: non-finite values in A");
  return check(L.dev_sync(nullptr), "sync");
}

inline int approximate_svd(const DevMat& A, const DevMat& U, const DevMat& Sv, const DevMat& V, int rank,
                           const char* params, uint64_t seed, uint64_t& ctr, void* comm = nullptr) {
  Lib& L = lib();
  if (!L.loaded) return fail(106, "device C API: " + L.err);
  if (A.dtype == F32 || A.dtype == F64) return approximate_svd_gen(A, U, Sv, V, rank, params, seed, ctr, comm);
  if (A.dtype != BF16) return fail(103, "device approximate_svd: A must be bf16, f32 or f64");
  if (U.dtype != F32 || Sv.dtype != F32 || V.dtype != F32) return fail(103, "device approximate_svd: U, S, V are f32");
  const int64_t m = A.m, n = A.n;
  if (m < n && !comm) return fail(103, "device approximate_svd: needs a tall A (m >= n); pass A^T and swap U / V");
  if (rank < 1 || rank > n) return fail(109, "device approximate_svd: bad rank");
  const SvdParams p = parse_svd_params(params);
  const int k = (int)std::max<int64_t>(rank, std::min<int64_t>(n, (int64_t)p.ratio * rank + p.additive));
  if (U.m != m || U.n != rank || V.m != n || V.n != rank || V.ld != rank || Sv.m * Sv.n != rank)
    return fail(104, "device approximate_svd: output shapes");
  if (n % 8 || n < 16 || n > 1024 || A.ld % 8 || k > 48)   // beyond the fused engine: the general one
    return approximate_svd_gen(A, U, Sv, V, rank, params, seed, ctr, comm);
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


// ------------------------------------------ NLA on host ("Matrix") operands
// Return value HOST_DECLINED: the call is outside the native coverage and the
// caller runs it on the runtime instead.
constexpr int HOST_DECLINED = -1;

// column-major host (m x n, ld m) <- row-major device-order host buffer (m x n, ld n)
inline void rm_to_cm(const double* rm, int64_t m, int64_t n, double* cm) {
  for (int64_t i = 0; i < m; ++i)
    for (int64_t j = 0; j < n; ++j) cm[i + j * m] = rm[i * n + j];
}

// ApproximateSVD of a column-major host A (m x n): U (m x rank), s (rank), V
// (n x rank), column-major.  The tall operand (A, or A^T for m < n) runs on
// the general-precision device engine in f64 with the sketch drawn from
// (seed, ctr) exactly as the runtime draws it (nla/svd.py
// _approximate_svd_device): JLT / CT dense, FJLT, CWT explicit.
inline int approximate_svd_host(const double* A, int64_t m, int64_t n, double* U, double* s, double* V, int rank,
                                const char* params, uint64_t seed, uint64_t& ctr) {
  Lib& L = lib();
  if (rank < 1 || rank > std::min(m, n)) return fail(109, "approximate_svd: incompatible matrix dimensions and rank");
  const SvdParams p = parse_svd_params(params);
  const bool tall = m >= n;
  const int64_t M = tall ? m : n, Nn = tall ? n : m;   // the tall operand T (M x Nn)
  const int k = (int)std::max<int64_t>(rank, std::min<int64_t>(Nn, (int64_t)p.ratio * rank + p.additive));
  if (k > 128 || k > Nn) return HOST_DECLINED;
  if (p.sketch != "JLT" && p.sketch != "CT" && p.sketch != "FJLT" && p.sketch != "CWT")
    return fail(109, "approximate_svd: sketch must be JLT, CT, FJLT or CWT");
  const int q = std::max(0, p.iters);
  Buf dA(m * n * 8), dT(tall ? m * n * 8 : 8), dU(M * rank * 8), dS(rank * 8), dV(Nn * rank * 8);
  if (!dA.p || !dT.p || !dU.p || !dS.p || !dV.p) return fail(101, "approximate_svd: device allocation failed");
  SLDEV_TRY(L.dev_memcpy(dA.p, A, m * n * 8, 0, nullptr), "copy");
  // the upload is the row-major n x m A^T: tall A needs the transpose
  const void* T = dA.p;
  if (tall) {
    SLDEV_TRY(L.transpose(dA.p, F64, n, m, m, dT.p, n, nullptr), "transpose");
    T = dT.p;
  }
  void* plan = nullptr;
  SLDEV_TRY(L.gen_create(M, Nn, Nn, k, rank, q, F64, &plan), "rsvd plan");
  struct Guard {
    void* p;
    ~Guard() { lib().gen_destroy(p); }
  } guard{plan};
  const uint64_t base = ctr;
  if (p.sketch == "JLT" || p.sketch == "CT") {
    const bool jlt = p.sketch == "JLT";
    SLDEV_TRY(L.gen_set_dense(plan, jlt ? sl::DIST_NORMAL : sl::DIST_CAUCHY, seed, base, 0.0, 0.0,
                              jlt ? std::sqrt(1.0 / k) : 1.0 / k),
              "sketch operator");
    ctr = base + (uint64_t)(Nn * k);
  } else if (p.sketch == "FJLT") {
    SLDEV_TRY(L.gen_set_fjlt(plan, seed, base, base + (uint64_t)Nn, std::sqrt((double)Nn / k)), "sketch operator");
    ctr = base + (uint64_t)(Nn + k);
  } else {
    slnat::Sketch cw;
    cw.type = "CWT";
    cw.N = Nn;
    cw.S = k;
    cw.seed = seed;
    cw.ctr0 = base;
    ctr = slnat::build(cw);
    std::vector<double> z((size_t)(Nn * k), 0.0);   // Z = Omega^T (Nn x k)
    for (int64_t j = 0; j < Nn; ++j) z[(size_t)(j * k + cw.idx[(size_t)j])] = cw.val[(size_t)j];
    Buf dz(Nn * k * 8);
    const int rc = upload(dz, z);
    if (rc) return rc;
    SLDEV_TRY(L.gen_set_z(plan, dz.p, nullptr), "sketch operator");
    SLDEV_TRY(L.dev_sync(nullptr), "sync");
  }
  SLDEV_TRY(L.gen_run(plan, T, dU.p, rank, dS.p, dV.p, nullptr), "rsvd run");
  int status = 0;
  SLDEV_TRY(L.gen_status(plan, &status, nullptr), "rsvd status");
  if (status & 2) return fail(108, "approximate_svd: non-finite values in A");
  std::vector<double> hU((size_t)(M * rank)), hV((size_t)(Nn * rank));
  SLDEV_TRY(L.dev_memcpy(hU.data(), dU.p, M * rank * 8, 1, nullptr), "copy");
  SLDEV_TRY(L.dev_memcpy(hV.data(), dV.p, Nn * rank * 8, 1, nullptr), "copy");
  SLDEV_TRY(L.dev_memcpy(s, dS.p, rank * 8, 1, nullptr), "copy");
  SLDEV_TRY(L.dev_sync(nullptr), "sync");
  rm_to_cm(hU.data(), M, rank, tall ? U : V);
  rm_to_cm(hV.data(), Nn, rank, tall ? V : U);
  return 0;
}

// ApproximateSymmetricSVD of the column-major host A (n x n, lower triangle
// read): V (n x rank), s (rank), column-major (sl_nat_sym_rsvd)
inline int approximate_symmetric_svd_host(const double* A, int64_t n, double* s, double* V, int rank,
                                          const char* params, uint64_t seed, uint64_t& ctr) {
  Lib& L = lib();
  if (rank < 1 || rank > n) return fail(109, "approximate_symmetric_svd: incompatible matrix dimensions and rank");
  const SvdParams p = parse_svd_params(params);
  const int k = (int)std::max<int64_t>(rank, std::min<int64_t>(n, (int64_t)p.ratio * rank + p.additive));
  Buf dA(n * n * 8), dV(n * rank * 8), dS(rank * 8);
  if (!dA.p || !dV.p || !dS.p) return fail(101, "approximate_symmetric_svd: device allocation failed");
  SLDEV_TRY(L.dev_memcpy(dA.p, A, n * n * 8, 0, nullptr), "copy");
  SLDEV_TRY(L.sym_rsvd((const double*)dA.p, n, n, 1, k, rank, std::max(0, p.iters), p.skip_qr ? 1 : 0, seed, ctr,
                       (double*)dV.p, n, (double*)dS.p, nullptr),
            "symmetric randSVD");
  ctr += (uint64_t)(n * k);
  SLDEV_TRY(L.dev_memcpy(V, dV.p, n * rank * 8, 1, nullptr), "copy");
  SLDEV_TRY(L.dev_memcpy(s, dS.p, rank * 8, 1, nullptr), "copy");
  return check(L.dev_sync(nullptr), "sync");
}

// FasterLeastSquares (Blendenpik) of the column-major host A (m x n; orientation
// 1: solve with A^T), B (rows x nrhs), X (cols x nrhs) (sl_nat_blendenpik)
inline int faster_least_squares_host(int orientation, const double* A, int64_t m, int64_t n, const double* B,
                                     int64_t bm, int64_t bn, double* X, int64_t xm, int64_t xn, const char* params,
                                     uint64_t seed, uint64_t& ctr) {
  Lib& L = lib();
  const bool adj = orientation != 0;
  const int64_t rows = adj ? n : m, cols = adj ? m : n;
  if (bm != rows || xm != cols || xn != bn) return fail(104, "faster_least_squares: dimension mismatch");
  if (rows < cols) return HOST_DECLINED;
  double tol = 1e-14, v;
  int iter_lim = 100;
  if (params && *params) {
    if (slnat::get_number(params, "tolerance", v)) tol = v;
    if (slnat::get_number(params, "iter_lim", v)) iter_lim = (int)v;
  }
  Buf dA(m * n * 8), dO(adj ? m * n * 8 : 8), dB(bm * bn * 8), dX(xm * xn * 8);
  if (!dA.p || !dO.p || !dB.p || !dX.p) return fail(101, "faster_least_squares: device allocation failed");
  SLDEV_TRY(L.dev_memcpy(dA.p, A, m * n * 8, 0, nullptr), "copy");
  SLDEV_TRY(L.dev_memcpy(dB.p, B, bm * bn * 8, 0, nullptr), "copy");
  const void* op = dA.p;
  if (adj) {   // column-major A^T (n x m) = the row-major transpose of the uploaded row-major A^T
    SLDEV_TRY(L.transpose(dA.p, F64, n, m, m, dO.p, n, nullptr), "transpose");
    op = dO.p;
  }
  int code = 0;
  SLDEV_TRY(L.blendenpik((const double*)op, rows, cols, rows, (const double*)dB.p, (int)bn, bm, (double*)dX.p, xm, seed,
                         &ctr, tol, iter_lim, &code, nullptr),
            "faster least squares");
  SLDEV_TRY(L.dev_memcpy(X, dX.p, xm * xn * 8, 1, nullptr), "copy");
  return check(L.dev_sync(nullptr), "sync");
}

// ApproximateSymmetricSVD of a DistMatrix A ([VC,*] / [VR,*] f64 rows of the
// symmetric n x n A, lower triangle read as the reference's El::LOWER): S
// (rank) replicated, V (n x rank) replicated ([*,*]) or in A's rows
// (sl_nat_sym_rsvd_comm: one n x k all-reduce per application of A).
inline int approximate_symmetric_svd_dist(const DistMat& A, const DistMat& Sv, int v_ly, const DistMat& V, int rank,
                                          const char* params, uint64_t seed, uint64_t& ctr) {
  Lib& L = lib();
  if (!L.loaded) return fail(106, "device C API: " + L.err);
  if (A.dtype != F64 || Sv.dtype != F64 || V.dtype != F64) return fail(103, "approximate_symmetric_svd: f64 operands");
  if (Sv.comm != A.comm || V.comm != A.comm) return fail(109, "approximate_symmetric_svd: operands on different communicators");
  const int64_t n = A.n;
  if (A.m != n) return fail(109, "approximate_symmetric_svd: matrix is not square -- symmetric matrix required");
  if (rank < 1 || rank > n) return fail(109, "approximate_symmetric_svd: incompatible matrix dimensions and rank");
  if (V.m != n || V.n != rank || Sv.m * Sv.n != rank) return fail(104, "approximate_symmetric_svd: output shapes");
  const SvdParams p = parse_svd_params(params);
  const int k = (int)std::max<int64_t>(rank, std::min<int64_t>(n, (int64_t)p.ratio * rank + p.additive));
  int rnk = 0, size = 1;
  int rc = comm_rank_size(A.comm, &rnk, &size);
  if (rc) return rc;
  int64_t r0, c0, lm, ln;
  shard_of(LY_ROWS, n, n, rnk, size, &r0, &c0, &lm, &ln);
  Buf Vc(n * rank * 8), Vr(n * rank * 8);
  if (!Vc.p || !Vr.p) return fail(101, "approximate_symmetric_svd: device allocation failed");
  SLDEV_TRY(L.sym_rsvd_comm((const double*)A.data, lm, n, A.ld, r0, 1, k, rank, std::max(0, p.iters),
                            p.skip_qr ? 1 : 0, seed, ctr, (double*)Vc.p, n, (double*)Sv.data, A.comm, nullptr),
            "symmetric randSVD");
  ctr += (uint64_t)(n * k);
  // V row-major (n x rank) = the transpose of the column-major result, then this rank's part
  SLDEV_TRY(L.transpose(Vc.p, F64, rank, n, n, Vr.p, rank, nullptr), "transpose");
  int64_t vr0, vc0, vlm, vln;
  shard_of(v_ly, n, rank, rnk, size, &vr0, &vc0, &vlm, &vln);
  rc = copy_block(DevMat{Vr.p, F64, n, rank, rank}, vr0, vc0, DevMat{V.data, F64, vlm, vln, V.ld}, 0, 0, vlm, vln);
  if (rc) return rc;
  return check(L.dev_sync(nullptr), "sync");
}

// FasterLeastSquares on DistMatrix operands: A (mg x n) and B (mg x nrhs) as
// [VC,*] / [VR,*] f64 device shards (row-major), X (n x nrhs) replicated
// ([*,*]); the same sketch-and-precondition LSQR as the host path with the
// sketch and A^T u summed over A's communicator (sl_nat_blendenpik_comm).
inline int faster_least_squares_dist(const DistMat& A, const DistMat& B, const DistMat& X, const char* params,
                                     uint64_t seed, uint64_t& ctr) {
  Lib& L = lib();
  if (!L.loaded) return fail(106, "device C API: " + L.err);
  if (A.dtype != F64 || B.dtype != F64 || X.dtype != F64) return fail(103, "faster_least_squares: f64 operands");
  if (B.comm != A.comm || X.comm != A.comm) return fail(109, "faster_least_squares: operands on different communicators");
  if (B.m != A.m || X.m != A.n || X.n != B.n) return fail(104, "faster_least_squares: dimension mismatch");
  if (A.m < A.n) return fail(103, "faster_least_squares: distributed A must be overdetermined (m >= n)");
  double tol = 1e-14, v;
  int iter_lim = 100;
  if (params && *params) {
    if (slnat::get_number(params, "tolerance", v)) tol = v;
    if (slnat::get_number(params, "iter_lim", v)) iter_lim = (int)v;
  }
  int rank = 0, size = 1;
  int rc = comm_rank_size(A.comm, &rank, &size);
  if (rc) return rc;
  int64_t r0, c0, lm, ln;
  shard_of(LY_ROWS, A.m, A.n, rank, size, &r0, &c0, &lm, &ln);
  const int64_t n = A.n, nrhs = B.n;
  // column-major shards: the row-major transposes
  Buf At(std::max<int64_t>(1, lm * n) * 8), Bt(std::max<int64_t>(1, lm * nrhs) * 8), Xc(n * nrhs * 8);
  if (!At.p || !Bt.p || !Xc.p) return fail(101, "faster_least_squares: device allocation failed");
  if (lm > 0) {
    SLDEV_TRY(L.transpose(A.data, F64, lm, n, A.ld, At.p, lm, nullptr), "transpose");
    SLDEV_TRY(L.transpose(B.data, F64, lm, nrhs, B.ld, Bt.p, lm, nullptr), "transpose");
  }
  int code = 0;
  SLDEV_TRY(L.blendenpik_comm((const double*)At.p, lm, n, std::max<int64_t>(lm, 1), (const double*)Bt.p, (int)nrhs,
                              std::max<int64_t>(lm, 1), (double*)Xc.p, n, A.m, r0, A.comm, seed, &ctr, tol, iter_lim,
                              &code, nullptr),
            "faster least squares");
  // X (row-major n x nrhs) = the transpose of the column-major result
  SLDEV_TRY(L.transpose(Xc.p, F64, nrhs, n, n, X.data, X.ld, nullptr), "transpose");
  return check(L.dev_sync(nullptr), "sync");
}

// ------------------------------------------------------------- LIBSVM input
struct Libsvm {
  std::vector<double> labels, vals;
  std::vector<int64_t> rowptr, cols;
  int64_t rows = 0, d = 0;
};

inline int read_libsvm(const char* fname, int64_t min_d, int64_t max_n, Libsvm& out) {
  Lib& L = lib();
  FILE* f = fopen(fname, "rb");
  if (!f) return fail(107, std::string("readlibsvm: cannot open ") + fname);
  std::vector<char> buf;
  char tmp[1 << 16];
  size_t got;
  while ((got = fread(tmp, 1, sizeof tmp, f)) > 0) buf.insert(buf.end(), tmp, tmp + got);
  fclose(f);
  const int nt = 16;
  int64_t stats[4] = {0, 0, 0, 0}, ranges[2 * nt], counts[2 * nt];
  int nch = 0;
  if (!buf.empty()) {
    if (L.libsvm_scan(buf.data(), (int64_t)buf.size(), nt, stats, ranges, counts, &nch))
      return fail(107, std::string("readlibsvm: ") + L.last_error());
  }
  const int64_t rows = max_n < 0 ? stats[0] : std::min<int64_t>(stats[0], max_n);
  out.labels.assign((size_t)rows, 0.0);
  out.rowptr.assign((size_t)rows + 1, 0);
  out.cols.assign((size_t)stats[1], 0);
  out.vals.assign((size_t)stats[1], 0.0);
  if (nch)
    L.libsvm_fill(buf.data(), ranges, counts, nch, max_n, out.labels.data(), out.rowptr.data(), out.cols.data(),
                  out.vals.data());
  out.rows = rows;
  out.d = std::max<int64_t>(stats[2], min_d);
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
  const bool xr = dirX != 1, yr = dirY != 1;   // 1 = SL_COLUMNS, anything else rows
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

// Host "Matrix" operands (column-major, f64) staged to the GPU, the same way
// apply_host_dense stages a sketch operand (reference capi/ckernel.cpp:34-128
// runs sl_kernel_gram on host matrices natively): a column-major m x n X is
// the row-major n x m X^T on the device, so its points flip direction (dir 1
// "columns" -> rows of the uploaded view), and the column-major K (#X x #Y)
// is the row-major K^T = Gram(Y, X) -- every kernel here is symmetric in its
// two arguments -- so nothing is transposed.  One copy each way.
inline int kernel_gram_host(const Kern& kk, int dirX, int dirY, const double* X, int64_t xm, int64_t xn,
                            const double* Y, int64_t ym, int64_t yn, double* K, int64_t km, int64_t kn) {
  Lib& L = lib();
  // SL_COLUMNS (1): points are the columns; any other value: rows (reference ckernel.cpp:112-115)
  const int64_t nx = dirX == 1 ? xn : xm, ny = dirY == 1 ? yn : ym;
  if (km != nx || kn != ny) return fail(104, "sl_kernel_gram: K must be (#X points) x (#Y points)");
  Buf dX(std::max<int64_t>(1, xm * xn) * 8), dY(std::max<int64_t>(1, ym * yn) * 8),
      dK(std::max<int64_t>(1, km * kn) * 8);
  if (!dX.p || !dY.p || !dK.p) return fail(101, "sl_kernel_gram: device allocation failed");
  SLDEV_TRY(L.dev_memcpy(dX.p, X, xm * xn * 8, 0, nullptr), "copy");
  if (Y != X || ym != xm || yn != xn) SLDEV_TRY(L.dev_memcpy(dY.p, Y, ym * yn * 8, 0, nullptr), "copy");
  const void* yd = (Y == X && ym == xm && yn == xn) ? dX.p : dY.p;
  // uploaded views: row-major xn x xm (points = rows iff dirX == 1), likewise Y
  const DevMat Xv{dX.p, F64, xn, xm, xm}, Yv{const_cast<void*>(yd), F64, yn, ym, ym};
  const DevMat Kv{dK.p, F64, kn, km, km};
  const int rc = kernel_gram(kk, dirY == 1 ? 2 : 1, dirX == 1 ? 2 : 1, Yv, Xv, Kv);
  if (rc) return rc;
  SLDEV_TRY(L.dev_memcpy(K, dK.p, km * kn * 8, 1, nullptr), "copy");
  return check(L.dev_sync(nullptr), "sync");
}

}  // namespace sldev
