// Plain library BLAS / LAPACK on the device for the general-precision paths:
// rocBLAS GEMMs and rocSOLVER dense factorisations / eigensolvers, resolved at
// run time (dlopen, no link-time dependency) with one handle per device.
// Hot fused kernels are hand-written elsewhere; these are the plain library
// products (GUIDE: hipBLASLt/rocBLAS only for plain library GEMMs).
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <mutex>
#include <string>

#include "sl_blas.hpp"

namespace {

struct Blas {
  bool tried = false, ok = false;
  std::string err;
  void* rb = nullptr;
  void* rs = nullptr;
  int (*create)(void**) = nullptr;
  int (*set_stream)(void*, hipStream_t) = nullptr;
  int (*dgemm)(void*, int, int, int, int, int, const double*, const double*, int, const double*, int, const double*,
               double*, int) = nullptr;
  int (*sgemm)(void*, int, int, int, int, int, const float*, const float*, int, const float*, int, const float*,
               float*, int) = nullptr;
  int (*gemm_ex)(void*, int, int, int, int, int, const void*, const void*, int, int, const void*, int, int,
                 const void*, const void*, int, int, void*, int, int, int, int, int, uint32_t) = nullptr;
  int (*dsyevd)(void*, int, int, int, double*, int, double*, double*, int*) = nullptr;
  int (*dtrtri)(void*, int, int, int, double*, int, int*) = nullptr;
  int (*dgeqrf)(void*, int, int, double*, int, double*) = nullptr;
  int (*dorgqr)(void*, int, int, int, double*, int, double*) = nullptr;
  int (*dgesvd)(void*, int, int, int, int, double*, int, double*, double*, int, double*, int, double*, int,
                int*) = nullptr;
  int (*dgemv)(void*, int, int, int, const double*, const double*, int, const double*, int, const double*, double*,
               int) = nullptr;
  int (*dnrm2)(void*, int, const double*, int, double*) = nullptr;
  int (*dgemm_sb)(void*, int, int, int, int, int, const double*, const double*, int, int64_t, const double*, int,
                  int64_t, const double*, double*, int, int64_t, int) = nullptr;
  int (*sgemm_sb)(void*, int, int, int, int, int, const float*, const float*, int, int64_t, const float*, int,
                  int64_t, const float*, float*, int, int64_t, int) = nullptr;
  int (*dtrsv)(void*, int, int, int, int, const double*, int, double*, int) = nullptr;
  int (*gemm_sb_ex)(void*, int, int, int, int, int, const void*, const void*, int, int, int64_t, const void*, int, int,
                    int64_t, const void*, const void*, int, int, int64_t, void*, int, int, int64_t, int, int, int, int,
                    uint32_t) = nullptr;
  void* handle[64] = {};
};

Blas& blas() {
  static Blas B;
  static std::mutex mu;
  std::lock_guard<std::mutex> g(mu);
  if (B.tried) return B;
  B.tried = true;
  B.rb = dlopen("librocblas.so", RTLD_NOW | RTLD_GLOBAL);
  if (!B.rb) B.rb = dlopen("/opt/rocm/lib/librocblas.so", RTLD_NOW | RTLD_GLOBAL);
  if (!B.rb) { B.err = "cannot load librocblas.so"; return B; }
  B.rs = dlopen("librocsolver.so", RTLD_NOW | RTLD_GLOBAL);
  if (!B.rs) B.rs = dlopen("/opt/rocm/lib/librocsolver.so", RTLD_NOW | RTLD_GLOBAL);
  auto sym = [&](void* h, const char* n) -> void* {
    void* p = h ? dlsym(h, n) : nullptr;
    if (!p && B.err.empty()) B.err = std::string("missing symbol ") + n;
    return p;
  };
  B.create = (decltype(B.create))sym(B.rb, "rocblas_create_handle");
  B.set_stream = (decltype(B.set_stream))sym(B.rb, "rocblas_set_stream");
  B.dgemm = (decltype(B.dgemm))sym(B.rb, "rocblas_dgemm");
  B.sgemm = (decltype(B.sgemm))sym(B.rb, "rocblas_sgemm");
  B.gemm_ex = (decltype(B.gemm_ex))sym(B.rb, "rocblas_gemm_ex");
  B.dgemv = (decltype(B.dgemv))sym(B.rb, "rocblas_dgemv");
  B.dnrm2 = (decltype(B.dnrm2))sym(B.rb, "rocblas_dnrm2");
  B.dgemm_sb = (decltype(B.dgemm_sb))sym(B.rb, "rocblas_dgemm_strided_batched");
  B.sgemm_sb = (decltype(B.sgemm_sb))sym(B.rb, "rocblas_sgemm_strided_batched");
  B.dtrsv = (decltype(B.dtrsv))sym(B.rb, "rocblas_dtrsv");
  B.gemm_sb_ex = (decltype(B.gemm_sb_ex))dlsym(B.rb, "rocblas_gemm_strided_batched_ex");
  if (B.rs) {
    B.dsyevd = (decltype(B.dsyevd))dlsym(B.rs, "rocsolver_dsyevd");
    B.dtrtri = (decltype(B.dtrtri))dlsym(B.rs, "rocsolver_dtrtri");
    B.dgeqrf = (decltype(B.dgeqrf))dlsym(B.rs, "rocsolver_dgeqrf");
    B.dorgqr = (decltype(B.dorgqr))dlsym(B.rs, "rocsolver_dorgqr");
    B.dgesvd = (decltype(B.dgesvd))dlsym(B.rs, "rocsolver_dgesvd");
  }
  B.ok = B.create && B.set_stream && B.dgemm && B.sgemm && B.gemm_ex && B.dgemv && B.dnrm2 && B.dtrsv && B.dgemm_sb && B.sgemm_sb;
  return B;
}

int handle(void** h, hipStream_t s) {
  Blas& B = blas();
  if (!B.ok) { sl_set_last_error(B.err.c_str()); return SL_ERR_UNSUPPORTED; }
  int dev = 0;
  SL_HIP_CHECK(hipGetDevice(&dev));
  if (dev < 0 || dev >= 64) { sl_set_last_error("device index"); return SL_ERR_INVALID; }
  {
    static std::mutex mu;
    std::lock_guard<std::mutex> g(mu);
    if (!B.handle[dev] && B.create(&B.handle[dev]) != 0) {
      sl_set_last_error("rocblas_create_handle failed");
      return SL_ERR_HIP;
    }
  }
  if (B.set_stream(B.handle[dev], s) != 0) { sl_set_last_error("rocblas_set_stream failed"); return SL_ERR_HIP; }
  *h = B.handle[dev];
  return SL_OK;
}

constexpr int OP_N = 111, OP_T = 112;
constexpr int DT_F32 = 151, DT_F64 = 152, DT_BF16 = 168;   // rocblas_datatype_{f32,f64,bf16}_r

int rc_of(int st, const char* what) {
  if (st == 0) return SL_OK;
  sl_set_last_error((std::string(what) + " failed (rocblas status " + std::to_string(st) + ")").c_str());
  return SL_ERR_HIP;
}

}  // namespace

bool slb_available() { return blas().ok; }
bool slb_solver_available() {
  Blas& B = blas();
  return B.ok && B.dsyevd && B.dtrtri && B.dgeqrf && B.dorgqr && B.dgesvd;
}

// Row-major C (M x N, ldc) = alpha op(A) op(B) + beta C, as the column-major
// C^T = op(B)^T op(A)^T.  dt: SL_F32 / SL_F64 (A, B, C all of it), or SL_BF16
// (A, B bf16, C f32, f32 accumulation).
int slb_gemm(int dt, bool ta, bool tb, int64_t M, int64_t N, int64_t K, double alpha, const void* A, int64_t lda,
             const void* B, int64_t ldb, double beta, void* C, int64_t ldc, hipStream_t s) {
  if (M <= 0 || N <= 0) return SL_OK;
  void* h = nullptr;
  const int rc = handle(&h, s);
  if (rc != SL_OK) return rc;
  Blas& L = blas();
  const int opA = ta ? OP_T : OP_N, opB = tb ? OP_T : OP_N;
  if (dt == SL_F64) {
    const double al = alpha, be = beta;
    return rc_of(L.dgemm(h, opB, opA, (int)N, (int)M, (int)K, &al, (const double*)B, (int)ldb, (const double*)A,
                         (int)lda, &be, (double*)C, (int)ldc), "rocblas_dgemm");
  }
  if (dt == SL_F32) {
    const float al = (float)alpha, be = (float)beta;
    return rc_of(L.sgemm(h, opB, opA, (int)N, (int)M, (int)K, &al, (const float*)B, (int)ldb, (const float*)A,
                         (int)lda, &be, (float*)C, (int)ldc), "rocblas_sgemm");
  }
  const float al = (float)alpha, be = (float)beta;
  return rc_of(L.gemm_ex(h, opB, opA, (int)N, (int)M, (int)K, &al, B, DT_BF16, (int)ldb, A, DT_BF16, (int)lda, &be,
                         C, DT_F32, (int)ldc, C, DT_F32, (int)ldc, DT_F32, 0, 0, 0), "rocblas_gemm_ex");
}

// batch of row-major products C_b = alpha op(A_b) op(B_b) + beta C_b with
// element strides sA / sB / sC between the operands of consecutive batches
// (SL_F32 / SL_F64, or SL_BF16: A, B bf16, C f32, f32 accumulation)
int slb_gemm_strided(int dt, bool ta, bool tb, int64_t M, int64_t N, int64_t K, double alpha, const void* A,
                     int64_t lda, int64_t sA, const void* B, int64_t ldb, int64_t sB, double beta, void* C, int64_t ldc,
                     int64_t sC, int batch, hipStream_t s) {
  if (M <= 0 || N <= 0 || batch <= 0) return SL_OK;
  void* h = nullptr;
  const int rc = handle(&h, s);
  if (rc != SL_OK) return rc;
  Blas& L = blas();
  const int opA = ta ? OP_T : OP_N, opB = tb ? OP_T : OP_N;
  if (dt == SL_BF16) {
    if (!L.gemm_sb_ex) {
      sl_set_last_error("rocblas_gemm_strided_batched_ex not found");
      return SL_ERR_UNSUPPORTED;
    }
    const float al = (float)alpha, be = (float)beta;
    return rc_of(L.gemm_sb_ex(h, opB, opA, (int)N, (int)M, (int)K, &al, B, DT_BF16, (int)ldb, sB, A, DT_BF16, (int)lda,
                              sA, &be, C, DT_F32, (int)ldc, sC, C, DT_F32, (int)ldc, sC, batch, DT_F32, 0, 0, 0),
                 "rocblas_gemm_strided_batched_ex");
  }
  if (dt == SL_F64) {
    const double al = alpha, be = beta;
    return rc_of(L.dgemm_sb(h, opB, opA, (int)N, (int)M, (int)K, &al, (const double*)B, (int)ldb, sB,
                            (const double*)A, (int)lda, sA, &be, (double*)C, (int)ldc, sC, batch),
                 "rocblas_dgemm_strided_batched");
  }
  const float al = (float)alpha, be = (float)beta;
  return rc_of(L.sgemm_sb(h, opB, opA, (int)N, (int)M, (int)K, &al, (const float*)B, (int)ldb, sB, (const float*)A,
                          (int)lda, sA, &be, (float*)C, (int)ldc, sC, batch),
               "rocblas_sgemm_strided_batched");
}

// Symmetric eigendecomposition of the row-major n x n f64 A in place
// (eigenvectors in A's ROWS on return: the column-major solver sees A^T = A
// and returns column-major eigenvectors, i.e. row-major transposed); D
// ascending; E scratch (n); info (device int).
int slb_dsyevd(int n, double* A, int lda, double* D, double* E, int* info, hipStream_t s) {
  void* h = nullptr;
  const int rc = handle(&h, s);
  if (rc != SL_OK) return rc;
  Blas& L = blas();
  if (!L.dsyevd) { sl_set_last_error("librocsolver.so: rocsolver_dsyevd unavailable"); return SL_ERR_UNSUPPORTED; }
  return rc_of(L.dsyevd(h, 211 /* evect_original */, 122 /* fill_lower */, n, A, lda, D, E, info), "rocsolver_dsyevd");
}

// ---------------------------------------------------------------- column-major
// LAPACK-style entry points of the C API's host-operand NLA paths
// (nla_native.cpp); every matrix column-major with its leading dimension.
int slb_dgeqrf_cm(int m, int n, double* A, int lda, double* tau, hipStream_t s) {
  void* h = nullptr;
  const int rc = handle(&h, s);
  if (rc != SL_OK) return rc;
  Blas& L = blas();
  if (!L.dgeqrf) { sl_set_last_error("librocsolver.so: rocsolver_dgeqrf unavailable"); return SL_ERR_UNSUPPORTED; }
  return rc_of(L.dgeqrf(h, m, n, A, lda, tau), "rocsolver_dgeqrf");
}

int slb_dorgqr_cm(int m, int n, int k, double* A, int lda, double* tau, hipStream_t s) {
  void* h = nullptr;
  const int rc = handle(&h, s);
  if (rc != SL_OK) return rc;
  Blas& L = blas();
  if (!L.dorgqr) { sl_set_last_error("librocsolver.so: rocsolver_dorgqr unavailable"); return SL_ERR_UNSUPPORTED; }
  return rc_of(L.dorgqr(h, m, n, k, A, lda, tau), "rocsolver_dorgqr");
}

// thin SVD A = U diag(S) VT (U m x min, VT min x n), E scratch (min - 1)
int slb_dgesvd_cm(int m, int n, double* A, int lda, double* S, double* U, int ldu, double* VT, int ldvt, double* E,
                  int* info, hipStream_t s) {
  void* h = nullptr;
  const int rc = handle(&h, s);
  if (rc != SL_OK) return rc;
  Blas& L = blas();
  if (!L.dgesvd) { sl_set_last_error("librocsolver.so: rocsolver_dgesvd unavailable"); return SL_ERR_UNSUPPORTED; }
  return rc_of(L.dgesvd(h, 192 /* singular */, 192, m, n, A, lda, S, U, ldu, VT, ldvt, E, 201 /* out of place */,
                        info), "rocsolver_dgesvd");
}

// upper (row-major lower) triangular inverse in place, column-major upper
int slb_dtrtri_upper_cm(int n, double* R, int ldr, int* info, hipStream_t s) {
  void* h = nullptr;
  const int rc = handle(&h, s);
  if (rc != SL_OK) return rc;
  Blas& L = blas();
  if (!L.dtrtri) { sl_set_last_error("librocsolver.so unavailable"); return SL_ERR_UNSUPPORTED; }
  return rc_of(L.dtrtri(h, 121 /* upper */, 131, n, R, ldr, info), "rocsolver_dtrtri");
}

int slb_dgemv_cm(bool trans, int m, int n, double alpha, const double* A, int lda, const double* x, double beta,
                 double* y, hipStream_t s) {
  void* h = nullptr;
  const int rc = handle(&h, s);
  if (rc != SL_OK) return rc;
  return rc_of(blas().dgemv(h, trans ? OP_T : OP_N, m, n, &alpha, A, lda, x, 1, &beta, y, 1), "rocblas_dgemv");
}

// Euclidean norm into a host double (synchronises the stream)
int slb_dnrm2(int n, const double* x, double* result, hipStream_t s) {
  void* h = nullptr;
  const int rc = handle(&h, s);
  if (rc != SL_OK) return rc;
  return rc_of(blas().dnrm2(h, n, x, 1, result), "rocblas_dnrm2");
}

// x = op(R)^{-1} x for the column-major upper triangular R
int slb_dtrsv_upper_cm(bool trans, int n, const double* R, int ldr, double* x, hipStream_t s) {
  void* h = nullptr;
  const int rc = handle(&h, s);
  if (rc != SL_OK) return rc;
  return rc_of(blas().dtrsv(h, 121, trans ? OP_T : OP_N, 131, n, R, ldr, x, 1), "rocblas_dtrsv");
}
