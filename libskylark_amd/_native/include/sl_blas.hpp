// Run-time resolved rocBLAS / rocSOLVER (sl_blas.cpp): plain library GEMMs and
// small dense LAPACK on the device, one handle per device, row-major API.
#pragma once
#include "sl_common.hpp"

bool slb_available();
bool slb_solver_available();
// row-major C (M x N) = alpha op(A) op(B) + beta C; dt SL_F32 / SL_F64, or
// SL_BF16 (bf16 A and B, f32 C and accumulation)
int slb_gemm(int dt, bool ta, bool tb, int64_t M, int64_t N, int64_t K, double alpha, const void* A, int64_t lda,
             const void* B, int64_t ldb, double beta, void* C, int64_t ldc, hipStream_t s);
// batched row-major products, element strides between batches (SL_F32 / SL_F64)
int slb_gemm_strided(int dt, bool ta, bool tb, int64_t M, int64_t N, int64_t K, double alpha, const void* A,
                     int64_t lda, int64_t sA, const void* B, int64_t ldb, int64_t sB, double beta, void* C, int64_t ldc,
                     int64_t sC, int batch, hipStream_t s);
// eigenvectors of the row-major symmetric A in its rows, eigenvalues ascending
int slb_dsyevd(int n, double* A, int lda, double* D, double* E, int* info, hipStream_t s);

// column-major LAPACK-style helpers (C API host-operand NLA paths)
int slb_dgeqrf_cm(int m, int n, double* A, int lda, double* tau, hipStream_t s);
int slb_dorgqr_cm(int m, int n, int k, double* A, int lda, double* tau, hipStream_t s);
int slb_dgesvd_cm(int m, int n, double* A, int lda, double* S, double* U, int ldu, double* VT, int ldvt, double* E,
                  int* info, hipStream_t s);
int slb_dtrtri_upper_cm(int n, double* R, int ldr, int* info, hipStream_t s);
int slb_dgemv_cm(bool trans, int m, int n, double alpha, const double* A, int lda, const double* x, double beta,
                 double* y, hipStream_t s);
int slb_dnrm2(int n, const double* x, double* result, hipStream_t s);
int slb_dtrsv_upper_cm(bool trans, int n, const double* R, int ldr, double* x, hipStream_t s);
