// Internal interface of the fp64 MFMA GEMM (gemm.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/botorch_amd.h"

int bo_gemm_f64_impl(int ta, int tb, int M, int N, int K, double alpha, const double* A,
                     int64_t lda, int64_t sA, const double* B, int64_t ldb, int64_t sB,
                     double beta, double* C, int64_t ldc, int64_t sC, int batch, int flags,
                     hipStream_t st);
