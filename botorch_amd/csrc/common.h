// Shared device/host helpers for the gfx950 (CDNA4) kernels of botorch_amd.
//
// Everything here is fp64: the reference path (BoTorch + GPyTorch on torch
// fp64) computes in double and the parity bar (1e-4 relative on posterior
// variances, where var = k** - ||r||^2 cancels by 1e3-1e4 near the data)
// excludes lower precision.  Dense contractions run on the fp64 matrix cores:
// v_mfma_f64_16x16x4_f64 (one f64 A and B element per lane, 4 f64
// accumulators per lane).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <stdint.h>

#include <cmath>
#include <cstdio>
#include <string>

#include "../../include/botorch_amd.h"

typedef double v4d __attribute__((ext_vector_type(4)));

#define BO_WAVE 64

// ---------------------------------------------------------------------------
// v_mfma_f64_16x16x4_f64 fragment maps (gfx950):
//   A (16x4):  lane l holds A[i = l & 15][k = l >> 4]
//   B (4x16):  lane l holds B[k = l >> 4][j = l & 15]
//   D (16x16): lane l, accumulator register r holds
//              D[row = (l >> 4) + 4 r][col = l & 15]
// The D map differs from the f32/bf16 families (row = 4 (l >> 4) + r); it is
// verified on hardware by bo_probe_mfma_f64_layout (tests/test_gpu_kernels.py).
// ---------------------------------------------------------------------------
__device__ __forceinline__ int mfma_row(int lane, int r) { return (lane >> 4) + 4 * r; }
__device__ __forceinline__ int mfma_col(int lane) { return lane & 15; }

__device__ __forceinline__ v4d mfma_f64(double a, double b, v4d c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// v broadcast from lane K of each 16-lane row (DPP row_newbcast on gfx950).
template <int K>
__device__ __forceinline__ double row_bcast(double v) {
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_mov_dpp((int)(x & 0xffffffffll), 0x150 + K, 0xf, 0xf, true);
  const int hi = __builtin_amdgcn_mov_dpp((int)(x >> 32), 0x150 + K, 0xf, 0xf, true);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ v4d v4d_zero() {
  v4d z = {0.0, 0.0, 0.0, 0.0};
  return z;
}

// Kernel families on the path (botorch/models/utils/gpytorch_modules.py:100-127,
// botorch/models/fully_bayesian.py:81-92).
enum BoKernelKind : int { BO_RBF = 0, BO_MATERN52 = 1 };

// Stationary kernel value from the squared distance of lengthscale-scaled inputs.
template <int KIND>
__device__ __forceinline__ double kernel_from_d2(double d2) {
  if (KIND == BO_RBF) {
    return exp(-0.5 * d2);
  } else {
    const double r = sqrt(fmax(d2, 1e-30));
    const double s5r = 2.23606797749978969641 * r;  // sqrt(5) r
    return (1.0 + s5r + (5.0 / 3.0) * d2) * exp(-s5r);
  }
}

// dk(x_i, x_k)/dx_i (scaled coordinates), as a factor g with dk = g * (x_i - x_k).
template <int KIND>
__device__ __forceinline__ double dkernel_factor(double d2, double outputscale) {
  if (KIND == BO_RBF) {
    return -outputscale * exp(-0.5 * d2);
  } else {
    const double r = sqrt(fmax(d2, 0.0));
    const double s5r = 2.23606797749978969641 * r;
    return -outputscale * (5.0 / 3.0) * (1.0 + s5r) * exp(-s5r);
  }
}

void bo_set_error(const char* fmt, ...);

#define BO_CHECK_ARG(cond, ...)        \
  do {                                 \
    if (!(cond)) {                     \
      bo_set_error(__VA_ARGS__);       \
      return BO_ERR_ARG;               \
    }                                  \
  } while (0)

#define BO_HIP(expr)                                                          \
  do {                                                                        \
    hipError_t _e = (expr);                                                   \
    if (_e != hipSuccess) {                                                   \
      bo_set_error("%s:%d %s: %s", __FILE__, __LINE__, #expr,                 \
                   hipGetErrorString(_e));                                    \
      return BO_ERR_HIP;                                                      \
    }                                                                         \
  } while (0)

#define BO_LAUNCH_CHECK() BO_HIP(hipGetLastError())

static inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

static inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// Stream-ordered scratch (hipMallocAsync) comes from the device's default
// pool; with its release threshold at 0 every synchronisation hands the
// memory back and the next allocation goes to the driver again.  Once per
// device the pool keeps what it has.
inline void keep_pool_warm() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return;
  static std::atomic<uint64_t> done{0};
  const uint64_t bit = uint64_t(1) << dev;
  if (done.load() & bit) return;
  hipMemPool_t pool;
  if (hipDeviceGetDefaultMemPool(&pool, dev) == hipSuccess) {
    uint64_t thr = ~uint64_t(0);
    (void)hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &thr);
  }
  done.fetch_or(bit);
}
