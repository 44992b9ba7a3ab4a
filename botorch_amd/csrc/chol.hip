// Exact-GP training caches on gfx950: kernel matrix, blocked Cholesky with the
// reference's jitter ladder, explicit triangular inverse, and the two solves.
//
// Replaces, for the exact-prediction path of SingleTaskGP
// (botorch/models/gpytorch.py:446 -> [G] DefaultPredictionStrategy):
//   L          = psd_safe_cholesky(K + s2 I)         (jitter 1e-8 * 10^i, 6 tries,
//                                                     botorch/__init__.py:47)
//   covar_cache = L^{-T}                               (root_inv_decomposition,
//                                                     fast_covar_root_decomposition
//                                                     off, botorch/__init__.py:44)
//   mean_cache  = (K + s2 I)^{-1} (y - c)
// The mean is later formed as R beta with beta = L^{-1}(y - c)  (K*x alpha =
// K*x L^{-T} L^{-1} (y - c) = R beta), so beta is cached beside alpha.
//
// Layout in HBM: every n x n cache is stored row-major at the padded order
// np = roundup(n, 128) with an identity pad, so the 128-wide diagonal blocks of
// the right-looking factorisation never straddle the edge.
#include <cstdarg>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "common.h"
#include "gemm.h"

int bo_chol_dag(double* A, double* Linv, int64_t np, int* info, void* work, hipStream_t st,
                long long* trace = nullptr, int nb = 1, double* Ainv = nullptr);

namespace {

constexpr int NBO = 128; // padded matrix order granule (n rounded up to 128)

// K[i][j] = outputscale * k(x_i, x_j) (+ diag_add on i == j), row-major with
// leading dimension ldk, over a `rows x cols` padded extent (identity pad).
// mode bit 1: zero the strict upper triangle (Cholesky input).
constexpr int CM_DMAX = 256;  // dimensions staged in LDS by covar_matrix_kernel
constexpr int CM_ROWS = 8;    // rows per workgroup

// K[i][j] = outputscale * k(x_i, x_j) (+ diag_add on i == j), row-major with
// leading dimension ldk, over a `rows x cols` padded extent (identity pad).
// mode bit 1: zero the strict upper triangle (Cholesky input).
// A workgroup takes CM_ROWS rows x 256 columns: the rows' inputs and the
// reciprocal lengthscales sit in LDS (one divide per dimension per workgroup),
// each thread reuses its column's input for all CM_ROWS rows, and each row's
// 256 values leave as one 2 KB coalesced store.  (One row per workgroup with
// per-element divides: 80 us for the n = 4096 Cholesky input.)
template <int KIND>
__global__ __launch_bounds__(256) void covar_matrix_kernel(
    const double* __restrict__ X1, int64_t n1, const double* __restrict__ X2, int64_t n2,
    int d, const double* __restrict__ ls, double outputscale, double diag_add, int mode,
    double* __restrict__ K, int64_t ldk, int64_t rows, int64_t cols) {
  __shared__ double invl[CM_DMAX], xi[CM_ROWS][CM_DMAX];
  const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t i0 = (int64_t)blockIdx.y * CM_ROWS;
  for (int t = threadIdx.x; t < d; t += blockDim.x) invl[t] = 1.0 / ls[t];
  __syncthreads();
  for (int e = threadIdx.x; e < CM_ROWS * d; e += blockDim.x) {
    const int r = e / d, t = e - r * d;
    xi[r][t] = (i0 + r < n1) ? X1[(i0 + r) * d + t] * invl[t] : 0.0;
  }
  __syncthreads();
  if (j >= cols) return;
  const bool jv = j < n2;
  double d2[CM_ROWS];
#pragma unroll
  for (int r = 0; r < CM_ROWS; ++r) d2[r] = 0.0;
  // rows of this workgroup that need a kernel value at column j
  const bool any = jv && i0 < n1 && !((mode & 1) && j > i0 + CM_ROWS - 1);
  if (any) {
    for (int t = 0; t < d; ++t) {
      const double v = X2[j * d + t] * invl[t];
#pragma unroll
      for (int r = 0; r < CM_ROWS; ++r) {
        const double diff = xi[r][t] - v;
        d2[r] = fma(diff, diff, d2[r]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < CM_ROWS; ++r) {
    const int64_t i = i0 + r;
    if (i >= rows) break;
    double val;
    if (i >= n1 || !jv) {
      val = (i == j) ? 1.0 : 0.0;
    } else if ((mode & 1) && j > i) {
      val = 0.0;
    } else {
      val = outputscale * kernel_from_d2<KIND>(d2[r]);
      if (i == j) val += diag_add;
    }
    K[i * ldk + j] = val;
  }
}

// Two-level batched covariance: batch z = o * inner + i reads its inputs at
// X1 + o s1o + i s1i (n1 x d), X2 + o s2o + i s2i (n2 x d), its lengthscales at
// ls + o slo + i sli (d) and outputscale os[o soo + i soi], and writes
// K + o sKo + i sKi (n1 x n2, leading dimension ldk).  The SAAS ensemble
// (models/fully_bayesian.py:276-281) evaluates all M members' K*x (outer = M,
// shared test rows) and all M x B q x q blocks K** (outer = M, inner = B) in
// one launch each.
constexpr int CB_ROWS = 8;     // X1 rows per workgroup (x2 loads reused across them)
constexpr int CB_DMAX = 512;   // inputs staged in LDS

template <int KIND>
__global__ __launch_bounds__(256) void covar_batched_kernel(
    const double* __restrict__ X1, int64_t s1o, int64_t s1i, int n1,
    const double* __restrict__ X2, int64_t s2o, int64_t s2i, int n2, int d,
    const double* __restrict__ ls, int64_t slo, int64_t sli, const double* __restrict__ os,
    int64_t soo, int64_t soi, double* __restrict__ K, int64_t sKo, int64_t sKi, int64_t ldk,
    int inner) {
  // The member's inverse lengthscales and its CB_ROWS scaled X1 rows live in
  // LDS (one reciprocal per dimension per workgroup, not one divide per
  // element); each thread owns one X2 column and reuses every x2 load for all
  // CB_ROWS rows.
  __shared__ double invl[CB_DMAX];
  __shared__ double x1s[CB_ROWS][CB_DMAX];
  const int z = blockIdx.z;
  const int o = z / inner, i = z % inner;
  const int row0 = blockIdx.y * CB_ROWS;
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  const double* l = ls + o * slo + i * sli;
  for (int t = threadIdx.x; t < d; t += blockDim.x) invl[t] = 1.0 / l[t];
  __syncthreads();
  const double* x1 = X1 + o * s1o + i * s1i;
  for (int e = threadIdx.x; e < CB_ROWS * d; e += blockDim.x) {
    const int r = e / d, t = e - r * d;
    x1s[r][t] = (row0 + r < n1) ? x1[(int64_t)(row0 + r) * d + t] * invl[t] : 0.0;
  }
  __syncthreads();
  if (col >= n2) return;
  const double* x2 = X2 + o * s2o + i * s2i + (int64_t)col * d;
  double d2[CB_ROWS];
#pragma unroll
  for (int r = 0; r < CB_ROWS; ++r) d2[r] = 0.0;
  for (int t = 0; t < d; ++t) {
    const double v = x2[t] * invl[t];
#pragma unroll
    for (int r = 0; r < CB_ROWS; ++r) {
      const double diff = x1s[r][t] - v;
      d2[r] = fma(diff, diff, d2[r]);
    }
  }
  const double scale = os[o * soo + i * soi];
  double* Kz = K + o * sKo + i * sKi;
#pragma unroll
  for (int r = 0; r < CB_ROWS; ++r)
    if (row0 + r < n1) Kz[(int64_t)(row0 + r) * ldk + col] = scale * kernel_from_d2<KIND>(d2[r]);
}

__global__ void transpose_kernel(const double* __restrict__ A, double* __restrict__ B,
                                 int64_t n, int64_t ld) {
  __shared__ double tile[32][33];
  const int64_t bx = blockIdx.x * 32, by = blockIdx.y * 32;
  const int tx = threadIdx.x, ty = threadIdx.y;  // 32 x 8
  for (int r = ty; r < 32; r += 8) {
    const int64_t gi = by + r, gj = bx + tx;
    tile[r][tx] = (gi < n && gj < n) ? A[gi * ld + gj] : 0.0;
  }
  __syncthreads();
  for (int r = ty; r < 32; r += 8) {
    const int64_t gi = bx + r, gj = by + tx;
    if (gi < n && gj < n) B[gi * ld + gj] = tile[tx][r];
  }
}

// y = op(M) x (+ shift), one wave per output row.  trans: use M^T.
__global__ __launch_bounds__(256) void gemv_kernel(const double* __restrict__ M, int64_t ld,
                                                   int64_t n, const double* __restrict__ x,
                                                   double xshift, double* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  double s = 0.0;
  for (int64_t k = lane; k < n; k += 64) s = fma(M[row * ld + k], x[k] - xshift, s);
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if (lane == 0) y[row] = s;
}

// gemv_kernel on a triangular M (uplo 1: lower, 2: upper): a row reads only
// its triangle.  Each lane keeps gemv_kernel's k = lane + 64 m order and
// skips only the zero products, so y is bit-identical to the full product.
__global__ __launch_bounds__(256) void gemv_tri_kernel(const double* __restrict__ M, int64_t ld,
                                                       int64_t n, const double* __restrict__ x,
                                                       double xshift, double* __restrict__ y,
                                                       int uplo) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= n) return;
  const int64_t k0 = uplo == 2 ? (row / 64) * 64 + lane : lane;
  const int64_t k1 = uplo == 1 ? row + 1 : n;
  double s = 0.0;
  for (int64_t k = k0; k < k1; k += 64)
    if (uplo != 2 || k >= row) s = fma(M[row * ld + k], x[k] - xshift, s);
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if (lane == 0) y[row] = s;
}

// y = M^T (x - xshift) for a lower-triangular M (y[c] = sum_{k >= c} M[k][c]
// (x[k] - xshift)) without forming M^T: block (column block of 64, row chunk of
// 256) -- lane = column, so every row is one coalesced 512-B read -- writes
// its partial sums part[chunk][c] (the 4 waves' row subsets summed in wave
// order through LDS); gemv_lt_sum_kernel adds the chunks in order.
constexpr int GLT_ROWS = 256;
__global__ __launch_bounds__(256) void gemv_lt_kernel(const double* __restrict__ M, int64_t ld,
                                                      int64_t n, const double* __restrict__ x,
                                                      double xshift, double* __restrict__ part,
                                                      int64_t ldp) {
  __shared__ double red[4][64];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int64_t c = (int64_t)blockIdx.x * 64 + lane;
  const int64_t k0 = (int64_t)blockIdx.y * GLT_ROWS;
  const int64_t k1 = k0 + GLT_ROWS < n ? k0 + GLT_ROWS : n;
  double s = 0.0;
  if (c < n) {
    const int64_t kb = k0 > c ? k0 : c;  // rows k >= c only
#pragma unroll 4
    for (int64_t k = kb + ((wave - kb) % 4 + 4) % 4; k < k1; k += 4)
      s = fma(M[k * ld + c], x[k] - xshift, s);
  }
  red[wave][lane] = s;
  __syncthreads();
  if (wave == 0) {
    s = red[0][lane];
    s += red[1][lane];
    s += red[2][lane];
    s += red[3][lane];
    if (c < n) part[(int64_t)blockIdx.y * ldp + c] = s;
  }
}

__global__ __launch_bounds__(256) void gemv_lt_sum_kernel(const double* __restrict__ part,
                                                          int64_t ldp, int nchunk, int64_t n,
                                                          double* __restrict__ y) {
  const int64_t c = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= n) return;
  double s = 0.0;
  for (int j = 0; j < nchunk; ++j) s += part[(int64_t)j * ldp + c];
  y[c] = s;
}

__global__ void scale_inputs_kernel(const double* __restrict__ X, int64_t n, int d,
                                    const double* __restrict__ ls, const double* __restrict__ center,
                                    int dp, double* __restrict__ Xs) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= n * dp) return;
  const int64_t i = idx / dp;
  const int t = (int)(idx % dp);
  Xs[idx] = (t < d) ? (X[i * d + t] - (center ? center[t] : 0.0)) / ls[t] : 0.0;
}

// A[i][i] += v[i], i < n: the observed noise variances of a fixed-noise
// likelihood on the kernel matrix's diagonal.
__global__ void add_diag_kernel(double* __restrict__ A, int64_t ld, int64_t n,
                                const double* __restrict__ v) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) A[i * ld + i] += v[i];
}

}  // namespace

// ---------------------------------------------------------------------------
thread_local char g_err[512];
void bo_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}

extern "C" {

const char* bo_last_error(void) { return g_err; }

int bo_version(void) { return BO_ABI_VERSION; }

// 128 = the fused posterior kernel's column tile (post.hip) = the Cholesky panel.
int64_t bo_padded_order(int64_t n) { return ceil_div(n, 128) * 128; }

int bo_covar_matrix(int kind, const double* X1, int64_t n1, const double* X2, int64_t n2,
                    int d, const double* lengthscale, double outputscale, double diag_add,
                    int mode, double* K, int64_t ldk, int64_t rows, int64_t cols, void* stream) {
  BO_CHECK_ARG(kind == BO_RBF || kind == BO_MATERN52, "bo_covar_matrix: bad kind %d", kind);
  BO_CHECK_ARG(d > 0 && d <= CM_DMAX && ldk >= cols && rows >= n1 && cols >= n2,
               "bo_covar_matrix: bad shape (d = %d, at most %d)", d, CM_DMAX);
  if (rows == 0 || cols == 0) return BO_OK;
  dim3 grid((unsigned)ceil_div(cols, 256), (unsigned)ceil_div(rows, CM_ROWS));
  hipStream_t st = as_stream(stream);
  if (kind == BO_RBF)
    covar_matrix_kernel<BO_RBF><<<grid, 256, 0, st>>>(X1, n1, X2, n2, d, lengthscale, outputscale, diag_add, mode, K, ldk, rows, cols);
  else
    covar_matrix_kernel<BO_MATERN52><<<grid, 256, 0, st>>>(X1, n1, X2, n2, d, lengthscale, outputscale, diag_add, mode, K, ldk, rows, cols);
  BO_LAUNCH_CHECK();
  return BO_OK;
}

int bo_covar_batched(int kind, const double* X1, int64_t s1o, int64_t s1i, int n1,
                     const double* X2, int64_t s2o, int64_t s2i, int n2, int d, const double* ls,
                     int64_t slo, int64_t sli, const double* os, int64_t soo, int64_t soi,
                     double* K, int64_t sKo, int64_t sKi, int64_t ldk, int outer, int inner,
                     void* stream) {
  BO_CHECK_ARG(kind == BO_RBF || kind == BO_MATERN52, "bo_covar_batched: bad kind %d", kind);
  BO_CHECK_ARG(d > 0 && n1 >= 0 && n2 >= 0 && ldk >= n2 && outer >= 1 && inner >= 1,
               "bo_covar_batched: bad shape");
  BO_CHECK_ARG(d <= CB_DMAX, "bo_covar_batched: d = %d > %d", d, CB_DMAX);
  BO_CHECK_ARG(ceil_div(n1, CB_ROWS) <= 65535 && (int64_t)outer * inner <= 65535,
               "bo_covar_batched: grid too large");
  if (n1 == 0 || n2 == 0) return BO_OK;
  const int threads = n2 >= 256 ? 256 : (int)(ceil_div(n2, 64) * 64);
  dim3 grid((unsigned)ceil_div(n2, threads), (unsigned)ceil_div(n1, CB_ROWS),
            (unsigned)(outer * inner));
  hipStream_t st = as_stream(stream);
  if (kind == BO_RBF)
    covar_batched_kernel<BO_RBF><<<grid, threads, 0, st>>>(X1, s1o, s1i, n1, X2, s2o, s2i, n2, d, ls,
                                                         slo, sli, os, soo, soi, K, sKo, sKi, ldk,
                                                         inner);
  else
    covar_batched_kernel<BO_MATERN52><<<grid, threads, 0, st>>>(X1, s1o, s1i, n1, X2, s2o, s2i, n2, d,
                                                              ls, slo, sli, os, soo, soi, K, sKo,
                                                              sKi, ldk, inner);
  BO_LAUNCH_CHECK();
  return BO_OK;
}

int bo_gemm_f64(int ta, int tb, int M, int N, int K, double alpha, const double* A, int64_t lda,
                int64_t sA, const double* B, int64_t ldb, int64_t sB, double beta, double* C,
                int64_t ldc, int64_t sC, int batch, int flags, void* stream) {
  return bo_gemm_f64_impl(ta, tb, M, N, K, alpha, A, lda, sA, B, ldb, sB, beta, C, ldc, sC,
                          batch, flags, as_stream(stream));
}

int bo_cholesky_inverse_batched(double* A, double* Linv, double* work, int nb, int64_t np,
                                int* info, void* stream) {
  BO_CHECK_ARG(nb >= 1 && nb <= 128 && np > 0 && np % NBO == 0,
               "bo_cholesky_inverse_batched: %d matrices of order %lld (1..128, multiple of %d)",
               nb, (long long)np, NBO);
  BO_CHECK_ARG(((uintptr_t)A & 15) == 0 && ((uintptr_t)Linv & 15) == 0,
               "bo_cholesky_inverse_batched: buffers must be 16-B aligned");
  return bo_chol_dag(A, Linv, np, info, work, as_stream(stream), nullptr, nb);
}

int bo_cholesky_inverse(double* A, double* Linv, double* work, int64_t np, int* info,
                        void* stream) {
  BO_CHECK_ARG(np > 0 && np % NBO == 0, "bo_cholesky_inverse: order %lld not a multiple of %d",
               (long long)np, NBO);
  BO_CHECK_ARG(((uintptr_t)A & 15) == 0 && ((uintptr_t)Linv & 15) == 0,
               "bo_cholesky_inverse: buffers must be 16-B aligned");
  return bo_chol_dag(A, Linv, np, info, work, as_stream(stream));
}

int bo_cholesky_inverse_ainv(double* A, double* Linv, double* Ainv, double* work, int64_t np,
                             int* info, void* stream) {
  BO_CHECK_ARG(np > 0 && np % NBO == 0, "bo_cholesky_inverse_ainv: order %lld not a multiple of %d",
               (long long)np, NBO);
  BO_CHECK_ARG(Ainv && ((uintptr_t)A & 15) == 0 && ((uintptr_t)Linv & 15) == 0 &&
                   ((uintptr_t)Ainv & 15) == 0,
               "bo_cholesky_inverse_ainv: buffers must be 16-B aligned (and Ainv given)");
  return bo_chol_dag(A, Linv, np, info, work, as_stream(stream), nullptr, 1, Ainv);
}

int bo_transpose(const double* A, double* B, int64_t n, int64_t ld, void* stream) {
  dim3 grid((unsigned)ceil_div(n, 32), (unsigned)ceil_div(n, 32));
  transpose_kernel<<<grid, dim3(32, 8), 0, as_stream(stream)>>>(A, B, n, ld);
  BO_LAUNCH_CHECK();
  return BO_OK;
}

int bo_gemv(const double* M, int64_t ld, int64_t n, const double* x, double xshift, double* y,
            void* stream) {
  if (n <= 0) return BO_OK;
  gemv_kernel<<<(unsigned)ceil_div(n, 4), 256, 0, as_stream(stream)>>>(M, ld, n, x, xshift, y);
  BO_LAUNCH_CHECK();
  return BO_OK;
}

int bo_gemv_tri(const double* M, int64_t ld, int64_t n, const double* x, double xshift, double* y,
                int uplo, void* stream) {
  BO_CHECK_ARG(uplo == 1 || uplo == 2, "bo_gemv_tri: uplo %d (1 lower, 2 upper)", uplo);
  if (n <= 0) return BO_OK;
  gemv_tri_kernel<<<(unsigned)ceil_div(n, 4), 256, 0, as_stream(stream)>>>(M, ld, n, x, xshift, y,
                                                                            uplo);
  BO_LAUNCH_CHECK();
  return BO_OK;
}

int bo_gemv_lt_work(int64_t n, int64_t* work_elems) {
  *work_elems = ceil_div(n, GLT_ROWS) * n;
  return BO_OK;
}

int bo_gemv_lt(const double* M, int64_t ld, int64_t n, const double* x, double xshift, double* y,
               double* work, void* stream) {
  BO_CHECK_ARG(M && x && y && work && ld >= n, "bo_gemv_lt: bad arguments");
  if (n <= 0) return BO_OK;
  const int nchunk = (int)ceil_div(n, GLT_ROWS);
  hipStream_t st = as_stream(stream);
  gemv_lt_kernel<<<dim3((unsigned)ceil_div(n, 64), (unsigned)nchunk), 256, 0, st>>>(M, ld, n, x,
                                                                                  xshift, work, n);
  BO_LAUNCH_CHECK();
  gemv_lt_sum_kernel<<<(unsigned)ceil_div(n, 256), 256, 0, st>>>(work, n, nchunk, n, y);
  BO_LAUNCH_CHECK();
  return BO_OK;
}

int bo_scale_inputs(const double* X, int64_t n, int d, const double* lengthscale,
                    const double* center, int dp, double* Xs, void* stream) {
  BO_CHECK_ARG(dp >= d, "bo_scale_inputs: dp < d");
  const int64_t tot = n * dp;
  if (tot == 0) return BO_OK;
  scale_inputs_kernel<<<(unsigned)ceil_div(tot, 256), 256, 0, as_stream(stream)>>>(
      X, n, d, lengthscale, center, dp, Xs);
  BO_LAUNCH_CHECK();
  return BO_OK;
}

}  // extern "C"

// Shared body of bo_gp_cache_build (homoskedastic noise) and
// bo_gp_cache_build_fixed (noise_vec: one observed variance per point).
static int gp_cache_build_impl(int kind, const double* Xt, int64_t n, int d,
                               const double* lengthscale, double outputscale, double noise,
                               const double* noise_vec, double constant, const double* y,
                               double* L, double* Linv, double* U, double* beta, double* alpha,
                               int max_tries, double jitter0, double* jitter_used, int* info_dev,
                               void* stream) {
  BO_CHECK_ARG(n > 0 && d > 0, "bo_gp_cache_build: empty training set");
  hipStream_t st = as_stream(stream);
  const int64_t np = bo_padded_order(n);
  double jitter = 0.0;
  int info_h = 0;
  for (int attempt = 0; attempt <= max_tries; ++attempt) {
    if (attempt > 0) jitter = jitter0 * std::pow(10.0, (double)(attempt - 1));
    int s = bo_covar_matrix(kind, Xt, n, Xt, n, d, lengthscale, outputscale, noise + jitter, 1,
                            L, np, np, np, stream);
    if (s) return s;
    if (noise_vec) {
      add_diag_kernel<<<(unsigned)ceil_div(n, 256), 256, 0, st>>>(L, np, n, noise_vec);
      BO_LAUNCH_CHECK();
    }
    s = bo_cholesky_inverse(L, Linv, U, np, info_dev, stream);
    if (s) return s;
    BO_HIP(hipMemcpyAsync(&info_h, info_dev, sizeof(int), hipMemcpyDeviceToHost, st));
    BO_HIP(hipStreamSynchronize(st));
    if (info_h < 0) {
      bo_set_error("bo_gp_cache_build: Cholesky task DAG timed out");
      return BO_ERR_HIP;
    }
    if (info_h == 0) break;
  }
  if (jitter_used) *jitter_used = jitter;
  if (info_h != 0) {
    bo_set_error("Matrix not positive definite after repeatedly adding jitter up to %.1e "
                 "(info %d)", jitter, info_h);
    return BO_ERR_NOT_PSD;
  }
  int s = bo_transpose(Linv, U, np, np, stream);  // U = L^{-T}
  if (s) return s;
  s = bo_gemv_tri(Linv, np, n, y, constant, beta, 1, stream);  // beta = L^{-1} (y - c)
  if (s) return s;
  // alpha = L^{-T} beta from L^{-1}'s columns (the MLL closure's path, which
  // forms no U, takes the same kernel: the two agree bit for bit); the chunk
  // partials in stream-ordered scratch
  int64_t we = 0;
  bo_gemv_lt_work(n, &we);
  double* work = nullptr;
  keep_pool_warm();
  BO_HIP(hipMallocAsync(reinterpret_cast<void**>(&work), sizeof(double) * we, st));
  s = bo_gemv_lt(Linv, np, n, beta, 0.0, alpha, work, stream);
  BO_HIP(hipFreeAsync(work, st));
  return s;
}

extern "C" {

int bo_gp_cache_build(int kind, const double* Xt, int64_t n, int d, const double* lengthscale,
                      double outputscale, double noise, double constant, const double* y,
                      double* L, double* Linv, double* U, double* beta, double* alpha,
                      int max_tries, double jitter0, double* jitter_used, int* info_dev,
                      void* stream) {
  return gp_cache_build_impl(kind, Xt, n, d, lengthscale, outputscale, noise, nullptr, constant,
                             y, L, Linv, U, beta, alpha, max_tries, jitter0, jitter_used,
                             info_dev, stream);
}

int bo_gp_cache_build_fixed(int kind, const double* Xt, int64_t n, int d,
                            const double* lengthscale, double outputscale,
                            const double* noise_vec, double constant, const double* y, double* L,
                            double* Linv, double* U, double* beta, double* alpha, int max_tries,
                            double jitter0, double* jitter_used, int* info_dev, void* stream) {
  BO_CHECK_ARG(noise_vec != nullptr, "bo_gp_cache_build_fixed: noise_vec is NULL");
  return gp_cache_build_impl(kind, Xt, n, d, lengthscale, outputscale, 0.0, noise_vec, constant,
                             y, L, Linv, U, beta, alpha, max_tries, jitter0, jitter_used,
                             info_dev, stream);
}

}  // extern "C"

namespace {

// K[b][a][c] = outputscale * k(X[b][a], X[b][c]) (+ diag_add on a == c),
// X: B x q x d.  One thread per entry.
template <int KIND>
__global__ void covar_blocks_kernel(const double* __restrict__ X, int64_t B, int q, int d,
                                    const double* __restrict__ ls, double outputscale,
                                    double diag_add, double* __restrict__ K) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= B * q * q) return;
  const int64_t b = idx / ((int64_t)q * q);
  const int a = (int)((idx / q) % q), c = (int)(idx % q);
  double v;
  if (a == c) {
    v = outputscale + diag_add;
  } else {
    const double* xa = X + (b * q + a) * d;
    const double* xc = X + (b * q + c) * d;
    double d2 = 0.0;
    for (int t = 0; t < d; ++t) {
      const double df = (xa[t] - xc[t]) / ls[t];
      d2 = fma(df, df, d2);
    }
    v = outputscale * kernel_from_d2<KIND>(d2);
  }
  K[idx] = v;
}

// Batched small Cholesky (q <= 64) with the [G] jitter ladder per member:
// one 64-thread workgroup per matrix, lane i owns row i in LDS.
__global__ __launch_bounds__(64) void chol_small_kernel(const double* __restrict__ A, int q,
                                                        int max_tries, double jitter0,
                                                        double* __restrict__ L,
                                                        int* __restrict__ info_out,
                                                        double* __restrict__ jitter_out) {
  __shared__ double M[64][65];
  __shared__ int s_fail;
  const int64_t b = blockIdx.x;
  const int i = threadIdx.x;
  const double* Ab = A + b * q * q;
  double jit = 0.0;
  int info = 0;
  for (int attempt = 0; attempt <= max_tries; ++attempt) {
    if (attempt > 0) jit = jitter0 * pow(10.0, (double)(attempt - 1));
    if (i < q)
      for (int c = 0; c < q; ++c) M[i][c] = (c <= i) ? Ab[i * q + c] + ((c == i) ? jit : 0.0) : 0.0;
    if (i == 0) s_fail = 0;
    __syncthreads();
    for (int j = 0; j < q; ++j) {
      const double ajj = M[j][j];
      if (i == 0 && !(ajj > 0.0) && s_fail == 0) s_fail = j + 1;
      const double djj = sqrt(ajj);
      __syncthreads();
      if (i == j) M[j][j] = djj;
      if (i > j && i < q) M[i][j] = M[i][j] / djj;
      __syncthreads();
      if (i > j && i < q) {
        const double lij = M[i][j];
        for (int l = j + 1; l <= i; ++l) M[i][l] = fma(-lij, M[l][j], M[i][l]);
      }
      __syncthreads();
    }
    info = s_fail;
    __syncthreads();
    if (info == 0) break;
  }
  if (i < q)
    for (int c = 0; c < q; ++c) L[(b * q + i) * q + c] = info ? NAN : ((c <= i) ? M[i][c] : 0.0);
  if (i == 0) {
    if (info_out) info_out[b] = info;
    if (jitter_out) jitter_out[b] = jit;
  }
}

// Keep the lower triangle of the n x n block, add jitter on its diagonal,
// identity on the pad diagonal.
__global__ void tril_jitter_kernel(double* __restrict__ L, int64_t n, int64_t np, double jitter) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= np * np) return;
  const int64_t i = idx / np, j = idx % np;
  if (i < n && j < n) {
    if (j > i) L[idx] = 0.0;
    else if (i == j) L[idx] += jitter;
  } else if (i == j) {
    L[idx] = 1.0;
  }
}

}  // namespace

extern "C" int bo_covar_blocks(int kind, const double* X, int64_t B, int q, int d,
                               const double* lengthscale, double outputscale, double diag_add,
                               double* K, void* stream) {
  const int64_t tot = B * q * q;
  if (tot == 0) return BO_OK;
  hipStream_t st = as_stream(stream);
  if (kind == BO_RBF)
    covar_blocks_kernel<BO_RBF><<<(unsigned)ceil_div(tot, 256), 256, 0, st>>>(X, B, q, d, lengthscale, outputscale, diag_add, K);
  else
    covar_blocks_kernel<BO_MATERN52><<<(unsigned)ceil_div(tot, 256), 256, 0, st>>>(X, B, q, d, lengthscale, outputscale, diag_add, K);
  BO_LAUNCH_CHECK();
  return BO_OK;
}

extern "C" int bo_chol_small(const double* A, int64_t B, int q, int max_tries, double jitter0,
                             double* L, int* info, double* jitter, void* stream) {
  BO_CHECK_ARG(q >= 1 && q <= 64, "bo_chol_small: q=%d (1..64)", q);
  if (B == 0) return BO_OK;
  chol_small_kernel<<<(unsigned)B, 64, 0, as_stream(stream)>>>(A, q, max_tries, jitter0, L, info,
                                                              jitter);
  BO_LAUNCH_CHECK();
  return BO_OK;
}

// Large single-matrix psd_safe_cholesky: factor (A + jitter I) for the ladder
// 0, jitter0, 10 jitter0, ... (one host read of the status per attempt).
// A: n x n (lower part read), L / Linv / work: np x np.
extern "C" int bo_cholesky_jitter(const double* A, int64_t n, double* L, double* Linv,
                                  double* work, int max_tries, double jitter0,
                                  double* jitter_used, int* info_dev, void* stream) {
  hipStream_t st = as_stream(stream);
  const int64_t np = bo_padded_order(n);
  double jitter = 0.0;
  int info_h = 0;
  for (int attempt = 0; attempt <= max_tries; ++attempt) {
    if (attempt > 0) jitter = jitter0 * std::pow(10.0, (double)(attempt - 1));
    // L <- tril(A) + jitter I, identity pad
    BO_HIP(hipMemsetAsync(L, 0, sizeof(double) * np * np, st));
    BO_HIP(hipMemcpy2DAsync(L, np * sizeof(double), A, n * sizeof(double), n * sizeof(double), n,
                            hipMemcpyDeviceToDevice, st));
    {
      const int64_t tot = np * np;
      tril_jitter_kernel<<<(unsigned)ceil_div(tot, 256), 256, 0, st>>>(L, n, np, jitter);
      BO_LAUNCH_CHECK();
    }
    int s = bo_cholesky_inverse(L, Linv, work, np, info_dev, (void*)st);
    if (s) return s;
    BO_HIP(hipMemcpyAsync(&info_h, info_dev, sizeof(int), hipMemcpyDeviceToHost, st));
    BO_HIP(hipStreamSynchronize(st));
    if (info_h < 0) {
      bo_set_error("bo_cholesky_jitter: Cholesky task DAG timed out");
      return BO_ERR_HIP;
    }
    if (info_h == 0) break;
  }
  if (jitter_used) *jitter_used = jitter;
  if (info_h != 0) {
    bo_set_error("Matrix not positive definite after repeatedly adding jitter up to %.1e", jitter);
    return BO_ERR_NOT_PSD;
  }
  return BO_OK;
}
