// Exact marginal log likelihood terms and their hyperparameter gradients.
//
// Reference: fit_gpytorch_mll -> fit_gpytorch_mll_scipy -> scipy L-BFGS-B over
// the closure -ExactMarginalLogLikelihood(model(X), y) (botorch/fit.py:75-258,
// optim/fit.py:47-110, optim/closures/model_closures.py:171-184), i.e. [G]
//   ll = -1/2 (y-c)^T A^{-1} (y-c) - 1/2 log|A| - n/2 log 2 pi,  A = K_theta + s2 I
// with its autograd gradient.  Here the gradient is closed-form:
//   dll/dtheta = 1/2 sum_ik (alpha_i alpha_k - A^{-1}_ik) dA_ik/dtheta,
// so after the Cholesky / inverse of bo_gp_cache_build and A^{-1} = U U^T
// (one triangular MFMA GEMM), a single pass over the lower triangle of the
// n x n pairs produces every term.  One workgroup per row i.
#include "common.h"

namespace {

constexpr int THREADS = 256;
constexpr int MAXD = 64;

template <int KIND, int DC>  // DC: compile-time input dimension (0 = runtime d <= MAXD)
__global__ __launch_bounds__(THREADS) void mll_terms_kernel(
    const double* __restrict__ X, int n, int d_rt, const double* __restrict__ ls, double outputscale,
    const double* __restrict__ L, const double* __restrict__ Ainv, int64_t ld,
    const double* __restrict__ alpha, const double* __restrict__ beta,
    double* __restrict__ partial) {
  // partial[i][0..d-1]: sum_k w W_ik g_ik Delta_ikj^2 ;  [d]: W_ii ;  [d+1]: sum_k w W_ik kbar_ik
  //                [d+2]: log L_ii ;  [d+3]: beta_i^2 ;  [d+4]: alpha_i      (w = 2 off-diagonal)
  const int d = DC > 0 ? DC : d_rt;
  constexpr int NA = DC > 0 ? DC + 1 : MAXD + 1;
  __shared__ double red[THREADS / 64][MAXD + 5];
  __shared__ double sl[MAXD];
  const int i = blockIdx.x;
  const int tid = threadIdx.x;
  if (tid < d) sl[tid] = 1.0 / ls[tid];
  __syncthreads();
  double acc[NA];
#pragma unroll
  for (int t = 0; t < NA; ++t) acc[t] = 0.0;
  const double ai = alpha[i];
  const double* xi = X + (int64_t)i * d;
  for (int k = tid; k <= i; k += THREADS) {
    const double* xk = X + (int64_t)k * d;
    double r2 = 0.0;
    for (int t = 0; t < d; ++t) {
      const double df = (xi[t] - xk[t]) * sl[t];
      r2 = fma(df, df, r2);
    }
    const double W = ai * alpha[k] - Ainv[(int64_t)i * ld + k];
    const double w = (k == i) ? W : 2.0 * W;
    double kbar, g;  // unit-outputscale kernel value; dk/dell_j = outputscale g Delta_j^2 / ell_j^3
    if (KIND == BO_RBF) {
      kbar = exp(-0.5 * r2);
      g = kbar;
    } else {
      const double r = sqrt(r2);
      const double s5r = 2.23606797749978969641 * r;
      const double e = exp(-s5r);
      kbar = (1.0 + s5r + (5.0 / 3.0) * r2) * e;
      g = (5.0 / 3.0) * (1.0 + s5r) * e;
    }
    const double wg = w * g * outputscale;
    for (int t = 0; t < d; ++t) {
      const double df = xi[t] - xk[t];
      acc[t] = fma(wg, df * df, acc[t]);
    }
    acc[d] = fma(w, kbar, acc[d]);
  }
  for (int t = 0; t <= d; ++t) {
    double v = acc[t];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if ((tid & 63) == 0) red[tid >> 6][t] = v;
  }
  __syncthreads();
  if (tid <= d) {
    double v = 0.0;
    for (int w = 0; w < THREADS / 64; ++w) v += red[w][tid];
    double* out = partial + (int64_t)i * (d + 5);
    if (tid < d) out[tid] = v;
    else out[d + 1] = v;
  }
  if (tid == 0) {
    double* out = partial + (int64_t)i * (d + 5);
    out[d] = ai * ai - Ainv[(int64_t)i * ld + i];
    out[d + 2] = log(L[(int64_t)i * ld + i]);
    out[d + 3] = beta[i] * beta[i];
    out[d + 4] = ai;
  }
}

}  // namespace

extern "C" int bo_mll_terms(int kind, const double* X, int64_t n, int d, const double* lengthscale,
                            double outputscale, const double* L, const double* Ainv, int64_t ld,
                            const double* alpha, const double* beta, double* partial,
                            void* stream) {
  BO_CHECK_ARG(d >= 1 && d <= MAXD, "bo_mll_terms: d=%d (1..%d)", d, MAXD);
  if (n == 0) return BO_OK;
  hipStream_t st = as_stream(stream);
#define BO_MLL(KIND, DC)                                                                   \
  mll_terms_kernel<KIND, DC><<<(unsigned)n, THREADS, 0, st>>>(X, (int)n, d, lengthscale,    \
                                                              outputscale, L, Ainv, ld, alpha, \
                                                              beta, partial)
  if (kind == BO_RBF) {
    if (d == 6) BO_MLL(BO_RBF, 6); else if (d <= 8 && d == 8) BO_MLL(BO_RBF, 8); else BO_MLL(BO_RBF, 0);
  } else {
    if (d == 6) BO_MLL(BO_MATERN52, 6); else BO_MLL(BO_MATERN52, 0);
  }
#undef BO_MLL
  BO_LAUNCH_CHECK();
  return BO_OK;
}
