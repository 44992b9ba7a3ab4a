// Batched Pareto (non-dominated) masks on the device.
//
// Reference: botorch/utils/multi_objective/pareto.py:16-64 (is_non_dominated),
// called S = 2048 times per prune_inferior_points_multi_objective
// (acquisition/multi_objective/utils.py:77-161) on n x m joint posterior
// samples.  The reference switches to a Python loop over the n points for
// large n (one small torch launch per point and sample chunk: 65536 launches at
// C4); here one thread owns one point and scans all others, the point set of a
// sample streaming through LDS in 256-point tiles.
//
//   nd[s][i] = no j with Y_j >= Y_i in every objective and > in one
//              (<= / < when minimising);
//   dedup:     additionally drop i if some j < i has Y_j == Y_i (keeps the
//              first of equal points, as the reference's argmax over matches).
#include "common.h"

namespace {

constexpr int PT = 256;   // points per tile / threads per block
constexpr int MMAX = 8;   // objectives

__global__ __launch_bounds__(PT) void pareto_mask_kernel(const double* __restrict__ Y, int n,
                                                         int m, int maximize, int dedup,
                                                         unsigned char* __restrict__ out) {
  __shared__ double tile[PT][MMAX];
  const int64_t s = blockIdx.y;
  const int i = blockIdx.x * PT + threadIdx.x;
  const double* Ys = Y + s * (int64_t)n * m;
  const double sign = maximize ? 1.0 : -1.0;
  double yi[MMAX];
#pragma unroll
  for (int t = 0; t < MMAX; ++t) yi[t] = (i < n && t < m) ? sign * Ys[(int64_t)i * m + t] : 0.0;
  bool keep = i < n;
  for (int j0 = 0; j0 < n; j0 += PT) {
    __syncthreads();
    const int jl = j0 + threadIdx.x;
    for (int t = 0; t < m; ++t) tile[threadIdx.x][t] = jl < n ? sign * Ys[(int64_t)jl * m + t] : 0.0;
    __syncthreads();
    if (!keep) continue;
    const int jn = min(PT, n - j0);
    for (int jj = 0; jj < jn; ++jj) {
      bool ge = true, gt = false, eq = true;
      for (int t = 0; t < m; ++t) {
        const double yj = tile[jj][t];
        ge = ge && (yj >= yi[t]);
        gt = gt || (yj > yi[t]);
        eq = eq && (yj == yi[t]);
      }
      const int j = j0 + jj;
      if ((ge && gt) || (dedup && eq && j < i)) {
        keep = false;
        break;
      }
    }
  }
  if (i < n) out[s * (int64_t)n + i] = keep ? 1 : 0;
}

}  // namespace

extern "C" int bo_pareto_mask(const double* Y, int64_t S, int n, int m, int maximize, int dedup,
                              unsigned char* out, void* stream) {
  BO_CHECK_ARG(S >= 0 && n >= 0 && m >= 1 && m <= MMAX, "bo_pareto_mask: 1 <= m <= %d (got %d)",
               MMAX, m);
  BO_CHECK_ARG(S <= 65535, "bo_pareto_mask: at most 65535 point sets per launch");
  if (S == 0 || n == 0) return BO_OK;
  dim3 grid((unsigned)ceil_div(n, PT), (unsigned)S);
  pareto_mask_kernel<<<grid, PT, 0, as_stream(stream)>>>(Y, n, m, maximize, dedup, out);
  BO_LAUNCH_CHECK();
  return BO_OK;
}
