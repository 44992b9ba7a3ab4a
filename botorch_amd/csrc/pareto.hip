// Batched Pareto (non-dominated) masks on the device.
//
// Reference: botorch/utils/multi_objective/pareto.py:16-64 (is_non_dominated),
// called S = 2048 times per prune_inferior_points_multi_objective
// (acquisition/multi_objective/utils.py:77-161) on n x m joint posterior
// samples.  The reference switches to a Python loop over the n points for
// large n (one small torch launch per point and sample chunk: 65536 launches at
// C4); here one thread owns one point and scans all others, the point set of a
// sample streaming through LDS in 256-point tiles (coalesced [point][objective]
// rows; every lane then reads the same tile entry: LDS broadcast).
//
//   nd[s][i] = no j with Y_j >= Y_i in every objective and > in one
//              (<= / < when minimising);
//   dedup:     additionally drop i if some j < i has Y_j == Y_i (keeps the
//              first of equal points, as the reference's argmax over matches).
//
// The objective count is a template parameter (the comparisons unroll and the
// point's own objectives stay in registers), "dominates" is tested as
// all(>=) && !all(==) (all(>=) excludes NaN, so !all(==) is any(>)), and a
// block stops streaming tiles once every point it owns is dominated.  At C4's
// prune (S = 2048 samples of n = 2048 points, m = 3) the scan is bound by the
// waves holding a front point, which must see all n.
#include "common.h"

namespace {

constexpr int PT = 256;   // points per tile / threads per block
constexpr int MMAX = 8;   // objectives

template <int M>
__global__ __launch_bounds__(PT) void pareto_mask_kernel(const double* __restrict__ Y, int n,
                                                         int maximize, int dedup,
                                                         unsigned char* __restrict__ out) {
  __shared__ double tile[PT * M];
  const int64_t s = blockIdx.y;
  const int i = blockIdx.x * PT + threadIdx.x;
  const double* Ys = Y + s * (int64_t)n * M;
  const double sign = maximize ? 1.0 : -1.0;
  double yi[M];
#pragma unroll
  for (int t = 0; t < M; ++t) yi[t] = i < n ? sign * Ys[(int64_t)i * M + t] : 0.0;
  bool keep = i < n;
  for (int j0 = 0; j0 < n; j0 += PT) {
    // also the barrier before the tile is overwritten
    if (!__syncthreads_or(keep)) break;
    const int64_t lim = (int64_t)(n - j0) * M;
#pragma unroll
    for (int e = threadIdx.x; e < PT * M; e += PT)
      tile[e] = e < lim ? sign * Ys[(int64_t)j0 * M + e] : 0.0;
    __syncthreads();
    if (!keep) continue;
    const int jn = min(PT, n - j0);
    for (int jj = 0; jj < jn; ++jj) {
      bool ge = true, eq = true;
#pragma unroll
      for (int t = 0; t < M; ++t) {
        const double yj = tile[jj * M + t];
        ge = ge && (yj >= yi[t]);
        eq = eq && (yj == yi[t]);
      }
      if ((ge && !eq) || (dedup && eq && j0 + jj < i)) {
        keep = false;
        break;
      }
    }
  }
  if (i < n) out[s * (int64_t)n + i] = keep ? 1 : 0;
}

template <int M>
void launch_pareto(const double* Y, int64_t S, int n, int maximize, int dedup, unsigned char* out,
                   hipStream_t stream) {
  dim3 grid((unsigned)ceil_div(n, PT), (unsigned)S);
  pareto_mask_kernel<M><<<grid, PT, 0, stream>>>(Y, n, maximize, dedup, out);
}

}  // namespace

extern "C" int bo_pareto_mask(const double* Y, int64_t S, int n, int m, int maximize, int dedup,
                              unsigned char* out, void* stream) {
  BO_CHECK_ARG(S >= 0 && n >= 0 && m >= 1 && m <= MMAX, "bo_pareto_mask: 1 <= m <= %d (got %d)",
               MMAX, m);
  BO_CHECK_ARG(S <= 65535, "bo_pareto_mask: at most 65535 point sets per launch");
  if (S == 0 || n == 0) return BO_OK;
  const hipStream_t st = as_stream(stream);
  switch (m) {
    case 1: launch_pareto<1>(Y, S, n, maximize, dedup, out, st); break;
    case 2: launch_pareto<2>(Y, S, n, maximize, dedup, out, st); break;
    case 3: launch_pareto<3>(Y, S, n, maximize, dedup, out, st); break;
    case 4: launch_pareto<4>(Y, S, n, maximize, dedup, out, st); break;
    case 5: launch_pareto<5>(Y, S, n, maximize, dedup, out, st); break;
    case 6: launch_pareto<6>(Y, S, n, maximize, dedup, out, st); break;
    case 7: launch_pareto<7>(Y, S, n, maximize, dedup, out, st); break;
    default: launch_pareto<8>(Y, S, n, maximize, dedup, out, st); break;
  }
  BO_LAUNCH_CHECK();
  return BO_OK;
}
