// Hit-and-run Markov chain over a polytope {y : A y <= b} on the host.
//
// Native replacement of the per-step Python loop of sample_polytope
// (botorch/utils/sampling.py:219-309), which the reference runs on the CPU
// ("a lot of looping going on", :683-684) for the raw samples of
// gen_batch_initial_conditions under linear constraints (optim/initializers.py:
// 178-240, 365-375): ~10^4 burn-in + 32 n q chained steps, one dependent step
// after another.  The chain is inherently sequential and each step is a few
// hundred flops, so it runs on one host core; the random draws it consumes
// (uniforms, unit directions and their products with A) are made by the caller
// with torch exactly as the reference makes them.
//
// Step t (direction r = R[t], its products a = AR[t], uniform u[t]):
//   s_i   = max(b_i - A_i y, 0)                      slack of constraint i
//   w_i   = s_i / a_i
//   hi    = min { w_i : w_i > 0 }   (no such i: FLT_MAX, torch.finfo().max)
//   lo    = max { w_i : w_i < 0 }   (no such i: -FLT_MAX)
//   a face the point sits on (w_i == 0) caps hi at 0 when a_i > 0 and lifts
//   lo to 0 when a_i < 0;
//   y    += (lo + u[t] (hi - lo)) r
// and after n0 burn-in steps every n_thin-th point is kept.
#include <stdint.h>

#include <cfloat>
#include <vector>

#include "../../include/botorch_amd.h"

void bo_set_error(const char* fmt, ...);

extern "C" int bo_hit_and_run_host(const double* A, const double* b, int64_t m, int64_t k,
                                   const double* y0, const double* R, const double* AR,
                                   const double* u, int64_t n_tot, int64_t n0, int64_t n_thin,
                                   double* out, int64_t n) {
  if (!A || !b || !y0 || !R || !AR || !u || !out || m < 0 || k < 1 || n_thin < 1 || n0 < 0 ||
      n < 0 || n_tot != n0 + n * n_thin) {
    bo_set_error("bo_hit_and_run_host: bad arguments (m=%lld k=%lld n_tot=%lld n0=%lld n=%lld "
                 "n_thin=%lld)", (long long)m, (long long)k, (long long)n_tot, (long long)n0,
                 (long long)n, (long long)n_thin);
    return BO_ERR_ARG;
  }
  // torch.finfo() is the default dtype's (float32) range
  const double big = (double)FLT_MAX;
  std::vector<double> y(y0, y0 + k);
  for (int64_t t = 0; t < n_tot; ++t) {
    const double* r = R + t * k;
    const double* a = AR + t * m;
    double hi = big, lo = -big;
    bool any_pos = false, any_neg = false, cap_hi = false, lift_lo = false;
    for (int64_t i = 0; i < m; ++i) {
      const double* Ai = A + i * k;
      double ay = 0.0;
      for (int64_t j = 0; j < k; ++j) ay += Ai[j] * y[j];
      double s = b[i] - ay;
      if (s < 0.0) s = 0.0;  // clamp(min=0) (NaN passes, as in torch)
      const double w = s / a[i];
      if (w > 0.0) {
        if (!any_pos || w < hi) hi = w;
        any_pos = true;
      } else if (w < 0.0) {
        if (!any_neg || w > lo) lo = w;
        any_neg = true;
      } else if (w == 0.0) {
        if (a[i] > 0.0) cap_hi = true;
        if (a[i] < 0.0) lift_lo = true;
      }
    }
    if (cap_hi && hi > 0.0) hi = 0.0;
    if (lift_lo && lo < 0.0) lo = 0.0;
    const double step = lo + u[t] * (hi - lo);
    for (int64_t j = 0; j < k; ++j) {
      const double dy = step * r[j];
      y[j] = y[j] + dy;
    }
    const int64_t kept = t - n0;
    if (kept >= 0 && kept % n_thin == 0) {
      double* o = out + (kept / n_thin) * k;
      for (int64_t j = 0; j < k; ++j) o[j] = y[j];
    }
  }
  return BO_OK;
}
