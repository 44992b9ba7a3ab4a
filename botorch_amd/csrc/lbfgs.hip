// Device-resident multi-start projected L-BFGS (the candidate generator of
// optimize_acqf without the host loop).
//
// Replaces, for box-constrained candidate generation, gen_candidates_scipy's
// scipy.optimize.minimize(method="L-BFGS-B") (botorch/generation/gen.py:
// 194-267), whose every function evaluation round-trips the b x q x d iterate
// and gradient through numpy on the host.  Here each restart is its own
// problem (the reference's objective is the SUM over restarts, whose gradient
// is block-separable, so the restarts never interact except through scipy's
// shared line search), and one launch advances all of them by one function
// evaluation:
//
//   caller: f_t, g_t = -acq(x_t), -d acq/dx at the current trial points (one
//           batched forward + backward of the fused acquisition kernels);
//   here  : Armijo test of the trial step  f_t <= f + c1 g^T (x_t - x);
//           accepted -> curvature pair (s, y) into the ring of the last m,
//                        convergence tests (projected-gradient sup-norm <= pgtol,
//                        relative decrease <= ftol: scipy's defaults), new
//                        direction d = -H g on the free variables (two-loop
//                        recursion; variables at a bound with the gradient
//                        pushing outwards are fixed, as L-BFGS-B's active set),
//                        unit step;
//           rejected -> halve the step (backtracking spread over launches);
//           next trial point x_t = clamp(x + alpha d, lower, upper).
// No host synchronisation per iteration: the driver reads the status vector
// only every few evaluations to stop early.
//
// One 256-thread workgroup per restart; vectors of length n = q * d.
#include "common.h"

namespace {

constexpr int THREADS = 256;
constexpr int MMAX = 32;

enum : int { ST_INIT = -1, ST_RUN = 0, ST_PGTOL = 1, ST_FTOL = 2, ST_LSFAIL = 3 };

__device__ __forceinline__ double block_sum(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double t = 0.0;
#pragma unroll
  for (int i = 0; i < THREADS / 64; ++i) t += red[i];
  return t;
}

__device__ __forceinline__ double block_max(double v, double* red) {
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double t = red[0];
#pragma unroll
  for (int i = 1; i < THREADS / 64; ++i) t = fmax(t, red[i]);
  return t;
}

__global__ __launch_bounds__(THREADS) void lbfgs_kernel(
    int n, int m, double* __restrict__ x, double* __restrict__ f, double* __restrict__ g,
    double* __restrict__ xt, const double* __restrict__ ft, const double* __restrict__ gt,
    double* __restrict__ d, double* __restrict__ alpha, double* __restrict__ S,
    double* __restrict__ Y, double* __restrict__ rho, int* __restrict__ hcount,
    int* __restrict__ hhead, int* __restrict__ status, int* __restrict__ nacc,
    const double* __restrict__ lower, const double* __restrict__ upper, double c1, double ftol,
    double pgtol, double min_alpha) {
  __shared__ double red[THREADS / 64];
  __shared__ double a_hist[MMAX];
  __shared__ double rho_sh[MMAX];  // the ring's rho values (block-visible copy)
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  double* xb = x + (int64_t)b * n;
  double* gb = g + (int64_t)b * n;
  double* xtb = xt + (int64_t)b * n;
  const double* gtb = gt + (int64_t)b * n;
  double* db = d + (int64_t)b * n;
  double* Sb = S + (int64_t)b * m * n;
  double* Yb = Y + (int64_t)b * m * n;
  double* rb = rho + (int64_t)b * m;

  int st = status[b];
  // ring state held in registers (uniform): read once, written back once
  int k = (st == ST_INIT) ? 0 : hcount[b];
  int head = (st == ST_INIT) ? 0 : hhead[b];
  if (tid < m) rho_sh[tid] = (st == ST_INIT) ? 0.0 : rb[tid];
  if (st > 0) {
    for (int i = tid; i < n; i += THREADS) xtb[i] = xb[i];
    return;
  }
  const double fnew = ft[b];
  if (st == ST_INIT) {
    for (int i = tid; i < n; i += THREADS) {
      xb[i] = xtb[i];
      gb[i] = gtb[i];
    }
    if (tid == 0) {
      f[b] = fnew;
      hcount[b] = 0;
      hhead[b] = 0;
      nacc[b] = 0;
    }
    // a non-finite start cannot be optimised: stop it where it is
    if (!isfinite(fnew)) {
      if (tid == 0) status[b] = ST_LSFAIL;
      return;
    }
  } else {
    // Armijo test of the trial step
    double gs = 0.0;
    for (int i = tid; i < n; i += THREADS) gs += gb[i] * (xtb[i] - xb[i]);
    gs = block_sum(gs, red);
    const double fcur = f[b];
    const bool accept = isfinite(fnew) && fnew <= fcur + c1 * gs;
    if (!accept) {
      const double a = 0.5 * alpha[b];
      __syncthreads();
      if (tid == 0) {
        alpha[b] = a;
        if (a < min_alpha) status[b] = ST_LSFAIL;
      }
      const bool stop = a < min_alpha;
      for (int i = tid; i < n; i += THREADS)
        xtb[i] = stop ? xb[i] : fmin(fmax(xb[i] + a * db[i], lower[i]), upper[i]);
      return;
    }
    // curvature pair (s, y): kept (in the ring slot after the newest) only
    // when s^T y > eps y^T y, so a rejected pair never overwrites the oldest one
    double sy = 0.0, yy = 0.0;
    for (int i = tid; i < n; i += THREADS) {
      const double s_i = xtb[i] - xb[i];
      const double y_i = gtb[i] - gb[i];
      sy += s_i * y_i;
      yy += y_i * y_i;
    }
    sy = block_sum(sy, red);
    yy = block_sum(yy, red);
    const bool keep = sy > 2.220446049250313e-16 * yy && sy > 0.0;
    double* sh = Sb + (int64_t)head * n;
    double* yh = Yb + (int64_t)head * n;
    for (int i = tid; i < n; i += THREADS) {
      if (keep) {
        sh[i] = xtb[i] - xb[i];
        yh[i] = gtb[i] - gb[i];
      }
      xb[i] = xtb[i];
      gb[i] = gtb[i];
    }
    __syncthreads();
    if (keep) {
      if (tid == 0) {
        rb[head] = 1.0 / sy;
        rho_sh[head] = 1.0 / sy;
      }
      head = (head + 1) % m;
      k = min(k + 1, m);
    }
    if (tid == 0) {
      hhead[b] = head;
      hcount[b] = k;
      f[b] = fnew;
      nacc[b] += 1;
    }
    // relative decrease (scipy L-BFGS-B: (f_k - f_{k+1}) / max(|f_k|, |f_{k+1}|, 1) <= ftol)
    if ((fcur - fnew) <= ftol * fmax(fmax(fabs(fcur), fabs(fnew)), 1.0)) {
      if (tid == 0) status[b] = ST_FTOL;
      for (int i = tid; i < n; i += THREADS) xtb[i] = xb[i];
      return;
    }
  }
  __syncthreads();
  // projected-gradient sup-norm
  double pg = 0.0;
  for (int i = tid; i < n; i += THREADS)
    pg = fmax(pg, fabs(fmin(fmax(xb[i] - gb[i], lower[i]), upper[i]) - xb[i]));
  pg = block_max(pg, red);
  if (pg <= pgtol) {
    if (tid == 0) status[b] = ST_PGTOL;
    for (int i = tid; i < n; i += THREADS) xtb[i] = xb[i];
    return;
  }
  // ---- direction: two-loop recursion on the free variables ----
  // q = g_F  (kept in d)
  for (int i = tid; i < n; i += THREADS) {
    const bool fixed = (xb[i] <= lower[i] && gb[i] > 0.0) || (xb[i] >= upper[i] && gb[i] < 0.0);
    db[i] = fixed ? 0.0 : gb[i];
  }
  __syncthreads();
  for (int j = 0; j < k; ++j) {  // newest -> oldest
    const int slot = (head - 1 - j + 2 * m) % m;
    const double* sj = Sb + (int64_t)slot * n;
    const double* yj = Yb + (int64_t)slot * n;
    double v = 0.0;
    for (int i = tid; i < n; i += THREADS) v += sj[i] * db[i];
    const double a = rho_sh[slot] * block_sum(v, red);
    if (tid == 0) a_hist[j] = a;
    for (int i = tid; i < n; i += THREADS) db[i] -= a * yj[i];
    __syncthreads();
  }
  double gamma;
  if (k > 0) {
    const int slot = (head - 1 + m) % m;
    const double* yj = Yb + (int64_t)slot * n;
    double yy = 0.0;
    for (int i = tid; i < n; i += THREADS) yy += yj[i] * yj[i];
    yy = block_sum(yy, red);
    gamma = (1.0 / rho_sh[slot]) / yy;  // s^T y / y^T y
  } else {
    // first step: unit sup-norm move, as scipy's initial step 1/||g||
    double gn = 0.0;
    for (int i = tid; i < n; i += THREADS) gn += db[i] * db[i];
    gn = sqrt(block_sum(gn, red));
    gamma = gn > 0.0 ? fmin(1.0, 1.0 / gn) : 1.0;
  }
  for (int i = tid; i < n; i += THREADS) db[i] *= gamma;
  __syncthreads();
  for (int j = k - 1; j >= 0; --j) {  // oldest -> newest
    const int slot = (head - 1 - j + 2 * m) % m;
    const double* sj = Sb + (int64_t)slot * n;
    const double* yj = Yb + (int64_t)slot * n;
    double v = 0.0;
    for (int i = tid; i < n; i += THREADS) v += yj[i] * db[i];
    const double beta = rho_sh[slot] * block_sum(v, red);
    const double a = a_hist[j];
    for (int i = tid; i < n; i += THREADS) db[i] += (a - beta) * sj[i];
    __syncthreads();
  }
  // d = -H g_F on the free variables; fall back to steepest descent if not a descent direction
  double gd = 0.0;
  for (int i = tid; i < n; i += THREADS) {
    const bool fixed = (xb[i] <= lower[i] && gb[i] > 0.0) || (xb[i] >= upper[i] && gb[i] < 0.0);
    const double v = fixed ? 0.0 : -db[i];
    db[i] = v;
    gd += gb[i] * v;
  }
  gd = block_sum(gd, red);
  if (!(gd < 0.0)) {
    for (int i = tid; i < n; i += THREADS) {
      const bool fixed = (xb[i] <= lower[i] && gb[i] > 0.0) || (xb[i] >= upper[i] && gb[i] < 0.0);
      db[i] = fixed ? 0.0 : -gb[i];
    }
    __syncthreads();
    if (tid == 0) hcount[b] = 0;
  }
  __syncthreads();
  if (tid == 0) {
    alpha[b] = 1.0;
    status[b] = ST_RUN;
  }
  for (int i = tid; i < n; i += THREADS) xtb[i] = fmin(fmax(xb[i] + db[i], lower[i]), upper[i]);
}

}  // namespace

extern "C" int bo_lbfgs_step(int B, int n, int m, double* x, double* f, double* g, double* xt,
                             const double* ft, const double* gt, double* d, double* alpha,
                             double* S, double* Y, double* rho, int* hcount, int* hhead,
                             int* status, int* nacc, const double* lower, const double* upper,
                             double c1, double ftol, double pgtol, double min_alpha,
                             void* stream) {
  BO_CHECK_ARG(n >= 1 && m >= 1 && m <= MMAX, "bo_lbfgs_step: n=%d, m=%d (1..%d)", n, m, MMAX);
  if (B == 0) return BO_OK;
  lbfgs_kernel<<<B, THREADS, 0, as_stream(stream)>>>(n, m, x, f, g, xt, ft, gt, d, alpha, S, Y,
                                                      rho, hcount, hhead, status, nacc, lower,
                                                      upper, c1, ftol, pgtol, min_alpha);
  BO_LAUNCH_CHECK();
  return BO_OK;
}
