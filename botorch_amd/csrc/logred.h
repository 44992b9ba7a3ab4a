// Smoothed log-improvement reductions of the LogEI family, per MC sample.
//
//   li_a = log_fatplus(f_a - best_f, tau_relu)    (fat)   botorch/utils/safe_math.py:293-320
//        | log_softplus(f_a - best_f, tau_relu)   (!fat)  :226-247
//   u    = fatmax_a(li_a, tau_max, alpha = 2)     (fat)   :323-352 via _inf_max_helper :149-187
//        | smooth_amax_a(li_a, tau_max)           (!fat)  :250-273
// (acquisition/logei.py:219-234, 509-534; q_reduction at :122), and the t-batch
// value is logmeanexp_s(u_s) (:209-223), reduced by the callers.
//
// The gradients follow torch autograd through the reference expressions,
// including the anchor path of fatmax: its value M + tau log sum_b p((M - li_b)/tau)
// is NOT invariant to the anchor M = max_b li_b, so d u / d li_a carries
// (1 + sum_b p'(x_b) / P) / #argmax on the maximal entries (amax splits ties
// evenly), beside the direct term -p'(x_a) / P.
#pragma once

#include "common.h"

struct LogRedParams {
  double tau_relu;
  double tau_max;
  int fat;
};

// torch.nn.functional.softplus(x) with beta = 1, threshold = 20, and its derivative.
__device__ __forceinline__ double torch_softplus(double x) { return x > 20.0 ? x : log1p(exp(x)); }
__device__ __forceinline__ double torch_softplus_grad(double x) {
  if (x > 20.0) return 1.0;
  const double z = exp(x);
  return z / (z + 1.0);
}

// log of the smoothed ReLU of z and d/dz.
__device__ __forceinline__ double log_soft_relu(double z, const LogRedParams& p, double* dz) {
  const double tau = p.tau_relu;
  if (p.fat) {
    // fatplus = tau (softplus(x) + 0.1 / (1 + x^2)),  x = z / tau
    const double x = z / tau;
    const double c = 1.0 / (1.0 + x * x);
    const double h = torch_softplus(x) + 0.1 * c;
    if (dz) *dz = (torch_softplus_grad(x) - 0.2 * x * c * c) / (h * tau);
    return log(tau * h);
  }
  // log_softplus (fp64 cutoffs lower = -35, upper = 32)
  const double beta = 1.0 / tau;
  const double x = z / tau;
  if (!(x > -35.0)) {
    if (dz) *dz = 1.0 / tau;
    return x + log(tau);
  }
  const double xb = z * beta;
  if (xb > 32.0) {
    if (dz) *dz = 1.0 / z;
    return log(z);
  }
  const double e = exp(xb);
  const double sp = log1p(e) / beta;
  if (dz) *dz = (e / (e + 1.0)) / sp;
  return log(sp);
}

// q-reduction of li[0..q) (fat: fatmax with alpha = 2; else smooth_amax).
// g (optional) receives d u / d li_a.
template <int QMAX>
__device__ __forceinline__ double log_q_reduce(const double (&li)[QMAX], int q,
                                               const LogRedParams& p, double (*g)[QMAX]) {
  const double tau = p.tau_max;
  double M = -INFINITY;
#pragma unroll
  for (int a = 0; a < QMAX; ++a)
    if (a < q) M = fmax(M, li[a]);
  if (p.fat) {
    // _pareto(x, alpha=2): beta_1 = 2, beta_0 = 2 -> 2 / (2 + 2 x + x^2)
    double P = 0.0, dP = 0.0;
    int cnt = 0;
#pragma unroll
    for (int a = 0; a < QMAX; ++a) {
      if (a < q) {
        const double x = (M - li[a]) / tau;
        const double den = 2.0 + 2.0 * x + x * x;
        P += 2.0 / den;
        dP += -2.0 * (2.0 + 2.0 * x) / (den * den);  // p'(x)
        cnt += (li[a] == M);
      }
    }
    if (g) {
      const double anchor = (1.0 + dP / P) / (double)cnt;
#pragma unroll
      for (int a = 0; a < QMAX; ++a) {
        if (a < q) {
          const double x = (M - li[a]) / tau;
          const double den = 2.0 + 2.0 * x + x * x;
          const double pd = -2.0 * (2.0 + 2.0 * x) / (den * den);
          (*g)[a] = -pd / P + ((li[a] == M) ? anchor : 0.0);
        } else {
          (*g)[a] = 0.0;
        }
      }
    }
    return M + tau * log(P);
  }
  // smooth_amax = tau * logsumexp(li / tau)  (softmax gradient)
  const double Ms = M / tau;
  double ssum = 0.0;
#pragma unroll
  for (int a = 0; a < QMAX; ++a)
    if (a < q) ssum += exp(li[a] / tau - Ms);
  if (g) {
#pragma unroll
    for (int a = 0; a < QMAX; ++a) (*g)[a] = (a < q) ? exp(li[a] / tau - Ms) / ssum : 0.0;
  }
  return tau * (Ms + log(ssum));
}

// Online logsumexp pair (max, sum of exp(v - max)) and its merge.
struct LseAcc {
  double m;
  double s;
};
__device__ __forceinline__ LseAcc lse_push(LseAcc a, double v) {
  if (v > a.m) {
    a.s = a.s * exp(a.m - v) + 1.0;
    a.m = v;
  } else {
    a.s += exp(v - a.m);
  }
  return a;
}
__device__ __forceinline__ LseAcc lse_merge(LseAcc a, LseAcc b) {
  if (b.m == -INFINITY) return a;
  if (a.m == -INFINITY) return b;
  const double m = fmax(a.m, b.m);
  return LseAcc{m, a.s * exp(a.m - m) + b.s * exp(b.m - m)};
}
