// Backward of the fused qEI/qNEI forward and of the batched exact posterior.
//
// gen_candidates_scipy differentiates -acqf(X).sum() w.r.t. X once per
// L-BFGS-B iteration (botorch/generation/gen.py:194-222).  The chain is
//   reduction (one-hot q-argmax of relu(f - best_f), 1/S)  ->  d mu', d L_q
//   -> Cholesky backward (torch's linalg.cholesky backward, Murray 2016)  -> d Sigma'
//   -> Standardize: d mu* = s d mu', d Sigma* = s^2 d Sigma'
//   -> exact prediction: mu* = c + K*x alpha,  Sigma* = K** - K*x A^{-1} K*x^T
//        d K*x = d mu* alpha^T - G W,   G = d Sigma* + d Sigma*^T,
//        W = K*x A^{-1} = R L^{-1}  (computed on the gradient path of the forward)
//        d K** = d Sigma*
//   -> kernel derivative  dk/dx_i = -k (x_i - x_k)/ell^2 (RBF) and the
//      Matern-5/2 form, reduced over the training points.
// The model caches carry no gradient (detach_test_caches, botorch/models/
// utils/assorted.py:286-298), so nothing flows to L^{-1} or alpha.
#include "common.h"

#include <algorithm>
#include "logred.h"

namespace {

constexpr int QMAX = 16;
constexpr int DP = 8;
constexpr int THREADS = 256;
constexpr int SMAX = 256;  // samples staged in LDS per pass (winner masks + base samples)
// row stride of the staged base samples: a lane per sample reads its own row,
// and a 16-double (128 B) stride put the wave's 64 rows on two bank groups
constexpr int ZST = QMAX + 1;

enum { MODE_QEI = 1, MODE_QNEI = 2, MODE_QLOGEI = 4, MODE_QLOGNEI = 5 };

// qNEI (cached root): the samples carry the baseline term F[s][row] =
// (Z_base T)[s][row] (row = b * Qp + a); its cotangent dF (same layout) is the
// winner weight, from which the host forms dT = Z_base^T dF.
// torch's linalg.cholesky backward (Murray 2016) for one q x q factor held in
// LDS: gA = L^{-T} Phi(L^T dL) L^{-1}, Phi = lower half with the diagonal
// halved, symmetrised.  Writes the q x q result to out (row-major).
__device__ __forceinline__ void chol_backward_lds(int q, double (*L)[QMAX + 1],
                                                  double (*dL)[QMAX + 1], double (*Li)[QMAX + 1],
                                                  double (*Pm)[QMAX + 1], double (*Tm)[QMAX + 1],
                                                  double* __restrict__ out, int tid) {
  // L^{-1} by forward substitution, one column per thread.
  if (tid < q) {
    const int c = tid;
    for (int r = 0; r < q; ++r) {
      double s = (r == c) ? 1.0 : 0.0;
      for (int k = c; k < r; ++k) s = fma(-L[r][k], Li[k][c], s);
      Li[r][c] = (r >= c) ? s / L[r][r] : 0.0;
    }
  }
  __syncthreads();
  // X = tril(L^T dL);  P = 0.5 (X + tril(X, -1)^T)   (torch cholesky_backward)
  if (tid < q * q) {
    const int i = tid / q, j = tid % q;
    const int lo = i > j ? i : j;
    double x = 0.0;
    for (int k = lo; k < q; ++k) x = fma(L[k][i], dL[k][j], x);  // (L^T dL)[i][j]
    if (i >= j) Tm[i][j] = x;
  }
  __syncthreads();
  if (tid < q * q) {
    const int i = tid / q, j = tid % q;
    Pm[i][j] = 0.5 * ((i >= j) ? Tm[i][j] : Tm[j][i]);
  }
  __syncthreads();
  // gA = L^{-T} P L^{-1}:  T = P L^{-1}, then gA = L^{-T} T
  if (tid < q * q) {
    const int i = tid / q, j = tid % q;
    double x = 0.0;
    for (int k = j; k < q; ++k) x = fma(Pm[i][k], Li[k][j], x);
    Tm[i][j] = x;
  }
  __syncthreads();
  if (tid < q * q) {
    const int i = tid / q, j = tid % q;
    double x = 0.0;
    for (int k = i; k < q; ++k) x = fma(Li[k][i], Tm[k][j], x);
    out[i * q + j] = x;
  }
}

// Standalone batched Cholesky backward: dL (B x q x q, lower) -> dA.
__global__ __launch_bounds__(THREADS) void chol_backward_kernel(int q, const double* __restrict__ Lg,
                                                                const double* __restrict__ dLg,
                                                                double* __restrict__ dA) {
  __shared__ double L[QMAX][QMAX + 1];
  __shared__ double dL[QMAX][QMAX + 1];
  __shared__ double Li[QMAX][QMAX + 1];
  __shared__ double Pm[QMAX][QMAX + 1];
  __shared__ double Tm[QMAX][QMAX + 1];
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  if (tid < q * q) {
    const int a = tid / q, c = tid % q;
    L[a][c] = Lg[((int64_t)b * q + a) * q + c];
    dL[a][c] = (c <= a) ? dLg[((int64_t)b * q + a) * q + c] : 0.0;
  }
  __syncthreads();
  chol_backward_lds(q, L, dL, Li, Pm, Tm, dA + (int64_t)b * q * q, tid);
}

// Batched Cholesky backward for 16 < q <= 64 (the joint (r+q) roots of the
// generic qNEI route and the q x q roots of large q-batches): the same algebra
// as chol_backward_lds with element loops over q x q and four 64 x 65 LDS
// planes (133 KB of gfx950's 160 KB); dL is read straight from global memory.
constexpr int QBIG = 64;
__global__ __launch_bounds__(THREADS) void chol_backward_big_kernel(
    int q, const double* __restrict__ Lg, const double* __restrict__ dLg, double* __restrict__ dA) {
  __shared__ double L[QBIG][QBIG + 1];
  __shared__ double Li[QBIG][QBIG + 1];
  __shared__ double Pm[QBIG][QBIG + 1];
  __shared__ double Tm[QBIG][QBIG + 1];
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int qq = q * q;
  const double* Lb = Lg + (int64_t)b * qq;
  const double* dLb = dLg + (int64_t)b * qq;
  for (int e = tid; e < qq; e += THREADS) L[e / q][e % q] = Lb[e];
  __syncthreads();
  // L^{-1}: one column per thread (forward substitution)
  for (int c = tid; c < q; c += THREADS) {
    for (int r = 0; r < q; ++r) {
      double s = (r == c) ? 1.0 : 0.0;
      for (int k = c; k < r; ++k) s = fma(-L[r][k], Li[k][c], s);
      Li[r][c] = (r >= c) ? s / L[r][r] : 0.0;
    }
  }
  // X = tril(L^T tril(dL))
  for (int e = tid; e < qq; e += THREADS) {
    const int i = e / q, j = e % q;
    if (i >= j) {
      double x = 0.0;
      for (int k = i; k < q; ++k) x = fma(L[k][i], dLb[k * q + j], x);
      Tm[i][j] = x;
    }
  }
  __syncthreads();
  for (int e = tid; e < qq; e += THREADS) {
    const int i = e / q, j = e % q;
    Pm[i][j] = 0.5 * ((i >= j) ? Tm[i][j] : Tm[j][i]);
  }
  __syncthreads();
  for (int e = tid; e < qq; e += THREADS) {  // T = P L^{-1}
    const int i = e / q, j = e % q;
    double x = 0.0;
    for (int k = j; k < q; ++k) x = fma(Pm[i][k], Li[k][j], x);
    Tm[i][j] = x;
  }
  __syncthreads();
  double* out = dA + (int64_t)b * qq;
  for (int e = tid; e < qq; e += THREADS) {  // gA = L^{-T} T
    const int i = e / q, j = e % q;
    double x = 0.0;
    for (int k = i; k < q; ++k) x = fma(Li[k][i], Tm[k][j], x);
    out[e] = x;
  }
}

template <int MODE>
__global__ __launch_bounds__(THREADS) void qmc_backward_kernel(
    int q, const double* __restrict__ mean, const double* __restrict__ Lq,
    const double* __restrict__ Z, int S, double best_f, const double* __restrict__ best_f_s,
    const double* __restrict__ dacq, double* __restrict__ dmean, double* __restrict__ dcov,
    const double* __restrict__ F, int64_t ldF, int Qp, double* __restrict__ dF) {
  __shared__ double L[QMAX][QMAX + 1];
  __shared__ double Li[QMAX][QMAX + 1];   // L^{-1}
  __shared__ double dL[QMAX][QMAX + 1];
  __shared__ double Pm[QMAX][QMAX + 1];
  __shared__ double Tm[QMAX][QMAX + 1];
  __shared__ double mu[QMAX];
  __shared__ unsigned short win[SMAX];
  __shared__ double wgt[SMAX];
  __shared__ double Zs[SMAX * ZST];    // the chunk's base samples (shared by every t-batch)

  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  if (tid < q * q) {
    const int a = tid / q, c = tid % q;
    L[a][c] = Lq[((int64_t)b * q + a) * q + c];
  }
  if (tid < q) mu[tid] = mean[(int64_t)b * q + tid];
  __syncthreads();
  const double g = dacq[b] / (double)S;

  double dmu_acc = 0.0, dl_acc = 0.0;
  // thread (a, j), j <= a, accumulates dL[a][j]; threads 0..q-1 also dmu.
  int ta = -1, tj = -1;
  if (tid < q * q) {
    ta = tid / q;
    tj = tid % q;
  }
  for (int s0 = 0; s0 < S; s0 += SMAX) {
    const int ns = min(SMAX, S - s0);
    for (int e = tid; e < ns * q; e += THREADS) Zs[(e / q) * ZST + e % q] = Z[(int64_t)s0 * q + e];
    // Pass 1: the winning (maximal, non-clamped) q-index set per sample.
    __syncthreads();  // Zs
    for (int s = tid; s < ns; s += THREADS) {
      const double* z = Zs + s * ZST;
      double zr[QMAX];  // the sample's row once, in registers
#pragma unroll
      for (int j = 0; j < QMAX; ++j) zr[j] = j < q ? z[j] : 0.0;
      const double bf = (MODE == MODE_QNEI) ? best_f_s[s0 + s] : best_f;
      double v[QMAX];
      double m = 0.0;
      const double* Fs = (MODE == MODE_QNEI) ? F + (int64_t)(s0 + s) * ldF + (int64_t)b * Qp : nullptr;
#pragma unroll
      for (int a = 0; a < QMAX; ++a) {
        if (a < q) {
          double f = mu[a];
          if (MODE == MODE_QNEI) f += Fs[a];
#pragma unroll
          for (int j = 0; j <= a; ++j) f = fma(L[a][j], zr[j], f);
          v[a] = f - bf;
          m = fmax(m, fmax(v[a], 0.0));
        }
      }
      // torch: amax splits the gradient evenly among all maximal entries;
      // clamp_min(0) passes it where f - best_f >= 0.
      unsigned mask = 0, cnt = 0;
#pragma unroll
      for (int a = 0; a < QMAX; ++a) {
        if (a < q && fmax(v[a], 0.0) == m) {
          ++cnt;
          if (v[a] >= 0.0) mask |= 1u << a;
        }
      }
      win[s] = (unsigned short)mask;
      wgt[s] = cnt ? g / (double)cnt : 0.0;
      if (MODE == MODE_QNEI) {
        double* dFs = dF + (int64_t)(s0 + s) * ldF + (int64_t)b * Qp;
        const double w = wgt[s];
        for (int a = 0; a < q; ++a) dFs[a] = (mask >> a & 1u) ? w : 0.0;
      }
    }
    __syncthreads();
    // Pass 2: deterministic accumulation per (a, j), operands from LDS (a
    // zero weight where a did not win: the same sums as a branch, in order).
    if (ta >= 0 && tj <= ta) {
#pragma unroll 8
      for (int s = 0; s < ns; ++s) {
        const double w = (win[s] >> ta & 1u) ? wgt[s] : 0.0;
        dl_acc = fma(w, Zs[s * ZST + tj], dl_acc);
        dmu_acc += w;
      }
    }
    __syncthreads();
  }
  if (ta >= 0) {
    dL[ta][tj] = (tj <= ta) ? dl_acc : 0.0;
    if (tj == 0) dmean[(int64_t)b * q + ta] = dmu_acc;
  }
  chol_backward_lds(q, L, dL, Li, Pm, Tm, dcov + (int64_t)b * q * q, tid);
}

// Backward of the qLogEI / qLogNEI reduction (logred.h):  with u_s the q-reduced
// smoothed log improvement of sample s and acq = logmeanexp_s u_s,
//   d acq / d u_s = exp(u_s - acq) / S,
//   w[s][a] = dacq * exp(u_s - acq) / S * du_s/dli_a * dli_a/dz_a   (z = f - best_f),
// then d mu'_a = sum_s w[s][a],  dL[a][j] = sum_s w[s][a] Z[s][j]  (dense weights,
// staged per sample chunk in LDS), and the q x q Cholesky backward as for qEI.
// LOGNEI also returns dF[s][b*Qp + a] = w[s][a] (the cached-root baseline term).
template <bool PERSAMPLE>
__global__ __launch_bounds__(THREADS) void qmc_log_backward_kernel(
    int q, const double* __restrict__ mean, const double* __restrict__ Lq,
    const double* __restrict__ Z, int S, double best_f, const double* __restrict__ best_f_s,
    const double* __restrict__ acq_fwd, LogRedParams lp, const double* __restrict__ dacq,
    double* __restrict__ dmean, double* __restrict__ dcov, const double* __restrict__ F,
    int64_t ldF, int Qp, double* __restrict__ dF) {
  constexpr int SL = 256;  // samples per LDS chunk (weights + base samples: two workgroups per CU)
  __shared__ double L[QMAX][QMAX + 1];
  __shared__ double Li[QMAX][QMAX + 1];
  __shared__ double dL[QMAX][QMAX + 1];
  __shared__ double Pm[QMAX][QMAX + 1];
  __shared__ double Tm[QMAX][QMAX + 1];
  __shared__ double mu[QMAX];
  __shared__ double w[SL][QMAX + 1];
  __shared__ double Zs[SL * ZST];

  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  if (tid < q * q) {
    const int a = tid / q, c = tid % q;
    L[a][c] = Lq[((int64_t)b * q + a) * q + c];
  }
  if (tid < q) mu[tid] = mean[(int64_t)b * q + tid];
  __syncthreads();
  const double g = dacq[b] / (double)S;
  const double a_fwd = acq_fwd[b];

  double dmu_acc = 0.0, dl_acc = 0.0;
  int ta = -1, tj = -1;
  if (tid < q * q) {
    ta = tid / q;
    tj = tid % q;
  }
  for (int s0 = 0; s0 < S; s0 += SL) {
    const int ns = min(SL, S - s0);
    for (int e = tid; e < ns * q; e += THREADS) Zs[(e / q) * ZST + e % q] = Z[(int64_t)s0 * q + e];
    __syncthreads();
    for (int s = tid; s < ns; s += THREADS) {
      const double* z = Zs + s * ZST;
      double zr[QMAX];
#pragma unroll
      for (int j = 0; j < QMAX; ++j) zr[j] = j < q ? z[j] : 0.0;
      const double bf = PERSAMPLE ? best_f_s[s0 + s] : best_f;
      const double* Fs = PERSAMPLE ? F + (int64_t)(s0 + s) * ldF + (int64_t)b * Qp : nullptr;
      double li[QMAX], dli[QMAX], gq[QMAX];
#pragma unroll
      for (int a = 0; a < QMAX; ++a) {
        li[a] = 0.0;
        dli[a] = 0.0;
        if (a < q) {
          double f = mu[a];
          if (PERSAMPLE) f += Fs[a];
#pragma unroll
          for (int j = 0; j <= a; ++j) f = fma(L[a][j], zr[j], f);
          li[a] = log_soft_relu(f - bf, lp, &dli[a]);
        }
      }
      const double u = log_q_reduce<QMAX>(li, q, lp, &gq);
      const double ws = g * exp(u - a_fwd);
#pragma unroll
      for (int a = 0; a < QMAX; ++a) {
        if (a < q) {
          const double v = ws * gq[a] * dli[a];
          w[s][a] = v;
          if (PERSAMPLE) dF[(int64_t)(s0 + s) * ldF + (int64_t)b * Qp + a] = v;
        }
      }
    }
    __syncthreads();
    if (ta >= 0 && tj <= ta) {
#pragma unroll 8
      for (int s = 0; s < ns; ++s) {
        const double v = w[s][ta];
        dl_acc = fma(v, Zs[s * ZST + tj], dl_acc);
        dmu_acc += v;
      }
    }
    __syncthreads();
  }
  if (ta >= 0) {
    dL[ta][tj] = (tj <= ta) ? dl_acc : 0.0;
    if (tj == 0) dmean[(int64_t)b * q + ta] = dmu_acc;
  }
  chol_backward_lds(q, L, dL, Li, Pm, Tm, dcov + (int64_t)b * q * q, tid);
}

static_assert(THREADS == QMAX * QMAX, "post_backward: one G entry per thread");

// dX for one t-batch per workgroup (training points [kb, ke): all of them, or
// one split of several -- see post_backward_kernel).  The G W term is a (16 x 16) x (16 x 16k)
// product per block of 16 training points, so each wave runs it on the matrix
// cores: A = G[a][j] (fixed for the kernel, in registers), B = W[j][k] (the
// t-batch's 16 W rows, 128-B row segments, each element read once), and the
// accumulator leaves lane (jq, kc) with D for rows jq + 4r and training point
// k0 + kc -- fixed rows per lane, so their coordinates stay in registers while
// the lane evaluates dk/dx for its 4 (row, point) pairs.  The waves stride over
// the 16-point blocks; per-row sums are combined by shuffles and LDS.
template <int KIND, int ND>
__device__ __forceinline__ void post_backward_body(
    int b, int q, int Qp, const double* __restrict__ Xq, const double* __restrict__ Xt, int n,
    const double* __restrict__ W, int64_t ldw, const double* __restrict__ alpha,
    const double* __restrict__ dmean, const double* __restrict__ dcov,
    const double* __restrict__ E, int64_t lde,
    const double* __restrict__ ls, double outputscale, double ystd, int d, int accumulate,
    double* __restrict__ dX, int wkm, int kb = 0, int ke = -1, double* __restrict__ part = nullptr) {
  if (ke < 0) ke = n;
  __shared__ double G[QMAX][QMAX + 1];
  __shared__ double dmu[QMAX];
  __shared__ double xs[QMAX][DP];
  __shared__ double red[THREADS / 64][QMAX][DP + 1];

  const int tid = threadIdx.x;
  const int row0 = b * Qp;
  const double s2 = ystd * ystd;
  {  // THREADS == QMAX * QMAX: one entry of G per thread, zero outside q x q
    const int a = tid / QMAX, c = tid % QMAX;
    const double* dc = dcov ? dcov + (int64_t)b * q * q : nullptr;
    G[a][c] = (dc && a < q && c < q) ? s2 * (dc[a * q + c] + dc[c * q + a]) : 0.0;
  }
  if (tid < QMAX) dmu[tid] = (dmean && tid < q) ? ystd * dmean[(int64_t)b * q + tid] : 0.0;
  if (tid < QMAX * DP) {
    const int a = tid / DP, t = tid % DP;
    xs[a][t] = a < q ? Xq[(int64_t)(row0 + a) * DP + t] : 0.0;
  }
  __syncthreads();

  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int kc = lane & 15;   // training point within a 16-block (MFMA column)
  const int jq = lane >> 4;   // MFMA inner index; output rows jq + 4 r
  double ga[4], dm[4], xa[4][ND], acc[4][ND];
#pragma unroll
  for (int s = 0; s < 4; ++s) ga[s] = G[kc][4 * s + jq];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    dm[r] = dmu[jq + 4 * r];
#pragma unroll
    for (int t = 0; t < ND; ++t) {
      xa[r][t] = xs[jq + 4 * r][t];
      acc[r][t] = 0.0;
    }
  }
  // two 16-point blocks per iteration (independent MFMA / exp chains); the
  // second one's points past n are masked like any ragged block
  auto block = [&](int k0) {
    const int k = k0 + kc;
    const bool kv = k < ke;
    v4d c = v4d_zero();
    if (W) {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int j = 4 * s + jq;
        const int64_t wi = wkm ? (int64_t)k * ldw + row0 + j : (int64_t)(row0 + j) * ldw + k;
        const double wb = (j < q && kv) ? W[wi] : 0.0;
        c = mfma_f64(ga[s], wb, c);
      }
    }
    const double al = (alpha && kv) ? alpha[k] : 0.0;
    double xt[ND];
#pragma unroll
    for (int t = 0; t < ND; ++t) xt[t] = kv ? Xt[(int64_t)k * DP + t] : 0.0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int a = jq + 4 * r;
      double D = fma(dm[r], al, -c[r]);
      if (E && a < q && kv) D += E[(int64_t)(row0 + a) * lde + k];
      double diff[ND];
      double d2 = 0.0;
#pragma unroll
      for (int t = 0; t < ND; ++t) {
        diff[t] = xa[r][t] - xt[t];
        d2 = fma(diff[t], diff[t], d2);
      }
      const double f = D * dkernel_factor<KIND>(d2, outputscale);
#pragma unroll
      for (int t = 0; t < ND; ++t) acc[r][t] = fma(f, diff[t], acc[r][t]);
    }
  };
  constexpr int KSTRIDE = 16 * (THREADS / 64);
  for (int k0 = kb + wave * 16; k0 < ke; k0 += 2 * KSTRIDE) {  // wave-uniform trip count
    block(k0);
    block(k0 + KSTRIDE);
  }
  // sum over the 16 lanes of a row group (kc), then over the waves
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int t = 0; t < ND; ++t) {
      double v = acc[r][t];
      v += __shfl_xor(v, 1);
      v += __shfl_xor(v, 2);
      v += __shfl_xor(v, 4);
      v += __shfl_xor(v, 8);
      if (kc == 0) red[wave][jq + 4 * r][t] = v;
    }
  __syncthreads();
  if (tid < q * d) {
    const int a = tid / d, t = tid % d;
    double s = 0.0;
#pragma unroll
    for (int w = 0; w < THREADS / 64; ++w) s += red[w][a][t];
    // K** terms: Sigma*[a][c] = K**(a, c) - ..., d K** = d Sigma* (c != a; the
    // diagonal is the constant outputscale) -- once, in the first split.
    if (dcov && kb == 0) {
      for (int c = 0; c < q; ++c) {
        if (c == a) continue;
        double d2 = 0.0;
#pragma unroll
        for (int u = 0; u < ND; ++u) {
          const double df = xs[a][u] - xs[c][u];
          d2 = fma(df, df, d2);
        }
        s = fma(G[a][c] * dkernel_factor<KIND>(d2, outputscale), xs[a][t] - xs[c][t], s);
      }
    }
    if (part) {  // one split's unscaled sum (post_backward_reduce_kernel finishes it)
      part[((int64_t)b * q + a) * d + t] = s;
    } else {
      double* o = dX + ((int64_t)b * q + a) * d + t;
      *o = accumulate ? *o + s / ls[t] : s / ls[t];
    }
  }
}

// grid (B, NS): with NS > 1 workgroup (b, s) takes the training points
// [s chunk, (s + 1) chunk) of t-batch b and writes its unscaled sums to
// part + s B q d; post_backward_reduce_kernel adds the NS splits in order.  A
// few t-batches (the tail of a compacted optimiser run: B = 2) otherwise left
// B workgroups walking all n points on a 256-CU chip (120 us at n = 4096).
template <int KIND, int ND>
__global__ __launch_bounds__(THREADS) void post_backward_kernel(
    int q, int Qp, const double* __restrict__ Xq, const double* __restrict__ Xt, int n,
    const double* __restrict__ W, int64_t ldw, const double* __restrict__ alpha,
    const double* __restrict__ dmean, const double* __restrict__ dcov,
    const double* __restrict__ E, int64_t lde,
    const double* __restrict__ ls, double outputscale, double ystd, int d, int accumulate,
    double* __restrict__ dX, int wkm, int chunk, double* __restrict__ part) {
  const int kb = blockIdx.y * chunk;
  const int ke = min(n, kb + chunk);
  post_backward_body<KIND, ND>(blockIdx.x, q, Qp, Xq, Xt, n, W, ldw, alpha, dmean, dcov, E, lde, ls,
                               outputscale, ystd, d, accumulate, dX, wkm, kb, ke,
                               part ? part + (int64_t)blockIdx.y * gridDim.x * q * d : nullptr);
}

// dX (+)= (sum over the NS splits, in split order) / lengthscale
__global__ __launch_bounds__(256) void post_backward_reduce_kernel(int ns, int64_t total, int d,
                                                                    const double* __restrict__ part,
                                                                    const double* __restrict__ ls,
                                                                    int accumulate, double* __restrict__ dX) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= total) return;
  double s = part[e];
  for (int j = 1; j < ns; ++j) s += part[(int64_t)j * total + e];
  const double v = s / ls[e % d];
  dX[e] = accumulate ? dX[e] + v : v;
}

// Several posterior backward passes of one (B, q, d, kind) in ONE launch
// (bo_post_backward_jobs: a ModelListGP's members, each with its training and
// baseline passes): grid (B, jobs), job j's dX written to its own slice (no
// accumulation across workgroups; the caller sums the slices).  One pass
// alone is B = 128 workgroups on 256 CUs.
constexpr int PB_MAXJ = 16;
struct PBJob {
  const double *Xq, *Xt, *W, *alpha, *dmean, *dcov, *E, *ls;
  double* dX;
  int64_t ldw, lde;
  double outputscale, ystd;
  int n, wkm;
};
struct PBJobs {
  PBJob j[PB_MAXJ];
};

template <int KIND, int ND>
__global__ __launch_bounds__(THREADS) void post_backward_jobs_kernel(int q, int Qp, int d, PBJobs jb) {
  const PBJob& J = jb.j[blockIdx.y];
  post_backward_body<KIND, ND>(blockIdx.x, q, Qp, J.Xq, J.Xt, J.n, J.W, J.ldw, J.alpha, J.dmean,
                               J.dcov, J.E, J.lde, J.ls, J.outputscale, J.ystd, d, 0, J.dX, J.wkm);
}

// Generic-d kernel-matrix gradient: dX[i][t] (+)= sum_k dK[i][k] d k(x_i, y_k) / d x_it
// for inputs in the ORIGINAL scale (lengthscale ls per dim).  group > 0: row i
// only sees the points of its own group (rows i / group * group ..; dK row
// holds `group` entries) -- the K** term of a q-batch.  One workgroup per row.
template <int KIND>
__global__ __launch_bounds__(THREADS) void kernel_grad_kernel(
    const double* __restrict__ X, const double* __restrict__ Y, int n, int d,
    const double* __restrict__ ls, double outputscale, const double* __restrict__ dK,
    int64_t ldk, int group, int accumulate, double* __restrict__ dX) {
  constexpr int CH = 1024;
  __shared__ double xi[128];
  __shared__ double il2[128];
  __shared__ double fk[CH];
  __shared__ double part[THREADS];
  const int64_t i = blockIdx.x;
  const int tid = threadIdx.x;
  const double* Yb = group > 0 ? Y + (i / group) * group * (int64_t)d : Y;
  const int npts = group > 0 ? group : n;
  for (int t = tid; t < d; t += THREADS) {
    xi[t] = X[i * d + t];
    il2[t] = 1.0 / (ls[t] * ls[t]);
  }
  __syncthreads();
  // thread layout for the second phase: TT threads per dimension slice
  double acc_t = 0.0;
  const int t_own = tid % 128;  // dimension handled (d <= 128)
  const int kslice = tid / 128;  // 2 slices of points
  for (int k0 = 0; k0 < npts; k0 += CH) {
    const int nk = min(CH, npts - k0);
    for (int kk = tid; kk < nk; kk += THREADS) {
      const double* y = Yb + (int64_t)(k0 + kk) * d;
      double d2 = 0.0;
      for (int t = 0; t < d; ++t) {
        const double df = xi[t] - y[t];
        d2 = fma(df * df, il2[t], d2);
      }
      const double D = dK[i * ldk + k0 + kk];
      fk[kk] = (group > 0 && (k0 + kk) == (int)(i % group)) ? 0.0
                                                            : D * dkernel_factor<KIND>(d2, outputscale);
    }
    __syncthreads();
    if (t_own < d) {
      for (int kk = kslice; kk < nk; kk += THREADS / 128) {
        const double* y = Yb + (int64_t)(k0 + kk) * d;
        acc_t = fma(fk[kk], xi[t_own] - y[t_own], acc_t);
      }
    }
    __syncthreads();
  }
  part[tid] = acc_t;
  __syncthreads();
  if (tid < d) {
    const double v = (part[tid] + part[tid + 128]) * il2[tid];
    dX[i * d + tid] = accumulate ? dX[i * d + tid] + v : v;
  }
}

}  // namespace

extern "C" int bo_kernel_grad(int kind, const double* X, int64_t rows, const double* Y, int64_t n,
                              int d, const double* lengthscale, double outputscale,
                              const double* dK, int64_t ldk, int group, int accumulate,
                              double* dX, void* stream) {
  BO_CHECK_ARG(kind == BO_RBF || kind == BO_MATERN52, "bo_kernel_grad: bad kind %d", kind);
  BO_CHECK_ARG(d >= 1 && d <= 128, "bo_kernel_grad: 1 <= d <= 128 (got %d)", d);
  BO_CHECK_ARG(group == 0 || rows % group == 0, "bo_kernel_grad: rows not a multiple of group");
  if (rows == 0) return BO_OK;
  hipStream_t st = as_stream(stream);
  if (kind == BO_RBF)
    kernel_grad_kernel<BO_RBF><<<(unsigned)rows, THREADS, 0, st>>>(X, Y, (int)n, d, lengthscale, outputscale, dK, ldk, group, accumulate, dX);
  else
    kernel_grad_kernel<BO_MATERN52><<<(unsigned)rows, THREADS, 0, st>>>(X, Y, (int)n, d, lengthscale, outputscale, dK, ldk, group, accumulate, dX);
  BO_LAUNCH_CHECK();
  return BO_OK;
}

extern "C" int bo_qmc_backward(int mode, int B, int q, const double* mean, const double* Lq,
                               const double* Z, int S, double best_f, const double* best_f_s,
                               const double* F, int64_t ldF, const double* dacq, double* dmean,
                               double* dcov, double* dF, const double* acq_fwd, int fat,
                               double tau_relu, double tau_max, void* stream) {
  BO_CHECK_ARG(q >= 1 && q <= QMAX, "bo_qmc_backward: q=%d out of range", q);
  BO_CHECK_ARG(mode == MODE_QEI || mode == MODE_QNEI || mode == MODE_QLOGEI || mode == MODE_QLOGNEI,
               "bo_qmc_backward: bad mode %d", mode);
  const bool per_sample = mode == MODE_QNEI || mode == MODE_QLOGNEI;
  const bool logm = mode == MODE_QLOGEI || mode == MODE_QLOGNEI;
  BO_CHECK_ARG(!per_sample || (best_f_s && F && dF),
               "bo_qmc_backward: qNEI / qLogNEI need best_f_s, F, dF");
  BO_CHECK_ARG(!logm || (acq_fwd && tau_relu > 0.0 && tau_max > 0.0),
               "bo_qmc_backward: log modes need the forward values and positive temperatures");
  if (B == 0) return BO_OK;
  int Qp = 1;
  while (Qp < q) Qp *= 2;
  BO_CHECK_ARG(!per_sample || ldF >= (int64_t)B * Qp, "bo_qmc_backward: ldF too small");
  hipStream_t st = as_stream(stream);
  const LogRedParams lp{tau_relu, tau_max, fat};
  if (mode == MODE_QEI)
    qmc_backward_kernel<MODE_QEI><<<B, THREADS, 0, st>>>(q, mean, Lq, Z, S, best_f, best_f_s, dacq, dmean, dcov, nullptr, 0, Qp, nullptr);
  else if (mode == MODE_QNEI)
    qmc_backward_kernel<MODE_QNEI><<<B, THREADS, 0, st>>>(q, mean, Lq, Z, S, best_f, best_f_s, dacq, dmean, dcov, F, ldF, Qp, dF);
  else if (mode == MODE_QLOGEI)
    qmc_log_backward_kernel<false><<<B, THREADS, 0, st>>>(q, mean, Lq, Z, S, best_f, best_f_s, acq_fwd, lp, dacq, dmean, dcov, nullptr, 0, Qp, nullptr);
  else
    qmc_log_backward_kernel<true><<<B, THREADS, 0, st>>>(q, mean, Lq, Z, S, best_f, best_f_s, acq_fwd, lp, dacq, dmean, dcov, F, ldF, Qp, dF);
  BO_LAUNCH_CHECK();
  return BO_OK;
}

extern "C" int bo_chol_backward(int B, int q, const double* L, const double* dL, double* dA,
                                void* stream) {
  BO_CHECK_ARG(q >= 1 && q <= QBIG, "bo_chol_backward: q=%d out of range (1..64)", q);
  if (B == 0) return BO_OK;
  if (q <= QMAX)
    chol_backward_kernel<<<B, THREADS, 0, as_stream(stream)>>>(q, L, dL, dA);
  else
    chol_backward_big_kernel<<<B, THREADS, 0, as_stream(stream)>>>(q, L, dL, dA);
  BO_LAUNCH_CHECK();
  return BO_OK;
}

extern "C" int bo_post_backward(int kind, int B, int q, int d, const double* Xq,
                                const double* Xt_scaled, int64_t n, const double* W, int64_t ldw,
                                const double* alpha, const double* dmean, const double* dcov,
                                const double* E, int64_t lde, const double* lengthscale,
                                double outputscale, double ystd, int accumulate, double* dX,
                                int w_kmajor, void* stream) {
  BO_CHECK_ARG(q >= 1 && q <= QMAX && d >= 1 && d <= DP, "bo_post_backward: bad q/d");
  if (B == 0) return BO_OK;
  int Qp = 1;
  while (Qp < q) Qp *= 2;
  hipStream_t st = as_stream(stream);
  // splits of >= 128 training points (one trip of the body's loop) until B NS
  // reaches ~256 workgroups; NS = 1 (B >= 256, or n <= 128) is the one-pass
  // kernel as before, bit for bit
  const int nchunks = (int)std::max<int64_t>(1, ceil_div(n, 128));
  const int ns = (int)std::min<int64_t>(nchunks, std::max<int64_t>(1, ceil_div(256, B)));
  const int chunk = (int)(ceil_div(nchunks, ns) * 128);
  const int ns_used = std::max(1, (int)ceil_div(n, chunk));
  double* part = nullptr;
  if (ns_used > 1) {
    keep_pool_warm();
    BO_HIP(hipMallocAsync(reinterpret_cast<void**>(&part),
                          sizeof(double) * (size_t)ns_used * B * q * d, st));
  }
  const dim3 grid((unsigned)B, (unsigned)ns_used);
#define BO_PB(KIND, ND)                                                                        \
  post_backward_kernel<KIND, ND><<<grid, THREADS, 0, st>>>(q, Qp, Xq, Xt_scaled, (int)n, W, ldw, \
                                                           alpha, dmean, dcov, E, lde,           \
                                                           lengthscale, outputscale, ystd, d,    \
                                                           accumulate, dX, w_kmajor,             \
                                                           ns_used > 1 ? chunk : (int)n, part)
  if (kind == BO_RBF) {
    if (d == 6) BO_PB(BO_RBF, 6); else BO_PB(BO_RBF, 8);
  } else {
    if (d == 6) BO_PB(BO_MATERN52, 6); else BO_PB(BO_MATERN52, 8);
  }
#undef BO_PB
  BO_LAUNCH_CHECK();
  if (part) {
    const int64_t total = (int64_t)B * q * d;
    post_backward_reduce_kernel<<<(unsigned)ceil_div(total, 256), 256, 0, st>>>(
        ns_used, total, d, part, lengthscale, accumulate, dX);
    BO_LAUNCH_CHECK();
    BO_HIP(hipFreeAsync(part, st));
  }
  return BO_OK;
}

extern "C" int bo_post_backward_jobs(int njobs, const BoPostBackwardArgs* const* jobs, double* dX_parts,
                                     void* stream) {
  BO_CHECK_ARG(njobs >= 1 && njobs <= PB_MAXJ, "bo_post_backward_jobs: %d jobs (1..%d)", njobs, PB_MAXJ);
  BO_CHECK_ARG(jobs && dX_parts, "bo_post_backward_jobs: null pointer");
  const BoPostBackwardArgs* a0 = jobs[0];
  BO_CHECK_ARG(a0 && a0->q >= 1 && a0->q <= QMAX && a0->d >= 1 && a0->d <= DP, "bo_post_backward_jobs: bad q/d");
  const int B = a0->B, q = a0->q, d = a0->d, kind = a0->kind;
  PBJobs jb{};
  for (int j = 0; j < njobs; ++j) {
    const BoPostBackwardArgs* a = jobs[j];
    BO_CHECK_ARG(a && a->B == B && a->q == q && a->d == d && a->kind == kind,
                 "bo_post_backward_jobs: job %d differs in B/q/d/kind", j);
    BO_CHECK_ARG(a->Xq && a->Xt_scaled && a->lengthscale && a->n >= 0,
                 "bo_post_backward_jobs: job %d lacks inputs", j);
    jb.j[j] = PBJob{a->Xq, a->Xt_scaled, a->W, a->alpha, a->dmean, a->dcov, a->E, a->lengthscale,
                    dX_parts + (int64_t)j * B * q * d, a->ldw, a->lde, a->outputscale, a->ystd,
                    (int)a->n, a->w_kmajor};
  }
  if (B == 0) return BO_OK;
  int Qp = 1;
  while (Qp < q) Qp *= 2;
  hipStream_t st = as_stream(stream);
  const dim3 grid((unsigned)B, (unsigned)njobs);
#define BO_PBJ(KIND, ND) post_backward_jobs_kernel<KIND, ND><<<grid, THREADS, 0, st>>>(q, Qp, d, jb)
  if (kind == BO_RBF) {
    if (d == 6) BO_PBJ(BO_RBF, 6); else BO_PBJ(BO_RBF, 8);
  } else {
    if (d == 6) BO_PBJ(BO_MATERN52, 6); else BO_PBJ(BO_MATERN52, 8);
  }
#undef BO_PBJ
  BO_LAUNCH_CHECK();
  return BO_OK;
}
