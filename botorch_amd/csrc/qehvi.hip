// qEHVI: Monte-Carlo expected hypervolume improvement over hypercells.
//
// Reference: qExpectedHypervolumeImprovement._compute_qehvi
// (botorch/acquisition/multi_objective/monte_carlo.py:230-317):
//   HVI(f) = sum_k sum_{nonempty T subset of [q]} (-1)^{|T|+1}
//            prod_t max(min(u_kt, min_{p in T} f_pt) - l_kt, 0)
//   acq    = mean_s HVI(f_s)
// Per cell, the subsets containing a point with an empty box
// (min(u_kt, f_pt) <= l_kt in some objective t) contribute exactly zero, so
// the inclusion-exclusion runs only over the nonempty submasks of the
// cell's active-point mask (the same sum, term for term, minus the zeros).
//
// Samples (ModelListGP: independent outputs, posteriors/base_samples.py:16-45
// non-interleaved base samples):  f[s][p][t] = mu_t[p] + sum_j L_t[p][j] Z[s][j m + t]
//
// One workgroup per t-batch: its samples go to LDS, the hypercells are read
// through L1/L2, threads stride over (sample, cell) pairs, the per-thread sums
// reduce with wavefront shuffles.
#include "common.h"

namespace {

constexpr int THREADS = 256;
constexpr int QMAX = 12;
constexpr int MMAX = 4;
constexpr int LDS_SAMPLES_DOUBLES = 6144;  // 48 KiB of samples per pass

template <int M>
__global__ __launch_bounds__(THREADS) void qehvi_kernel(
    int B, int q, const double* __restrict__ mean, const double* __restrict__ L,
    const double* __restrict__ Z, int S, const double* __restrict__ lo,
    const double* __restrict__ hi, int K, double* __restrict__ acq) {
  __shared__ double f[LDS_SAMPLES_DOUBLES];
  __shared__ double red[THREADS / 64];
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int per_sample = q * M;
  const int chunk = LDS_SAMPLES_DOUBLES / per_sample;
  double sum = 0.0;
  for (int s0 = 0; s0 < S; s0 += chunk) {
    const int ns = min(chunk, S - s0);
    __syncthreads();
    for (int e = tid; e < ns * per_sample; e += THREADS) {
      const int s = e / per_sample;
      const int p = (e / M) % q;
      const int t = e % M;
      const double* Lt = L + (((int64_t)t * B + b) * q + p) * q;
      const double* zs = Z + (int64_t)(s0 + s) * q * M;
      double v = mean[((int64_t)t * B + b) * q + p];
      for (int j = 0; j <= p; ++j) v = fma(Lt[j], zs[j * M + t], v);
      f[e] = v;
    }
    __syncthreads();
    for (int e = tid; e < ns * K; e += THREADS) {
      const int s = e / K;
      const int k = e % K;
      double l[M], u[M];
#pragma unroll
      for (int t = 0; t < M; ++t) {
        l[t] = lo[k * M + t];
        u[t] = hi[k * M + t];
      }
      const double* fs = f + s * per_sample;
      double a[QMAX][M];
      unsigned act = 0;
#pragma unroll
      for (int p = 0; p < QMAX; ++p) {
        bool ok = p < q;
#pragma unroll
        for (int t = 0; t < M; ++t) {
          const double v = p < q ? fmin(u[t], fs[p * M + t]) - l[t] : 0.0;
          a[p][t] = v;
          ok = ok && (v > 0.0);
        }
        if (ok) act |= 1u << p;
      }
      double cell = 0.0;
      for (unsigned sub = act; sub; sub = (sub - 1) & act) {
        double mn[M];
#pragma unroll
        for (int t = 0; t < M; ++t) mn[t] = INFINITY;
#pragma unroll
        for (int p = 0; p < QMAX; ++p)
          if (sub & (1u << p))
#pragma unroll
            for (int t = 0; t < M; ++t) mn[t] = fmin(mn[t], a[p][t]);
        double vol = 1.0;
#pragma unroll
        for (int t = 0; t < M; ++t) vol *= mn[t];
        cell += (__popc(sub) & 1) ? vol : -vol;
      }
      sum += cell;
    }
  }
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
  if ((tid & 63) == 0) red[tid >> 6] = sum;
  __syncthreads();
  if (tid == 0) {
    double t = 0.0;
    for (int w = 0; w < THREADS / 64; ++w) t += red[w];
    acq[b] = t / S;
  }
}

// Generic MC qEI / qNEI reduction of given samples (S x B x q): the reduction
// kernel of the non-fused path (custom posteriors), same semantics as the
// fused one (acquisition/monte_carlo.py:405-414, 580-589).
__global__ __launch_bounds__(THREADS) void mc_reduce_kernel(
    int S, int B, int q, const double* __restrict__ samples, double best_f,
    const double* __restrict__ best_f_s, double* __restrict__ acq) {
  __shared__ double red[THREADS / 64];
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  double sum = 0.0;
  for (int s = tid; s < S; s += THREADS) {
    const double bf = best_f_s ? best_f_s[s] : best_f;
    const double* fs = samples + ((int64_t)s * B + b) * q;
    double m = 0.0;
    for (int a = 0; a < q; ++a) m = fmax(m, fs[a] - bf);
    sum += m;
  }
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
  if ((tid & 63) == 0) red[tid >> 6] = sum;
  __syncthreads();
  if (tid == 0) {
    double t = 0.0;
    for (int w = 0; w < THREADS / 64; ++w) t += red[w];
    acq[b] = t / S;
  }
}

}  // namespace

extern "C" int bo_qehvi(int B, int q, int m, const double* mean, const double* L, const double* Z,
                        int S, const double* cell_lo, const double* cell_hi, int K, double* acq,
                        void* stream) {
  BO_CHECK_ARG(q >= 1 && q <= QMAX, "bo_qehvi: 1 <= q <= %d (got %d)", QMAX, q);
  BO_CHECK_ARG(m >= 2 && m <= MMAX, "bo_qehvi: 2 <= m <= %d (got %d)", MMAX, m);
  BO_CHECK_ARG(S > 0 && K >= 0, "bo_qehvi: bad S/K");
  if (B == 0) return BO_OK;
  hipStream_t st = as_stream(stream);
  if (m == 2)
    qehvi_kernel<2><<<B, THREADS, 0, st>>>(B, q, mean, L, Z, S, cell_lo, cell_hi, K, acq);
  else if (m == 3)
    qehvi_kernel<3><<<B, THREADS, 0, st>>>(B, q, mean, L, Z, S, cell_lo, cell_hi, K, acq);
  else
    qehvi_kernel<4><<<B, THREADS, 0, st>>>(B, q, mean, L, Z, S, cell_lo, cell_hi, K, acq);
  BO_LAUNCH_CHECK();
  return BO_OK;
}

extern "C" int bo_mc_reduce(int S, int B, int q, const double* samples, double best_f,
                            const double* best_f_s, double* acq, void* stream) {
  if (B == 0) return BO_OK;
  mc_reduce_kernel<<<B, THREADS, 0, as_stream(stream)>>>(S, B, q, samples, best_f, best_f_s, acq);
  BO_LAUNCH_CHECK();
  return BO_OK;
}
