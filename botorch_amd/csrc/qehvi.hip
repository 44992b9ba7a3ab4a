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
// reduce with wavefront shuffles.  C4 has only 128 t-batches for 256 CUs and
// every (sample, cell) step waits on L1 / LDS loads and a data-dependent
// subset loop, so the workgroups are wide: 16 waves (forward) / 8 waves
// (backward, 220 VGPRs) per t-batch hide that latency (at 4 waves the forward
// kernel issued one VALU instruction per ~25 cycles per wave, PMC r03).
#include "common.h"

#include <cstdlib>

#include <algorithm>

namespace {

constexpr int THREADS = 256;   // mc_reduce_kernel
constexpr int FWD_THREADS = 1024;
constexpr int BWD_THREADS = 512;
constexpr int QMAX = 12;
constexpr int MMAX = 4;
constexpr int LDS_SAMPLES_DOUBLES = 6144;  // 48 KiB of samples per pass
constexpr int GROUP = 16;                  // lanes per sample in the backward

// Optional extensions used by qNEHVI (cached baseline root, per-sample box
// decompositions): cstride > 0 gives every sample its own K cells
// (lo/hi + s * cstride); F (m x S x ldF, output stride sF) adds the baseline
// term Z_base T of the cached-root samples at row b * Qp + p.
struct QehviExt {
  int64_t cstride;
  const double* F;
  int64_t ldF, sF;
  int Qp;
};

template <int M>
__device__ __forceinline__ double sample_value(int B, int b, int q, int p, int t, int s,
                                               const double* __restrict__ mean,
                                               const double* __restrict__ L,
                                               const double* __restrict__ Z, const QehviExt& ex) {
  const double* Lt = L + (((int64_t)t * B + b) * q + p) * q;
  const double* zs = Z + (int64_t)s * q * M;
  double v = mean[((int64_t)t * B + b) * q + p];
  if (ex.F) v += ex.F[t * ex.sF + (int64_t)s * ex.ldF + (int64_t)b * ex.Qp + p];
  for (int j = 0; j <= p; ++j) v = fma(Lt[j], zs[j * M + t], v);
  return v;
}

// CELLS_LDS: the K hypercells (shared by all samples: cell_stride 0) staged in
// LDS once, so the (sample, cell) loop reads only LDS
constexpr int LDS_CELL_DOUBLES = 2048;  // K * M <= 1024 (C4: 294 x 3)

// QB: the q bucket (4, 8 or QMAX) the per-point arrays are sized for -- the
// backward's a / gacc arrays at QMAX spilled to scratch (300-400 B per lane).
template <int M, int NT = FWD_THREADS, bool CELLS_LDS = false, int QB = QMAX>
__global__ __launch_bounds__(NT) void qehvi_kernel(
    int B, int q, const double* __restrict__ mean, const double* __restrict__ L,
    const double* __restrict__ Z, int S, const double* __restrict__ lo,
    const double* __restrict__ hi, int K, QehviExt ex, double* __restrict__ acq, int H = 1,
    double* __restrict__ part = nullptr) {
  // H > 1: the t-batch's samples are split over H workgroups (C4's 128
  // t-batches would leave half the CUs idle); workgroup h sums the samples
  // [h S / H, (h + 1) S / H) into part[b H + h], qehvi_part_reduce_kernel
  // adds the H partials in order
  __shared__ double f[LDS_SAMPLES_DOUBLES];
  __shared__ double red[NT / 64];
  __shared__ double cells[CELLS_LDS ? LDS_CELL_DOUBLES : 1];
  const int b = blockIdx.x / H;
  const int h = blockIdx.x - b * H;
  const int sbeg = (int)((int64_t)S * h / H), send = (int)((int64_t)S * (h + 1) / H);
  const int tid = threadIdx.x;
  const int per_sample = q * M;
  // a chunk's samples, then their per-objective maxima over the points
  const int chunk = LDS_SAMPLES_DOUBLES / (per_sample + M);
  double* const fmx = f + chunk * per_sample;
  if constexpr (CELLS_LDS) {
    for (int e = tid; e < K * M; e += NT) {
      cells[e] = lo[e];
      cells[LDS_CELL_DOUBLES / 2 + e] = hi[e];
    }
  }
  double sum = 0.0;
  for (int s0 = sbeg; s0 < send; s0 += chunk) {
    const int ns = min(chunk, send - s0);
    __syncthreads();
    for (int e = tid; e < ns * per_sample; e += NT) {
      const int s = e / per_sample;
      f[e] = sample_value<M>(B, b, q, (e / M) % q, e % M, s0 + s, mean, L, Z, ex);
    }
    __syncthreads();
    for (int e = tid; e < ns * M; e += NT) {
      const double* fs = f + (e / M) * per_sample + e % M;
      double mx = fs[0];
      for (int p = 1; p < q; ++p) mx = fmax(mx, fs[p * M]);
      fmx[e] = mx;
    }
    __syncthreads();
    for (int e = tid; e < ns * K; e += NT) {
      const int s = e / K;
      const int k = e % K;
      double l[M], u[M];
      const int64_t co = (int64_t)(s0 + s) * ex.cstride + (int64_t)k * M;
      // a point is active in the cell only if it exceeds the lower corner in
      // every objective, so no point is unless each objective's maximum over
      // the points does: such pairs contribute exactly zero (skipped; at C4
      // over 90% of the (sample, cell) pairs have no active point)
      bool any = true;
#pragma unroll
      for (int t = 0; t < M; ++t) {
        l[t] = CELLS_LDS ? cells[k * M + t] : lo[co + t];
        any = any && (fmx[s * M + t] > l[t]);
      }
      if (!any) continue;
#pragma unroll
      for (int t = 0; t < M; ++t) u[t] = CELLS_LDS ? cells[LDS_CELL_DOUBLES / 2 + k * M + t] : hi[co + t];
      const double* fs = f + s * per_sample;
      double a[QB][M];
      unsigned act = 0;
#pragma unroll
      for (int p = 0; p < QB; ++p) {
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
        for (int p = 0; p < QB; ++p)
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
    for (int w = 0; w < NT / 64; ++w) t += red[w];
    if (H == 1) acq[b] = t / S;
    else part[blockIdx.x] = t;
  }
}

__global__ __launch_bounds__(64) void qehvi_part_reduce_kernel(const double* __restrict__ part, int B,
                                                               int H, int S, double* __restrict__ acq) {
  const int b = blockIdx.x * 64 + threadIdx.x;
  if (b >= B) return;
  double t = 0.0;
  for (int h = 0; h < H; ++h) t += part[(int64_t)b * H + h];
  acq[b] = t / S;
}

// Backward of qehvi_kernel (gen_candidates_scipy's autograd.grad through
// _compute_qehvi, monte_carlo.py:230-317): for every (sample, cell, subset T)
// term sign * prod_t mn_t, the derivative w.r.t. f[s][p*][t] is
// sign * prod_{t' != t} mn_t' where p* = argmin_{p in T} f_pt and the min is
// not the cell's upper bound (min(u, .) passes no gradient to f there; a
// clamped-at-lower term is zero with zero gradient).  df[s] is summed by one
// 16-lane group over the cells in a fixed order (no atomics), then dmean_t[p] = sum_s df[s][p][t] and
// dL_t[p][j] = sum_s df[s][p][t] Z[s][j m + t] (j <= p), scaled by dacq / S.
// CELLS_LDS (shared cells, K m <= LDS_CELL_DOUBLES / 2): the cells staged in
// LDS once; the chunk's base samples are staged in LDS always (read by the
// sample values and again by the dmean / dL sums).
template <int M, int NT = BWD_THREADS, int QB = QMAX, bool CELLS_LDS = false>
__global__ __launch_bounds__(NT) void qehvi_backward_kernel(
    int B, int q, const double* __restrict__ mean, const double* __restrict__ L,
    const double* __restrict__ Z, int S, const double* __restrict__ lo,
    const double* __restrict__ hi, int K, QehviExt ex, const double* __restrict__ dacq,
    double* __restrict__ dmean, double* __restrict__ dL, double* __restrict__ dF, int H = 1,
    double* __restrict__ part = nullptr) {
  // H > 1: samples split over H workgroups as in qehvi_kernel; workgroup h
  // writes its (dmean, dL) entries to part[(b H + h) nent + .] (dF rows are
  // per sample: written directly), qehvi_backward_reduce_kernel sums them
  constexpr int CH = LDS_SAMPLES_DOUBLES / 2;
  __shared__ double f[CH];
  __shared__ double df[CH];
  __shared__ double zc[CH];  // the chunk's base samples, Z[s0 + s][.]
  __shared__ double cells[CELLS_LDS ? LDS_CELL_DOUBLES : 1];
  const int b = blockIdx.x / H;
  const int h = blockIdx.x - b * H;
  const int sbeg = (int)((int64_t)S * h / H), send = (int)((int64_t)S * (h + 1) / H);
  const int tid = threadIdx.x;
  const int per_sample = q * M;
  // a chunk's samples (then their per-objective maxima over the points in f)
  const int chunk = CH / (per_sample + M);
  double* const fmx = f + chunk * per_sample;
  const double g = dacq[b] / (double)S;
  // entries owned by this thread: (t, p, j) with j <= p (j == p + 1 -> dmean)
  const int nent = M * q * (q + 3) / 2;
  double accv[2] = {0.0, 0.0};
  if constexpr (CELLS_LDS) {
    for (int e = tid; e < K * M; e += NT) {
      cells[e] = lo[e];
      cells[LDS_CELL_DOUBLES / 2 + e] = hi[e];
    }
  }
  for (int s0 = sbeg; s0 < send; s0 += chunk) {
    const int ns = min(chunk, send - s0);
    __syncthreads();
    for (int e = tid; e < ns * per_sample; e += NT) zc[e] = Z[(int64_t)s0 * per_sample + e];
    __syncthreads();
    for (int e = tid; e < ns * per_sample; e += NT) {
      // sample_value with the base samples from LDS (the same sum, in order)
      const int s = e / per_sample, p = (e / M) % q, t = e % M;
      const double* Lt = L + (((int64_t)t * B + b) * q + p) * q;
      const double* zs = zc + s * per_sample;
      double v = mean[((int64_t)t * B + b) * q + p];
      if (ex.F) v += ex.F[t * ex.sF + (int64_t)(s0 + s) * ex.ldF + (int64_t)b * ex.Qp + p];
      for (int j = 0; j <= p; ++j) v = fma(Lt[j], zs[j * M + t], v);
      f[e] = v;
    }
    __syncthreads();
    for (int e = tid; e < ns * M; e += NT) {
      const double* fs = f + (e / M) * per_sample + e % M;
      double mx = fs[0];
      for (int p = 1; p < q; ++p) mx = fmax(mx, fs[p * M]);
      fmx[e] = mx;
    }
    __syncthreads();
    // GROUP consecutive lanes share one sample: lane g of the group takes the
    // cells k = g, g + GROUP, ...; the group's partial gradients reduce in a
    // fixed butterfly, so df (and every gradient) is bitwise reproducible
    for (int s = tid / GROUP; s < ns; s += NT / GROUP) {
      const double* fs = f + s * per_sample;
      double gacc[QB][M];
#pragma unroll
      for (int p = 0; p < QB; ++p)
#pragma unroll
        for (int t = 0; t < M; ++t) gacc[p][t] = 0.0;
      for (int k = tid % GROUP; k < K; k += GROUP) {
        double l[M], u[M];
        const int64_t co = (int64_t)(s0 + s) * ex.cstride + (int64_t)k * M;
        bool any = true;  // as the forward: no active point -> no gradient
#pragma unroll
        for (int t = 0; t < M; ++t) {
          l[t] = CELLS_LDS ? cells[k * M + t] : lo[co + t];
          any = any && (fmx[s * M + t] > l[t]);
        }
        if (!any) continue;
#pragma unroll
        for (int t = 0; t < M; ++t) u[t] = CELLS_LDS ? cells[LDS_CELL_DOUBLES / 2 + k * M + t] : hi[co + t];
        double a[QB][M];
        unsigned act = 0;
#pragma unroll
        for (int p = 0; p < QB; ++p) {
          bool ok = p < q;
#pragma unroll
          for (int t = 0; t < M; ++t) {
            const double v = p < q ? fmin(u[t], fs[p * M + t]) - l[t] : 0.0;
            a[p][t] = v;
            ok = ok && (v > 0.0);
          }
          if (ok) act |= 1u << p;
        }
        for (unsigned sub = act; sub; sub = (sub - 1) & act) {
          double mn[M];
          int am[M];
#pragma unroll
          for (int t = 0; t < M; ++t) {
            mn[t] = INFINITY;
            am[t] = 0;
          }
#pragma unroll
          for (int p = 0; p < QB; ++p)
            if (sub & (1u << p))
#pragma unroll
              for (int t = 0; t < M; ++t)
                if (a[p][t] < mn[t]) {
                  mn[t] = a[p][t];
                  am[t] = p;
                }
          const double sg = (__popc(sub) & 1) ? 1.0 : -1.0;
#pragma unroll
          for (int t = 0; t < M; ++t) {
            double o = sg;
#pragma unroll
            for (int t2 = 0; t2 < M; ++t2)
              if (t2 != t) o *= mn[t2];
            // the min reaches f only where f < u (else the upper bound is active)
#pragma unroll
            for (int p = 0; p < QB; ++p)
              if (p == am[t] && fs[p * M + t] < u[t]) gacc[p][t] += o;
          }
        }
      }
#pragma unroll
      for (int p = 0; p < QB; ++p) {
        if (p >= q) break;
#pragma unroll
        for (int t = 0; t < M; ++t) {
          double v = gacc[p][t];
#pragma unroll
          for (int o = GROUP / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, GROUP);
          if (tid % GROUP == 0) df[s * per_sample + p * M + t] = v;
        }
      }
    }
    __syncthreads();
    if (dF) {  // cotangent of the cached-root baseline term (rows b * Qp + p)
      for (int e = tid; e < ns * per_sample; e += NT) {
        const int s = e / per_sample, p = (e / M) % q, t = e % M;
        dF[t * ex.sF + (int64_t)(s0 + s) * ex.ldF + (int64_t)b * ex.Qp + p] = g * df[e];
      }
    }
    for (int w = 0; w < 2; ++w) {
      const int ent = tid + w * NT;
      if (ent >= nent) continue;
      const int per_t = q * (q + 3) / 2;
      const int t = ent / per_t;
      int r = ent % per_t;
      int p = 0;
      while (r >= p + 2) {
        r -= p + 2;
        ++p;
      }
      const int j = r;  // 0..p -> dL[p][j]; p + 1 -> dmean[p]
      double acc = 0.0;
      for (int s = 0; s < ns; ++s) {
        const double d = df[s * per_sample + p * M + t];
        acc = fma(d, (j <= p) ? zc[s * per_sample + j * M + t] : 1.0, acc);
      }
      accv[w] += acc;
    }
  }
  if (H > 1) {
    for (int w = 0; w < 2; ++w) {
      const int ent = tid + w * NT;
      if (ent < nent) part[(int64_t)blockIdx.x * nent + ent] = g * accv[w];
    }
    return;
  }
  for (int w = 0; w < 2; ++w) {
    const int ent = tid + w * NT;
    if (ent >= nent) continue;
    const int per_t = q * (q + 3) / 2;
    const int t = ent / per_t;
    int r = ent % per_t;
    int p = 0;
    while (r >= p + 2) {
      r -= p + 2;
      ++p;
    }
    const int j = r;
    const double v = g * accv[w];
    if (j <= p) {
      double* dLt = dL + (((int64_t)t * B + b) * q + p) * q;
      dLt[j] = v;
    } else {
      dmean[((int64_t)t * B + b) * q + p] = v;
    }
  }
  // strict upper triangle of dL
  for (int e = tid; e < M * q * q; e += NT) {
    const int t = e / (q * q), p = (e / q) % q, j = e % q;
    if (j > p) dL[(((int64_t)t * B + b) * q + p) * q + j] = 0.0;
  }
}

// Sum of the H sample-split partials of qehvi_backward_kernel (in order), then
// its output layout: dL lower triangle + dmean, strict upper triangle zero.
__global__ __launch_bounds__(256) void qehvi_backward_reduce_kernel(const double* __restrict__ part,
                                                                    int B, int q, int M, int H,
                                                                    double* __restrict__ dmean,
                                                                    double* __restrict__ dL) {
  const int b = blockIdx.x;
  const int nent = M * q * (q + 3) / 2;
  const int per_t = q * (q + 3) / 2;
  for (int ent = threadIdx.x; ent < nent; ent += 256) {
    double v = 0.0;
    for (int h = 0; h < H; ++h) v += part[((int64_t)b * H + h) * nent + ent];
    const int t = ent / per_t;
    int r = ent % per_t;
    int p = 0;
    while (r >= p + 2) {
      r -= p + 2;
      ++p;
    }
    if (r <= p) dL[(((int64_t)t * B + b) * q + p) * q + r] = v;
    else dmean[((int64_t)t * B + b) * q + p] = v;
  }
  for (int e = threadIdx.x; e < M * q * q; e += 256) {
    const int t = e / (q * q), p = (e / q) % q, j = e % q;
    if (j > p) dL[(((int64_t)t * B + b) * q + p) * q + j] = 0.0;
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

extern "C" int bo_qehvi_ext(int B, int q, int m, const double* mean, const double* L,
                            const double* Z, int S, const double* cell_lo, const double* cell_hi,
                            int K, int64_t cell_stride, const double* F, int64_t ldF, int64_t sF,
                            int Qp, double* acq, double* work, int64_t work_elems, void* stream);

extern "C" int bo_qehvi(int B, int q, int m, const double* mean, const double* L, const double* Z,
                        int S, const double* cell_lo, const double* cell_hi, int K,
                        int64_t cell_stride, const double* F, int64_t ldF, int64_t sF, int Qp,
                        double* acq, void* stream) {
  return bo_qehvi_ext(B, q, m, mean, L, Z, S, cell_lo, cell_hi, K, cell_stride, F, ldF, sF, Qp, acq,
                      nullptr, 0, stream);
}

// work (>= 2 B doubles, optional): the samples of each t-batch split over H =
// min(8, 1024 / B, work_elems / B) workgroups when B leaves CUs idle.
extern "C" int bo_qehvi_ext(int B, int q, int m, const double* mean, const double* L,
                            const double* Z, int S, const double* cell_lo, const double* cell_hi,
                            int K, int64_t cell_stride, const double* F, int64_t ldF, int64_t sF,
                            int Qp, double* acq, double* work, int64_t work_elems, void* stream) {
  BO_CHECK_ARG(q >= 1 && q <= QMAX, "bo_qehvi: 1 <= q <= %d (got %d)", QMAX, q);
  BO_CHECK_ARG(m >= 2 && m <= MMAX, "bo_qehvi: 2 <= m <= %d (got %d)", MMAX, m);
  BO_CHECK_ARG(S > 0 && K >= 0 && cell_stride >= 0, "bo_qehvi: bad S/K/cell_stride");
  BO_CHECK_ARG(F == nullptr || (Qp >= q && ldF >= (int64_t)B * Qp), "bo_qehvi: bad F layout");
  if (B == 0) return BO_OK;
  hipStream_t st = as_stream(stream);
  const QehviExt ex{cell_stride, F, ldF, sF, Qp};
  const bool cl = cell_stride == 0 && (int64_t)K * m <= LDS_CELL_DOUBLES / 2;
  int H = 1;
  // Sample split toward ~1024 workgroups (4 per CU): C4 (B = 128, H = 8) step
  // 0.395 -> 0.380-0.383 ms against a 256-workgroup target (one per CU; 512:
  // 0.386-0.391; tools/ab_qehvi_wg.sh) -- more resident waves hide the
  // inclusion-exclusion's latency.  BO_QEHVI_WG overrides (A/B knob).
  static const int target = [] {
    const char* e = std::getenv("BO_QEHVI_WG");
    const int v = e ? std::atoi(e) : 1024;
    return v >= 1 && v <= 4096 ? v : 1024;
  }();
  if (work != nullptr && work_elems >= 2 * (int64_t)B) {
    H = (int)std::min<int64_t>(std::min(8, std::max(1, target / B)), work_elems / B);
    H = std::max(1, std::min(H, S));
  }
  const unsigned grid = (unsigned)((int64_t)B * H);
#define BO_QF(MM, QQ)                                                                          \
  if (cl)                                                                                      \
    qehvi_kernel<MM, FWD_THREADS, true, QQ><<<grid, FWD_THREADS, 0, st>>>(                     \
        B, q, mean, L, Z, S, cell_lo, cell_hi, K, ex, acq, H, work);                           \
  else                                                                                         \
    qehvi_kernel<MM, FWD_THREADS, false, QQ><<<grid, FWD_THREADS, 0, st>>>(                    \
        B, q, mean, L, Z, S, cell_lo, cell_hi, K, ex, acq, H, work)
#define BO_QFM(MM)          \
  if (q <= 4) {             \
    BO_QF(MM, 4);           \
  } else if (q <= 8) {      \
    BO_QF(MM, 8);           \
  } else {                  \
    BO_QF(MM, QMAX);        \
  }
  if (m == 2) {
    BO_QFM(2);
  } else if (m == 3) {
    BO_QFM(3);
  } else {
    BO_QFM(4);
  }
#undef BO_QFM
#undef BO_QF
  BO_LAUNCH_CHECK();
  if (H > 1) {
    qehvi_part_reduce_kernel<<<(unsigned)ceil_div(B, 64), 64, 0, st>>>(work, B, H, S, acq);
    BO_LAUNCH_CHECK();
  }
  return BO_OK;
}

extern "C" int bo_qehvi_backward_ext(int B, int q, int m, const double* mean, const double* L,
                                     const double* Z, int S, const double* cell_lo,
                                     const double* cell_hi, int K, int64_t cell_stride,
                                     const double* F, int64_t ldF, int64_t sF, int Qp,
                                     const double* dacq, double* dmean, double* dL, double* dF,
                                     double* work, int64_t work_elems, void* stream);

extern "C" int bo_qehvi_backward(int B, int q, int m, const double* mean, const double* L,
                                 const double* Z, int S, const double* cell_lo,
                                 const double* cell_hi, int K, int64_t cell_stride,
                                 const double* F, int64_t ldF, int64_t sF, int Qp,
                                 const double* dacq, double* dmean, double* dL, double* dF,
                                 void* stream) {
  return bo_qehvi_backward_ext(B, q, m, mean, L, Z, S, cell_lo, cell_hi, K, cell_stride, F, ldF, sF,
                               Qp, dacq, dmean, dL, dF, nullptr, 0, stream);
}

// work (>= 2 B nent doubles, nent = m q (q + 3) / 2, optional): the sample
// split of bo_qehvi_ext for the backward.
extern "C" int bo_qehvi_backward_ext(int B, int q, int m, const double* mean, const double* L,
                                 const double* Z, int S, const double* cell_lo,
                                 const double* cell_hi, int K, int64_t cell_stride,
                                 const double* F, int64_t ldF, int64_t sF, int Qp,
                                 const double* dacq, double* dmean, double* dL, double* dF,
                                 double* work, int64_t work_elems, void* stream) {
  BO_CHECK_ARG(q >= 1 && q <= QMAX, "bo_qehvi_backward: 1 <= q <= %d (got %d)", QMAX, q);
  BO_CHECK_ARG(m >= 2 && m <= MMAX, "bo_qehvi_backward: 2 <= m <= %d (got %d)", MMAX, m);
  BO_CHECK_ARG(S > 0 && K >= 0 && cell_stride >= 0, "bo_qehvi_backward: bad S/K/cell_stride");
  BO_CHECK_ARG((F == nullptr) == (dF == nullptr), "bo_qehvi_backward: F and dF go together");
  BO_CHECK_ARG(F == nullptr || (Qp >= q && ldF >= (int64_t)B * Qp), "bo_qehvi_backward: bad F layout");
  if (B == 0) return BO_OK;
  hipStream_t st = as_stream(stream);
  const QehviExt ex{cell_stride, F, ldF, sF, Qp};
  const int64_t nent = (int64_t)m * q * (q + 3) / 2;
  int H = 1;
  // BO_QEHVI_BWD_WG: target workgroups of the backward's sample split (A/B knob)
  static const int target = [] {
    const char* e = std::getenv("BO_QEHVI_BWD_WG");
    const int v = e ? std::atoi(e) : 256;
    return v >= 1 && v <= 4096 ? v : 256;
  }();
  if (work != nullptr && work_elems >= 2 * (int64_t)B * nent) {
    H = (int)std::min<int64_t>(std::min(8, std::max(1, target / B)), work_elems / ((int64_t)B * nent));
    H = std::max(1, std::min(H, S));
  }
  const unsigned grid = (unsigned)((int64_t)B * H);
  const bool cl = cell_stride == 0 && (int64_t)K * m <= LDS_CELL_DOUBLES / 2;
#define BO_QB(MM, NT, QQ)                                                                      \
  if (cl)                                                                                      \
    qehvi_backward_kernel<MM, NT, QQ, true><<<grid, NT, 0, st>>>(                              \
        B, q, mean, L, Z, S, cell_lo, cell_hi, K, ex, dacq, dmean, dL, dF, H, work);           \
  else                                                                                         \
    qehvi_backward_kernel<MM, NT, QQ, false><<<grid, NT, 0, st>>>(                             \
        B, q, mean, L, Z, S, cell_lo, cell_hi, K, ex, dacq, dmean, dL, dF, H, work)
#define BO_QBM(MM, NT)        \
  if (q <= 4) {               \
    BO_QB(MM, NT, 4);         \
  } else if (q <= 8) {        \
    BO_QB(MM, NT, 8);         \
  } else {                    \
    BO_QB(MM, NT, QMAX);      \
  }
  if (m == 2) {
    BO_QBM(2, BWD_THREADS);
  } else if (m == 3) {
    BO_QBM(3, BWD_THREADS);
  } else {
    BO_QBM(4, 256);  // m = 4 needs 256 VGPRs: 4 waves per workgroup
  }
#undef BO_QBM
#undef BO_QB
  BO_LAUNCH_CHECK();
  if (H > 1) {
    qehvi_backward_reduce_kernel<<<(unsigned)B, 256, 0, st>>>(work, B, q, m, H, dmean, dL);
    BO_LAUNCH_CHECK();
  }
  return BO_OK;
}

extern "C" int bo_mc_reduce(int S, int B, int q, const double* samples, double best_f,
                            const double* best_f_s, double* acq, void* stream) {
  if (B == 0) return BO_OK;
  mc_reduce_kernel<<<B, THREADS, 0, as_stream(stream)>>>(S, B, q, samples, best_f, best_f_s, acq);
  BO_LAUNCH_CHECK();
  return BO_OK;
}
