// Per-t-batch posterior finalisation + Monte-Carlo acquisition reduction.
//
// One workgroup per t-batch b (restart / raw sample):
//   1. Sigma*_b = K**_b - sum_ct Spart[ct],  mu*_b = c + sum_ct mpart[ct]
//      (the column-tile partials of post_partials_kernel, post.hip), then
//      Standardize.untransform_posterior: mu' = ybar + s mu*, Sigma' = s^2 Sigma*
//      (botorch/models/transforms/outcome.py:373-447).
//   2. L_q = psd_safe_cholesky(Sigma') with the [G] jitter ladder applied per
//      batch member: plain, then jitter0 * 10^i for i = 0..max_tries-1
//      (linear_operator psd_safe_cholesky; botorch/__init__.py:47 sets 6 tries).
//      A member that still fails reports info > 0; the host raises NotPSDError.
//   3. f[s,a] = mu'_a + sum_{j<=a} L_q[a][j] Z[s][j]   (posteriors/gpytorch.py:85-126)
//      and the acquisition reduction:
//        qEI  : mean_s max_a relu(f - best_f)           (acquisition/monte_carlo.py:405-414)
//        qNEI : mean_s max_a relu(f - best_f[s])        (:580-589, cached baseline best)
//        qLogEI / qLogNEI : logmeanexp_s fatmax_a log_fatplus(f - best_f(s))
//                           (acquisition/logei.py:122, 219-234, 347-362; logred.h)
//      q-max and the sample sum are wavefront shuffle reductions (an online
//      (max, sum-exp) pair for logmeanexp).
#include "common.h"

#include <cstring>
#include "logred.h"

namespace {

constexpr int QMAX = 16;

__device__ __forceinline__ double rsq_nr(double v) {
  double r = __builtin_amdgcn_rsq(v);
  r = r * fma(-0.5 * v * r, r, 1.5);
  r = r * fma(-0.5 * v * r, r, 1.5);
  return r;
}

__device__ __forceinline__ double readlane_d(double v, int l) {
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(x & 0xffffffffll), l);
  const int hi = __builtin_amdgcn_readlane((int)(x >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
constexpr int DP = 8;
constexpr int THREADS = 256;

// Phase clocks of the tools-only build (-DBO_QMC_PHASES, tools/qmc_phases.sh):
// workgroup b's 100 MHz wall clock at entry (0), the finalised covariance (1),
// the factor (2), the reduced value (3) and its exit (4); never in the product.
#ifdef BO_QMC_PHASES
constexpr int PH_N = 5, PH_WG = 1024;
__device__ unsigned long long g_qmc_phase[PH_WG * PH_N];
#define QMC_PHASE(k)                                                     \
  do {                                                                   \
    if (threadIdx.x == 0 && blockIdx.x < PH_WG)                          \
      g_qmc_phase[blockIdx.x * PH_N + (k)] = wall_clock64();             \
  } while (0)
#else
#define QMC_PHASE(k) \
  do {               \
  } while (0)
#endif

enum QmcMode : int {
  QMC_POSTERIOR = 0,
  QMC_QEI = 1,
  QMC_QNEI = 2,
  QMC_CHOL = 3,
  QMC_QLOGEI = 4,
  QMC_QLOGNEI = 5
};

__host__ __device__ constexpr bool per_sample_best(int mode) {
  return mode == QMC_QNEI || mode == QMC_QLOGNEI;
}
__host__ __device__ constexpr bool log_mode(int mode) {
  return mode == QMC_QLOGEI || mode == QMC_QLOGNEI;
}

// sum_{ct < n} p[ct * stride] with U independent partial sums, so U of the
// partials' loads are in flight together instead of one latency per partial
// (U = 16 for the quad plan's long partial lists: C2 has 136 block pairs).
template <int U = 8>
__device__ __forceinline__ double strided_sum(const double* __restrict__ p, int64_t stride, int n) {
  double s[U];
#pragma unroll
  for (int u = 0; u < U; ++u) s[u] = 0.0;
  int ct = 0;
  for (; ct + U <= n; ct += U) {
    double v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = p[(int64_t)(ct + u) * stride];
#pragma unroll
    for (int u = 0; u < U; ++u) s[u] += v[u];
  }
#pragma unroll
  for (int u = 0; u < U; ++u)
    if (ct + u < n) s[u] += p[(int64_t)(ct + u) * stride];
#pragma unroll
  for (int w = U / 2; w > 0; w >>= 1)
#pragma unroll
    for (int u = 0; u < w; ++u) s[u] += s[u + w];
  return s[0];
}

// strided_sum<U> at the narrowest width that holds n partials in one pass:
// the same bits (with n <= U' every partial sits alone in its slot and the
// wider tree only adds exact zeros in the same pairing order), without the
// wide form's predicated tail -- a compare, a 64-bit address and a branch per
// slot for 16 slots when C2's threads hold one or two partials.
template <int U>
__device__ __forceinline__ double strided_sum_fit(const double* __restrict__ p, int64_t stride, int n) {
  if (n <= 2) return strided_sum<2>(p, stride, n);
  if (n <= 4) return strided_sum<4>(p, stride, n);
  if (U > 8 && n <= 8) return strided_sum<8>(p, stride, n);
  return strided_sum<U>(p, stride, n);
}

// z_J of this lane's group of G lanes: lane J of the group (DPP row
// broadcast; G = 8: the row's two groups take lanes J and 8 + J)
template <int G, int J>
__device__ __forceinline__ double group_bcast(double z, bool upper) {
  if constexpr (G == 16) {
    return row_bcast<J>(z);
  } else {
    const double lo = row_bcast<J>(z), hi = row_bcast<8 + J>(z);
    return upper ? hi : lo;
  }
}

// f + sum_{j >= J} Lr[j] z_j (j ascending: the serial form's FMA chain)
template <int G, int J>
__device__ __forceinline__ double lq_chain(const double (&Lr)[QMAX], double z, bool upper, double f) {
  f = fma(Lr[J], group_bcast<G, J>(z, upper), f);
  if constexpr (J + 1 < G) return lq_chain<G, J + 1>(Lr, z, upper, f);
  return f;
}

// max / sum over the G lanes of a group (xor shuffles inside the group)
template <int G>
__device__ __forceinline__ double group_max(double v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  return v;
}
template <int G>
__device__ __forceinline__ double group_sum(double v) {
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// log_q_reduce (logred.h) across a group: li of the active lanes
template <int G>
__device__ __forceinline__ double group_log_q_reduce(double li, bool act, const LogRedParams& p) {
  const double tau = p.tau_max;
  const double M = group_max<G>(act ? li : -INFINITY);
  if (p.fat) {
    const double x = (M - li) / tau;
    const double den = 2.0 + 2.0 * x + x * x;
    const double P = group_sum<G>(act ? 2.0 / den : 0.0);
    return M + tau * log(P);
  }
  const double Ms = M / tau;
  const double ssum = group_sum<G>(act ? exp(li / tau - Ms) : 0.0);
  return tau * (Ms + log(ssum));
}

// Samples and the MC reduction of one t-batch.  Lane (slot = lane / G,
// a = lane % G) of wave w holds row a of L_q in registers and takes test
// point a of sample s = s0 + (64 / G) w + slot: z[s][a] is one coalesced load,
// z[s][j] reaches the group by DPP broadcast, f_a is the same FMA chain (j
// ascending) as the serial form, and the q-reductions are shuffles inside the
// group.  SB samples' loads per lane are in flight at once.  (The serial
// per-sample loop read L_q from LDS once per FMA and paid one L2 latency per
// sample: 22 us of C3's 38 us finalisation, profiles/r04/qmc.)  Accumulates
// the qEI sum / the log modes' (max, sum-exp) pair in the group's lane 0.
template <int G, int MODE>
__device__ __forceinline__ void sample_phase(int tid, int q, int S, int row0,
                                             const double (&Lq)[QMAX][QMAX + 1],
                                             const double (&mu)[QMAX], const double* __restrict__ Z,
                                             const double* __restrict__ F, int64_t ldF, double best_f,
                                             const double* __restrict__ best_f_s,
                                             const LogRedParams& lp, double& sum, LseAcc& lse) {
  constexpr int SLOTS = 64 / G;             // samples per wave per pass
  constexpr int PER = SLOTS * (THREADS / 64);  // samples per workgroup per pass
  constexpr int SB = 8;
  const int lane = tid & 63, a_ = lane % G, slot = lane / G, wv = tid >> 6;
  const bool upper = (lane & 8) != 0;  // G = 8: the row's second group
  const bool arow = a_ < q;
  double Lr[QMAX];
#pragma unroll
  for (int j = 0; j < QMAX; ++j) Lr[j] = (arow && j <= a_) ? Lq[a_][j] : 0.0;
  const double mu_a = arow ? mu[a_] : 0.0;
  for (int s0 = 0; s0 < S; s0 += SB * PER) {
    double zb[SB], fb[SB], bb[SB];
#pragma unroll
    for (int u = 0; u < SB; ++u) {
      const int s = s0 + u * PER + SLOTS * wv + slot;
      const bool act = s < S && arow;
      zb[u] = act ? Z[(int64_t)s * q + a_] : 0.0;
      fb[u] = (F != nullptr && act) ? F[(int64_t)s * ldF + row0 + a_] : 0.0;
      bb[u] = per_sample_best(MODE) ? (s < S ? best_f_s[s] : 0.0) : best_f;
    }
#pragma unroll
    for (int u = 0; u < SB; ++u) {
      const int s = s0 + u * PER + SLOTS * wv + slot;
      const bool sv = s < S;
      const bool act = sv && arow;
      const double f = lq_chain<G, 0>(Lr, zb[u], upper, mu_a + fb[u]);
      const double bf = bb[u];
      if (log_mode(MODE)) {
        const double li = act ? log_soft_relu(f - bf, lp, nullptr) : -INFINITY;
        const double uu = group_log_q_reduce<G>(li, act, lp);
        if (a_ == 0 && sv) lse = lse_push(lse, uu);
      } else {
        // max_a relu(f_a - best_f) = relu(max_a (f_a - best_f)): fmax is exact
        const double v = group_max<G>(act ? f - bf : -INFINITY);
        if (a_ == 0 && sv) sum += fmax(v, 0.0);
      }
    }
  }
}

// One sample per thread (S <= THREADS): the z row (zs) and the sample's best
// (bf) were loaded at the kernel's entry, L_q from LDS.
template <int MODE>
__device__ __forceinline__ void sample_serial(int tid, int q, int S, int row0,
                                              const double (&Lq)[QMAX][QMAX + 1],
                                              const double (&mu)[QMAX], const double (&zs)[QMAX],
                                              double bf, const double* __restrict__ F, int64_t ldF,
                                              const LogRedParams& lp, double& sum, LseAcc& lse) {
  const int s = tid;
  if (s >= S) return;
  double vmax = 0.0;
  double li[QMAX];
#pragma unroll
  for (int a = 0; a < QMAX; ++a) {
    li[a] = 0.0;
    if (a < q) {
      double f = mu[a] + ((F != nullptr) ? F[(int64_t)s * ldF + row0 + a] : 0.0);
#pragma unroll
      for (int j = 0; j <= a; ++j) f = fma(Lq[a][j], zs[j], f);
      if (log_mode(MODE)) li[a] = log_soft_relu(f - bf, lp, nullptr);
      else vmax = fmax(vmax, f - bf);
    }
  }
  if (log_mode(MODE)) lse = lse_push(lse, log_q_reduce<QMAX>(li, q, lp, nullptr));
  else sum += vmax;
}

// psd_safe_cholesky's ladder on the q x q covariance, one wave.  Lane l owns
// the entries (a0 + RS k, c) of a W-wide layout (c = l % W, a0 = l / W, RS =
// 64 / W rows apart; W = 8: one entry, W = 16: four).  Column j: the pivot by
// v_readlane, l_aj = a_aj / sqrt(a_jj) written to colb by the column's lanes,
// then every trailing entry a_ac -= l_aj l_cj with both factors from colb (in
// order within the wave: no barrier).  Per entry the FMA sequence (j
// ascending, fma(-l_aj, l_cj, .)) is the row-per-lane form's: the same bits.
// (The row-per-lane form broadcast each column entry by a v_readlane pair per
// row: ~2700 instructions on one wave, 3.8 us of C2's 11.5 us kernel span.)
template <int W>
__device__ __forceinline__ void ladder_factor(int lane, int q, const double (&Sig)[QMAX][QMAX + 1],
                                              double (&Lq)[QMAX][QMAX + 1], double* colb,
                                              int max_tries, double jitter0, int& s_info,
                                              double& s_jit) {
  constexpr int RS = 64 / W, R = W / RS;  // rows apart, entries per lane
  const int c = lane % W, a0 = lane / W;
  double jit = 0.0;
  int info = 0;
  for (int attempt = 0; attempt <= max_tries; ++attempt) {
    if (attempt > 0) jit = jitter0 * pow(10.0, (double)(attempt - 1));
    double v[R];
#pragma unroll
    for (int k = 0; k < R; ++k) {
      const int a = a0 + RS * k;
      v[k] = (a < q && c <= a) ? Sig[a][c] + ((a == c) ? jit : 0.0) : 0.0;
    }
    info = 0;
#pragma unroll
    for (int j = 0; j < W; ++j) {
      if (j < q) {
        const double ajj = readlane_d(v[j / RS], (j % RS) * W + j);
        if (!(ajj > 0.0) && info == 0) info = j + 1;
        const double rinv = rsq_nr(ajj);
        if (c == j) {
#pragma unroll
          for (int k = 0; k < R; ++k) {
            const int a = a0 + RS * k;
            if (a >= j && a < q) {
              const double l = (a == j) ? ajj * rinv : v[k] * rinv;
              v[k] = l;
              colb[a] = l;
            }
          }
        }
        if (c > j && c < q) {
          const double lc = colb[c];
#pragma unroll
          for (int k = 0; k < R; ++k) {
            const int a = a0 + RS * k;
            if (a >= c && a < q) v[k] = fma(-colb[a], lc, v[k]);
          }
        }
      }
    }
    if (info == 0) {
#pragma unroll
      for (int k = 0; k < R; ++k) {
        const int a = a0 + RS * k;
        Lq[a][c] = (c <= a && a < q) ? v[k] : 0.0;
      }
      break;
    }
  }
  if (lane == 0) {
    s_info = info;
    s_jit = jit;
  }
}

// A ModelListGP's members finalised in one launch (bo_qmc_finalize_members,
// root-only mode): member blockIdx.y's rows, partials, scalars and outputs
// replace the kernel's own arguments.
constexpr int QMC_MAXM = 8;
struct QmcMembers {
  const double* Xq[QMC_MAXM];
  const double* Spart[QMC_MAXM];
  const double* mpart[QMC_MAXM];
  double outputscale[QMC_MAXM], constant[QMC_MAXM], ymean[QMC_MAXM], ystd[QMC_MAXM];
  double* mean_out[QMC_MAXM];
  double* L_out[QMC_MAXM];
  int* info_out[QMC_MAXM];
  double* jitter_out[QMC_MAXM];
  double* status_out[QMC_MAXM];
  int* status_count[QMC_MAXM];
  const double* Tm[QMC_MAXM];  // cached-root qNEHVI: per member T (r x ldT) and F (S x ldF)
  const double* F[QMC_MAXM];
  int nm;  // 0: the kernel's own arguments
};

template <int KIND, int MODE>
__global__ __launch_bounds__(THREADS) void qmc_kernel(
    int q, int Qp, const double* __restrict__ Xq, const double* __restrict__ Spart,
    const double* __restrict__ mpart, int nC, int nrows_pad, double outputscale,
    double constant, double ymean, double ystd, const double* __restrict__ Z, int S,
    double best_f, const double* __restrict__ best_f_s, int max_tries, double jitter0,
    double* __restrict__ acq, double* __restrict__ mean_out, double* __restrict__ cov_out,
    double* __restrict__ L_out, int* __restrict__ info_out, double* __restrict__ jitter_out,
    const double* __restrict__ Tm, int r, int64_t ldT, const double* __restrict__ F,
    int64_t ldF, LogRedParams lp, int sym, double* __restrict__ status_out,
    int* __restrict__ status_count, QmcMembers qm = QmcMembers{}) {
  if (qm.nm > 0) {
    const int m = blockIdx.y;
    Xq = qm.Xq[m];
    Spart = qm.Spart[m];
    mpart = qm.mpart[m];
    outputscale = qm.outputscale[m];
    constant = qm.constant[m];
    ymean = qm.ymean[m];
    ystd = qm.ystd[m];
    mean_out = qm.mean_out[m];
    L_out = qm.L_out[m];
    info_out = qm.info_out[m];
    jitter_out = qm.jitter_out[m];
    status_out = qm.status_out[m];
    status_count = qm.status_count[m];
    Tm = qm.Tm[m];
    F = qm.F[m];
  }
  // qNEI with the cached baseline root (utils/low_rank.py:85-173): Tm (r x ldT)
  // holds bl_chol^T = L_rr^{-1} Sigma'(X_base, X) per padded test row and F
  // (S x ldF) the samples' baseline term Z_base T; then
  //   br = Sigma'_qq - T^T T,  f = mu' + F + chol(br) Z_q.
  __shared__ double Sig[QMAX][QMAX + 1];
  __shared__ double Lq[QMAX][QMAX + 1];
  __shared__ double mu[QMAX];
  __shared__ double red[THREADS / 64];
  __shared__ double red2[THREADS / 64];
  __shared__ int s_info;
  __shared__ double s_jit;
  __shared__ int s_last;
  __shared__ double colb[QMAX];
  __shared__ double psum[THREADS];
  __shared__ double msum[THREADS];

  QMC_PHASE(0);
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int row0 = b * Qp;               // first padded test row of this t-batch
  const int tile = row0 >> 4;            // its 16-row MFMA tile
  const int off = row0 & 15;             // offset inside the tile
  const int nrows16 = nrows_pad >> 4;
  const double s2 = ystd * ystd;

  // The one-sample-per-thread form's z row and best first (S <= THREADS, C2):
  // their loads are in flight with the partials' instead of after the q x q
  // Cholesky
  const bool serial = S <= THREADS && MODE != QMC_POSTERIOR && MODE != QMC_CHOL;
  double zs[QMAX];
  double bf_s = best_f;
#pragma unroll
  for (int j = 0; j < QMAX; ++j) zs[j] = 0.0;
  if (serial && tid < S) {
    const double* z = Z + (int64_t)tid * q;
#pragma unroll
    for (int j = 0; j < QMAX; ++j)
      if (j < q) zs[j] = z[j];
    if (per_sample_best(MODE)) bf_s = best_f_s[tid];
  }

  // 1. finalise the q x q covariance and the mean.  The partial sums use all
  // threads: nsplit threads per entry (q = 8: 4) each take every nsplit-th
  // partial, combined in a fixed order below -- the quad plan's partial count
  // (C2: 136 block pairs, summed as P + P^T) would otherwise put ~35 dependent
  // load rounds on 64 threads.
  const int E = q * q;
  const int nsplit = THREADS / E;  // >= 1 (q <= 16)
  // K** of this thread's entry first: its row loads are in flight with the
  // partials' below instead of after them
  double kxx = 0.0;
  if (tid < E) {
    const int a = tid / q, c = tid % q;
    if (a == c) {
      kxx = outputscale;
    } else {
      const double* xa = Xq + (int64_t)(row0 + a) * DP;
      const double* xc = Xq + (int64_t)(row0 + c) * DP;
      double d2 = 0.0;
#pragma unroll
      for (int t = 0; t < DP; ++t) {
        const double df = xa[t] - xc[t];
        d2 = fma(df, df, d2);
      }
      kxx = outputscale * kernel_from_d2<KIND>(d2);
    }
  }
  if (tid < E * nsplit) {
    const int e = tid % E, j = tid / E;
    const int a = e / q, c = e % q;
    const int64_t pstride = (int64_t)nrows16 * 256;
    const int cnt = nC > j ? (nC - 1 - j) / nsplit + 1 : 0;
    const double* sp = Spart + (int64_t)j * pstride + (int64_t)tile * 256 + (off + a) * 16 + (off + c);
    double part = strided_sum_fit<16>(sp, pstride * nsplit, cnt);
    if (sym) {  // quad plan partials (quad.hip): Sigma = sum_p P_p + P_p^T
      const double* spt =
          Spart + (int64_t)j * pstride + (int64_t)tile * 256 + (off + c) * 16 + (off + a);
      part += strided_sum_fit<16>(spt, pstride * nsplit, cnt);
    }
    psum[tid] = part;
  }
  {  // the mean's partials likewise: THREADS / q threads per test row
    const int ms = THREADS / q;
    const int a = tid % q, j = tid / q;
    if (j < ms) {
      const int cnt = nC > j ? (nC - 1 - j) / ms + 1 : 0;
      msum[tid] = strided_sum_fit<16>(mpart + (int64_t)j * nrows_pad + row0 + a, (int64_t)nrows_pad * ms, cnt);
    }
  }
  __syncthreads();
  if (tid < E) {
    const int a = tid / q, c = tid % q;
    double acc = 0.0;
    for (int j = 0; j < nsplit; ++j) acc += psum[j * E + tid];
    double v = s2 * (kxx - acc);
    if (Tm != nullptr) {
      // T^T T over the r baseline rows: unrolled so eight rows' loads are in
      // flight per wait (one L2 round trip per row had made this loop most of
      // qNEHVI's finalisation, 68 us at C4); the FMA chain keeps its order
      double tt = 0.0;
#pragma unroll 8
      for (int j = 0; j < r; ++j) tt = fma(Tm[j * ldT + row0 + a], Tm[j * ldT + row0 + c], tt);
      v -= tt;
    }
    Sig[a][c] = v;
    if (cov_out) cov_out[((int64_t)b * q + a) * q + c] = v;
  }
  if (tid < q) {
    double m = 0.0;
    for (int j = 0; j < THREADS / q; ++j) m += msum[j * q + tid];
    const double v = ymean + ystd * (constant + m);
    mu[tid] = v;
    if (mean_out) mean_out[(int64_t)b * q + tid] = v;
  }
  __syncthreads();
  QMC_PHASE(1);
  if (MODE == QMC_POSTERIOR) return;

  // 2. Cholesky with the jitter ladder (wave 0, one lane per entry: ladder_factor)
  if (tid < 64) {
    if (q <= 8)
      ladder_factor<8>(tid, q, Sig, Lq, colb, max_tries, jitter0, s_info, s_jit);
    else
      ladder_factor<16>(tid, q, Sig, Lq, colb, max_tries, jitter0, s_info, s_jit);
  }
  __syncthreads();
  QMC_PHASE(2);
  const int info = s_info;
  if (tid == 0) {
    // agent-scope (write-through) stores: the fused status reads them from
    // other XCDs' workgroups without an L2 write-back fence
    if (info_out) __hip_atomic_store(info_out + b, info, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (jitter_out)
      __hip_atomic_store(jitter_out + b, s_jit, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // The batch's ladder status (bo_ladder_status's [max info, max jitter])
  // folded in at the workgroup's exit: every workgroup counts itself in once
  // its entries are drained, the last to arrive reduces all B of them and
  // re-arms the counter.  Counting at the exit keeps the counter's round trip
  // (one address for the whole grid) off the sampling.  The hand-off follows
  // MI355X_MICROARCH.md's inter-workgroup recipe (as chol_dag.hip):
  // write-through stores drained (vmcnt(0)) before the agent-scope count,
  // agent-scope loads on the reading side -- an agent-scope release fence
  // would write back the whole L2 per workgroup.  Called by every thread.
  auto status_arrive = [&]() {
    QMC_PHASE(3);
    if (status_out == nullptr) return;
    __syncthreads();  // red / red2 free (the reduction below is done with them)
    if (tid == 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      s_last = __hip_atomic_fetch_add(status_count, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
               (int)gridDim.x - 1;
    }
    __syncthreads();
    if (!s_last) {
      QMC_PHASE(4);
      return;
    }
    double mi = 0.0, mj = 0.0;
    for (int bb = tid; bb < (int)gridDim.x; bb += THREADS) {
      mi = fmax(mi, (double)__hip_atomic_load(info_out + bb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      mj = fmax(mj, __hip_atomic_load(jitter_out + bb, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    }
    for (int o = 32; o > 0; o >>= 1) {
      mi = fmax(mi, __shfl_xor(mi, o));
      mj = fmax(mj, __shfl_xor(mj, o));
    }
    if ((tid & 63) == 0) {
      red[tid >> 6] = mi;
      red2[tid >> 6] = mj;
    }
    __syncthreads();
    if (tid == 0) {
      // folded into what the words hold (sticky): the eager calls' ring slots
      // are zeroed by the host before each use, a captured graph's buffer is
      // zeroed only when its status has been acted on, so it collects the max
      // over every replay since (graphs.GraphedAcquisition)
      status_out[0] = fmax(status_out[0], fmax(fmax(red[0], red[1]), fmax(red[2], red[3])));
      status_out[1] = fmax(status_out[1], fmax(fmax(red2[0], red2[1]), fmax(red2[2], red2[3])));
      __hip_atomic_store(status_count, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    QMC_PHASE(4);
  };
  if (L_out && tid < q * q) {
    const int a = tid / q, c = tid % q;
    L_out[((int64_t)b * q + a) * q + c] = info ? NAN : Lq[a][c];
  }
  if (MODE == QMC_CHOL) {
    status_arrive();
    return;
  }
  if (info) {
    if (tid == 0) acq[b] = NAN;
    status_arrive();
    return;
  }

  // 3. samples and the reduction (sample_phase): groups of G = 16 lanes for
  // q > 8, G = 8 for q <= 8 (twice the samples per pass).
  // At most one sample per thread (S <= THREADS, C2) the serial form is
  // shorter: one latency for its z row, q(q+1)/2 FMAs (measured at C2: 12.8 us
  // serial against 14.0 grouped).
  double sum = 0.0;
  LseAcc lse{-INFINITY, 0.0};
  if (serial)
    sample_serial<MODE>(tid, q, S, row0, Lq, mu, zs, bf_s, F, ldF, lp, sum, lse);
  else if (q > 8)
    sample_phase<16, MODE>(tid, q, S, row0, Lq, mu, Z, F, ldF, best_f, best_f_s, lp, sum, lse);
  else
    sample_phase<8, MODE>(tid, q, S, row0, Lq, mu, Z, F, ldF, best_f, best_f_s, lp, sum, lse);
  if (log_mode(MODE)) {
    for (int o = 32; o > 0; o >>= 1) {
      LseAcc other{__shfl_xor(lse.m, o), __shfl_xor(lse.s, o)};
      lse = lse_merge(lse, other);
    }
    if ((tid & 63) == 0) {
      red[tid >> 6] = lse.m;
      red2[tid >> 6] = lse.s;
    }
    __syncthreads();
    if (tid == 0) {
      LseAcc t{-INFINITY, 0.0};
      for (int w = 0; w < THREADS / 64; ++w) t = lse_merge(t, LseAcc{red[w], red2[w]});
      acq[b] = t.m + log(t.s) - log((double)S);
    }
    status_arrive();
    return;
  }
  for (int o = 32; o > 0; o >>= 1) sum += __shfl_xor(sum, o);
  if ((tid & 63) == 0) red[tid >> 6] = sum;
  __syncthreads();
  if (tid == 0) {
    double t = 0.0;
    for (int w = 0; w < THREADS / 64; ++w) t += red[w];
    acq[b] = t / S;
  }
  status_arrive();
}

struct QmcArgs {
  int q, Qp;
  const double *Xq, *Spart, *mpart;
  int nC, nrows_pad;
  double outputscale, constant, ymean, ystd;
  const double* Z;
  int S;
  double best_f;
  const double* best_f_s;
  int max_tries;
  double jitter0;
  double *acq, *mean_out, *cov_out, *L_out;
  int* info_out;
  double* jitter_out;
  const double* Tm;
  int r;
  int64_t ldT;
  const double* F;
  int64_t ldF;
  LogRedParams lp;
  int sym;
  double* status_out;
  int* status_count;
};

template <int KIND, int MODE>
void launch_mode(int B, const QmcArgs& a, hipStream_t st) {
  qmc_kernel<KIND, MODE><<<B, THREADS, 0, st>>>(
      a.q, a.Qp, a.Xq, a.Spart, a.mpart, a.nC, a.nrows_pad, a.outputscale, a.constant, a.ymean,
      a.ystd, a.Z, a.S, a.best_f, a.best_f_s, a.max_tries, a.jitter0, a.acq, a.mean_out,
      a.cov_out, a.L_out, a.info_out, a.jitter_out, a.Tm, a.r, a.ldT, a.F, a.ldF, a.lp, a.sym,
      a.status_out, a.status_count);
}

template <int KIND>
void launch_qmc(int mode, int B, const QmcArgs& a, hipStream_t st) {
  if (mode == QMC_POSTERIOR) launch_mode<KIND, QMC_POSTERIOR>(B, a, st);
  else if (mode == QMC_QEI) launch_mode<KIND, QMC_QEI>(B, a, st);
  else if (mode == QMC_QNEI) launch_mode<KIND, QMC_QNEI>(B, a, st);
  else if (mode == QMC_QLOGEI) launch_mode<KIND, QMC_QLOGEI>(B, a, st);
  else if (mode == QMC_QLOGNEI) launch_mode<KIND, QMC_QLOGNEI>(B, a, st);
  else launch_mode<KIND, QMC_CHOL>(B, a, st);
}

}  // namespace

extern "C" int bo_post_geometry(int64_t B, int q, int64_t n, int* Qp, int* nrows_pad, int* nC);

extern "C" int bo_qmc_finalize_ext(int kind, int mode, int B, int q, const double* Xq,
                                   const double* Spart, const double* mpart, int64_t n,
                                   double outputscale, double constant, double ymean,
                                   double ystd, const double* Z, int S, double best_f,
                                   const double* best_f_s, int max_tries, double jitter0,
                                   double* acq, double* mean_out, double* cov_out, double* L_out,
                                   int* info_out, double* jitter_out, const double* Tm, int r,
                                   int64_t ldT, const double* F, int64_t ldF, int fat,
                                   double tau_relu, double tau_max, int nparts, int sym_parts,
                                   double* status_out, int* status_count, void* stream);

extern "C" int bo_qmc_finalize(int kind, int mode, int B, int q, const double* Xq,
                               const double* Spart, const double* mpart, int64_t n,
                               double outputscale, double constant, double ymean, double ystd,
                               const double* Z, int S, double best_f, const double* best_f_s,
                               int max_tries, double jitter0, double* acq, double* mean_out,
                               double* cov_out, double* L_out, int* info_out,
                               double* jitter_out, const double* Tm, int r, int64_t ldT,
                               const double* F, int64_t ldF, int fat, double tau_relu,
                               double tau_max, void* stream) {
  return bo_qmc_finalize_ext(kind, mode, B, q, Xq, Spart, mpart, n, outputscale, constant, ymean,
                             ystd, Z, S, best_f, best_f_s, max_tries, jitter0, acq, mean_out,
                             cov_out, L_out, info_out, jitter_out, Tm, r, ldT, F, ldF, fat,
                             tau_relu, tau_max, 0, 0, nullptr, nullptr, stream);
}

extern "C" int bo_qmc_finalize_ext(int kind, int mode, int B, int q, const double* Xq,
                               const double* Spart, const double* mpart, int64_t n,
                               double outputscale, double constant, double ymean, double ystd,
                               const double* Z, int S, double best_f, const double* best_f_s,
                               int max_tries, double jitter0, double* acq, double* mean_out,
                               double* cov_out, double* L_out, int* info_out,
                               double* jitter_out, const double* Tm, int r, int64_t ldT,
                               const double* F, int64_t ldF, int fat, double tau_relu,
                               double tau_max, int nparts, int sym_parts, double* status_out,
                               int* status_count, void* stream) {
  BO_CHECK_ARG(mode >= 0 && mode <= 5, "bo_qmc_finalize: bad mode %d", mode);
  BO_CHECK_ARG(nparts >= 0 && (sym_parts == 0 || nparts > 0),
               "bo_qmc_finalize: nparts %d / sym_parts %d", nparts, sym_parts);
  BO_CHECK_ARG(status_out == nullptr ||
                   (status_count && info_out && jitter_out && mode != QMC_POSTERIOR),
               "bo_qmc_finalize: the fused ladder status needs a counter, info and jitter outputs");
  if (B == 0) return BO_OK;  // no t-batches (empty outputs may carry null pointers)
  BO_CHECK_ARG(!log_mode(mode) || (tau_relu > 0.0 && tau_max > 0.0),
               "bo_qmc_finalize: tau_relu and tau_max must be positive");
  BO_CHECK_ARG(mode == QMC_POSTERIOR || mode == QMC_CHOL || (acq && Z && S > 0),
               "bo_qmc_finalize: missing MC args");
  BO_CHECK_ARG(!per_sample_best(mode) || best_f_s,
               "bo_qmc_finalize: qNEI / qLogNEI need per-sample best_f");
  BO_CHECK_ARG((Tm == nullptr) == (F == nullptr) && (Tm == nullptr || r > 0),
               "bo_qmc_finalize: cached-root qNEI needs both T and F");
  int Qp, nrows_pad, nC;
  int s = bo_post_geometry(B, q, n, &Qp, &nrows_pad, &nC);
  if (s) return s;
  if (B == 0) return BO_OK;
  if (nparts > 0) nC = nparts;
  QmcArgs a{q,      Qp,     Xq,       Spart,     mpart,     nC,      nrows_pad, outputscale,
            constant, ymean, ystd,   Z,        S,         best_f,  best_f_s,  max_tries,
            jitter0, acq,    mean_out, cov_out,  L_out,     info_out, jitter_out, Tm,
            r,       ldT,    F,        ldF,      LogRedParams{tau_relu, tau_max, fat},
            sym_parts, status_out, status_count};
  hipStream_t st = as_stream(stream);
  if (kind == BO_RBF) launch_qmc<BO_RBF>(mode, B, a, st);
  else launch_qmc<BO_MATERN52>(mode, B, a, st);
  BO_LAUNCH_CHECK();
  return BO_OK;
}

// The root-only finalisation (BO_QMC_CHOL: mean + jittered q x q Cholesky) of
// nm <= 8 models of one shape and kernel kind in ONE launch (grid B x nm):
// per member its rows, partials (nparts as bo_qmc_finalize_ext), scalars,
// outputs and optional fused-status words.
extern "C" int bo_qmc_finalize_members(int nm, int kind, int B, int q, const double* const* Xq,
                                       const double* const* Spart, const double* const* mpart,
                                       int64_t n, const double* outputscale, const double* constant,
                                       const double* ymean, const double* ystd, int max_tries,
                                       double jitter0, double* const* mean_out,
                                       double* const* L_out, int* const* info_out,
                                       double* const* jitter_out, int nparts,
                                       double* const* status_out, int* const* status_count,
                                       const double* const* Tm, int r, int64_t ldT,
                                       const double* const* F, int64_t ldF, void* stream) {
  BO_CHECK_ARG(nm >= 1 && nm <= QMC_MAXM, "bo_qmc_finalize_members: %d models (1..%d)", nm, QMC_MAXM);
  BO_CHECK_ARG(kind == BO_RBF || kind == BO_MATERN52, "bad kernel kind %d", kind);
  BO_CHECK_ARG(nparts >= 0, "bo_qmc_finalize_members: nparts %d", nparts);
  BO_CHECK_ARG(Xq && Spart && mpart && outputscale && constant && ymean && ystd && mean_out && L_out &&
                   info_out && jitter_out,
               "bo_qmc_finalize_members: null pointer array");
  if (B == 0) return BO_OK;
  int Qp, nrows_pad, nC;
  int s = bo_post_geometry(B, q, n, &Qp, &nrows_pad, &nC);
  if (s) return s;
  if (nparts > 0) nC = nparts;
  QmcMembers qm{};
  qm.nm = nm;
  for (int m = 0; m < nm; ++m) {
    BO_CHECK_ARG(Xq[m] && Spart[m] && mpart[m] && mean_out[m] && L_out[m] && info_out[m] && jitter_out[m],
                 "bo_qmc_finalize_members: null buffer");
    BO_CHECK_ARG(!status_out || (status_out[m] && status_count && status_count[m]),
                 "bo_qmc_finalize_members: status words need their counters");
    qm.Xq[m] = Xq[m];
    qm.Spart[m] = Spart[m];
    qm.mpart[m] = mpart[m];
    qm.outputscale[m] = outputscale[m];
    qm.constant[m] = constant[m];
    qm.ymean[m] = ymean[m];
    qm.ystd[m] = ystd[m];
    qm.mean_out[m] = mean_out[m];
    qm.L_out[m] = L_out[m];
    qm.info_out[m] = info_out[m];
    qm.jitter_out[m] = jitter_out[m];
    qm.status_out[m] = status_out ? status_out[m] : nullptr;
    qm.status_count[m] = status_out ? status_count[m] : nullptr;
    BO_CHECK_ARG((Tm == nullptr) == (F == nullptr) && (Tm == nullptr || (r > 0 && Tm[m] && F[m])),
                 "bo_qmc_finalize_members: cached-root members need T and F (r > 0)");
    qm.Tm[m] = Tm ? Tm[m] : nullptr;
    qm.F[m] = F ? F[m] : nullptr;
  }
  hipStream_t st = as_stream(stream);
  const dim3 grid((unsigned)B, (unsigned)nm);
#define BO_QMC_M(KIND)                                                                            \
  qmc_kernel<KIND, QMC_CHOL><<<grid, THREADS, 0, st>>>(                                           \
      q, Qp, Xq[0], Spart[0], mpart[0], nC, nrows_pad, outputscale[0], constant[0], ymean[0],     \
      ystd[0], nullptr, 0, 0.0, nullptr, max_tries, jitter0, nullptr, mean_out[0], nullptr,       \
      L_out[0], info_out[0], jitter_out[0], qm.Tm[0], Tm ? r : 0, ldT, qm.F[0], ldF,               \
      LogRedParams{1.0, 1.0, 1}, 0, qm.status_out[0], qm.status_count[0], qm)
  if (kind == BO_RBF) BO_QMC_M(BO_RBF);
  else BO_QMC_M(BO_MATERN52);
#undef BO_QMC_M
  BO_LAUNCH_CHECK();
  return BO_OK;
}

namespace {

// out[0] = max_b info[b] (as double), out[1] = max_b jitter[b]: the two facts
// the host needs after a batched jitter ladder (fail -> NotPSDError, jitter
// added -> NumericalWarning), in one launch and one 16-byte read-back.
__global__ __launch_bounds__(256) void ladder_status_kernel(const int* __restrict__ info,
                                                            const double* __restrict__ jitter,
                                                            int64_t B, double* __restrict__ out) {
  __shared__ double red[2][4];
  double mi = 0.0, mj = 0.0;
  for (int64_t b = threadIdx.x; b < B; b += 256) {
    mi = fmax(mi, (double)info[b]);
    mj = fmax(mj, jitter[b]);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    mi = fmax(mi, __shfl_xor(mi, o));
    mj = fmax(mj, __shfl_xor(mj, o));
  }
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][wave] = mi;
    red[1][wave] = mj;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    out[0] = fmax(fmax(red[0][0], red[0][1]), fmax(red[0][2], red[0][3]));
    out[1] = fmax(fmax(red[1][0], red[1][1]), fmax(red[1][2], red[1][3]));
  }
}

}  // namespace

extern "C" int bo_ladder_status(const int* info, const double* jitter, int64_t B, double* out,
                                void* stream) {
  BO_CHECK_ARG(B >= 0 && info && jitter && out, "bo_ladder_status: bad arguments");
  ladder_status_kernel<<<1, 256, 0, as_stream(stream)>>>(info, jitter, B, out);
  BO_LAUNCH_CHECK();
  return BO_OK;
}

extern "C" int bo_pinned_alloc(int64_t bytes, void** host, void** dev) {
  BO_CHECK_ARG(bytes > 0 && host && dev, "bo_pinned_alloc: bad arguments");
  BO_HIP(hipHostMalloc(host, (size_t)bytes, hipHostMallocMapped | hipHostMallocCoherent));
  std::memset(*host, 0, (size_t)bytes);
  BO_HIP(hipHostGetDevicePointer(dev, *host, 0));
  return BO_OK;
}

extern "C" int bo_pinned_free(void* host) {
  if (host) BO_HIP(hipHostFree(host));
  return BO_OK;
}

#ifdef BO_QMC_PHASES
extern "C" int bo_qmc_phase_dump(unsigned long long* out, int n) {
  if (n > PH_WG * PH_N) n = PH_WG * PH_N;
  return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_qmc_phase), sizeof(unsigned long long) * n, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}
#endif
