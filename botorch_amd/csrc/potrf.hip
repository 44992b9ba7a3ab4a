// 128 x 128 diagonal-block Cholesky + triangular inverse, one workgroup, in LDS.
//
// Building block of the blocked right-looking factorisation in chol.hip
// (psd_safe_cholesky of the training covariance, botorch/models/gpytorch.py:446
// -> [G] DefaultPredictionStrategy; the explicit inverse is [G]
// root_inv_decomposition's L^{-T}, botorch/__init__.py:44).  The block is
// held in LDS (128 rows at pitch 130 doubles = 133 KB of the CU's 160 KB) and
// factored as four 32-column sub-panels:
//   F1  waves 0 and 1 factor the 32 x 32 diagonal sub-block AND build its
//       inverse in one sweep: each lane owns a 4 x 4 tile, of L on wave 0 and
//       of X = L^{-1} on wave 1; a step factors a 2 x 2 pivot block and applies
//       rank-2 updates (right-looking Cholesky on wave 0, right-looking forward
//       substitution on wave 1, one step behind, columns and pivots passed
//       through LDS), 16 steps with one barrier each;
//   F2  the sub-panel below is solved against that inverse on the fp64 MFMA
//       (each wave owns whole 16-row strips and updates them in place);
//   F3  the trailing lower triangle of the block takes the rank-32 update on the
//       MFMA (16 x 16 tiles dealt round-robin over the 4 waves, two at a time).
// The 32-block inverses are then merged into the 128-block inverse by recursive
// doubling, X21 = -X22 L21 X11, again on the MFMA, and L and L^{-1} are written
// to HBM.  The strictly-upper 32 x 32 blocks of the LDS tile are free space:
// they hold the sub-block inverses (F1) and the products T = L21 X11 of the
// merge.
//
// A non-positive or NaN pivot records info = 1-based order of the first failing
// leading minor (torch.linalg.cholesky_ex semantics), as the jitter ladder of
// bo_cholesky_jitter / bo_gp_cache_build expects.
#include "common.h"

namespace {

constexpr int DB = 128;  // diagonal block
constexpr int SP = 130;  // LDS pitch (doubles): rows of a 16-row MFMA fragment hit distinct banks

__device__ __forceinline__ double readlane_d(double v, int l) {
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(x & 0xffffffffll), l);
  const int hi = __builtin_amdgcn_readlane((int)(x >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// acc[t] += A(16 x K) B_t(K x 16) from LDS, t < NT, sharing the A fragments
// (NT independent accumulation chains keep the matrix pipe busy).
// A(m, k) = Ab[m * SP + k].  B_t = Bb + t * bstep;
// BT: B(k, j) = B_t[j * SP + k]; else B(k, j) = B_t[k * SP + j].
// Optional triangular masks (block coordinates): A(m, k) := 0 when
// k > a_m0 + m (lower A, k counted from 0); B_t(k, j) := 0 when k < t * 16 + j
// (lower B whose column tiles start at 16 t).
template <int NT, int K, bool BT, bool AMASK, bool BMASK>
__device__ __forceinline__ void mma16(const double* Ab, const double* Bb, int bstep, int lane,
                                      v4d (&acc)[NT], int a_m0 = 0) {
  const int mm = lane & 15;
  const int kq = lane >> 4;
#pragma unroll
  for (int k0 = 0; k0 < K; k0 += 4) {
    const int kk = k0 + kq;
    double a = Ab[mm * SP + kk];
    if (AMASK && kk > a_m0 + mm) a = 0.0;
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      const double* Bt = Bb + t * bstep;
      double b = BT ? Bt[mm * SP + kk] : Bt[kk * SP + mm];
      if (BMASK && kk < t * 16 + mm) b = 0.0;
      acc[t] = mfma_f64(a, b, acc[t]);
    }
  }
}

// Store a 16 x 16 accumulator tile into LDS at D (row pitch SP), scaled.
__device__ __forceinline__ void put16(double* D, v4d acc, int lane, double scale) {
#pragma unroll
  for (int r = 0; r < 4; ++r) D[mfma_row(lane, r) * SP + mfma_col(lane)] = scale * acc[r];
}

__device__ __forceinline__ void tri_index(int t, int& tr, int& tc) {
  tr = 0;
  while ((tr + 1) * (tr + 2) / 2 <= t) ++tr;
  tc = t - tr * (tr + 1) / 2;
}

// Factor the 32 x 32 block at Sd (in place, lower; upper zeroed) and write its
// inverse (lower, upper zeroed) at Dd.  Called by all four waves of the
// workgroup; two of them work.  Lane = (ti, tj) owns rows 4 ti.., cols 4 tj..
// of its wave's matrix: wave 0 holds L (right-looking Cholesky), wave 1 holds
// X = L^{-1} (right-looking forward substitution).  A step factors a 2 x 2
// pivot block and applies a rank-2 update, 16 steps in all.  Wave 0 publishes
// the step's two L columns and pivot scalars in LDS (double-buffered by step
// parity); wave 1 applies step s - 1 while wave 0 runs step s, one workgroup
// barrier per step, so the two halves of the fp64 work (1024 FMAs per lane
// each) overlap instead of queueing on one wave.  Returns (wave 0) the
// 1-based failing pivot or 0.
__device__ __forceinline__ int factor32(double* Sd, double* Dd, double* colbuf, double* pivbuf,
                                        double* rowbuf, int lane, int wave) {
  const int ti = lane >> 3, tj = lane & 7;
  const bool wL = wave == 0, wX = wave == 1;
  double m[4][4];  // wave 0: a (-> L), wave 1: x (-> X)
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int i = 4 * ti + u, l = 4 * tj + v;
      m[u][v] = wL ? ((l <= i) ? Sd[i * SP + l] : 0.0) : ((l == i) ? 1.0 : 0.0);
    }
  int fail = 0;
  // 1/sqrt by v_rsq_f64 + two Newton steps (full fp64 accuracy).
  auto rsq_nr = [](double v) {
    double r = __builtin_amdgcn_rsq(v);
    r = r * fma(-0.5 * v * r, r, 1.5);
    r = r * fma(-0.5 * v * r, r, 1.5);
    return r;
  };
  double p00 = 0.0, p10 = 0.0, p11 = 0.0, inv0 = 0.0, L10 = 0.0, s11 = 0.0, inv1 = 0.0;
  if (wL) {
    p00 = readlane_d(m[0][0], 0);
    p10 = readlane_d(m[1][0], 0);
    p11 = readlane_d(m[1][1], 0);
    inv0 = rsq_nr(p00);
    L10 = p10 * inv0;
    s11 = fma(-L10, L10, p11);
    inv1 = rsq_nr(s11);
  }

  // Wave 0, step j: columns j, j+1 -> colbuf[buf], pivot scalars -> pivbuf[buf],
  // rank-2 Cholesky update (next pivot block first).
#define BO_L_STEP(JU)                                                                     \
  {                                                                                       \
    const int ju = (JU);                                                                  \
    const int j = 4 * jt + ju;                                                            \
    const int buf = (j >> 1) & 1;                                                         \
    double* cb = colbuf + buf * 64;                                                       \
    if (fail == 0) {                                                                      \
      if (!(p00 > 0.0)) fail = j + 1;                                                     \
      else if (!(s11 > 0.0)) fail = j + 2;                                                \
    }                                                                                     \
    const double L00 = p00 * inv0, L11 = s11 * inv1;                                      \
    if (tj == jt) {                                                                       \
      _Pragma("unroll") for (int u = 0; u < 4; ++u) {                                    \
        const int i = 4 * ti + u;                                                         \
        const double c0 = (i > j) ? m[u][ju] * inv0 : ((i == j) ? L00 : 0.0);            \
        const double c1 =                                                                 \
            (i > j + 1) ? fma(-c0, L10, m[u][ju + 1]) * inv1 : ((i == j + 1) ? L11 : 0.0); \
        m[u][ju] = c0;                                                                    \
        m[u][ju + 1] = c1;                                                                \
        cb[i] = c0;                                                                       \
        cb[32 + i] = c1;                                                                  \
      }                                                                                   \
    }                                                                                     \
    if (lane == 0) {                                                                      \
      pivbuf[buf * 4 + 0] = inv0;                                                         \
      pivbuf[buf * 4 + 1] = L10;                                                          \
      pivbuf[buf * 4 + 2] = inv1;                                                         \
    }                                                                                     \
    asm volatile("" ::: "memory");                                                        \
    double Lr0[4], Lr1[4], Lcm0[4], Lcm1[4];                                              \
    _Pragma("unroll") for (int h = 0; h < 2; ++h) {                                      \
      const double2 r0 = *reinterpret_cast<const double2*>(cb + 4 * ti + 2 * h);          \
      const double2 r1 = *reinterpret_cast<const double2*>(cb + 32 + 4 * ti + 2 * h);     \
      const double2 q0 = *reinterpret_cast<const double2*>(cb + 4 * tj + 2 * h);          \
      const double2 q1 = *reinterpret_cast<const double2*>(cb + 32 + 4 * tj + 2 * h);     \
      Lr0[2 * h] = r0.x; Lr0[2 * h + 1] = r0.y;                                           \
      Lr1[2 * h] = r1.x; Lr1[2 * h + 1] = r1.y;                                           \
      Lcm0[2 * h] = q0.x; Lcm0[2 * h + 1] = q0.y;                                         \
      Lcm1[2 * h] = q1.x; Lcm1[2 * h + 1] = q1.y;                                         \
    }                                                                                     \
    asm volatile("" ::: "memory");                                                        \
    _Pragma("unroll") for (int v = 0; v < 4; ++v) {                                      \
      const bool cl = 4 * tj + v > j + 1;                                                 \
      Lcm0[v] = cl ? -Lcm0[v] : 0.0;                                                      \
      Lcm1[v] = cl ? -Lcm1[v] : 0.0;                                                      \
    }                                                                                     \
    const int j1 = j + 2;                                                                 \
    const int u1 = (ju + 2) & 3;                                                          \
    if (j1 < 32) {                                                                        \
      m[u1][u1] = fma(Lr1[u1], Lcm1[u1], fma(Lr0[u1], Lcm0[u1], m[u1][u1]));              \
      m[u1 + 1][u1] = fma(Lr1[u1 + 1], Lcm1[u1], fma(Lr0[u1 + 1], Lcm0[u1], m[u1 + 1][u1])); \
      m[u1 + 1][u1 + 1] =                                                                 \
          fma(Lr1[u1 + 1], Lcm1[u1 + 1], fma(Lr0[u1 + 1], Lcm0[u1 + 1], m[u1 + 1][u1 + 1])); \
      const int src = (j1 >> 2) * 9;                                                      \
      p00 = readlane_d(m[u1][u1], src);                                                   \
      p10 = readlane_d(m[u1 + 1][u1], src);                                               \
      p11 = readlane_d(m[u1 + 1][u1 + 1], src);                                           \
      inv0 = rsq_nr(p00);                                                                 \
      L10 = p10 * inv0;                                                                   \
      s11 = fma(-L10, L10, p11);                                                          \
      inv1 = rsq_nr(s11);                                                                 \
    }                                                                                     \
    _Pragma("unroll") for (int u = 0; u < 4; ++u)                                        \
      _Pragma("unroll") for (int v = 0; v < 4; ++v) {                                    \
        const bool early = j1 < 32 && ((u == u1 && v == u1) || (u == u1 + 1 && v == u1) || \
                                       (u == u1 + 1 && v == u1 + 1));                     \
        if (!early) m[u][v] = fma(Lr1[u], Lcm1[v], fma(Lr0[u], Lcm0[v], m[u][v]));        \
      }                                                                                   \
  }
  // Wave 1, step j (published by wave 0 one barrier earlier): rows j, j+1 of X
  // scaled by the pivot block, then the rank-2 substitution update.
#define BO_X_STEP(JT, JU)                                                                 \
  {                                                                                       \
    const int jtx = (JT), ju = (JU);                                                      \
    const int j = 4 * jtx + ju;                                                           \
    const int buf = (j >> 1) & 1;                                                         \
    const double* cb = colbuf + buf * 64;                                                 \
    const double xi0 = pivbuf[buf * 4 + 0], xl10 = pivbuf[buf * 4 + 1],                   \
                 xi1 = pivbuf[buf * 4 + 2];                                               \
    if (ti == jtx) {                                                                      \
      _Pragma("unroll") for (int v = 0; v < 4; ++v) {                                    \
        const double xj = m[ju][v] * xi0;                                                 \
        const double xj1 = fma(-xl10, xj, m[ju + 1][v]) * xi1;                            \
        m[ju][v] = xj;                                                                    \
        m[ju + 1][v] = xj1;                                                               \
        rowbuf[4 * tj + v] = xj;                                                          \
        rowbuf[32 + 4 * tj + v] = xj1;                                                    \
      }                                                                                   \
    }                                                                                     \
    asm volatile("" ::: "memory");                                                        \
    double Lrm0[4], Lrm1[4], X0[4], X1[4];                                                \
    _Pragma("unroll") for (int h = 0; h < 2; ++h) {                                      \
      const double2 r0 = *reinterpret_cast<const double2*>(cb + 4 * ti + 2 * h);          \
      const double2 r1 = *reinterpret_cast<const double2*>(cb + 32 + 4 * ti + 2 * h);     \
      const double2 y0 = *reinterpret_cast<const double2*>(rowbuf + 4 * tj + 2 * h);      \
      const double2 y1 = *reinterpret_cast<const double2*>(rowbuf + 32 + 4 * tj + 2 * h); \
      Lrm0[2 * h] = r0.x; Lrm0[2 * h + 1] = r0.y;                                         \
      Lrm1[2 * h] = r1.x; Lrm1[2 * h + 1] = r1.y;                                         \
      X0[2 * h] = y0.x; X0[2 * h + 1] = y0.y;                                             \
      X1[2 * h] = y1.x; X1[2 * h + 1] = y1.y;                                             \
    }                                                                                     \
    asm volatile("" ::: "memory");                                                        \
    _Pragma("unroll") for (int u = 0; u < 4; ++u) {                                      \
      const bool rw = 4 * ti + u > j + 1;                                                 \
      Lrm0[u] = rw ? -Lrm0[u] : 0.0;                                                      \
      Lrm1[u] = rw ? -Lrm1[u] : 0.0;                                                      \
    }                                                                                     \
    _Pragma("unroll") for (int u = 0; u < 4; ++u)                                        \
      _Pragma("unroll") for (int v = 0; v < 4; ++v)                                      \
        m[u][v] = fma(Lrm1[u], X1[v], fma(Lrm0[u], X0[v], m[u][v]));                      \
  }

  // Iteration (jt, ju): wave 0 runs step 4 jt + ju, wave 1 the step before it.
  // The outer loop is not unrolled (instruction-cache footprint); the inner
  // pair is, so register indices stay compile-time.
#pragma unroll 1
  for (int jt = 0; jt < 8; ++jt) {
    if (wL) BO_L_STEP(0)
    if (wX && jt > 0) BO_X_STEP(jt - 1, 2)
    __syncthreads();
    if (wL) BO_L_STEP(2)
    if (wX) BO_X_STEP(jt, 0)
    __syncthreads();
  }
  if (wX) BO_X_STEP(7, 2)
#undef BO_L_STEP
#undef BO_X_STEP
#pragma unroll
  for (int u = 0; u < 4; ++u)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int i = 4 * ti + u, l = 4 * tj + v;
      if (wL) Sd[i * SP + l] = (l <= i) ? m[u][v] : 0.0;
      if (wX) Dd[i * SP + l] = (l <= i) ? m[u][v] : 0.0;
    }
  return fail;
}

#define BO_TSC(I)                                      \
  do {                                                 \
    if (tsc && tid == 0) tsc[I] = (long long)clock64(); \
  } while (0)

__global__ __launch_bounds__(256) void potrf_block_kernel(double* __restrict__ A, int64_t lda,
                                                          int64_t k0, double* __restrict__ Linv,
                                                          int64_t ldi, int* __restrict__ info,
                                                          long long* __restrict__ tsc) {
  __shared__ __attribute__((aligned(16))) double S[DB * SP];
  __shared__ __attribute__((aligned(16))) double colbuf[2 * 64];
  __shared__ __attribute__((aligned(16))) double pivbuf[8];
  __shared__ __attribute__((aligned(16))) double rowbuf[64];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  BO_TSC(0);

  // Load the lower triangle of the block (upper -> 0): 16-B vector loads,
  // eight in flight per thread before their LDS stores.
#pragma unroll
  for (int e0 = 0; e0 < DB * DB / 2; e0 += 8 * 256) {
    double2 v[8];
#pragma unroll
    for (int w = 0; w < 8; ++w) {
      const int e = e0 + w * 256 + tid;
      v[w] = *reinterpret_cast<const double2*>(A + (k0 + (e >> 6)) * lda + k0 + 2 * (e & 63));
    }
#pragma unroll
    for (int w = 0; w < 8; ++w) {
      const int e = e0 + w * 256 + tid;
      const int r = e >> 6, c = 2 * (e & 63);
      S[r * SP + c] = (c <= r) ? v[w].x : 0.0;
      S[r * SP + c + 1] = (c + 1 <= r) ? v[w].y : 0.0;
    }
  }
  __syncthreads();
  BO_TSC(1);

  // Location of the inverse of diagonal sub-block s inside the free upper blocks.
  auto dinv_at = [](int s) -> int {
    return s < 3 ? (32 * s) * SP + 32 * (s + 1) : 64;  // (s, s+1); s = 3 -> block (0, 2)
  };

  for (int s = 0; s < 4; ++s) {
    const int c = 32 * s;
    // ---- F1: factor + invert the 32 x 32 diagonal sub-block (wave 0) ----
    {
      const int fail = factor32(S + c * SP + c, S + dinv_at(s), colbuf, pivbuf, rowbuf, lane, wave);
      if (wave == 0 && fail && lane == 0) atomicCAS(info, 0, (int)(k0 + c + fail));
    }
    __syncthreads();
    BO_TSC(2 + 3 * s);
    if (s == 3) break;
    // ---- F2: sub-panel below: L[r][c..c+32) = A[r][c..c+32) * Dinv^T ----
    const int nstrip = (DB - c - 32) / 16;
    const double* D = S + dinv_at(s);
    for (int st = wave; st < nstrip; st += 4) {
      double* Ar = S + (c + 32 + 16 * st) * SP + c;
      v4d acc[2] = {v4d_zero(), v4d_zero()};
      mma16<2, 32, true, false, false>(Ar, D, 16 * SP, lane, acc);
      put16(Ar, acc[0], lane, 1.0);
      put16(Ar + 16, acc[1], lane, 1.0);
    }
    __syncthreads();
    BO_TSC(3 + 3 * s);
    // ---- F3: trailing lower triangle -= L_panel L_panel^T (rank 32) ----
    const int T = nstrip;
    const int ntile = T * (T + 1) / 2;
    for (int t = wave; t < ntile; t += 8) {
      const bool two = t + 4 < ntile;
      int tr0, tc0, tr1, tc1;
      tri_index(t, tr0, tc0);
      tri_index(two ? t + 4 : t, tr1, tc1);
      const int r0 = c + 32 + 16 * tr0, q0 = c + 32 + 16 * tc0;
      const int r1 = c + 32 + 16 * tr1, q1 = c + 32 + 16 * tc1;
      v4d a0[1] = {v4d_zero()}, a1[1] = {v4d_zero()};
      // two independent chains interleaved by the unrolled k loops
      mma16<1, 32, true, false, false>(S + r0 * SP + c, S + q0 * SP + c, 0, lane, a0);
      mma16<1, 32, true, false, false>(S + r1 * SP + c, S + q1 * SP + c, 0, lane, a1);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gr = r0 + mfma_row(lane, r), gq = q0 + mfma_col(lane);
        if (gr >= gq) S[gr * SP + gq] -= a0[0][r];
      }
      if (two) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int gr = r1 + mfma_row(lane, r), gq = q1 + mfma_col(lane);
          if (gr >= gq) S[gr * SP + gq] -= a1[0][r];
        }
      }
    }
    __syncthreads();
    BO_TSC(4 + 3 * s);
  }

  // L -> HBM (upper triangle of the block zeroed).
  for (int e = tid; e < DB * DB / 2; e += 256) {
    const int r = e >> 6;
    const int c = 2 * (e & 63);
    double2 v;
    v.x = (c <= r) ? S[r * SP + c] : 0.0;
    v.y = (c + 1 <= r) ? S[r * SP + c + 1] : 0.0;
    *reinterpret_cast<double2*>(A + (k0 + r) * lda + k0 + c) = v;
  }
  __syncthreads();
  // Sub-block inverses into the diagonal 32-blocks (their L is saved above).
  for (int e = tid; e < 4 * 32 * 32; e += 256) {
    const int s = e >> 10, r = (e >> 5) & 31, cc = e & 31;
    S[(32 * s + r) * SP + 32 * s + cc] = S[dinv_at(s) + r * SP + cc];
  }
  __syncthreads();
  BO_TSC(12);

  // ---- merge to 64-blocks: pairs (0,1), (2,3); waves 2p, 2p+1 ----
  {
    const int p = wave >> 1, h = wave & 1;
    const int c1 = 64 * p, c2 = c1 + 32;
    double* L21 = S + c2 * SP + c1;
    double* X11 = S + c1 * SP + c1;
    double* X22 = S + c2 * SP + c2;
    double* Tb = S + c1 * SP + c2;  // free upper block (2p, 2p+1)
    // T = L21 X11: wave h takes output row strip h (16 rows), both column tiles.
    v4d acc[2] = {v4d_zero(), v4d_zero()};
    mma16<2, 32, false, false, false>(L21 + 16 * h * SP, X11, 16, lane, acc);
    put16(Tb + 16 * h * SP, acc[0], lane, 1.0);
    put16(Tb + 16 * h * SP + 16, acc[1], lane, 1.0);
    __syncthreads();
    // X21 = -X22 T  (written over L21, which is no longer read)
    acc[0] = v4d_zero();
    acc[1] = v4d_zero();
    mma16<2, 32, false, false, false>(X22 + 16 * h * SP, Tb, 16, lane, acc);
    put16(L21 + 16 * h * SP, acc[0], lane, -1.0);
    put16(L21 + 16 * h * SP + 16, acc[1], lane, -1.0);
  }
  __syncthreads();
  BO_TSC(13);
  // ---- merge to the 128-block: X21 = -X22 L21 X11 with 64-blocks ----
  {
    // the strictly-upper 32-blocks of X11 / X22 hold T garbage -> masked
    double* L21 = S + 64 * SP;       // rows 64.., cols 0..
    double* X11 = S;                 // rows 0.., cols 0..
    double* X22 = S + 64 * SP + 64;  // rows 64.., cols 64..
    double* Tb = S + 64;             // rows 0..63, cols 64..127 (free upper)
    v4d acc[4] = {v4d_zero(), v4d_zero(), v4d_zero(), v4d_zero()};
    // T = L21 X11: wave w owns output row strip w (16 rows x 64 cols).
    mma16<4, 64, false, false, true>(L21 + 16 * wave * SP, X11, 16, lane, acc);
    __syncthreads();  // all (masked) reads of the upper T-garbage done before overwrite
#pragma unroll
    for (int jt = 0; jt < 4; ++jt) put16(Tb + 16 * wave * SP + 16 * jt, acc[jt], lane, 1.0);
    __syncthreads();
    // X21 = -X22 T
#pragma unroll
    for (int jt = 0; jt < 4; ++jt) acc[jt] = v4d_zero();
    mma16<4, 64, false, true, false>(X22 + 16 * wave * SP, Tb, 16, lane, acc, 16 * wave);
#pragma unroll
    for (int jt = 0; jt < 4; ++jt) put16(L21 + 16 * wave * SP + 16 * jt, acc[jt], lane, -1.0);
  }
  __syncthreads();
  BO_TSC(14);
  // L^{-1} block -> HBM (upper zeroed).
  for (int e = tid; e < DB * DB / 2; e += 256) {
    const int r = e >> 6;
    const int c = 2 * (e & 63);
    double2 v;
    v.x = (c <= r) ? S[r * SP + c] : 0.0;
    v.y = (c + 1 <= r) ? S[r * SP + c + 1] : 0.0;
    *reinterpret_cast<double2*>(Linv + (k0 + r) * ldi + k0 + c) = v;
  }
  BO_TSC(15);
}

}  // namespace

// Factor the 128 x 128 diagonal block at (k0, k0) of A in place and write its
// inverse to Linv at (k0, k0).  lda, ldi even; A, Linv 16-B aligned.
int bo_potrf_block128(double* A, int64_t lda, int64_t k0, double* Linv, int64_t ldi, int* info,
                      hipStream_t st) {
  potrf_block_kernel<<<1, 256, 0, st>>>(A, lda, k0, Linv, ldi, info, nullptr);
  BO_LAUNCH_CHECK();
  return BO_OK;
}

// Phase timing probe (s_memtime ticks at 16 points of one block factorisation
// of the leading 128 x 128 block): load, per sub-panel F1/F2/F3, L store,
// 64-merge, 128-merge, L^{-1} store.
extern "C" int bo_probe_potrf_phases(double* A, int64_t lda, double* Linv, int* info,
                                     long long* tsc, void* stream) {
  potrf_block_kernel<<<1, 256, 0, as_stream(stream)>>>(A, lda, 0, Linv, lda, info, tsc);
  BO_LAUNCH_CHECK();
  return BO_OK;
}
