// Batched exact-GP posterior over q-batches of candidates, fused with the
// kernel-row builder, on the gfx950 fp64 matrix cores.
//
// Reference path (botorch/models/gpytorch.py:405-466 -> [G] exact prediction
// under fast_pred_var, botorch/models/utils/assorted.py:286-298):
//   K*x = k(X*, X_tr)          (b q) x n
//   R   = K*x L^{-T}           (b q) x n      <- the dominant dense contraction
//   mu  = c + K*x alpha = c + R beta,   beta = L^{-1}(y - c)
//   Sigma_b = K**_b - R_b R_b^T         q x q per t-batch b
//
// post_partials_kernel computes R^T tile by tile as an MFMA GEMM
//   R^T[c][i] = sum_k U[k][c] K*x[i][k],   U = L^{-T} (upper triangular)
// with the K*x tile read from K*x^T (built once per call by kxt_build_kernel)
// or, above the memory cap, generated on the fly from the lengthscale-scaled
// inputs, and U streamed from HBM/L2.  Because the R^T tile's
// MFMA accumulators have the test row on the lane and the training column on
// (lane>>4, register), the same accumulator register is simultaneously a
// valid A and B operand of a second MFMA, so  R_b R_b^T  over the tile's 128
// columns is accumulated with 4 MFMAs per 16x16 accumulator and no data
// movement.  Each workgroup writes its 16x16 partial blocks and its partial
// R beta; post_finalize sums them over the column tiles.  R itself is never
// materialised (C3: 268 MB saved per forward).
//
// Small problems (C2: 8 column tiles x 4 row tiles = 32 workgroups for 256
// CUs; a rank's b = 64 share of C3: 256 tiles of very unequal triangular
// k-ranges) run split: a host-built segment table gives every workgroup a list
// of (tile, k-range) segments.  The stream-K plan cuts the concatenated
// k-steps of all tiles (heaviest column tile first, row tiles inner) into one
// equal share per resident slot, so no slot idles behind the longest column
// tile; the uniform plan cuts every tile into chunks of kc_len.  A segment
// that covers its whole tile runs the epilogue itself; the others write their
// partial R^T accumulators to a workspace and post_splitk_reduce_kernel sums
// each tile's chunks in k order (deterministic) and runs the same epilogue.
//
// Test rows are laid out per t-batch: row b*Qp + a, a < q, Qp = q rounded up
// to a power of two <= 16, so every t-batch sits inside one 16-row MFMA tile.
#include "common.h"

#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>
#include <vector>

namespace {

constexpr int PC = 128;   // training columns c per workgroup
constexpr int PI = 128;   // test rows i per workgroup
constexpr int PK = 16;    // k-step
constexpr int PLD = 144;  // LDS row pitch (doubles): 2 x 144 dwords = 32 mod 64 banks
constexpr int DP = 8;     // padded input dimension held in registers
constexpr int kSlots = 512;            // resident workgroups: 256 CUs x 2 (launch bounds)
constexpr int kTileDoubles = 32 * 64;  // one 16-row x 128-column R^T tile
#ifndef KXT_K
#define KXT_K 16  // training points per thread of kxt_build_kernel
#endif

// One kernel value k(x_i, x_k) from scaled coordinates (0 beyond n / invalid rows).
template <int KIND, int ND>
__device__ __forceinline__ double eval_kernel_row(const double (&xi)[ND], const double* __restrict__ Xt,
                                                  int n, int k, double outputscale, bool ivalid) {
  if (k >= n || !ivalid) return 0.0;
  const double* xt = Xt + (int64_t)k * DP;
  double d2 = 0.0;
#pragma unroll
  for (int t = 0; t < ND; ++t) {
    const double df = xi[t] - xt[t];
    d2 = fma(df, df, d2);
  }
#ifdef BO_PROBE_CHEAP_KERNEL  // timing probe only (tools): no exp, wrong values
  return outputscale * d2 * 0.0;  // keeps the distance FMAs, drops the exp
#else
  return outputscale * kernel_from_d2<KIND>(d2);
#endif
}

// Number of k-chunks of column tile ci, and the chunks of all tiles before it
// (the split-k workspace stores only non-empty chunks).
__host__ __device__ __forceinline__ int splitk_chunks(int ci, int n, int kc_len) {
  const int e = ci * PC + PC;
  const int kfull = n < e ? n : e;
  return (kfull + kc_len - 1) / kc_len;
}
__host__ __device__ __forceinline__ int64_t splitk_base(int ci, int n, int kc_len) {
  int64_t s = 0;
  for (int c = 0; c < ci; ++c) s += splitk_chunks(c, n, kc_len);
  return s;
}

// Epilogue of one 16-row tile (rows row0..row0+15) of column tile ci, given
// its R^T accumulators acc[ct] (columns ci*128 + 16 ct + mfma_row, rows row0 +
// mfma_col).  post_store_rt: the R^T store of the gradient path (lanes 0-15
// hold consecutive test rows, so each store writes 128-B row segments).
// post_epilogue: the 16 x 16 block of R R^T over the tile's 128 columns (the
// accumulator register is a valid A and B operand at once: 4 MFMAs per
// accumulator, no data movement) and the partial R beta.
__device__ __forceinline__ void post_store_rt(const v4d (&acc)[8], int ci, int row0, int lane,
                                              int nI, double* __restrict__ Rt) {
  const int c0 = ci * PC;
  const int nrows_pad = nI * PI;
#pragma unroll
  for (int ct = 0; ct < 8; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = c0 + ct * 16 + mfma_row(lane, r);
      Rt[(int64_t)c * nrows_pad + row0 + mfma_col(lane)] = acc[ct][r];
    }
}

__device__ __forceinline__ void post_epilogue(const v4d (&acc)[8], int ci, int row0, int lane,
                                              int n, const double* __restrict__ beta, int nI,
                                              double* __restrict__ Spart,
                                              double* __restrict__ mpart) {
  const int c0 = ci * PC;
  const int nrows16 = nI * (PI / 16);
  const int nrows_pad = nI * PI;
  v4d P = v4d_zero();
#pragma unroll
  for (int ct = 0; ct < 8; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) P = mfma_f64(acc[ct][r], acc[ct][r], P);
  double* sp = Spart + ((int64_t)ci * nrows16 + row0 / 16) * 256;
#pragma unroll
  for (int r = 0; r < 4; ++r) sp[mfma_row(lane, r) * 16 + mfma_col(lane)] = P[r];

  double m = 0.0;
#pragma unroll
  for (int ct = 0; ct < 8; ++ct)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = c0 + ct * 16 + mfma_row(lane, r);
      m = fma(acc[ct][r], (c < n) ? beta[c] : 0.0, m);
    }
  m += __shfl_xor(m, 16);
  m += __shfl_xor(m, 32);
  if (lane < 16) mpart[(int64_t)ci * nrows_pad + row0 + lane] = m;
}

// Fused posterior-backward epilogue of the LOWERK (W^T) tiles (bo_post_w_dx):
// what the dX reduction needs besides the W tile itself.
struct FusedDx {
  const double* dmean;  // B x q (standardised-space scale applied here: ystd)
  const double* dcov;   // B x q x q
  const double* alpha;  // n
  const double* Xq;     // nrows_pad x 8 test rows (scaled)
  const double* Xt;     // n x 8 training rows (scaled)
  double ystd, outputscale;
  int B, q, Qp;
  double* part;         // nC x nrows_pad x 8 partial dX (scaled coordinates)
};

// Member-batched stream-K plans (bo_post_partials_members): the buffers of up
// to 8 models of one shape (a ModelListGP's members); a segment's member is
// bits 24.. of its kbeg word (of the column-tile word in the reduction list).
constexpr int POST_MAXM = 8;
struct PostMembers {
  const double* U[POST_MAXM];
  const double* beta[POST_MAXM];
  const double* Kt[POST_MAXM];
  double* Spart[POST_MAXM];
  double* mpart[POST_MAXM];
  double* Rt[POST_MAXM];
  int nm;  // 0: the kernel's own pointer arguments
};

// The next k-step's U rows are stored to the other LDS stage on every step,
// the last one included (its rows are the current step's, the stage is not
// read again before the next segment's prologue rewrites it behind a
// barrier): with the store behind `if (more)` the compiler sank the U loads
// into that branch, after the step's MFMAs, and every step waited the full
// load latency before its store.
#ifndef BO_POST_PAIRED_REV
#define BO_POST_PAIRED_REV 1
#endif
#ifndef BO_USTORE_ALWAYS
#define BO_USTORE_ALWAYS 1
#endif
template <int KIND, int ND, bool SPLIT, bool CROSS, bool PRE = false, bool LOWERK = false,
          bool FUSEDX = false>
__global__ __launch_bounds__(256, 2) void post_partials_kernel(
    const double* __restrict__ Xq, int nrows, const double* __restrict__ Xt, int n,
    const double* __restrict__ U, int64_t ldu, const double* __restrict__ beta,
    double outputscale, int nC, int nI, double* __restrict__ Spart, double* __restrict__ mpart,
    double* __restrict__ Rt, const int4* __restrict__ segs, const int* __restrict__ wg_off,
    double* __restrict__ work, const double* __restrict__ Qc, int rq, int64_t ldq,
    double* __restrict__ Cx, const double* __restrict__ Kt, int grouped, FusedDx fx = FusedDx{},
    int rt_blk = 0, PostMembers pm = PostMembers{}) {
  // Two LDS stages: while the MFMAs consume stage t, the U rows of step t+1
  // are in flight to registers and this thread evaluates its 8 kernel values
  // of step t+1 between the MFMAs (VALU work hidden under the matrix pipe);
  // one barrier per k-step.
  __shared__ __attribute__((aligned(16))) double Us[2][PK][PLD];
  __shared__ __attribute__((aligned(16))) double Ks[2][PK][PLD];

  const int bid = blockIdx.x;
  int ci = 0, ii = 0, kbeg = 0, kend = 0;
  int ci_long = 0, ci_short = 0;  // paired schedule: the workgroup's two column tiles
  if constexpr (SPLIT) {
    // segments come from the table below
  } else if (grouped == 2) {
    // Paired super-tiles (nC a multiple of 16): the grouped schedule below,
    // but every workgroup runs a LONG column tile and then its SHORT partner
    // of the mirrored column group (cg and nC/8 - 1 - cg), ci_long + ci_short
    // = nC - 1, so every workgroup does nC + 1 k-blocks: the triangular
    // k-ranges even out inside each workgroup instead of across the launch's
    // tail (the heaviest-first grouped order still lost ~7% there).  The 8
    // workgroups sharing a row tile and the 8 sharing a column tile stay on
    // one XCD in both halves.
    const int xcd = bid & 7;
    const int slot = bid >> 3;
    const int t = (slot >> 6) * 8 + xcd;
    const int w = slot & 63;
    const int nIG = nI >> 3;
    const int p = t / nIG;
    if (p >= (nC >> 4)) return;
    ci_long = ((nC >> 3) - 1 - p) * 8 + 7 - (w & 7);
    ci_short = p * 8 + (w & 7);
    ii = (t % nIG) * 8 + (w >> 3);
  } else if (grouped) {
    // Grouped XCD schedule (nC, nI multiples of 8): consecutive block ids are
    // dealt round-robin over the 8 XCDs, so block b and b+8 share an L2.  The
    // 64 slots an XCD fills at once hold one super-tile of 8 column tiles x 8
    // row tiles, which walk their k-ranges together: each k-step's U slice is
    // shared by 8 workgroups and each K*x slice by 8, instead of one U slice by
    // all 64 and 64 private K*x slices (the precomputed K*x^T was re-read from
    // HBM once per column tile).  Super-tiles go heaviest column group first,
    // one per XCD per round.  Placement only affects speed.
    const int xcd = bid & 7;
    const int slot = bid >> 3;
    const int t = (slot >> 6) * 8 + xcd;
    const int w = slot & 63;
    const int nIG = nI >> 3;
    const int cg = (nC >> 3) - 1 - t / nIG;
    if (cg < 0) return;
    ci = cg * 8 + 7 - (w & 7);
    ii = (t % nIG) * 8 + (w >> 3);
    kend = min(n, ci * PC + PC);
  } else {
    // XCD-aware schedule: consecutive block ids are dealt round-robin over the
    // 8 XCDs, so block b and b+8 share an L2.  XCD x takes the column tiles
    // ci with (descending position) % 8 == x, heaviest (largest ci, longest
    // triangular k-range) first, and sweeps all test-row tiles of a column
    // tile back to back: the U panel of that column tile is read once into the
    // XCD's L2 and reused by all of them.  Placement only affects speed.
    const int xcd = bid & 7;
    const int slot = bid >> 3;
    const int jj = slot / nI;
    ii = slot - jj * nI;
    const int pos = jj * 8 + xcd;
    if (pos >= nC) return;
    ci = nC - 1 - pos;
    kend = min(n, ci * PC + PC);
  }
  if (LOWERK && !SPLIT && grouped != 2) {
    // W^T = L^{-T} R^T (bo_post_w): column tile ci reads k in [128 ci, n),
    // so the heaviest tiles are the SMALLEST ci -- mirror the schedule's order.
    ci = nC - 1 - ci;
    kbeg = ci * PC;
    kend = n;
  }
  // Split plans: this workgroup's segments (uniform control flow: every
  // thread walks the same list; the last k-step's barrier frees the LDS
  // stages before the next segment's prologue writes them).
  const double* const U_all = U;
  const double* const beta_all = beta;
  const double* const Kt_all = Kt;
  double* const Spart_all = Spart;
  double* const mpart_all = mpart;
  double* const Rt_all = Rt;
  int sbeg = 0, send = 1;
  if constexpr (SPLIT) {
    sbeg = wg_off[bid];
    send = wg_off[bid + 1];
  } else {
    if (grouped == 2) send = 2;
  }
  for (int sidx = sbeg; sidx < send; ++sidx) {
  int chunk = -1;
  if (!SPLIT && grouped == 2) {
    ci = sidx == 0 ? ci_long : ci_short;
    kbeg = 0;
    kend = min(n, ci * PC + PC);
    if constexpr (LOWERK) {
      ci = nC - 1 - ci;
      kbeg = ci * PC;
      kend = n;
    }
  }
  int mem = 0;
  if constexpr (SPLIT) {
    const int4 sg = segs[sidx];
    ci = sg.x & 0xffff;
    ii = sg.x >> 16;
    kbeg = sg.y & 0xffffff;
    mem = sg.y >> 24;
    kend = sg.z;
    chunk = sg.w;  // -1: the segment covers its whole tile
  }
  // this segment's model (member-batched plans), else the arguments
  const bool memb = SPLIT && pm.nm > 0;
  const double* U = memb ? pm.U[mem] : U_all;
  const double* beta = memb ? pm.beta[mem] : beta_all;
  const double* Kt = memb ? pm.Kt[mem] : Kt_all;
  double* Spart = memb ? pm.Spart[mem] : Spart_all;
  double* mpart = memb ? pm.mpart[mem] : mpart_all;
  double* Rt = memb ? pm.Rt[mem] : Rt_all;
  const int c0 = ci * PC;
  const int i0 = ii * PI;
  const int nsteps = (kend - kbeg + PK - 1) / PK;
  // Paired schedule: every workgroup's long + short k-ranges add up to the
  // same count, so a super-tile's 64 workgroups stay in step (and share each
  // k-slice of K*x^T and U in the XCD's L2) only if both tiles walk relative to
  // the common end of the ranges: k = 0 for the upper ranges [0, kend) -- the
  // long tile ascending, the short one descending and ending at k = 0 at the
  // same moment in every workgroup -- and k = n for the lower (LOWERK) ranges.
  // Ascending short tiles started 8 k-steps apart per column offset and re-read
  // K*x^T from HBM about once per column tile.  Only the summation order
  // differs between the walks.
  const bool rev = BO_POST_PAIRED_REV && !SPLIT && grouped == 2 && ((sidx == 1) != LOWERK);
  const int kfirst = rev ? kbeg + (nsteps - 1) * PK : kbeg;
  const int kdir = rev ? -PK : PK;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;

  // K*x tile role: this thread evaluates test row ti against 8 of the 16
  // training points of each k-step (kh is wave-uniform -> scalar loads of Xt).
  const int ti = tid & (PI - 1);
  const int kh = __builtin_amdgcn_readfirstlane(tid >> 7);
  const bool ivalid = (i0 + ti) < nrows;
  double xi[ND];
#pragma unroll
  for (int t = 0; t < ND; ++t) xi[t] = ivalid ? Xq[(int64_t)(i0 + ti) * DP + t] : 0.0;

  v4d acc[8][2];  // [16-column sub-tile ct][16-row sub-tile it]
#pragma unroll
  for (int a = 0; a < 8; ++a) {
    acc[a][0] = v4d_zero();
    acc[a][1] = v4d_zero();
  }
  // Cross term (CROSS): while K*x streams through LDS, accumulate
  // Cx = Qc K*x^T for rq <= 16 extra rows of Qc (2 MFMAs per 16 of the tile's
  // own) -- the qNEI cross-covariance P_b R^T = Q_b K*x^T without
  // materialising R.  Column tile ci takes the k-block [128 ci, 128 ci + 128),
  // the last steps of its own range, and writes a partial Cx[ci]; spreading
  // the extra MFMAs over all tiles keeps the longest tiles' length unchanged.
  const bool cross = CROSS;
  v4d accx[2] = {v4d_zero(), v4d_zero()};
  double qa[4] = {0.0, 0.0, 0.0, 0.0};
  const bool qrow = CROSS && (lane & 15) < rq;
#define BO_LOAD_Q(K0)                                                              \
  if (cross) {                                                                     \
    _Pragma("unroll") for (int ks = 0; ks < 4; ++ks) {                            \
      const int kk = (K0) + ks * 4 + (lane >> 4);                                  \
      qa[ks] = (qrow && kk < n) ? Qc[(int64_t)(lane & 15) * ldq + kk] : 0.0;       \
    }                                                                              \
  }

  // Per-thread staging registers: 4 x 16 B of U rows, 8 kernel values.
  double u0x, u0y, u1x, u1y, u2x, u2y, u3x, u3y;
  double kv[8];
  const int urow = tid >> 6;          // + 4 p
  const int ucol = c0 + 2 * (tid & 63);
#define BO_LOAD_U(K0)                                                             \
  {                                                                               \
    const double* src = U + (int64_t)((K0) + urow) * ldu + ucol;                  \
    const double2 v0 = *reinterpret_cast<const double2*>(src);                    \
    const double2 v1 = *reinterpret_cast<const double2*>(src + 4 * ldu);          \
    const double2 v2 = *reinterpret_cast<const double2*>(src + 8 * ldu);          \
    const double2 v3 = *reinterpret_cast<const double2*>(src + 12 * ldu);         \
    u0x = v0.x; u0y = v0.y; u1x = v1.x; u1y = v1.y;                               \
    u2x = v2.x; u2y = v2.y; u3x = v3.x; u3y = v3.y;                               \
  }
#define BO_STORE(BUF)                                                             \
  {                                                                               \
    double* dst = &Us[BUF][urow][2 * (tid & 63)];                                 \
    *reinterpret_cast<double2*>(dst) = make_double2(u0x, u0y);                    \
    *reinterpret_cast<double2*>(dst + 4 * PLD) = make_double2(u1x, u1y);          \
    *reinterpret_cast<double2*>(dst + 8 * PLD) = make_double2(u2x, u2y);          \
    *reinterpret_cast<double2*>(dst + 12 * PLD) = make_double2(u3x, u3y);         \
    if (!PRE) {                                                                   \
      _Pragma("unroll") for (int kk = 0; kk < 8; ++kk) Ks[BUF][kh * 8 + kk][ti] = kv[kk]; \
    }                                                                             \
  }

  // K*x value (row ti, training point k): read from the K*x^T that
  // bo_post_kxt built (PRE), or evaluated in registers between the MFMAs.
#define BO_KVAL(K)                                                                         \
  (PRE ? Kt[(int64_t)(K) * (nI * PI) + i0 + ti]                                            \
       : eval_kernel_row<KIND, ND>(xi, Xt, n, (K), outputscale, ivalid))
  // PRE: the MFMA B operands (K*x^T rows k, 16 consecutive test rows per
  // 16 lanes = one 128-B segment) go from L2 straight into registers one
  // k-step ahead (bn -> bc); only U is staged through LDS.
  double bc[2][4], bn[2][4];
  const double* ktw = PRE ? Kt + i0 + wave * 32 + (lane & 15) + (int64_t)(lane >> 4) * (nI * PI)
                          : nullptr;
  // FUSEDX reads R^T in the blocked layout (BO_RT_BLOCKED): one 512-B
  // segment per load instruction
  const double* ktb = FUSEDX ? Kt + (int64_t)((i0 + wave * 32) >> 4) * 256 + lane : nullptr;
#define BO_LOAD_B(K0, DST)                                                          \
  _Pragma("unroll") for (int it = 0; it < 2; ++it)                                 \
    _Pragma("unroll") for (int ks = 0; ks < 4; ++ks)                              \
      DST[it][ks] = FUSEDX ? ktb[((int64_t)((K0) >> 4) * (nI * (PI / 16)) + it) * 256 + ks * 64] \
                           : ktw[(int64_t)((K0) + 4 * ks) * (nI * PI) + it * 16];
  BO_LOAD_U(kfirst);
  if (PRE) {
    BO_LOAD_B(kfirst, bc);
  } else {
#pragma unroll
    for (int kk = 0; kk < 8; ++kk)
      kv[kk] = BO_KVAL(kfirst + kh * 8 + kk);
  }
  BO_STORE(0);
  __syncthreads();
  // One k-step; XMFMA = the cross-term MFMAs (cross workgroups only: a
  // separate copy of the loop keeps the common loop free of branches, which
  // would split its MFMA / kernel-evaluation interleaving).
#define BO_KSTEP(XLOAD, XMFMA)                                                       \
  {                                                                                  \
    const int cur = t & 1;                                                           \
    const bool more = t + 1 < nsteps;                                                \
    const int knext = kfirst + (more ? t + 1 : t) * kdir;                            \
    XLOAD                                                                            \
    BO_LOAD_U(knext);                                                                \
    if (PRE) { BO_LOAD_B(knext, bn); }                                               \
    _Pragma("unroll") for (int ks = 0; ks < PK / 4; ++ks) {                         \
      const int kr = ks * 4 + (lane >> 4);                                           \
      double a[8], b[2];                                                             \
      _Pragma("unroll") for (int ct = 0; ct < 8; ++ct) a[ct] = Us[cur][kr][ct * 16 + (lane & 15)]; \
      _Pragma("unroll") for (int it = 0; it < 2; ++it)                              \
        b[it] = PRE ? bc[it][ks] : Ks[cur][kr][wave * 32 + it * 16 + (lane & 15)];   \
      _Pragma("unroll") for (int ct = 0; ct < 8; ++ct)                              \
        _Pragma("unroll") for (int it = 0; it < 2; ++it)                            \
          acc[ct][it] = FUSEDX ? mfma_f64(b[it], a[ct], acc[ct][it])                \
                               : mfma_f64(a[ct], b[it], acc[ct][it]);                \
      XMFMA                                                                          \
      if (!PRE) {                                                                    \
        kv[2 * ks] = BO_KVAL(knext + kh * 8 + 2 * ks);                              \
        kv[2 * ks + 1] = BO_KVAL(knext + kh * 8 + 2 * ks + 1);                      \
      }                                                                              \
    }                                                                                \
    if (BO_USTORE_ALWAYS || more) BO_STORE(cur ^ 1);                                 \
    if (PRE) {                                                                       \
      _Pragma("unroll") for (int it = 0; it < 2; ++it)                              \
        _Pragma("unroll") for (int ks = 0; ks < 4; ++ks) bc[it][ks] = bn[it][ks];   \
    }                                                                                \
    __syncthreads();                                                                 \
  }
  int t = 0;
  if (cross) {
    // the cross term's steps are those with k >= c0: the last ones ascending,
    // the first ones on a reversed walk
    const int tc = min(nsteps, c0 / PK);
    const int t0 = rev ? 0 : tc, t1 = rev ? nsteps - tc : nsteps;
    for (; t < t0; ++t) BO_KSTEP(, )
    for (; t < t1; ++t)
      BO_KSTEP(BO_LOAD_Q(kfirst + t * kdir),
               accx[0] = mfma_f64(qa[ks], b[0], accx[0]);
               accx[1] = mfma_f64(qa[ks], b[1], accx[1]);)
    for (; t < nsteps; ++t) BO_KSTEP(, )
  } else {
    for (; t < nsteps; ++t) BO_KSTEP(, )
  }
#undef BO_KSTEP
#undef BO_KVAL
#undef BO_LOAD_U
#undef BO_STORE
#undef BO_LOAD_Q
#undef BO_LOAD_B
  if (cross) {
    const int nrows_pad = nI * PI;
#pragma unroll
    for (int it = 0; it < 2; ++it)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = mfma_row(lane, r);
        if (j < rq)
          Cx[((int64_t)ci * rq + j) * nrows_pad + i0 + wave * 32 + it * 16 + mfma_col(lane)] =
              accx[it][r];
      }
  }

  if constexpr (FUSEDX) {
    // The operands were swapped in the k-loop, so acc[ct][it] holds W = R L^-1
    // itself: lane l, register r: test row i = row16 + (l >> 4) + 4 r,
    // training point c = c0 + 16 ct + (l & 15).  Per 16-row tile:
    //   (G W)[a][c] = sum_j G[a][j] W[j][c]: 4 MFMAs per 16 x 16 block, the W
    //   accumulator register being the B operand as it stands (j = (l >> 4) +
    //   4 r) and G (block-diagonal over the tile's t-batches, G_b = s^2
    //   (dcov_b + dcov_b^T)) the A operand;
    //   dK*x[a][c] = s dmean[a] alpha[c] - (G W)[a][c]  (post_backward's D),
    //   dX[a][t] += dK*x[a][c] dk(x_a, x_c)/dx_a,t summed over this tile's 128
    //   training points -> part[ci][a][t] (scaled coordinates; the reduction
    //   over ci, the K** term and the 1 / lengthscale are post_dx_reduce's).
    // W itself is never written.
    const int ncol = lane & 15, grp = lane >> 4;
    const double s2 = fx.ystd * fx.ystd;
    const int nrows_pad = nI * PI;
    // the tile's 128 training rows (+ alpha) and 128 test rows, staged in the
    // (now free) U stages: the epilogue then holds only G, the G W block and
    // the dX sums in registers beside the W accumulators
    double* xc_s = &Us[0][0][0];       // 128 x 8
    double* al_s = xc_s + PC * DP;     // 128
    double* xa_s = al_s + PC;          // 128 x 8
    for (int e = tid; e < PC * DP; e += 256) {
      const int c = c0 + e / DP;
      xc_s[e] = c < n ? fx.Xt[(int64_t)c * DP + (e % DP)] : 0.0;
      xa_s[e] = fx.Xq[(int64_t)i0 * DP + e];
    }
    if (tid < PC) al_s[tid] = (c0 + tid) < n ? fx.alpha[c0 + tid] : 0.0;
    __syncthreads();
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int row16 = i0 + wave * 32 + it * 16;
      const int rl = wave * 32 + it * 16;  // row16 - i0
      double ga[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ra = row16 + ncol, rj = row16 + grp + 4 * r;
        const int ba = ra / fx.Qp, bj = rj / fx.Qp;
        const int aa = ra - ba * fx.Qp, jj = rj - bj * fx.Qp;
        ga[r] = (ba == bj && ba < fx.B && aa < fx.q && jj < fx.q)
                    ? s2 * (fx.dcov[((int64_t)ba * fx.q + aa) * fx.q + jj] +
                            fx.dcov[((int64_t)ba * fx.q + jj) * fx.q + aa])
                    : 0.0;
      }
      double dmu[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int ra = row16 + grp + 4 * r;
        const int b = ra / fx.Qp, aa = ra - b * fx.Qp;
        dmu[r] = (b < fx.B && aa < fx.q) ? fx.ystd * fx.dmean[(int64_t)b * fx.q + aa] : 0.0;
      }
      // two rows of the lane's four at a time (the G W block is recomputed per
      // half: 4 more MFMAs, fewer live registers beside the W accumulators)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        double dx[2][ND];
#pragma unroll
        for (int rr = 0; rr < 2; ++rr)
#pragma unroll
          for (int t = 0; t < ND; ++t) dx[rr][t] = 0.0;
#pragma unroll
        for (int ct = 0; ct < 8; ++ct) {
          v4d gw = v4d_zero();
#pragma unroll
          for (int r = 0; r < 4; ++r) gw = mfma_f64(ga[r], acc[ct][it][r], gw);
          const int cl = ct * 16 + ncol;  // training row within the tile
          const double al = al_s[cl];
          const bool cv = c0 + cl < n;
#pragma unroll
          for (int rr = 0; rr < 2; ++rr) {
            const int r = 2 * h + rr;
            const double D = cv ? fma(dmu[r], al, -gw[r]) : 0.0;
            const double* xa = xa_s + (rl + grp + 4 * r) * DP;
            const double* xc = xc_s + cl * DP;
            double diff[ND];
            double d2 = 0.0;
#pragma unroll
            for (int t = 0; t < ND; ++t) {
              diff[t] = xa[t] - xc[t];
              d2 = fma(diff[t], diff[t], d2);
            }
            const double f = D * dkernel_factor<KIND>(d2, fx.outputscale);
#pragma unroll
            for (int t = 0; t < ND; ++t) dx[rr][t] = fma(f, diff[t], dx[rr][t]);
          }
        }
#pragma unroll
        for (int rr = 0; rr < 2; ++rr)
#pragma unroll
          for (int t = 0; t < ND; ++t) {
            double v = dx[rr][t];
            v += __shfl_xor(v, 1);
            v += __shfl_xor(v, 2);
            v += __shfl_xor(v, 4);
            v += __shfl_xor(v, 8);
            dx[rr][t] = v;
          }
        if (ncol == 0) {
#pragma unroll
          for (int rr = 0; rr < 2; ++rr) {
            double* o = fx.part + ((int64_t)ci * nrows_pad + row16 + grp + 4 * (2 * h + rr)) * DP;
#pragma unroll
            for (int t = 0; t < ND; ++t) o[t] = dx[rr][t];
          }
        }
      }
    }
    __syncthreads();  // the next segment's prologue rewrites the U stages
  } else if (SPLIT && chunk >= 0) {
    // Partial R^T of this chunk: register-major, lane-minor per 16-row tile,
    // so every store instruction writes 512 contiguous bytes.
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      double* w = work + ((int64_t)chunk * (PI / 16) + wave * 2 + it) * kTileDoubles + lane;
#pragma unroll
      for (int ct = 0; ct < 8; ++ct)
#pragma unroll
        for (int r = 0; r < 4; ++r) w[(ct * 4 + r) * 64] = acc[ct][it][r];
    }
  } else {
    // Same epilogue as post_store_rt + post_epilogue, written out over the
    // [ct][it] accumulators (passing sub-arrays costs this kernel spills).
    const int nrows16 = nI * (PI / 16);
    const int nrows_pad = nI * PI;
    if (Rt != nullptr && rt_blk) {
      // BO_RT_BLOCKED: each 16 x 16 block as its accumulator registers stand,
      // register-major, lane-minor -- one 512-B segment per store
#pragma unroll
      for (int ct = 0; ct < 8; ++ct)
#pragma unroll
        for (int it = 0; it < 2; ++it) {
          double* blk = Rt + ((int64_t)((c0 >> 4) + ct) * nrows16 +
                              ((i0 + wave * 32 + it * 16) >> 4)) * 256 + lane;
#pragma unroll
          for (int r = 0; r < 4; ++r) blk[r * 64] = acc[ct][it][r];
        }
    } else if (Rt != nullptr) {
#pragma unroll
      for (int ct = 0; ct < 8; ++ct)
#pragma unroll
        for (int it = 0; it < 2; ++it)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int c = c0 + ct * 16 + mfma_row(lane, r);
            const int i = i0 + wave * 32 + it * 16 + mfma_col(lane);
            Rt[(int64_t)c * nrows_pad + i] = acc[ct][it][r];
          }
    }
    if constexpr (!LOWERK) {  // LOWERK: W^T only
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      v4d P = v4d_zero();
#pragma unroll
      for (int ct = 0; ct < 8; ++ct)
#pragma unroll
        for (int r = 0; r < 4; ++r) P = mfma_f64(acc[ct][it][r], acc[ct][it][r], P);
      const int row0 = i0 + wave * 32 + it * 16;
      double* sp = Spart + ((int64_t)ci * nrows16 + row0 / 16) * 256;
#pragma unroll
      for (int r = 0; r < 4; ++r) sp[mfma_row(lane, r) * 16 + mfma_col(lane)] = P[r];
      double m = 0.0;
#pragma unroll
      for (int ct = 0; ct < 8; ++ct)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = c0 + ct * 16 + mfma_row(lane, r);
          m = fma(acc[ct][it][r], (c < n) ? beta[c] : 0.0, m);
        }
      m += __shfl_xor(m, 16);
      m += __shfl_xor(m, 32);
      if (lane < 16) mpart[(int64_t)ci * nrows_pad + row0 + lane] = m;
    }
    }
  }
  }  // segments
}

// K*x^T once per call: Kt[k][i] = outputscale k(x_i, x_k), zero for k >= n
// or padding rows; np x nrows_pad.  The one-pass grid re-reads each K*x tile
// from L2/HBM for every column tile whose k-range covers it (nC / 2 times on
// average) instead of re-evaluating its exponentials each time: at C3 the
// posterior kernel runs 3.0 ms from precomputed values against 3.7 ms with
// the exponentials between its MFMAs, for 0.08 ms of build.
// RowsFromX (bo_post_kxt_rows): the thread takes its test row straight from
// X (B x q x d) divided by the lengthscale, and the blockIdx.y == 0 threads
// write the padded row layout Xq (prepare_rows_kernel's output) on the way --
// one launch instead of two.
struct RowsFromX {
  const double* X;
  const double* ls;
  int B, q, d, Qp;
  double* Xq_out;
};

// Several models' K*x^T from one X in one launch (bo_post_kxt_rows_members):
// model blockIdx.z's lengthscale, training rows, outputscale and outputs.
struct KxtMembers {
  const double* ls[8];
  const double* Xt[8];
  double os[8];
  double* Xq[8];
  double* Kt[8];
  int nm;  // 0: the kernel's own arguments
};

template <int KIND, int ND, int KK = KXT_K, bool FROMX = false>
__global__ __launch_bounds__(256) void kxt_build_kernel(const double* __restrict__ Xq, int nrows,
                                                        const double* __restrict__ Xt, int n,
                                                        int np, int nrows_pad, double outputscale,
                                                        double* __restrict__ Kt,
                                                        RowsFromX rx = RowsFromX{},
                                                        KxtMembers km = KxtMembers{}) {
  if (km.nm > 0) {
    const int m = blockIdx.z;
    rx.ls = km.ls[m];
    rx.Xq_out = km.Xq[m];
    Xt = km.Xt[m];
    outputscale = km.os[m];
    Kt = km.Kt[m];
  }
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int k0 = blockIdx.y * KK;
  const bool iv = i < nrows;
  double xi[ND];
  if constexpr (FROMX) {
    const int b = i / rx.Qp, a = i - (i / rx.Qp) * rx.Qp;
    const bool real = iv && b < rx.B && a < rx.q;
#pragma unroll
    for (int t = 0; t < ND; ++t)
      xi[t] = (real && t < rx.d) ? rx.X[((int64_t)b * rx.q + a) * rx.d + t] / rx.ls[t] : 0.0;
    if (blockIdx.y == 0 && i < nrows_pad) {
#pragma unroll
      for (int t = 0; t < DP; ++t)
        rx.Xq_out[(int64_t)i * DP + t] =
            (real && t < rx.d) ? rx.X[((int64_t)b * rx.q + a) * rx.d + t] / rx.ls[t] : 0.0;
    }
  } else {
#pragma unroll
    for (int t = 0; t < ND; ++t) xi[t] = iv ? Xq[(int64_t)i * DP + t] : 0.0;
  }
  if (i >= nrows_pad) return;
#pragma unroll 4
  for (int kk = 0; kk < KK; ++kk) {
    const int k = k0 + kk;
    if (k < np) Kt[(int64_t)k * nrows_pad + i] = eval_kernel_row<KIND, ND>(xi, Xt, n, k, outputscale, iv);
  }
}

// Split reduction: one workgroup of four waves per 16-row tile of every tile
// split over several chunks (red: column tile, row tile, first chunk, chunk
// count).  Wave w sums the chunks first + w, first + w + 4, ... in k order
// (two chunks' loads in flight per round), waves 1-3 hand their sums to wave 0
// through LDS, which adds them in wave order and runs the epilogue: four
// times the loads in flight per tile of the one-wave form (C2's longest tiles
// have 16 chunks, each round one memory latency), a fixed summation order.
__global__ __launch_bounds__(256) void post_splitk_reduce_kernel(
    const double* __restrict__ work, const int4* __restrict__ red, int n, int nI,
    const double* __restrict__ beta_all, double* __restrict__ Spart_all,
    double* __restrict__ mpart_all, double* __restrict__ Rt_all, PostMembers pm = PostMembers{}) {
  __shared__ double part[3][32][64];
  const int4 r4 = red[blockIdx.x / (PI / 16)];
  const int sub = blockIdx.x % (PI / 16);
  const int ci = r4.x & 0xffffff, rt = r4.y * (PI / 16) + sub;
  const int mem = r4.x >> 24;
  const bool memb = pm.nm > 0;
  const double* beta = memb ? pm.beta[mem] : beta_all;
  double* Spart = memb ? pm.Spart[mem] : Spart_all;
  double* mpart = memb ? pm.mpart[mem] : mpart_all;
  double* Rt = memb ? pm.Rt[mem] : Rt_all;
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  v4d acc[8];
#pragma unroll
  for (int ct = 0; ct < 8; ++ct) acc[ct] = v4d_zero();
  const int cend = r4.z + r4.w;
  int c = r4.z + wave;
  for (; c + 4 < cend; c += 8) {
    const double* w0 = work + ((int64_t)c * (PI / 16) + sub) * kTileDoubles + lane;
    const double* w1 = w0 + 4 * (PI / 16) * kTileDoubles;
    double v0[32], v1[32];
#pragma unroll
    for (int e = 0; e < 32; ++e) {
      v0[e] = w0[e * 64];
      v1[e] = w1[e * 64];
    }
#pragma unroll
    for (int ct = 0; ct < 8; ++ct)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[ct][r] += v0[ct * 4 + r];
#pragma unroll
    for (int ct = 0; ct < 8; ++ct)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[ct][r] += v1[ct * 4 + r];
  }
  if (c < cend) {
    const double* w = work + ((int64_t)c * (PI / 16) + sub) * kTileDoubles + lane;
#pragma unroll
    for (int ct = 0; ct < 8; ++ct)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[ct][r] += w[(ct * 4 + r) * 64];
  }
  if (wave > 0) {
#pragma unroll
    for (int ct = 0; ct < 8; ++ct)
#pragma unroll
      for (int r = 0; r < 4; ++r) part[wave - 1][ct * 4 + r][lane] = acc[ct][r];
  }
  __syncthreads();
  if (wave != 0) return;
#pragma unroll
  for (int w = 0; w < 3; ++w)
#pragma unroll
    for (int ct = 0; ct < 8; ++ct)
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[ct][r] += part[w][ct * 4 + r][lane];
  if (Rt != nullptr) post_store_rt(acc, ci, rt * 16, lane, nI, Rt);
  if (Spart != nullptr) post_epilogue(acc, ci, rt * 16, lane, n, beta, nI, Spart, mpart);
}

// dX of the fused posterior backward (bo_post_w_dx): the per-column-tile
// partials summed in column-tile order (deterministic), the K** term of the
// q x q blocks (post_backward_kernel's), and the 1 / lengthscale of the
// scaled coordinates.  One workgroup per t-batch, one thread per (a, t).
template <int KIND>
__global__ __launch_bounds__(256) void post_dx_reduce_kernel(
    const double* __restrict__ part, int nC, int nrows_pad, int q, int Qp, int d,
    const double* __restrict__ Xq, const double* __restrict__ dcov,
    const double* __restrict__ ls, double outputscale, double ystd, double* __restrict__ dX) {
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  if (tid >= q * d) return;
  const int a = tid / d, t = tid - (tid / d) * d;
  const int64_t row = (int64_t)b * Qp + a;
  double s = 0.0;
  for (int ci = 0; ci < nC; ++ci) s += part[((int64_t)ci * nrows_pad + row) * DP + t];
  const double s2 = ystd * ystd;
  for (int c = 0; c < q; ++c) {
    if (c == a) continue;
    const int64_t rc = (int64_t)b * Qp + c;
    double d2 = 0.0;
#pragma unroll
    for (int u = 0; u < DP; ++u) {
      const double df = Xq[row * DP + u] - Xq[rc * DP + u];
      d2 = fma(df, df, d2);
    }
    const double g = s2 * (dcov[((int64_t)b * q + a) * q + c] + dcov[((int64_t)b * q + c) * q + a]);
    s = fma(g * dkernel_factor<KIND>(d2, outputscale), Xq[row * DP + t] - Xq[rc * DP + t], s);
  }
  dX[((int64_t)b * q + a) * d + t] = s / ls[t];
}

// Scatter X (B x q x d) into the padded, lengthscale-scaled row layout
// Xq[(b*Qp + a) * DP + t] = X[b][a][t] / ls[t]  (zeros elsewhere).
__global__ void prepare_rows_kernel(const double* __restrict__ X, int B, int q, int d,
                                    int Qp, const double* __restrict__ ls, int nrows_pad,
                                    double* __restrict__ Xq) {
  const int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= (int64_t)nrows_pad * DP) return;
  const int64_t row = idx / DP;
  const int t = (int)(idx % DP);
  const int64_t b = row / Qp;
  const int a = (int)(row % Qp);
  double v = 0.0;
  if (b < B && a < q && t < d) v = X[(b * q + a) * d + t] / ls[t];
  Xq[idx] = v;
}

// ---- small grids: 32 x 32 units over column-tile pairs (round 5) -------------------
// Forward-only posteriors too small for the 128 x 128 tiles (C2: 32 tiles for
// 256 CUs) ran stream-K: k-ranges cut into shares, each cut share writing a
// 128 KB partial R^T tile that post_splitk_reduce_kernel read back (37 MB per
// C2 call, 21% of its kernel time).  Here the unit is 32 test rows x a PAIR of
// 32-column tiles (ct, nct - 1 - ct): the pair's triangular k-ranges add up to
// the same 32 (nct + 1) for every pair, so the units are equal and each covers
// whole k-ranges -- R R^T and R beta are complete per unit and the partials
// are 16 x 16 blocks per pair (nct / 2 of them per 16-row tile), summed by
// qmc_kernel as it sums the column-tile partials.  No split-k workspace and no
// reduction launch.  The 4 waves of a unit take the pair's 16-deep k-steps in
// turn (wave w: steps w, w + 4, ...), each wave its own 32 x 32 accumulators
// fed straight from L2 (U rows and K*x^T rows: 16 lanes = one 128-B segment per
// load), two k-steps of operands in flight; the four partial accumulators are
// summed in LDS in wave order (deterministic), then wave (t, h) runs the
// epilogue of tile t, row half h.
constexpr int SMU = 32;  // test rows and training columns per unit tile
#ifndef SMALL_DEPTH
#define SMALL_DEPTH 2  // k-steps of operands in flight per wave (A/B: -DSMALL_DEPTH=3)
#endif
#ifndef SMALL_PAIRED
#define SMALL_PAIRED 1  // both tiles of a pair over their common k-range (A/B: 0)
#endif
#ifndef SMALL_WAVES
#define SMALL_WAVES 8  // waves per unit, taking the k-steps in turn (round 6 A/B: 8 over 4, C2 eager 44.1 -> 42.4 us)
#endif
constexpr int SMW = SMALL_WAVES;

__device__ __forceinline__ void small_load(const double* __restrict__ U, int64_t ldu,
                                           const double* __restrict__ Kt, int64_t ldk, int kb,
                                           int c0, int r0, int lane, double (&a)[4][2],
                                           double (&b)[4][2]) {
  const int kr = lane >> 4, cl = lane & 15;
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const int64_t k = kb + 4 * ks + kr;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      a[ks][h] = U[k * ldu + c0 + 16 * h + cl];
      b[ks][h] = Kt[k * ldk + r0 + 16 * h + cl];
    }
  }
}

// Steps s = first, first + 4, ... < nsteps of one 32-column tile at c0 into acc.
__device__ __forceinline__ void small_tile(const double* __restrict__ U, int64_t ldu,
                                           const double* __restrict__ Kt, int64_t ldk, int c0,
                                           int r0, int nsteps, int first, int lane,
                                           v4d (&acc)[2][2]) {
  double a0[4][2], b0[4][2], a1[4][2], b1[4][2];
  int s = first;
  if (s < nsteps) small_load(U, ldu, Kt, ldk, PK * s, c0, r0, lane, a0, b0);
  if (s + SMW < nsteps) small_load(U, ldu, Kt, ldk, PK * (s + SMW), c0, r0, lane, a1, b1);
#if SMALL_DEPTH >= 3
  // a third step of operands in flight (BO A/B: SMALL_DEPTH)
  double a2[4][2], b2[4][2];
  if (s + 2 * SMW < nsteps) small_load(U, ldu, Kt, ldk, PK * (s + 2 * SMW), c0, r0, lane, a2, b2);
  for (; s < nsteps; s += SMW) {
    double a3[4][2], b3[4][2];
    const bool more = s + 3 * SMW < nsteps;
    if (more) small_load(U, ldu, Kt, ldk, PK * (s + 3 * SMW), c0, r0, lane, a3, b3);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int hc = 0; hc < 2; ++hc)
#pragma unroll
        for (int hr = 0; hr < 2; ++hr) acc[hc][hr] = mfma_f64(a0[ks][hc], b0[ks][hr], acc[hc][hr]);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        a0[ks][h] = a1[ks][h];
        b0[ks][h] = b1[ks][h];
        a1[ks][h] = a2[ks][h];
        b1[ks][h] = b2[ks][h];
        if (more) {
          a2[ks][h] = a3[ks][h];
          b2[ks][h] = b3[ks][h];
        }
      }
  }
#else
  for (; s < nsteps; s += SMW) {
    double a2[4][2], b2[4][2];
    const bool more = s + 2 * SMW < nsteps;
    if (more) small_load(U, ldu, Kt, ldk, PK * (s + 2 * SMW), c0, r0, lane, a2, b2);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int hc = 0; hc < 2; ++hc)
#pragma unroll
        for (int hr = 0; hr < 2; ++hr) acc[hc][hr] = mfma_f64(a0[ks][hc], b0[ks][hr], acc[hc][hr]);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        a0[ks][h] = a1[ks][h];
        b0[ks][h] = b1[ks][h];
        if (more) {
          a1[ks][h] = a2[ks][h];
          b1[ks][h] = b2[ks][h];
        }
      }
  }
#endif
}

// Both tiles of a pair together over their common k-range (round 5): the
// K*x^T operand (rows k, the unit's 32 test rows) is the same for both
// column tiles there, so it is loaded once for the two tiles' 8 MFMAs per
// 4-deep step -- half the K*x^T traffic of the common range and 8
// independent accumulator chains per wave instead of 4.  Steps s of the
// common range go to wave s % 4 (first = wave), each tile's own sum in
// k order.  Tile B's remaining steps follow in small_tile.
__device__ __forceinline__ void small_load2(const double* __restrict__ U, int64_t ldu,
                                            const double* __restrict__ Kt, int64_t ldk, int kb,
                                            int cA, int cB, int r0, int lane, double (&aA)[4][2],
                                            double (&aB)[4][2], double (&b)[4][2]) {
  const int kr = lane >> 4, cl = lane & 15;
#pragma unroll
  for (int ks = 0; ks < 4; ++ks) {
    const int64_t k = kb + 4 * ks + kr;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      aA[ks][h] = U[k * ldu + cA + 16 * h + cl];
      aB[ks][h] = U[k * ldu + cB + 16 * h + cl];
      b[ks][h] = Kt[k * ldk + r0 + 16 * h + cl];
    }
  }
}

__device__ __forceinline__ void small_pair(const double* __restrict__ U, int64_t ldu,
                                           const double* __restrict__ Kt, int64_t ldk, int cA, int cB,
                                           int r0, int nsteps, int first, int lane,
                                           v4d (&accA)[2][2], v4d (&accB)[2][2]) {
  double aA0[4][2], aB0[4][2], b0[4][2], aA1[4][2], aB1[4][2], b1[4][2];
  int s = first;
  if (s < nsteps) small_load2(U, ldu, Kt, ldk, PK * s, cA, cB, r0, lane, aA0, aB0, b0);
  if (s + SMW < nsteps) small_load2(U, ldu, Kt, ldk, PK * (s + SMW), cA, cB, r0, lane, aA1, aB1, b1);
  for (; s < nsteps; s += SMW) {
    double aA2[4][2], aB2[4][2], b2[4][2];
    const bool more = s + 2 * SMW < nsteps;
    if (more) small_load2(U, ldu, Kt, ldk, PK * (s + 2 * SMW), cA, cB, r0, lane, aA2, aB2, b2);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int hc = 0; hc < 2; ++hc)
#pragma unroll
        for (int hr = 0; hr < 2; ++hr) {
          accA[hc][hr] = mfma_f64(aA0[ks][hc], b0[ks][hr], accA[hc][hr]);
          accB[hc][hr] = mfma_f64(aB0[ks][hc], b0[ks][hr], accB[hc][hr]);
        }
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        aA0[ks][h] = aA1[ks][h];
        aB0[ks][h] = aB1[ks][h];
        b0[ks][h] = b1[ks][h];
        if (more) {
          aA1[ks][h] = aA2[ks][h];
          aB1[ks][h] = aB2[ks][h];
          b1[ks][h] = b2[ks][h];
        }
      }
  }
}

// One launch serves up to 8 models of one shape (the members of a
// ModelListGP: C4's three outputs): block b -> member b / units, unit b % units.
constexpr int SMALL_MAXM = 8;
struct SmallMember {
  const double* Kt;    // np x ldk
  const double* U;     // np x ldu
  const double* beta;  // n
  double* Spart;       // nparts x ldk/16 x 16 x 16
  double* mpart;       // nparts x ldk
  double* Rt;          // np x ldk, row-major R^T (the gradient path), or null
};
struct SmallArgs {
  SmallMember m[SMALL_MAXM];
  int64_t ldk, ldu;
  int n, nct, units;
};

// SMW waves per unit (round 5: 8, two per SIMD -- with one, half of every
// wave's cycles waited on its operand loads at C2, SQ_WAIT_INST_ANY /
// SQ_WAVE_CYCLES = 0.52, MFMA busy 0.27; tools/pmc_small.sh)
__global__ __launch_bounds__(64 * SMW, 8 / SMW) void post_small_kernel(const SmallArgs a) {
  // [source wave][tile][hc][hr][register][lane]: 16 KB per wave
  __shared__ __attribute__((aligned(16))) double red[SMW][2][2][2][4][64];
  const int npair = a.nct >> 1;
  const int mem = blockIdx.x / a.units;
  const int unit = blockIdx.x - mem * a.units;
  const SmallMember& M = a.m[mem];
  const double* __restrict__ Kt = M.Kt;
  const double* __restrict__ U = M.U;
  const int64_t ldk = a.ldk, ldu = a.ldu;
  const int n = a.n, nct = a.nct;
  // consecutive blocks go to different XCDs: the units of one row tile spread
  // over the XCDs and share K*x^T rows through the MALL, each XCD's L2 holds
  // the U columns of its pairs
  const int p = unit % npair, ru = unit / npair;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int r0 = ru * SMU;
  const int ctA = p, ctB = nct - 1 - p;
  v4d acc[2][2][2];  // [tile][hc][hr]
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int hc = 0; hc < 2; ++hc)
#pragma unroll
      for (int hr = 0; hr < 2; ++hr) acc[t][hc][hr] = v4d_zero();
  // tile t: k in [0, 32 (ct + 1)), 2 (ct + 1) steps of 16; the second tile's
  // steps are dealt from the wave after the one that took the first's last step
  const int sA = 2 * (ctA + 1), sB = 2 * (ctB + 1);
#if SMALL_PAIRED
  // the common k-range of both tiles (sA <= sB: ctA < ctB), then tile B's rest
  small_pair(U, ldu, Kt, ldk, SMU * ctA, SMU * ctB, r0, sA, wave, lane, acc[0], acc[1]);
  if (sB > sA) {
    // tile B's steps sA.. continue the round robin: step s on wave s % 4
    const int firstB = sA + ((wave - sA % SMW + SMW) % SMW);
    small_tile(U, ldu, Kt, ldk, SMU * ctB, r0, sB, firstB, lane, acc[1]);
  }
#else
  small_tile(U, ldu, Kt, ldk, SMU * ctA, r0, sA, wave, lane, acc[0]);
  small_tile(U, ldu, Kt, ldk, SMU * ctB, r0, sB, (wave - sA % SMW + SMW) % SMW, lane, acc[1]);
#endif
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int hc = 0; hc < 2; ++hc)
#pragma unroll
      for (int hr = 0; hr < 2; ++hr)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[wave][t][hc][hr][r][lane] = acc[t][hc][hr][r];
  __syncthreads();
  // wave (t, hr) < 4: the unit's R^T block of tile t, row half hr, summed in
  // wave order (waves 4.. only meet the barriers)
  const bool role = wave < 4;
  const int t = (wave >> 1) & 1, hr = wave & 1;
  double v[2][4];
#pragma unroll
  for (int hc = 0; hc < 2; ++hc)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      double x = red[0][t][hc][hr][r][lane];
#pragma unroll
      for (int w = 1; w < SMW; ++w) x += red[w][t][hc][hr][r][lane];
      v[hc][r] = x;
    }
  const int c0 = SMU * (t ? ctB : ctA);
  if (role && M.Rt != nullptr) {  // row-major R^T: 16 lanes = one 128-B row segment
#pragma unroll
    for (int hc = 0; hc < 2; ++hc)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        M.Rt[(int64_t)(c0 + 16 * hc + mfma_row(lane, r)) * ldk + r0 + 16 * hr + mfma_col(lane)] =
            v[hc][r];
  }
  v4d P = v4d_zero();
  double m = 0.0;
#pragma unroll
  for (int hc = 0; hc < 2; ++hc)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      P = mfma_f64(v[hc][r], v[hc][r], P);
      const int c = c0 + 16 * hc + mfma_row(lane, r);
      m = fma(v[hc][r], c < n ? M.beta[c] : 0.0, m);
    }
  m += __shfl_xor(m, 16);
  m += __shfl_xor(m, 32);
  __syncthreads();  // every wave's reads of red done
  double* xP = &red[0][0][0][0][0][0];  // tile 1's blocks handed to tile 0's waves
  double* xm = xP + 2 * 4 * 64;
  if (role && t == 1) {
#pragma unroll
    for (int r = 0; r < 4; ++r) xP[(hr * 4 + r) * 64 + lane] = P[r];
    xm[hr * 64 + lane] = m;
  }
  __syncthreads();
  if (role && t == 0) {
    const int nrows16 = (int)(ldk >> 4);
    const int row16 = (r0 >> 4) + hr;
    double* sp = M.Spart + ((int64_t)p * nrows16 + row16) * 256;
#pragma unroll
    for (int r = 0; r < 4; ++r)
      sp[mfma_row(lane, r) * 16 + mfma_col(lane)] = P[r] + xP[(hr * 4 + r) * 64 + lane];
    if (lane < 16) M.mpart[(int64_t)p * ldk + row16 * 16 + lane] = m + xm[hr * 64 + lane];
  }
}

// Small-grid plan switch: BO_POST_SMALL=0 off, 1 whenever it applies, unset /
// auto: where the 128-tile plan would be stream-K (read once).
static int small_mode() {
  static const int v = [] {
    const char* e = std::getenv("BO_POST_SMALL");
    if (!e) return 2;
    return e[0] == '0' ? 0 : (e[0] == '1' ? 1 : 2);
  }();
  return v;
}

// Paired super-tile schedule switch (default on; BO_POST_PAIRED=0: off), read once.
static bool paired_enabled() {
  static const bool on = [] {
    const char* e = std::getenv("BO_POST_PAIRED");
    return !(e && e[0] == '0');
  }();
  return on;
}

// ---- split plans (host) ----------------------------------------------------------
// Segment (ci | ii << 16, kbeg, kend, chunk or -1) lists per workgroup, and the
// reduction list of the tiles split over several chunks.
struct SplitPlan {
  std::vector<int4> segs, red;
  std::vector<int> wg_off;
  int nchunks = 0, max_segs = 0;
  int64_t max_steps = 0;  // k-steps of the busiest workgroup
};

// Fewest k-steps per stream-K segment (BO_SK_MIN_SHARE, default 4; read once).
// Every cut segment costs a 128 KB partial R^T tile written and read back by
// the reduction, so tiny grids trade parallelism against that traffic.
static int sk_min_share() {
  static const int v = [] {
    const char* e = std::getenv("BO_SK_MIN_SHARE");
    const int x = e ? std::atoi(e) : 4;
    return x >= 1 ? x : 4;
  }();
  return v;
}

// kc_len > 0: uniform chunks of kc_len; kc_len < 0: stream-K over `slots`.
// mode PLAN_POST: posterior tiles, k-range [0, min(n, 128 ci + 128));
// PLAN_AINV: the tiles of A^{-1} = L^{-T} L^{-1} (bo_ainv), column tiles ci >=
// row tiles ii, k-range [128 ci, n); PLAN_LOWER: every tile, k-range
// [128 ci, n) (W^T = L^{-T} R^T, bo_post_w).
enum { PLAN_POST = 0, PLAN_AINV = 1, PLAN_LOWER = 2 };
SplitPlan build_split_plan(int nC, int nI, int n, int kc_len, int slots, int mode = PLAN_POST,
                           int nm = 1) {
  struct Seg { int ci, ii, kb, ke, m = 0; };
  std::vector<std::vector<Seg>> wg;
  auto kfull = [n](int ci) { return std::min(n, ci * PC + PC); };
  const bool ainv = mode == PLAN_AINV;
  // k-range of column tile ci, and the column tiles heaviest first
  auto kbeg_of = [&](int ci) { return mode == PLAN_POST ? 0 : ci * PC; };
  auto kend_of = [&](int ci) { return mode == PLAN_POST ? kfull(ci) : n; };
  auto ci_at = [&](int t) { return mode == PLAN_POST ? nC - 1 - t : t; };
  if (ainv) {
    // Stream-K per row tile (lane ii holds column tiles ci = nC-1 .. ii, the
    // shortest k-ranges first); every lane gets workgroups in proportion to
    // its k-steps so the shares come out equal.
    std::vector<int64_t> lane(nI, 0);
    int64_t total = 0;
    for (int ii = 0; ii < nI; ++ii) {
      for (int ci = ii; ci < nC; ++ci) lane[ii] += ceil_div(n - ci * PC, PK);
      total += lane[ii];
    }
    // sum over lanes of ceil(lane / share) <= total / share + nI <= slots
    const int64_t share = std::max<int64_t>(16, ceil_div(total, std::max(1, slots - nI)));
    for (int ii = 0; ii < nI; ++ii) {
      const size_t base = wg.size();
      int64_t pos = 0;
      for (int ci = nC - 1; ci >= ii; --ci) {
        const int L = (int)ceil_div(n - ci * PC, PK);
        int s0 = 0;
        while (s0 < L) {
          const int64_t j = pos / share;
          if (base + (size_t)j >= wg.size()) wg.resize(base + (size_t)j + 1);
          const int take = (int)std::min<int64_t>(L - s0, (j + 1) * share - pos);
          wg[base + (size_t)j].push_back(Seg{ci, ii, ci * PC + s0 * PK,
                                             std::min(n, ci * PC + (s0 + take) * PK)});
          s0 += take;
          pos += take;
        }
      }
    }
  } else if (kc_len > 0) {
    for (int t = 0; t < nC; ++t) {
      const int ci = ci_at(t);
      for (int kb = kbeg_of(ci); kb < kend_of(ci); kb += kc_len)
        for (int ii = 0; ii < nI; ++ii) wg.push_back({Seg{ci, ii, kb, std::min(kend_of(ci), kb + kc_len)}});
    }
  } else {
    // One lane of workgroups per row tile ii, each lane cutting the same
    // sequence (column tiles heaviest first, k ascending) into equal shares:
    // workgroup j of every lane covers the same k-steps of the same column
    // tiles, so the nI workgroups of one j read the same U slices at the same
    // time; they are placed on one XCD (block b: XCD b % 8, slot b / 8) so
    // those slices are fetched into its L2 once.
    // (member-batched plans: nm x nI lanes, member-major; the lanes of one
    // member's j sit on one XCD as before -- they share that member's U)
    const int lanes = nI * nm;
    int64_t lane_total = 0;
    for (int ci = 0; ci < nC; ++ci) lane_total += ceil_div(kend_of(ci) - kbeg_of(ci), PK);
    const int64_t per_lane = std::max<int64_t>(
        1, std::min<int64_t>(std::max(1, slots / lanes), lane_total / sk_min_share()));
    const int64_t share = ceil_div(lane_total, per_lane);
    const int64_t jn = ceil_div(lane_total, share);  // workgroups used per lane
    // Workgroup of (member m, lane ii, share j).  One model: ((j / 8) nI + ii)
    // 8 + j % 8 -- the nI workgroups of one j on one XCD (block b runs on XCD
    // b % 8), jn padded to a multiple of 8.  Several: that padding would push
    // the grid past the resident slots (C4: 21 shares x 24 lanes -> 576 > 512,
    // a second round for the last workgroups), so the (m, j) groups of nI
    // workgroups are dealt round-robin over the XCDs, each XCD's slots filled
    // in turn.
    std::vector<int64_t> xcd_next(8, 0);
    std::vector<int64_t> group_base((size_t)(nm * jn), 0);
    if (nm > 1)
      for (int64_t g = 0; g < nm * jn; ++g) {
        const int x = (int)(g % 8);
        group_base[(size_t)g] = xcd_next[x];
        xcd_next[x] += nI;
      }
    auto wg_of = [&](int m, int ii, int64_t j) -> int64_t {
      if (nm == 1) return ((j / 8) * lanes + ii) * 8 + (j % 8);
      const int64_t g = m * jn + j;
      return (group_base[(size_t)g] + ii) * 8 + (g % 8);
    };
    int64_t wmax = 0;
    for (int x = 0; x < 8; ++x) wmax = std::max(wmax, xcd_next[x]);
    wg.resize(nm == 1 ? (size_t)(ceil_div(jn, 8) * 8 * lanes) : (size_t)(wmax * 8));
    for (int m = 0; m < nm; ++m)
      for (int ii = 0; ii < nI; ++ii) {
        int64_t pos = 0;
        for (int t = 0; t < nC; ++t) {
          const int ci = ci_at(t), kb0 = kbeg_of(ci), ke0 = kend_of(ci);
          const int L = (int)ceil_div(ke0 - kb0, PK);
          int s0 = 0;
          while (s0 < L) {
            const int64_t j = pos / share;
            const int take = (int)std::min<int64_t>(L - s0, (j + 1) * share - pos);
            const int64_t b = wg_of(m, ii, j);
            wg[(size_t)b].push_back(
                Seg{ci, ii, kb0 + s0 * PK, std::min(ke0, kb0 + (s0 + take) * PK), m});
            s0 += take;
            pos += take;
          }
        }
      }
  }
  // chunk numbers: the segments of every split tile, in k order
  std::map<std::tuple<int, int, int>, std::vector<std::pair<int, int>>> tiles;  // -> (wg, idx), k order
  for (int w = 0; w < (int)wg.size(); ++w)
    for (int j = 0; j < (int)wg[w].size(); ++j)
      tiles[std::make_tuple(wg[w][j].m, wg[w][j].ci, wg[w][j].ii)].push_back({w, j});
  std::vector<std::vector<int>> chunk_of(wg.size());
  for (size_t w = 0; w < wg.size(); ++w) chunk_of[w].assign(wg[w].size(), -1);
  SplitPlan p;
  for (auto& kv : tiles) {
    auto& lst = kv.second;
    std::sort(lst.begin(), lst.end(), [&](const std::pair<int, int>& a, const std::pair<int, int>& b) {
      return wg[a.first][a.second].kb < wg[b.first][b.second].kb;
    });
    if (lst.size() == 1) continue;  // whole tile in one segment: epilogue in place
    p.red.push_back(make_int4(std::get<1>(kv.first) | (std::get<0>(kv.first) << 24),
                              std::get<2>(kv.first), p.nchunks, (int)lst.size()));
    for (auto& e : lst) chunk_of[e.first][e.second] = p.nchunks++;
  }
  p.wg_off.push_back(0);
  for (size_t w = 0; w < wg.size(); ++w) {
    int64_t steps = 0;
    for (size_t j = 0; j < wg[w].size(); ++j) {
      const Seg& g = wg[w][j];
      p.segs.push_back(make_int4(g.ci | (g.ii << 16), g.kb | (g.m << 24), g.ke, chunk_of[w][j]));
      steps += ceil_div(g.ke - g.kb, PK);
    }
    p.wg_off.push_back((int)p.segs.size());
    p.max_segs = std::max(p.max_segs, (int)wg[w].size());
    p.max_steps = std::max(p.max_steps, steps);
  }
  return p;
}

// The chunk count of a plan (its workspace size), memoised: building a plan
// walks every segment of the grid (C2's stream-K plan: ~56 us of host time,
// b = 128 at n = 4096: ~255 us), and the eager operator asks for the
// workspace on every call.
std::mutex g_chunks_mu;
std::map<std::tuple<int, int, int, int, int, int>, int> g_chunks;  // (nC, nI, n, kc, slots, mode|nm)

int plan_chunks(int nC, int nI, int n, int kc_len, int slots, int mode, int nm = 1) {
  const auto key = std::make_tuple(nC, nI, n, kc_len, slots, mode | (nm << 8));
  {
    std::lock_guard<std::mutex> lk(g_chunks_mu);
    auto it = g_chunks.find(key);
    if (it != g_chunks.end()) return it->second;
  }
  const int c = build_split_plan(nC, nI, n, kc_len, slots, mode, nm).nchunks;
  std::lock_guard<std::mutex> lk(g_chunks_mu);
  g_chunks[key] = c;
  return c;
}

struct DevPlan {
  int4 *segs = nullptr, *red = nullptr;
  int* wg_off = nullptr;
  int W = 0, nred = 0, nchunks = 0;
};
std::mutex g_plan_mu;
std::map<std::tuple<int, int, int, int, int, int>, DevPlan> g_plans;  // (dev, nC, nI, n, kc, mode)

int device_plan(int nC, int nI, int n, int kc_len, DevPlan** out, int mode = PLAN_POST, int nm = 1) {
  int dev = 0;
  BO_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_plan_mu);
  DevPlan& dp = g_plans[std::make_tuple(dev, nC, nI, n, kc_len, mode | (nm << 8))];
  if (!dp.wg_off) {
    const SplitPlan p = build_split_plan(nC, nI, n, kc_len, kSlots, mode, nm);
    BO_HIP(hipMalloc(&dp.segs, sizeof(int4) * std::max<size_t>(1, p.segs.size())));
    BO_HIP(hipMalloc(&dp.red, sizeof(int4) * std::max<size_t>(1, p.red.size())));
    BO_HIP(hipMalloc(&dp.wg_off, sizeof(int) * p.wg_off.size()));
    BO_HIP(hipMemcpy(dp.segs, p.segs.data(), sizeof(int4) * p.segs.size(), hipMemcpyHostToDevice));
    if (!p.red.empty())
      BO_HIP(hipMemcpy(dp.red, p.red.data(), sizeof(int4) * p.red.size(), hipMemcpyHostToDevice));
    BO_HIP(hipMemcpy(dp.wg_off, p.wg_off.data(), sizeof(int) * p.wg_off.size(), hipMemcpyHostToDevice));
    dp.W = (int)p.wg_off.size() - 1;
    dp.nred = (int)p.red.size();
    dp.nchunks = p.nchunks;
  }
  *out = &dp;
  return BO_OK;
}

}  // namespace

extern "C" {

int bo_post_geometry(int64_t B, int q, int64_t n, int* Qp, int* nrows_pad, int* nC) {
  BO_CHECK_ARG(q >= 1 && q <= 16, "posterior kernels support 1 <= q <= 16 (got %d)", q);
  int qp = 1;
  while (qp < q) qp *= 2;
  *Qp = qp;
  *nrows_pad = (int)(ceil_div(B * qp, PI) * PI);
  *nC = (int)ceil_div(n, PC);
  return BO_OK;
}

int bo_post_split_plan(int64_t B, int q, int64_t n, int slots, int* kc_len,
                       int64_t* work_elems) {
  int Qp, nrows_pad, nC;
  int s = bo_post_geometry(B, q, n, &Qp, &nrows_pad, &nC);
  if (s) return s;
  const int64_t nI = nrows_pad / PI;
  if (slots <= 0) slots = kSlots;
  *kc_len = 0;
  *work_elems = 0;
  if (nI == 0) return BO_OK;  // no t-batches
  // Stream-K wherever the one-pass grid is imbalance-bound: fewer than four
  // tiles per slot (the heaviest-first rounds cannot even out the triangular
  // k-ranges) and at least one k-step per slot to share.  Measured at n = 4096,
  // q = 16 (tools/time_posterior.py, us, one pass -> stream-K): b = 64
  // 1026 -> 411, 128 1033 -> 693, 256 1552 -> 1261, 512 (2048 tiles) 2403 ->
  // 2432 (the grouped 8 x 8 super-tile schedule keeps its edge there).
  const int64_t steps = nI * splitk_base(nC, (int)n, PK);
  const int64_t tiles = (int64_t)nC * nI;
  // The paired one-pass grid (nC % 16 == 0, equal work per workgroup) already
  // fills the slots from two tiles per slot: b = 256 at n = 4096 measured 1134
  // (paired one pass) vs 1266 us (stream-K) (profiles/r03/time_posterior_paired.json).
  const bool paired = nC % 16 == 0 && nI % 8 == 0 && paired_enabled();
  if (paired && tiles >= 2 * (int64_t)slots) return BO_OK;
  // ... or wherever one tile's k-range alone is long: a one-pass grid of a few
  // row tiles runs its longest column tile as one workgroup's chain of k-steps
  // (b = 1, q = 8, n = 1024: 8 workgroups, 64 steps in a row, ~165 us per
  // call against ~60 us cut into shares)
  const int64_t longest = ceil_div(std::min<int64_t>(n, (int64_t)nC * PC), PK);
  if (tiles < 4 * (int64_t)slots && (steps >= slots || longest > 4 * sk_min_share())) {
    *kc_len = -1;
    *work_elems = (int64_t)plan_chunks(nC, (int)nI, (int)n, -1, slots, PLAN_POST) * PI * PC;
  }
  return BO_OK;
}

// Small-grid posterior plan (post_small_kernel): *nparts = the number of
// pair partials per 16-row tile (np / 64), 0 when the 128-tile plan is kept.
int bo_post_small_plan(int64_t B, int q, int64_t n, int* nparts) {
  int Qp, nrows_pad, nC;
  int s = bo_post_geometry(B, q, n, &Qp, &nrows_pad, &nC);
  if (s) return s;
  *nparts = 0;
  const int mode = small_mode();
  if (mode == 0 || B <= 0) return BO_OK;
  if (mode == 2) {
    int kc = 0;
    int64_t we = 0;
    s = bo_post_split_plan(B, q, n, 0, &kc, &we);
    if (s) return s;
    if (kc == 0) return BO_OK;
    // ... and only small: the 32-row units stream both operands from L2 / the
    // MALL with no reuse across waves, so past ~5e8 MACs the stream-K 128-tile
    // plan wins (forward ms per call, tools/time_small.py, small vs stream-K:
    // n = 1024 q = 8 b = 64 0.041 vs 0.052; n = 2048 q = 8 b = 32 0.055 vs
    // 0.063; n = 4096 q = 16 b = 1 0.095 vs 0.097; but n = 2048 q = 8 b = 128
    // 0.135 vs 0.124, n = 4096 q = 16 b = 64 0.44 vs 0.35)
    const double np_ = (double)nC * PC;
    if ((double)B * Qp * np_ * np_ > 1.2e9) return BO_OK;
  }
  *nparts = (int)(ceil_div(n, PC) * PC / (2 * SMU));
  return BO_OK;
}

// R R^T and R beta partials of the posterior from K*x^T (Kt, np x nrows_pad,
// bo_post_kxt) and U = L^{-T} (np x np, ld ldu) for nm <= 8 models of one
// shape in one launch: Spart[m] nparts x nrows_pad/16 x 16 x 16, mpart[m]
// nparts x nrows_pad (nparts from bo_post_small_plan); Rt[m] (optional, null
// array or entries): R^T row-major, np x nrows_pad.
int bo_post_small_batched(int nm, const double* const* Kt, const double* const* U,
                          const double* const* beta, double* const* Spart, double* const* mpart,
                          double* const* Rt, int64_t B, int q, int64_t n, int64_t ldu,
                          void* stream) {
  int Qp, nrows_pad, nC;
  int s = bo_post_geometry(B, q, n, &Qp, &nrows_pad, &nC);
  if (s) return s;
  BO_CHECK_ARG(nm >= 1 && nm <= SMALL_MAXM, "bo_post_small_batched: %d models (1..%d)", nm,
               SMALL_MAXM);
  BO_CHECK_ARG(Kt && U && beta && Spart && mpart, "bo_post_small_batched: null pointer array");
  const int64_t np = (int64_t)nC * PC;
  BO_CHECK_ARG(ldu >= np, "bo_post_small: ldu %lld < padded order %lld", (long long)ldu,
               (long long)np);
  SmallArgs a{};
  for (int m = 0; m < nm; ++m) {
    BO_CHECK_ARG(Kt[m] && U[m] && beta[m] && Spart[m] && mpart[m], "bo_post_small: null buffer");
    a.m[m] = SmallMember{Kt[m], U[m], beta[m], Spart[m], mpart[m], Rt ? Rt[m] : nullptr};
  }
  if (B == 0) return BO_OK;
  a.ldk = nrows_pad;
  a.ldu = ldu;
  a.n = (int)n;
  a.nct = (int)(np / SMU);
  a.units = (int)(ceil_div(B * Qp, SMU) * (a.nct / 2));
  post_small_kernel<<<(unsigned)(a.units * nm), 64 * SMW, 0, as_stream(stream)>>>(a);
  BO_LAUNCH_CHECK();
  return BO_OK;
}

int bo_post_small(const double* Kt, int64_t B, int q, int64_t n, const double* U, int64_t ldu,
                  const double* beta, double* Spart, double* mpart, double* Rt, void* stream) {
  return bo_post_small_batched(1, &Kt, &U, &beta, &Spart, &mpart, &Rt, B, q, n, ldu, stream);
}

// Member-batched stream-K posterior (nm models of one shape, K*x^T given):
// *work_elems = the shared split-k workspace in doubles, or -1 where the
// one-model plan is not stream-K (the caller then runs one launch per model).
int bo_post_members_work(int nm, int64_t B, int q, int64_t n, int64_t* work_elems) {
  BO_CHECK_ARG(nm >= 1 && nm <= POST_MAXM, "bo_post_members_work: %d models (1..%d)", nm, POST_MAXM);
  int Qp, nrows_pad, nC;
  int s = bo_post_geometry(B, q, n, &Qp, &nrows_pad, &nC);
  if (s) return s;
  int kc = 0;
  int64_t we = 0;
  s = bo_post_split_plan(B, q, n, 0, &kc, &we);
  if (s) return s;
  *work_elems = -1;
  if (kc != -1 || nrows_pad == 0) return BO_OK;
  *work_elems = (int64_t)plan_chunks(nC, nrows_pad / PI, (int)n, -1, kSlots, PLAN_POST, nm) * PI * PC;
  return BO_OK;
}

// R R^T / R beta column-tile partials (and R^T, row-major, where Rt[m] is
// given) of nm models of one shape in ONE stream-K launch over all their
// tiles (+ one reduction launch): Kt[m] np x nrows_pad (bo_post_kxt_rows),
// U[m] np x np (ld ldu), Spart[m] nC x nrows_pad/16 x 16 x 16, mpart[m] nC x
// nrows_pad.  The one-model plan cut C4's 8 x 16 tiles into ~4 shares each
// (a 128 KB partial R^T per share, written and read back); over the three
// members' 24 row lanes the shares are three times as long.
int bo_post_partials_members(int nm, const double* const* Kt, const double* const* U,
                             const double* const* beta, double* const* Spart, double* const* mpart,
                             double* const* Rt, const double* Xq0, int64_t B, int q, int64_t n,
                             int64_t ldu, double* work, void* stream) {
  BO_CHECK_ARG(nm >= 1 && nm <= POST_MAXM, "bo_post_partials_members: %d models (1..%d)", nm,
               POST_MAXM);
  BO_CHECK_ARG(Kt && U && beta && Spart && mpart && Xq0, "bo_post_partials_members: null pointer");
  int Qp, nrows_pad, nC;
  int s = bo_post_geometry(B, q, n, &Qp, &nrows_pad, &nC);
  if (s) return s;
  if (nrows_pad == 0) return BO_OK;
  BO_CHECK_ARG(ldu % 2 == 0 && ldu >= (int64_t)nC * PC, "U leading dim %lld too small", (long long)ldu);
  int64_t we = 0;
  s = bo_post_members_work(nm, B, q, n, &we);
  if (s) return s;
  BO_CHECK_ARG(we >= 0, "bo_post_partials_members: the one-model plan is not stream-K here");
  BO_CHECK_ARG(we == 0 || work != nullptr, "bo_post_partials_members: workspace of %lld doubles needed",
               (long long)we);
  PostMembers pm{};
  pm.nm = nm;
  for (int m = 0; m < nm; ++m) {
    BO_CHECK_ARG(Kt[m] && U[m] && beta[m] && Spart[m] && mpart[m], "bo_post_partials_members: null buffer");
    pm.U[m] = U[m];
    pm.beta[m] = beta[m];
    pm.Kt[m] = Kt[m];
    pm.Spart[m] = Spart[m];
    pm.mpart[m] = mpart[m];
    pm.Rt[m] = Rt ? Rt[m] : nullptr;
  }
  const int nI = nrows_pad / PI;
  DevPlan* plan = nullptr;
  s = device_plan(nC, nI, (int)n, -1, &plan, PLAN_POST, nm);
  if (s) return s;
  hipStream_t st = as_stream(stream);
  // K*x^T given: the kernel kind and input dimension do not enter (PRE)
  post_partials_kernel<BO_RBF, 1, true, false, true><<<(unsigned)plan->W, 256, 0, st>>>(
      Xq0, B * Qp, nullptr, (int)n, U[0], ldu, beta[0], 1.0, nC, nI, Spart[0], mpart[0], nullptr,
      plan->segs, plan->wg_off, work, nullptr, 0, 0, nullptr, Kt[0], 0, FusedDx{}, 0, pm);
  BO_LAUNCH_CHECK();
  if (plan->nred > 0) {
    post_splitk_reduce_kernel<<<(unsigned)(plan->nred * (PI / 16)), 256, 0, st>>>(
        work, plan->red, (int)n, nI, beta[0], Spart[0], mpart[0], nullptr, pm);
    BO_LAUNCH_CHECK();
  }
  return BO_OK;
}

int bo_post_split_work(int64_t B, int q, int64_t n, int kc_len, int64_t* work_elems) {
  int Qp, nrows_pad, nC;
  int s = bo_post_geometry(B, q, n, &Qp, &nrows_pad, &nC);
  if (s) return s;
  *work_elems = 0;
  if (kc_len == 0 || nrows_pad == 0) return BO_OK;
  *work_elems = (int64_t)plan_chunks(nC, nrows_pad / PI, (int)n, kc_len, kSlots, PLAN_POST) * PI * PC;
  return BO_OK;
}

// The segment table of a plan (host only, tests): up to cap segments as 4 ints
// (ci | ii << 16, kbeg, kend, chunk or -1) and up to wcap + 1 workgroup
// offsets; *nseg / *nwg receive the sizes.
int bo_post_split_table(int64_t B, int q, int64_t n, int kc_len, int* segs, int cap, int* wg_off,
                        int wcap, int* nseg, int* nwg) {
  int Qp, nrows_pad, nC;
  int s = bo_post_geometry(B, q, n, &Qp, &nrows_pad, &nC);
  if (s) return s;
  BO_CHECK_ARG(kc_len != 0 && nrows_pad > 0, "bo_post_split_table: a split plan of a non-empty batch");
  const SplitPlan p = build_split_plan(nC, nrows_pad / PI, (int)n, kc_len, kSlots);
  *nseg = (int)p.segs.size();
  *nwg = (int)p.wg_off.size() - 1;
  for (int i = 0; i < *nseg && i < cap; ++i) {
    segs[4 * i] = p.segs[i].x;
    segs[4 * i + 1] = p.segs[i].y;
    segs[4 * i + 2] = p.segs[i].z;
    segs[4 * i + 3] = p.segs[i].w;
  }
  for (int i = 0; i <= *nwg && i <= wcap; ++i) wg_off[i] = p.wg_off[i];
  return BO_OK;
}

int bo_prepare_rows(const double* X, int B, int q, int d, const double* lengthscale,
                    double* Xq, void* stream) {
  BO_CHECK_ARG(d <= DP, "fused posterior kernel supports d <= %d (got %d)", DP, d);
  int Qp, nrows_pad, nC;
  int s = bo_post_geometry(B, q, 1, &Qp, &nrows_pad, &nC);
  if (s) return s;
  const int64_t tot = (int64_t)nrows_pad * DP;
  if (tot == 0) return BO_OK;  // no t-batches
  prepare_rows_kernel<<<(unsigned)ceil_div(tot, 256), 256, 0, as_stream(stream)>>>(
      X, B, q, d, Qp, lengthscale, nrows_pad, Xq);
  BO_LAUNCH_CHECK();
  return BO_OK;
}

int bo_post_kxt(int kind, const double* Xq, int B, int q, int d, const double* Xt_scaled,
                int64_t n, double outputscale, double* Kt, void* stream) {
  BO_CHECK_ARG(kind == BO_RBF || kind == BO_MATERN52, "bad kernel kind %d", kind);
  BO_CHECK_ARG(d >= 1 && d <= DP, "fused posterior kernel supports 1 <= d <= %d", DP);
  int Qp, nrows_pad, nC;
  int s = bo_post_geometry(B, q, n, &Qp, &nrows_pad, &nC);
  if (s) return s;
  if (nrows_pad == 0) return BO_OK;
  const int np = nC * PC;
  const int nrows = B * Qp;
  hipStream_t st = as_stream(stream);
  // 16 training points per thread where the grid fills the chip (C3: 4096
  // workgroups); small grids (C2: 128 workgroups at 16) take 2 per thread
  const bool small = ceil_div(nrows_pad, 256) * ceil_div(np, KXT_K) < 1024;
  const dim3 grid((unsigned)ceil_div(nrows_pad, 256), (unsigned)ceil_div(np, small ? 2 : KXT_K));
#define BO_KXT(KIND, ND)                                                                        \
  if (small)                                                                                    \
    kxt_build_kernel<KIND, ND, 2><<<grid, 256, 0, st>>>(Xq, nrows, Xt_scaled, (int)n, np,       \
                                                        nrows_pad, outputscale, Kt);            \
  else                                                                                          \
    kxt_build_kernel<KIND, ND><<<grid, 256, 0, st>>>(Xq, nrows, Xt_scaled, (int)n, np, nrows_pad, \
                                                     outputscale, Kt)
#define BO_KXT_D(KIND)                       \
  switch (d) {                               \
    case 1: BO_KXT(KIND, 1); break;          \
    case 2: BO_KXT(KIND, 2); break;          \
    case 3: BO_KXT(KIND, 3); break;          \
    case 4: BO_KXT(KIND, 4); break;          \
    case 5: BO_KXT(KIND, 5); break;          \
    case 6: BO_KXT(KIND, 6); break;          \
    default: BO_KXT(KIND, 8); break;         \
  }
  if (kind == BO_RBF) {
    BO_KXT_D(BO_RBF)
  } else {
    BO_KXT_D(BO_MATERN52)
  }
#undef BO_KXT_D
#undef BO_KXT
  BO_LAUNCH_CHECK();
  return BO_OK;
}

// Points per thread of the small-grid K*x^T build: BO_KXT_SMALL (1, 2, 4 or
// 8; default 2), read once -- an A/B knob for tools/time_kxt.py.
static int kxt_small_k() {
  static const int k = [] {
    const char* e = std::getenv("BO_KXT_SMALL");
    const int v = e ? std::atoi(e) : 2;
    return (v == 1 || v == 2 || v == 4 || v == 8) ? v : 2;
  }();
  return k;
}

// bo_post_kxt_rows for nm <= 8 models of one shape and kernel kind (a
// ModelListGP's members) in ONE launch (grid z = model).
int bo_post_kxt_rows_members(int nm, int kind, const double* X, int B, int q, int d,
                             const double* const* lengthscale, const double* const* Xt_scaled,
                             const double* outputscale, int64_t n, double* const* Xq,
                             double* const* Kt, void* stream) {
  BO_CHECK_ARG(nm >= 1 && nm <= 8, "bo_post_kxt_rows_members: %d models (1..8)", nm);
  BO_CHECK_ARG(kind == BO_RBF || kind == BO_MATERN52, "bad kernel kind %d", kind);
  BO_CHECK_ARG(d >= 1 && d <= DP, "fused posterior kernel supports 1 <= d <= %d", DP);
  int Qp, nrows_pad, nC;
  int s = bo_post_geometry(B, q, n, &Qp, &nrows_pad, &nC);
  if (s) return s;
  if (nrows_pad == 0) return BO_OK;
  BO_CHECK_ARG(X && lengthscale && Xt_scaled && outputscale && Xq && Kt,
               "bo_post_kxt_rows_members: null pointer");
  KxtMembers km{};
  km.nm = nm;
  for (int m = 0; m < nm; ++m) {
    BO_CHECK_ARG(lengthscale[m] && Xt_scaled[m] && Xq[m] && Kt[m], "bo_post_kxt_rows_members: null buffer");
    km.ls[m] = lengthscale[m];
    km.Xt[m] = Xt_scaled[m];
    km.os[m] = outputscale[m];
    km.Xq[m] = Xq[m];
    km.Kt[m] = Kt[m];
  }
  const int np = nC * PC;
  const int nrows = B * Qp;
  hipStream_t st = as_stream(stream);
  const RowsFromX rx{X, lengthscale[0], B, q, d, Qp, Xq[0]};
  // points per thread: the one-model rule over the whole (z-stacked) grid
  const bool small = ceil_div(nrows_pad, 256) * ceil_div(np, KXT_K) * nm < 1024;
  const int kk = small ? kxt_small_k() : KXT_K;
  const dim3 grid((unsigned)ceil_div(nrows_pad, 256), (unsigned)ceil_div(np, kk), (unsigned)nm);
#define BO_KXTM_K(KIND, ND, K)                                                                 \
  kxt_build_kernel<KIND, ND, K, true><<<grid, 256, 0, st>>>(nullptr, nrows, Xt_scaled[0], (int)n, \
                                                            np, nrows_pad, outputscale[0], Kt[0], rx, km)
#define BO_KXTM(KIND, ND)                  \
  switch (kk) {                            \
    case 1: BO_KXTM_K(KIND, ND, 1); break; \
    case 2: BO_KXTM_K(KIND, ND, 2); break; \
    case 4: BO_KXTM_K(KIND, ND, 4); break; \
    case 8: BO_KXTM_K(KIND, ND, 8); break; \
    default: BO_KXTM_K(KIND, ND, KXT_K); break; \
  }
#define BO_KXTM_D(KIND)                      \
  switch (d) {                               \
    case 1: BO_KXTM(KIND, 1); break;         \
    case 2: BO_KXTM(KIND, 2); break;         \
    case 3: BO_KXTM(KIND, 3); break;         \
    case 4: BO_KXTM(KIND, 4); break;         \
    case 5: BO_KXTM(KIND, 5); break;         \
    case 6: BO_KXTM(KIND, 6); break;         \
    default: BO_KXTM(KIND, 8); break;        \
  }
  if (kind == BO_RBF) {
    BO_KXTM_D(BO_RBF)
  } else {
    BO_KXTM_D(BO_MATERN52)
  }
#undef BO_KXTM_D
#undef BO_KXTM
#undef BO_KXTM_K
  BO_LAUNCH_CHECK();
  return BO_OK;
}

// bo_prepare_rows + bo_post_kxt in one launch: Xq and K*x^T from X itself.
int bo_post_kxt_rows(int kind, const double* X, int B, int q, int d, const double* lengthscale,
                     const double* Xt_scaled, int64_t n, double outputscale, double* Xq, double* Kt,
                     void* stream) {
  BO_CHECK_ARG(kind == BO_RBF || kind == BO_MATERN52, "bad kernel kind %d", kind);
  BO_CHECK_ARG(d >= 1 && d <= DP, "fused posterior kernel supports 1 <= d <= %d", DP);
  int Qp, nrows_pad, nC;
  int s = bo_post_geometry(B, q, n, &Qp, &nrows_pad, &nC);
  if (s) return s;
  if (nrows_pad == 0) return BO_OK;  // no t-batches (empty outputs may carry null pointers)
  BO_CHECK_ARG(X && lengthscale && Xt_scaled && Xq && Kt, "bo_post_kxt_rows: null buffer");
  const int np = nC * PC;
  const int nrows = B * Qp;
  hipStream_t st = as_stream(stream);
  const RowsFromX rx{X, lengthscale, B, q, d, Qp, Xq};
  const bool small = ceil_div(nrows_pad, 256) * ceil_div(np, KXT_K) < 1024;
  const int kk = small ? kxt_small_k() : KXT_K;
  const dim3 grid((unsigned)ceil_div(nrows_pad, 256), (unsigned)ceil_div(np, kk));
#define BO_KXTR_K(KIND, ND, K)                                                                 \
  kxt_build_kernel<KIND, ND, K, true><<<grid, 256, 0, st>>>(nullptr, nrows, Xt_scaled, (int)n,  \
                                                            np, nrows_pad, outputscale, Kt, rx)
#define BO_KXTR(KIND, ND)                  \
  switch (kk) {                            \
    case 1: BO_KXTR_K(KIND, ND, 1); break; \
    case 2: BO_KXTR_K(KIND, ND, 2); break; \
    case 4: BO_KXTR_K(KIND, ND, 4); break; \
    case 8: BO_KXTR_K(KIND, ND, 8); break; \
    default: BO_KXTR_K(KIND, ND, KXT_K); break; \
  }
#define BO_KXTR_D(KIND)                      \
  switch (d) {                               \
    case 1: BO_KXTR(KIND, 1); break;         \
    case 2: BO_KXTR(KIND, 2); break;         \
    case 3: BO_KXTR(KIND, 3); break;         \
    case 4: BO_KXTR(KIND, 4); break;         \
    case 5: BO_KXTR(KIND, 5); break;         \
    case 6: BO_KXTR(KIND, 6); break;         \
    default: BO_KXTR(KIND, 8); break;        \
  }
  if (kind == BO_RBF) {
    BO_KXTR_D(BO_RBF)
  } else {
    BO_KXTR_D(BO_MATERN52)
  }
#undef BO_KXTR_D
#undef BO_KXTR
#undef BO_KXTR_K
  BO_LAUNCH_CHECK();
  return BO_OK;
}

int bo_post_partials_layout(int kind, const double* Xq, int B, int q, int d,
                            const double* Xt_scaled, int64_t n, const double* U, int64_t ldu,
                            const double* beta, double outputscale, double* Spart, double* mpart,
                            double* Rt, int kc_len, double* work, const double* Qc, int rq,
                            int64_t ldq, double* Cx, const double* Kt, int rt_layout, void* stream);

int bo_post_partials(int kind, const double* Xq, int B, int q, int d,
                     const double* Xt_scaled, int64_t n, const double* U, int64_t ldu, const double* beta,
                     double outputscale, double* Spart, double* mpart, double* Rt,
                     int kc_len, double* work, const double* Qc, int rq, int64_t ldq, double* Cx,
                     const double* Kt, void* stream) {
  return bo_post_partials_layout(kind, Xq, B, q, d, Xt_scaled, n, U, ldu, beta, outputscale, Spart,
                                 mpart, Rt, kc_len, work, Qc, rq, ldq, Cx, Kt, BO_RT_ROWMAJOR,
                                 stream);
}

int bo_post_partials_layout(int kind, const double* Xq, int B, int q, int d,
                            const double* Xt_scaled, int64_t n, const double* U, int64_t ldu,
                            const double* beta, double outputscale, double* Spart, double* mpart,
                            double* Rt, int kc_len, double* work, const double* Qc, int rq,
                            int64_t ldq, double* Cx, const double* Kt, int rt_layout, void* stream) {
  BO_CHECK_ARG(rt_layout == BO_RT_ROWMAJOR || (rt_layout == BO_RT_BLOCKED && kc_len == 0 && !Qc),
               "rt_layout %d: the blocked R^T is stored by one-pass grids without a cross term",
               rt_layout);
  BO_CHECK_ARG(Qc == nullptr || (kc_len == 0 && rq >= 1 && rq <= 16 && ldq >= n && Cx != nullptr),
               "cross term: one-pass only, 1 <= rq <= 16 rows (got %d), ldq >= n, Cx given", rq);
  BO_CHECK_ARG(kind == BO_RBF || kind == BO_MATERN52, "bad kernel kind %d", kind);
  BO_CHECK_ARG(ldu % 2 == 0 && ldu >= ceil_div(n, PC) * PC, "U leading dim %lld too small",
               (long long)ldu);
  if (B == 0) return BO_OK;  // no t-batches: nothing to launch
  const bool pre = Kt != nullptr;
  BO_CHECK_ARG(kc_len == 0 || kc_len == -1 || (kc_len > 0 && kc_len % PK == 0),
               "split chunk %d must be 0, -1 (stream-K) or a positive multiple of %d", kc_len, PK);
  int Qp, nrows_pad, nC;
  int s = bo_post_geometry(B, q, n, &Qp, &nrows_pad, &nC);
  if (s) return s;
  const int nI = nrows_pad / PI;
  const int nrows = B * Qp;
  if (nI == 0) return BO_OK;  // no t-batches: nothing to launch
  BO_CHECK_ARG(d >= 1 && d <= DP, "fused posterior kernel supports 1 <= d <= %d", DP);
  // Grouped 8 x 8 super-tile schedule where the grid divides (C3: 2.68 -> 2.49 ms,
  // HBM 4.5 -> 3.7 GB per launch against the per-column-tile order).
  // Paired where the column groups pair up (nC % 16 == 0; BO_POST_PAIRED=0
  // keeps the unpaired grouped order for A/B timing).
  const int grouped = (kc_len == 0 && nC % 8 == 0 && nI % 8 == 0)
                          ? ((nC % 16 == 0 && paired_enabled()) ? 2 : 1) : 0;
  DevPlan* plan = nullptr;
  if (kc_len != 0) {
    s = device_plan(nC, nI, (int)n, kc_len, &plan);
    if (s) return s;
    BO_CHECK_ARG(plan->nchunks == 0 || work != nullptr, "split plan needs a workspace of %lld doubles",
                 (long long)plan->nchunks * PI * PC);
  }
  const int64_t blocks = kc_len != 0    ? plan->W
                         : grouped == 2 ? 512 * (int64_t)ceil_div((nC / 16) * (nI / 8), 8)
                         : grouped      ? 512 * (int64_t)ceil_div((nC / 8) * (nI / 8), 8)
                                        : 8 * ceil_div(nC, 8) * (int64_t)nI;
  const int4* segs = plan ? plan->segs : nullptr;
  const int* wg_off = plan ? plan->wg_off : nullptr;
  hipStream_t st = as_stream(stream);
  // One instantiation per active input dimension (the padded coordinates
  // beyond d are zero, so fewer distance terms are exact, not approximate).
#define BO_POST_GO(KIND, ND, SPL, CRS, PRE_)                                                \
  post_partials_kernel<KIND, ND, SPL, CRS, PRE_><<<(unsigned)blocks, 256, 0, st>>>(          \
      Xq, nrows, Xt_scaled, (int)n, U, ldu, beta, outputscale, nC, nI, Spart, mpart, Rt,    \
      segs, wg_off, work, Qc, rq, ldq, Cx, Kt, grouped, FusedDx{}, rt_layout == BO_RT_BLOCKED)
#define BO_POST_LAUNCH(KIND, ND)                                                            \
  if (kc_len != 0) {                                                                        \
    if (pre) BO_POST_GO(KIND, ND, true, false, true);                                       \
    else BO_POST_GO(KIND, ND, true, false, false);                                          \
  } else if (Qc != nullptr) {                                                               \
    if (pre) BO_POST_GO(KIND, ND, false, true, true);                                       \
    else BO_POST_GO(KIND, ND, false, true, false);                                          \
  } else {                                                                                  \
    if (pre) BO_POST_GO(KIND, ND, false, false, true);                                      \
    else BO_POST_GO(KIND, ND, false, false, false);                                         \
  }
#define BO_POST_DISPATCH_D(KIND)                   \
  switch (d) {                                     \
    case 1: BO_POST_LAUNCH(KIND, 1); break;        \
    case 2: BO_POST_LAUNCH(KIND, 2); break;        \
    case 3: BO_POST_LAUNCH(KIND, 3); break;        \
    case 4: BO_POST_LAUNCH(KIND, 4); break;        \
    case 5: BO_POST_LAUNCH(KIND, 5); break;        \
    case 6: BO_POST_LAUNCH(KIND, 6); break;        \
    default: BO_POST_LAUNCH(KIND, 8); break;       \
  }
  if (kind == BO_RBF) {
    BO_POST_DISPATCH_D(BO_RBF)
  } else {
    BO_POST_DISPATCH_D(BO_MATERN52)
  }
#undef BO_POST_DISPATCH_D
#undef BO_POST_LAUNCH
#undef BO_POST_GO
  BO_LAUNCH_CHECK();
  if (plan && plan->nred > 0) {
    post_splitk_reduce_kernel<<<(unsigned)(plan->nred * (PI / 16)), 256, 0, st>>>(
        work, plan->red, (int)n, nI, beta, Spart, mpart, Rt);
    BO_LAUNCH_CHECK();
  }
  return BO_OK;
}

int bo_post_w(const double* Linv, int64_t ldl, const double* Rt, int B, int q, int64_t n,
              double* Wt, void* stream) {
  BO_CHECK_ARG(ldl % 2 == 0 && ldl >= ceil_div(n, PC) * PC, "L^{-1} leading dim %lld too small",
               (long long)ldl);
  if (B == 0) return BO_OK;
  int Qp, nrows_pad, nC;
  int s = bo_post_geometry(B, q, n, &Qp, &nrows_pad, &nC);
  if (s) return s;
  const int nI = nrows_pad / PI;
  if (nI == 0) return BO_OK;
  if (nC % 8 != 0 || nI % 8 != 0) {
    bo_set_error("bo_post_w: %d column x %d row tiles do not form 8 x 8 super-tiles", nC, nI);
    return BO_ERR_ARG;
  }
  const int grouped = (nC % 16 == 0 && paired_enabled()) ? 2 : 1;
  const int64_t blocks = grouped == 2 ? 512 * (int64_t)ceil_div((nC / 16) * (nI / 8), 8)
                                      : 512 * (int64_t)ceil_div((nC / 8) * (nI / 8), 8);
  post_partials_kernel<BO_RBF, 1, false, false, true, true><<<(unsigned)blocks, 256, 0,
                                                                as_stream(stream)>>>(
      Rt, 0, Rt, (int)n, Linv, ldl, nullptr, 0.0, nC, nI, nullptr, nullptr, Wt, nullptr,
      nullptr, nullptr, nullptr, 0, 0, nullptr, Rt, grouped);
  BO_LAUNCH_CHECK();
  return BO_OK;
}

// The posterior backward with W = R L^{-1} never stored (bo_post_w_dx): the
// one-pass W tiles of bo_post_w with the dK*x -> dX reduction fused into their
// epilogue, then post_dx_reduce.  Applies where bo_post_w's one-pass grid does
// (no stream-K plan, 8 x 8 super-tiles); elsewhere *work_elems = 0.
int bo_post_w_dx_work(int B, int q, int64_t n, int64_t* work_elems) {
  int Qp, nrows_pad, nC;
  int s = bo_post_geometry(B, q, n, &Qp, &nrows_pad, &nC);
  if (s) return s;
  *work_elems = 0;
  const int nI = nrows_pad / PI;
  int kc = 0;
  int64_t we = 0;
  s = bo_post_w_work(B, q, n, &kc, &we);
  if (s) return s;
  if (nI > 0 && kc == 0 && nC % 8 == 0 && nI % 8 == 0)
    *work_elems = (int64_t)nC * nrows_pad * DP;
  return BO_OK;
}

int bo_post_w_dx(int kind, const double* Linv, int64_t ldl, const double* Rt, int B, int q, int d,
                 int64_t n, const double* Xq, const double* Xt_scaled, const double* alpha,
                 const double* dmean, const double* dcov, const double* lengthscale,
                 double outputscale, double ystd, double* work, double* dX, void* stream) {
  BO_CHECK_ARG(kind == BO_RBF || kind == BO_MATERN52, "bad kernel kind %d", kind);
  BO_CHECK_ARG(d >= 1 && d <= DP && q >= 1 && q <= 16, "bo_post_w_dx: q=%d d=%d", q, d);
  BO_CHECK_ARG(ldl % 2 == 0 && ldl >= ceil_div(n, PC) * PC, "L^{-1} leading dim %lld too small",
               (long long)ldl);
  BO_CHECK_ARG(Linv && Rt && Xq && Xt_scaled && alpha && dmean && dcov && lengthscale && work && dX,
               "bo_post_w_dx: null buffer");
  if (B == 0) return BO_OK;
  int64_t we = 0;
  int s = bo_post_w_dx_work(B, q, n, &we);
  if (s) return s;
  if (we == 0) {
    bo_set_error("bo_post_w_dx: no one-pass W grid at B=%d q=%d n=%lld (use bo_post_w_split)", B,
                 q, (long long)n);
    return BO_ERR_ARG;
  }
  int Qp, nrows_pad, nC;
  s = bo_post_geometry(B, q, n, &Qp, &nrows_pad, &nC);
  if (s) return s;
  const int nI = nrows_pad / PI;
  const int grouped = (nC % 16 == 0 && paired_enabled()) ? 2 : 1;
  const int64_t blocks = grouped == 2 ? 512 * (int64_t)ceil_div((nC / 16) * (nI / 8), 8)
                                      : 512 * (int64_t)ceil_div((nC / 8) * (nI / 8), 8);
  FusedDx fx{dmean, dcov, alpha, Xq, Xt_scaled, ystd, outputscale, B, q, Qp, work};
  hipStream_t st = as_stream(stream);
#define BO_WDX(KIND, ND)                                                                     \
  post_partials_kernel<KIND, ND, false, false, true, true, true><<<(unsigned)blocks, 256, 0, st>>>( \
      Rt, 0, Rt, (int)n, Linv, ldl, nullptr, 0.0, nC, nI, nullptr, nullptr, nullptr, nullptr,   \
      nullptr, nullptr, nullptr, 0, 0, nullptr, Rt, grouped, fx);                             \
  BO_LAUNCH_CHECK();                                                                         \
  post_dx_reduce_kernel<KIND><<<(unsigned)B, 256, 0, st>>>(work, nC, nrows_pad, q, Qp, d, Xq, \
                                                          dcov, lengthscale, outputscale, ystd, dX)
  if (kind == BO_RBF) {
    if (d == 6) { BO_WDX(BO_RBF, 6); } else { BO_WDX(BO_RBF, 8); }
  } else {
    if (d == 6) { BO_WDX(BO_MATERN52, 6); } else { BO_WDX(BO_MATERN52, 8); }
  }
#undef BO_WDX
  BO_LAUNCH_CHECK();
  return BO_OK;
}

// W^T = L^{-T} R^T under a stream-K plan (the k-ranges [128 ci, n) are very
// unequal; grids below four tiles per slot).  *kc_len = -1 and the workspace
// when the plan applies, else 0 (use bo_post_w or a GEMM).
int bo_post_w_work(int B, int q, int64_t n, int* kc_len, int64_t* work_elems) {
  int Qp, nrows_pad, nC;
  int s = bo_post_geometry(B, q, n, &Qp, &nrows_pad, &nC);
  if (s) return s;
  const int nI = nrows_pad / PI;
  *kc_len = 0;
  *work_elems = 0;
  int64_t steps = 0;
  for (int ci = 0; ci < nC; ++ci) steps += (int64_t)nI * ceil_div(n - ci * PC, PK);
  const bool paired = nC % 16 == 0 && nI % 8 == 0 && paired_enabled();  // as bo_post_split_plan
  if (paired && (int64_t)nC * nI >= 2 * (int64_t)kSlots) return BO_OK;
  const int64_t longest = ceil_div(n, PK);  // tile 0's k-range [0, n)
  if (nI > 0 && (int64_t)nC * nI < 4 * (int64_t)kSlots &&
      (steps >= kSlots || longest > 4 * sk_min_share())) {
    *kc_len = -1;
    *work_elems = (int64_t)plan_chunks(nC, nI, (int)n, -1, kSlots, PLAN_LOWER) * PI * PC;
  }
  return BO_OK;
}

int bo_post_w_split(const double* Linv, int64_t ldl, const double* Rt, int B, int q, int64_t n,
                    double* Wt, double* work, void* stream) {
  BO_CHECK_ARG(ldl % 2 == 0 && ldl >= ceil_div(n, PC) * PC, "L^{-1} leading dim %lld too small",
               (long long)ldl);
  if (B == 0) return BO_OK;
  int Qp, nrows_pad, nC;
  int s = bo_post_geometry(B, q, n, &Qp, &nrows_pad, &nC);
  if (s) return s;
  const int nI = nrows_pad / PI;
  if (nI == 0) return BO_OK;
  DevPlan* plan = nullptr;
  s = device_plan(nC, nI, (int)n, -1, &plan, PLAN_LOWER);
  if (s) return s;
  BO_CHECK_ARG(plan->nchunks == 0 || work != nullptr, "bo_post_w_split needs a workspace of %lld doubles",
               (long long)plan->nchunks * PI * PC);
  hipStream_t st = as_stream(stream);
  post_partials_kernel<BO_RBF, 1, true, false, true, true><<<(unsigned)plan->W, 256, 0, st>>>(
      Rt, 0, Rt, (int)n, Linv, ldl, nullptr, 0.0, nC, nI, nullptr, nullptr, Wt, plan->segs,
      plan->wg_off, work, nullptr, 0, 0, nullptr, Rt, 0);
  BO_LAUNCH_CHECK();
  if (plan->nred > 0) {
    post_splitk_reduce_kernel<<<(unsigned)(plan->nred * (PI / 16)), 256, 0, st>>>(
        work, plan->red, (int)n, nI, nullptr, nullptr, nullptr, Wt);
    BO_LAUNCH_CHECK();
  }
  return BO_OK;
}

// W^T = L^{-T} R^T of nm models of one shape in ONE stream-K launch (+ one
// reduction launch): the members' (m, row tile) lanes share the slots as in
// bo_post_partials_members.  *work_elems = the shared workspace in doubles, or
// -1 where the one-model W plan is not stream-K (then one call per model).
int bo_post_w_members_work(int nm, int B, int q, int64_t n, int64_t* work_elems) {
  BO_CHECK_ARG(nm >= 1 && nm <= POST_MAXM, "bo_post_w_members_work: %d models (1..%d)", nm, POST_MAXM);
  int kc = 0;
  int64_t we = 0;
  int s = bo_post_w_work(B, q, n, &kc, &we);
  if (s) return s;
  *work_elems = -1;
  int Qp, nrows_pad, nC;
  s = bo_post_geometry(B, q, n, &Qp, &nrows_pad, &nC);
  if (s) return s;
  if (kc != -1 || nrows_pad == 0) return BO_OK;
  *work_elems = (int64_t)plan_chunks(nC, nrows_pad / PI, (int)n, -1, kSlots, PLAN_LOWER, nm) * PI * PC;
  return BO_OK;
}

int bo_post_w_split_members(int nm, const double* const* Linv, int64_t ldl, const double* const* Rt,
                            int B, int q, int64_t n, double* const* Wt, double* work, void* stream) {
  BO_CHECK_ARG(nm >= 1 && nm <= POST_MAXM, "bo_post_w_split_members: %d models (1..%d)", nm, POST_MAXM);
  BO_CHECK_ARG(Linv && Rt && Wt, "bo_post_w_split_members: null pointer");
  BO_CHECK_ARG(ldl % 2 == 0 && ldl >= ceil_div(n, PC) * PC, "L^{-1} leading dim %lld too small",
               (long long)ldl);
  if (B == 0) return BO_OK;
  int Qp, nrows_pad, nC;
  int s = bo_post_geometry(B, q, n, &Qp, &nrows_pad, &nC);
  if (s) return s;
  const int nI = nrows_pad / PI;
  if (nI == 0) return BO_OK;
  int64_t we = 0;
  s = bo_post_w_members_work(nm, B, q, n, &we);
  if (s) return s;
  BO_CHECK_ARG(we >= 0, "bo_post_w_split_members: the one-model W plan is not stream-K here");
  BO_CHECK_ARG(we == 0 || work != nullptr, "bo_post_w_split_members: workspace of %lld doubles needed",
               (long long)we);
  PostMembers pm{};
  pm.nm = nm;
  for (int m = 0; m < nm; ++m) {
    BO_CHECK_ARG(Linv[m] && Rt[m] && Wt[m], "bo_post_w_split_members: null buffer");
    pm.U[m] = Linv[m];
    pm.Kt[m] = Rt[m];
    pm.Rt[m] = Wt[m];  // beta / Spart / mpart stay null, as in bo_post_w_split
  }
  DevPlan* plan = nullptr;
  s = device_plan(nC, nI, (int)n, -1, &plan, PLAN_LOWER, nm);
  if (s) return s;
  hipStream_t st = as_stream(stream);
  post_partials_kernel<BO_RBF, 1, true, false, true, true><<<(unsigned)plan->W, 256, 0, st>>>(
      Rt[0], 0, Rt[0], (int)n, Linv[0], ldl, nullptr, 0.0, nC, nI, nullptr, nullptr, Wt[0], plan->segs,
      plan->wg_off, work, nullptr, 0, 0, nullptr, Rt[0], 0, FusedDx{}, 0, pm);
  BO_LAUNCH_CHECK();
  if (plan->nred > 0) {
    post_splitk_reduce_kernel<<<(unsigned)(plan->nred * (PI / 16)), 256, 0, st>>>(
        work, plan->red, (int)n, nI, nullptr, nullptr, nullptr, Wt[0], pm);
    BO_LAUNCH_CHECK();
  }
  return BO_OK;
}

// A^{-1} = L^{-T} L^{-1} (lower tiles: Ainv[r][c] for tile row >= tile column)
// from L^{-1} (np x np, ld = np, identity pad): the posterior kernel's lower
// k-range MFMA tiles with L^{-1} as both operands, under a stream-K plan (the
// k-ranges [128 ci, n) are very unequal), partial tiles reduced in k order.
int bo_ainv_work(int64_t n, int64_t* work_elems) {
  const int nC = (int)ceil_div(n, PC);
  *work_elems = (int64_t)plan_chunks(nC, nC, (int)n, -1, kSlots, PLAN_AINV) * PI * PC;
  return BO_OK;
}

int bo_ainv(const double* Linv, int64_t ld, int64_t n, double* Ainv, double* work, void* stream) {
  const int nC = (int)ceil_div(n, PC);
  BO_CHECK_ARG(n > 0 && ld == (int64_t)nC * PC, "bo_ainv: ld %lld must be n rounded up to %d",
               (long long)ld, PC);
  DevPlan* plan = nullptr;
  int s = device_plan(nC, nC, (int)n, -1, &plan, PLAN_AINV);
  if (s) return s;
  BO_CHECK_ARG(plan->nchunks == 0 || work != nullptr, "bo_ainv needs a workspace of %lld doubles",
               (long long)plan->nchunks * PI * PC);
  hipStream_t st = as_stream(stream);
  post_partials_kernel<BO_RBF, 1, true, false, true, true><<<(unsigned)plan->W, 256, 0, st>>>(
      Linv, 0, Linv, (int)n, Linv, ld, nullptr, 0.0, nC, nC, nullptr, nullptr, Ainv, plan->segs,
      plan->wg_off, work, nullptr, 0, 0, nullptr, Linv, 0);
  BO_LAUNCH_CHECK();
  if (plan->nred > 0) {
    post_splitk_reduce_kernel<<<(unsigned)(plan->nred * (PI / 16)), 256, 0, st>>>(
        work, plan->red, (int)n, nC, nullptr, nullptr, nullptr, Ainv);
    BO_LAUNCH_CHECK();
  }
  return BO_OK;
}

}  // extern "C"
