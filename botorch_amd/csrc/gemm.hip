// Batched fp64 GEMM on the gfx950 matrix cores (v_mfma_f64_16x16x4_f64).
//
//   C[b] = alpha * op(A[b]) * op(B[b]) + beta * C[b]      (row-major storage)
//
// Used by the blocked Cholesky (TRSM-as-GEMM against the inverted diagonal
// block, SYRK trailing update restricted to the lower triangle), the
// recursive-doubling triangular inverse, the MLL gradient's K^{-1} = U U^T,
// the qNEI cross-covariance and the generic posterior.  Triangular operands
// skip the all-zero k-range of each tile (flags), which halves the flops of
// L^{-1}-type products that a dense GEMM would spend on zeros.
//
// Workgroup: 256 threads = 4 waves in a 2 x 2 grid; tile BM x BN, k-step 16.
// LDS holds op(A) as As[k][m] and op(B) as Bs[k][n] in two stages; each k-step
// issues the next stage's global loads (16-B vector loads along the
// contiguous dimension of the operand) before the MFMAs of the current stage
// and writes them to the other stage after, so there is ONE barrier per
// k-step and the HBM/L2 latency hides under 64 (128-tile) or 16 (64-tile)
// MFMAs per wave.  Row pitch BM + 16 doubles puts the four 16-lane groups of
// an operand read on alternating bank halves.
//
// Grid: a 1-D tile list (lower-triangle tiles only under BO_GEMM_LOWER_C),
// dealt XCD-major: hardware hands consecutive block ids round-robin to the 8
// XCDs, so block b runs on XCD b % 8; tile t = (b % 8) * per_xcd + b / 8 gives
// each XCD a contiguous run of tiles that share A row panels in its own L2.
#include "common.h"

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include "gemm.h"

namespace {

constexpr int BK = 16;
constexpr int PAD = 16;

struct TileMap {
  int tilesN;      // tiles along n
  int ntiles;      // tiles per batch member
  int per_xcd;     // ceil(ntiles / 8)
  int lower;       // enumerate lower-triangle tiles only (BM == BN)
};

__device__ __forceinline__ void tile_coords(const TileMap& tm, int t, int& ti, int& tj) {
  if (tm.lower) {
    // t -> (ti, tj), tj <= ti, row-major over the lower triangle
    int r = (int)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
    while ((r + 1) * (r + 2) / 2 <= t) ++r;
    while (r * (r + 1) / 2 > t) --r;
    ti = r;
    tj = t - r * (r + 1) / 2;
  } else {
    ti = t / tm.tilesN;
    tj = t - ti * tm.tilesN;
  }
}

// Stage loader for one operand.  KCONTIG: element (r, k) at P[r * ld + k]
// (k contiguous), else at P[k * ld + r] (r contiguous).  R = tile extent along
// the non-k dimension.  Each thread moves NV pairs of doubles per k-step.
template <int R, bool KCONTIG>
struct Stage {
  static constexpr int NV = R * BK / 512;  // double2 per thread
  double2 v[NV];

  __device__ __forceinline__ void load(const double* __restrict__ P, int64_t ld, int r0, int k0,
                                       int Rlim, int Klim, bool vec_ok, int tid) {
#pragma unroll
    for (int p = 0; p < NV; ++p) {
      const int e = tid + p * 256;
      int r, k;
      if (KCONTIG) { k = 2 * (e % (BK / 2)); r = e / (BK / 2); }
      else         { r = 2 * (e % (R / 2));  k = e / (R / 2); }
      const int gr = r0 + r, gk = k0 + k;
      double x = 0.0, y = 0.0;
      if (KCONTIG) {
        const double* src = P + (int64_t)gr * ld + gk;
        if (gr < Rlim) {
          if (vec_ok && gk + 1 < Klim) {
            const double2 t = *reinterpret_cast<const double2*>(src);
            x = t.x; y = t.y;
          } else {
            if (gk < Klim) x = src[0];
            if (gk + 1 < Klim) y = src[1];
          }
        }
      } else {
        const double* src = P + (int64_t)gk * ld + gr;
        if (gk < Klim) {
          if (vec_ok && gr + 1 < Rlim) {
            const double2 t = *reinterpret_cast<const double2*>(src);
            x = t.x; y = t.y;
          } else {
            if (gr < Rlim) x = src[0];
            if (gr + 1 < Rlim) y = src[1];
          }
        }
      }
      v[p] = make_double2(x, y);
    }
  }

  __device__ __forceinline__ void store(double (*S)[R + PAD], int tid) const {
#pragma unroll
    for (int p = 0; p < NV; ++p) {
      const int e = tid + p * 256;
      if (KCONTIG) {
        const int k = 2 * (e % (BK / 2)), r = e / (BK / 2);
        S[k][r] = v[p].x;
        S[k + 1][r] = v[p].y;
      } else {
        const int r = 2 * (e % (R / 2)), k = e / (R / 2);
        *reinterpret_cast<double2*>(&S[k][r]) = v[p];
      }
    }
  }
};

template <int BM, int BN, bool TA, bool TB, int MINB>
__global__ __launch_bounds__(256, MINB) void gemm_f64_kernel(
    int M, int N, int K, double alpha, const double* __restrict__ A, int64_t lda,
    int64_t sA, const double* __restrict__ B, int64_t ldb, int64_t sB, double beta,
    double* __restrict__ C, int64_t ldc, int64_t sC, int flags, TileMap tm, int vecA,
    int vecB, int ksplit = 1, double* __restrict__ work = nullptr) {
  constexpr int TM = BM / 32;  // MFMA tiles per wave along m (2 x 2 waves)
  constexpr int TN = BN / 32;
  __shared__ __attribute__((aligned(16))) double As[2][BK][BM + PAD];
  __shared__ __attribute__((aligned(16))) double Bs[2][BK][BN + PAD];

  const int b = blockIdx.x;
  const int t = (b & 7) * tm.per_xcd + (b >> 3);
  if (t >= tm.ntiles) return;
  int ti, tj;
  tile_coords(tm, t, ti, tj);
  const int m0 = ti * BM, n0 = tj * BN;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = (wave >> 1) * (BM / 2);
  const int wn = (wave & 1) * (BN / 2);
  const int64_t bz = blockIdx.y;
  A += bz * sA;
  B += bz * sB;
  C += bz * sC;

  // k-range restricted by triangular operands (zero regions are skipped).
  int kbeg = 0, kend = K;
  if (flags & BO_GEMM_A_LOWER) kend = min(kend, m0 + BM);  // op(A)[m][k] = 0 for k > m
  if (flags & BO_GEMM_B_UPPER) kend = min(kend, n0 + BN);  // op(B)[k][n] = 0 for k > n
  if (flags & BO_GEMM_A_UPPER) kbeg = max(kbeg, m0);       // op(A)[m][k] = 0 for k < m
  if (flags & BO_GEMM_B_LOWER) kbeg = max(kbeg, n0);       // op(B)[k][n] = 0 for k < n
  kbeg = (kbeg / BK) * BK;
  int nsteps = kend > kbeg ? (kend - kbeg + BK - 1) / BK : 0;
  if (ksplit > 1) {  // split-k: chunk blockIdx.z of the k-steps (partials to work)
    const int per = (nsteps + ksplit - 1) / ksplit;
    const int s0 = min(nsteps, (int)blockIdx.z * per);
    const int s1 = min(nsteps, s0 + per);
    kbeg += s0 * BK;
    nsteps = s1 - s0;
  }

  v4d acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = v4d_zero();

  // op(A) = A (row m, col k) stored [M][K] -> k contiguous unless TA.
  Stage<BM, !TA> sa;
  // op(B)[k][n]: stored [K][N] (n contiguous) unless TB ([N][K], k contiguous).
  Stage<BN, TB> sb;

  if (nsteps > 0) {
    sa.load(A, lda, m0, kbeg, M, K, vecA, tid);
    sb.load(B, ldb, n0, kbeg, N, K, vecB, tid);
    sa.store(As[0], tid);
    sb.store(Bs[0], tid);
  }
  __syncthreads();
  for (int s = 0; s < nsteps; ++s) {
    const int cur = s & 1;
    const bool more = s + 1 < nsteps;
    if (more) {
      const int kn = kbeg + (s + 1) * BK;
      sa.load(A, lda, m0, kn, M, K, vecA, tid);
      sb.load(B, ldb, n0, kn, N, K, vecB, tid);
    }
#pragma unroll
    for (int ks = 0; ks < BK / 4; ++ks) {
      const int kr = ks * 4 + (lane >> 4);
      double a[TM], bb[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = As[cur][kr][wm + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < TN; ++j) bb[j] = Bs[cur][kr][wn + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma_f64(a[i], bb[j], acc[i][j]);
    }
    if (more) {
      sa.store(As[cur ^ 1], tid);
      sb.store(Bs[cur ^ 1], tid);
    }
    __syncthreads();
  }

  if (ksplit > 1) {  // the chunk's raw partial (every element: empty chunks write zeros)
    double* W = work + ((int64_t)blockIdx.z * gridDim.y + bz) * (int64_t)M * N;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int gm = m0 + wm + i * 16 + mfma_row(lane, r);
          const int gn = n0 + wn + j * 16 + mfma_col(lane);
          if (gm < M && gn < N) W[(int64_t)gm * N + gn] = acc[i][j][r];
        }
    return;
  }
  // Epilogue.  The beta * C reads of one 16-row strip are all issued before
  // any of its stores (a load after a store to the same array cannot be
  // hoisted by the compiler, which would otherwise serialise one HBM round
  // trip per element).
  const bool lower = flags & BO_GEMM_LOWER_C;
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    double cv[TN][4];
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gm = m0 + wm + i * 16 + mfma_row(lane, r);
        const int gn = n0 + wn + j * 16 + mfma_col(lane);
        const bool ok = gm < M && gn < N && (!lower || gm >= gn);
        cv[j][r] = (ok && beta != 0.0) ? C[(int64_t)gm * ldc + gn] : 0.0;
      }
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int gm = m0 + wm + i * 16 + mfma_row(lane, r);
        const int gn = n0 + wn + j * 16 + mfma_col(lane);
        if (gm < M && gn < N && (!lower || gm >= gn))
          C[(int64_t)gm * ldc + gn] = fma(beta, cv[j][r], alpha * acc[i][j][r]);
      }
  }
}

inline bool aligned16(const void* p) { return ((uintptr_t)p & 15) == 0; }


// C = alpha * (sum of the ksplit chunk partials, in chunk order) + beta * C.
__global__ __launch_bounds__(256) void gemm_splitk_reduce_kernel(int M, int N, int batch, int ksplit,
                                                                 const double* __restrict__ work,
                                                                 double alpha, double beta,
                                                                 double* __restrict__ C, int64_t ldc,
                                                                 int64_t sC) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t mn = (int64_t)M * N;
  if (e >= mn * batch) return;
  const int64_t z = e / mn, r = e - z * mn;
  const int m = (int)(r / N), n = (int)(r - (int64_t)m * N);
  double acc = 0.0;
  for (int s = 0; s < ksplit; ++s) acc += work[((int64_t)s * batch + z) * mn + r];
  double* c = C + z * sC + (int64_t)m * ldc + n;
  *c = beta != 0.0 ? fma(beta, *c, alpha * acc) : alpha * acc;
}

template <int BM, int BN, int MINB>
int launch_gemm(bool ta, bool tb, int M, int N, int K, double alpha, const double* A,
                int64_t lda, int64_t sA, const double* B, int64_t ldb, int64_t sB,
                double beta, double* C, int64_t ldc, int64_t sC, int batch, int flags,
                hipStream_t st, int ksplit = 1) {
  TileMap tm;
  const int tilesM = (int)ceil_div(M, BM);
  tm.tilesN = (int)ceil_div(N, BN);
  tm.lower = (BM == BN) && (flags & BO_GEMM_LOWER_C) ? 1 : 0;
  if (tm.lower) {
    // tiles with ti >= tj cover the lower triangle (N beyond M never needed)
    const int tn = tm.tilesN < tilesM ? tm.tilesN : tilesM;
    // rows ti < tilesM, cols tj <= min(ti, tn - 1): count = full triangle of tn
    // rows plus (tilesM - tn) full rows of tn tiles.
    if (tn == tilesM) {
      tm.ntiles = tilesM * (tilesM + 1) / 2;
    } else {
      tm.lower = 0;  // ragged (N < M) lower request: plain grid, masked epilogue
      tm.ntiles = tilesM * tm.tilesN;
    }
  } else {
    tm.ntiles = tilesM * tm.tilesN;
  }
  tm.per_xcd = (int)ceil_div(tm.ntiles, 8);
  // vector loads need 16-B aligned rows: base aligned, even leading dim and
  // even batch stride
  const int vecA = aligned16(A) && lda % 2 == 0 && (batch == 1 || sA % 2 == 0);
  const int vecB = aligned16(B) && ldb % 2 == 0 && (batch == 1 || sB % 2 == 0);
  double* work = nullptr;
  if (ksplit > 1) {
    keep_pool_warm();
    BO_HIP(hipMallocAsync(reinterpret_cast<void**>(&work),
                          sizeof(double) * (size_t)ksplit * batch * M * N, st));
  }
  dim3 grid((unsigned)(8 * tm.per_xcd), (unsigned)batch, (unsigned)ksplit);
#define BO_GEMM_GO(TA_, TB_)                                                                 \
  gemm_f64_kernel<BM, BN, TA_, TB_, MINB><<<grid, 256, 0, st>>>(                            \
      M, N, K, alpha, A, lda, sA, B, ldb, sB, beta, C, ldc, sC, flags, tm, vecA, vecB,      \
      ksplit, work)
  if (ta && tb) BO_GEMM_GO(true, true);
  else if (ta) BO_GEMM_GO(true, false);
  else if (tb) BO_GEMM_GO(false, true);
  else BO_GEMM_GO(false, false);
#undef BO_GEMM_GO
  BO_LAUNCH_CHECK();
  if (ksplit > 1) {
    const int64_t tot = (int64_t)batch * M * N;
    gemm_splitk_reduce_kernel<<<(unsigned)ceil_div(tot, 256), 256, 0, st>>>(M, N, batch, ksplit, work,
                                                                         alpha, beta, C, ldc, sC);
    BO_LAUNCH_CHECK();
    BO_HIP(hipFreeAsync(work, st));
  }
  return BO_OK;
}

}  // namespace

namespace {

// Narrow products (N <= 16 with M <= 16 or a short k-range, e.g. the q x q
// blocks R_b R_b^T of the SAAS ensemble -- 1024 members of 4 x 256 x 4 -- or
// the reparameterised samples Z L_b^T, 256 x 4 x 4 per member): one wave per
// (batch member, 16-row block), one 16 x 16 MFMA accumulator, k in steps of 4
// (a 128 x 128 tile would spend orders of magnitude more flops on padding).
// Structure flags mask the operands exactly as the tiled kernel's k-range
// skipping does.
__global__ __launch_bounds__(256) void gemm_small_kernel(
    int M, int N, int K, double alpha, const double* __restrict__ A, int64_t lda, int64_t sA,
    int ta, const double* __restrict__ B, int64_t ldb, int64_t sB, int tb, double beta,
    double* __restrict__ C, int64_t ldc, int64_t sC, int batch, int flags) {
  const int lane = threadIdx.x & 63;
  const int mblocks = (M + 15) >> 4;
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (w >= (int64_t)batch * mblocks) return;
  const int64_t z = w / mblocks;
  const int m0 = (int)(w - z * mblocks) * 16;
  const double* Az = A + z * sA;
  const double* Bz = B + z * sB;
  const int r16 = lane & 15;  // A fragment row m0 + r16 / B fragment column j
  const int kq = lane >> 4;
  const int ia = m0 + r16;
  v4d acc = v4d_zero();
  for (int k0 = 0; k0 < K; k0 += 4) {
    const int k = k0 + kq;
    double a = 0.0, b = 0.0;
    if (ia < M && k < K) {
      a = ta ? Az[(int64_t)k * lda + ia] : Az[(int64_t)ia * lda + k];
      if (((flags & BO_GEMM_A_LOWER) && k > ia) || ((flags & BO_GEMM_A_UPPER) && k < ia)) a = 0.0;
    }
    if (r16 < N && k < K) {
      b = tb ? Bz[(int64_t)r16 * ldb + k] : Bz[(int64_t)k * ldb + r16];
      if (((flags & BO_GEMM_B_UPPER) && k > r16) || ((flags & BO_GEMM_B_LOWER) && k < r16)) b = 0.0;
    }
    acc = mfma_f64(a, b, acc);
  }
  double* Cz = C + z * sC;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = m0 + mfma_row(lane, r), j = mfma_col(lane);
    if (i < M && j < N && (!(flags & BO_GEMM_LOWER_C) || i >= j)) {
      double c = alpha * acc[r];
      if (beta != 0.0) c = fma(beta, Cz[(int64_t)i * ldc + j], c);
      Cz[(int64_t)i * ldc + j] = c;
    }
  }
}

}  // namespace

int bo_gemm_f64_impl(int ta, int tb, int M, int N, int K, double alpha, const double* A,
                     int64_t lda, int64_t sA, const double* B, int64_t ldb, int64_t sB,
                     double beta, double* C, int64_t ldc, int64_t sC, int batch, int flags,
                     hipStream_t st) {
  if (M <= 0 || N <= 0 || batch <= 0) return BO_OK;
  if (K < 0) K = 0;  // C = beta * C (the alpha term is empty)
  if (N <= 16 && (M <= 16 || K <= 256)) {
    const int64_t waves = (int64_t)batch * ceil_div(M, 16);
    gemm_small_kernel<<<(unsigned)ceil_div(waves, 4), 256, 0, st>>>(
        M, N, K, alpha, A, lda, sA, ta, B, ldb, sB, tb, beta, C, ldc, sC, batch, flags);
    BO_LAUNCH_CHECK();
    return BO_OK;
  }
  // Large problems: 128 x 128 tiles (16 MFMA accumulators per wave); smaller
  // ones keep 64 x 64 so the grid still covers the 256 CUs.  Triangular
  // operands (long, unbalanced k-ranges) also use 64 x 64 so the heaviest tile
  // does not set the duration.
  const int64_t tiles128 = ceil_div(M, 128) * ceil_div(N, 128) * (int64_t)batch;
  const bool tri = flags & (BO_GEMM_A_UPPER | BO_GEMM_B_LOWER | BO_GEMM_A_LOWER | BO_GEMM_B_UPPER);
  if (tiles128 >= 512 && !(tri && K > 1024))
    return launch_gemm<128, 128, 1>(ta, tb, M, N, K, alpha, A, lda, sA, B, ldb, sB, beta, C, ldc,
                                    sC, batch, flags, st);
  // Split-k where the 64 x 64 grid leaves most CUs idle on a long k-range
  // (qNEHVI's cached-root cross term at C4: P_b R^T, 248 x 1024 x 2048 --
  // 64 tiles, 160 us unsplit): chunk partials in a stream-ordered workspace,
  // summed in chunk order (deterministic) by one reduction launch.
  // BO_GEMM_SPLITK=0 keeps one pass (A/B knob).
  static const bool splitk_on = [] {
    const char* e = std::getenv("BO_GEMM_SPLITK");
    return !(e && e[0] == '0');
  }();
  const int64_t tiles64 = ceil_div(M, 64) * ceil_div(N, 64) * (int64_t)batch;
  int ksplit = 1;
  // (BO_GEMM_SPLITK_KMIN: the shortest k-range split, default 1024; chunks
  // of >= KMIN / 4)
  static const int kmin = [] {
    const char* e = std::getenv("BO_GEMM_SPLITK_KMIN");
    const int v = e ? std::atoi(e) : 1024;
    return v >= 128 ? v : 1024;
  }();
  if (splitk_on && !(flags & BO_GEMM_LOWER_C) && tiles64 < 256 && K >= kmin)
    ksplit = (int)std::min<int64_t>(std::min<int64_t>(8, std::max<int64_t>(1, 512 / tiles64)),
                                    K / (kmin / 4));
  return launch_gemm<64, 64, 2>(ta, tb, M, N, K, alpha, A, lda, sA, B, ldb, sB, beta, C, ldc, sC,
                                batch, flags, st, ksplit);
}
