// Batched fp64 GEMM on the gfx950 matrix cores (v_mfma_f64_16x16x4_f64).
//
//   C[b] = alpha * op(A[b]) * op(B[b]) + beta * C[b]      (row-major storage)
//
// Used by the blocked Cholesky (TRSM-as-GEMM against the inverted diagonal
// block, SYRK trailing update restricted to the lower triangle), the
// recursive-doubling triangular inverse, the MLL gradient's K^{-1} = U U^T
// and the qNEI cross-covariance.  Triangular operands skip the all-zero
// k-range of each tile (flags below), which halves the flops of L^{-1}-type
// products exactly like the reference's dense GEMM would not.
//
// Tile: BM x BN per 256-thread workgroup (4 waves in a 2 x 2 grid), BK = 16.
// LDS holds op(A) as As[k][m] and op(B) as Bs[k][n] (rows padded by 16
// doubles so the two 16-lane halves of each ds_read_b64 lane group fall on
// opposite bank halves); the next k-tile is prefetched into registers while
// the current one feeds the MFMAs.
#include "common.h"
#include "gemm.h"

namespace {

constexpr int BK = 16;
constexpr int PAD = 16;

template <int BM, int BN, bool TA, bool TB>
__global__ __launch_bounds__(256) void gemm_f64_kernel(
    int M, int N, int K, double alpha, const double* __restrict__ A, int64_t lda,
    int64_t sA, const double* __restrict__ B, int64_t ldb, int64_t sB, double beta,
    double* __restrict__ C, int64_t ldc, int64_t sC, int flags) {
  constexpr int TM = BM / 32;  // MFMA tiles per wave along m (2x2 waves)
  constexpr int TN = BN / 32;
  constexpr int LA = BM * BK / 256;  // A elements staged per thread
  constexpr int LB = BN * BK / 256;
  __shared__ double As[BK][BM + PAD];
  __shared__ double Bs[BK][BN + PAD];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = (wave >> 1) * (BM / 2);
  const int wn = (wave & 1) * (BN / 2);
  const int m0 = blockIdx.y * BM;
  const int n0 = blockIdx.x * BN;
  const int64_t bz = blockIdx.z;
  A += bz * sA;
  B += bz * sB;
  C += bz * sC;

  if ((flags & BO_GEMM_LOWER_C) && n0 > m0 + BM - 1) return;  // tile strictly above diagonal

  // k-range restricted by triangular operands (zero regions are skipped).
  int kbeg = 0, kend = K;
  if (flags & BO_GEMM_A_LOWER) kend = min(kend, m0 + BM);  // op(A)[m][k] = 0 for k > m
  if (flags & BO_GEMM_B_UPPER) kend = min(kend, n0 + BN);  // op(B)[k][n] = 0 for k > n
  if (flags & BO_GEMM_A_UPPER) kbeg = max(kbeg, m0);       // op(A)[m][k] = 0 for k < m
  if (flags & BO_GEMM_B_LOWER) kbeg = max(kbeg, n0);       // op(B)[k][n] = 0 for k < n
  kbeg = (kbeg / BK) * BK;

  v4d acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = v4d_zero();

  double ra[LA], rb[LB];

  auto load_tiles = [&](int k0) {
#pragma unroll
    for (int p = 0; p < LA; ++p) {
      int e = tid + p * 256;
      int m, k;
      if (TA) { m = e % BM; k = e / BM; }  // A stored [K][M]: m contiguous
      else    { k = e % BK; m = e / BK; }  // A stored [M][K]: k contiguous
      int gm = m0 + m, gk = k0 + k;
      double v = 0.0;
      if (gm < M && gk < K) v = TA ? A[(int64_t)gk * lda + gm] : A[(int64_t)gm * lda + gk];
      ra[p] = v;
    }
#pragma unroll
    for (int p = 0; p < LB; ++p) {
      int e = tid + p * 256;
      int n, k;
      if (TB) { k = e % BK; n = e / BK; }  // B stored [N][K]: k contiguous
      else    { n = e % BN; k = e / BN; }  // B stored [K][N]: n contiguous
      int gn = n0 + n, gk = k0 + k;
      double v = 0.0;
      if (gn < N && gk < K) v = TB ? B[(int64_t)gn * ldb + gk] : B[(int64_t)gk * ldb + gn];
      rb[p] = v;
    }
  };
  auto store_tiles = [&]() {
#pragma unroll
    for (int p = 0; p < LA; ++p) {
      int e = tid + p * 256;
      int m, k;
      if (TA) { m = e % BM; k = e / BM; }
      else    { k = e % BK; m = e / BK; }
      As[k][m] = ra[p];
    }
#pragma unroll
    for (int p = 0; p < LB; ++p) {
      int e = tid + p * 256;
      int n, k;
      if (TB) { k = e % BK; n = e / BK; }
      else    { n = e % BN; k = e / BN; }
      Bs[k][n] = rb[p];
    }
  };

  if (kbeg < kend) load_tiles(kbeg);
  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    __syncthreads();
    store_tiles();
    __syncthreads();
    if (k0 + BK < kend) load_tiles(k0 + BK);
#pragma unroll
    for (int ks = 0; ks < BK / 4; ++ks) {
      const int kr = ks * 4 + (lane >> 4);
      double a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = As[kr][wm + i * 16 + (lane & 15)];
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = Bs[kr][wn + j * 16 + (lane & 15)];
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma_f64(a[i], b[j], acc[i][j]);
    }
  }

  // Epilogue.
  const bool lower = flags & BO_GEMM_LOWER_C;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        int gm = m0 + wm + i * 16 + mfma_row(lane, r);
        int gn = n0 + wn + j * 16 + mfma_col(lane);
        if (gm < M && gn < N && (!lower || gm >= gn)) {
          double* c = C + (int64_t)gm * ldc + gn;
          double v = alpha * acc[i][j][r];
          if (beta != 0.0) v += beta * (*c);
          *c = v;
        }
      }
}

template <int BM, int BN>
int launch_gemm(bool ta, bool tb, int M, int N, int K, double alpha, const double* A,
                int64_t lda, int64_t sA, const double* B, int64_t ldb, int64_t sB,
                double beta, double* C, int64_t ldc, int64_t sC, int batch, int flags,
                hipStream_t st) {
  dim3 grid((unsigned)ceil_div(N, BN), (unsigned)ceil_div(M, BM), (unsigned)batch);
  if (ta && tb)
    gemm_f64_kernel<BM, BN, true, true><<<grid, 256, 0, st>>>(M, N, K, alpha, A, lda, sA, B, ldb, sB, beta, C, ldc, sC, flags);
  else if (ta)
    gemm_f64_kernel<BM, BN, true, false><<<grid, 256, 0, st>>>(M, N, K, alpha, A, lda, sA, B, ldb, sB, beta, C, ldc, sC, flags);
  else if (tb)
    gemm_f64_kernel<BM, BN, false, true><<<grid, 256, 0, st>>>(M, N, K, alpha, A, lda, sA, B, ldb, sB, beta, C, ldc, sC, flags);
  else
    gemm_f64_kernel<BM, BN, false, false><<<grid, 256, 0, st>>>(M, N, K, alpha, A, lda, sA, B, ldb, sB, beta, C, ldc, sC, flags);
  BO_LAUNCH_CHECK();
  return BO_OK;
}

}  // namespace

int bo_gemm_f64_impl(int ta, int tb, int M, int N, int K, double alpha, const double* A,
                     int64_t lda, int64_t sA, const double* B, int64_t ldb, int64_t sB,
                     double beta, double* C, int64_t ldc, int64_t sC, int batch, int flags,
                     hipStream_t st) {
  if (M <= 0 || N <= 0 || batch <= 0) return BO_OK;
  if (K <= 0) {
    // C = beta * C (alpha term is empty).
    return launch_gemm<64, 64>(ta, tb, M, N, 0, alpha, A, lda, sA, B, ldb, sB, beta, C, ldc, sC, batch, flags, st);
  }
  // Large problems: 128 x 128 tiles (16 MFMA accumulators per wave); small
  // ones keep 64 x 64 so the grid still covers the 256 CUs.
  int64_t tiles128 = ceil_div(M, 128) * ceil_div(N, 128) * (int64_t)batch;
  if (tiles128 >= 256)
    return launch_gemm<128, 128>(ta, tb, M, N, K, alpha, A, lda, sA, B, ldb, sB, beta, C, ldc, sC, batch, flags, st);
  return launch_gemm<64, 64>(ta, tb, M, N, K, alpha, A, lda, sA, B, ldb, sB, beta, C, ldc, sC, batch, flags, st);
}
