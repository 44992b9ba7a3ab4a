// Small-grid posterior partials through A^{-1} (the "quad" plan).
//
// The one-pass posterior (post.hip) forms R = K*x L^{-T} and squares it, so a
// workgroup's 128 x 128 tile must finish its whole k-range before its
// epilogue: on small grids (C2: n = 1024, 512 test rows = 32 tiles for 256
// CUs) the k-ranges are split across workgroups and the partial R tiles
// (128 KB each) go through a workspace and a reduction launch.  The same
// posterior written through A^{-1} = L^{-T} L^{-1} = (K + s2 I)^{-1}
// ([G] exact_predictive_covar, mean_cache alpha = A^{-1}(y - c)):
//
//   Sigma_b = K**_b - sum_{k, l} K*x[b, k] A^{-1}[k, l] K*x[b, l]
//   mu_b    = c + sum_k K*x[b, k] alpha[k]
//
// is LINEAR in the blocks of A^{-1}: every (k-block, l-block) pair of 64 x 64
// blocks contributes an independent q x q term, so the work splits into equal
// units (pair, 128 test rows) whose partials are 16 x 16 per row tile instead
// of 128 x 128 R tiles.  Pairs kb < lb stand for both (kb, lb) and (lb, kb)
// (A^{-1} symmetric): the unit stores P = K_kb A^{-1}_{kb,lb} K_lb^T and the
// finalisation sums P + P^T (diagonal pairs store P / 2).  The flops equal the
// triangular R's (B q n^2 / 2 multiply-adds) plus one K_lb contraction per
// unit (16 MFMAs per 16-row tile).
//
// A^{-1} is a model cache here (bo_ainv + bo_sym_lower, built once per
// model); R is never formed, so this plan serves forward-only calls (the
// gradient path keeps R for its W = R L^{-1}).
#include "common.h"

#include <cstdlib>

namespace {

constexpr int QB = 64;    // A^{-1} block edge (k and l)
constexpr int QI = 128;   // test rows per unit (4 waves x 32)
constexpr int QLD = 68;   // LDS pitch of the A^{-1} block (doubles)

// Unit u -> (chunk, row tile).  The block pairs (kb, lb), kb <= lb, of one
// block row kb are cut into chunks of G consecutive lb; a chunk's pairs share
// the k-loop's K*x^T operands (loaded once) and ONE partial (their P's summed
// in registers), so the finalisation reads sum_kb ceil((nb - kb) / G)
// partials per row tile instead of nb (nb + 1) / 2.  Inside a chunk the next
// pair's A^{-1} block is fetched into registers under the current pair's
// MFMAs and parked in the other LDS buffer.  Consecutive units share a chunk:
// the grid deals them XCD by XCD (block b runs on XCD b % 8), so the row
// tiles of one chunk meet in one L2.
__global__ __launch_bounds__(256, 2) void post_quad_kernel(
    const double* __restrict__ Kt, int nrows_pad, const double* __restrict__ Ainv, int64_t lda,
    const double* __restrict__ alpha, int n, int nb, int G, int nI, int units,
    double* __restrict__ Spart, double* __restrict__ mpart) {
  __shared__ __attribute__((aligned(16))) double As[2][QB][QLD];
  const int bid = blockIdx.x;
  const int per_xcd = gridDim.x >> 3;  // the grid is a multiple of 8
  const int u = (bid & 7) * per_xcd + (bid >> 3);
  if (u >= units) return;  // whole workgroup: no barrier below is skipped by part of it
  const int chunk = u / nI;
  const int ii = u - chunk * nI;
  int kb = 0, rem = chunk;
  for (;;) {
    const int nc = (nb - kb + G - 1) / G;
    if (rem < nc) break;
    rem -= nc;
    ++kb;
  }
  const int lb_begin = kb + rem * G;
  const int lb_end = min(nb, lb_begin + G);
  const int k0 = kb * QB, i0 = ii * QI;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;

  // A^{-1} block (kb, lb): 64 x 64, 8 x 16 B per thread
  auto load_a = [&](int lb, double2 (&v)[(QB * QB / 2) / 256]) {
#pragma unroll
    for (int j = 0; j < (QB * QB / 2) / 256; ++j) {
      const int e = tid + 256 * j;
      v[j] = *reinterpret_cast<const double2*>(Ainv + (int64_t)(k0 + (e >> 5)) * lda + lb * QB +
                                               (e & 31) * 2);
    }
  };
  auto park_a = [&](int buf, const double2 (&v)[(QB * QB / 2) / 256]) {
#pragma unroll
    for (int j = 0; j < (QB * QB / 2) / 256; ++j) {
      const int e = tid + 256 * j;
      *reinterpret_cast<double2*>(&As[buf][e >> 5][(e & 31) * 2]) = v[j];
    }
  };
  double2 av[(QB * QB / 2) / 256];
  load_a(lb_begin, av);
  // MFMA B operands of the k-loop (K*x^T rows k0 + 4 ks + (lane >> 4), 16
  // consecutive test rows per 16 lanes): loaded once for the chunk
  const double* kt = Kt + i0 + wave * 32 + (lane & 15) + (int64_t)(lane >> 4) * nrows_pad;
  double b[QB / 4][2];
#pragma unroll
  for (int ks = 0; ks < QB / 4; ++ks)
#pragma unroll
    for (int it = 0; it < 2; ++it) b[ks][it] = kt[(int64_t)(k0 + 4 * ks) * nrows_pad + 16 * it];
  park_a(0, av);
  __syncthreads();

  // the chunk's P, one accumulator chain per 16-row tile (the two chains
  // interleave)
  v4d Pc[2] = {v4d_zero(), v4d_zero()};
  double m[2] = {0.0, 0.0};
  for (int lb = lb_begin; lb < lb_end; ++lb) {
    const int cur = (lb - lb_begin) & 1;
    const int l0 = lb * QB;
    // epilogue operands (K*x^T rows l0 + 16 ct + 4 r + (lane >> 4)) and the
    // next pair's A^{-1} block: in flight under this pair's k-loop
    double e[QB / 16][4][2];
#pragma unroll
    for (int ct = 0; ct < QB / 16; ++ct)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int it = 0; it < 2; ++it)
          e[ct][r][it] = kt[(int64_t)(l0 + 16 * ct + 4 * r) * nrows_pad + 16 * it];
    const bool more = lb + 1 < lb_end;
    if (more) load_a(lb + 1, av);

    // T^T[l][i] = sum_{k in kb} A^{-1}[k][l] K*x[i][k]: lane l, register r of
    // acc[ct][it] holds l = l0 + 16 ct + (lane >> 4) + 4 r, i = row16 + (lane & 15)
    v4d acc[QB / 16][2];
#pragma unroll
    for (int ct = 0; ct < QB / 16; ++ct) {
      acc[ct][0] = v4d_zero();
      acc[ct][1] = v4d_zero();
    }
#pragma unroll
    for (int ks = 0; ks < QB / 4; ++ks) {
      double a[QB / 16];
#pragma unroll
      for (int ct = 0; ct < QB / 16; ++ct)
        a[ct] = As[cur][4 * ks + (lane >> 4)][16 * ct + (lane & 15)];
#pragma unroll
      for (int ct = 0; ct < QB / 16; ++ct)
#pragma unroll
        for (int it = 0; it < 2; ++it) acc[ct][it] = mfma_f64(a[ct], b[ks][it], acc[ct][it]);
    }
    // the diagonal pair stands for itself only: P / 2 (summed as P + P^T),
    // applied to T (exact: a power of two)
    if (lb == kb) {
#pragma unroll
      for (int ct = 0; ct < QB / 16; ++ct) {
        acc[ct][0] *= 0.5;
        acc[ct][1] *= 0.5;
      }
    }
    // P[i][j] += sum_{l in lb} T[i][l] K*x[j][l]: the accumulator register is
    // the A operand as it stands (k index = (lane >> 4) + 4 r), K*x^T the B
#pragma unroll
    for (int ct = 0; ct < QB / 16; ++ct)
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int it = 0; it < 2; ++it)
          Pc[it] = mfma_f64(acc[ct][it][r], e[ct][r][it], Pc[it]);
    // mean K*x[j, kb] alpha[kb] from the diagonal pair's operands
    if (lb == kb) {
#pragma unroll
      for (int it = 0; it < 2; ++it)
#pragma unroll
        for (int ct = 0; ct < QB / 16; ++ct)
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int l = l0 + 16 * ct + 4 * r + (lane >> 4);
            m[it] = fma(e[ct][r][it], l < n ? alpha[l] : 0.0, m[it]);
          }
    }
    if (more) park_a(cur ^ 1, av);
    __syncthreads();
  }

  const int nrows16 = nrows_pad >> 4;
#pragma unroll
  for (int it = 0; it < 2; ++it) {
    const v4d P = Pc[it];
    const int row16 = i0 + wave * 32 + it * 16;
    double* sp = Spart + ((int64_t)chunk * nrows16 + (row16 >> 4)) * 256;
#pragma unroll
    for (int r = 0; r < 4; ++r) sp[mfma_row(lane, r) * 16 + mfma_col(lane)] = P[r];
    double mm = m[it];
    mm += __shfl_xor(mm, 16);
    mm += __shfl_xor(mm, 32);
    if (lane < 16) mpart[(int64_t)chunk * nrows_pad + row16 + lane] = mm;
  }
}

// Partials per row tile of the quad plan: sum_kb ceil((nb - kb) / G).
int quad_chunks(int nb, int G) {
  int c = 0;
  for (int kb = 0; kb < nb; ++kb) c += (nb - kb + G - 1) / G;
  return c;
}

// Pairs per chunk: BO_QUAD_G (1..16) or 1 (chunks of 4 measured slower at C2:
// 35 vs 26-31 us for the posterior, the finalisation 17 vs 21 us).
int quad_group() {
  static const int g = [] {
    const char* e = std::getenv("BO_QUAD_G");
    const int v = e ? std::atoi(e) : 0;
    return (v >= 1 && v <= 16) ? v : 1;
  }();
  return g;
}

// A[r][c] = A[c][r] for r < c (the upper triangle from the lower), 32 x 32
// tiles through LDS so both sides are read and written along rows.
__global__ __launch_bounds__(256) void sym_lower_kernel(double* __restrict__ A, int64_t ld, int n) {
  __shared__ double t[32][33];
  const int tr = blockIdx.y, tc = blockIdx.x;  // destination tile (tile row < tile col, or diagonal)
  if (tr > tc) return;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  // source: tile (tc, tr) of the lower triangle
  for (int y = ty; y < 32; y += 8) {
    const int r = tc * 32 + y, c = tr * 32 + tx;
    t[y][tx] = (r < n && c < n) ? A[(int64_t)r * ld + c] : 0.0;
  }
  __syncthreads();
  for (int y = ty; y < 32; y += 8) {
    const int r = tr * 32 + y, c = tc * 32 + tx;
    if (r < n && c < n && r < c) A[(int64_t)r * ld + c] = t[tx][y];
  }
}

}  // namespace

extern "C" {

int bo_post_geometry(int64_t B, int q, int64_t n, int* Qp, int* nrows_pad, int* nC);
int bo_post_split_plan(int64_t B, int q, int64_t n, int slots, int* kc_len, int64_t* work_elems);

// The quad plan (opt-in, BO_POST_QUAD=auto) applies to forward-only calls
// whose one-pass grid would be split (bo_post_split_plan: stream-K) with
// n <= 2048 and at most ~1000 pair units; =1 forces it wherever the geometry
// allows, =0 / unset keeps the R route.
int bo_post_quad_plan(int64_t B, int q, int64_t n, int* npairs) {
  int Qp, nrows_pad, nC;
  int s = bo_post_geometry(B, q, n, &Qp, &nrows_pad, &nC);
  if (s) return s;
  *npairs = 0;
  if (nrows_pad == 0 || n <= 0) return BO_OK;
  // Opt-in (BO_POST_QUAD=1 or =auto): measured at C2 the quad posterior takes
  // 26-31 us against 25 + 13 us for the R route's stream-K pass and split-k
  // reduction, but its 136 partials (40 in chunks of 4) cost the
  // finalisation 10-14 us more than the R route's 8, so the eager call is no
  // faster (0.064-0.066 ms both, profiles/r03/c2/).  Default: the R route.
  const char* env = std::getenv("BO_POST_QUAD");
  const int force = env ? (env[0] == '0' ? 0 : (env[0] == '1' ? 1 : -1)) : 0;
  if (force == 0) return BO_OK;
  const int nb = (int)ceil_div(n, QB);
  bool use = force == 1;
  if (!use) {
    int kc = 0;
    int64_t we = 0;
    s = bo_post_split_plan(B, q, n, 0, &kc, &we);
    if (s) return s;
    // measured (tools/time_quad.py, profiles/r03/time_quad*.json): the quad
    // units run at ~57% of the MFMA peak against the R route's ~75%, so the
    // plan wins only where the R route's split-k reduction dominates -- up to
    // ~1000 units (C2: 544 units, 30 vs 41 us; n = 1024, b = 256: 2176 units,
    // 74 vs 67 us)
    const int64_t units = (int64_t)nb * (nb + 1) / 2 * (nrows_pad / QI);
    use = kc != 0 && n <= 2048 && units <= 1024;  // counted in pairs
  }
  if (use) *npairs = quad_chunks(nb, quad_group());
  return BO_OK;
}

int bo_post_quad(const double* Kt, const double* Ainv, int64_t lda, const double* alpha, int64_t B,
                 int q, int64_t n, double* Spart, double* mpart, void* stream) {
  int Qp, nrows_pad, nC;
  int s = bo_post_geometry(B, q, n, &Qp, &nrows_pad, &nC);
  if (s) return s;
  if (nrows_pad == 0) return BO_OK;  // no t-batches
  BO_CHECK_ARG(Kt && Ainv && alpha && Spart && mpart, "bo_post_quad: null buffer");
  BO_CHECK_ARG(lda % 2 == 0 && lda >= (int64_t)nC * 128,
               "bo_post_quad: A^{-1} leading dim %lld must be even and >= %d", (long long)lda,
               nC * 128);
  const int nb = (int)ceil_div(n, QB);
  const int nI = nrows_pad / QI;
  const int G = quad_group();
  const int64_t units = (int64_t)quad_chunks(nb, G) * nI;
  BO_CHECK_ARG(units < (1LL << 30), "bo_post_quad: %lld units", (long long)units);
  const int64_t grid = ceil_div(units, 8) * 8;
  // Kt (np x nrows_pad) has rows up to nC * 128 >= nb * 64: every block row read exists
  post_quad_kernel<<<(unsigned)grid, 256, 0, as_stream(stream)>>>(
      Kt, nrows_pad, Ainv, lda, alpha, (int)n, nb, G, nI, (int)units, Spart, mpart);
  BO_LAUNCH_CHECK();
  return BO_OK;
}

int bo_sym_lower(double* A, int64_t ld, int64_t n, void* stream) {
  BO_CHECK_ARG(A && n >= 0 && ld >= n, "bo_sym_lower: bad arguments");
  if (n == 0) return BO_OK;
  const unsigned t = (unsigned)ceil_div(n, 32);
  sym_lower_kernel<<<dim3(t, t), 256, 0, as_stream(stream)>>>(A, ld, (int)n);
  BO_LAUNCH_CHECK();
  return BO_OK;
}

}  // extern "C"
