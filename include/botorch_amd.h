/*
 * botorch_amd -- C ABI of the MI355X (gfx950) GP-posterior + MC-acquisition
 * hot path.  Plain pointers and sizes only; every pointer argument named for
 * a tensor is a DEVICE pointer (HBM) unless documented as host; every `stream`
 * is a hipStream_t passed as void* (enqueue only -- the calls never
 * synchronise, except bo_gp_cache_build, which reads the Cholesky status back
 * once per jitter attempt, as the reference's psd_safe_cholesky does).
 *
 * All matrices are row-major fp64.  Return value: BO_OK (0) or a BO_ERR_*
 * code; bo_last_error() describes the last failure of the calling thread.
 *
 * The reference (anand-12/botorch @ 2024-10-08) is pure Python over
 * GPyTorch/linear_operator; it has no FFI.  Each entry point cites the
 * reference interface whose computation it replaces; INTEGRATION.md shows the
 * ctypes binding (botorch_amd/_lib.py) a maintainer adds on the reference side.
 */
#ifndef BOTORCH_AMD_H
#define BOTORCH_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BO_ABI_VERSION 11

/* status codes */
#define BO_OK 0
#define BO_ERR_ARG 1
#define BO_ERR_HIP 2
#define BO_ERR_NOT_PSD 3 /* maps to NotPSDError (botorch/exceptions/errors.py) */
#define BO_ERR_NAN 4     /* maps to NanError */

/* kernel families (botorch/models/utils/gpytorch_modules.py:100-127,
 * botorch/models/fully_bayesian.py:81-92) */
#define BO_KIND_RBF 0
#define BO_KIND_MATERN52 1

/* bo_gemm_f64 flags: structure of the operands (zero regions are skipped) */
#define BO_GEMM_LOWER_C 1 /* write only C[m][n] with m >= n */
#define BO_GEMM_A_LOWER 2 /* op(A)[m][k] == 0 for k > m */
#define BO_GEMM_B_UPPER 4 /* op(B)[k][n] == 0 for k > n */
#define BO_GEMM_A_UPPER 8 /* op(A)[m][k] == 0 for k < m */
#define BO_GEMM_B_LOWER 16 /* op(B)[k][n] == 0 for k < n */

/* layouts of the stored R^T (BoPostPartialsArgs.rt_layout): row-major
 * (nC*128) x nrows_pad, or blocked in the posterior kernel's MFMA accumulator
 * order -- 16 x 16 blocks (training block kb, test block ib) at
 * (kb * nrows_pad / 16 + ib) * 256, element (k, i) of a block at
 * ((k % 16) / 4) * 64 + (k % 4) * 16 + i % 16 -- so every store and every
 * load of it is one 512-B segment per instruction.  bo_post_w_dx reads the
 * blocked layout; every other consumer (bo_post_w, bo_post_w_split,
 * bo_gemm_f64) the row-major one. */
#define BO_RT_ROWMAJOR 0
#define BO_RT_BLOCKED 1

/* qmc modes */
#define BO_QMC_POSTERIOR 0
#define BO_QMC_QEI 1
#define BO_QMC_QNEI 2
#define BO_QMC_CHOL 3 /* finalise + jittered q x q Cholesky only (no MC) */
#define BO_QMC_QLOGEI 4  /* qLogExpectedImprovement (acquisition/logei.py:137-234) */
#define BO_QMC_QLOGNEI 5 /* qLogNoisyExpectedImprovement, cached root (logei.py:236-507) */

const char* bo_last_error(void);
int bo_version(void);

/* Hardware probe of the fp64 MFMA accumulator map; out: 64 x 8 doubles (the
 * layout the kernels assume, checked by tests/test_gpu_kernels.py).  The
 * timing/trace probes of the development tools are not part of this ABI: they
 * live in tools/bo_tools.h (tools/libbotorch_amd_tools.so, `make tools`). */
int bo_probe_mfma_f64_layout(double* out, void* stream);

/* Peak-rate probe: `blocks` x 256 threads, each wave issuing iters x 8
 * independent fp64 MFMAs (2048 flop each).  out: 1 double (kept live). */
int bo_probe_mfma_f64_rate(int blocks, int iters, double* out, void* stream);



/* Queue of the Cholesky task DAG for T = np/64 tile rows (HOST function, no
 * device work): 4 ints per task (type | fin << 8, k, j, i0 | i1 << 16) into
 * out (capacity cap tasks); returns the task count. */
int bo_chol_dag_tasks(int T, int* out, int cap);
/* The same queue with the A^{-1} tasks (bo_cholesky_inverse_ainv). */
int bo_chol_dag_tasks_ainv(int T, int* out, int cap);

/* Batched C = alpha op(A) op(B) + beta C on the fp64 matrix cores (strides sA,
 * sB, sC between batch members).  Building block of the Cholesky/inverse and
 * of the qNEI cross-covariance; replaces the dense torch.matmul calls inside
 * [G] linear_operator (e.g. MatmulLinearOperator under
 * botorch/models/gpytorch.py:446). */
int bo_gemm_f64(int transA, int transB, int M, int N, int K, double alpha, const double* A,
                int64_t lda, int64_t sA, const double* B, int64_t ldb, int64_t sB,
                double beta, double* C, int64_t ldc, int64_t sC, int batch, int flags,
                void* stream);

/* K[i][j] = outputscale * k(X1_i, X2_j) + diag_add * [i == j] over a rows x cols
 * extent with an identity pad beyond (n1, n2); mode bit 1 zeroes the strict
 * upper triangle.  X1: n1 x d, X2: n2 x d, lengthscale: d.
 * Replaces [G] RBFKernel/MaternKernel(+ScaleKernel).forward
 * (SingleTaskGP.forward, botorch/models/gp_regression.py:249-254). */
int bo_covar_matrix(int kind, const double* X1, int64_t n1, const double* X2, int64_t n2,
                    int d, const double* lengthscale, double outputscale, double diag_add,
                    int mode, double* K, int64_t ldk, int64_t rows, int64_t cols, void* stream);

/* Padded order np used by every n x n cache below (multiple of 128). */
int64_t bo_padded_order(int64_t n);

/* Two-level batched covariance (batch z = o * inner + i, o < outer, i < inner):
 * K[o][i] (n1 x n2, leading dim ldk, at K + o sKo + i sKi) =
 *   os[o soo + i soi] * k((X1[o][i] - X2[o][i]) / ls[o][i]),
 * X1 at X1 + o s1o + i s1i (n1 x d), X2 likewise, ls at ls + o slo + i sli (d).
 * Strides are in elements (0 = shared); d <= 512.  The SAAS ensemble's K*x of all M
 * members and K** of all M x B t-batches (models/fully_bayesian.py:276-281),
 * one launch each. */
int bo_covar_batched(int kind, const double* X1, int64_t s1o, int64_t s1i, int n1,
                     const double* X2, int64_t s2o, int64_t s2i, int n2, int d, const double* ls,
                     int64_t slo, int64_t sli, const double* os, int64_t soo, int64_t soi,
                     double* K, int64_t sKo, int64_t sKi, int64_t ldk, int outer, int inner,
                     void* stream);

/* In-place blocked Cholesky of the lower-stored SPD matrix A (np x np, upper
 * triangle zero) and its explicit inverse Linv (np x np).  work: np x np
 * scratch.  *info (device int) = 0 or the 1-based order of the first failing
 * leading minor (torch.linalg.cholesky_ex convention). */
int bo_cholesky_inverse(double* A, double* Linv, double* work, int64_t np, int* info,
                        void* stream);
/* bo_cholesky_inverse plus A^{-1} = L^{-T} L^{-1} (the lower 64 x 64 tiles,
 * diagonal tiles whole) in the SAME persistent launch (round 5): the MLL
 * gradient's tr(A^{-1} dK/dtheta) (botorch/optim/closures/model_closures.py:
 * 171-184 -> [G] ExactMarginalLogLikelihood's backward).  Its tile products run
 * as soon as the rows of L^{-1} they read are final, in the CUs the
 * factorisation's chain-bound tail leaves idle.  work >= (16 + 5 (np/64)^2)
 * 4-byte counters. */
int bo_cholesky_inverse_ainv(double* A, double* Linv, double* Ainv, double* work, int64_t np,
                             int* info, void* stream);

/* nb independent bo_cholesky_inverse problems in ONE persistent launch: A and
 * Linv hold nb np x np matrices back to back, info nb device ints, work >=
 * (16 + 4 nb (np/64)^2) * 4 bytes.  The matrices' task queues are interleaved,
 * so one matrix's diagonal chain overlaps the others' MFMA updates.  Results
 * are bit-identical to nb separate calls.  Replaces the per-output
 * factorisations of a batched multi-output GP ([G] batched
 * psd_safe_cholesky over the output batch, models/gpytorch.py:327-355) and of
 * a ModelListGP's members (models/model_list_gp_regression.py). */
int bo_cholesky_inverse_batched(double* A, double* Linv, double* work, int nb, int64_t np,
                                int* info, void* stream);

/* psd_safe_cholesky of one n x n matrix ([G] linear_operator, the ladder of
 * botorch/__init__.py:47): factor A + jitter I for jitter = 0, jitter0,
 * 10 jitter0, ... (max_tries increments).  L, Linv, work: np x np (identity
 * pad); jitter_used: HOST double.  Used for the joint posterior over the qNEI
 * baseline (acquisition/cached_cholesky.py:94-120, acquisition/utils.py:245-349). */
int bo_cholesky_jitter(const double* A, int64_t n, double* L, double* Linv, double* work,
                       int max_tries, double jitter0, double* jitter_used, int* info_dev,
                       void* stream);

/* Outcome of a batched jitter ladder (info, jitter: B entries from
 * bo_qmc_finalize / bo_chol_small): out[0] = max info (0: all factored),
 * out[1] = max jitter added.  One launch; the caller reads 16 bytes back, as
 * [G] psd_safe_cholesky's torch.any(info) check does. */
int bo_ladder_status(const int* info, const double* jitter, int64_t B, double* out, void* stream);

/* Pinned, device-mapped, coherent host memory (zeroed): *host for the CPU,
 * *dev for kernels -- the status words bo_qmc_finalize folds a ladder's
 * outcome into (BoQmcFinalizeArgs.status_out), read by the host after a
 * stream sync without a status launch or copy (a ModelListGP's members in
 * the qEHVI forward).  bo_pinned_free releases it. */
int bo_pinned_alloc(int64_t bytes, void** host, void** dev);
/* bo_qmc_finalize_ext in BO_QMC_CHOL mode (mean + jittered q x q root) for
 * nm <= 8 models of one shape and kernel kind in ONE launch: per member its
 * rows Xq[m], partials Spart[m] / mpart[m] (nparts as bo_qmc_finalize_ext),
 * scalars and outputs; status_out (optional, with status_count) per member as
 * BoQmcFinalizeArgs.status_out; Tm / F (optional, with r, ldT, ldF): each
 * member's cached-root qNEHVI terms as BoQmcFinalizeArgs.Tm / F.  A
 * ModelListGP's members in the qEHVI / qNEHVI forward. */
int bo_qmc_finalize_members(int nm, int kind, int B, int q, const double* const* Xq,
                            const double* const* Spart, const double* const* mpart, int64_t n,
                            const double* outputscale, const double* constant, const double* ymean,
                            const double* ystd, int max_tries, double jitter0,
                            double* const* mean_out, double* const* L_out, int* const* info_out,
                            double* const* jitter_out, int nparts, double* const* status_out,
                            int* const* status_count, const double* const* Tm, int r,
                            int64_t ldT, const double* const* F, int64_t ldF, void* stream);
int bo_pinned_free(void* host);

/* Pareto masks of S point sets (Y: S x n x m, m <= 8; out: S x n bytes, 1 =
 * non-dominated): no other point is >= in every objective and > in one
 * (maximize; <= / < otherwise); dedup also drops later copies of equal points.
 * botorch/utils/multi_objective/pareto.py:16-64 over the S joint samples of
 * prune_inferior_points_multi_objective (acquisition/multi_objective/utils.py:77-161). */
int bo_pareto_mask(const double* Y, int64_t S, int n, int m, int maximize, int dedup,
                   unsigned char* out, void* stream);

/* Batched small psd_safe_cholesky (q <= 64), ladder applied per member
 * ([G] MultivariateNormal root_decomposition, posteriors/gpytorch.py:121-123).
 * A, L: B x q x q; info (B, nullable), jitter (B, nullable). */
int bo_chol_small(const double* A, int64_t B, int q, int max_tries, double jitter0, double* L,
                  int* info, double* jitter, void* stream);

/* K[b] = outputscale * k(X[b], X[b]) (+ diag_add I), X: B x q x d, K: B x q x q. */
int bo_covar_blocks(int kind, const double* X, int64_t B, int q, int d,
                    const double* lengthscale, double outputscale, double diag_add, double* K,
                    void* stream);

/* B = A^T for n x n matrices with leading dimension ld. */
int bo_transpose(const double* A, double* B, int64_t n, int64_t ld, void* stream);

/* y[i] = sum_k M[i][k] (x[k] - xshift), i, k < n. */
int bo_gemv(const double* M, int64_t ld, int64_t n, const double* x, double xshift, double* y,
            void* stream);
/* bo_gemv for a triangular M (uplo 1: lower, 2: upper), reading only the
 * triangle; bit-identical to bo_gemv on the same (zero-filled) matrix.  The
 * cache builds' beta = L^{-1}(y - c). */
int bo_gemv_tri(const double* M, int64_t ld, int64_t n, const double* x, double xshift, double* y,
                int uplo, void* stream);
/* y = M^T (x - xshift) for a lower-triangular M (y[c] = sum_{k >= c} M[k][c]
 * (x[k] - xshift)) read column-wise, without forming M^T: the caches' alpha =
 * L^{-T} beta = (K + s2 I)^{-1}(y - c), [G] mean_cache (botorch/models/
 * gpytorch.py:446; the MLL closure, optim/closures/model_closures.py:171-184,
 * forms no L^{-T}).  work >= bo_gemv_lt_work(n) doubles. */
int bo_gemv_lt_work(int64_t n, int64_t* work_elems);
int bo_gemv_lt(const double* M, int64_t ld, int64_t n, const double* x, double xshift, double* y,
               double* work, void* stream);

/* Xs[i][t] = (X[i][t] - center[t]) / lengthscale[t] for t < d, 0 for d <= t < dp
 * (center may be NULL). */
int bo_scale_inputs(const double* X, int64_t n, int d, const double* lengthscale,
                    const double* center, int dp, double* Xs, void* stream);

/* Exact-GP training caches of an eval-mode SingleTaskGP ([G]
 * DefaultPredictionStrategy.mean_cache / covar_cache, reached at
 * botorch/models/gpytorch.py:446 under gpt_posterior_settings,
 * botorch/models/utils/assorted.py:286-298):
 *   L = psd_safe_cholesky(K + noise I)   (jitter ladder: 0, then jitter0*10^i,
 *                                          i < max_tries; botorch/__init__.py:47)
 *   Linv = L^{-1},  U = L^{-T} (covar_cache),
 *   beta = L^{-1}(y - constant),  alpha = U beta (mean_cache).
 * Xt: n x d, y: n (standardized targets).  L, Linv, U: np x np device buffers,
 * beta, alpha: n.  jitter_used: HOST double (may be NULL).  info_dev: device int.
 * Returns BO_ERR_NOT_PSD when the ladder is exhausted. */
int bo_gp_cache_build(int kind, const double* Xt, int64_t n, int d, const double* lengthscale,
                      double outputscale, double noise, double constant, const double* y,
                      double* L, double* Linv, double* U, double* beta, double* alpha,
                      int max_tries, double jitter0, double* jitter_used, int* info_dev,
                      void* stream);
/* The same caches under a fixed-noise likelihood (SingleTaskGP with train_Yvar,
 * botorch/models/gp_regression.py:187-194 -> [G] FixedNoiseGaussianLikelihood):
 * K + diag(noise_vec), noise_vec: n observed variances (device, standardised
 * like the targets), then the same jitter ladder. */
int bo_gp_cache_build_fixed(int kind, const double* Xt, int64_t n, int d,
                            const double* lengthscale, double outputscale,
                            const double* noise_vec, double constant, const double* y, double* L,
                            double* Linv, double* U, double* beta, double* alpha, int max_tries,
                            double jitter0, double* jitter_used, int* info_dev, void* stream);

/* Geometry of the fused posterior kernels for B t-batches of q points (1 <= q
 * <= 16) over n training points: Qp = q rounded up to a power of two,
 * nrows_pad = roundup(B*Qp, 128) test rows, nC = ceil(n/128) column tiles.
 * Host pointers. */
int bo_post_geometry(int64_t B, int q, int64_t n, int* Qp, int* nrows_pad, int* nC);

/* Xq[(b*Qp + a)*8 + t] = X[b][a][t] / lengthscale[t] (X: B x q x d, d <= 8);
 * Xq: nrows_pad x 8. */
int bo_prepare_rows(const double* X, int B, int q, int d, const double* lengthscale,
                    double* Xq, void* stream);

/* Fused K*x build + R^T = U^T K*x^T GEMM + R R^T / R beta epilogue
 * ([G] exact_predictive_mean / exact_predictive_covar under fast_pred_var,
 * botorch/models/gpytorch.py:446).  Xt_scaled: n x 8 lengthscale-scaled
 * training inputs; U: >= np x np with leading dim ldu; beta: n.
 * Spart: nC x (nrows_pad/16) x 16 x 16,  mpart: nC x nrows_pad.
 * Rt (nullable, gradient path): R^T, (nC*128) x nrows_pad.
 * kc_len = 0: one workgroup per (column tile, row tile), work unused;
 * kc_len > 0: split (every tile cut into chunks of kc_len training rows);
 * kc_len = -1: stream-K (the tiles' k-steps cut into one equal share per
 * resident slot).  Split plans reduce each cut tile's chunks in k order, with
 * `work` >= the work_elems of bo_post_split_plan / bo_post_split_work.
 * Qc (nullable, one-pass only): rq <= 16 rows (leading dim ldq >= n) whose
 * products with K*x are returned as nC column-tile partials
 * Cx[ci] (nC x rq x nrows_pad; sum over ci = Qc K*x^T) -- the
 * qNEI cross-covariance P_b R^T = Q_b K*x^T, Q_b = P_b U^T
 * (acquisition/cached_cholesky.py:94-120), without storing R.
 * Kt (nullable): K*x^T from bo_post_kxt (read instead of evaluated). */
int bo_post_partials(int kind, const double* Xq, int B, int q, int d,
                     const double* Xt_scaled, int64_t n, const double* U, int64_t ldu, const double* beta,
                     double outputscale, double* Spart, double* mpart, double* Rt,
                     int kc_len, double* work, const double* Qc, int rq, int64_t ldq, double* Cx,
                     const double* Kt, void* stream);

/* K*x^T of the same call, np x nrows_pad (np = 128 nC): Kt[k][i] =
 * outputscale k(x_i, x_k), zero for k >= n and padding rows.  Passed to
 * bo_post_partials as Kt, the posterior kernel reads these values instead of
 * evaluating each one again for every column tile that covers it. */
int bo_post_kxt(int kind, const double* Xq, int B, int q, int d, const double* Xt_scaled,
                int64_t n, double outputscale, double* Kt, void* stream);

/* bo_prepare_rows and bo_post_kxt in one launch (ABI 11): Xq (nrows_pad x 8)
 * and Kt from X (B x q x d) and the lengthscale directly. */
int bo_post_kxt_rows(int kind, const double* X, int B, int q, int d, const double* lengthscale,
                     const double* Xt_scaled, int64_t n, double outputscale, double* Xq, double* Kt,
                     void* stream);

/* W^T = L^{-T} R^T = (K*x (K + s2 I)^{-1})^T for the posterior backward, np x
 * nrows_pad, from bo_post_partials' stored R^T (np x nrows_pad) and L^{-1}
 * (lower, ld ldl): the posterior kernel's MFMA tiles over the lower k-range
 * k >= c of each column (the second forward-size contraction of the gradient,
 * SURVEY.md 8(a) a14).  BO_ERR_ARG when the tile grid does not form 8 x 8
 * super-tiles (the caller then uses bo_gemm_f64). */
int bo_post_w(const double* Linv, int64_t ldl, const double* Rt, int B, int q, int64_t n,
              double* Wt, void* stream);
/* The same W^T under a stream-K plan (grids below four tiles per resident
 * slot, where the k-ranges [128 c, n) leave the one-pass grid imbalanced; no
 * super-tile condition).  bo_post_w_work: *kc_len = -1 and the workspace
 * doubles when the plan applies, else *kc_len = 0. */
int bo_post_w_work(int B, int q, int64_t n, int* kc_len, int64_t* work_elems);
int bo_post_w_split(const double* Linv, int64_t ldl, const double* Rt, int B, int q, int64_t n,
                    double* Wt, double* work, void* stream);
/* The same W^T of nm <= 8 models of one shape (a ModelListGP's members:
 * Linv[m], Rt[m], Wt[m]) in one stream-K launch + one reduction.
 * bo_post_w_members_work: the shared workspace in doubles, or -1 where the
 * one-model plan is not stream-K (then bo_post_w_split per model). */
int bo_post_w_members_work(int nm, int B, int q, int64_t n, int64_t* work_elems);
int bo_post_w_split_members(int nm, const double* const* Linv, int64_t ldl, const double* const* Rt,
                            int B, int q, int64_t n, double* const* Wt, double* work, void* stream);

/* The posterior backward without W: dX (B x q x d) of the posterior moments'
 * cotangents (dmean B x q, dcov B x q x q, standardised by ystd as in
 * bo_post_backward) from bo_post_partials' stored R^T and L^{-1}: the one-pass
 * W^T = L^{-T} R^T tiles of bo_post_w with the reduction dK*x = s dmean alpha^T
 * - G W (G_b = s^2 (dcov_b + dcov_b^T)) -> dX fused into their epilogue, W
 * never written; then the K** term and 1 / lengthscale (generation/gen.py:
 * 194-222 -> autograd through [G] exact prediction).
 * Rt in the BO_RT_BLOCKED layout (bo_post_partials_v with rt_layout =
 * BO_RT_BLOCKED).  work >= bo_post_w_dx_work doubles (nC x nrows_pad x 8 partials); a zero
 * size means the one-pass grid does not apply (stream-K plans: use
 * bo_post_w_split + bo_post_backward) and bo_post_w_dx returns BO_ERR_ARG. */
int bo_post_w_dx_work(int B, int q, int64_t n, int64_t* work_elems);
int bo_post_w_dx(int kind, const double* Linv, int64_t ldl, const double* Rt, int B, int q, int d,
                 int64_t n, const double* Xq, const double* Xt_scaled, const double* alpha,
                 const double* dmean, const double* dcov, const double* lengthscale,
                 double outputscale, double ystd, double* work, double* dX, void* stream);

/* Plan of bo_post_partials (host pointers): kc_len = 0 (one pass) or -1
 * (stream-K), whichever a k-step cost model of the triangular grid over
 * `slots` resident workgroups (slots <= 0: 512 = 256 CUs x 2) rates faster,
 * and the workspace size in doubles. */
int bo_post_split_plan(int64_t B, int q, int64_t n, int slots, int* kc_len,
                       int64_t* work_elems);
/* Workspace doubles of bo_post_partials under a given kc_len (0, -1 or a
 * chunk length). */
int bo_post_split_work(int64_t B, int q, int64_t n, int kc_len, int64_t* work_elems);

/* Small-grid forward posterior (round 5; replaces the stream-K split + split-k
 * reduction of small forward-only grids such as C2, the R R^T / R beta
 * contraction of [G] exact prediction, botorch/models/gpytorch.py:446 under
 * acquisition/monte_carlo.py:405-414): units of 32 test rows x a pair of
 * 32-column tiles of U = L^{-T} whose triangular k-ranges sum to a constant,
 * so every unit covers whole k-ranges and emits finished 16 x 16 partials.
 * bo_post_small_plan: *nparts = np / 64 partials per 16-row tile where the
 * library takes this route (BO_POST_SMALL: 0 never, 1 always, default where
 * the 128-tile plan would be stream-K), else 0.  bo_post_small: Kt = K*x^T
 * (np x nrows_pad, bo_post_kxt), U (ld ldu >= np), beta (n); writes Spart
 * (nparts x nrows_pad/16 x 16 x 16) and mpart (nparts x nrows_pad), the
 * bo_qmc_finalize inputs with nparts = *nparts, sym_parts = 0, and with Rt
 * non-null R^T row-major (np x nrows_pad) for the gradient's W^T routes. */
int bo_post_small_plan(int64_t B, int q, int64_t n, int* nparts);
int bo_post_small(const double* Kt, int64_t B, int q, int64_t n, const double* U, int64_t ldu,
                  const double* beta, double* Spart, double* mpart, double* Rt, void* stream);
/* nm <= 8 models of one shape (B, q, n, ldu) in ONE launch -- the members of
 * a ModelListGP (botorch/models/gpytorch.py:629-726: C4's three outputs), each
 * with its own K*x^T, U, beta and outputs (host arrays of device pointers; Rt
 * may be null, or hold nulls).  Rt[m]: R^T row-major (np x nrows_pad), the
 * gradient path's input to the W^T routes. */
int bo_post_small_batched(int nm, const double* const* Kt, const double* const* U,
                          const double* const* beta, double* const* Spart, double* const* mpart,
                          double* const* Rt, int64_t B, int q, int64_t n, int64_t ldu,
                          void* stream);
/* The same nm <= 8 models' partials where the one-model plan is stream-K
 * (C4: ModelListGP(3), n = 2048, q = 8, b = 128): ONE stream-K launch over
 * every member's 128 x 128 tiles plus one split-k reduction, replacing one
 * bo_post_partials per member (models/model_list_gp.py -> [G]
 * ModelListGP.posterior's per-model loop).  Spart[m] / mpart[m] hold nC
 * column-tile partials (bo_post_partials' layout); Rt[m] (optional) R^T
 * row-major; Xq0 any member's padded rows (bo_post_kxt_rows).
 * bo_post_members_work: the shared workspace in doubles, -1 where the
 * one-model plan is not stream-K (one launch per model then). */
int bo_post_members_work(int nm, int64_t B, int q, int64_t n, int64_t* work_elems);
/* bo_post_kxt_rows for nm <= 8 models of one shape and kernel kind sharing X
 * (lengthscale[m], Xt_scaled[m], outputscale[m] -> Xq[m], Kt[m]) in one
 * launch. */
int bo_post_kxt_rows_members(int nm, int kind, const double* X, int B, int q, int d,
                             const double* const* lengthscale, const double* const* Xt_scaled,
                             const double* outputscale, int64_t n, double* const* Xq,
                             double* const* Kt, void* stream);
int bo_post_partials_members(int nm, const double* const* Kt, const double* const* U,
                             const double* const* beta, double* const* Spart, double* const* mpart,
                             double* const* Rt, const double* Xq0, int64_t B, int q, int64_t n,
                             int64_t ldu, double* work, void* stream);
/* A^{-1} = L^{-T} L^{-1} for the MLL gradient (replaces the U U^T GEMM of
 * fit.py's closure, optim/closures/model_closures.py:171-184 -> [G]
 * ExactMarginalLogLikelihood backward): Linv np x np (ld = np = n rounded up
 * to 128, identity pad), Ainv np x np receives the lower tiles (tile row >=
 * tile column; diagonal tiles whole).  work >= bo_ainv_work doubles. */
int bo_ainv_work(int64_t n, int64_t* work_elems);
int bo_ainv(const double* Linv, int64_t ld, int64_t n, double* Ainv, double* work, void* stream);

/* A[r][c] = A[c][r] for r < c < n: the full symmetric A^{-1} from bo_ainv's
 * lower tiles (call with n = np so the identity pad is mirrored too). */
int bo_sym_lower(double* A, int64_t ld, int64_t n, void* stream);

/* Forward-only posterior partials of small grids through A^{-1} (the "quad"
 * plan, csrc/quad.hip): Sigma_b = K**_b - sum_{kb <= lb} (P + P^T) over 64 x 64
 * block pairs of the full symmetric A^{-1} = (K + s2 I)^{-1} (bo_ainv +
 * bo_sym_lower), mu_b = c + K*x alpha -- the same [G] exact_predictive_mean /
 * covar as bo_post_partials (models/gpytorch.py:405-466), linear in the blocks
 * of A^{-1}, so the units' partials are 16 x 16 blocks and no split-k
 * reduction runs; the pairs of one block row are taken in chunks of G (one
 * partial per chunk and row tile).  bo_post_quad_plan: *npairs = the partial
 * count (> 0) when the plan applies to (B, q, n) (opt-in: BO_POST_QUAD=auto
 * for stream-K geometries with n <= 2048 and <= 1024 pair units, =1 forces
 * it; unset / 0: the R route, measured as fast at C2; BO_QUAD_G sets the
 * chunk, default 1); the caller then sizes Spart as npairs x
 * nrows_pad/16 x 16 x 16 and mpart as npairs x nrows_pad and finalises with
 * BoQmcFinalizeArgs nparts = npairs, sym_parts = 1.  Kt: bo_post_kxt's K*x^T
 * (np x nrows_pad). */
int bo_post_quad_plan(int64_t B, int q, int64_t n, int* npairs);
int bo_post_quad(const double* Kt, const double* Ainv, int64_t lda, const double* alpha, int64_t B,
                 int q, int64_t n, double* Spart, double* mpart, void* stream);

/* The segment table of a split plan (host only; tests): up to cap segments as
 * 4 ints (ci | ii << 16, kbeg, kend, chunk or -1 = whole tile in place) and
 * up to wcap + 1 per-workgroup offsets; *nseg, *nwg receive the sizes. */
int bo_post_split_table(int64_t B, int q, int64_t n, int kc_len, int* segs, int cap, int* wg_off,
                        int wcap, int* nseg, int* nwg);

/* Finalise the posterior of each t-batch and (mode != POSTERIOR) run the
 * fused q x q psd_safe_cholesky + reparameterised sampling + MC reduction:
 *   mean_out (B x q) = ymean + ystd (constant + R beta)
 *   cov_out (B x q x q) = ystd^2 (K** - R R^T)       [Standardize.untransform_posterior,
 *                                                     botorch/models/transforms/outcome.py:373-447]
 *   L_out (B x q x q), info_out (B), jitter_out (B)  [posteriors/gpytorch.py:85-126]
 *   acq (B): qEI  mean_s max_a relu(f - best_f)      [acquisition/monte_carlo.py:405-414]
 *            qNEI mean_s max_a relu(f - best_f_s[s])  [acquisition/monte_carlo.py:580-589]
 *            qLogEI / qLogNEI (best_f / best_f_s[s]):
 *              logmeanexp_s fatmax_a log_fatplus(f - best_f, tau_relu)   (fat != 0)
 *              logmeanexp_s smooth_amax_a log_softplus(f - best_f, tau_relu) (fat == 0)
 *              with the q-reduction at temperature tau_max
 *              [acquisition/logei.py:122, 219-234, 347-362, 509-534;
 *               utils/safe_math.py:209-352]; fat/tau_* are ignored by other modes
 * Z: S x q base samples (SobolQMCNormalSampler, sampling/normal.py:178-209).
 * Output pointers may be NULL when not needed (acq required for QEI/QNEI).
 * Cached-root qNEI (utils/low_rank.py:85-173, acquisition/cached_cholesky.py):
 * Tm (r x ldT) = L_rr^{-1} Sigma'(X_baseline, X) columns per padded test row,
 * F (S x ldF) = Z_baseline Tm; then Sigma'_qq <- Sigma'_qq - Tm^T Tm and
 * f = mean' + F + chol(.) Z (Z: the q new Sobol columns).  NULL otherwise. */
int bo_qmc_finalize(int kind, int mode, int B, int q, const double* Xq, const double* Spart,
                    const double* mpart, int64_t n, double outputscale, double constant,
                    double ymean, double ystd, const double* Z, int S, double best_f,
                    const double* best_f_s, int max_tries, double jitter0, double* acq,
                    double* mean_out, double* cov_out, double* L_out, int* info_out,
                    double* jitter_out, const double* Tm, int r, int64_t ldT, const double* F,
                    int64_t ldF, int fat, double tau_relu, double tau_max, void* stream);

/* Backward of the MC reduction + q x q Cholesky (gen_candidates_scipy's
 * autograd.grad, botorch/generation/gen.py:194-222):
 * dacq (B) -> dmean (B x q), dcov (B x q x q, symmetric) w.r.t. the outcome-
 * space posterior (mean', Sigma'), given mean' and L_q from bo_qmc_finalize.
 * mode: BO_QMC_QEI or BO_QMC_QNEI (best_f_s per sample).  torch semantics:
 * amax splits ties evenly, clamp_min(0) passes the gradient at >= 0.
 * qNEI (cached root, utils/low_rank.py:85-173): the forward samples include
 * F = Z_base T (S x ldF, rows b*Qp + a, as passed to bo_qmc_finalize); dF (same
 * layout) receives its cotangent, from which dT = Z_base^T dF.  F/dF may be
 * NULL for qEI.  Log modes (BO_QMC_QLOGEI / BO_QMC_QLOGNEI) also take the
 * forward values acq_fwd (B) and the forward's fat / tau_relu / tau_max; their
 * weights are dense over (sample, q) rather than one-hot. */
int bo_qmc_backward(int mode, int B, int q, const double* mean, const double* Lq,
                    const double* Z, int S, double best_f, const double* best_f_s,
                    const double* F, int64_t ldF, const double* dacq, double* dmean,
                    double* dcov, double* dF, const double* acq_fwd, int fat, double tau_relu,
                    double tau_max, void* stream);

/* Backward of the batched exact posterior w.r.t. the candidates X (B x q x d):
 *   dK*x = ystd dmean alpha^T - G W,  G = ystd^2 (dcov + dcov^T),
 *   W = R L^{-1} (nrows_pad x ldw, rows b*Qp + a; w_kmajor != 0: W^T as
 *   bo_post_w writes it, np x ldw), dK** = ystd^2 dcov,
 *   + E (optional extra dK*x, nrows_pad x lde, same rows: the qNEI cross-
 *     covariance terms),
 * reduced through dk/dx.  Xq / Xt_scaled as for bo_post_partials.  W, alpha,
 * dmean, dcov and E may each be NULL (term absent); accumulate != 0 adds into
 * dX.  With Xt_scaled = the qNEI baseline points and only E, this is the
 * gradient through K(X_baseline, X).  Caches carry no gradient ([G]
 * detach_test_caches, botorch/models/utils/assorted.py:286-298). */
int bo_post_backward(int kind, int B, int q, int d, const double* Xq, const double* Xt_scaled,
                     int64_t n, const double* W, int64_t ldw, const double* alpha,
                     const double* dmean, const double* dcov, const double* E, int64_t lde,
                     const double* lengthscale, double outputscale, double ystd, int accumulate,
                     double* dX, int w_kmajor, void* stream);

/* Kernel-matrix gradient for any d <= 128 (inputs in the original scale):
 *   dX[i][t] (+)= sum_k dK[i][k] d k(X_i, Y_k) / d X_it,
 * group > 0: row i pairs only with the `group` rows of its own block of Y
 * (dK row = group entries) -- the K** term of q-batches.  Generic-d path of
 * the posterior backward (SAAS, d = 50: models/fully_bayesian.py:509-546). */
int bo_kernel_grad(int kind, const double* X, int64_t rows, const double* Y, int64_t n, int d,
                   const double* lengthscale, double outputscale, const double* dK, int64_t ldk,
                   int group, int accumulate, double* dX, void* stream);

/* Exact-MLL terms for fit_gpytorch_mll (botorch/fit.py:75-258 ->
 * optim/closures/model_closures.py:171-184, [G] ExactMarginalLogLikelihood),
 * given bo_gp_cache_build's L, alpha, beta and Ainv = U U^T (lower triangle
 * read; ld = np).  partial: n x (d+5) per-row sums
 *   [0..d-1] sum_k w_ik W_ik outputscale g_ik (x_ij - x_kj)^2,   W = alpha alpha^T - Ainv
 *   [d]      W_ii        [d+1] sum_k w_ik W_ik kbar_ik   [d+2] log L_ii
 *   [d+3]    beta_i^2    [d+4] alpha_i          (w_ik = 2 for k < i, 1 for k = i)
 * from which the host forms the loss and its gradient in (ell, noise, constant,
 * outputscale) exactly. */
int bo_mll_terms(int kind, const double* X, int64_t n, int d, const double* lengthscale,
                 double outputscale, const double* L, const double* Ainv, int64_t ld,
                 const double* alpha, const double* beta, double* partial, void* stream);

/* qEHVI over hypercells ([lo, hi] K x m from the non-dominated partitioning,
 * botorch/acquisition/multi_objective/monte_carlo.py:230-317) for B t-batches of
 * q points of an m-output independent model (ModelListGP):
 *   f[s][p][t] = mean[t][b][p] + sum_j L[t][b][p][j] Z[s][j m + t]
 *   acq[b] = mean_s sum_k inclusion-exclusion volume.
 * mean: m x B x q, L: m x B x q x q, Z: S x (q m).  2 <= m <= 4, q <= 12.
 * cell_stride 0: one set of K cells for every sample; > 0 (qNEHVI,
 * NoisyExpectedHypervolumeMixin, botorch/utils/multi_objective/hypervolume.py:
 * 507-835): sample s reads its own cells at cell_lo/hi + s * cell_stride (padded
 * with empty cells as BoxDecompositionList does).  F (nullable): the cached-root
 * baseline term added to f (m x S x ldF, output stride sF, row b * Qp + p). */
int bo_qehvi(int B, int q, int m, const double* mean, const double* L, const double* Z, int S,
             const double* cell_lo, const double* cell_hi, int K, int64_t cell_stride,
             const double* F, int64_t ldF, int64_t sF, int Qp, double* acq, void* stream);

/* Backward of bo_qehvi (autograd through _compute_qehvi,
 * multi_objective/monte_carlo.py:230-317): dacq (B) -> dmean (m x B x q) and
 * dL (m x B x q x q, lower) of the per-output posterior roots, and (with F)
 * dF (the cotangent of F, same layout) from which dT = Z_base^T dF. */
int bo_qehvi_backward(int B, int q, int m, const double* mean, const double* L, const double* Z,
                      int S, const double* cell_lo, const double* cell_hi, int K,
                      int64_t cell_stride, const double* F, int64_t ldF, int64_t sF, int Qp,
                      const double* dacq, double* dmean, double* dL, double* dF, void* stream);

/* Batched Cholesky backward (torch linalg.cholesky backward): L, dL (B x q x q,
 * lower) -> dA (B x q x q, symmetric), q <= 64. */
int bo_chol_backward(int B, int q, const double* L, const double* dL, double* dA, void* stream);

/* MC qEI / qNEI reduction of given samples (S x B x q):
 * acq[b] = mean_s max(max_a samples[s][b][a] - bf_s, 0), bf_s = best_f_s[s] or best_f. */
int bo_mc_reduce(int S, int B, int q, const double* samples, double best_f,
                 const double* best_f_s, double* acq, void* stream);

/* Scrambled Sobol N(0,1) samples, points skip..skip+n-1: out (n x dim).
 * state: dim x 30 int64 scrambled direction numbers, shift: dim int64
 * (torch.quasirandom.SobolEngine(dim, scramble=True, seed) state).
 * first_f32: the engine's first point was formed in float32 (torch's default
 * dtype at construction), so point 0 is rounded through float32 like it.
 * Replaces draw_sobol_normal_samples (botorch/utils/sampling.py:108-137). */
int bo_sobol_normal(const int64_t* state, const int64_t* shift, int dim, int64_t n,
                    int64_t skip, int first_f32, double* out, void* stream);

/* The scrambled engine state itself: state (dim x 30) and shift (dim) of
 * SobolEngine(dim, scramble=True, seed) from state0 (dim x 30, the unscrambled
 * direction numbers, torch._sobol_engine_initialize_state_) and bits (uint8,
 * 0/1): the engine's two draws from its seeded generator, in order -- dim x 30
 * shift bits, then dim x 30 x 30 matrix bits.  Replaces SobolEngine._scramble
 * (torch/quasirandom.py; torch._sobol_engine_scramble_), which the reference's
 * samplers run at every construction (sampling/qmc.py:56). */
int bo_sobol_scramble(int dim, const int64_t* state0, const uint8_t* bits, int64_t* state,
                      int64_t* shift, void* stream);

/* One function evaluation of the device-resident multi-start projected L-BFGS
 * (replaces scipy L-BFGS-B in gen_candidates_scipy, botorch/generation/gen.py:
 * 194-267).  B restarts of dimension n, history m (<= 32).  The caller fills
 * ft (B) / gt (B x n) with the objective (-acq) and its gradient at the trial
 * points xt; the step accepts (Armijo, c1) or backtracks, updates x / f / g
 * and the (S, Y, rho) ring, tests convergence (status: 1 projected gradient
 * <= pgtol, 2 relative decrease <= ftol, 3 step below min_alpha; -1 on the first
 * call = take xt as the start), and writes the next trial points to xt.
 * x, g, xt, gt, d: B x n; S, Y: B x m x n; f, alpha: B; rho: B x m;
 * hcount, hhead, status, nacc (accepted steps): B int32; lower, upper: n. */
int bo_lbfgs_step(int B, int n, int m, double* x, double* f, double* g, double* xt,
                  const double* ft, const double* gt, double* d, double* alpha, double* S,
                  double* Y, double* rho, int* hcount, int* hhead, int* status, int* nacc,
                  const double* lower, const double* upper, double c1, double ftol,
                  double pgtol, double min_alpha, void* stream);

/* One function evaluation of the device-resident multi-start L-BFGS-B: scipy
 * 1.15's L-BFGS-B (generalized Cauchy point, subspace minimisation with the
 * v3.0 projection, More-Thuente line search; the optimiser of
 * gen_candidates_scipy, botorch/generation/gen.py:252-267) as a reverse-
 * communication state machine, one 64-lane wave per restart.  The caller
 * writes ft (B) / gt (B x n) = objective and gradient at the trial points xt
 * (B x n); the call advances every restart to its next evaluation and
 * overwrites xt.  Zeroed state (v, iv, ws, wy, mat, ds, is) means "start at
 * xt".  ftol / pgtol / maxls / maxiter / maxfun are scipy's options of the same
 * names (m = maxcor <= 20).  Per restart: v = V x n doubles, iv = IV x n ints,
 * ws / wy = m x n, mat = MAT doubles, ds = DS doubles, is = IS ints, with
 * (V, IV, MAT, DS, IS) from bo_lbfgsb_layout; is[1] is the status (0 running,
 * 1 projected gradient <= pgtol, 2 relative reduction <= ftol, 3 abnormal line
 * search, 4 maxiter, 5 maxfun, 6 error), is[10] the iterations, ds[0] f and
 * v[0..n) x. */
int bo_lbfgsb_step(int B, int n, int m, int maxls, int maxiter, int maxfun, double ftol,
                   double pgtol, const double* lower, const double* upper, double* xt,
                   const double* ft, const double* gt, double* v, int* iv, double* ws, double* wy,
                   double* mat, double* ds, int* is, void* stream);
/* HOST: out[0..5] = V, IV, MAT, DS, IS, maximum m. */
int bo_lbfgsb_layout(int* out);
/* Profiling aid: subsequent bo_lbfgsb_step launches of at most `capacity`
 * restarts add each restart's phase times (wall-clock ticks: load, Cauchy
 * point, free set, formk, cmprlb, subsm, line search + update, store) into prof
 * (capacity x 8, device memory); larger launches are not profiled; NULL stops. */
int bo_lbfgsb_set_profile(unsigned long long* prof, int capacity);
/* Timing aid: 0 keeps every restart's working set in HBM; 1 (default) stages it
 * in LDS for each launch when it fits (8 (10 + 2m) n + 8 n bytes <= ~40 KB). */
int bo_lbfgsb_set_staging(int on);
/* Route of a single restart (B == 1, the joint problem of
 * gen_candidates_device(joint=True)): 0 (default) runs n >= 2048 on the
 * grid-wide kernel (one workgroup per 256 variables, the S / Y ring in LDS;
 * n <= 16384 and maxcor small enough for its LDS), 1 every single restart
 * that fits, -1 never (the one-workgroup kernel).  Same state layout. */
int bo_lbfgsb_set_grid(int mode);
/* Number of grid-wide L-BFGS-B launches this process has made (tests assert
 * the route). */
int64_t bo_lbfgsb_grid_launches(void);

/* HOST function (plain host pointers; no GPU involved): exact non-dominated
 * box decompositions of S point sets Y (S x n x m, maximisation) w.r.t. ref (m),
 * FastNondominatedPartitioning per set (botorch/utils/multi_objective/
 * box_decompositions/non_dominated.py:353-457, utils.py:103-288), padded with
 * empty all-zero cells to the common maximum K (box_decomposition_list.py:
 * 62-94).  *K_out receives K; with cell_lo / cell_hi NULL the call only sizes,
 * else they receive S x K_cap x m (BO_ERR_ARG if K > K_cap).  The per-sample
 * decompositions of qNEHVI (utils/multi_objective/hypervolume.py:680-700) run
 * on `nthreads` host threads. */
int bo_nd_partition_host(const double* Y, int64_t S, int64_t n, int m, const double* ref,
                         int64_t K_cap, int64_t* K_out, double* cell_lo, double* cell_hi,
                         int nthreads);

/* HOST function: bo_nd_partition_host's contract with NondominatedPartitioning's
 * binary partitioning instead (botorch/utils/multi_objective/box_decompositions/
 * non_dominated.py:81-192 + get_hypercell_bounds :248-335): cells that straddle
 * the front are halved until adjacent, and with alpha > 0 dropped once their
 * volume is at most alpha of the box around the front (the approximate
 * decomposition qNEHVI uses for alpha > 0, m > 2:
 * utils/multi_objective/hypervolume.py:606-612, 744-758). */
int bo_nd_partition_alpha_host(const double* Y, int64_t S, int64_t n, int m, const double* ref,
                               double alpha, int64_t K_cap, int64_t* K_out, double* cell_lo,
                               double* cell_hi, int nthreads);

/* HOST function (plain host pointers; no GPU involved): the hit-and-run chain
 * of sample_polytope (botorch/utils/sampling.py:219-309) over {y : A y <= b}
 * (A m x k row-major, b m), from y0 (k).  Step t moves along the unit direction
 * R[t] (n_tot x k) by lo + u[t] (hi - lo), [lo, hi] the feasible segment from
 * the slacks max(b - A y, 0) / AR[t] (AR = R A^T, n_tot x m, made by the caller
 * with torch as the reference makes it); after n0 burn-in steps every n_thin-th
 * point goes to out (n x k); n_tot must equal n0 + n * n_thin.  Replaces the
 * Python loop at sampling.py:278-308 that gen_batch_initial_conditions runs
 * under linear constraints (optim/initializers.py:365-375). */
int bo_hit_and_run_host(const double* A, const double* b, int64_t m, int64_t k, const double* y0,
                        const double* R, const double* AR, const double* u, int64_t n_tot,
                        int64_t n0, int64_t n_thin, double* out, int64_t n);

/* Scrambled Sobol raw designs in a box, points skip..skip+n-1: out (n x dim),
 * dim = q * d, out[i][j] = lower[j % d] + range[j % d] * u_i[j] (device
 * lower/range of length d).  Same engine state as bo_sobol_normal.
 * Replaces draw_sobol_samples (botorch/utils/sampling.py:66-105) in
 * gen_batch_initial_conditions (botorch/optim/initializers.py:350-362). */
int bo_sobol_box(const int64_t* state, const int64_t* shift, int dim, int64_t n, int64_t skip,
                 int first_f32, const double* lower, const double* range, int d, double* out,
                 void* stream);

/* ---- Parameter-struct entry points (ABI 9; ABI 10 adds rt_layout, ABI 11 the
 * quad-plan and fused-status fields of BoQmcFinalizeArgs) ------------------------
 * The widest calls above also take one struct of named fields, so a binding
 * declares a record instead of a positional list of 20-33 arguments.  Every
 * struct opens with struct_size = sizeof(struct) and abi_version =
 * BO_ABI_VERSION; a mismatch returns BO_ERR_ARG (never a misread field).  Field
 * meanings are those of the positional function named in each comment; each
 * _v function forwards to it. */
#define BO_STRUCT_HEADER \
  uint32_t struct_size;  \
  uint32_t abi_version

typedef struct BoPostPartialsArgs { /* bo_post_partials */
  BO_STRUCT_HEADER;
  int32_t kind, B, q, d;
  const double* Xq;
  const double* Xt_scaled;
  int64_t n;
  const double* U;
  int64_t ldu;
  const double* beta;
  double outputscale;
  double *Spart, *mpart, *Rt;
  int32_t kc_len, rq;
  double* work;
  const double* Qc;
  int64_t ldq;
  double* Cx;
  const double* Kt;
  int32_t rt_layout, _pad; /* ABI 10: BO_RT_ROWMAJOR or BO_RT_BLOCKED (the layout of Rt) */
} BoPostPartialsArgs;
int bo_post_partials_v(const BoPostPartialsArgs* a, void* stream);

typedef struct BoQmcFinalizeArgs { /* bo_qmc_finalize */
  BO_STRUCT_HEADER;
  int32_t kind, mode, B, q;
  const double *Xq, *Spart, *mpart;
  int64_t n;
  double outputscale, constant, ymean, ystd;
  const double* Z;
  int32_t S, max_tries;
  double best_f;
  const double* best_f_s;
  double jitter0;
  double *acq, *mean_out, *cov_out, *L_out;
  int* info_out;
  double* jitter_out;
  const double* Tm;
  int32_t r, fat;
  int64_t ldT;
  const double* F;
  int64_t ldF;
  double tau_relu, tau_max;
  /* ABI 11.  nparts: the number of partials in Spart / mpart (0: the column
   * tiles of bo_post_geometry); sym_parts = 1: the quad plan's partials
   * (bo_post_quad), summed as P + P^T.  status_out (2 doubles) + status_count
   * (one int, zero before the first call): the batch's [max info, max jitter]
   * of bo_ladder_status computed by the same launch (the last workgroup to
   * finish reduces them and re-zeroes the counter); null: not computed. */
  int32_t nparts, sym_parts;
  double* status_out;
  int32_t* status_count;
} BoQmcFinalizeArgs;
int bo_qmc_finalize_v(const BoQmcFinalizeArgs* a, void* stream);

typedef struct BoQmcBackwardArgs { /* bo_qmc_backward */
  BO_STRUCT_HEADER;
  int32_t mode, B, q, S;
  const double *mean, *Lq, *Z;
  double best_f;
  const double *best_f_s, *F;
  int64_t ldF;
  const double* dacq;
  double *dmean, *dcov, *dF;
  const double* acq_fwd;
  int32_t fat, _pad;
  double tau_relu, tau_max;
} BoQmcBackwardArgs;
int bo_qmc_backward_v(const BoQmcBackwardArgs* a, void* stream);

typedef struct BoPostBackwardArgs { /* bo_post_backward */
  BO_STRUCT_HEADER;
  int32_t kind, B, q, d;
  const double *Xq, *Xt_scaled;
  int64_t n;
  const double* W;
  int64_t ldw;
  const double *alpha, *dmean, *dcov, *E;
  int64_t lde;
  const double* lengthscale;
  double outputscale, ystd;
  int32_t accumulate, w_kmajor;
  double* dX;
} BoPostBackwardArgs;
int bo_post_backward_v(const BoPostBackwardArgs* a, void* stream);
/* njobs <= 16 posterior backward passes of one (B, q, d, kind) in one launch
 * (a ModelListGP's members, each with its training and baseline passes):
 * job j's dX (its dX / accumulate fields ignored) is written to dX_parts + j B q d;
 * the caller sums the slices. */
int bo_post_backward_jobs(int njobs, const BoPostBackwardArgs* const* jobs, double* dX_parts,
                          void* stream);

typedef struct BoQehviArgs { /* bo_qehvi and bo_qehvi_backward (d* fields: backward only) */
  BO_STRUCT_HEADER;
  int32_t B, q, m, S;
  const double *mean, *L, *Z, *cell_lo, *cell_hi;
  int32_t K, Qp;
  int64_t cell_stride;
  const double* F;
  int64_t ldF, sF;
  double* acq;
  const double* dacq;
  double *dmean, *dL, *dF;
  /* ABI 11 (optional): a workspace lets the samples of each t-batch split
   * over several workgroups when B leaves CUs idle -- forward >= 2 B doubles,
   * backward >= 2 B m q (q + 3) / 2 */
  double* work;
  int64_t work_elems;
} BoQehviArgs;
int bo_qehvi_v(const BoQehviArgs* a, void* stream);
int bo_qehvi_backward_v(const BoQehviArgs* a, void* stream);

typedef struct BoLbfgsStepArgs { /* bo_lbfgs_step */
  BO_STRUCT_HEADER;
  int32_t B, n, m, _pad;
  double *x, *f, *g, *xt;
  const double *ft, *gt;
  double *d, *alpha, *S, *Y, *rho;
  int *hcount, *hhead, *status, *nacc;
  const double *lower, *upper;
  double c1, ftol, pgtol, min_alpha;
} BoLbfgsStepArgs;
int bo_lbfgs_step_v(const BoLbfgsStepArgs* a, void* stream);

typedef struct BoLbfgsbArgs { /* bo_lbfgsb_step */
  BO_STRUCT_HEADER;
  int32_t B, n, m, maxls, maxiter, maxfun;
  double ftol, pgtol;
  const double *lower, *upper;
  double* xt;
  const double *ft, *gt;
  double* v;
  int* iv;
  double *ws, *wy, *mat, *ds;
  int* is;
} BoLbfgsbArgs;
int bo_lbfgsb_step_v(const BoLbfgsbArgs* a, void* stream);

/* HOST: sizeof the named record ("BoPostPartialsArgs", ...), -1 if unknown --
 * lets a binding check its declared layout once at load time. */
int64_t bo_struct_size(const char* name);

#ifdef __cplusplus
}
#endif

#endif /* BOTORCH_AMD_H */
