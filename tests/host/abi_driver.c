/* A non-Python caller of include/botorch_amd.h: plain C99, linked against
 * botorch_amd/libbotorch_amd.so (and, for the device part, the HIP runtime's
 * C API).  Test infrastructure (tests/test_abi_c.py builds and runs it).
 *
 *   abi_driver host  -- ABI version, every parameter record's size as this
 *                       compiler lays it out vs. bo_struct_size, a
 *                       box decomposition through bo_nd_partition_host, and
 *                       an argument error reported through bo_last_error.
 *   abi_driver gpu   -- the device L-BFGS-B (bo_lbfgsb_step_v) minimising a
 *                       box-constrained quadratic for 64 restarts, with the
 *                       objective evaluated on the host: device memory from
 *                       hipMalloc, no PyTorch anywhere.
 * Prints "ok ..." lines and exits 0, or prints the failure and exits 1. */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/botorch_amd.h"

#define FAIL(...)                     \
  do {                                \
    fprintf(stderr, "FAIL: ");        \
    fprintf(stderr, __VA_ARGS__);     \
    fprintf(stderr, "\n");            \
    return 1;                         \
  } while (0)

#define CHECK_SIZE(T)                                                                    \
  do {                                                                                   \
    if (bo_struct_size(#T) != (int64_t)sizeof(T))                                        \
      FAIL("%s: library %lld vs C %zu", #T, (long long)bo_struct_size(#T), sizeof(T)); \
  } while (0)

static int host_checks(void) {
  if (bo_version() != BO_ABI_VERSION) FAIL("ABI %d vs header %d", bo_version(), BO_ABI_VERSION);
  CHECK_SIZE(BoPostPartialsArgs);
  CHECK_SIZE(BoQmcFinalizeArgs);
  CHECK_SIZE(BoQmcBackwardArgs);
  CHECK_SIZE(BoPostBackwardArgs);
  CHECK_SIZE(BoQehviArgs);
  CHECK_SIZE(BoLbfgsStepArgs);
  CHECK_SIZE(BoLbfgsbArgs);
  if (bo_struct_size("NoSuchRecord") != -1) FAIL("unknown record size");
  printf("ok records\n");

  /* two objectives, Pareto set {(1,3), (2,2), (3,1)}, ref (0,0): the
   * non-dominated region below the front is covered by cells whose volumes
   * sum to the hypervolume 6 */
  const double Y[6] = {1, 3, 2, 2, 3, 1};
  const double ref[2] = {0, 0};
  int64_t K = 0;
  if (bo_nd_partition_host(Y, 1, 3, 2, ref, 0, &K, NULL, NULL, 1) != BO_OK)
    FAIL("nd_partition sizing: %s", bo_last_error());
  double* lo = (double*)malloc(sizeof(double) * K * 2);
  double* hi = (double*)malloc(sizeof(double) * K * 2);
  if (bo_nd_partition_host(Y, 1, 3, 2, ref, K, &K, lo, hi, 1) != BO_OK)
    FAIL("nd_partition: %s", bo_last_error());
  /* FastNondominatedPartitioning cells cover the region no Pareto point
   * dominates: in two objectives the n + 1 = 4 strips between and beyond the
   * three points (upper bounds +inf), none with a point strictly inside */
  if (K != 4) FAIL("K = %lld cells, expected 4", (long long)K);
  for (int64_t k = 0; k < K; ++k)
    for (int p = 0; p < 3; ++p) {
      const int inside = Y[2 * p] > lo[2 * k] && Y[2 * p] < hi[2 * k] &&
                         Y[2 * p + 1] > lo[2 * k + 1] && Y[2 * p + 1] < hi[2 * k + 1];
      if (inside) FAIL("point %d inside cell %lld", p, (long long)k);
      if (lo[2 * k] < ref[0] || lo[2 * k + 1] < ref[1]) FAIL("cell %lld below ref", (long long)k);
    }
  free(lo);
  free(hi);
  printf("ok nd_partition K=%lld\n", (long long)K);

  /* argument errors come back as a status plus a message */
  BoLbfgsbArgs bad;
  memset(&bad, 0, sizeof bad);
  bad.struct_size = sizeof bad;
  bad.abi_version = BO_ABI_VERSION + 1;
  if (bo_lbfgsb_step_v(&bad, NULL) == BO_OK) FAIL("a wrong abi_version was accepted");
  if (strlen(bo_last_error()) == 0) FAIL("empty error message");
  printf("ok errors: %s\n", bo_last_error());
  return 0;
}

/* ---- device part: HIP runtime C API ---- */
typedef int hipError_t;
extern hipError_t hipMalloc(void** ptr, size_t size);
extern hipError_t hipFree(void* ptr);
extern hipError_t hipMemcpy(void* dst, const void* src, size_t size, int kind);
extern hipError_t hipMemset(void* dst, int value, size_t size);
extern hipError_t hipDeviceSynchronize(void);
enum { H2D = 1, D2H = 2 };

static void* dalloc(size_t bytes) {
  void* p = NULL;
  if (hipMalloc(&p, bytes) != 0) return NULL;
  hipMemset(p, 0, bytes);
  return p;
}

static int gpu_checks(void) {
  enum { B = 64, N = 12, M = 10 };
  int lay[6];
  bo_lbfgsb_layout(lay);
  const int NV = lay[0], NIV = lay[1], NMAT = lay[2], NDS = lay[3], NIS = lay[4];
  double target[N], lower[N], upper[N], xt[B * N], ft[B], gt[B * N], x[B * N];
  int is[B * 16];
  for (int i = 0; i < N; ++i) {
    target[i] = -0.5 + 0.2 * i; /* partly outside [0, 1]: active bounds */
    lower[i] = 0.0;
    upper[i] = 1.0;
  }
  unsigned s = 12345u;
  for (int k = 0; k < B * N; ++k) {
    s = s * 1103515245u + 12345u;
    xt[k] = (double)((s >> 8) & 0xffff) / 65535.0;
  }
  double *d_lo = dalloc(sizeof lower), *d_hi = dalloc(sizeof upper), *d_xt = dalloc(sizeof xt);
  double *d_ft = dalloc(sizeof ft), *d_gt = dalloc(sizeof gt);
  double* d_v = dalloc(sizeof(double) * B * NV * N);
  int* d_iv = dalloc(sizeof(int) * B * NIV * N);
  double *d_ws = dalloc(sizeof(double) * B * M * N), *d_wy = dalloc(sizeof(double) * B * M * N);
  double *d_mat = dalloc(sizeof(double) * B * NMAT), *d_ds = dalloc(sizeof(double) * B * NDS);
  int* d_is = dalloc(sizeof(int) * B * NIS);
  if (!d_lo || !d_is) FAIL("hipMalloc");
  hipMemcpy(d_lo, lower, sizeof lower, H2D);
  hipMemcpy(d_hi, upper, sizeof upper, H2D);
  hipMemcpy(d_xt, xt, sizeof xt, H2D);
  BoLbfgsbArgs a;
  memset(&a, 0, sizeof a);
  a.struct_size = sizeof a;
  a.abi_version = BO_ABI_VERSION;
  a.B = B; a.n = N; a.m = M; a.maxls = 20; a.maxiter = 2000; a.maxfun = 15000;
  a.ftol = 2.2204460492503131e-09; a.pgtol = 1e-5;
  a.lower = d_lo; a.upper = d_hi; a.xt = d_xt; a.ft = d_ft; a.gt = d_gt;
  a.v = d_v; a.iv = d_iv; a.ws = d_ws; a.wy = d_wy; a.mat = d_mat; a.ds = d_ds; a.is = d_is;
  int evals = 0, all_done = 0;
  for (; evals < 200 && !all_done; ++evals) {
    hipMemcpy(xt, d_xt, sizeof xt, D2H);
    for (int b = 0; b < B; ++b) { /* f = sum (x - target)^2 * (1 + i/N) */
      double f = 0.0;
      for (int i = 0; i < N; ++i) {
        const double w = 1.0 + (double)i / N, r = xt[b * N + i] - target[i];
        f += w * r * r;
        gt[b * N + i] = 2.0 * w * r;
      }
      ft[b] = f;
    }
    hipMemcpy(d_ft, ft, sizeof ft, H2D);
    hipMemcpy(d_gt, gt, sizeof gt, H2D);
    if (bo_lbfgsb_step_v(&a, NULL) != BO_OK) FAIL("bo_lbfgsb_step_v: %s", bo_last_error());
    hipMemcpy(is, d_is, sizeof(int) * B * NIS, D2H);
    all_done = 1;
    for (int b = 0; b < B; ++b)
      if (is[b * NIS + 1] == 0) all_done = 0;
  }
  hipDeviceSynchronize();
  if (!all_done) FAIL("not converged after %d evaluations", evals);
  /* x = v[0..n) of each restart */
  for (int b = 0; b < B; ++b) hipMemcpy(x + b * N, d_v + (size_t)b * NV * N, sizeof(double) * N, D2H);
  double err = 0.0;
  for (int b = 0; b < B; ++b)
    for (int i = 0; i < N; ++i) {
      const double sol = fmin(fmax(target[i], 0.0), 1.0);
      err = fmax(err, fabs(x[b * N + i] - sol));
    }
  /* stopped by pgtol = 1e-5 or the relative reduction test: |x - x*| <= ~1e-5 */
  for (int b = 0; b < B; ++b)
    if (is[b * NIS + 1] != 1 && is[b * NIS + 1] != 2) FAIL("restart %d status %d", b, is[b * NIS + 1]);
  if (err > 1e-4) FAIL("max |x - clamp(target)| = %g", err);
  printf("ok gpu lbfgsb: %d restarts, %d evaluations, max err %.2e\n", B, evals, err);
  hipFree(d_lo); hipFree(d_hi); hipFree(d_xt); hipFree(d_ft); hipFree(d_gt); hipFree(d_v);
  hipFree(d_iv); hipFree(d_ws); hipFree(d_wy); hipFree(d_mat); hipFree(d_ds); hipFree(d_is);
  return 0;
}

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "host";
  if (!strcmp(mode, "host")) return host_checks();
  if (!strcmp(mode, "gpu")) return host_checks() || gpu_checks();
  fprintf(stderr, "usage: %s host|gpu\n", argv[0]);
  return 2;
}
