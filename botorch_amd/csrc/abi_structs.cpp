// Parameter-struct entry points of the C ABI (include/botorch_amd.h, ABI 9-11):
// each validates the struct header and forwards to the positional function.
// Host code only (g++): no device work of its own.
#include <cstdio>
#include <string>

#include "../../include/botorch_amd.h"

void bo_set_error(const char* fmt, ...);

namespace {

template <class T>
bool header_ok(const T* a, const char* name) {
  if (!a) {
    bo_set_error("%s: null argument struct", name);
    return false;
  }
  if (a->struct_size != sizeof(T) || a->abi_version != BO_ABI_VERSION) {
    bo_set_error("%s: struct size %u / ABI %u, library expects %zu / %d", name, a->struct_size,
                 a->abi_version, sizeof(T), BO_ABI_VERSION);
    return false;
  }
  return true;
}

}  // namespace

extern "C" {

// bo_post_partials with the R^T layout of ABI 10 (post.hip)
int bo_post_partials_layout(int kind, const double* Xq, int B, int q, int d,
                            const double* Xt_scaled, int64_t n, const double* U, int64_t ldu,
                            const double* beta, double outputscale, double* Spart, double* mpart,
                            double* Rt, int kc_len, double* work, const double* Qc, int rq,
                            int64_t ldq, double* Cx, const double* Kt, int rt_layout, void* stream);

// bo_qmc_finalize with the quad-plan partials and the fused ladder status of
// ABI 11 (qmc.hip)
int bo_qmc_finalize_ext(int kind, int mode, int B, int q, const double* Xq, const double* Spart,
                        const double* mpart, int64_t n, double outputscale, double constant,
                        double ymean, double ystd, const double* Z, int S, double best_f,
                        const double* best_f_s, int max_tries, double jitter0, double* acq,
                        double* mean_out, double* cov_out, double* L_out, int* info_out,
                        double* jitter_out, const double* Tm, int r, int64_t ldT, const double* F,
                        int64_t ldF, int fat, double tau_relu, double tau_max, int nparts,
                        int sym_parts, double* status_out, int* status_count, void* stream);

// bo_qehvi with the sample-split workspace of ABI 11 (qehvi.hip)
int bo_qehvi_ext(int B, int q, int m, const double* mean, const double* L, const double* Z, int S,
                 const double* cell_lo, const double* cell_hi, int K, int64_t cell_stride,
                 const double* F, int64_t ldF, int64_t sF, int Qp, double* acq, double* work,
                 int64_t work_elems, void* stream);

int bo_qehvi_backward_ext(int B, int q, int m, const double* mean, const double* L, const double* Z,
                          int S, const double* cell_lo, const double* cell_hi, int K,
                          int64_t cell_stride, const double* F, int64_t ldF, int64_t sF, int Qp,
                          const double* dacq, double* dmean, double* dL, double* dF, double* work,
                          int64_t work_elems, void* stream);

int bo_post_partials_v(const BoPostPartialsArgs* a, void* stream) {
  if (!header_ok(a, "bo_post_partials_v")) return BO_ERR_ARG;
  return bo_post_partials_layout(a->kind, a->Xq, a->B, a->q, a->d, a->Xt_scaled, a->n, a->U,
                                 a->ldu, a->beta, a->outputscale, a->Spart, a->mpart, a->Rt,
                                 a->kc_len, a->work, a->Qc, a->rq, a->ldq, a->Cx, a->Kt,
                                 a->rt_layout, stream);
}

int bo_qmc_finalize_v(const BoQmcFinalizeArgs* a, void* stream) {
  if (!header_ok(a, "bo_qmc_finalize_v")) return BO_ERR_ARG;
  return bo_qmc_finalize_ext(a->kind, a->mode, a->B, a->q, a->Xq, a->Spart, a->mpart, a->n,
                             a->outputscale, a->constant, a->ymean, a->ystd, a->Z, a->S,
                             a->best_f, a->best_f_s, a->max_tries, a->jitter0, a->acq,
                             a->mean_out, a->cov_out, a->L_out, a->info_out, a->jitter_out, a->Tm,
                             a->r, a->ldT, a->F, a->ldF, a->fat, a->tau_relu, a->tau_max,
                             a->nparts, a->sym_parts, a->status_out, a->status_count, stream);
}

int bo_qmc_backward_v(const BoQmcBackwardArgs* a, void* stream) {
  if (!header_ok(a, "bo_qmc_backward_v")) return BO_ERR_ARG;
  return bo_qmc_backward(a->mode, a->B, a->q, a->mean, a->Lq, a->Z, a->S, a->best_f, a->best_f_s,
                         a->F, a->ldF, a->dacq, a->dmean, a->dcov, a->dF, a->acq_fwd, a->fat,
                         a->tau_relu, a->tau_max, stream);
}

int bo_post_backward_v(const BoPostBackwardArgs* a, void* stream) {
  if (!header_ok(a, "bo_post_backward_v")) return BO_ERR_ARG;
  return bo_post_backward(a->kind, a->B, a->q, a->d, a->Xq, a->Xt_scaled, a->n, a->W, a->ldw,
                          a->alpha, a->dmean, a->dcov, a->E, a->lde, a->lengthscale,
                          a->outputscale, a->ystd, a->accumulate, a->dX, a->w_kmajor, stream);
}

int bo_qehvi_v(const BoQehviArgs* a, void* stream) {
  if (!header_ok(a, "bo_qehvi_v")) return BO_ERR_ARG;
  return bo_qehvi_ext(a->B, a->q, a->m, a->mean, a->L, a->Z, a->S, a->cell_lo, a->cell_hi, a->K,
                      a->cell_stride, a->F, a->ldF, a->sF, a->Qp, a->acq, a->work, a->work_elems,
                      stream);
}

int bo_qehvi_backward_v(const BoQehviArgs* a, void* stream) {
  if (!header_ok(a, "bo_qehvi_backward_v")) return BO_ERR_ARG;
  return bo_qehvi_backward_ext(a->B, a->q, a->m, a->mean, a->L, a->Z, a->S, a->cell_lo,
                               a->cell_hi, a->K, a->cell_stride, a->F, a->ldF, a->sF, a->Qp,
                               a->dacq, a->dmean, a->dL, a->dF, a->work, a->work_elems, stream);
}

int bo_lbfgs_step_v(const BoLbfgsStepArgs* a, void* stream) {
  if (!header_ok(a, "bo_lbfgs_step_v")) return BO_ERR_ARG;
  return bo_lbfgs_step(a->B, a->n, a->m, a->x, a->f, a->g, a->xt, a->ft, a->gt, a->d, a->alpha,
                       a->S, a->Y, a->rho, a->hcount, a->hhead, a->status, a->nacc, a->lower,
                       a->upper, a->c1, a->ftol, a->pgtol, a->min_alpha, stream);
}

int bo_lbfgsb_step_v(const BoLbfgsbArgs* a, void* stream) {
  if (!header_ok(a, "bo_lbfgsb_step_v")) return BO_ERR_ARG;
  return bo_lbfgsb_step(a->B, a->n, a->m, a->maxls, a->maxiter, a->maxfun, a->ftol, a->pgtol,
                        a->lower, a->upper, a->xt, a->ft, a->gt, a->v, a->iv, a->ws, a->wy, a->mat,
                        a->ds, a->is, stream);
}

}  // extern "C"

// sizeof of each argument record (HOST, for bindings to verify their layouts).
extern "C" int64_t bo_struct_size(const char* name) {
  const std::string s = name ? name : "";
  if (s == "BoPostPartialsArgs") return sizeof(BoPostPartialsArgs);
  if (s == "BoQmcFinalizeArgs") return sizeof(BoQmcFinalizeArgs);
  if (s == "BoQmcBackwardArgs") return sizeof(BoQmcBackwardArgs);
  if (s == "BoPostBackwardArgs") return sizeof(BoPostBackwardArgs);
  if (s == "BoQehviArgs") return sizeof(BoQehviArgs);
  if (s == "BoLbfgsStepArgs") return sizeof(BoLbfgsStepArgs);
  if (s == "BoLbfgsbArgs") return sizeof(BoLbfgsbArgs);
  return -1;
}
