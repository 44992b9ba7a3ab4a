"""PyTorch custom operators (``torch.ops.bo.*``) over the C ABI.

SURVEY.md section 8(b) asks for the hot path "bound as PyTorch-ROCm custom
ops": this module registers them with ``torch.library`` (schema, ROCm kernel,
fake/meta implementation for tracing, and an autograd formula for the
differentiable ones).  The model and acquisition classes call these ops; each
op's implementation is the ctypes binding of ``include/botorch_amd.h`` through
``botorch_amd.kernels`` (device pointers, the current HIP stream), so the ops
and the C ABI are one path, not two.

Ops (reference computation each replaces):
  bo::sobol_normal    SobolEngine + NormalQMCEngine draw        (sampling/qmc.py:60-98)
  bo::gp_cache        L, L^{-1}, L^{-T}, beta, alpha (+ jitter)  ([G] prediction caches,
                                                                 models/gpytorch.py:446)
  bo::chol_jitter     psd_safe_cholesky of a batch (+ autograd)  ([G] psd_safe_cholesky)
  bo::post_partials   column-tile partials of R R^T and R beta  ([G] exact_predictive_covar)
  bo::qmc_finalize    posterior moments / q x q root / MC reduction
  bo::gp_posterior    outcome-space mean and covariance (+ autograd, posteriors/gpytorch.py)
  bo::qmc_acq         fused qEI / qLogEI value of B t-batches (+ autograd,
                      acquisition/monte_carlo.py:405-414, logei.py:137-234)
  bo::qehvi           inclusion-exclusion qEHVI on the hypercells (+ autograd,
                      multi_objective/monte_carlo.py:230-317)
  bo::mll             exact marginal log likelihood data term and its gradient
                      (optim/closures/model_closures.py:171-184)
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Tuple

import torch
from torch import Tensor

from . import _lib, kernels

F64 = torch.float64


def _geometry(B, q, n):
    """bo_post_geometry restated for symbolic shapes (the fake implementations
    run under tracing): (Qp, nrows_pad, nC) of B t-batches of q <= 16 points
    against n training points -- 16-row t-batch tiles padded to 128 rows,
    128-column training tiles."""
    Qp = 1
    while Qp < q:
        Qp *= 2
    return Qp, ((B * Qp + 127) // 128) * 128, (n + 127) // 128


def _padded(n: int) -> int:
    return ((n + 127) // 128) * 128


def _cache_from(Xt, Xt_scaled, lengthscale, U, beta, alpha, kind, outputscale, constant,
                Linv=None) -> kernels.GPCache:
    n, d = Xt.shape
    np_ = U.shape[0]
    empty = U.new_empty(0)
    return kernels.GPCache(kind, n, d, np_, Xt, Xt_scaled, lengthscale, float(outputscale), 0.0,
                           float(constant), empty, Linv if Linv is not None else empty, U, beta,
                           alpha, 0.0)


def _pp_from(B, q, n, Xq, Spart, mpart, Rt) -> kernels.PostPartials:
    Qp, nrows_pad, nC = kernels.geometry(B, q, n)
    return kernels.PostPartials(B, q, Qp, nrows_pad, nC, Xq, Spart, mpart,
                                Rt if Rt.numel() else None)


# ---- bo::sobol_normal ------------------------------------------------------------------
@torch.library.custom_op("bo::sobol_normal", mutates_args=(), device_types="cuda")
def sobol_normal(state: Tensor, shift: Tensor, n: int, skip: int, first_f32: bool) -> Tensor:
    """n x D standard-normal Sobol points from SobolEngine's scrambled direction
    numbers (state D x 30, int64) and digital shift (D, int64)."""
    dim = shift.shape[0]
    out = torch.empty(n, dim, dtype=F64, device=state.device)
    kernels.check(kernels.lib().bo_sobol_normal(kernels._p(state.contiguous()),
                                                kernels._p(shift.contiguous()), dim, n, skip,
                                                int(first_f32), kernels._p(out),
                                                kernels._stream(state.device)), "sobol_normal")
    return out


@sobol_normal.register_fake
def _(state, shift, n, skip, first_f32):
    return state.new_empty(n, shift.shape[0], dtype=F64)


# ---- bo::gp_cache --------------------------------------------------------------------------
@torch.library.custom_op("bo::gp_cache", mutates_args=(), device_types="cuda")
def gp_cache(Xt: Tensor, y: Tensor, lengthscale: Tensor, outputscale: float, noise: float,
             constant: float, kind: int, noise_vec: Optional[Tensor] = None
             ) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor]:
    """(L, L^{-1}, U = L^{-T}: np x np; beta, alpha: n; Xt_scaled: n x 8; jitter: 1).
    noise_vec (n): a fixed-noise likelihood's observed variances (noise ignored)."""
    c = kernels.build_gp_cache(Xt, y, lengthscale, noise if noise_vec is None else noise_vec,
                               constant, kind=kind,
                               outputscale=outputscale)
    jit = torch.full((1,), c.jitter, dtype=F64, device=Xt.device)
    return c.L, c.Linv, c.U, c.beta, c.alpha, c.Xt_scaled, jit


@gp_cache.register_fake
def _(Xt, y, lengthscale, outputscale, noise, constant, kind, noise_vec=None):
    n = Xt.shape[0]
    np_ = _padded(n)
    mk = lambda *s: Xt.new_empty(*s, dtype=F64)  # noqa: E731
    return mk(np_, np_), mk(np_, np_), mk(np_, np_), mk(n), mk(n), mk(n, kernels.DP), mk(1)


# ---- bo::chol_jitter -------------------------------------------------------------------------
@torch.library.custom_op("bo::chol_jitter", mutates_args=(), device_types="cuda")
def chol_jitter(A: Tensor) -> Tensor:
    """psd_safe_cholesky of (..., k, k): jitter ladder per member; NotPSDError
    (with the reference's message) when the ladder is exhausted."""
    return kernels.chol_jitter(A.contiguous())


@chol_jitter.register_fake
def _(A):
    return torch.empty_like(A)


@torch.library.custom_op("bo::chol_backward", mutates_args=(), device_types="cuda")
def chol_backward(L: Tensor, dL: Tensor) -> Tensor:
    """dA of A = L L^T (torch.linalg.cholesky's backward), batched, k <= 64."""
    q = L.shape[-1]
    batch = L.shape[:-2]
    dA = kernels.chol_backward(L.reshape(-1, q, q).contiguous(),
                               dL.reshape(-1, q, q).tril().contiguous())
    return dA.reshape(*batch, q, q)


@chol_backward.register_fake
def _(L, dL):
    return torch.empty_like(L)


def _chol_setup(ctx, inputs, output):
    ctx.save_for_backward(output)


def _chol_bwd(ctx, dL):
    (L,) = ctx.saved_tensors
    return torch.ops.bo.chol_backward(L, dL)


chol_jitter.register_autograd(_chol_bwd, setup_context=_chol_setup)


# ---- bo::post_partials / bo::qmc_finalize (the primitive posterior pair) ------------------------
@torch.library.custom_op("bo::post_partials", mutates_args=(), device_types="cuda")
def post_partials(X: Tensor, Xt: Tensor, Xt_scaled: Tensor, U: Tensor, beta: Tensor,
                  lengthscale: Tensor, kind: int, outputscale: float,
                  store_R: bool) -> Tuple[Tensor, Tensor, Tensor, Tensor]:
    """Column-tile partials of R R^T and R beta for X (B x q x d), R = K*x L^{-T}:
    (Spart nC x B Qp/16 x 16 x 16, mpart nC x B Qp, Xq B Qp x 8, R^T or empty)."""
    c = _cache_from(Xt, Xt_scaled, lengthscale, U, beta, beta, kind, outputscale, 0.0)
    pp = kernels.post_partials(c, X, store_R=store_R, small=False)  # the schema's nC partials
    Rt = pp.Rt if pp.Rt is not None else X.new_empty(0, dtype=F64)
    return pp.Spart, pp.mpart, pp.Xq, Rt


@post_partials.register_fake
def _(X, Xt, Xt_scaled, U, beta, lengthscale, kind, outputscale, store_R):
    B, q, _ = X.shape
    Qp, nrows_pad, nC = _geometry(B, q, Xt.shape[0])
    mk = lambda *s: X.new_empty(*s, dtype=F64)  # noqa: E731
    return (mk(nC, nrows_pad // 16, 16, 16), mk(nC, nrows_pad), mk(nrows_pad, kernels.DP),
            mk(nC * 128, nrows_pad) if store_R else mk(0))


@torch.library.custom_op("bo::qmc_finalize", mutates_args=(), device_types="cuda")
def qmc_finalize(Spart: Tensor, mpart: Tensor, Xq: Tensor, Z: Optional[Tensor],
                 best_f_s: Optional[Tensor], B: int, q: int, n: int, kind: int, mode: int,
                 outputscale: float, constant: float, ymean: float, ystd: float, best_f: float,
                 fat: bool, tau_relu: float, tau_max: float
                 ) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor, Tensor]:
    """Per t-batch: moments (outcome space), jittered q x q root and, in the MC
    modes, the acquisition value: (acq, mean, cov, L, info, jitter)."""
    pp = _pp_from(B, q, n, Xq, Spart, mpart, Xq.new_empty(0))
    c = kernels.GPCache(kind, n, 0, 0, Xq, Xq, Xq, float(outputscale), 0.0, float(constant),
                        Xq, Xq, Xq, Xq, Xq, 0.0)
    out = kernels.qmc_finalize(c, pp, mode, ymean, ystd, Z=Z, best_f=best_f, best_f_s=best_f_s,
                               want_mean=True, want_cov=True, want_L=True,
                               log_params=(fat, tau_relu, tau_max))
    def e(dtype=F64):
        return Xq.new_empty(0, dtype=dtype)
    return (out["acq"] if out["acq"] is not None else e(), out["mean"], out["cov"], out["L"],
            out["info"] if out["info"] is not None else e(torch.int32),
            out["jitter"] if out["jitter"] is not None else e())


@qmc_finalize.register_fake
def _(Spart, mpart, Xq, Z, best_f_s, B, q, n, kind, mode, outputscale, constant, ymean, ystd,
      best_f, fat, tau_relu, tau_max):
    mk = lambda *s: Xq.new_empty(*s, dtype=F64)  # noqa: E731
    mc = mode in (_lib.QMC_QEI, _lib.QMC_QNEI) + _lib.LOG_MODES
    post = mode == _lib.QMC_POSTERIOR
    return (mk(B) if mc else mk(0), mk(B, q), mk(B, q, q), mk(B, q, q),
            Xq.new_empty(0 if post else B, dtype=torch.int32), mk(0 if post else B))


# ---- bo::gp_posterior ----------------------------------------------------------------------
@torch.library.custom_op("bo::gp_posterior", mutates_args=(), device_types="cuda")
def gp_posterior(X: Tensor, Xt: Tensor, Xt_scaled: Tensor, U: Tensor, Linv: Tensor, beta: Tensor,
                 alpha: Tensor, lengthscale: Tensor, kind: int, outputscale: float,
                 constant: float, ymean: float, ystd: float, need_grad: bool
                 ) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor]:
    """(mean B x q, cov B x q x q) of the outcome-space exact posterior
    ([G] exact_predictive_mean/covar + Standardize.untransform_posterior), plus
    what the gradient needs when need_grad: (Xq, R^T, W) (else empty)."""
    c = _cache_from(Xt, Xt_scaled, lengthscale, U, beta, alpha, kind, outputscale, constant, Linv)
    pp = kernels.post_partials(c, X, store_R=need_grad)
    out = kernels.qmc_finalize(c, pp, _lib.QMC_POSTERIOR, ymean, ystd)
    if not need_grad:
        return (out["mean"], out["cov"], X.new_empty(0, dtype=F64), X.new_empty(0, dtype=F64),
                X.new_empty(0, dtype=F64))
    W = kernels.w_matrix(c, pp)
    Wt = W.t if W.kmajor else W.t.T.contiguous()  # stored k-major (np x B Qp) either way
    return out["mean"], out["cov"], pp.Xq, pp.Rt, Wt


@gp_posterior.register_fake
def _(X, Xt, Xt_scaled, U, Linv, beta, alpha, lengthscale, kind, outputscale, constant, ymean,
      ystd, need_grad):
    B, q, _ = X.shape
    mk = lambda *s: X.new_empty(*s, dtype=F64)  # noqa: E731
    if not need_grad:
        return mk(B, q), mk(B, q, q), mk(0), mk(0), mk(0)
    Qp, nrows_pad, nC = _geometry(B, q, Xt.shape[0])
    return (mk(B, q), mk(B, q, q), mk(nrows_pad, kernels.DP), mk(nC * 128, nrows_pad),
            mk(U.shape[0], nrows_pad))


@torch.library.custom_op("bo::gp_posterior_backward", mutates_args=(), device_types="cuda")
def gp_posterior_backward(dmean: Tensor, dcov: Tensor, Xq: Tensor, Rt: Tensor, Wt: Tensor,
                          Xt: Tensor, Xt_scaled: Tensor, alpha: Tensor, lengthscale: Tensor,
                          kind: int, outputscale: float, ystd: float, q: int) -> Tensor:
    """dX (B x q x d) of the posterior moments: dK*x = s dmean alpha^T - G W,
    reduced through dk/dx over the training points (bo_post_backward)."""
    B = dmean.shape[0]
    c = _cache_from(Xt, Xt_scaled, lengthscale, Wt, alpha, alpha, kind, outputscale, 0.0)
    pp = _pp_from(B, q, Xt.shape[0], Xq, Xq, Xq, Rt)
    return kernels.post_backward(c, pp, kernels.WMat(Wt, True), dmean.contiguous(),
                                 dcov.contiguous(), ystd)


@gp_posterior_backward.register_fake
def _(dmean, dcov, Xq, Rt, Wt, Xt, Xt_scaled, alpha, lengthscale, kind, outputscale, ystd, q):
    return dmean.new_empty(dmean.shape[0], q, Xt.shape[1])


def _post_setup(ctx, inputs, output):
    X, Xt, Xt_scaled, U, Linv, beta, alpha, lengthscale, kind, outputscale, constant, ymean, ystd, \
        need_grad = inputs
    _, _, Xq, Rt, Wt = output
    # the saved intermediates carry no gradient: without this autograd would
    # zero-fill a grad for each of them (R^T and W^T: 268 MB each at C3)
    ctx.mark_non_differentiable(Xq, Rt, Wt)
    ctx.set_materialize_grads(False)
    ctx.save_for_backward(Xq, Rt, Wt, Xt, Xt_scaled, alpha, lengthscale)
    ctx.meta = (kind, outputscale, ystd, X.shape[0], X.shape[1])


def _post_bwd(ctx, dmean, dcov, *_):
    Xq, Rt, Wt, Xt, Xt_scaled, alpha, lengthscale = ctx.saved_tensors
    kind, outputscale, ystd, B, q = ctx.meta
    if Rt.numel() == 0:
        raise RuntimeError("bo::gp_posterior was called with need_grad=False")
    if dmean is None and dcov is None:
        return (None,) * 14
    if dmean is None:
        dmean = Wt.new_zeros(B, q)
    if dcov is None:
        dcov = Wt.new_zeros(B, q, q)
    dX = torch.ops.bo.gp_posterior_backward(dmean, dcov, Xq, Rt, Wt, Xt, Xt_scaled, alpha,
                                            lengthscale, kind, outputscale, ystd, q)
    return (dX,) + (None,) * 13


gp_posterior.register_autograd(_post_bwd, setup_context=_post_setup)


# ---- bo::qmc_acq (fused qEI / qLogEI) -------------------------------------------------------
@torch.library.custom_op("bo::qmc_acq", mutates_args=(), device_types="cuda")
def qmc_acq(X: Tensor, Xt: Tensor, Xt_scaled: Tensor, U: Tensor, Linv: Tensor, beta: Tensor,
            alpha: Tensor, lengthscale: Tensor, Z: Tensor, best_f_s: Optional[Tensor], kind: int,
            mode: int, outputscale: float, constant: float, ymean: float, ystd: float,
            best_f: float, fat: bool, tau_relu: float, tau_max: float, need_grad: bool,
            Ainv: Optional[Tensor] = None
            ) -> Tuple[Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor, Tensor]:
    """MC acquisition value (B) of B t-batches on the fused path: posterior
    partials, finalisation with the per-member jitter ladder, reparameterised
    Sobol samples and the qEI / qLogEI reduction, one launch each.  With
    need_grad also (mean, L, Xq, R^T) for the registered backward (the W^T slot
    stays empty: the backward forms W itself); the last output is the ladder
    status tensor (info).  Ainv (forward only): the model's full A^{-1}
    (kernels.quad_ainv) where the quad plan applies to this geometry."""
    # the whole host sequence is one native call (csrc/torch/bo_torch.cpp)
    n = Xt.shape[0]
    out = _lib.torch_ops().qmc_acq_native(
        X.contiguous(), Xt_scaled, U, Linv, beta, lengthscale, Z.reshape(-1, X.shape[1]).contiguous(),
        best_f_s, kind, mode, n, outputscale, constant, ymean, ystd, best_f, fat, tau_relu, tau_max,
        need_grad, kernels.kxt_cap(X.device), False, Ainv, alpha)
    acq, mean, L, Xq, Rt, Wt, jit, info, _ = out
    return acq, mean, L, Xq, Rt, Wt, jit, info


@qmc_acq.register_fake
def _(X, Xt, Xt_scaled, U, Linv, beta, alpha, lengthscale, Z, best_f_s, kind, mode, outputscale,
      constant, ymean, ystd, best_f, fat, tau_relu, tau_max, need_grad, Ainv=None):
    B, q, _ = X.shape
    mk = lambda *s: X.new_empty(*s, dtype=F64)  # noqa: E731
    info = X.new_empty(B, dtype=torch.int32)
    if not need_grad:
        return mk(B), mk(0), mk(0), mk(0), mk(0), mk(0), mk(B), info
    Qp, nrows_pad, nC = _geometry(B, q, Xt.shape[0])
    # R^T's layout is carried by its shape (csrc/torch/bo_torch.cpp): blocked
    # where the backward's fused W -> dX pass applies
    Rt = (mk(nC * 8, nrows_pad // 16, 256) if kernels.rt_blocked_plan(B, q, Xt.shape[0])
          else mk(nC * 128, nrows_pad))
    return (mk(B), mk(B, q), mk(B, q, q), mk(nrows_pad, kernels.DP), Rt, mk(0), mk(B), info)


@torch.library.custom_op("bo::qmc_acq_backward", mutates_args=(), device_types="cuda")
def qmc_acq_backward(dacq: Tensor, acq: Tensor, mean: Tensor, L: Tensor, Z: Tensor,
                     best_f_s: Optional[Tensor], Xq: Tensor, Rt: Tensor, Linv: Tensor, U: Tensor,
                     Xt: Tensor, Xt_scaled: Tensor, alpha: Tensor, lengthscale: Tensor, kind: int,
                     mode: int, outputscale: float, ystd: float, best_f: float, fat: bool,
                     tau_relu: float, tau_max: float) -> Tensor:
    """dX of qmc_acq: the reduction + sampling + q x q Cholesky backward
    (bo_qmc_backward), then the posterior backward with W = R L^-1 reduced into
    dX as it is formed (bo_post_w_dx) -- one native call
    (bo::qmc_acq_backward_native)."""
    return _lib.torch_ops().qmc_acq_backward_native(
        dacq.contiguous(), acq, mean, L, Z.reshape(-1, mean.shape[1]).contiguous(), best_f_s, Xq,
        Rt, Linv, U, Xt_scaled, alpha, lengthscale, kind, mode, Xt.shape[1], Xt.shape[0],
        outputscale, ystd, best_f, fat, tau_relu, tau_max)


@qmc_acq_backward.register_fake
def _(dacq, acq, mean, L, Z, best_f_s, Xq, Rt, Linv, U, Xt, Xt_scaled, alpha, lengthscale, kind,
      mode, outputscale, ystd, best_f, fat, tau_relu, tau_max):
    return mean.new_empty(mean.shape[0], mean.shape[1], Xt.shape[1])


def _acq_setup(ctx, inputs, output):
    (X, Xt, Xt_scaled, U, Linv, beta, alpha, lengthscale, Z, best_f_s, kind, mode, outputscale,
     constant, ymean, ystd, best_f, fat, tau_relu, tau_max, need_grad, *_) = inputs
    acq, mean, L, Xq, Rt, Wt, jit, info = output
    # only acq is differentiable; unmaterialised grads keep autograd from
    # zero-filling R^T (268 MB at C3) on every backward
    ctx.mark_non_differentiable(mean, L, Xq, Rt, Wt, jit, info)
    ctx.set_materialize_grads(False)
    ctx.save_for_backward(acq, mean, L, Z, Xq, Rt, Linv, U, Xt, Xt_scaled, alpha, lengthscale)
    ctx.best_f_s = best_f_s
    ctx.meta = (kind, mode, outputscale, ystd, best_f, fat, tau_relu, tau_max)


def _acq_bwd(ctx, dacq, *_):
    acq, mean, L, Z, Xq, Rt, Linv, U, Xt, Xt_scaled, alpha, lengthscale = ctx.saved_tensors
    if Rt.numel() == 0:
        raise RuntimeError("bo::qmc_acq was called with need_grad=False")
    kind, mode, outputscale, ystd, best_f, fat, tau_relu, tau_max = ctx.meta
    if dacq is None:
        return (None,) * 22
    dX = torch.ops.bo.qmc_acq_backward(dacq, acq, mean, L, Z, ctx.best_f_s, Xq, Rt, Linv, U, Xt,
                                       Xt_scaled, alpha, lengthscale, kind, mode, outputscale,
                                       ystd, best_f, fat, tau_relu, tau_max)
    # the forward's deferred ladder status, now that the backward is queued
    # (waits only for the forward's event; raises NotPSDError / warns here)
    if not torch.cuda.is_current_stream_capturing():
        kernels.check_ladder_status(dX.device)
    return (dX,) + (None,) * 21


qmc_acq.register_autograd(_acq_bwd, setup_context=_acq_setup)


class QmcAcqGrad(torch.autograd.Function):
    """bo::qmc_acq with need_grad, as a plain autograd Function: the same two
    native calls (qmc_acq_native, qmc_acq_backward_native) and the semantics
    of _acq_setup / _acq_bwd (only acq differentiable, no materialised zero
    grads, the ladder status read once the backward is queued), without the
    torch.library autograd wrapper around the registered op -- its per-call
    schema handling (fill_defaults over 22 arguments) and redispatch cost ~90
    us of host time per C2 forward + backward (tools/host_c2_fwd_bwd.py), the
    per-iteration path of gen_candidates_scipy.  The registered op stays the
    interface for opcheck / fake tensors and the forward-only calls."""

    @staticmethod
    def forward(ctx, X, Xt, Xt_scaled, U, Linv, beta, alpha, lengthscale, Z, best_f_s, kind, mode,
                outputscale, constant, ymean, ystd, best_f, fat, tau_relu, tau_max):
        out = _lib.torch_ops().qmc_acq_native(
            X.contiguous(), Xt_scaled, U, Linv, beta, lengthscale,
            Z.reshape(-1, X.shape[1]).contiguous(), best_f_s, kind, mode, Xt.shape[0], outputscale,
            constant, ymean, ystd, best_f, fat, tau_relu, tau_max, True, kernels.kxt_cap(X.device),
            False, None, alpha)
        acq, mean, L, Xq, Rt, _, jit, info, _ = out
        ctx.mark_non_differentiable(jit, info)
        ctx.set_materialize_grads(False)
        # every tensor through save_for_backward (the output acq included): a
        # tensor held as a plain ctx attribute, above all an output, forms an
        # output -> grad_fn -> ctx -> output cycle that keeps R^T (268 MB at C3)
        # and the whole graph alive until the cyclic GC runs, and skips the
        # saved-tensor version check on the cached U / L^-1 / alpha
        ctx.save_for_backward(acq, mean, L, Z, Xq, Rt, Linv, U, Xt_scaled, alpha, lengthscale,
                              best_f_s)
        ctx.meta = (kind, mode, outputscale, ystd, best_f, fat, tau_relu, tau_max, Xt.shape[1],
                    Xt.shape[0])
        return acq, jit, info

    @staticmethod
    def backward(ctx, dacq, *_):
        if dacq is None:
            return (None,) * 20
        acq, mean, L, Z, Xq, Rt, Linv, U, Xt_scaled, alpha, lengthscale, best_f_s = \
            ctx.saved_tensors
        kind, mode, outputscale, ystd, best_f, fat, tau_relu, tau_max, d, n = ctx.meta
        dX = _lib.torch_ops().qmc_acq_backward_native(
            dacq.contiguous(), acq, mean, L, Z.reshape(-1, mean.shape[1]).contiguous(), best_f_s,
            Xq, Rt, Linv, U, Xt_scaled, alpha, lengthscale, kind, mode, d, n, outputscale, ystd,
            best_f, fat, tau_relu, tau_max)
        if not torch.cuda.is_current_stream_capturing():
            kernels.check_ladder_status(dX.device)
        return (dX,) + (None,) * 19


# ---- bo::qehvi ---------------------------------------------------------------------------
@torch.library.custom_op("bo::qehvi", mutates_args=(), device_types="cuda")
def qehvi(mean: Tensor, L: Tensor, Z: Tensor, cell_lo: Tensor, cell_hi: Tensor) -> Tensor:
    """qEHVI (B) of m independent outputs: mean m x B x q, roots m x B x q x q,
    Z S x (q m), hypercells K x m (or S x K x m)."""
    return kernels.qehvi(mean, L, Z, cell_lo, cell_hi)


@qehvi.register_fake
def _(mean, L, Z, cell_lo, cell_hi):
    return mean.new_empty(mean.shape[1])


@torch.library.custom_op("bo::qehvi_backward", mutates_args=(), device_types="cuda")
def qehvi_backward(dacq: Tensor, mean: Tensor, L: Tensor, Z: Tensor, cell_lo: Tensor,
                   cell_hi: Tensor) -> Tuple[Tensor, Tensor]:
    return kernels.qehvi_backward(mean, L, Z, cell_lo, cell_hi, dacq)


@qehvi_backward.register_fake
def _(dacq, mean, L, Z, cell_lo, cell_hi):
    return torch.empty_like(mean), torch.empty_like(L)


def _qehvi_setup(ctx, inputs, output):
    mean, L, Z, cell_lo, cell_hi = inputs
    ctx.save_for_backward(mean, L, Z, cell_lo, cell_hi)


def _qehvi_bwd(ctx, dacq):
    mean, L, Z, lo, hi = ctx.saved_tensors
    dmean, dL = torch.ops.bo.qehvi_backward(dacq, mean, L, Z, lo, hi)
    return dmean, dL, None, None, None


qehvi.register_autograd(_qehvi_bwd, setup_context=_qehvi_setup)


# ---- bo::mll -----------------------------------------------------------------------------------
@torch.library.custom_op("bo::mll", mutates_args=(), device_types="cuda")
def mll(Xt: Tensor, y: Tensor, lengthscale: Tensor, noise: float, constant: float,
        outputscale: float, kind: int, noise_vec: Optional[Tensor] = None) -> Tuple[Tensor, Tensor]:
    """Data term of the exact marginal log likelihood, log N(y | c, K + s2 I)
    (no priors, not divided by n), and its gradient w.r.t. [noise, constant,
    lengthscale_1..d, (outputscale)]: one Cholesky + inverse (task DAG), the
    triangular A^{-1} = U U^T and one bo_mll_terms pass.  noise_vec (n): a
    fixed-noise likelihood (K + diag(noise_vec); the noise entry of the
    gradient is then meaningless and unused)."""
    from .fit import mll_terms
    val, grad = mll_terms(Xt, y, lengthscale, noise if noise_vec is None else noise_vec,
                          constant, outputscale, kind)
    return (torch.tensor([val], dtype=F64, device=Xt.device),
            torch.as_tensor(grad, dtype=F64).to(Xt.device))


@mll.register_fake
def _(Xt, y, lengthscale, noise, constant, outputscale, kind, noise_vec=None):
    d = Xt.shape[1]
    return Xt.new_empty(1, dtype=F64), Xt.new_empty(d + 3, dtype=F64)


OPS: List[str] = ["sobol_normal", "gp_cache", "chol_jitter", "chol_backward", "post_partials",
                  "qmc_finalize", "gp_posterior", "gp_posterior_backward", "qmc_acq",
                  "qmc_acq_backward", "qehvi", "qehvi_backward", "mll"]
