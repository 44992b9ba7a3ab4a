"""Acquisition functions on the accelerated path (BoTorch-compatible API).

MC family: acquisition/monte_carlo.py:60-645 (SampleReducingMCAcquisitionFunction,
qExpectedImprovement, qNoisyExpectedImprovement); multi-objective qEHVI:
acquisition/multi_objective/monte_carlo.py:146-322; analytic EI / PI / UCB:
acquisition/analytic.py.

For a SingleTaskGP with the identity objective and no constraints, ``forward``
runs the fused gfx950 path -- post_partials (K*x + R = K*x L^{-T} + R R^T on
the fp64 matrix cores) and qmc_finalize (q x q psd_safe_cholesky, Sobol
reparameterisation, q-max / sample-mean reduction) -- as one autograd node whose
backward is bo_qmc_backward + bo_post_backward.  Other objectives / models take
the generic route (device posterior -> sampler -> torch reduction).
"""
from __future__ import annotations

import copy
import math
import os
import warnings
from typing import Callable, List, Optional, Union

import torch
from torch import nn

from . import _lib, kernels
from .exceptions import BotorchError, BotorchWarning, NanError, NotPSDError, UnsupportedError
from .safe_math import TAU_MAX, TAU_RELU, fatmax, log_improvement, logmeanexp, smooth_amax
from .objective import (ConstrainedMCObjective, GenericMCObjective, IdentityMCObjective,
                        MCAcquisitionObjective, MCObjective, compute_best_feasible_objective,
                        compute_feasibility_indicator, compute_smoothed_feasibility_indicator,
                        repeat_to_match_aug_dim)
from .models import prime_prediction_caches
from .posteriors import FUSED_QMAX
from .sampling import MCSampler, ShapeOnlyPosterior, SobolQMCNormalSampler, get_sampler


# -- input handling (utils/transforms.py:146-336) -----------------------------
def t_batch_mode(X: torch.Tensor, expected_q: Optional[int] = None) -> torch.Tensor:
    if X.dim() == 2:
        X = X.unsqueeze(0)
    if expected_q is not None and X.shape[-2] != expected_q:
        raise AssertionError(f"Expected X to be `batch_shape x q={expected_q} x d`, but got X with shape {tuple(X.shape)}.")
    return X


class AcquisitionFunction(nn.Module):
    """acquisition/acquisition.py:33-74."""

    def __init__(self, model):
        super().__init__()
        self.model = model
        self.X_pending = None

    def set_X_pending(self, X_pending: Optional[torch.Tensor] = None) -> None:
        if X_pending is not None:
            if X_pending.requires_grad:
                warnings.warn("Pending points require a gradient but the acquisition function"
                              " will not provide a gradient to these points.", BotorchWarning)
            self.X_pending = X_pending.detach().clone()
        else:
            self.X_pending = X_pending

    def _concat_pending(self, X: torch.Tensor) -> torch.Tensor:
        """utils/transforms.py:312-336."""
        if self.X_pending is not None:
            Xp = self.X_pending.to(X).expand(*X.shape[:-2], *self.X_pending.shape[-2:])
            X = torch.cat([X, Xp], dim=-2)
        return X


class MCAcquisitionFunction(AcquisitionFunction):
    """acquisition/acquisition.py:77-146 + SampleReducingMCAcquisitionFunction
    (acquisition/monte_carlo.py:155-330): samples -> objective -> per-sample
    utility -> constraint weighting -> q reduction -> sample reduction.

    Subclasses run a fused gfx950 kernel chain when the configuration allows
    (``_fused_eligible``) and otherwise this generic route, whose posterior,
    root decomposition and base samples are still the device kernels."""

    _default_sample_shape = torch.Size([512])
    _log = False

    def __init__(self, model, sampler: Optional[MCSampler] = None, objective=None,
                 posterior_transform=None, X_pending=None, constraints=None, eta=1e-3,
                 fat: bool = False):
        super().__init__(model)
        if constraints is not None and isinstance(objective, ConstrainedMCObjective):
            raise ValueError("ConstrainedMCObjective as well as constraints passed to constructor."
                             "Choose one or the other, preferably the latter.")
        if objective is None and model.num_outputs != 1 and posterior_transform is None:
            raise UnsupportedError("Must specify an objective or a posterior transform when "
                                   "using a multi-output model.")
        self.sampler = sampler
        self.objective = objective if objective is not None else IdentityMCObjective()
        self.posterior_transform = posterior_transform
        self._constraints = constraints
        self._eta = eta
        self._fat = fat
        self.set_X_pending(X_pending)

    @property
    def sample_shape(self) -> torch.Size:
        return self.sampler.sample_shape if self.sampler is not None else self._default_sample_shape

    def _ensure_sampler(self, posterior=None):
        if self.sampler is None:
            self.sampler = get_sampler(posterior, sample_shape=self._default_sample_shape)
        return self.sampler

    def get_posterior_samples(self, posterior):
        """acquisition/acquisition.py:109-146."""
        return self._ensure_sampler(posterior)(posterior)

    def _fused_eligible(self, X: torch.Tensor) -> bool:
        m = self.model
        return (hasattr(m, "prediction_cache") and type(self.objective) is IdentityMCObjective
                and self.posterior_transform is None and self._constraints is None
                and X.shape[-2] <= FUSED_QMAX and X.shape[-1] <= kernels.DP and X.is_cuda
                and len(self.sample_shape) == 1)

    # -- generic route (monte_carlo.py:253-330) -----------------------------------------
    def _sample_forward(self, obj: torch.Tensor) -> torch.Tensor:
        raise NotImplementedError

    def _q_reduction(self, acqval: torch.Tensor) -> torch.Tensor:
        return acqval.amax(dim=-1)

    def _sample_reduction(self, acqval: torch.Tensor) -> torch.Tensor:
        return acqval.mean(dim=tuple(range(len(self.sample_shape))))

    def _apply_constraints(self, acqval: torch.Tensor, samples: torch.Tensor) -> torch.Tensor:
        """monte_carlo.py:305-330: weight (or, in log space, shift) the utility by
        the smoothed feasibility indicator."""
        if self._constraints is not None:
            if not self._log and (acqval < 0).any():
                raise ValueError("Constraint-weighting requires unconstrained "
                                 "acquisition values to be non-negative.")
            ind = compute_smoothed_feasibility_indicator(constraints=self._constraints,
                                                         samples=samples, eta=self._eta,
                                                         log=self._log, fat=self._fat)
            acqval = acqval.add(ind) if self._log else acqval.mul(ind)
        return acqval

    def _get_samples_and_objectives(self, X: torch.Tensor):
        posterior = self.model.posterior(X, posterior_transform=self.posterior_transform)
        samples = self.get_posterior_samples(posterior)
        return samples, self.objective(samples, X=X)

    def _generic_forward(self, X: torch.Tensor) -> torch.Tensor:
        samples, obj = self._get_samples_and_objectives(X)
        samples = repeat_to_match_aug_dim(target_tensor=samples, reference_tensor=obj)
        acqval = self._apply_constraints(self._sample_forward(obj), samples)
        return _ensemble_mean(self.model, self._sample_reduction(self._q_reduction(acqval)))


def _fused_mc(X3: torch.Tensor, acqf, mode: int, best_f: float, best_f_s, Z: torch.Tensor):
    """qEI / qLogEI value of B t-batches on the gfx950 fused path through
    bo::qmc_acq (one torch.ops call; its registered backward gives dX).  The
    jitter-ladder status is read at the end of the backward when a gradient
    follows, else one call later (kernels.raise_not_psd_deferred)."""
    from . import ops  # torch.ops.bo registration, QmcAcqGrad
    model = acqf.model
    cache = model.prediction_cache()
    ymean, ystd = model.outcome_stats()
    need_grad = torch.is_grad_enabled() and X3.requires_grad
    lp = getattr(acqf, "_log_params", None)
    fat, tau_relu, tau_max = lp if lp is not None else (True, 1.0, 1.0)
    dev = X3.device
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    if X3.dtype != torch.float64:  # the model computes in fp64; the value returns in X's dtype
        return _fused_mc(X3.to(torch.float64), acqf, mode, best_f, best_f_s, Z).to(X3.dtype)
    cap = kernels._CAPTURE_STATUS.get(idx) if idx in kernels._CAPTURE else None
    if not need_grad and not kernels.SYNC_LADDER and (idx not in kernels._CAPTURE or cap):
        # eager forward-only: ONE native call issues the whole chain and defers
        # the ladder status (the previous call's is returned and acted on here);
        # under a graph capture the same call, its status folded into the
        # graph's pinned words by the finalisation kernel itself
        acq, prev = _lib.torch_ops().qmc_acq_eager(
            X3.contiguous(), cache.Xt_scaled, cache.U, cache.beta, cache.lengthscale,
            Z, best_f_s, int(cache.kind), int(mode), int(cache.n), float(cache.outputscale),
            float(cache.constant), float(ymean), float(ystd), float(best_f), bool(fat),
            float(tau_relu), float(tau_max), kernels.kxt_cap(dev),
            kernels.quad_ainv(cache, X3.shape[0], X3.shape[1]), cache.alpha,
            cap[0] if cap else None, cap[1] if cap else None)
        if cap:
            kernels.record_capture_status(idx, None, type(acqf).__name__)
        else:
            kernels.ladder_prev_outcome(prev, idx, type(acqf).__name__)
        return acq
    if need_grad:  # the registered op's semantics without its autograd wrapper
        acq, jit, info = ops.QmcAcqGrad.apply(
            X3, cache.Xt, cache.Xt_scaled, cache.U, cache.Linv, cache.beta, cache.alpha,
            cache.lengthscale, Z, best_f_s, int(cache.kind), int(mode), float(cache.outputscale),
            float(cache.constant), float(ymean), float(ystd), float(best_f), bool(fat),
            float(tau_relu), float(tau_max))
    else:
        outs = torch.ops.bo.qmc_acq(
            X3, cache.Xt, cache.Xt_scaled, cache.U, cache.Linv, cache.beta, cache.alpha,
            cache.lengthscale, Z, best_f_s, int(cache.kind), int(mode), float(cache.outputscale),
            float(cache.constant), float(ymean), float(ystd), float(best_f), bool(fat),
            float(tau_relu), float(tau_max), False,
            kernels.quad_ainv(cache, X3.shape[0], X3.shape[1]))
        acq, jit, info = outs[0], outs[6], outs[7]
    # deferred either way: with a gradient the status is read at the end of the
    # registered backward (ops._acq_bwd), once the backward's launches are
    # queued behind the forward -- so the evaluation that produced a failed
    # root raises NotPSDError (as gen.py's closure sees the reference's) but
    # the device does not drain between the forward and the backward
    kernels.raise_not_psd_deferred(info, jit, type(acqf).__name__)
    return acq

def _host_scalar(module, name: str) -> float:
    """float(module.<name>) read once per value: a best_f on the device (the
    usual ``best_f=train_Y.max()``) would otherwise be a device-to-host read,
    i.e. a stream drain, in every forward.  The cache holds the tensor itself
    (so a replacement can never reuse its identity) and its version counter:
    a new tensor or an in-place change is read again."""
    t = getattr(module, name)
    cache = module.__dict__.setdefault("_host_scalars", {})
    hit = cache.get(name)
    if hit is None or hit[0] is not t or hit[1] != t._version:
        hit = (t, t._version, float(t))
        cache[name] = hit
    return hit[2]


def _ensemble_mean(model, acq: torch.Tensor) -> torch.Tensor:
    """Average over the MCMC batch of ensemble models (utils/transforms.py:289-293)."""
    return acq.mean(dim=-1) if getattr(model, "_is_ensemble", False) else acq


class qExpectedImprovement(MCAcquisitionFunction):
    """MC batch EI (acquisition/monte_carlo.py:332-414):
    qEI(X) = E[max_j max(Y_j - best_f, 0)], optionally weighted by smoothed
    outcome constraints (``constraints``, ``eta``)."""

    def __init__(self, model, best_f: Union[float, torch.Tensor], sampler=None, objective=None,
                 posterior_transform=None, X_pending=None, constraints=None, eta=1e-3):
        super().__init__(model, sampler, objective, posterior_transform, X_pending,
                         constraints=constraints, eta=eta)
        self.register_buffer("best_f", torch.as_tensor(best_f, dtype=torch.float64))

    def _sample_forward(self, obj: torch.Tensor) -> torch.Tensor:
        """monte_carlo.py:405-414."""
        return (obj - self.best_f.unsqueeze(-1).to(obj)).clamp_min(0)

    def forward(self, X: torch.Tensor) -> torch.Tensor:
        X = self._concat_pending(t_batch_mode(X))
        batch = X.shape[:-2]
        q, d = X.shape[-2], X.shape[-1]
        X3 = X.reshape(-1, q, d)
        if self._fused_eligible(X) and self.best_f.numel() == 1:
            sampler = self._ensure_sampler()
            Z = sampler.base_samples_2d(q, X.device)
            acq = _fused_mc(X3, self, _lib.QMC_QEI, _host_scalar(self, "best_f"), None, Z)
            return acq.reshape(batch)
        if (getattr(self.model, "_is_fully_bayesian", False) and X.is_cuda and not self._log
                and type(self.objective) is IdentityMCObjective and self.posterior_transform is None
                and self._constraints is None and len(self.sample_shape) == 1
                and self.best_f.numel() == 1 and q <= FUSED_QMAX):
            sampler = self._ensure_sampler()
            Z = sampler.base_samples_2d(q, X.device)
            return _SaasQEI.apply(X3, self, _host_scalar(self, "best_f"), Z).reshape(batch)
        return self._generic_forward(X)


class _SaasQEI(torch.autograd.Function):
    """qEI over the MCMC ensemble of a SAAS model (models/fully_bayesian.py:509-546,
    averaged over MCMC_DIM as utils/transforms.py:289-293), any d <= 128, with
    all M members batched into each launch.

    Forward: K*x of every member (one bo_covar_batched, Matern-5/2 x outputscale),
    R = K*x L_m^{-T} and the means (batched MFMA GEMMs over M), the R R^T blocks
    (batched over M x B), K** (one bo_covar_batched over M x B), the jittered
    q x q roots (bo_chol_small over M x B), reparameterised samples (one batched
    GEMM) and the qEI reduction (bo_mc_reduce over M x B), averaged over M.
    Backward: bo_qmc_backward over M x B -> d mu, d Sigma; d K*x = d mu alpha^T
    - G W (W = R L^{-1}, batched GEMMs); bo_kernel_grad per member for K*x and K**."""

    @staticmethod
    def forward(ctx, X3, acqf, best_f, Z):
        model = acqf.model
        B, q, d = X3.shape
        dev = X3.device
        X2 = X3.detach().reshape(B * q, d).contiguous()
        need_grad = ctx.needs_input_grad[0]
        ym, ys = model.outcome_stats()
        ens = model.ensemble_cache()
        M, n = ens["U"].shape[0], ens["n"]
        f64 = dict(dtype=torch.float64, device=dev)
        Bq = B * q
        Kx = torch.empty(M, Bq, n, **f64)
        kernels.covar_batched(ens["kind"], X2, (0, 0), Bq, ens["Xt"], (0, 0), n, d, ens["ls"],
                              (d, 0), ens["os"], (1, 0), Kx, (Bq * n, 0), n, M, 1)
        R = kernels.gemm(Kx, ens["U"], flags=_lib.GEMM_B_UPPER)              # M x Bq x n
        mean = kernels.gemm(Kx, ens["alpha"].unsqueeze(-1)).reshape(M, B, q)
        RR = kernels.gemm(R.view(M * B, q, n), R.view(M * B, q, n), transB=True)  # MB x q x q
        Kxx = torch.empty(M * B, q, q, **f64)
        kernels.covar_batched(ens["kind"], X2, (0, q * d), q, X2, (0, q * d), q, d, ens["ls"],
                              (d, 0), ens["os"], (1, 0), Kxx, (B * q * q, q * q), q, M, B)
        cov = (Kxx - RR) * (ys * ys)
        mean = ym + ys * (mean + ens["const"].view(M, 1, 1))
        L = kernels.chol_jitter(cov)                                          # MB x q x q
        f = kernels.sample_mvn(mean.reshape(M * B, q), L, Z)                  # S x MB x q
        acq = kernels.mc_reduce(f, best_f).view(M, B).mean(dim=0)
        if need_grad:
            ctx.ens, ctx.X2, ctx.Z, ctx.best_f, ctx.shape, ctx.ys = ens, X2, Z, best_f, (B, q, d), ys
            ctx.R, ctx.mean, ctx.L = R, mean.reshape(M * B, q), L
        return acq

    @staticmethod
    def backward(ctx, dacq):
        B, q, d = ctx.shape
        ens, ys = ctx.ens, ctx.ys
        M, n = ens["U"].shape[0], ens["n"]
        da = (dacq / M).repeat(M).contiguous()                                # MB
        dmean, dcov = kernels.qmc_backward(_lib.QMC_QEI, ctx.mean, ctx.L, ctx.Z, da, ctx.best_f)
        dmu = (ys * dmean).reshape(M, B * q)                                  # standardized
        G = ((ys * ys) * (dcov + dcov.mT)).contiguous()                       # MB x q x q
        W = kernels.gemm(ctx.R, ens["U"], transB=True, flags=_lib.GEMM_B_LOWER)  # M x Bq x n
        dK = (dmu.unsqueeze(-1) * ens["alpha"].unsqueeze(1)).contiguous()    # M x Bq x n
        kernels.gemm(G, W.view(M * B, q, n), alpha=-1.0, beta=1.0, C=dK.view(M * B, q, n))
        Gm = G.view(M, B * q, q)
        dX = None
        for mi in range(M):
            ls = ens["ls"][mi]
            os_ = ens["os_host"][mi]
            dX = kernels.kernel_grad(ctx.X2, ens["Xt"], dK[mi], ls, ens["kind"], os_, dX=dX)
            dX = kernels.kernel_grad(ctx.X2, ctx.X2, Gm[mi].contiguous(), ls, ens["kind"], os_,
                                     group=q, dX=dX)
        return dX.reshape(B, q, d), None, None, None


# -- analytic ------------------------------------------------------------------------
_INV_SQRT_2PI = 1 / math.sqrt(2 * math.pi)  # utils/probability/utils.py:27-29
_NEG_INV_SQRT_2 = -(1 / math.sqrt(2))


def _ndtr(x):
    """Standard normal CDF (utils/probability/utils.py:133-136)."""
    return 0.5 * torch.erfc(_NEG_INV_SQRT_2 * x)


def _phi(x):
    """Standard normal PDF (utils/probability/utils.py:139-142)."""
    return _INV_SQRT_2PI * (-0.5 * x.square()).exp()


class AnalyticAcquisitionFunction(AcquisitionFunction):
    def __init__(self, model, posterior_transform=None):
        super().__init__(model)
        self.posterior_transform = posterior_transform

    def set_X_pending(self, X_pending=None) -> None:
        """acquisition/analytic.py:78-82."""
        raise UnsupportedError("Analytic acquisition functions do not account for X_pending yet.")

    def _mean_and_sigma(self, X, compute_sigma=True, min_var=1e-12):
        """acquisition/analytic.py:84-108."""
        posterior = self.model.posterior(X, posterior_transform=self.posterior_transform)
        mean = posterior.mean.squeeze(-2).squeeze(-1)
        if not compute_sigma:
            return mean, None
        sigma = posterior.variance.clamp_min(min_var).sqrt().view(mean.shape)
        return mean, sigma


class ExpectedImprovement(AnalyticAcquisitionFunction):
    """acquisition/analytic.py:298-354: sigma (phi(u) + u Phi(u)), u = (mu - best_f)/sigma."""

    def __init__(self, model, best_f, posterior_transform=None, maximize=True):
        super().__init__(model, posterior_transform)
        self.register_buffer("best_f", torch.as_tensor(best_f, dtype=torch.float64))
        self.maximize = maximize

    def forward(self, X):
        X = t_batch_mode(X, expected_q=1)
        mean, sigma = self._mean_and_sigma(X)
        u = (mean - self.best_f.to(mean)) / sigma
        if not self.maximize:
            u = -u
        return sigma * (_phi(u) + u * _ndtr(u))


class ProbabilityOfImprovement(AnalyticAcquisitionFunction):
    """acquisition/analytic.py (PI): Phi((mu - best_f)/sigma)."""

    def __init__(self, model, best_f, posterior_transform=None, maximize=True):
        super().__init__(model, posterior_transform)
        self.register_buffer("best_f", torch.as_tensor(best_f, dtype=torch.float64))
        self.maximize = maximize

    def forward(self, X):
        X = t_batch_mode(X, expected_q=1)
        mean, sigma = self._mean_and_sigma(X)
        u = (mean - self.best_f.to(mean)) / sigma
        return _ndtr(u if self.maximize else -u)


class UpperConfidenceBound(AnalyticAcquisitionFunction):
    """acquisition/analytic.py (UCB): mu + sqrt(beta) sigma."""

    def __init__(self, model, beta, posterior_transform=None, maximize=True):
        super().__init__(model, posterior_transform)
        self.register_buffer("beta", torch.as_tensor(beta, dtype=torch.float64))
        self.maximize = maximize

    def forward(self, X):
        X = t_batch_mode(X, expected_q=1)
        mean, sigma = self._mean_and_sigma(X)
        return (mean if self.maximize else -mean) + self.beta.to(mean).sqrt() * sigma


# -- qNEI -------------------------------------------------------------------------------
def prune_inferior_points(model, X, objective=None, posterior_transform=None, constraints=None,
                          num_samples: int = 2048, max_frac: float = 1.0, sampler=None,
                          marginalize_dim=None):
    """acquisition/utils.py:245-349: keep the points with non-zero empirical
    probability of being the best (feasible) point under ``num_samples`` joint
    posterior samples.  The joint n x n posterior, its jittered Cholesky and the
    sample GEMM run on the device."""
    if marginalize_dim is None and getattr(model, "_is_ensemble", False):
        marginalize_dim = MCMC_DIM
    if X.ndim > 2:
        raise UnsupportedError("Batched inputs `X` are currently unsupported by prune_inferior_points")
    if X.size(-2) == 0:
        raise ValueError("X must have at least one point.")
    if max_frac <= 0 or max_frac > 1.0:
        raise ValueError(f"max_frac must take values in (0, 1], is {max_frac}")
    max_points = math.ceil(max_frac * X.size(-2))
    with torch.no_grad():
        posterior = model.posterior(X=X, posterior_transform=posterior_transform)
        if sampler is None:
            sampler = get_sampler(posterior, sample_shape=torch.Size([num_samples]))
        samples = sampler(posterior)
        if objective is None:
            objective = IdentityMCObjective()
        obj_vals = objective(samples, X=X)
    if obj_vals.ndim > 2:
        if obj_vals.ndim == 3 and marginalize_dim is not None:
            if marginalize_dim < 0:
                marginalize_dim = 1 + (marginalize_dim % obj_vals.ndim)
            obj_vals = obj_vals.mean(dim=marginalize_dim)
        else:
            raise UnsupportedError("Models with multiple batch dims are currently unsupported by"
                                   " prune_inferior_points.")
    infeas = ~compute_feasibility_indicator(constraints=constraints, samples=samples,
                                            marginalize_dim=marginalize_dim)
    if infeas.any():
        obj_vals[infeas] = obj_vals.min() - 1
    is_best = torch.argmax(obj_vals, dim=-1)
    idcs, counts = torch.unique(is_best, return_counts=True)
    if len(idcs) > max_points:
        counts, order_idcs = torch.sort(counts, descending=True)
        idcs = order_idcs[:max_points]  # reference quirk kept (utils.py:345-347)
    return X[idcs]


MCMC_DIM = -3  # models/fully_bayesian.py


def supports_cache_root(model, posterior_transform=None) -> bool:
    """acquisition/cached_cholesky.py:34-51, for the models built here: exact
    GPs (SingleTaskGP, the SAAS ensemble) with a linear (Standardize) outcome
    transform.  A ModelListGP is cached here only under a scalarising posterior
    transform (its joint root is then single-output); without one the full
    joint samples are drawn instead."""
    if hasattr(model, "models"):
        return posterior_transform is not None and all(supports_cache_root(m) for m in model.models)
    return hasattr(model, "prediction_cache") or getattr(model, "_is_fully_bayesian", False)


def sample_cached_cholesky(posterior, baseline_L: torch.Tensor, q: int, base_samples: torch.Tensor,
                           sample_shape: torch.Size, max_tries: int = 6) -> torch.Tensor:
    """utils/low_rank.py:85-173 for a single-output joint posterior over
    (X_baseline, X): the q new rows of the joint Cholesky from the cached
    baseline root (bl = K_qb L_bb^{-T}, br = psd_safe_cholesky(K_qq - bl bl^T)),
    then samples = mean_q + [bl, br] Z (Z the joint base samples).  Raises
    NanError on non-finite samples."""
    from .exceptions import NanError
    from .posteriors import _CholJitter
    mvn = posterior.distribution
    cov = mvn.covariance_matrix
    bottom = cov[..., -q:, :]
    bl, br = bottom.split([bottom.shape[-1] - q, q], dim=-1)
    bl_chol = torch.linalg.solve_triangular(baseline_L.to(bl), bl.transpose(-2, -1),
                                            upper=False).transpose(-2, -1)
    br_to_chol = br - bl_chol @ bl_chol.transpose(-2, -1)
    if torch.is_grad_enabled() and br_to_chol.requires_grad:
        br_chol = _CholJitter.apply(br_to_chol)
    else:
        br_chol = kernels.chol_jitter(br_to_chol, max_tries=max_tries)
    new_Lq = torch.cat([bl_chol, br_chol], dim=-1)                     # batch x q x (r + q)
    mean = mvn.mean[..., -q:]                                          # batch x q
    n_tot = new_Lq.shape[-1]
    Z = base_samples.reshape(*sample_shape, -1, n_tot)
    if Z.shape[len(sample_shape)] != 1:
        raise UnsupportedError("sample_cached_cholesky here takes base samples shared over t-batches")
    Z = Z.reshape(-1, n_tot).to(new_Lq)                               # S' x (r + q)
    f = torch.matmul(Z, new_Lq.reshape(-1, q, n_tot).mT)              # B' x S' x q
    f = f.permute(1, 0, 2) + mean.reshape(1, -1, q)
    res = f.reshape(*sample_shape, *mean.shape[:-1], q, 1)
    bad_nan, bad_inf = bool(torch.isnan(res).any()), bool(torch.isinf(res).any())
    if bad_nan or bad_inf:
        what = " and ".join(w for w, b in (("nans", bad_nan), ("infs", bad_inf)) if b)
        raise NanError(f"Samples contain {what}.")
    return res


class _CachedBaselineRoot:
    """Cached-root state of one exact-GP output over X_baseline
    (acquisition/cached_cholesky.py:94-120, utils/low_rank.py:85-173) and the
    fused-path pieces built on it.

    Construction: the baseline posterior (outcome space), its jittered
    Cholesky L_rr with inverse, the baseline samples mean_b + Z_base L_rr^T, and
    P_b = L_rr^{-1} K(X_b, X_tr) L^{-T} (r x np), Q_b = P_b U^T, the scaled
    baseline inputs.  forward(): T = L_rr^{-1} Sigma'(X_b, X) = s^2 (L_rr^{-1}
    K_bX - P_b R^T) (two MFMA GEMMs) and the sample term F = Z_base T.
    backward(): dT = Z_base^T dF - T G (G = dSigma + dSigma^T) pushed through
    both GEMMs to dK*x (E = -s^2 dT^T Q_b) and d K_bX (s^2 L_rr^{-T} dT)."""

    def __init__(self, model, X_baseline, Z_base, posterior_transform=None):
        r = X_baseline.shape[-2]
        self.Z_base = Z_base
        with torch.no_grad():
            post = model.posterior(X_baseline, posterior_transform=posterior_transform)
            mean_b = post.distribution.mean.reshape(1, r)
            cov_b = post.distribution.covariance_matrix.reshape(r, r)
            L_rr, Linv_rr, _ = kernels.cholesky_with_inverse(cov_b)
            base = kernels.sample_mvn(mean_b, L_rr.unsqueeze(0).contiguous(), Z_base)
            self.samples = base.reshape(Z_base.shape[0], r)
            self.L = L_rr.contiguous()
            self.Linv = Linv_rr.contiguous()
            self.fused_ready = False
            if hasattr(model, "prediction_cache") and X_baseline.shape[-1] <= kernels.DP:
                cache = model.prediction_cache()
                Kb = kernels.covar_matrix(X_baseline.contiguous(), cache.Xt, cache.lengthscale,
                                          cache.kind, cache.outputscale)
                R_b = kernels.gemm(Kb, cache.U[: cache.n, : cache.n], flags=_lib.GEMM_B_UPPER)
                P_b = torch.zeros(r, cache.np, dtype=torch.float64, device=Kb.device)
                P_b[:, : cache.n] = kernels.gemm(self.Linv, R_b, flags=_lib.GEMM_A_LOWER)
                self.P_b = P_b
                # Q_b = P_b U^T = L_rr^{-1} K(X_b, X_tr) A^{-1}  (gradient of the
                # cross-covariance through R = K*x L^{-T})
                self.Q_b = kernels.gemm(P_b, cache.U, transB=True, flags=_lib.GEMM_B_LOWER)
                self.Xb_scaled = torch.zeros(r, kernels.DP, dtype=torch.float64, device=Kb.device)
                self.Xb_scaled[:, : cache.d] = X_baseline / cache.lengthscale
                self.fused_ready = True

    def forward(self, cache, pp, ystd, F_out=None):
        """T and F (F written into F_out when given: the stacked qEHVI input)."""
        s2 = ystd * ystd
        ones = self.__dict__.get("_ones")
        if ones is None or ones.device != pp.Xq.device:
            ones = self._ones = torch.ones(kernels.DP, dtype=torch.float64, device=pp.Xq.device)
        Kbx = kernels.covar_matrix(self.Xb_scaled, pp.Xq, ones, cache.kind, cache.outputscale)
        T = kernels.gemm(self.Linv, Kbx, alpha=s2, flags=_lib.GEMM_A_LOWER)
        if pp.Cx is not None:   # P_b R^T = Q_b K*x^T, fused into the posterior pass
            T.add_(pp.Cx, alpha=-s2)
        else:
            T = kernels.gemm(self.P_b, pp.Rt, alpha=-s2, beta=1.0, C=T)
        F = kernels.gemm(self.Z_base, T, C=F_out)
        return T, F

    def backward(self, cache, pp, W, dmean, dcov, dF, T, ystd, dX=None):
        s2 = ystd * ystd
        B, q, Qp, nrows = pp.B, pp.q, pp.Qp, pp.nrows_pad
        r = self.Linv.shape[0]
        dT = kernels.gemm(self.Z_base, dF, transA=True)            # r x nrows_pad
        G = (dcov + dcov.mT).contiguous()                          # B x q x q
        kernels.gemm_strided(r, q, q, T, nrows, Qp, G, q, q * q, dT, nrows, Qp, B,
                             alpha=-1.0, beta=1.0)                  # dT_b -= T_b G_b
        E = kernels.gemm(dT, self.Q_b, transA=True, alpha=-s2)     # nrows_pad x np
        dKbx = kernels.gemm(self.Linv, dT, transA=True, alpha=s2, flags=_lib.GEMM_A_UPPER)
        dX = kernels.post_backward(cache, pp, W, dmean, dcov, ystd, E=E, dX=dX)
        return kernels.post_backward(cache, pp, None, None, None, ystd, E=dKbx.mT.contiguous(),
                                     Xt_scaled=self.Xb_scaled, n=r, dX=dX)


class qNoisyExpectedImprovement(MCAcquisitionFunction):
    """MC batch noisy EI (acquisition/monte_carlo.py:417-645, cached_cholesky.py:
    63-186, utils/low_rank.py:85-173):
    qNEI(X) = E[max(max_j Y_j - max_i Y_base_i, 0)].

    ``cache_root=True`` (default): the baseline posterior, its jittered root
    L_rr and the baseline samples are computed once; ``base_sampler`` keeps the
    baseline base samples and every forward reuses them as the leading columns
    of the joint (r + q) draw (sampling/normal.py:68-131).  For a SingleTaskGP
    with the identity objective, q <= 16 and d <= 8 the forward is the fused
    chain (post_partials with the cross term, T = L_rr^{-1} Sigma'(X_b, X),
    F = Z_b T, qmc_finalize(QNEI)); otherwise the joint posterior over
    (X_baseline, X) goes through sample_cached_cholesky.  A NotPSD/NaN failure
    of either falls back to standard joint sampling with a BotorchWarning
    (cached_cholesky.py:141-165).  ``cache_root=False``: every forward samples
    the joint (r + q) posterior and takes the baseline best from those samples.
    """

    _fused_mode = _lib.QMC_QNEI

    def __init__(self, model, X_baseline, sampler=None, objective=None, posterior_transform=None,
                 X_pending=None, prune_baseline=True, cache_root=True, constraints=None,
                 eta=1e-3, marginalize_dim=None):
        super().__init__(model, sampler, objective, posterior_transform, X_pending,
                         constraints=constraints, eta=eta)
        self._init_baseline(model, X_baseline, prune_baseline, cache_root, marginalize_dim)

    def _init_baseline(self, model, X_baseline, prune_baseline, cache_root, marginalize_dim):
        if cache_root and not supports_cache_root(model, self.posterior_transform):
            warnings.warn("`cache_root` is only supported here for exact GPs (or a ModelListGP "
                          f"under a scalarising posterior transform); got {type(model)}. "
                          "Setting `cache_root = False`.", RuntimeWarning)
            cache_root = False
        self._cache_root = cache_root
        if prune_baseline:
            X_baseline = prune_inferior_points(model, X_baseline, objective=self.objective,
                                               posterior_transform=self.posterior_transform,
                                               constraints=self._constraints,
                                               marginalize_dim=marginalize_dim)
        self.register_buffer("X_baseline", X_baseline)
        self.baseline_samples = None
        self.baseline_obj = None
        self.base_sampler = None
        self._root = None
        self._zq = None
        if not self._cache_root:
            return
        self.q_in = -1
        r = X_baseline.shape[-2]
        fusable = (hasattr(model, "prediction_cache") and type(self.objective) is IdentityMCObjective
                   and self.posterior_transform is None and self._constraints is None
                   and X_baseline.ndim == 2 and X_baseline.shape[-1] <= kernels.DP
                   and X_baseline.is_cuda and len(self.sample_shape) == 1)
        with torch.no_grad():
            if fusable:
                # the sampler's own base samples over X_baseline (S x r), then the
                # device root + fused precomputations on them
                sampler = self._ensure_sampler()
                sampler._construct_base_samples(ShapeOnlyPosterior(torch.Size(), r, X_baseline.device))
                Z_base = sampler.base_samples.reshape(-1, r).contiguous()
                self._root = _CachedBaselineRoot(model, X_baseline, Z_base)
                baseline_samples = self._root.samples.reshape(*self.sample_shape, r, 1)
                baseline_L = self._root.L
            else:
                posterior = self.model.posterior(X_baseline, posterior_transform=self.posterior_transform)
                baseline_samples = self.get_posterior_samples(posterior)
                baseline_L = posterior.distribution.scale_tril
            baseline_obj = self.objective(baseline_samples, X=X_baseline)
        self.base_sampler = copy.deepcopy(self.sampler)
        self.baseline_samples = baseline_samples
        self.baseline_obj = baseline_obj
        self.register_buffer("_baseline_best_f", self._compute_best_feasible_objective(
            samples=baseline_samples, obj=baseline_obj).contiguous())
        self._baseline_L_t = baseline_L

    @property
    def _baseline_L(self) -> torch.Tensor:
        return self._baseline_L_t

    @_baseline_L.setter
    def _baseline_L(self, L: torch.Tensor) -> None:
        # a replaced root invalidates the fused precomputations built on the old one
        self._baseline_L_t = L
        self._root = None

    @property
    def _fused_ready(self) -> bool:
        return self._root is not None and self._root.fused_ready

    def _compute_best_feasible_objective(self, samples, obj):
        """monte_carlo.py:628-645."""
        return compute_best_feasible_objective(samples=samples, obj=obj,
                                               constraints=self._constraints, model=self.model,
                                               objective=self.objective,
                                               posterior_transform=self.posterior_transform,
                                               X_baseline=self.X_baseline)

    def compute_best_f(self, obj: torch.Tensor) -> torch.Tensor:
        """monte_carlo.py:540-563: the (cached or per-forward) best feasible
        baseline objective, viewed against obj without its q dimension."""
        if self._cache_root:
            val = self._baseline_best_f
        else:
            val = self._compute_best_feasible_objective(samples=self.baseline_samples,
                                                        obj=self.baseline_obj)
        n_sample_dims = len(self.sample_shape)
        view_shape = torch.Size([*val.shape[:n_sample_dims],
                                 *(1,) * (obj.ndim - val.ndim - 1),
                                 *val.shape[n_sample_dims:]])
        return val.view(view_shape).to(obj)

    def _sample_forward(self, obj: torch.Tensor) -> torch.Tensor:
        """monte_carlo.py:565-575."""
        return (obj - self.compute_best_f(obj).unsqueeze(-1)).clamp_min(0)

    # -- joint base samples (cached_cholesky.py:167-186) ----------------------------------
    def _set_sampler(self, q_in: int, posterior) -> None:
        if self.q_in != q_in and self.base_sampler is not None:
            self.sampler._update_base_samples(posterior=posterior, base_sampler=self.base_sampler)
            self.q_in = q_in
            self._zq = None

    def _base_samples_q(self, q: int, device) -> torch.Tensor:
        """The q new columns of the joint (r + q) base samples (S x q) for the
        fused path; the leading r columns are the cached baseline ones."""
        r = self.X_baseline.shape[-2]
        S = self.sample_shape.numel()
        bs = self.sampler.base_samples
        if self.q_in != q or bs is None or bs.numel() != S * (r + q):
            self.q_in = -1
            self._set_sampler(q, ShapeOnlyPosterior(torch.Size([1]), r + q, device))
            bs = self.sampler.base_samples
        key = (q, bs.data_ptr(), bs._version)
        if self._zq is None or self._zq[0] != key:
            self._zq = (key, bs.reshape(S, r + q)[:, r:].contiguous())
        return self._zq[1]

    def _get_f_X_samples(self, posterior, q_in: int) -> torch.Tensor:
        """cached_cholesky.py:122-165."""
        if self._cache_root and self._baseline_L is not None:
            try:
                return sample_cached_cholesky(posterior=posterior, baseline_L=self._baseline_L,
                                              q=q_in, base_samples=self.sampler.base_samples,
                                              sample_shape=self.sampler.sample_shape)
            except (NanError, NotPSDError):
                warnings.warn("Low-rank cholesky updates failed due NaNs or due to an "
                              "ill-conditioned covariance matrix. Falling back to standard "
                              "sampling.", BotorchWarning)
        samples = self.get_posterior_samples(posterior)
        return samples[..., -q_in:, :]

    def _joint_posterior(self, X: torch.Tensor):
        Xb = self.X_baseline
        X_full = torch.cat([Xb.expand(*X.shape[:-2], *Xb.shape[-2:]), X], dim=-2)
        return X_full, self.model.posterior(X_full, posterior_transform=self.posterior_transform)

    def _get_samples_and_objectives(self, X: torch.Tensor):
        """monte_carlo.py:577-626."""
        q = X.shape[-2]
        X_full, posterior = self._joint_posterior(X)
        if not self._cache_root:
            samples_full = self.get_posterior_samples(posterior)
            samples = samples_full[..., -q:, :]
            obj_full = self.objective(samples_full, X=X_full)
            self.baseline_obj, obj = obj_full[..., :-q], obj_full[..., -q:]
            self.baseline_samples = samples_full[..., :-q, :]
        else:
            self._set_sampler(q_in=q, posterior=posterior)
            samples = self._get_f_X_samples(posterior=posterior, q_in=q)
            obj = self.objective(samples, X=X_full[..., -q:, :])
        return samples, obj

    def _fallback_forward(self, X: torch.Tensor) -> torch.Tensor:
        """Standard joint sampling after a failed low-rank update of the fused path
        (cached_cholesky.py:147-165): the cached baseline best is kept."""
        q = X.shape[-2]
        X_full, posterior = self._joint_posterior(X)
        self._set_sampler(q_in=q, posterior=posterior)
        samples = self.get_posterior_samples(posterior)[..., -q:, :]
        obj = self.objective(samples, X=X)
        acqval = self._apply_constraints(self._sample_forward(obj), samples)
        return _ensemble_mean(self.model, self._sample_reduction(self._q_reduction(acqval)))

    def forward(self, X: torch.Tensor) -> torch.Tensor:
        X = self._concat_pending(t_batch_mode(X))
        batch = X.shape[:-2]
        q, d = X.shape[-2], X.shape[-1]
        if self._fused_ready and self._fused_eligible(X):
            try:
                return _FusedQNEI.apply(X.reshape(-1, q, d), self).reshape(batch)
            except (NotPSDError, NanError):
                warnings.warn("Low-rank cholesky updates failed due NaNs or due to an "
                              "ill-conditioned covariance matrix. Falling back to standard "
                              "sampling.", BotorchWarning)
                return self._fallback_forward(X)
        return self._generic_forward(X)


class _FusedQNEI(torch.autograd.Function):
    """qNEI value of B t-batches on the cached-root fused path, with its gradient.

    Forward: post_partials (+ R^T), T = L_rr^{-1} Sigma'(X_b, X) =
    s^2 (L_rr^{-1} K_bX - P_b R^T), F = Z_b T, qmc_finalize(QNEI) on
    Sigma_cond = Sigma' - T^T T.
    Backward (utils/low_rank.py:85-173 differentiated):
      qmc_backward -> d mu', d Sigma_cond, dF;   dT = Z_b^T dF - T (G_b), G_b = dS + dS^T
      d K*x += -s^2 dT^T Q_b   (Q_b = P_b U^T, through R = K*x L^{-T})
      d K_bX = s^2 L_rr^{-T} dT (through K(X_b, X))
    and post_backward reduces both through dk/dx."""

    @staticmethod
    def forward(ctx, X3, acqf):
        model = acqf.model
        cache = model.prediction_cache()
        ymean, ystd = model.outcome_stats()
        q = X3.shape[-2]
        need_grad = ctx.needs_input_grad[0]
        pp = kernels.post_partials(cache, X3.detach(), store_R=need_grad, cross=acqf._root.Q_b)
        T, F = acqf._root.forward(cache, pp, ystd)
        Zq = acqf._base_samples_q(q, X3.device)
        lp = getattr(acqf, "_log_params", None)
        out = kernels.qmc_finalize(cache, pp, acqf._fused_mode, ymean, ystd, Z=Zq,
                                   best_f_s=acqf._baseline_best_f, want_mean=need_grad,
                                   want_cov=False, want_L=need_grad, T=T, F=F, log_params=lp)
        kernels._raise_not_psd(out["info"], out["jitter"], type(acqf).__name__)
        if need_grad:
            ctx.acqf, ctx.cache, ctx.pp, ctx.ystd = acqf, cache, pp, ystd
            ctx.lp, ctx.acq = lp, out["acq"].detach().clone()
            ctx.T, ctx.F, ctx.Zq = T, F, Zq
            ctx.mean, ctx.L = out["mean"], out["L"]
            ctx.W = kernels.w_matrix(cache, pp)
        return out["acq"]

    @staticmethod
    def backward(ctx, dacq):
        acqf, cache, pp, ystd = ctx.acqf, ctx.cache, ctx.pp, ctx.ystd
        dmean, dcov, dF = kernels.qmc_backward(acqf._fused_mode, ctx.mean, ctx.L, ctx.Zq,
                                               dacq.contiguous(), best_f_s=acqf._baseline_best_f,
                                               F=ctx.F, acq_fwd=ctx.acq, log_params=ctx.lp)
        dX = acqf._root.backward(cache, pp, ctx.W, dmean, dcov, dF, ctx.T, ystd)
        return dX, None


# -- LogEI family ---------------------------------------------------------------------
def _check_tau(tau, name: str):
    """acquisition/logei.py:537-544."""
    if isinstance(tau, torch.Tensor) and tau.numel() != 1:
        raise ValueError(name + f" is not a scalar: {tau.numel() = }.")
    if not (tau > 0):
        raise ValueError(name + f" is non-positive: {tau = }.")
    return tau


class qLogExpectedImprovement(qExpectedImprovement):
    """MC batch log expected improvement (acquisition/logei.py:71-234):
    qLogEI(X) = logmeanexp_s q_reduce_j log_soft_clamp(Y_sj - best_f), with
    q_reduce = fatmax(tau_max) and log_soft_clamp = log_fatplus(tau_relu) when
    fat (default), else smooth_amax / log_softplus; constraints add the
    log-feasibility (fatmoid when fat).

    Fused path: bo_qmc_finalize in BO_QMC_QLOGEI mode (the same post_partials
    posterior and q x q root as qEI; only the per-sample reduction differs),
    backward through bo_qmc_backward's dense log-mode weights."""

    _log = True

    def __init__(self, model, best_f, sampler=None, objective=None, posterior_transform=None,
                 X_pending=None, constraints=None, eta=1e-3, fat: bool = True,
                 tau_max: float = TAU_MAX, tau_relu: float = TAU_RELU):
        super().__init__(model, best_f, sampler, objective, posterior_transform, X_pending,
                         constraints=constraints, eta=eta)
        self.tau_max = _check_tau(tau_max, "tau_max")
        self.tau_relu = _check_tau(tau_relu, "tau_relu")
        self._fat = fat
        self._log_params = (int(bool(fat)), float(tau_relu), float(tau_max))

    def _sample_forward(self, obj: torch.Tensor) -> torch.Tensor:
        """logei.py:219-234."""
        return log_improvement(obj, self.best_f, tau=self.tau_relu, fat=self._fat)

    def _q_reduction(self, acqval: torch.Tensor) -> torch.Tensor:
        return (fatmax if self._fat else smooth_amax)(acqval, dim=-1, tau=self.tau_max)

    def _sample_reduction(self, acqval: torch.Tensor) -> torch.Tensor:
        return logmeanexp(acqval, dim=tuple(range(len(self.sample_shape))))

    def forward(self, X: torch.Tensor) -> torch.Tensor:
        X = self._concat_pending(t_batch_mode(X))
        batch = X.shape[:-2]
        q, d = X.shape[-2], X.shape[-1]
        if self._fused_eligible(X) and self.best_f.numel() == 1:
            sampler = self._ensure_sampler()
            Z = sampler.base_samples_2d(q, X.device)
            acq = _fused_mc(X.reshape(-1, q, d), self, _lib.QMC_QLOGEI,
                            _host_scalar(self, "best_f"), None, Z)
            return acq.reshape(batch)
        return self._generic_forward(X)


class qLogNoisyExpectedImprovement(qNoisyExpectedImprovement):
    """MC batch log noisy expected improvement (acquisition/logei.py:236-507):
    the qNEI samples (cached root or full joint, as qNoisyExpectedImprovement)
    under the LogEI reductions against the per-sample baseline best.  Unlike
    qNEI, ``prune_baseline`` defaults to False (logei.py:270).  Fused path:
    bo_qmc_finalize / bo_qmc_backward in BO_QMC_QLOGNEI mode."""

    _log = True
    _fused_mode = _lib.QMC_QLOGNEI

    def __init__(self, model, X_baseline, sampler=None, objective=None, posterior_transform=None,
                 X_pending=None, constraints=None, eta=1e-3, fat: bool = True,
                 prune_baseline: bool = False, cache_root: bool = True,
                 tau_max: float = TAU_MAX, tau_relu: float = TAU_RELU, marginalize_dim=None):
        MCAcquisitionFunction.__init__(self, model, sampler, objective, posterior_transform,
                                       X_pending, constraints=constraints, eta=eta, fat=fat)
        self.tau_max = _check_tau(tau_max, "tau_max")
        self.tau_relu = _check_tau(tau_relu, "tau_relu")
        self._log_params = (int(bool(fat)), float(tau_relu), float(tau_max))
        self._init_baseline(model, X_baseline, prune_baseline, cache_root, marginalize_dim)

    def _sample_forward(self, obj: torch.Tensor) -> torch.Tensor:
        """logei.py:347-362."""
        return log_improvement(obj, self.compute_best_f(obj), tau=self.tau_relu, fat=self._fat)

    def _q_reduction(self, acqval: torch.Tensor) -> torch.Tensor:
        return (fatmax if self._fat else smooth_amax)(acqval, dim=-1, tau=self.tau_max)

    def _sample_reduction(self, acqval: torch.Tensor) -> torch.Tensor:
        return logmeanexp(acqval, dim=tuple(range(len(self.sample_shape))))


# -- qEHVI ---------------------------------------------------------------------------
def _qehvi_members_eager(acqf, X3: torch.Tensor):
    """Forward-only qEHVI through ONE native call (bo::qehvi_members_eager:
    every member's rows, K*x^T, posterior partials, finalisation and the
    qEHVI launch, issued from C++).  The members' ladder outcomes are
    deferred as the eager qEI's (a ring of pinned slots: the previous calls'
    outcomes are acted on here, kernels.check_ladder_status waits for all);
    with BO_SYNC_LADDER=1, one stream sync and the members' outcomes raised /
    warned in member order.
    None where it does not apply (graph capture; members of unequal shape or
    kernel; more than 8 members): the caller takes _FusedQEHVI."""
    dev = X3.device
    idx = kernels._dev_index(dev)
    if idx in kernels._CAPTURE:
        return None
    models = acqf.model.models
    if len(models) > 8:
        return None
    keys = prime_prediction_caches(models)
    key = (tuple(keys), idx)
    args = acqf.__dict__.get("_native_args")
    if args is None or args[0] != key:
        caches = [mm.prediction_cache(key=k) for mm, k in zip(models, keys)]
        c0 = caches[0]
        if not all(c.n == c0.n and c.np == c0.np and c.d == c0.d and c.kind == c0.kind
                   and c.U.numel() for c in caches):
            return None
        stats = [mm.outcome_stats() for mm in models]
        args = (key, [c.Xt_scaled for c in caches], [c.U for c in caches],
                [c.beta for c in caches], [c.lengthscale for c in caches],
                [float(c.outputscale) for c in caches], [float(c.constant) for c in caches],
                [float(m_) for m_, _ in stats], [float(s_) for _, s_ in stats], int(c0.kind),
                int(c0.n))
        acqf.__dict__["_native_args"] = args
    q = X3.shape[-2]
    Z = acqf._ensure_sampler().base_samples_2d(q * len(models), dev)
    lo, hi = acqf._cells(dev)
    defer = not kernels.SYNC_LADDER
    acq, status = _lib.torch_ops().qehvi_members_eager(
        X3.contiguous(), *args[1:], Z, lo, hi, kernels.kxt_cap(dev), defer)
    if defer:
        # as the eager qEI: the previous calls' outcomes, this one's pending
        # (kernels.check_ladder_status / the optimisers' end-of-loop poll)
        kernels.ladder_prev_outcome(status, idx, "qEHVI posterior root")
    else:
        kernels._stream_sync(dev)
        kernels.raise_status_words(status.tolist(), "qEHVI posterior root")
    return acq


class _FusedQEHVI(torch.autograd.Function):
    """qEHVI of B t-batches over a ModelListGP, with its gradient.

    Forward: per output, post_partials + qmc_finalize(CHOL) (posterior mean and
    jittered q x q root), then bo_qehvi over (sample, cell) pairs.
    Backward: bo_qehvi_backward (inclusion-exclusion derivative) -> d mu_t, d L_t;
    bo_chol_backward -> d Sigma_t; bo_post_backward per output model."""

    @staticmethod
    def forward(ctx, X3, acqf):
        models = acqf.model.models
        need_grad = ctx.needs_input_grad[0]
        q = X3.shape[-2]
        saved = []
        keys = prime_prediction_caches(models)
        caches = [mm.prediction_cache(key=key) for mm, key in zip(models, keys)]
        # every member's posterior partials in one launch where the small-grid
        # plan applies (C4: the three outputs of the ModelListGP)
        pps = kernels.post_partials_members(caches, X3.detach(), store_R=need_grad)
        status = []
        # every member's mean and q x q root written straight into its slice of
        # the stacked m x B x q (x q) inputs of the qEHVI launch (no stack copies)
        f64 = dict(dtype=torch.float64, device=X3.device)
        mean = torch.empty(len(models), X3.shape[0], q, **f64)
        L = torch.empty(len(models), X3.shape[0], q, q, **f64)
        # outside graph capture the finalisation launches fold their ladder
        # outcomes straight into pinned words (no status launches or copy); on
        # the gradient path those words are read at the end of the backward
        # (kernels._LadderRing), else once behind the qEHVI launch
        idx = kernels._dev_index(X3.device)
        pinned = idx not in kernels._CAPTURE and len(models) <= 8
        ring = (kernels.ladder_ring(X3.device) if pinned and need_grad and not kernels.SYNC_LADDER
                else None)
        ps = kernels.pinned_status(X3.device) if pinned and ring is None else None
        if ring is not None:
            token, words = ring.take(len(models), "qEHVI posterior root")
        else:
            words = ps.arm(len(models)) if ps is not None else [None] * len(models)
        stats = [mm.outcome_stats() for mm in models]
        if (len(models) <= 8 and all(p_.Spart.shape == pps[0].Spart.shape for p_ in pps)
                and all(c.kind == caches[0].kind for c in caches)):
            # every member's finalisation in one launch
            info, jit = kernels.qmc_finalize_members(caches, pps, stats, mean, L,
                                                     status=words if pinned else None)
            status = [(info[t], jit[t]) for t in range(len(models))]
        else:
            for t, (cache, pp) in enumerate(zip(caches, pps)):
                out = kernels.qmc_finalize(cache, pp, _lib.QMC_CHOL, *stats[t], want_mean=True,
                                           want_cov=False, want_L=True, mean_out=mean[t],
                                           L_out=L[t], status=words[t])
                status.append((out["info"], out["jitter"]))
        if need_grad:
            Ws = kernels.w_matrix_members(caches, pps)   # one launch where stream-K
            for t, (cache, pp) in enumerate(zip(caches, pps)):
                saved.append((cache, pp, stats[t][1], Ws[t]))
        sampler = acqf._ensure_sampler()
        Z = sampler.base_samples_2d(q * len(models), X3.device)
        lo, hi = acqf._cells(X3.device)
        # the kernel itself (as the backward below): this Function already is
        # the autograd node, the registered op's wrapper would only add host time
        acq = kernels.qehvi(mean, L, Z, lo, hi)
        # the members' ladders checked once, behind the qEHVI launch (one host
        # read per forward instead of one per member, each of which drained
        # the queue: ~40 us of idle device between members at C4)
        ctx.ladder = None
        if ring is not None:
            ring.record(token)
            ctx.ladder = (ring, token)
        elif ps is not None:
            kernels.raise_not_psd_members(ps, len(models), X3.device, "qEHVI posterior root")
        else:
            kernels.raise_not_psd_many(status, "qEHVI posterior root")
        if need_grad:
            ctx.saved, ctx.mean, ctx.L, ctx.Z, ctx.cells = saved, mean, L, Z, (lo, hi)
        return acq

    @staticmethod
    def backward(ctx, dacq):
        lo, hi = ctx.cells
        dmean, dL = kernels.qehvi_backward(ctx.mean, ctx.L, ctx.Z, lo, hi, dacq)
        dX = None
        sv = ctx.saved
        if (_PB_JOBS and 1 < len(sv) <= 16 and all(
                c.kind == sv[0][0].kind and c.d == sv[0][0].d for c, _, _, _ in sv)):
            # every member's Cholesky backward, then posterior backward pass, in one launch each
            q_ = ctx.L.shape[-1]
            dcovs = kernels.chol_backward(ctx.L.reshape(-1, q_, q_),
                                          dL.reshape(-1, q_, q_)).reshape(ctx.L.shape)
            dX = kernels.post_backward_jobs([
                dict(cache=cache, pp=pp, W=W, dmean=dmean[t], ystd=ystd, dcov=dcovs[t])
                for t, (cache, pp, ystd, W) in enumerate(sv)])
        else:
            for t, (cache, pp, ystd, W) in enumerate(sv):
                dcov = kernels.chol_backward(ctx.L[t], dL[t])
                dX = kernels.post_backward(cache, pp, W, dmean[t], dcov, ystd, dX=dX)
        _settle_ladder(ctx)
        return dX, None


def _settle_ladder(ctx) -> None:
    """The forward's deferred ladder outcome (kernels._LadderRing), read once
    the backward's launches are queued behind it."""
    lad = getattr(ctx, "ladder", None)
    if lad is not None:
        ctx.ladder = None
        lad[0].settle(lad[1])


class IdentityMCMultiOutputObjective(MCObjective):
    """acquisition/multi_objective/objective.py (identity over outputs)."""

    def forward(self, samples, X=None):
        return samples


class qExpectedHypervolumeImprovement(MCAcquisitionFunction):
    """MC qEHVI (acquisition/multi_objective/monte_carlo.py:146-322) over the
    hypercells of a non-dominated partitioning.

    Fused path (ModelListGP of SingleTaskGPs, identity objective): per output,
    the exact posterior of the B t-batches (post_partials + the per-t-batch
    jittered Cholesky, qmc_finalize in CHOL mode), then one bo_qehvi launch that
    draws the non-interleaved Sobol samples and evaluates the inclusion-exclusion
    hypervolume improvement over (sample, hypercell) pairs."""

    _default_sample_shape = torch.Size([128])

    def __init__(self, model, ref_point, partitioning, sampler=None, objective=None,
                 constraints=None, X_pending=None, eta=1e-3, fat=False):
        if len(ref_point) != partitioning.num_outcomes:
            raise ValueError(
                "The length of the reference point must match the number of outcomes. "
                f"Got ref_point with {len(ref_point)} elements, but expected "
                f"{partitioning.num_outcomes}.")
        if constraints is not None:
            raise UnsupportedError("outcome constraints are not on the accelerated path")
        AcquisitionFunction.__init__(self, model)
        self.sampler = sampler
        self.objective = objective if objective is not None else IdentityMCMultiOutputObjective()
        self.posterior_transform = None
        self.set_X_pending(X_pending)
        self.ref_point = torch.as_tensor(ref_point, dtype=torch.float64)
        lo, hi = partitioning.get_hypercell_bounds()
        self.cell_lower_bounds = lo.to(torch.float64)
        self.cell_upper_bounds = hi.to(torch.float64)
        self._dev_cells = {}

    def _cells(self, device):
        key = str(device)
        if key not in self._dev_cells:
            self._dev_cells[key] = (self.cell_lower_bounds.to(device).contiguous(),
                                    self.cell_upper_bounds.to(device).contiguous())
        return self._dev_cells[key]

    def forward(self, X: torch.Tensor) -> torch.Tensor:
        X = self._concat_pending(t_batch_mode(X))
        batch = X.shape[:-2]
        q, d = X.shape[-2], X.shape[-1]
        X3 = X.reshape(-1, q, d)
        models = getattr(self.model, "models", None)
        if models is None or not all(hasattr(mm, "prediction_cache") for mm in models):
            raise UnsupportedError("qEHVI here runs on a ModelListGP of SingleTaskGPs")
        if not isinstance(self.objective, IdentityMCMultiOutputObjective):
            raise UnsupportedError("only the identity multi-output objective is accelerated")
        if q > 12 or d > kernels.DP:
            raise UnsupportedError("fused qEHVI supports q <= 12 and d <= 8")
        acq = None
        if not (torch.is_grad_enabled() and X3.requires_grad) and X3.dtype == torch.float64:
            acq = _qehvi_members_eager(self, X3)
        if acq is None:
            acq = _FusedQEHVI.apply(X3, self)
        return acq.reshape(batch)


# -- qNEHVI ------------------------------------------------------------------------------
def prune_inferior_points_multi_objective(model, X, ref_point, objective=None, constraints=None,
                                          num_samples: int = 2048, max_frac: float = 1.0,
                                          marginalize_dim=None, chunk: int = 64):
    """acquisition/multi_objective/utils.py:77-161 (unconstrained, identity
    objective): keep the points with a positive probability of being
    Pareto-optimal and better than ref_point under ``num_samples`` joint
    posterior samples (drawn on the device; Pareto masks in sample chunks)."""
    from .multi_objective import is_non_dominated
    if X.ndim > 2:
        raise UnsupportedError("Batched inputs `X` are currently unsupported by "
                               "prune_inferior_points_multi_objective")
    if max_frac <= 0 or max_frac > 1.0:
        raise ValueError(f"max_frac must take values in (0, 1], is {max_frac}")
    if constraints is not None:
        raise UnsupportedError("constraints are not on the accelerated path")
    max_points = math.ceil(max_frac * X.size(-2))
    ref = torch.as_tensor(ref_point, dtype=torch.float64, device=X.device)
    models = getattr(model, "models", [model])
    n, m = X.shape[-2], len(models)
    with torch.no_grad():
        # joint samples of the independent outputs: Sobol dimension n m,
        # point-major / output-minor base samples (get_sampler on the MTMVN),
        # seeded as the reference's sampler seeds itself from the global
        # generator (sampling/base.py: torch.randint(0, 1000000, (1,)))
        if n * m <= 21201:
            seed = int(torch.randint(0, 1000000, (1,)).item())
            Z = kernels.sobol_normal(n * m, num_samples, seed, X.device).view(num_samples, n, m)
        else:
            Z = torch.randn(num_samples, n, m, dtype=torch.float64, device=X.device)
        cols = []
        for t, mm in enumerate(models):
            post = mm.posterior(X)
            mean = post.distribution.mean.reshape(1, n)
            L, _, _ = kernels.cholesky_with_inverse(post.distribution.covariance_matrix.reshape(n, n))
            cols.append(kernels.sample_mvn(mean, L.unsqueeze(0).contiguous(),
                                           Z[:, :, t].contiguous()).reshape(num_samples, n))
        obj = torch.stack(cols, dim=-1)  # S x n x m
        if objective is not None:
            obj = objective(obj, X=X)
        hits = torch.zeros(n, dtype=torch.float64, device=X.device)
        # one device launch for all samples (bo_pareto_mask); host tensors chunked
        step = obj.shape[0] if obj.is_cuda else chunk
        for s0 in range(0, obj.shape[0], step):
            o = obj[s0:s0 + step]
            mask = is_non_dominated(o, deduplicate=False) & (o > ref).all(dim=-1)
            hits += mask.to(torch.float64).sum(dim=0)
    probs = hits / obj.shape[0]
    idcs = probs.nonzero().view(-1)
    if idcs.shape[0] > max_points:
        counts, order_idcs = torch.sort(probs, descending=True)
        idcs = order_idcs[:max_points]
    return X[idcs]


class _FusedQNEHVI(torch.autograd.Function):
    """qNEHVI of B t-batches over a ModelListGP with cached baseline roots,
    with its gradient.

    Forward, per output t: post_partials (+ R^T), the cached-root terms
    T_t = L_rr,t^{-1} Sigma'_t(X_b, X) and F_t = Z_b,t T_t (two MFMA GEMMs + one),
    qmc_finalize(CHOL) on Sigma'_t - T_t^T T_t -> mean_t, L_t; then one bo_qehvi
    launch over (sample, per-sample hypercell) pairs with f = mean + F + L Z_q.
    Backward: bo_qehvi_backward (d mean, d L, d F) -> bo_chol_backward ->
    the cached-root backward of each output (dT = Z_b^T dF - T G)."""

    @staticmethod
    def forward(ctx, X3, acqf):
        models = acqf.model.models
        need_grad = ctx.needs_input_grad[0]
        q = X3.shape[-2]
        saved, status = [], []
        pp = None
        keys = prime_prediction_caches(models)
        caches = [mm.prediction_cache(key=key) for mm, key in zip(models, keys)]
        # where the one-model plan splits k (C4), the cross term cannot ride in
        # the posterior pass and R^T is stored anyway: then every member's
        # partials + R^T in one launch (post_partials_members)
        B, q_, _ = X3.shape
        c0 = caches[0]
        pps = None
        if (1 < len(models) <= 8 and kernels.split_plan(B, q_, c0.n)[0] != 0
                and all(c.n == c0.n and c.np == c0.np and c.d == c0.d for c in caches)):
            pps = kernels.post_partials_members(caches, X3.detach(), store_R=True)
        # the members' means, roots and baseline terms written straight into
        # the stacked qEHVI inputs; outside graph capture their ladder
        # outcomes folded into pinned words (as qEHVI's forward)
        f64 = dict(dtype=torch.float64, device=X3.device)
        M = len(models)
        mean = torch.empty(M, B, q_, **f64)
        L = torch.empty(M, B, q_, q_, **f64)
        F = None
        idx = kernels._dev_index(X3.device)
        # forward-only calls defer the ladder outcome (the eager qEI's ring:
        # no stream sync per call); the gradient path folds it into pinned
        # words read at the end of the backward (kernels._LadderRing)
        defer = not need_grad and not kernels.SYNC_LADDER and idx not in kernels._CAPTURE
        pinned = not defer and idx not in kernels._CAPTURE and M <= 8
        ring = kernels.ladder_ring(X3.device) if pinned and not kernels.SYNC_LADDER else None
        ps = kernels.pinned_status(X3.device) if pinned and ring is None else None
        if ring is not None:
            token, words = ring.take(M, "qNEHVI posterior root")
        else:
            words = ps.arm(M) if ps is not None else [None] * M
        stats = [mm.outcome_stats() for mm in models]
        batched = pps is not None and _roots_batched(acqf, caches, pps, stats)
        if batched:
            # every member's T and F in three batched GEMMs over the members
            Ts, F = _roots_forward_batched(acqf, caches, pps, stats)
            pp_list = list(pps)
            if need_grad:
                Ws = kernels.w_matrix_members(caches, pps)
                for t in range(M):
                    saved.append((caches[t], pps[t], stats[t][1], Ts[t], Ws[t]))
        else:
            Ts, pp_list = [], []
            for t, mm in enumerate(models):
                cache = caches[t]
                ystd = stats[t][1]
                pp = pps[t] if pps is not None else kernels.post_partials(
                    cache, X3.detach(), store_R=need_grad, cross=acqf._roots[t].Q_b)
                pp_list.append(pp)
                if F is None:
                    F = torch.empty(M, acqf._roots[t].Z_base.shape[0], pp.nrows_pad, **f64)
                T, _ = acqf._roots[t].forward(cache, pp, ystd, F_out=F[t])
                Ts.append(T)
                if need_grad:
                    saved.append((cache, pp, ystd, T, kernels.w_matrix(cache, pp)))
        pp = pp_list[-1]
        same_parts = all(p_.Spart.shape == pp_list[0].Spart.shape for p_ in pp_list)
        if M <= 8 and same_parts and all(c.kind == caches[0].kind for c in caches):
            # every member's finalisation in one launch
            info, jit = kernels.qmc_finalize_members(
                caches, pp_list, stats, mean, L, status=words if pinned else None,
                Ts=Ts, F=F)
            status = [(info[t], jit[t]) for t in range(M)]
        else:
            for t in range(M):
                out = kernels.qmc_finalize(caches[t], pp_list[t], _lib.QMC_CHOL, *stats[t],
                                           want_mean=True, want_cov=False, want_L=True, T=Ts[t],
                                           F=F[t], mean_out=mean[t], L_out=L[t], status=words[t])
                status.append((out["info"], out["jitter"]))
        Zq = acqf._base_samples_q(q, X3.device)
        lo, hi = acqf._cells
        acq = kernels.qehvi(mean, L, Zq, lo, hi, F=F, Qp=pp.Qp)
        ctx.ladder = None
        if defer:
            kernels.raise_not_psd_deferred(torch.cat([i_.reshape(-1) for i_, _ in status]),
                                           torch.cat([j_.reshape(-1) for _, j_ in status]),
                                           "qNEHVI posterior root")
        elif ring is not None:
            ring.record(token)
            ctx.ladder = (ring, token)
        elif ps is not None:
            kernels.raise_not_psd_members(ps, M, X3.device, "qNEHVI posterior root")
        else:
            kernels.raise_not_psd_many(status, "qNEHVI posterior root")  # one read (as qEHVI)
        if need_grad:
            ctx.acqf, ctx.saved, ctx.mean, ctx.L, ctx.F, ctx.Zq, ctx.Qp = (
                acqf, saved, mean, L, F, Zq, pp.Qp)
            ctx.batched = batched
        return acq

    @staticmethod
    def backward(ctx, dacq):
        lo, hi = ctx.acqf._cells
        dmean, dL, dF = kernels.qehvi_backward(ctx.mean, ctx.L, ctx.Zq, lo, hi, dacq, F=ctx.F,
                                               Qp=ctx.Qp)
        dX = None
        if ctx.batched and _BWD_BATCHED:
            dX = _roots_backward_batched(ctx, dmean, dL, dF)
        else:
            for t, (cache, pp, ystd, T, W) in enumerate(ctx.saved):
                dcov = kernels.chol_backward(ctx.L[t], dL[t])
                dX = ctx.acqf._roots[t].backward(cache, pp, W, dmean[t], dcov, dF[t].contiguous(),
                                                 T, ystd, dX=dX)
        _settle_ladder(ctx)
        return dX, None


# BO_QNEHVI_BWD_BATCHED=0: the per-member backward on the batched forward (A/B)
_BWD_BATCHED = os.environ.get("BO_QNEHVI_BWD_BATCHED", "1") != "0"
# BO_PB_JOBS=0: the members' post_backward passes one launch each (A/B)
_PB_JOBS = os.environ.get("BO_PB_JOBS", "1") != "0"


def _roots_backward_batched(ctx, dmean, dL, dF):
    """_CachedBaselineRoot.backward for all members at once (the forward's
    batched route): dT = Z_base^T dF and the dK*x / dK(X_b, X) GEMMs batched
    over the members (s^2 folded into the stacked operands), the per-t-batch
    dT -= T G and the two post_backward passes per member."""
    acqf = ctx.acqf
    roots = acqf._roots
    M = len(roots)
    _, Linv_s, _, Zb, _ = acqf.__dict__["_root_stack"]
    Qb_s = acqf.__dict__.get("_root_stack_qb")
    key = acqf.__dict__["_root_stack"][0]
    if Qb_s is None or Qb_s[0] != key:
        s2 = [float(sv) ** 2 for sv in key[0]]
        Qb_s = (key, torch.stack([rt.Q_b * (-s2[t]) for t, rt in enumerate(roots)]).contiguous())
        acqf.__dict__["_root_stack_qb"] = Qb_s
    Qb_s = Qb_s[1]
    dT = kernels.gemm(Zb, dF.contiguous(), transA=True)                 # M x r x N
    r = dT.shape[1]
    q_ = ctx.L.shape[-1]
    dcovs = kernels.chol_backward(ctx.L.reshape(-1, q_, q_), dL.reshape(-1, q_, q_)).reshape(
        ctx.L.shape)                                                    # all members, one launch
    for t, (cache, pp, ystd, T, W) in enumerate(ctx.saved):
        dcov = dcovs[t]
        G = (dcov + dcov.mT).contiguous()
        q, Qp, nrows, B = pp.q, pp.Qp, pp.nrows_pad, pp.B
        kernels.gemm_strided(r, q, q, T, nrows, Qp, G, q, q * q, dT[t], nrows, Qp, B,
                             alpha=-1.0, beta=1.0)                      # dT_b -= T_b G_b
    E = kernels.gemm(dT, Qb_s, transA=True)                             # M x N x np
    # (s^2 L_rr^-T dT)^T = dT^T (s^2 L_rr^-1): already in post_backward's layout
    dKbxT = kernels.gemm(dT, Linv_s, transA=True, flags=_lib.GEMM_B_LOWER)  # M x N x r
    if _PB_JOBS and 2 * M <= 16:
        # every member's training and baseline passes in one launch
        jobs = []
        for t, (cache, pp, ystd, T, W) in enumerate(ctx.saved):
            jobs.append(dict(cache=cache, pp=pp, W=W, dmean=dmean[t], dcov=dcovs[t], ystd=ystd,
                             E=E[t]))
            jobs.append(dict(cache=cache, pp=pp, ystd=ystd, E=dKbxT[t],
                             Xt_scaled=roots[t].Xb_scaled, n=r))
        return kernels.post_backward_jobs(jobs)
    dX = None
    for t, (cache, pp, ystd, T, W) in enumerate(ctx.saved):
        dX = kernels.post_backward(cache, pp, W, dmean[t], dcovs[t], ystd, E=E[t], dX=dX)
        dX = kernels.post_backward(cache, pp, None, None, None, ystd, E=dKbxT[t],
                                   Xt_scaled=roots[t].Xb_scaled, n=r, dX=dX)
    return dX


def _roots_batched(acqf, caches, pps, stats) -> bool:
    """Whether the members' cached-root terms can go as batched GEMMs: R^T
    stacked by the members' route, equal baseline sizes and sample counts."""
    roots = acqf._roots
    if any(p_.Rt is None or p_.Cx is not None for p_ in pps):
        return False
    r0, S0 = roots[0].Linv.shape[0], roots[0].Z_base.shape[0]
    if any(rt.Linv.shape[0] != r0 or rt.Z_base.shape[0] != S0 for rt in roots):
        return False
    base = pps[0].Rt
    step = base.numel()
    return all(p_.Rt.data_ptr() == base.data_ptr() + 8 * step * t and p_.Rt.is_contiguous()
               for t, p_ in enumerate(pps))


def _roots_forward_batched(acqf, caches, pps, stats):
    """_CachedBaselineRoot.forward for all members at once: T_t = s_t^2
    (L_rr,t^-1 K(X_b, X)_t - P_b,t R_t^T), F_t = Z_base,t T_t as three batched
    GEMMs over the members (the s_t^2 folded into stacked copies of L_rr^-1
    and P_b, rebuilt when the outcome scales change)."""
    roots = acqf._roots
    M = len(roots)
    p0 = pps[0]
    dev = p0.Xq.device
    # keyed by the roots too (their identity and baseline size), not only by
    # the outcome scales: _set_cell_bounds rebuilds the roots
    key = (tuple(float(s_[1]) for s_ in stats), str(dev),
           tuple((id(rt), rt.Linv.data_ptr(), rt.Linv.shape[0]) for rt in roots))
    stk = acqf.__dict__.get("_root_stack")
    if stk is None or stk[0] != key:
        s2 = [float(s_[1]) ** 2 for s_ in stats]
        stk = (key, torch.stack([rt.Linv * s2[t] for t, rt in enumerate(roots)]).contiguous(),
               torch.stack([rt.P_b * s2[t] for t, rt in enumerate(roots)]).contiguous(),
               torch.stack([rt.Z_base for rt in roots]).contiguous(),
               torch.ones(kernels.DP, dtype=torch.float64, device=dev))
        acqf.__dict__["_root_stack"] = stk
    _, Linv_s, Pb_s, Zb, ones = stk
    r = Linv_s.shape[1]
    Kbx = torch.empty(M, r, p0.nrows_pad, dtype=torch.float64, device=dev)
    for t, (rt, c, p_) in enumerate(zip(roots, caches, pps)):
        kernels.covar_matrix(rt.Xb_scaled, p_.Xq, ones, c.kind, c.outputscale, out=Kbx[t])
    T = kernels.gemm(Linv_s, Kbx, flags=_lib.GEMM_A_LOWER)
    Rt_all = p0.Rt.as_strided((M,) + tuple(p0.Rt.shape), (p0.Rt.numel(),) + tuple(p0.Rt.stride()))
    T = kernels.gemm(Pb_s, Rt_all, alpha=-1.0, beta=1.0, C=T)
    F = kernels.gemm(Zb, T)
    return [T[t] for t in range(M)], F


class _QEHVIFromRoots(torch.autograd.Function):
    """The fused hypervolume-improvement kernel (bo_qehvi) on caller-made
    sample roots, f_s = mean + F_s + L z_s (mean m x B x q, L m x B x q x q,
    F m x S x B q), as a differentiable function of (mean, L, F)."""

    @staticmethod
    def forward(ctx, mean, L, F, Zq, lo, hi, q):
        acq = kernels.qehvi(mean, L, Zq, lo, hi, F=F, Qp=q)
        ctx.save_for_backward(mean, L, F, Zq, lo, hi)
        ctx.q = q
        return acq

    @staticmethod
    def backward(ctx, dacq):
        mean, L, F, Zq, lo, hi = ctx.saved_tensors
        dmean, dL, dF = kernels.qehvi_backward(mean, L, Zq, lo, hi, dacq.contiguous(), F=F,
                                               Qp=ctx.q)
        return dmean, dL, dF, None, None, None, None


class qNoisyExpectedHypervolumeImprovement(qExpectedHypervolumeImprovement):
    """MC q-noisy expected hypervolume improvement (acquisition/multi_objective/
    monte_carlo.py:325-468; NoisyExpectedHypervolumeMixin,
    utils/multi_objective/hypervolume.py:507-835) for a ModelListGP of
    SingleTaskGPs:

      qNEHVI(X) = mean_s HVI(f_s(X, X_pending) | Pareto front of f_s(X_baseline))
                  + prev_nehvi.

    Construction: the joint baseline samples (Sobol dimension r m), one box
    decomposition of the non-dominated region per sample (exact:
    FastNondominatedPartitioning; alpha > 0: the approximate binary
    partitioning of NondominatedPartitioning, m > 2; both in native host code,
    as the reference runs them on the CPU for m > 2), padded with empty cells to
    a common count (BoxDecompositionList), resident on the device as S x K x m.
    Forward / backward: _FusedQNEHVI over the q new points and the pending
    points not yet in the baseline.

    cache_root=False: every forward samples the joint posterior of each
    t-batch with its own root (_joint_forward) instead of the cached baseline
    root and its low-rank update; the same quantity up to the jitter of the
    (r + q) root.

    Pending points (hypervolume.py:778-822): with cache_pending, more than
    max_iep new ones join the baseline and the decompositions are rebuilt
    (without incremental_nehvi, the hypervolume they add to every sample's
    front, mean_s (HV_s - HV0_s)+, is carried in prev_nehvi); up to max_iep, or
    all of them without cache_pending, are appended to every forward's q-batch
    (concatenate_pending_points)."""

    _default_sample_shape = torch.Size([128])

    def __init__(self, model, ref_point, X_baseline, sampler=None, objective=None,
                 constraints=None, X_pending=None, eta=1e-3, fat=False, prune_baseline=False,
                 alpha=0.0, cache_pending=True, max_iep=0, incremental_nehvi=True,
                 cache_root=True, marginalize_dim=None):
        if len(ref_point) < 2:
            raise ValueError("NoisyExpectedHypervolumeMixin supports m>=2 outcomes "
                             f"but ref_point has length {len(ref_point)}, which is smaller than 2.")
        if X_baseline.ndim > 2:
            raise UnsupportedError("NoisyExpectedHypervolumeMixin does not support batched "
                                   f"X_baseline. Expected 2 dims, got {X_baseline.ndim}.")
        if constraints is not None:
            raise UnsupportedError("outcome constraints are not on the accelerated path")
        models = getattr(model, "models", None)
        if models is None or not all(hasattr(mm, "prediction_cache") for mm in models):
            raise UnsupportedError("qNEHVI here runs on a ModelListGP of SingleTaskGPs")
        if len(models) != len(ref_point):
            raise ValueError("The length of the reference point must match the number of outcomes.")
        AcquisitionFunction.__init__(self, model)
        self.sampler = sampler
        self.objective = objective if objective is not None else IdentityMCMultiOutputObjective()
        if not isinstance(self.objective, IdentityMCMultiOutputObjective):
            raise UnsupportedError("only the identity multi-output objective is accelerated")
        self.posterior_transform = None
        self.ref_point = torch.as_tensor(ref_point, dtype=torch.float64, device=X_baseline.device)
        self.fat = fat
        self.alpha = alpha
        self.cache_pending = bool(cache_pending)
        self._max_iep = int(max_iep)
        self.incremental_nehvi = bool(incremental_nehvi)
        self._cache_root = bool(cache_root)
        self.X_pending = None
        if prune_baseline:
            X_baseline = prune_inferior_points_multi_objective(model, X_baseline, self.ref_point)
        self._X_baseline = X_baseline
        self._X_baseline_and_pending = X_baseline
        self._partitioned = False
        # on the baseline's device, as the reference's tkwargs buffer
        # (hypervolume.py:619-622): a host scalar here made every forward's
        # ``+ prev_nehvi`` a pageable copy that drained the stream (C4
        # qNEHVI forward + backward: ~150 us of idle device per call)
        self.register_buffer("_prev_nehvi", torch.tensor(0.0, dtype=torch.float64,
                                                         device=X_baseline.device))
        if X_pending is not None:
            self.set_X_pending(X_pending)
        # hypervolume.py:643-644: the first decomposition, unless set_X_pending
        # already made it (more than max_iep pending points joined the
        # baseline).  Without cache_pending nothing joins, and the reference's
        # condition would skip the decomposition altogether (its first forward
        # then fails on the missing cell bounds): it is made here.
        if not self._partitioned:
            self._set_cell_bounds()

    @property
    def X_baseline(self) -> torch.Tensor:
        return self._X_baseline_and_pending

    def set_X_pending(self, X_pending=None) -> None:
        """hypervolume.py:778-822."""
        if X_pending is None:
            self.X_pending = None
            return
        if X_pending.requires_grad:
            warnings.warn("Pending points require a gradient but the acquisition function"
                          " will not provide a gradient to these points.", BotorchWarning)
        X_pending = X_pending.detach().clone()
        if not self.cache_pending:
            self.X_pending = X_pending
            return
        joined = torch.cat([self._X_baseline, X_pending], dim=-2)
        num_new = joined.shape[0] - self.X_baseline.shape[0]
        if num_new <= 0:
            return
        if num_new > self._max_iep:
            self._X_baseline_and_pending = joined
            self._set_cell_bounds()
            if not self.incremental_nehvi:
                self._prev_nehvi = (self._hypervolumes - self._initial_hvs).clamp_min(0.0).mean()
            self.X_pending = None
        else:
            self.X_pending = X_pending[-num_new:]

    def _set_cell_bounds(self) -> None:
        """hypervolume.py:680-776: baseline samples and one box decomposition per
        MC sample (native host threads), padded to a common cell count
        (box_decomposition_list.py:62-94), then resident on the device.  The
        first decomposition of a non-incremental qNEHVI records every sample's
        baseline hypervolume (_compute_initial_hvs, :654-678)."""
        Xb = self.X_baseline
        models = self.model.models
        r, m = Xb.shape[-2], len(models)
        if r == 0:
            raise UnsupportedError("qNEHVI here needs at least one baseline point")
        sampler = self._ensure_sampler()
        S = sampler.sample_shape.numel()
        Zb = kernels.sobol_normal(r * m, S, sampler.seed, Xb.device).view(S, r, m)
        self._roots = [_CachedBaselineRoot(mm, Xb, Zb[:, :, t].contiguous())
                       for t, mm in enumerate(models)]
        # the members' stacked root operands (_roots_forward_batched /
        # _roots_backward_batched) belong to the previous roots: a baseline
        # that grew by pending points has a different r
        self.__dict__.pop("_root_stack", None)
        self.__dict__.pop("_root_stack_qb", None)
        if not all(rt.fused_ready for rt in self._roots):
            raise UnsupportedError(f"qNEHVI here needs d <= {kernels.DP}")
        Y = torch.stack([rt.samples for rt in self._roots], dim=-1).cpu()  # S x r x m
        if self.alpha > 0 and m > 2:  # NondominatedPartitioning(alpha); m = 2 is exact there
            lo, hi = kernels.nd_partition_host(Y, self.ref_point.cpu(), alpha=self.alpha)
        else:
            lo, hi = kernels.nd_partition_host(Y, self.ref_point.cpu())  # native, threaded
        self.cell_lower_bounds = lo.to(Xb.device)
        self.cell_upper_bounds = hi.to(Xb.device)
        self._cells = (self.cell_lower_bounds, self.cell_upper_bounds)
        self.baseline_samples = Y
        self._zq = {}
        if not self._partitioned and not self.incremental_nehvi:
            self._initial_hvs = dominated_hypervolume(Y, self.ref_point.cpu()).to(self.ref_point)
        self._partitioned = True

    @property
    def _hypervolumes(self) -> torch.Tensor:
        """hypervolume.py:824-835: every sample's hypervolume over the current
        baseline, from its cells (non_dominated.py:445-457)."""
        return cells_hypervolume(self.baseline_samples, self.ref_point.cpu(),
                                 self.cell_lower_bounds.cpu(),
                                 self.cell_upper_bounds.cpu()).to(self.ref_point)

    def _base_samples_q(self, q: int, device) -> torch.Tensor:
        """The q m new columns of the (r+q) m-dim Sobol draw (sampling/normal.py:
        68-131): point-major, output-minor, i.e. column p m + t for new point p."""
        if q not in self._zq:
            r, m = self.X_baseline.shape[-2], len(self.model.models)
            S = self.sampler.sample_shape.numel()
            full = kernels.sobol_normal((r + q) * m, S, self.sampler.seed, device)
            self._zq[q] = full[:, r * m:].contiguous()
        return self._zq[q]

    def forward(self, X: torch.Tensor) -> torch.Tensor:
        X = self._concat_pending(t_batch_mode(X))
        batch = X.shape[:-2]
        q, d = X.shape[-2], X.shape[-1]
        if q > 12 or d > kernels.DP or not X.is_cuda:
            raise UnsupportedError(f"fused qNEHVI supports q <= 12 (pending points included) "
                                   f"and d <= {kernels.DP} on the device")
        X3 = X.reshape(-1, q, d)
        if self._cache_root:
            acq = _FusedQNEHVI.apply(X3, self)
        else:
            acq = self._joint_forward(X3)
        return acq.reshape(batch) + self._prev_nehvi.to(acq)

    def _joint_forward(self, X3: torch.Tensor) -> torch.Tensor:
        """cache_root=False (monte_carlo.py:444-468, cached_cholesky.py:161-165):
        every forward samples the joint posterior over [X_baseline; X] of each
        t-batch -- its own jittered (r + q) Cholesky -- with the cached
        baseline base samples in the leading r columns (the base sampler's)
        and the new point's columns after them, and keeps the new rows:
        f = mean_X + Z_b L[X, b]^T + L[X, X] z.  The hypervolume improvement
        over the per-sample cells is the fused kernel's; moments, the joint
        root and its gradient are the general differentiable kernels'."""
        B, q, d = X3.shape
        Xb = self.X_baseline.to(X3)
        r = Xb.shape[-2]
        Xf = torch.cat([Xb.expand(B, r, d), X3], dim=-2)
        means, Ls, Fs = [], [], []
        for t, mm in enumerate(self.model.models):
            post = mm.posterior(Xf)
            mean = post.distribution.mean.reshape(B, r + q)
            Lj = post.distribution.scale_tril.reshape(B, r + q, r + q)
            Zb = self._roots[t].Z_base.to(Lj)                              # S x r
            F = torch.matmul(Zb, Lj[:, r:, :r].mT).permute(1, 0, 2)       # S x B x q
            means.append(mean[:, r:])
            Ls.append(Lj[:, r:, r:])
            Fs.append(F.reshape(Zb.shape[0], B * q))
        Zq = self._base_samples_q(q, X3.device)
        lo, hi = self._cells
        return _QEHVIFromRoots.apply(torch.stack(means), torch.stack(Ls), torch.stack(Fs), Zq,
                                     lo, hi, q)


def cells_hypervolume(Y: torch.Tensor, ref: torch.Tensor, lo: torch.Tensor,
                      hi: torch.Tensor) -> torch.Tensor:
    """FastNondominatedPartitioning.compute_hypervolume (box_decompositions/
    non_dominated.py:445-457) per sample: the box [ref, ideal] less the
    non-dominated cells clipped to it; ideal = the best value of every outcome
    over the points above ref (those of the Pareto front); 0 without one.
    Y: S x n x m, lo / hi: S x K x m (padded cells are empty)."""
    above = (Y > ref).all(dim=-1, keepdim=True)
    ideal = torch.where(above, Y, torch.full_like(Y, float("-inf"))).max(dim=-2, keepdim=True).values
    has = above.any(dim=-2).squeeze(-1)
    total = (ideal.squeeze(-2) - ref).clamp_min(0.0).prod(dim=-1)
    clip_lo, clip_hi = torch.minimum(lo, ideal), torch.minimum(hi, ideal)
    non_dom = (clip_hi - clip_lo).clamp_min(0.0).prod(dim=-1).sum(dim=-1)
    return torch.where(has, total - non_dom, torch.zeros_like(total))


def dominated_hypervolume(Y: torch.Tensor, ref: torch.Tensor) -> torch.Tensor:
    """Every sample's dominated hypervolume (DominatedPartitioning.
    compute_hypervolume, box_decompositions/dominated.py:51-62, as
    _compute_initial_hvs uses it): through the exact non-dominated cells of the
    same points, whose complement in [ref, ideal] it is."""
    lo, hi = kernels.nd_partition_host(Y, ref)
    return cells_hypervolume(Y, ref, lo, hi)


def _acq_device(acqf) -> Optional[torch.device]:
    """The device an acquisition's model lives on (its training inputs, or a
    ModelListGP member's), None when it has none."""
    model = getattr(acqf, "model", None)
    for m in [model] + list(getattr(model, "models", None) or []):
        ti = getattr(m, "train_inputs", None) if m is not None else None
        if ti:
            return ti[0].device
    return None


class FixedFeatureAcquisitionFunction(AcquisitionFunction):
    """acquisition/fixed_feature.py:54-200: the base acquisition over the full
    d-dim input, evaluated on X of dim d' = d - d_f with the ``columns`` filled
    from ``values``.  The optimisers use it to drop fixed features from the
    search space (generation/utils.py:102-196).  The fixed values live on the
    base acquisition's device from construction, and filling the columns is one
    concatenation and one index_select with a device index, so no host data
    moves per call and the fused forward of the base acquisition (and its
    HIP-graph capture) is unchanged."""

    def __init__(self, acq_function: AcquisitionFunction, d: int, columns: List[int], values):
        nn.Module.__init__(self)
        self.acq_func = acq_function
        self.d = d
        home = _acq_device(acq_function)
        if torch.is_tensor(values):
            vals = values.detach().clone()
        else:
            # python numbers are fp64 (fixed_feature.py:25-37); tensors keep shape
            single = all(torch.is_tensor(v) and v.dtype == torch.float32 for v in values)
            dtype = torch.float32 if single else torch.float64
            dev = next((v.device for v in values if torch.is_tensor(v) and v.is_cuda),
                       home or torch.device("cpu"))
            parts = []
            for v in values:
                t = torch.tensor([float(v)], dtype=dtype) if not torch.is_tensor(v) else (
                    v.detach().clone().reshape(1) if v.ndim == 0 else v.detach().clone())
                parts.append(t.to(dtype=dtype, device=dev))
            vals = torch.cat(torch.broadcast_tensors(*parts), dim=-1)
        if home is not None:
            vals = vals.to(home)
        self.register_buffer("values", vals)
        # column i of X_full: from X (free) or from the appended values (fixed)
        d_f = vals.shape[-1]
        cols = set(columns)
        free = iter(range(d - d_f))
        fixed = iter(range(d - d_f, d))
        self._selector = [next(fixed) if i in cols else next(free) for i in range(d)]
        self._placed = {}  # (device, dtype) -> (values, device index of the selector)

    @property
    def model(self):
        return self.acq_func.model

    @property
    def X_pending(self):
        try:
            return self.acq_func.X_pending
        except AttributeError:
            raise ValueError(f"Base acquisition function {type(self.acq_func).__name__} does not "
                             "have an `X_pending` attribute.")

    @X_pending.setter
    def X_pending(self, X_pending):
        if "acq_func" not in self._modules:  # AcquisitionFunction.__init__ is skipped
            return
        self.acq_func.X_pending = (self._construct_X_full(X_pending) if X_pending is not None
                                   else None)

    def set_X_pending(self, X_pending=None) -> None:
        self.acq_func.set_X_pending(self._construct_X_full(X_pending) if X_pending is not None
                                    else None)

    def _on(self, X: torch.Tensor):
        """The values and the column selector on X's device and dtype (placed
        once per device / dtype: a call under stream capture copies nothing)."""
        key = (X.device, X.dtype)
        hit = self._placed.get(key)
        v = self.values
        # rebuilt if values was replaced or updated in place (version counter,
        # storage): .to() may have made a copy that an in-place update misses
        src = (v, v._version, v.data_ptr())
        if hit is None or hit[2][0] is not v or hit[2][1:] != src[1:]:
            vals = v.to(device=X.device, dtype=X.dtype)
            sel = torch.tensor(self._selector, dtype=torch.long, device=X.device)
            hit = (vals, sel, src)
            self._placed[key] = hit
        return hit[0], hit[1]

    def _construct_X_full(self, X: torch.Tensor) -> torch.Tensor:
        d_prime, d_f = X.shape[-1], self.values.shape[-1]
        if d_prime + d_f != self.d:
            raise ValueError(f"Feature dimension d' ({d_prime}) of input must be "
                             f"d - d_f ({self.d - d_f}).")
        vals, sel = self._on(X)
        vals = vals.expand(*X.shape[:-1], d_f)
        return torch.cat([X, vals], dim=-1).index_select(-1, sel)

    def forward(self, X: torch.Tensor) -> torch.Tensor:
        return self.acq_func(self._construct_X_full(X))
