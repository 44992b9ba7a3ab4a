"""GP hyperparameter fitting: fit_gpytorch_mll with an on-device exact MLL.

Reference: botorch/fit.py:75-258 (fit_gpytorch_mll -> _fit_fallback: up to 5
attempts, prior resampling between attempts, rollback, NotPSDError caught),
optim/fit.py:47-110 (fit_gpytorch_mll_scipy: L-BFGS-B with bounds from the
constraints, optim/utils/model_utils.py:69-109) and the closure
optim/closures/model_closures.py:171-184 (-[G] ExactMarginalLogLikelihood).

Each closure call: kernel matrix + blocked MFMA Cholesky with the jitter ladder
+ explicit inverse (bo_gp_cache_build), A^{-1} = L^{-T} L^{-1} (bo_ainv),
one pass of bo_mll_terms; the host reads back n x (d+5) row sums and forms
the loss and its exact gradient (plus the LogNormal prior terms).
"""
from __future__ import annotations

import logging
import math
import re
import time
import warnings
from dataclasses import dataclass
from enum import Enum, auto
from typing import Optional

import numpy as np
import torch
from scipy.optimize import minimize

from . import _lib, kernels
from ._lib import check, lib
from .exceptions import NotPSDError, OptimizationWarning, UnsupportedError
from .models import FixedNoiseGaussianLikelihood, LogNormalPrior, ScaleKernel, SingleTaskGP

logger = logging.getLogger("botorch_amd")


class ExactMarginalLogLikelihood:
    """[G] ExactMarginalLogLikelihood(likelihood, model)."""

    def __init__(self, likelihood, model: SingleTaskGP):
        self.likelihood = likelihood
        self.model = model

    def train(self):
        self.model.train()
        return self

    def eval(self):
        self.model.eval()
        return self

    @property
    def training(self):
        return self.model.training


def _prior_terms(prior: Optional[LogNormalPrior], x: np.ndarray):
    if prior is None:
        return 0.0, np.zeros_like(x)
    lx = np.log(x)
    val = np.sum(-((lx - prior.loc) ** 2) / (2 * prior.scale ** 2) - math.log(prior.scale)
                 - 0.5 * math.log(2 * math.pi) - lx)
    grad = -(lx - prior.loc) / (prior.scale ** 2 * x) - 1.0 / x
    return float(val), grad


class _Layout:
    """Flat parameter vector <-> model hyperparameters (order of
    get_parameters_and_bounds: noise, constant, lengthscales[, outputscale];
    a fixed-noise likelihood has no noise entry)."""

    def __init__(self, model: SingleTaskGP):
        self.model = model
        self.d = model.train_inputs[0].shape[-1]
        self.fixed = isinstance(model.likelihood, FixedNoiseGaussianLikelihood)
        self.o = 0 if self.fixed else 1  # offset of the constant
        self.has_os = isinstance(model.covar_module, ScaleKernel)
        base = model.covar_module.base_kernel if self.has_os else model.covar_module
        self.base = base
        lo = ([] if self.fixed else [model.likelihood.noise_lower]) + [-np.inf]
        lo += [base.lengthscale_lower] * self.d
        if self.has_os:
            lo.append(0.0)
        self.bounds = [(None if not np.isfinite(l) else l, None) for l in lo]
        # (name, start, size) segments, the order above
        self.segments = ([] if self.fixed else [("noise", 0, 1)]) + [
            ("constant", self.o, 1), ("lengthscale", self.o + 1, self.d)] + (
            [("outputscale", self.o + 1 + self.d, 1)] if self.has_os else [])
        self.size = self.o + 1 + self.d + (1 if self.has_os else 0)

    def get(self) -> np.ndarray:
        m = self.model
        v = [] if self.fixed else [float(m.likelihood.noise.detach())]
        v.append(float(m.mean_module.constant.detach()))
        v += self.base.lengthscale.detach().reshape(-1).cpu().tolist()
        if self.has_os:
            v.append(float(m.covar_module.outputscale.detach()))
        return np.asarray(v, dtype=np.float64)

    def set(self, x: np.ndarray) -> None:
        m, o = self.model, self.o
        if not self.fixed:
            m.likelihood.noise = torch.tensor([float(x[0])], dtype=torch.float64)
        m.mean_module.constant = float(x[o])
        self.base.lengthscale = torch.as_tensor(x[o + 1:o + 1 + self.d]).reshape(1, -1)
        if self.has_os:
            m.covar_module.outputscale = float(x[o + 1 + self.d])

    def value_and_grad(self, x: np.ndarray):
        # the closure reads x, not the module: the parameters are written once,
        # at the optimum (fit_gpytorch_mll_scipy), not per evaluation (four
        # constrained-parameter writes = a dozen small host-to-device copies)
        return mll_value_and_grad(self.model, x, self, sync_model=False)


class _MultiLayout:
    """The m members of a multi-output SingleTaskGP as one flat vector in the
    batched model's parameter order (each parameter's m entries together:
    noise_1..m, constant_1..m, lengthscale m x d, outputscale_1..m).  The loss
    is the sum of the members' losses (the closure's Tensor.sum reducer over
    the batched MLL, optim/closures/model_closures.py:171-184), so one
    L-BFGS-B runs over all of them jointly, as the reference's does."""

    def __init__(self, model: SingleTaskGP):
        self.model = model
        self.parts = [_Layout(mm) for mm in model.models]
        p0, L = self.parts[0], self.parts[0].size
        self.perm = np.asarray([t * L + start + j for _, start, size in p0.segments
                                for t in range(len(self.parts)) for j in range(size)])
        self.bounds = [b for p in self.parts for b in p.bounds]
        self.bounds = [self.bounds[i] for i in self.perm]
        self.size = L * len(self.parts)

    def _split(self, x: np.ndarray):
        cat = np.empty(self.size)
        cat[self.perm] = x
        L = self.parts[0].size
        return [cat[t * L:(t + 1) * L] for t in range(len(self.parts))]

    def get(self) -> np.ndarray:
        return np.concatenate([p.get() for p in self.parts])[self.perm]

    def set(self, x: np.ndarray) -> None:
        for p, v in zip(self.parts, self._split(x)):
            p.set(v)

    def value_and_grad(self, x: np.ndarray):
        """All members' K + s2 I factorised in ONE batched DAG launch
        (kernels.build_gp_caches; bit-identical to per-member builds), then
        each member's A^{-1}, data term and priors."""
        xs = self._split(x)
        caches = [None] * len(self.parts)
        if not any(p.fixed for p in self.parts):
            specs = []
            for p, v in zip(self.parts, xs):
                mm = p.model
                noise, const, ls, os_ = _hyper_of(mm, v, p)
                specs.append(dict(Xt=mm.train_inputs[0], y=mm.train_targets,
                                  lengthscale=torch.as_tensor(ls, dtype=torch.float64,
                                                              device=mm.train_inputs[0].device),
                                  noise=float(noise), constant=float(const), kind=int(mm.kind),
                                  outputscale=float(os_)))
            caches = kernels.build_gp_caches(specs, check_nan=False)
        loss, grads = 0.0, []
        for p, v, cache in zip(self.parts, xs, caches):
            lt, gt = mll_value_and_grad(p.model, v, p, cache=cache, sync_model=False)
            loss += lt
            grads.append(gt)
        return loss, np.concatenate(grads)[self.perm]


def _layout(model):
    return _MultiLayout(model) if getattr(model, "_is_multi_output", False) else _Layout(model)


def mll_terms(Xt: torch.Tensor, y: torch.Tensor, ls_t: torch.Tensor, noise, const: float,
              os_: float, kind: int, cache=None):
    """Data term of [G] ExactMarginalLogLikelihood, ll = log N(y | c, K + s2 I)
    (no priors, not divided by n), and d ll / d [noise, constant,
    lengthscale_1..d, outputscale] (bo::mll's implementation).  ``noise`` may
    be an n-vector (fixed-noise likelihood: K + diag(noise); its gradient
    entry is then meaningless).  ``cache``: the caches of exactly these
    hyperparameters, already built (the batched multi-output closure)."""
    n, d = Xt.shape
    dev = Xt.device
    ls = ls_t.detach().cpu().numpy().astype(np.float64) if torch.is_tensor(ls_t) else np.asarray(ls_t)
    ls_t = torch.as_tensor(ls, dtype=torch.float64, device=dev)
    fixed = torch.is_tensor(noise) and noise.numel() > 1
    info = None
    if cache is None and not fixed:
        # optimistic: the jitter-free factorisation and everything after it are
        # enqueued at once; its status comes back with the MLL sums (one
        # device-to-host transfer per closure instead of two)
        cache, info = kernels.build_gp_cache_optimistic(Xt, y, ls_t, float(noise), const,
                                                        kind=kind, outputscale=os_)
    elif cache is None:
        cache = kernels.build_gp_cache(Xt, y, ls_t, noise, const, kind=kind, outputscale=os_,
                                       check_nan=False)  # checked once in fit_gpytorch_mll_scipy

    def _sums(cache, info):
        # A^{-1} = L^{-T} L^{-1}, lower tiles (n^3/3 flops on the posterior
        # kernel's MFMA tiles, stream-K over the unequal k-ranges)
        Ainv = cache.Ainv if cache.Ainv is not None else kernels.ainv(cache)
        st = kernels._stream(dev)
        part = torch.empty(n, d + 5, dtype=torch.float64, device=dev)
        check(lib().bo_mll_terms(kind, kernels._p(Xt.contiguous()), n, d, kernels._p(ls_t), os_,
                                 kernels._p(cache.L), kernels._p(Ainv), cache.np,
                                 kernels._p(cache.alpha), kernels._p(cache.beta), kernels._p(part),
                                 st), "mll_terms")
        sums = part.sum(dim=0)
        if info is not None:
            sums = torch.cat([sums, info.to(torch.float64)])
        return sums.cpu().numpy()

    s = _sums(cache, info)
    if info is not None:
        status = int(s[-1])
        s = s[:-1]
        if status < 0:
            raise RuntimeError("bo_cholesky_inverse: the Cholesky task DAG timed out")
        if status != 0:  # not p.d. without jitter: the ladder, then the sums again
            cache = kernels.build_gp_cache(Xt, y, ls_t, noise, const, kind=kind, outputscale=os_,
                                           check_nan=False)
            s = _sums(cache, None)
    quad, logdet_half, sum_alpha = s[d + 3], s[d + 2], s[d + 4]
    ll = -0.5 * quad - logdet_half - 0.5 * n * math.log(2 * math.pi)
    g = np.zeros(d + 3)
    g[0] = 0.5 * s[d]                       # d ll / d noise
    g[1] = sum_alpha                        # d ll / d constant
    g[2:2 + d] = 0.5 * s[:d] / ls ** 3      # d ll / d lengthscale
    g[2 + d] = 0.5 * s[d + 1]               # d ll / d outputscale
    return float(ll), g


def _hyper_of(model: SingleTaskGP, x: np.ndarray, layout: _Layout):
    d = model.train_inputs[0].shape[1]
    o = layout.o
    noise = 0.0 if layout.fixed else x[0]
    return noise, x[o], x[o + 1:o + 1 + d], (x[o + 1 + d] if layout.has_os else 1.0)


def mll_value_and_grad(model: SingleTaskGP, x: np.ndarray, layout: _Layout, cache=None,
                       sync_model: bool = True):
    """Loss = -(log N(y | c, K + s2 I) + log priors) / n and its gradient: the
    data term through bo::mll (torch.ops), the LogNormal priors on the host.
    Fixed noise: K + diag(observed variances), no noise entry or prior.
    ``cache``: prebuilt caches at x (the batched multi-output closure); the
    data term then comes from fit.mll_terms on them directly.  ``sync_model``
    (default True): also write x into the model's parameters, as the
    reference's closure leaves them."""
    from . import ops  # noqa: F401  (registers torch.ops.bo)
    if sync_model:
        layout.set(x)
    Xt = model.train_inputs[0]
    y = model.train_targets
    n, d = Xt.shape
    o = layout.o
    noise = 0.0 if layout.fixed else x[0]
    nv = model.likelihood.noise if layout.fixed else None
    const = x[o]
    ls = x[o + 1:o + 1 + d]
    os_ = x[o + 1 + d] if layout.has_os else 1.0
    if cache is not None or not sync_model:
        # the fit's own closure: bo::mll's implementation with the host
        # lengthscales (no device-to-host read of them)
        ll, gall = mll_terms(Xt, y, np.asarray(ls, dtype=np.float64),
                             nv if nv is not None else float(noise), float(const), float(os_),
                             int(model.kind), cache=cache)
    else:
        ls_t = torch.as_tensor(ls, dtype=torch.float64, device=Xt.device)
        llt, gt = torch.ops.bo.mll(Xt, y, ls_t, float(noise), float(const), float(os_),
                                   int(model.kind), nv)
        ll = float(llt.item())
        gall = gt.cpu().numpy()
    g = np.zeros_like(x)
    if not layout.fixed:
        g[0] = gall[0]
        pv, pg = _prior_terms(model.likelihood.noise_prior, np.array([noise]))
        ll += pv
        g[0] += pg[0]
    g[o:o + 1 + d] = gall[1:2 + d]
    if layout.has_os:
        g[o + 1 + d] = gall[2 + d]
    pv, pg = _prior_terms(layout.base.lengthscale_prior, ls)
    ll += pv
    g[o + 1:o + 1 + d] += pg
    return -ll / n, -g / n


class OptimizationStatus(int, Enum):
    """optim/core.py:39-43."""
    RUNNING = auto()
    SUCCESS = auto()
    FAILURE = auto()
    STOPPED = auto()


@dataclass
class OptimizationResult:
    """optim/core.py:46-52."""
    step: int
    fval: float
    status: OptimizationStatus
    runtime: Optional[float] = None
    message: Optional[str] = None


# optim/core.py:34-36 matches the iteration / evaluation limit messages of
# scipy <= 1.14's Fortran L-BFGS-B ("TOTAL NO. of ITERATIONS REACHED LIMIT",
# "TOTAL NO. of f AND g EVALUATIONS EXCEEDS LIMIT").  scipy 1.15 (installed
# here) spells them "TOTAL NO. OF ITERATIONS REACHED LIMIT" and "TOTAL NO. OF
# F,G EVALUATIONS EXCEEDS LIMIT", which the reference's case-sensitive pattern
# misses (a maxiter stop would then count as a failed fit).  Both spellings are
# matched here: the reference's intent with the scipy the box has.
LBFGSB_MAXITER_MAXFUN_REGEX = re.compile(
    r"TOTAL NO\. OF (ITERATIONS REACHED LIMIT|F AND G EVALUATIONS EXCEEDS LIMIT|"
    r"F,G EVALUATIONS EXCEEDS LIMIT)", re.IGNORECASE)


def _param_bounds_by_name(layout):
    """get_parameters_and_bounds names (optim/utils/model_utils.py:69-109) of
    the single-output layout's segments."""
    return {"likelihood.noise_covar.raw_noise": "noise", "mean_module.raw_constant": "constant",
            "covar_module.raw_lengthscale": "lengthscale",
            "covar_module.base_kernel.raw_lengthscale": "lengthscale",
            "covar_module.raw_outputscale": "outputscale"}


def _apply_user_bounds(layout, bounds) -> list:
    """fit_gpytorch_mll_scipy's ``bounds`` dict (updating the defaults,
    optim/fit.py:83-84) onto the flat vector's scipy bounds."""
    out = list(layout.bounds)
    if not bounds:
        return out
    if isinstance(layout, _MultiLayout):
        raise UnsupportedError("user bounds for a multi-output SingleTaskGP fit")
    names = _param_bounds_by_name(layout)
    segs = {name: (start, size) for name, start, size in layout.segments}
    for pname, (lo, hi) in bounds.items():
        seg = names.get(pname)
        if seg is None or seg not in segs:
            raise UnsupportedError(f"bounds for unknown parameter {pname!r}")
        start, size = segs[seg]
        for j in range(start, start + size):
            out[j] = (lo, hi)
    return out


def fit_gpytorch_mll_scipy(mll: ExactMarginalLogLikelihood, parameters=None, bounds=None,
                           closure=None, closure_kwargs=None, method="L-BFGS-B", options=None,
                           callback=None, timeout_sec=None) -> OptimizationResult:
    """optim/fit.py:47-110 + optim/core.py:55-140: L-BFGS-B over the flat
    hyperparameter vector, the closure being the device MLL (value and exact
    gradient from bo::mll), bounded by ``timeout_sec``; the parameters are
    written at the optimum; an OptimizationWarning when the run did not end in
    SUCCESS.  ``callback(parameters, OptimizationResult)`` is called after
    each iteration as the reference's wrapped callback does.  ``parameters`` /
    ``closure``: the device closure is the only one on this path (a custom
    torch closure raises UnsupportedError)."""
    if parameters is not None or closure is not None or closure_kwargs:
        raise UnsupportedError("custom parameters / closures: the MLL closure here is the "
                               "device one (bo::mll)")
    from .optim import minimize_with_timeout
    t0 = time.monotonic()
    model = mll.model
    layout = _layout(model)
    x0 = layout.get()
    if torch.isnan(model.train_inputs[0]).any() or torch.isnan(model.train_targets).any():
        from .exceptions import NanError
        raise NanError("training data contains NaN")
    wrapped = None
    if callback is not None:
        step = [0]

        def wrapped(x):
            step[0] += 1
            # the iterate goes into the model first (the reference's closure
            # writes its state into the parameters before the callback runs)
            layout.set(x)
            res = OptimizationResult(step=step[0], fval=float(layout.value_and_grad(x)[0]),
                                     status=OptimizationStatus.RUNNING,
                                     runtime=time.monotonic() - t0)
            return callback(dict(model.named_parameters()), res)

    raw = minimize_with_timeout(layout.value_and_grad, x0, jac=True, method=method,
                                bounds=_apply_user_bounds(layout, bounds), options=options or {},
                                callback=wrapped, timeout_sec=timeout_sec)
    layout.set(raw.x)
    msg = raw.message if isinstance(raw.message, str) else raw.message.decode("ascii")
    if raw.success:
        status = OptimizationStatus.SUCCESS
    elif LBFGSB_MAXITER_MAXFUN_REGEX.search(msg) or "Optimization timed out after" in msg:
        status = OptimizationStatus.STOPPED
    else:
        status = OptimizationStatus.FAILURE
    result = OptimizationResult(step=int(getattr(raw, "nit", 0)), fval=float(raw.fun),
                                status=status, runtime=time.monotonic() - t0, message=msg)
    if status != OptimizationStatus.SUCCESS:
        warnings.warn(f"`scipy_minimize` terminated with status {status}, displaying original "
                      f"message from `scipy.optimize.minimize`: {msg}", OptimizationWarning)
    return result


def _sample_prior_values(prior: LogNormalPrior, shape, device) -> torch.Tensor:
    """[G] LogNormalPrior.sample(shape) in fp64 on the model's device:
    exp(torch.normal(loc, scale)) from the global generator of that device."""
    loc = torch.full(shape, prior.loc, dtype=torch.float64, device=device)
    scale = torch.full(shape, prior.scale, dtype=torch.float64, device=device)
    with torch.no_grad():
        return torch.normal(loc, scale).exp()


def sample_all_priors(model) -> None:
    """optim/utils/model_utils.py:153-193 sample_all_priors: each free
    hyperparameter with a prior gets a draw of its own shape, in the order of
    [G] named_priors (the module's own priors, then its children's in
    registration order: likelihood noise, then the covariance module -- a
    ScaleKernel's outputscale before its base kernel's lengthscale).  The
    draws come from the global generator of the parameters' device, as the
    reference's do; the constraints have ``transform=None``, so a draw is set
    as is (L-BFGS-B clips it into the bounds)."""
    if getattr(model, "_is_multi_output", False):
        members = list(model.models)
        dev = model.train_inputs[0].device
        m, d = len(members), model.train_inputs[0].shape[-1]
        # the batched model (batch shape [m]) draws each prior once, m-wide
        p = members[0].likelihood.noise_prior
        if p is not None and not isinstance(members[0].likelihood, FixedNoiseGaussianLikelihood):
            v = _sample_prior_values(p, (m, 1), dev)
            for t, mm in enumerate(members):
                mm.likelihood.noise = v[t]
        ck = members[0].covar_module
        if isinstance(ck, ScaleKernel) and ck.outputscale_prior is not None:
            v = _sample_prior_values(ck.outputscale_prior, (m,), dev)
            for t, mm in enumerate(members):
                mm.covar_module.outputscale = float(v[t])
        base = ck.base_kernel if isinstance(ck, ScaleKernel) else ck
        if base.lengthscale_prior is not None:
            v = _sample_prior_values(base.lengthscale_prior, (m, 1, d), dev)
            for t, mm in enumerate(members):
                b = mm.covar_module.base_kernel if isinstance(mm.covar_module, ScaleKernel) \
                    else mm.covar_module
                b.lengthscale = v[t]
        return
    dev = model.train_inputs[0].device
    lik = model.likelihood
    if not isinstance(lik, FixedNoiseGaussianLikelihood) and lik.noise_prior is not None:
        lik.noise = _sample_prior_values(lik.noise_prior, (1,), dev)
    ck = model.covar_module
    if isinstance(ck, ScaleKernel) and ck.outputscale_prior is not None:
        ck.outputscale = float(_sample_prior_values(ck.outputscale_prior, (), dev))
    base = ck.base_kernel if isinstance(ck, ScaleKernel) else ck
    if base.lengthscale_prior is not None:
        base.lengthscale = _sample_prior_values(base.lengthscale_prior,
                                                tuple(base.lengthscale.shape), dev)


def _debug_warn(w) -> bool:
    return bool(LBFGSB_MAXITER_MAXFUN_REGEX.search(str(w.message)))


def _rethrow_warn(w) -> bool:
    if not issubclass(w.category, OptimizationWarning):
        return True
    return "Optimization timed out after" in str(w.message)


def DEFAULT_WARNING_HANDLER(w) -> bool:
    """fit.py:51-71 (_warning_handler_template with _debug_warn / _rethrow_warn):
    True when the warning is resolved -- iteration / evaluation limits are
    logged, non-optimisation warnings and timeouts are re-emitted -- False when
    it should trigger a retry."""
    if _debug_warn(w):
        logger.debug(str(w.message))
        return True
    if _rethrow_warn(w):
        warnings.warn_explicit(str(w.message), w.category, w.filename, w.lineno)
        return True
    return False


class SumMarginalLogLikelihood:
    """[G] SumMarginalLogLikelihood(likelihood, ModelListGP): one exact MLL per
    member."""

    def __init__(self, likelihood, model):
        self.likelihood = likelihood
        self.model = model
        self.mlls = [ExactMarginalLogLikelihood(mm.likelihood, mm) for mm in model.models]

    def train(self):
        self.model.train()
        return self

    def eval(self):
        self.model.eval()
        return self

    @property
    def training(self):
        return any(m.training for m in self.mlls)


def fit_gpytorch_mll(mll, closure=None, optimizer=None, closure_kwargs=None,
                     optimizer_kwargs=None, **kwargs):
    """botorch/fit.py:75-113: dispatch on the MLL type -- a
    SumMarginalLogLikelihood over a ModelListGP fits each member (_fit_list,
    fit.py:262-283), anything else goes to _fit_fallback."""
    if optimizer is not None:
        kwargs["optimizer"] = optimizer
    if isinstance(mll, SumMarginalLogLikelihood):
        mll.train()
        for sub in mll.mlls:
            fit_gpytorch_mll(sub, closure=closure, closure_kwargs=closure_kwargs,
                             optimizer_kwargs=optimizer_kwargs, **kwargs)
        return mll.eval() if not mll.training else mll
    return _fit_fallback(mll, closure=closure, closure_kwargs=closure_kwargs,
                         optimizer_kwargs=optimizer_kwargs, **kwargs)


def _fit_fallback(mll, *, closure=None, optimizer=fit_gpytorch_mll_scipy, closure_kwargs=None,
                  optimizer_kwargs=None, max_attempts: int = 5,
                  pick_best_of_all_attempts: bool = False,
                  warning_handler=DEFAULT_WARNING_HANDLER,
                  caught_exception_types=(NotPSDError,), **ignore):
    """botorch/fit.py:116-259.  Each attempt starts from the state the fit was
    called with (the rollback of module_rollback_ctx); attempts after the first
    resample the priors from the global generator first.  Warnings the
    ``warning_handler`` does not resolve are re-emitted and make the attempt a
    failure; exceptions of ``caught_exception_types`` are logged and count as
    failed attempts.  The first successful attempt is kept, or with
    ``pick_best_of_all_attempts`` the successful attempt of largest MLL.  When
    no attempt succeeded: ModelFittingError, with the model back at its
    starting state and in train mode."""
    from .exceptions import ModelFittingError
    from .settings import debug
    if closure is not None or closure_kwargs:
        raise UnsupportedError("custom closures: the MLL closure here is the device one "
                               "(bo::mll)")
    optimizer_kwargs = {} if optimizer_kwargs is None else optimizer_kwargs
    model = mll.model
    mll.train()
    layout = _layout(model)
    ckpt = layout.get()   # module_rollback_ctx's checkpoint
    best_mll, best_x = -math.inf, None
    for attempt in range(1, max_attempts + 1):
        layout.set(ckpt)
        if attempt > 1:
            sample_all_priors(model)
        try:
            with warnings.catch_warnings(record=True) as wlist, debug(True):
                warnings.simplefilter("always", category=OptimizationWarning)
                result = optimizer(mll, closure=None, **optimizer_kwargs)
            success = True
            for w in wlist:
                if not warning_handler(w):
                    warnings.warn_explicit(str(w.message), w.category, w.filename, w.lineno)
                    success = False
            if success and not pick_best_of_all_attempts:
                return mll.eval()
            if success:
                cur = -float(result.fval)
                if cur > best_mll:
                    best_mll, best_x = cur, layout.get()
                    logger.debug(f"Fit attempt #{attempt}: New best MLL: {best_mll}.")
                else:
                    logger.debug(f"Fit attempt #{attempt}: Current MLL {cur} did not beat best "
                                 f"MLL so far {best_mll}.")
            mll.train()
            if not success:
                logger.debug(f"Fit attempt #{attempt} of {max_attempts} triggered retry policy"
                             f"{'.' if attempt == max_attempts else '; retrying...'}")
        except caught_exception_types as err:
            logger.debug(f"Fit attempt #{attempt} of {max_attempts} failed with exception:\n{err}")
    if best_x is not None:
        layout.set(best_x)
        return mll.eval()
    layout.set(ckpt)
    mll.train()
    msg = "All attempts to fit the model have failed."
    if debug.off():
        msg += " For more information, try enabling botorch.settings.debug mode."
    raise ModelFittingError(msg)
