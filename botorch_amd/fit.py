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

import math
import time
import warnings
from typing import Optional

import numpy as np
import torch
from scipy.optimize import minimize

from . import _lib, kernels
from ._lib import check, lib
from .exceptions import NotPSDError, OptimizationWarning
from .models import FixedNoiseGaussianLikelihood, LogNormalPrior, ScaleKernel, SingleTaskGP


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

    def sample_priors(self, gen: torch.Generator) -> None:
        _sample_all_priors(self.model, self, gen)


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

    def sample_priors(self, gen: torch.Generator) -> None:
        for p in self.parts:
            p.sample_priors(gen)


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
        Ainv = kernels.ainv(cache)
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


def fit_gpytorch_mll_scipy(mll: ExactMarginalLogLikelihood, method="L-BFGS-B", options=None,
                           callback=None, timeout_sec=None):
    model = mll.model
    layout = _layout(model)
    x0 = layout.get()
    if torch.isnan(model.train_inputs[0]).any() or torch.isnan(model.train_targets).any():
        from .exceptions import NanError
        raise NanError("training data contains NaN")

    def f(x):
        return layout.value_and_grad(x)

    res = minimize(f, x0, jac=True, method=method, bounds=layout.bounds, options=options or {},
                   callback=callback)
    layout.set(res.x)
    if not res.success:
        warnings.warn(f"`scipy_minimize` terminated with status {res.status}, displaying original "
                      f"message from `scipy.optimize.minimize`: {res.message}", OptimizationWarning)
    return res


def _sample_all_priors(model: SingleTaskGP, layout: _Layout, gen: torch.Generator):
    """sample_all_priors: draw free hyperparameters from their priors."""
    x = layout.get()
    base, o = layout.base, layout.o
    if not layout.fixed and model.likelihood.noise_prior is not None:
        p = model.likelihood.noise_prior
        x[0] = max(math.exp(p.loc + p.scale * torch.randn(1, generator=gen).item()),
                   model.likelihood.noise_lower)
    if base.lengthscale_prior is not None:
        p = base.lengthscale_prior
        z = torch.randn(layout.d, generator=gen, dtype=torch.float64).numpy()
        x[o + 1:o + 1 + layout.d] = np.maximum(np.exp(p.loc + p.scale * z), base.lengthscale_lower)
    layout.set(x)


def fit_gpytorch_mll(mll: ExactMarginalLogLikelihood, optimizer_kwargs=None, max_attempts=5,
                     **kwargs) -> ExactMarginalLogLikelihood:
    """botorch/fit.py:75-258 (_fit_fallback)."""
    optimizer_kwargs = optimizer_kwargs or {}
    model = mll.model
    mll.train()
    layout = _layout(model)
    gen = torch.Generator().manual_seed(0)
    ckpt = layout.get()
    for attempt in range(1, max_attempts + 1):
        if attempt > 1:
            layout.set(ckpt)
            layout.sample_priors(gen)
        try:
            with warnings.catch_warnings(record=True) as ws:
                warnings.simplefilter("always", category=OptimizationWarning)
                fit_gpytorch_mll_scipy(mll, **optimizer_kwargs)
            bad = [w for w in ws if issubclass(w.category, OptimizationWarning)
                   and "ITERATIONS REACHED LIMIT" not in str(w.message).upper()
                   and "timed out" not in str(w.message)]
            if not bad:
                return mll.eval()
        except NotPSDError:
            pass
    layout.set(ckpt)
    warnings.warn("All attempts to fit the model have failed.", OptimizationWarning)
    return mll
