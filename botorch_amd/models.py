"""Exact GP models with BoTorch's posterior API, backed by the gfx950 kernels.

Mirrors botorch/models/gp_regression.py:68-254 (SingleTaskGP), the default
modules of botorch/models/utils/gpytorch_modules.py:74-127, the Standardize
outcome transform (botorch/models/transforms/outcome.py:217-447) and
ModelListGP (botorch/models/model_list_gp_regression.py:24).  Hyperparameters
are plain fp64 ``nn.Parameter``s holding the constrained values directly (the
reference's constraints use ``transform=None``: raw value == value); their
lower bounds are enforced by L-BFGS-B in ``fit.py`` exactly as
botorch/optim/utils/model_utils.py:69-109 does.

Eval-mode prediction caches (Cholesky factor, L^{-T}, alpha, beta) live on the
device and are rebuilt when any hyperparameter or training tensor changes
version, or on ``train()`` (mirrors [G] ExactGP dropping prediction_strategy).
"""
from __future__ import annotations

import math
import warnings
from typing import List, Optional, Sequence, Union

import torch
from torch import nn

from . import _lib
from .exceptions import InputDataWarning, UnsupportedError

MIN_INFERRED_NOISE_LEVEL = 1e-4  # gpytorch_modules.py:29
LENGTHSCALE_LOWER = 2.5e-2       # gpytorch_modules.py:123
SQRT2, SQRT3 = math.sqrt(2), math.sqrt(3)


# Generation of the model trees' structure: bumped whenever a parameter or a
# submodule is (re)assigned inside one (an in-place change of a parameter's
# values bumps its tensor _version instead).  SingleTaskGP._key() reuses its
# list of parameters until this changes -- walking the module tree on every
# acquisition call was its largest host cost.
_STRUCTURE = [0]


class _TrackedModule(nn.Module):
    """nn.Module whose parameter / submodule (re)assignments bump _STRUCTURE."""

    def __setattr__(self, name, value):
        super().__setattr__(name, value)
        if isinstance(value, (nn.Parameter, nn.Module)):
            _STRUCTURE[0] += 1

    def __delattr__(self, name):
        super().__delattr__(name)
        _STRUCTURE[0] += 1

    def register_parameter(self, name, param):
        super().register_parameter(name, param)
        _STRUCTURE[0] += 1

    def add_module(self, name, module):
        super().add_module(name, module)
        _STRUCTURE[0] += 1


class LogNormalPrior:
    """[G] LogNormalPrior(loc, scale) (torch LogNormal)."""

    def __init__(self, loc: float, scale: float):
        self.loc, self.scale = float(loc), float(scale)

    @property
    def mode(self) -> float:
        return math.exp(self.loc - self.scale ** 2)

    def log_prob(self, x: torch.Tensor) -> torch.Tensor:
        lx = torch.log(x)
        return (-((lx - self.loc) ** 2) / (2 * self.scale ** 2) - math.log(self.scale)
                - 0.5 * math.log(2 * math.pi) - lx)


class _Kernel(_TrackedModule):
    kind = _lib.RBF

    def __init__(self, ard_num_dims: int, lengthscale_prior: Optional[LogNormalPrior] = None,
                 lengthscale_lower: float = LENGTHSCALE_LOWER, initial: Optional[float] = None):
        super().__init__()
        self.ard_num_dims = ard_num_dims
        self.lengthscale_prior = lengthscale_prior
        self.lengthscale_lower = lengthscale_lower
        init = initial if initial is not None else (
            lengthscale_prior.mode if lengthscale_prior is not None else 1.0)
        self.raw_lengthscale = nn.Parameter(torch.full((1, ard_num_dims), init, dtype=torch.float64))

    @property
    def lengthscale(self) -> torch.Tensor:
        return self.raw_lengthscale

    @lengthscale.setter
    def lengthscale(self, value):
        with torch.no_grad():
            self.raw_lengthscale.copy_(torch.as_tensor(value, dtype=torch.float64).expand_as(self.raw_lengthscale))

    outputscale = 1.0


class RBFKernel(_Kernel):
    """exp(-||(x - x')/ell||^2 / 2)  ([G] RBFKernel)."""
    kind = _lib.RBF


class MaternKernel(_Kernel):
    """Matern-5/2 ([G] MaternKernel(nu=2.5))."""
    kind = _lib.MATERN52

    def __init__(self, nu: float = 2.5, **kw):
        if nu != 2.5:
            raise UnsupportedError("only nu = 2.5 is on the accelerated path")
        super().__init__(**kw)


class ScaleKernel(_TrackedModule):
    """outputscale * base_kernel ([G] ScaleKernel)."""

    def __init__(self, base_kernel: _Kernel, outputscale: float = 1.0, outputscale_prior=None):
        super().__init__()
        self.base_kernel = base_kernel
        self.outputscale_prior = outputscale_prior
        self.raw_outputscale = nn.Parameter(torch.tensor(float(outputscale), dtype=torch.float64))

    kind = property(lambda self: self.base_kernel.kind)
    ard_num_dims = property(lambda self: self.base_kernel.ard_num_dims)

    @property
    def lengthscale(self):
        return self.base_kernel.lengthscale

    @property
    def outputscale(self):
        return self.raw_outputscale

    @outputscale.setter
    def outputscale(self, v):
        with torch.no_grad():
            self.raw_outputscale.fill_(float(v))


class GaussianLikelihood(_TrackedModule):
    """Homoskedastic Gaussian noise ([G] GaussianLikelihood) with BoTorch's
    LogNormal(-4, 1) prior and noise >= 1e-4 (gpytorch_modules.py:74-97)."""

    def __init__(self, noise_prior: Optional[LogNormalPrior] = None,
                 noise_lower: float = MIN_INFERRED_NOISE_LEVEL, initial: Optional[float] = None):
        super().__init__()
        self.noise_prior = noise_prior
        self.noise_lower = noise_lower
        init = initial if initial is not None else (noise_prior.mode if noise_prior else 1e-4)
        self.raw_noise = nn.Parameter(torch.tensor([init], dtype=torch.float64))

    @property
    def noise(self):
        return self.raw_noise

    @noise.setter
    def noise(self, v):
        with torch.no_grad():
            self.raw_noise.copy_(torch.as_tensor(v, dtype=torch.float64).reshape(1))


class FixedNoiseGaussianLikelihood(_TrackedModule):
    """Observed per-point noise variances ([G] FixedNoiseGaussianLikelihood with
    learn_additional_noise=False), the likelihood SingleTaskGP builds from
    train_Yvar (botorch/models/gp_regression.py:187-194).  Nothing is learned:
    ``noise`` is a buffer, there is no prior, and the MLL's K + s2 I becomes
    K + diag(noise)."""

    noise_prior = None
    noise_lower = 0.0

    def __init__(self, noise: torch.Tensor):
        super().__init__()
        self.register_buffer("noise", torch.as_tensor(noise, dtype=torch.float64).reshape(-1).clone())


class ConstantMean(_TrackedModule):
    def __init__(self):
        super().__init__()
        self.raw_constant = nn.Parameter(torch.tensor(0.0, dtype=torch.float64))

    @property
    def constant(self):
        return self.raw_constant

    @constant.setter
    def constant(self, v):
        with torch.no_grad():
            self.raw_constant.fill_(float(v))


def get_covar_module_with_dim_scaled_prior(ard_num_dims: int, use_rbf_kernel: bool = True):
    """gpytorch_modules.py:100-127: LogNormal(sqrt2 + ln(d)/2, sqrt3) lengthscale
    prior, initialised at its mode, lengthscale >= 0.025."""
    prior = LogNormalPrior(SQRT2 + 0.5 * math.log(ard_num_dims), SQRT3)
    cls = RBFKernel if use_rbf_kernel else MaternKernel
    return cls(ard_num_dims=ard_num_dims, lengthscale_prior=prior)


def get_gaussian_likelihood_with_lognormal_prior():
    """gpytorch_modules.py:74-97."""
    return GaussianLikelihood(noise_prior=LogNormalPrior(-4.0, 1.0))


class Standardize(_TrackedModule):
    """Outcome standardisation (botorch/models/transforms/outcome.py:217-447)."""

    def __init__(self, m: int, min_stdv: float = 1e-8):
        super().__init__()
        self._m = m
        self._min_stdv = min_stdv
        self.register_buffer("means", torch.zeros(1, m, dtype=torch.float64))
        self.register_buffer("stdvs", torch.ones(1, m, dtype=torch.float64))
        self._is_trained = False

    def forward(self, Y: torch.Tensor, Yvar: Optional[torch.Tensor] = None):
        if self.training:
            if Y.shape[-2] < 1:
                raise ValueError("Can't standardize with no observations.")
            if Y.shape[-2] == 1:
                stdvs = torch.ones(1, Y.shape[-1], dtype=Y.dtype, device=Y.device)
            else:
                stdvs = Y.std(dim=-2, keepdim=True)
            stdvs = stdvs.where(stdvs >= self._min_stdv, torch.full_like(stdvs, 1.0))
            self.means = Y.mean(dim=-2, keepdim=True)
            self.stdvs = stdvs
            self._is_trained = True
            self._generation = getattr(self, "_generation", 0) + 1
        Y_tf = (Y - self.means) / self.stdvs
        Yvar_tf = Yvar / self.stdvs.pow(2) if Yvar is not None else None
        return Y_tf, Yvar_tf

    def untransform(self, Y, Yvar=None):
        return self.means + self.stdvs * Y, (self.stdvs.pow(2) * Yvar if Yvar is not None else None)


class _StackedView:
    """Read-only view of one module of a multi-output SingleTaskGP's members,
    stacking an attribute over the outputs in the reference's batched shapes
    (likelihood.noise m x 1, covar_module.lengthscale m x 1 x d,
    mean_module.constant m)."""

    def __init__(self, members, name: str):
        object.__setattr__(self, "_mods", [getattr(mm, name) for mm in members])

    def __getattr__(self, attr):
        vals = [getattr(mod, attr) for mod in self._mods]
        if all(torch.is_tensor(v) for v in vals):
            return torch.stack([v.detach() for v in vals])
        if all(isinstance(v, (int, float)) for v in vals):
            return torch.tensor(vals, dtype=torch.float64)
        return vals

    def __setattr__(self, attr, value):
        raise AttributeError("set the hyperparameters of a multi-output SingleTaskGP through "
                             "model.models[t]")


class Model(_TrackedModule):
    """Abstract model with BoTorch's ``posterior`` contract (models/model.py:82-117)."""

    _num_outputs = 1

    @property
    def num_outputs(self) -> int:
        return self._num_outputs

    def posterior(self, X, output_indices=None, observation_noise=False, posterior_transform=None):
        raise NotImplementedError

    def outcome_stats(self):
        """(mean, std) of the Standardize transform as host floats, read back once
        per change of the buffers (not per acquisition call: each read is a
        device-to-host sync)."""
        ot = self._modules.get("outcome_transform")
        if ot is None:
            return 0.0, 1.0
        bufs = ot._buffers  # (direct: nn.Module attribute lookups cost per call)
        m, s = bufs["means"], bufs["stdvs"]
        key = (ot.__dict__.get("_generation", 0), m.data_ptr(), m._version, s.data_ptr(),
               s._version)
        if getattr(self, "_ostats_key", None) != key:
            self._ostats = (float(m.reshape(-1)[0]), float(s.reshape(-1)[0]))
            self._ostats_key = key
        return self._ostats


class SingleTaskGP(Model):
    """Single-output exact GP (botorch/models/gp_regression.py:130-254).

    Defaults: RBF-ARD kernel without outputscale, LogNormal priors,
    ConstantMean, GaussianLikelihood, Standardize(m=1) outcome transform.
    """

    def __init__(self, train_X: torch.Tensor, train_Y: torch.Tensor,
                 train_Yvar: Optional[torch.Tensor] = None, likelihood=None, covar_module=None,
                 mean_module=None, outcome_transform="DEFAULT", input_transform=None):
        super().__init__()
        if input_transform is not None:
            raise UnsupportedError("input transforms are not on the accelerated path")
        if train_X.dim() != 2 or train_Y.dim() != 2 or train_X.shape[0] != train_Y.shape[0]:
            raise UnsupportedError("SingleTaskGP here takes train_X n x d and train_Y n x m")
        if train_Yvar is not None and train_Yvar.shape != train_Y.shape:
            raise ValueError(f"train_Yvar of shape {tuple(train_Yvar.shape)} does not match "
                             f"train_Y of shape {tuple(train_Y.shape)}")
        train_X = train_X.to(torch.float64)
        train_Y = train_Y.to(torch.float64)
        from .exceptions import InputDataError
        if torch.isnan(train_X).any() or torch.isnan(train_Y).any():
            raise InputDataError("Input data contains NaN values.")
        if train_Yvar is not None:
            train_Yvar = train_Yvar.to(torch.float64)
            if torch.isnan(train_Yvar).any():
                raise InputDataError("Input data contains NaN values.")
            if (train_Yvar < 0).any():  # models/utils/assorted.py validate_input_scaling
                raise InputDataError("Input data contains negative variances.")
        if train_Y.shape[-1] > 1:
            self._init_multi_output(train_X, train_Y, train_Yvar, likelihood, covar_module,
                                    mean_module, outcome_transform)
            return
        if outcome_transform == "DEFAULT":
            outcome_transform = Standardize(m=1)
        if outcome_transform is not None:
            outcome_transform.train()
            train_Y_tf, train_Yvar_tf = outcome_transform(train_Y, train_Yvar)
            self.outcome_transform = outcome_transform
        else:
            train_Y_tf, train_Yvar_tf = train_Y, train_Yvar
        self._check_scaling(train_X, train_Y_tf)
        self.train_inputs = (train_X,)
        self.train_targets = train_Y_tf.squeeze(-1)
        self._raw_train_Y = train_Y
        d = train_X.shape[-1]
        if likelihood is None and train_Yvar_tf is not None:
            likelihood = FixedNoiseGaussianLikelihood(train_Yvar_tf.squeeze(-1))
        self.likelihood = likelihood if likelihood is not None else get_gaussian_likelihood_with_lognormal_prior()
        self.mean_module = mean_module if mean_module is not None else ConstantMean()
        self.covar_module = covar_module if covar_module is not None else get_covar_module_with_dim_scaled_prior(d)
        self._cache = None
        self._cache_key = None
        self.to(train_X.device)

    def _init_multi_output(self, train_X, train_Y, train_Yvar, likelihood, covar_module,
                           mean_module, outcome_transform):
        """m > 1 outputs: the reference's batched multi-output model
        (models/gpytorch.py:327-355 BatchedMultiOutputGPyTorchModel, batch shape
        [m] of independent GPs with their own hyperparameters) as m single-output
        members sharing train_X.  Standardize(m) standardises each column on its
        own, so each member's Standardize(1) holds exactly its column's
        statistics; the posterior is the members' block-diagonal joint (the
        from_batch_mvn MTMVN), which the ModelListGP routes (qEHVI / qNEHVI /
        scalarised qEI) consume through ``models``; fit_gpytorch_mll minimises
        the summed loss jointly over all members' parameters."""
        m = train_Y.shape[-1]
        if likelihood is not None or covar_module is not None or mean_module is not None:
            raise UnsupportedError("custom modules of a multi-output SingleTaskGP (batched "
                                   "modules) are not on the accelerated path")
        if outcome_transform == "DEFAULT":
            outcome_transform = Standardize(m=m)
        if outcome_transform is not None and not (isinstance(outcome_transform, Standardize)
                                                  and outcome_transform._m == m):
            raise UnsupportedError("a multi-output SingleTaskGP takes Standardize(m) or no "
                                   "outcome transform here")
        if outcome_transform is not None:
            # statistics of the full n x m Y (the reference's reduction), each
            # member then holds its column of them
            outcome_transform.train()
            Y_tf, Yvar_tf = outcome_transform(train_Y, train_Yvar)
            outcome_transform.eval()
            self.outcome_transform = outcome_transform
        else:
            Y_tf, Yvar_tf = train_Y, train_Yvar
        members = []
        for t in range(m):
            mm = SingleTaskGP(train_X, Y_tf[:, t:t + 1],
                              None if Yvar_tf is None else Yvar_tf[:, t:t + 1],
                              outcome_transform=None)
            if outcome_transform is not None:
                col = Standardize(m=1, min_stdv=outcome_transform._min_stdv)
                col.means = outcome_transform.means[..., t:t + 1].clone()
                col.stdvs = outcome_transform.stdvs[..., t:t + 1].clone()
                col._is_trained = True
                col.eval()
                mm.outcome_transform = col
                mm._raw_train_Y = train_Y[:, t:t + 1]
            members.append(mm)
        self.models = nn.ModuleList(members)
        self._num_outputs = m
        for name in ("likelihood", "covar_module", "mean_module"):
            setattr(self, name, _StackedView(members, name))
        self.train_inputs = (train_X,)
        self.train_targets = torch.stack([mm.train_targets for mm in members])  # m x n
        self._cache = None
        self._cache_key = None

    @property
    def _is_multi_output(self) -> bool:
        return self._num_outputs > 1

    @staticmethod
    def _check_scaling(X, Y):
        """botorch/models/utils/assorted.py:219-261 (warnings only)."""
        if X.numel() and (X.min() < -1e-8 or X.max() > 1 + 1e-8):
            warnings.warn("Input data is not contained to the unit cube. Please consider "
                          "min-max scaling the input data.", InputDataWarning)

    # -- hyperparameter accessors ------------------------------------------------
    @property
    def kind(self) -> int:
        return self.covar_module.kind

    def hyper(self):
        if self._is_multi_output:
            raise UnsupportedError("hyper() of a multi-output SingleTaskGP: use model.models[t]")
        ls = self.covar_module.lengthscale.detach().reshape(-1)
        os_ = float(self.covar_module.outputscale.detach()) if isinstance(self.covar_module, ScaleKernel) else 1.0
        return ls, os_, float(self.likelihood.noise.detach().mean()), float(self.mean_module.constant.detach())

    def train(self, mode: bool = True):
        if mode:
            self._cache = None
            self._cache_key = None
        return super().train(mode)

    @property
    def batch_shape(self) -> torch.Size:
        return torch.Size([])

    def _key(self):
        if self._is_multi_output:
            return tuple(mm._key() for mm in self.models)
        d = self.__dict__
        if d.get("_plist_gen") != _STRUCTURE[0]:
            d["_plist"] = list(self.parameters())
            d["_plist_gen"] = _STRUCTURE[0]
        ps = [self.train_inputs[0], self.train_targets] + d["_plist"]
        return tuple((p.data_ptr(), p._version) for p in ps)

    def prediction_cache(self, key=None):
        """Device caches of [G] exact prediction; rebuilt on any change.
        ``key``: this model's _key(), when the caller has just computed it."""
        from . import kernels
        if self._is_multi_output:
            raise UnsupportedError("a multi-output SingleTaskGP keeps one cache per output "
                                   "(model.models[t].prediction_cache())")
        from .settings import propagate_grads
        if propagate_grads.on() and (self.train_inputs[0].requires_grad or self.train_targets.requires_grad):
            from .exceptions import UnsupportedError
            raise UnsupportedError(
                "settings.propagate_grads: posterior gradients to the training data are not "
                "supported (the prediction caches are built without a backward to them)")
        if key is None:
            key = self._key()
        if self._cache is None or self._cache_key != key:
            from . import ops  # noqa: F401  (torch.ops.bo registration)
            ls, os_, noise, c = self.hyper()
            Xt = self.train_inputs[0].contiguous()
            nv = self.likelihood.noise if isinstance(self.likelihood, FixedNoiseGaussianLikelihood) else None
            L, Linv, U, beta, alpha, Xs, jit = torch.ops.bo.gp_cache(
                Xt, self.train_targets.contiguous(), ls.contiguous(), float(os_), float(noise),
                float(c), int(self.kind), nv)
            n, d = Xt.shape
            self._cache = kernels.GPCache(self.kind, n, d, U.shape[0], Xt, Xs, ls.contiguous(),
                                          float(os_), float(noise), float(c), L, Linv, U, beta,
                                          alpha, 0.0)
            self._cache_key = key
        return self._cache

    def posterior(self, X: torch.Tensor, output_indices=None, observation_noise=False,
                  posterior_transform=None):
        """botorch/models/gpytorch.py:405-466 (m > 1: :327-355).  The model
        computes in fp64: X of another floating dtype is promoted (the
        gradient flows back through the cast)."""
        from .posteriors import GPyTorchPosterior, PosteriorList
        if X.dtype != torch.float64:
            X = X.to(torch.float64)
        if self._is_multi_output:
            idx = output_indices if output_indices is not None else range(self._num_outputs)
            prime_prediction_caches([self.models[i] for i in idx])
            post = PosteriorList(*[self.models[i].posterior(X, observation_noise=observation_noise)
                                   for i in idx])
            return post if posterior_transform is None else posterior_transform(post)
        if output_indices not in (None, [0]):
            raise UnsupportedError("single-output model")
        self.eval()
        post = GPyTorchPosterior.from_model(self, X, observation_noise=observation_noise)
        if posterior_transform is not None:
            return posterior_transform(post)
        return post


def prime_prediction_caches(models):
    """Build the missing prediction caches of several single-output exact GPs
    (a ModelListGP's members, the outputs of a multi-output SingleTaskGP, the
    SAAS ensemble's members) with ONE batched factorisation
    (kernels.build_gp_caches: the members' K + s2 I in one persistent DAG
    launch, one status read-back); each model.prediction_cache() then returns
    its cache without a launch.  When every model already holds a cache this
    returns at once (a stale cache, after new hyperparameters, is rebuilt by
    its own prediction_cache()).  The caches are bit-identical to the
    per-model builds; fixed-noise members and unequal orders keep the
    per-model path.  Returns each model's version key (None where not
    computed), for prediction_cache(key=...): one key computation per model
    and forward."""
    from . import kernels
    from .settings import propagate_grads
    if all(getattr(mm, "_cache", None) is not None for mm in models):
        # every model has a cache: a stale one (new hyperparameters) is rebuilt
        # by its own prediction_cache(); this keeps the per-forward host cost
        # of the common case (all fresh) at one attribute read per model
        return [None] * len(models)
    stale, keys = [], []
    pg = propagate_grads.on()
    for mm in models:
        keys.append(None)
        if not isinstance(mm, SingleTaskGP) or mm._is_multi_output:
            continue
        if isinstance(mm.likelihood, FixedNoiseGaussianLikelihood):
            continue
        if pg and (mm.train_inputs[0].requires_grad or mm.train_targets.requires_grad):
            continue  # prediction_cache raises the reference's error
        key = keys[-1] = mm._key()
        if mm._cache is not None and mm._cache_key == key:
            continue
        stale.append((mm, key))
    if len(stale) < 2:
        return keys
    specs = []
    for mm, _ in stale:
        ls, os_, noise, c = mm.hyper()
        specs.append(dict(Xt=mm.train_inputs[0].contiguous(), y=mm.train_targets.contiguous(),
                          lengthscale=ls.contiguous(), noise=float(noise), constant=float(c),
                          kind=int(mm.kind), outputscale=float(os_)))
    for (mm, key), cache in zip(stale, kernels.build_gp_caches(specs)):
        mm._cache = cache
        mm._cache_key = key
    return keys


class ModelListGP(Model):
    """Independent single-output GPs (botorch/models/model_list_gp_regression.py:24);
    its posterior is block-diagonal across outputs (models/gpytorch.py:629-726)."""

    def __init__(self, *models: SingleTaskGP):
        super().__init__()
        self.models = nn.ModuleList(models)
        self._num_outputs = len(models)

    def posterior(self, X, output_indices=None, observation_noise=False, posterior_transform=None):
        from .posteriors import PosteriorList
        idx = output_indices if output_indices is not None else range(len(self.models))
        prime_prediction_caches([self.models[i] for i in idx])
        post = PosteriorList(*[self.models[i].posterior(X, observation_noise=observation_noise) for i in idx])
        if posterior_transform is not None:
            return posterior_transform(post)
        return post

    def train(self, mode: bool = True):
        for m in self.models:
            m.train(mode)
        return super().train(mode)


MCMC_DIM = -3  # models/fully_bayesian.py: posterior batch dim of the MCMC samples


def sample_saas_prior(d: int, num_samples: int, seed: int = 0, dtype=torch.float64):
    """Hyperparameter sets from the SAAS prior (models/fully_bayesian.py:168-247):
    outputscale ~ Gamma(2, 0.15), mean ~ N(0, 1), noise = 1e-4 + Gamma(0.9, 10),
    tau^2 ~ HalfCauchy(0.1), inv_len^2 ~ HalfCauchy(1)^d, lengthscale =
    (tau^2 inv_len^2)^{-1/2}.  (NUTS itself is out of scope: pyro is absent.)"""
    g = torch.Generator().manual_seed(seed)
    M = num_samples

    def gamma(conc, rate, shape):
        # Marsaglia-Tsang through torch's generator-aware _standard_gamma
        return torch._standard_gamma(torch.full(shape, conc, dtype=dtype), generator=g) / rate

    def half_cauchy(scale, shape):
        u = torch.rand(shape, generator=g, dtype=dtype)
        return scale * torch.tan(0.5 * math.pi * u)

    tausq = half_cauchy(0.1, (M, 1))
    inv_len_sq = half_cauchy(1.0, (M, d))
    return {
        "outputscale": gamma(2.0, 0.15, (M,)),
        "mean": torch.randn(M, generator=g, dtype=dtype),
        "noise": MIN_INFERRED_NOISE_LEVEL + gamma(0.9, 10.0, (M,)),
        "lengthscale": (tausq * inv_len_sq).rsqrt(),
    }


class SaasFullyBayesianSingleTaskGP(Model):
    """Fully Bayesian SAAS GP (models/fully_bayesian.py:315-546): M hyperparameter
    sets (MCMC samples) of a ScaleKernel(Matern-5/2) GP with constant mean and
    Gaussian noise, evaluated as an ensemble.  The posterior at X (b x q x d) has
    batch shape b x M (X is broadcast over MCMC_DIM = -3); acquisition values are
    averaged over M (utils/transforms.py:289-293).

    Each member is an exact GP with its own device caches (Matern-5/2 kernel
    matrix, blocked MFMA Cholesky, L^{-T}); the q-batch posterior runs through
    the generic kernels (d = 50 exceeds the fused kernel's register-resident
    inputs)."""

    _is_fully_bayesian = True
    _is_ensemble = True

    def __init__(self, train_X, train_Y, train_Yvar=None, outcome_transform=None,
                 input_transform=None, pyro_model=None):
        super().__init__()
        if not (train_X.ndim == train_Y.ndim == 2 and len(train_X) == len(train_Y)
                and train_Y.shape[-1] == 1):
            raise ValueError("Expected train_X to have shape n x d and train_Y to have shape n x 1")
        if train_Yvar is not None or input_transform is not None:
            raise UnsupportedError("fixed noise / input transforms are not on the accelerated path")
        train_X = train_X.to(torch.float64)
        train_Y = train_Y.to(torch.float64)
        if outcome_transform is not None:
            outcome_transform.train()
            train_Y, _ = outcome_transform(train_Y)
            self.outcome_transform = outcome_transform
        self.train_inputs = (train_X,)
        self.train_targets = train_Y.squeeze(-1)
        self._members = None
        self._ens = None
        self._ens_key = None

    def ensemble_cache(self):
        """The members' prediction caches stacked for the batched ensemble path:
        U (M x n x n, each L_m^{-T}), alpha (M x n), lengthscale (M x d),
        outputscale (M), constant (M); rebuilt whenever a member's cache is."""
        keys = prime_prediction_caches(self._members)
        caches = [m.prediction_cache(key=k) for m, k in zip(self._members, keys)]
        key = tuple(id(c) for c in caches)
        if self._ens is None or self._ens_key != key:
            n = caches[0].n
            dev = caches[0].U.device
            f64 = dict(dtype=torch.float64, device=dev)
            self._ens = dict(
                n=n, kind=caches[0].kind, Xt=caches[0].Xt.contiguous(),
                U=torch.stack([c.U[:n, :n] for c in caches]).contiguous(),
                alpha=torch.stack([c.alpha.reshape(-1)[:n] for c in caches]).contiguous(),
                ls=torch.stack([c.lengthscale.reshape(-1) for c in caches]).contiguous(),
                os=torch.tensor([c.outputscale for c in caches], **f64),
                os_host=[float(c.outputscale) for c in caches],
                const=torch.tensor([c.constant for c in caches], **f64))
            self._ens_key = key
        return self._ens

    def load_mcmc_samples(self, mcmc_samples) -> None:
        """models/fully_bayesian.py:249-312 (batched modules from the samples)."""
        X = self.train_inputs[0]
        d = X.shape[-1]
        M = len(mcmc_samples["mean"])
        members = []
        for i in range(M):
            base = MaternKernel(ard_num_dims=d, lengthscale_lower=0.0, initial=1.0)
            base.lengthscale = mcmc_samples["lengthscale"][i].reshape(1, d)
            k = ScaleKernel(base, outputscale=float(mcmc_samples["outputscale"][i]))
            lik = GaussianLikelihood(noise_lower=MIN_INFERRED_NOISE_LEVEL, initial=max(
                float(mcmc_samples["noise"][i]), MIN_INFERRED_NOISE_LEVEL))
            mean = ConstantMean()
            mean.constant = float(mcmc_samples["mean"][i])
            mdl = SingleTaskGP(X, self.train_targets.unsqueeze(-1), likelihood=lik, covar_module=k,
                               mean_module=mean, outcome_transform=None)
            members.append(mdl.eval())
        self._members = nn.ModuleList(members)
        self._ens = None

    @property
    def num_mcmc_samples(self) -> int:
        if self._members is None:
            raise RuntimeError("Model has not been fitted. You need to call "
                               "`fit_fully_bayesian_model_nuts` to fit the model.")
        return len(self._members)

    @property
    def batch_shape(self) -> torch.Size:
        return torch.Size([self.num_mcmc_samples])

    def train(self, mode: bool = True):
        super().train(mode)
        if mode:
            self._members = None
        return self

    def posterior(self, X, output_indices=None, observation_noise=False, posterior_transform=None):
        """models/fully_bayesian.py:509-546 -> GaussianMixturePosterior (batch b x M)."""
        from .posteriors import GPyTorchPosterior, MultivariateNormal, posterior_moments
        M = self.num_mcmc_samples
        batch, q, d = X.shape[:-2], X.shape[-2], X.shape[-1]
        X3 = X.reshape(-1, q, d)
        means, covs = [], []
        for mdl in self._members:
            mu, cov = posterior_moments(mdl, X3)  # differentiable (generic kernels at d > 8)
            if observation_noise is True:
                # noise joins in the model's (standardised) space, before the
                # outcome untransform (models/gpytorch.py:446-466)
                cov = cov + mdl.likelihood.noise.reshape(()) * torch.eye(q, dtype=cov.dtype, device=cov.device)
            if hasattr(self, "outcome_transform"):
                tf = self.outcome_transform
                s = float(tf.stdvs.reshape(-1)[0])
                mu = float(tf.means.reshape(-1)[0]) + s * mu
                cov = cov * (s * s)
            means.append(mu)
            covs.append(cov)
        mean = torch.stack(means, dim=1).reshape(*batch, M, q)
        cov = torch.stack(covs, dim=1).reshape(*batch, M, q, q)
        post = GPyTorchPosterior(MultivariateNormal(mean, cov), model=self, X=X)
        post._is_ensemble = True
        return post if posterior_transform is None else posterior_transform(post)


def fit_fully_bayesian_model_nuts(model, **kwargs):
    """botorch/fit.py:335-391 -- NUTS over the SAAS prior needs pyro, which is not
    available (out of scope); load hyperparameters with ``load_mcmc_samples``."""
    raise UnsupportedError("NUTS fitting (pyro) is out of scope; use load_mcmc_samples")
