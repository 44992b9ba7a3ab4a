"""Posterior objects with BoTorch's interface (botorch/posteriors/gpytorch.py:35-179).

The moments are produced by the gfx950 kernels (fused K*x build + R = K*x L^{-T}
GEMM + R R^T epilogue, then the per-t-batch finalisation) and are
differentiable w.r.t. the inputs through ``bo_post_backward``.
"""
from __future__ import annotations

from typing import List, Optional

import torch

from . import _lib, kernels
from .exceptions import NotPSDError, UnsupportedError

FUSED_QMAX = 16  # q limit of the fused posterior kernels (1 t-batch per 16-row MFMA tile)


def _fused_ok(q: int, d: int) -> bool:
    return q <= FUSED_QMAX and d <= kernels.DP


class _PosteriorMoments(torch.autograd.Function):
    """(mean', Sigma') of B t-batches of q points, outcome space."""

    @staticmethod
    def forward(ctx, X3, model):
        cache = model.prediction_cache()
        ymean, ystd = model.outcome_stats()
        need_grad = ctx.needs_input_grad[0]
        pp = kernels.post_partials(cache, X3.detach(), store_R=need_grad)
        out = kernels.qmc_finalize(cache, pp, _lib.QMC_POSTERIOR, ymean, ystd)
        if need_grad:
            ctx.cache, ctx.pp, ctx.ystd = cache, pp, ystd
            ctx.W = kernels.w_matrix(cache, pp)
        return out["mean"], out["cov"]

    @staticmethod
    def backward(ctx, dmean, dcov):
        pp = ctx.pp
        if dmean is None:
            dmean = torch.zeros(pp.B, pp.q, dtype=torch.float64, device=ctx.W.device)
        if dcov is None:
            dcov = torch.zeros(pp.B, pp.q, pp.q, dtype=torch.float64, device=ctx.W.device)
        dX = kernels.post_backward(ctx.cache, pp, ctx.W, dmean, dcov, ctx.ystd)
        return dX, None


def posterior_moments(model, X: torch.Tensor):
    """mean' (batch x q), Sigma' (batch x q x q) for X (batch x q x d)."""
    batch = X.shape[:-2]
    q, d = X.shape[-2], X.shape[-1]
    X3 = X.reshape(-1, q, d).to(torch.float64)
    if not _fused_ok(q, d):
        if X.requires_grad:
            raise UnsupportedError(
                f"gradients need q <= {FUSED_QMAX} and d <= {kernels.DP} (got q={q}, d={d})")
        mean, cov = kernels.posterior_general(model, X3)
    else:
        mean, cov = _PosteriorMoments.apply(X3, model)
    return mean.reshape(*batch, q), cov.reshape(*batch, q, q)


class MultivariateNormal:
    """Minimal [G] MultivariateNormal view over computed moments."""

    def __init__(self, mean: torch.Tensor, covariance_matrix: torch.Tensor):
        self.loc = mean
        self.covariance_matrix = covariance_matrix
        self._scale_tril = None

    mean = property(lambda self: self.loc)
    lazy_covariance_matrix = property(lambda self: self.covariance_matrix)
    batch_shape = property(lambda self: self.loc.shape[:-1])
    event_shape = property(lambda self: self.loc.shape[-1:])
    base_sample_shape = property(lambda self: self.loc.shape[-1:])
    islazy = False

    @property
    def variance(self) -> torch.Tensor:
        return self.covariance_matrix.diagonal(dim1=-2, dim2=-1)

    @property
    def scale_tril(self) -> torch.Tensor:
        """psd_safe_cholesky root (jitter ladder), as [G] root_decomposition."""
        if self._scale_tril is None:
            self._scale_tril = kernels.chol_jitter(self.covariance_matrix)
        return self._scale_tril


class GPyTorchPosterior:
    """botorch/posteriors/gpytorch.py:35-179 for single-output exact GPs."""

    def __init__(self, distribution: MultivariateNormal, model=None, X=None):
        self.distribution = distribution
        self.model = model
        self.X = X
        self._is_mt = False

    @classmethod
    def from_model(cls, model, X: torch.Tensor, observation_noise=False):
        mean, cov = posterior_moments(model, X)
        if observation_noise is True:
            _, ystd = model.outcome_stats()
            noise = model.likelihood.noise.reshape(()) * ystd * ystd
            cov = cov + noise * torch.eye(cov.shape[-1], dtype=cov.dtype, device=cov.device)
        elif torch.is_tensor(observation_noise):
            cov = cov + torch.diag_embed(observation_noise.squeeze(-1))
        return cls(MultivariateNormal(mean, cov), model=model, X=X)

    mvn = property(lambda self: self.distribution)
    device = property(lambda self: self.distribution.loc.device)
    dtype = property(lambda self: self.distribution.loc.dtype)
    batch_shape = property(lambda self: self.distribution.batch_shape)

    @property
    def base_sample_shape(self) -> torch.Size:
        return self.distribution.batch_shape + self.distribution.base_sample_shape

    @property
    def batch_range(self):
        return (0, -1)

    def _extended_shape(self, sample_shape=torch.Size()) -> torch.Size:
        return torch.Size(sample_shape) + self.distribution.batch_shape + self.distribution.event_shape + torch.Size([1])

    @property
    def mean(self) -> torch.Tensor:
        return self.distribution.mean.unsqueeze(-1)

    @property
    def variance(self) -> torch.Tensor:
        return self.distribution.variance.unsqueeze(-1)

    @property
    def covariance_matrix(self) -> torch.Tensor:
        return self.distribution.covariance_matrix

    def rsample_from_base_samples(self, sample_shape: torch.Size, base_samples: torch.Tensor):
        """posteriors/gpytorch.py:85-126: mean' + L base_samples, L the jittered
        Cholesky root.  base_samples: sample_shape x (batch) x q."""
        sample_shape = torch.Size(sample_shape)
        if base_samples.shape[: len(sample_shape)] != sample_shape:
            raise RuntimeError("`sample_shape` disagrees with shape of `base_samples`.")
        L = self.distribution.scale_tril
        mean = self.distribution.mean
        batch, q = mean.shape[:-1], mean.shape[-1]
        Z = base_samples.to(L)
        nb = len(batch)
        bstrides = Z.stride()[len(sample_shape): len(sample_shape) + nb]
        if not torch.is_grad_enabled() or not (mean.requires_grad or L.requires_grad):
            if all(s == 0 for s in bstrides) or all(b == 1 for b in Z.shape[len(sample_shape):-1]):
                # base samples shared across t-batches (the collapsed sampler layout):
                # one batched MFMA GEMM with the samples broadcast.
                Z2 = Z.reshape(-1, *Z.shape[len(sample_shape):])[(slice(None),) + (0,) * nb]
                f = kernels.sample_mvn(mean.reshape(-1, q), L.reshape(-1, q, q), Z2)
                return f.reshape(*sample_shape, *batch, q, 1)
        samples = mean + (L @ Z.unsqueeze(-1)).squeeze(-1)
        return samples.unsqueeze(-1)

    def rsample(self, sample_shape: Optional[torch.Size] = None):
        sample_shape = torch.Size([1]) if sample_shape is None else torch.Size(sample_shape)
        Z = torch.randn(sample_shape + self.base_sample_shape, dtype=self.dtype, device=self.device)
        return self.rsample_from_base_samples(sample_shape, Z)


class PosteriorList:
    """Independent per-output posteriors (botorch/posteriors/posterior_list.py)."""

    def __init__(self, *posteriors):
        self.posteriors = list(posteriors)

    @property
    def mean(self):
        return torch.cat([p.mean for p in self.posteriors], dim=-1)

    @property
    def variance(self):
        return torch.cat([p.variance for p in self.posteriors], dim=-1)

    device = property(lambda self: self.posteriors[0].device)
    dtype = property(lambda self: self.posteriors[0].dtype)
