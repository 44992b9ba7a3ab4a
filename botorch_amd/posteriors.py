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


def _fused_moments(X3: torch.Tensor, model):
    """(mean', Sigma') of B t-batches of q <= 16 points (outcome space) through
    bo::gp_posterior, differentiable w.r.t. X3 (the op's registered backward)."""
    from . import ops  # noqa: F401  (torch.ops.bo registration)
    cache = model.prediction_cache()
    ymean, ystd = model.outcome_stats()
    need_grad = torch.is_grad_enabled() and X3.requires_grad
    mean, cov, _, _, _ = torch.ops.bo.gp_posterior(
        X3, cache.Xt, cache.Xt_scaled, cache.U, cache.Linv, cache.beta, cache.alpha,
        cache.lengthscale, int(cache.kind), float(cache.outputscale), float(cache.constant),
        float(ymean), float(ystd), bool(need_grad))
    return mean, cov


class _GeneralMoments(torch.autograd.Function):
    """(mean', Sigma') of B t-batches of any q and any d <= 128 through the
    generic kernels, differentiable w.r.t. X.

    Forward ([G] exact prediction): K*x (bo_covar_matrix), R = K*x L^{-T}
    (triangular MFMA GEMM against the cached U, leading dimension np), the
    R_b R_b^T blocks (batched GEMM), K** (bo_covar_blocks), mean = c + K*x alpha.
    Backward: d mu* = s d mu', G = s^2 (dS + dS^T); d K*x = d mu* alpha^T - G_b W_b
    with W = R L^{-1} = K*x A^{-1} (GEMM against U^T); d K** = G through
    bo_kernel_grad over the training points and over the t-batch's own points."""

    @staticmethod
    def forward(ctx, X3, model):
        cache = model.prediction_cache()
        ymean, ystd = model.outcome_stats()
        B, q, d = X3.shape
        n, np_ = cache.n, cache.np
        X2 = X3.detach().reshape(B * q, d).contiguous()
        Kx = kernels.covar_matrix(X2, cache.Xt, cache.lengthscale, cache.kind, cache.outputscale)
        R = torch.empty(B * q, n, dtype=torch.float64, device=X2.device)
        kernels.gemm_strided(B * q, n, n, Kx, n, 0, cache.U, np_, 0, R, n, 0, 1,
                             flags=_lib.GEMM_B_UPPER)
        mean = kernels.gemm(Kx, cache.alpha.reshape(n, 1)).reshape(B, q)
        RR = kernels.gemm(R.view(B, q, n), R.view(B, q, n), transB=True)
        Kxx = kernels.covar_blocks(X3.detach(), cache.lengthscale, cache.kind, cache.outputscale)
        cov = (Kxx - RR) * (ystd * ystd)
        mean = ymean + ystd * (mean + cache.constant)
        if ctx.needs_input_grad[0]:
            ctx.cache, ctx.ystd, ctx.X2, ctx.R, ctx.shape = cache, ystd, X2, R, (B, q, d)
        return mean, cov

    @staticmethod
    def backward(ctx, dmean, dcov):
        cache, ystd = ctx.cache, ctx.ystd
        B, q, d = ctx.shape
        n, np_ = cache.n, cache.np
        dev = ctx.R.device
        if dmean is None:
            dmean = torch.zeros(B, q, dtype=torch.float64, device=dev)
        if dcov is None:
            dcov = torch.zeros(B, q, q, dtype=torch.float64, device=dev)
        G = ((ystd * ystd) * (dcov + dcov.mT)).contiguous()
        W = torch.empty(B * q, n, dtype=torch.float64, device=dev)      # R L^{-1} = R U^T
        kernels.gemm_strided(B * q, n, n, ctx.R, n, 0, cache.U, np_, 0, W, n, 0, 1,
                             transB=True, flags=_lib.GEMM_B_LOWER)
        dK = ((ystd * dmean).reshape(B * q, 1) * cache.alpha.reshape(1, n)).contiguous()
        kernels.gemm(G, W.view(B, q, n), alpha=-1.0, beta=1.0, C=dK.view(B, q, n))
        dX = kernels.kernel_grad(ctx.X2, cache.Xt, dK, cache.lengthscale, cache.kind,
                                 cache.outputscale)
        dX = kernels.kernel_grad(ctx.X2, ctx.X2, G.view(B * q, q), cache.lengthscale, cache.kind,
                                 cache.outputscale, group=q, dX=dX)
        return dX.reshape(B, q, d), None


class _CholJitter(torch.autograd.Function):
    """psd_safe_cholesky with its gradient ([G] MultivariateNormal
    root_decomposition under autograd): forward = the jitter ladder
    (bo_chol_small / blocked MFMA Cholesky), backward = torch's
    linalg.cholesky backward (bo_chol_backward, q <= 64)."""

    @staticmethod
    def forward(ctx, A):
        L = kernels.chol_jitter(A.detach())
        ctx.save_for_backward(L)
        return L

    @staticmethod
    def backward(ctx, dL):
        (L,) = ctx.saved_tensors
        q = L.shape[-1]
        batch = L.shape[:-2]
        L3 = L.reshape(-1, q, q).contiguous()
        dL3 = dL.reshape(-1, q, q).tril().contiguous()
        if q <= 64:
            dA = kernels.chol_backward(L3, dL3)
        else:  # blocked roots beyond 64: the same formula as device GEMM/TRSM calls
            P = (L3.mT @ dL3).tril()
            P = 0.5 * (P + P.tril(-1).mT)
            Li = torch.linalg.solve_triangular(L3, torch.eye(q, dtype=L3.dtype, device=L3.device)
                                               .expand_as(L3), upper=False)
            dA = Li.mT @ P @ Li
        return dA.reshape(*batch, q, q)


def posterior_moments(model, X: torch.Tensor):
    """mean' (batch x q), Sigma' (batch x q x q) for X (batch x q x d): the fused
    kernels for q <= 16 and d <= 8, the generic kernels otherwise (both
    differentiable)."""
    batch = X.shape[:-2]
    q, d = X.shape[-2], X.shape[-1]
    X3 = X.reshape(-1, q, d).to(torch.float64)
    if not _fused_ok(q, d):
        mean, cov = _GeneralMoments.apply(X3, model)
    else:
        mean, cov = _fused_moments(X3, model)
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
            C = self.covariance_matrix
            if torch.is_grad_enabled() and C.requires_grad:
                self._scale_tril = _CholJitter.apply(C)
            else:
                self._scale_tril = kernels.chol_jitter(C)
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
            # homoskedastic: the one noise level; fixed noise: the mean of the
            # observed variances (models/gpytorch.py _apply_noise, FixedNoise case)
            noise = model.likelihood.noise.mean() * ystd * ystd
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
        if all(s == 0 for s in bstrides) or all(b == 1 for b in Z.shape[len(sample_shape):-1]):
            # shared base samples under autograd: one broadcast GEMM Z L^T
            Z2 = Z.reshape(-1, *Z.shape[len(sample_shape):])[(slice(None),) + (0,) * nb]
            f = torch.matmul(Z2, L.reshape(-1, q, q).mT)                    # B x S' x q
            f = f.permute(1, 0, 2) + mean.reshape(1, -1, q)
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

    def _reshape_and_cat(self, tensors):
        """posteriors/posterior_list.py: concatenate per-output samples (... x q x 1)."""
        return torch.cat(tensors, dim=-1)

    def rsample(self, sample_shape=None):
        return self._reshape_and_cat([p.rsample(sample_shape) for p in self.posteriors])
