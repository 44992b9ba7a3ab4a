"""Smooth, numerically safe reductions of the LogEI family on device tensors
(botorch/utils/safe_math.py).  Used by the non-fused (generic) acquisition
route; the fused gfx950 route evaluates the same expressions inside
bo_qmc_finalize (botorch_amd/csrc/logred.h).
"""
from __future__ import annotations

import math
from typing import Tuple, Union

import torch
from torch.nn.functional import softplus

TAU_RELU = 1e-6  # acquisition/logei.py:66
TAU_MAX = 1e-2   # acquisition/logei.py:67

Dim = Union[int, Tuple[int, ...]]


def _any(x: torch.Tensor, dim: Dim, keepdim: bool = False) -> torch.Tensor:
    """safe_math.py:190-206."""
    dims = dim if isinstance(dim, tuple) else (dim,)
    for d in dims:
        x = x.any(dim=d, keepdim=True)
    return x if keepdim else x.squeeze(dim)


def _inf_max_helper(max_fun, x: torch.Tensor, dim: Dim, keepdim: bool) -> torch.Tensor:
    """safe_math.py:149-187: anchor at the maximum, with +inf maxima passed through."""
    M = x.amax(dim=dim, keepdim=True)
    is_inf_max = torch.logical_and(*torch.broadcast_tensors(M.isinf(), x == M))
    has_inf_max = _any(is_inf_max, dim=dim, keepdim=True)
    y_inf = x.masked_fill(~is_inf_max, 0.0)
    M_no_inf = M.masked_fill(M.isinf(), 0.0)
    y_no_inf = x.masked_fill(has_inf_max, 0.0) - M_no_inf
    res = torch.where(has_inf_max, y_inf.sum(dim=dim, keepdim=True),
                      M_no_inf + max_fun(y_no_inf, dim=dim, keepdim=True))
    return res if keepdim else res.sum(dim=dim)


def logsumexp(x: torch.Tensor, dim: Dim, keepdim: bool = False) -> torch.Tensor:
    """safe_math.py:124-146."""
    return _inf_max_helper(torch.logsumexp, x=x, dim=dim, keepdim=keepdim)


def logmeanexp(X: torch.Tensor, dim: Dim, keepdim: bool = False) -> torch.Tensor:
    """safe_math.py:209-223."""
    n = X.shape[dim] if isinstance(dim, int) else math.prod(X.shape[i] for i in dim)
    return logsumexp(X, dim=dim, keepdim=keepdim) - math.log(n)


def log_softplus(x: torch.Tensor, tau=1.0) -> torch.Tensor:
    """safe_math.py:226-247 (fp64 cutoffs -35 / 32, fp32 -15 / 16)."""
    tau = torch.as_tensor(tau, dtype=x.dtype, device=x.device)
    upper = 16 if x.dtype == torch.float32 else 32
    lower = -15 if x.dtype == torch.float32 else -35
    mask = x / tau > lower
    return torch.where(mask, softplus(x.masked_fill(~mask, lower), beta=(1 / tau), threshold=upper).log(),
                       x / tau + tau.log())


def smooth_amax(X: torch.Tensor, dim: Dim = -1, keepdim: bool = False, tau=1.0) -> torch.Tensor:
    """safe_math.py:250-273."""
    return logsumexp(X / tau, dim=dim, keepdim=keepdim) * tau


def fatplus(x: torch.Tensor, tau=1.0) -> torch.Tensor:
    """safe_math.py:302-320: tau (softplus(x/tau) + 0.1 cauchy(x/tau))."""
    z = x / tau
    return tau * (softplus(z) + 1e-1 / (1 + z.square()))


def log_fatplus(x: torch.Tensor, tau=1.0) -> torch.Tensor:
    """safe_math.py:293-299."""
    return fatplus(x, tau=tau).log()


def _pareto(x: torch.Tensor, alpha: float) -> torch.Tensor:
    """safe_math.py:454-478."""
    alpha = alpha / 2
    beta_1 = 2 * alpha
    beta_0 = alpha * beta_1
    return (beta_0 / (beta_0 + beta_1 * x + x.square())).pow(alpha)


def fatmax(x: torch.Tensor, dim: Dim, keepdim: bool = False, tau=1.0, alpha: float = 2.0):
    """safe_math.py:323-352."""

    def max_fun(y, dim, keepdim=False):
        return tau * _pareto(-y / tau, alpha=alpha).sum(dim=dim, keepdim=keepdim).log()

    return _inf_max_helper(max_fun=max_fun, x=x, dim=dim, keepdim=keepdim)


def log_improvement(Y: torch.Tensor, best_f: torch.Tensor, tau, fat: bool) -> torch.Tensor:
    """acquisition/logei.py:509-534: log of the smoothed (Y - best_f)_+;
    best_f broadcasts against Y without its q dimension."""
    log_soft_clamp = log_fatplus if fat else log_softplus
    return log_soft_clamp(Y - best_f.unsqueeze(-1).to(Y), tau=tau)


def log1pexp(x: torch.Tensor) -> torch.Tensor:
    """safe_math.py:84-94: log(1 + exp(x)), switching form above x = 18."""
    mask = x <= 18
    return torch.where(mask, x.masked_fill(~mask, 0).exp().log1p(),
                       (lambda z: z + (-z).exp())(x.masked_fill(mask, 0)))


def logexpit(X: torch.Tensor) -> torch.Tensor:
    """safe_math.py:97-99: log of the logistic sigmoid."""
    return -log1pexp(-X)


_INV_SQRT_3 = math.sqrt(1 / 3)


def cauchy(x: torch.Tensor) -> torch.Tensor:
    """safe_math.py:449-451: un-normalised Cauchy density."""
    return 1 / (1 + x.square())


def fatmoid(X: torch.Tensor, tau=1.0) -> torch.Tensor:
    """safe_math.py:429-446: fat-tailed smooth Heaviside (inflection at 1/sqrt 3)."""
    X = X / tau
    m = _INV_SQRT_3
    return torch.where(X < 0, 2 / 3 * cauchy(X - m), 1 - 2 / 3 * cauchy(X + m))


def log_fatmoid(X: torch.Tensor, tau=1.0) -> torch.Tensor:
    """safe_math.py:422-426."""
    return fatmoid(X, tau=tau).log()
