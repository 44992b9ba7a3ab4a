"""Smooth, overflow-safe reductions of the LogEI family (the functions of
botorch/utils/safe_math.py that acquisition/logei.py composes), restated for
the generic acquisition route on device tensors.  The fused gfx950 route
evaluates the same expressions inside bo_qmc_finalize (csrc/logred.h); both
are pinned to the reference's own outputs, values and gradients, by
tests/test_logei_golden.py.

Conventions.  ``tau`` is a temperature: every smooth function f_tau(x) equals
tau * f_1(x / tau).  Reductions over ``dim`` (an int or a tuple) are anchored
at the maximum M over ``dim``: R(x) = M + r(x - M), so the exponentials see
non-positive arguments.  The anchored form is also the definition of the fat
maximum (its inner sum is not shift-equivariant), so M keeps its autograd path.
"""
from __future__ import annotations

import math
from typing import Callable, Tuple, Union

import torch
from torch.nn.functional import softplus

TAU_RELU = 1e-6  # acquisition/logei.py:66
TAU_MAX = 1e-2   # acquisition/logei.py:67

Dim = Union[int, Tuple[int, ...]]


def _dims(dim: Dim) -> Tuple[int, ...]:
    return (dim,) if isinstance(dim, int) else tuple(dim)


def _count(x: torch.Tensor, dim: Dim) -> int:
    return math.prod(x.shape[d] for d in _dims(dim))


def _anchored(inner: Callable[[torch.Tensor, Tuple[int, ...]], torch.Tensor], x: torch.Tensor,
              dim: Dim, keepdim: bool) -> torch.Tensor:
    """M + inner(x - M) over ``dim`` (safe_math.py:149-187's contract).

    An infinite maximum cannot anchor: a slice whose maximum is +-inf returns
    the sum of its entries equal to that maximum (so +inf stays +inf and an
    all -inf slice stays -inf) and its other entries get no gradient; the
    finite slices see x - M, with the infinite slices' entries replaced by 0
    so that no inf - inf reaches the autograd graph."""
    ds = _dims(dim)
    m = x.amax(dim=ds, keepdim=True)
    m_inf = torch.isinf(m)
    at_inf_max = m_inf & (x == m)
    slice_inf = at_inf_max
    for d in ds:
        slice_inf = slice_inf.any(dim=d, keepdim=True)
    anchor = torch.where(m_inf, torch.zeros_like(m), m)
    inf_value = torch.where(at_inf_max, x, torch.zeros_like(x)).sum(dim=ds, keepdim=True)
    finite_value = anchor + inner(torch.where(slice_inf, torch.zeros_like(x), x) - anchor, ds)
    out = torch.where(slice_inf, inf_value, finite_value)
    return out if keepdim else out.squeeze(ds)


def logsumexp(x: torch.Tensor, dim: Dim, keepdim: bool = False) -> torch.Tensor:
    """log sum exp over ``dim`` (safe_math.py:124-146)."""
    return _anchored(lambda y, ds: torch.logsumexp(y, dim=ds, keepdim=True), x, dim, keepdim)


def logmeanexp(X: torch.Tensor, dim: Dim, keepdim: bool = False) -> torch.Tensor:
    """log mean exp over ``dim`` (safe_math.py:209-223): the MC sample
    reduction of the LogEI family."""
    return logsumexp(X, dim=dim, keepdim=keepdim) - math.log(_count(X, dim))


def smooth_amax(X: torch.Tensor, dim: Dim = -1, keepdim: bool = False, tau=1.0) -> torch.Tensor:
    """tau log sum exp(x / tau) (safe_math.py:250-273): the q reduction with
    fat=False."""
    return tau * logsumexp(X / tau, dim=dim, keepdim=keepdim)


def _pareto_tail(z: torch.Tensor, alpha: float) -> torch.Tensor:
    """(b0 / (b0 + b1 z + z^2))^(alpha/2), b1 = alpha, b0 = alpha^2 / 2: equal
    to 1 with slope -1 at z = 0 and decaying like z^-alpha (safe_math.py:
    454-478)."""
    a = 0.5 * alpha
    b1 = 2.0 * a
    b0 = a * b1
    return (b0 / (b0 + b1 * z + z * z)) ** a


def fatmax(x: torch.Tensor, dim: Dim, keepdim: bool = False, tau=1.0, alpha: float = 2.0):
    """Fat-tailed smooth maximum (safe_math.py:323-352):
    M + tau log sum_j tail((M - x_j) / tau), M the maximum over ``dim``."""
    def inner(y, ds):
        return tau * _pareto_tail(-y / tau, alpha).sum(dim=ds, keepdim=True).log()
    return _anchored(inner, x, dim, keepdim)


def log_softplus(x: torch.Tensor, tau=1.0) -> torch.Tensor:
    """log(tau softplus(x / tau)) (safe_math.py:226-247).  Below z = x / tau =
    -35 (fp64; -15 in fp32) softplus(z) = exp(z) to working precision, so the
    log is z + log tau, taken in closed form; above z = 32 (16) softplus is the
    identity (torch's threshold)."""
    t = torch.as_tensor(tau, dtype=x.dtype, device=x.device)
    lo, hi = (-15, 16) if x.dtype == torch.float32 else (-35, 32)
    z = x / t
    tiny = z <= lo
    body = softplus(torch.where(tiny, torch.full_like(x, lo), x), beta=1 / t, threshold=hi).log()
    return torch.where(tiny, z + t.log(), body)


def fatplus(x: torch.Tensor, tau=1.0) -> torch.Tensor:
    """tau (softplus(z) + 0.1 / (1 + z^2)), z = x / tau (safe_math.py:
    302-320): a softplus whose left tail decays only quadratically."""
    z = x / tau
    return tau * (softplus(z) + 0.1 / (1 + z * z))


def log_fatplus(x: torch.Tensor, tau=1.0) -> torch.Tensor:
    """log fatplus (safe_math.py:293-299)."""
    return torch.log(fatplus(x, tau=tau))


def log_improvement(Y: torch.Tensor, best_f: torch.Tensor, tau, fat: bool) -> torch.Tensor:
    """log of the smoothed improvement (Y - best_f)_+ (acquisition/logei.py:
    509-534); best_f broadcasts against Y without its q dimension."""
    diff = Y - best_f.unsqueeze(-1).to(Y)
    return log_fatplus(diff, tau=tau) if fat else log_softplus(diff, tau=tau)


def log1pexp(x: torch.Tensor) -> torch.Tensor:
    """log(1 + e^x) (safe_math.py:84-94): log1p(e^x) up to x = 18, x + e^-x
    above (where e^x would lose log1p's precision)."""
    small = x <= 18
    xs = torch.where(small, x, torch.zeros_like(x))
    xl = torch.where(small, torch.zeros_like(x), x)
    return torch.where(small, torch.log1p(torch.exp(xs)), xl + torch.exp(-xl))


def logexpit(X: torch.Tensor) -> torch.Tensor:
    """log sigmoid(x) = -log(1 + e^-x) (safe_math.py:97-99)."""
    return -log1pexp(-X)


def cauchy(x: torch.Tensor) -> torch.Tensor:
    """1 / (1 + x^2), the un-normalised Cauchy density (safe_math.py:449-451)."""
    return 1 / (1 + x * x)


def fatmoid(X: torch.Tensor, tau=1.0) -> torch.Tensor:
    """Fat-tailed smooth step (safe_math.py:429-446): two Cauchy halves
    shifted by 1/sqrt(3) (the inflection points) and joined at 0 with value
    1/2."""
    z = X / tau
    s = 1 / math.sqrt(3)
    return torch.where(z < 0, (2 / 3) * cauchy(z - s), 1 - (2 / 3) * cauchy(z + s))


def log_fatmoid(X: torch.Tensor, tau=1.0) -> torch.Tensor:
    """log fatmoid (safe_math.py:422-426)."""
    return torch.log(fatmoid(X, tau=tau))
