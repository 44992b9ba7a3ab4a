"""CPU restatement of the exact-GP numerics on the reference's hot path.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).  fp64 torch on CPU.

[G] = gpytorch 1.12 / linear_operator 0.5.2 (pinned at requirements.txt:5-6),
whose sources are not available here; their published algorithms are restated.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

import torch

RBF, MATERN52 = 0, 1

# botorch/__init__.py:47 -- linop cholesky_max_tries overridden to 6.
CHOLESKY_MAX_TRIES = 6
# [G] linear_operator.settings.cholesky_jitter defaults: float 1e-6, double 1e-8.
CHOLESKY_JITTER = {torch.float32: 1e-6, torch.float64: 1e-8}
# botorch/models/utils/gpytorch_modules.py:29
MIN_INFERRED_NOISE_LEVEL = 1e-4
LENGTHSCALE_LOWER = 2.5e-2  # gpytorch_modules.py:123


class NotPSDError(RuntimeError):
    pass


class NanError(RuntimeError):
    pass


def sq_dist(x1: torch.Tensor, x2: torch.Tensor, x1_eq_x2: bool = False) -> torch.Tensor:
    """[G] gpytorch.kernels.kernel.sq_dist: mean-centred quadratic expansion, clamped at 0."""
    adjustment = x1.mean(-2, keepdim=True)
    x1 = x1 - adjustment
    x2 = x2 - adjustment
    x1_norm = x1.pow(2).sum(dim=-1, keepdim=True)
    x2_norm = x2.pow(2).sum(dim=-1, keepdim=True)
    x1_ = torch.cat([-2.0 * x1, x1_norm, torch.ones_like(x1_norm)], dim=-1)
    x2_ = torch.cat([x2, torch.ones_like(x2_norm), x2_norm], dim=-1)
    res = x1_.matmul(x2_.transpose(-2, -1))
    if x1_eq_x2:
        res.diagonal(dim1=-2, dim2=-1).fill_(0)
    return res.clamp_min_(0)


def covar(x1, x2, lengthscale, kind=RBF, outputscale=1.0, x1_eq_x2=False):
    """[G] RBFKernel / MaternKernel(nu=2.5) forward (+ ScaleKernel).

    RBF: exp(-d2/2) on x/ell (botorch default kernel,
    botorch/models/utils/gpytorch_modules.py:100-127).
    Matern-5/2: (1 + sqrt5 r + 5/3 r^2) exp(-sqrt5 r), inputs centred by the
    mean of x1 before scaling ([G] MaternKernel.forward; restated by the
    reference at botorch/models/fully_bayesian.py:81-92).
    """
    if kind == RBF:
        d2 = sq_dist(x1 / lengthscale, x2 / lengthscale, x1_eq_x2)
        return d2.div(-2).exp() * outputscale
    mean = x1.mean(dim=-2, keepdim=True)
    x1_ = (x1 - mean) / lengthscale
    x2_ = (x2 - mean) / lengthscale
    r = sq_dist(x1_, x2_, x1_eq_x2).clamp_min(1e-30).sqrt()
    e = torch.exp(-math.sqrt(5) * r)
    return (1 + math.sqrt(5) * r + 5.0 / 3.0 * r * r) * e * outputscale


def psd_safe_cholesky(A: torch.Tensor, jitter: Optional[float] = None,
                      max_tries: int = CHOLESKY_MAX_TRIES):
    """[G] linear_operator.utils.cholesky.psd_safe_cholesky.

    Plain Cholesky first; on failure add ``jitter * 10**i`` (i = 0..max_tries-1)
    to the diagonal of only the *currently failing* batch members (increments
    ``jitter_new - jitter_prev``), retrying after each increment.  NaN input
    raises NanError; still failing after the ladder raises NotPSDError.

    Returns ``(L, jitter_added)`` with the total jitter per batch member.
    """
    L, info = torch.linalg.cholesky_ex(A)
    added = torch.zeros(A.shape[:-2], dtype=A.dtype)
    if not torch.any(info):
        return L, added
    if torch.isnan(A).any():
        raise NanError("cholesky input contains NaN")
    if jitter is None:
        jitter = CHOLESKY_JITTER[A.dtype]
    Aprime = A.clone()
    jitter_prev = 0.0
    for i in range(max_tries):
        jitter_new = jitter * (10 ** i)
        inc = (info > 0).to(A.dtype) * (jitter_new - jitter_prev)
        Aprime.diagonal(dim1=-1, dim2=-2).add_(inc.unsqueeze(-1))
        added = added + inc
        jitter_prev = jitter_new
        L, info = torch.linalg.cholesky_ex(Aprime)
        if not torch.any(info):
            return L, added
    raise NotPSDError(f"not p.d. after jitter up to {jitter_new:.1e}")


def standardize_fit(Y: torch.Tensor, min_stdv: float = 1e-8):
    """botorch/models/transforms/outcome.py:253-307 (train-mode Standardize.forward)."""
    if Y.shape[-2] == 1:
        stdvs = torch.ones(*Y.shape[:-2], 1, Y.shape[-1], dtype=Y.dtype)
    else:
        stdvs = Y.std(dim=-2, keepdim=True)
    stdvs = stdvs.where(stdvs >= min_stdv, torch.full_like(stdvs, 1.0))
    means = Y.mean(dim=-2, keepdim=True)
    return means, stdvs


@dataclass
class GPHyper:
    """SingleTaskGP hyperparameters (transform=None constraints: raw == value)."""
    lengthscale: torch.Tensor  # (d,)
    noise: float  # or an (n,) tensor: a fixed-noise likelihood's variances, K + diag(noise)
    constant: float
    outputscale: float = 1.0
    kind: int = RBF

    @staticmethod
    def default(d: int, dtype=torch.float64) -> "GPHyper":
        # LogNormal(sqrt2 + ln(d)/2, sqrt3) mode; LogNormal(-4, 1) mode
        # (gpytorch_modules.py:74-127).
        ls_mode = math.exp(math.sqrt(2) + 0.5 * math.log(d) - 3.0)
        return GPHyper(torch.full((d,), ls_mode, dtype=dtype), math.exp(-5.0), 0.0)


class ExactGPOracle:
    """SingleTaskGP(train_X, train_Y) + Standardize in eval mode.

    Caches follow [G] DefaultPredictionStrategy under botorch's settings
    (botorch/__init__.py:44-49, models/utils/assorted.py:286-298):
      L       = psd_safe_cholesky(K + s2 I)
      covar_cache = L^{-T}   (root_inv_decomposition, Cholesky method)
      mean_cache  = (K + s2 I)^{-1} (y - c)   (cholesky_solve)
    Exact prediction (fast_pred_var): mu = c + K*x alpha,
      Sigma = K** - (K*x L^{-T}) (K*x L^{-T})^T.
    """

    def __init__(self, train_X, train_Y, hyper: GPHyper, standardize: bool = True):
        self.train_X = train_X.double()
        Y = train_Y.double()
        if Y.ndim == 1:
            Y = Y.unsqueeze(-1)
        if standardize:
            self.ymean, self.ystd = standardize_fit(Y)
        else:
            self.ymean = torch.zeros(1, 1, dtype=torch.float64)
            self.ystd = torch.ones(1, 1, dtype=torch.float64)
        self.train_y = ((Y - self.ymean) / self.ystd).squeeze(-1)
        self.h = hyper
        self._build()

    def _k(self, x1, x2, x1_eq_x2=False):
        return covar(x1, x2, self.h.lengthscale, self.h.kind, self.h.outputscale, x1_eq_x2)

    def _build(self):
        n = self.train_X.shape[0]
        K = self._k(self.train_X, self.train_X, x1_eq_x2=True)
        A = K + self.h.noise * torch.eye(n, dtype=torch.float64)
        self.L, self.jitter = psd_safe_cholesky(A)
        eye = torch.eye(n, dtype=torch.float64)
        Linv = torch.linalg.solve_triangular(self.L, eye, upper=False)
        self.LinvT = Linv.mT.contiguous()
        resid = (self.train_y - self.h.constant).unsqueeze(-1)
        self.alpha = torch.cholesky_solve(resid, self.L).squeeze(-1)

    # -- exact prediction ---------------------------------------------------
    def latent(self, X):
        """Standardized-space posterior: mean (..., q), covariance (..., q, q)."""
        Ktx = self._k(X, self.train_X)
        mean = Ktx @ self.alpha + self.h.constant
        R = Ktx @ self.LinvT
        Kxx = self._k(X, X, x1_eq_x2=True)
        cov = Kxx - R @ R.mT
        return mean, cov, R

    def posterior(self, X):
        """Outcome-space posterior (Standardize.untransform_posterior,
        botorch/models/transforms/outcome.py:373-447): mu' = ybar + s mu,
        Sigma' = s Sigma s."""
        mean, cov, _ = self.latent(X)
        s = self.ystd.squeeze()
        return self.ymean.squeeze() + s * mean, cov * (s * s)

    def mean_var(self, X):
        m, c = self.posterior(X)
        return m, c.diagonal(dim1=-2, dim2=-1)


# -- marginal log likelihood ------------------------------------------------
def lognormal_log_prob(x, loc, scale):
    """torch LogNormal(loc, scale).log_prob(x) ([G] LogNormalPrior)."""
    lx = torch.log(x)
    return -((lx - loc) ** 2) / (2 * scale ** 2) - math.log(scale) - 0.5 * math.log(2 * math.pi) - lx


def neg_mll(train_X, train_y, lengthscale, noise, constant, fixed_noise: bool = False):
    """Loss of botorch's exact-MLL closure (optim/closures/model_closures.py:171-184).

    [G] ExactMarginalLogLikelihood: (log N(y | c, K + s2 I) + sum of prior
    log-probs) / n, negated; priors = LogNormal(sqrt2 + ln(d)/2, sqrt3) on each
    lengthscale and LogNormal(-4, 1) on the noise (gpytorch_modules.py:74-127).
    Differentiable (autograd) in lengthscale, noise, constant.
    fixed_noise: ``noise`` is the n observed variances of a fixed-noise
    likelihood ([G] FixedNoiseGaussianLikelihood, gp_regression.py:187-194):
    K + diag(noise), no noise prior.
    """
    n, d = train_X.shape
    K = covar(train_X, train_X, lengthscale, RBF, 1.0, x1_eq_x2=True)
    A = K + noise * torch.eye(n, dtype=train_X.dtype)
    L = torch.linalg.cholesky(A)
    diff = (train_y - constant).unsqueeze(-1)
    v = torch.linalg.solve_triangular(L, diff, upper=False)
    inv_quad = (v * v).sum()
    logdet = 2 * torch.log(torch.diagonal(L)).sum()
    ll = -0.5 * (inv_quad + logdet + n * math.log(2 * math.pi))
    ls_loc = math.sqrt(2) + 0.5 * math.log(d)
    prior = lognormal_log_prob(lengthscale, ls_loc, math.sqrt(3)).sum()
    if not fixed_noise:
        prior = prior + lognormal_log_prob(noise.reshape(-1), -4.0, 1.0).sum()
    return -(ll + prior) / n


def fit_scipy(train_X, train_y, x0, bounds, options=None):
    """fit_gpytorch_mll_scipy (optim/fit.py:47-110 -> optim/core.py:55-140):
    scipy L-BFGS-B over the flat parameter vector [noise, constant,
    lengthscale_1..d] (the order of get_parameters_and_bounds for
    SingleTaskGP), with bounds from the constraints and the closure's loss and
    autograd gradient (neg_mll).  Returns the scipy OptimizeResult."""
    import numpy as np
    from scipy.optimize import minimize

    def f(x):
        noise = torch.tensor(float(x[0]), dtype=torch.float64, requires_grad=True)
        c = torch.tensor(float(x[1]), dtype=torch.float64, requires_grad=True)
        ls = torch.tensor(np.asarray(x[2:]), dtype=torch.float64, requires_grad=True)
        loss = neg_mll(train_X, train_y, ls, noise, c)
        loss.backward()
        g = np.concatenate([[noise.grad.item(), c.grad.item()], ls.grad.numpy()])
        return loss.item(), g

    return minimize(f, np.asarray(x0, dtype=np.float64), jac=True, method="L-BFGS-B",
                    bounds=bounds, options=options or {})
