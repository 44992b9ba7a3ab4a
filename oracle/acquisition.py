"""CPU restatement of the MC (and analytic) acquisition functions on the path.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).
"""
from __future__ import annotations

import itertools
import math

import torch

from .gp import ExactGPOracle, psd_safe_cholesky
from .sampling import draw_sobol_normal_samples


def mc_samples(mean, cov, Z):
    """posteriors/gpytorch.py:85-126 -> [G] MultivariateNormal.rsample with base
    samples: L = psd_safe_cholesky(Sigma'), f[s,b,i] = mu'[b,i] + sum_j L[b,i,j] Z[s,j]."""
    L, _ = psd_safe_cholesky(cov)
    return mean.unsqueeze(0) + torch.einsum("...ij,sj->s...i", L, Z)


def qei_from_samples(samples, best_f):
    """acquisition/monte_carlo.py:405-414 (_sample_forward) + q_reduction=amax,
    sample_reduction=mean (:246-274)."""
    return (samples - best_f).clamp_min(0).amax(dim=-1).mean(dim=0)


def qei(model: ExactGPOracle, X, Z, best_f):
    """qExpectedImprovement.forward (acquisition/monte_carlo.py:253-289, 405-414)."""
    mean, cov = model.posterior(X)
    return qei_from_samples(mc_samples(mean, cov, Z), best_f)


def ei_analytic(model: ExactGPOracle, X, best_f, maximize=True):
    """ExpectedImprovement.forward (acquisition/analytic.py:338-354, 84-108, 968-972)."""
    mean, var = model.mean_var(X)
    mean = mean.squeeze(-1)
    sigma = var.squeeze(-1).clamp_min(1e-12).sqrt()
    u = (mean - best_f) / sigma
    if not maximize:
        u = -u
    return sigma * ei_helper(u)


def ei_helper(u):
    """phi(u) + u Phi(u) (analytic.py:968-972; utils/probability/utils.py:133-142)."""
    phi = torch.exp(-0.5 * u * u) / math.sqrt(2 * math.pi)
    Phi = 0.5 * torch.erfc(-u / math.sqrt(2))
    return phi + u * Phi


# -- qNEI with cached baseline root ----------------------------------------------
def prune_inferior_points(model: ExactGPOracle, X, num_samples=2048, seed=0, max_frac=1.0):
    """acquisition/utils.py:245-349 (unconstrained, identity objective; the
    sampler seed is made explicit for determinism)."""
    mean, cov = model.posterior(X)
    Z = draw_sobol_normal_samples(X.shape[-2], num_samples, seed)
    samples = mc_samples(mean, cov, Z)  # S x n
    is_best = torch.argmax(samples, dim=-1)
    idcs, counts = torch.unique(is_best, return_counts=True)
    max_points = math.ceil(max_frac * X.size(-2))
    if len(idcs) > max_points:
        counts, order_idcs = torch.sort(counts, descending=True)
        idcs = order_idcs[:max_points]  # reference quirk kept (utils.py:345-347)
    return X[idcs]


def prune_inferior_points_multi_objective(models, X, ref_point, num_samples=2048, seed=0,
                                          max_frac=1.0):
    """acquisition/multi_objective/utils.py:77-161 (unconstrained, identity
    objective; the sampler seed -- the reference's SobolQMCNormalSampler draws
    it with torch.randint(0, 1000000, (1,)) -- made explicit): joint samples of
    the independent outputs from the point-major / output-minor base samples
    (Sobol dim n m), a point kept when it is Pareto-optimal (pareto.py:16-64,
    deduplicate=False) and better than ref_point in every objective in any
    sample."""
    from .sampling import base_samples_multi_output
    n, m = X.shape[-2], len(models)
    Z = base_samples_multi_output(num_samples, n, m, seed)  # S x m x n
    cols = []
    for t, mod in enumerate(models):
        mean, cov = mod.posterior(X)
        cols.append(mc_samples(mean, cov, Z[:, t]))  # S x n
    obj = torch.stack(cols, dim=-1)  # S x n x m
    # dominated[s, a] = some b with obj[s, b] >= obj[s, a] everywhere and > somewhere
    Ya, Yb = obj.unsqueeze(-2), obj.unsqueeze(-3)  # [s, a, 1, m], [s, 1, b, m]
    dominates = (Yb >= Ya).all(dim=-1) & (Yb > Ya).any(dim=-1)  # [s, a, b]
    mask = ~dominates.any(dim=-1) & (obj > torch.as_tensor(ref_point, dtype=obj.dtype)).all(dim=-1)
    probs = mask.to(obj.dtype).mean(dim=0)
    idcs = probs.nonzero().view(-1)
    max_points = math.ceil(max_frac * n)
    if idcs.shape[0] > max_points:
        _, order = torch.sort(probs, descending=True)
        idcs = order[:max_points]
    return X[idcs]


class QNEIOracle:
    """qNoisyExpectedImprovement with cache_root=True (acquisition/monte_carlo.py:
    441-625, cached_cholesky.py:94-186, utils/low_rank.py:85-173,
    sampling/normal.py:68-131)."""

    def __init__(self, model: ExactGPOracle, X_baseline, S: int, seed: int):
        self.model = model
        self.Xb = X_baseline
        self.S = S
        self.seed = seed
        r = X_baseline.shape[-2]
        mean_b, cov_b = model.posterior(X_baseline)
        self.Zb = draw_sobol_normal_samples(r, S, seed)  # S x r
        Lb, _ = psd_safe_cholesky(cov_b)
        base_samples = mean_b.unsqueeze(0) + self.Zb @ Lb.mT  # S x r
        self.best_f = base_samples.amax(dim=-1)  # S
        self.L_rr = Lb  # root decomposition of the baseline covariance
        self._zq = {}

    def base_samples_q(self, q):
        if q not in self._zq:
            r = self.Xb.shape[-2]
            full = draw_sobol_normal_samples(r + q, self.S, self.seed)
            full[:, :r] = self.Zb
            self._zq[q] = full
        return self._zq[q]

    def samples(self, X):
        b, q, d = X.shape
        r = self.Xb.shape[-2]
        Xf = torch.cat([self.Xb.expand(b, r, d), X], dim=-2)
        mean, cov = self.model.posterior(Xf)
        bottom = cov[..., -q:, :]
        bl, br = bottom[..., :r], bottom[..., r:]
        bl_chol = torch.linalg.solve_triangular(self.L_rr, bl.mT, upper=False).mT
        br_chol, _ = psd_safe_cholesky(br - bl_chol @ bl_chol.mT)
        Lq = torch.cat([bl_chol, br_chol], dim=-1)  # b x q x (r+q)
        Z = self.base_samples_q(q)  # S x (r+q)
        return mean[..., -q:].unsqueeze(0) + torch.einsum("bij,sj->sbi", Lq, Z)

    def __call__(self, X):
        f = self.samples(X)
        return (f - self.best_f.view(-1, 1, 1)).clamp_min(0).amax(dim=-1).mean(dim=0)


def qnei_full_joint(model: ExactGPOracle, X_baseline, X, Z_joint, sample_slice=None):
    """qNoisyExpectedImprovement with cache_root=False (acquisition/monte_carlo.py:
    577-626, 540-575): samples of the joint posterior over (X_baseline, X) with
    the joint base samples Z_joint (S x (r+q)); per-sample best over the
    baseline columns, improvement of the last q columns."""
    b, q, d = X.shape
    r = X_baseline.shape[-2]
    Xf = torch.cat([X_baseline.expand(b, r, d), X], dim=-2)
    mean, cov = model.posterior(Xf)
    f = mc_samples(mean, cov, Z_joint)                  # S x b x (r+q)
    best = f[..., :r].amax(dim=-1)                      # S x b
    return (f[..., r:] - best.unsqueeze(-1)).clamp_min(0).amax(dim=-1).mean(dim=0)


def smoothed_feasibility(constraints, samples, eta):
    """utils/objective.py:134-180 (log=False, fat=False): prod_i sigmoid(-c_i / eta)."""
    ind = torch.ones_like(samples[..., 0])
    for c in constraints:
        ind = ind * torch.sigmoid(-c(samples) / eta)
    return ind


def qei_constrained(model: ExactGPOracle, X, Z, best_f, constraints, eta=1e-3):
    """qExpectedImprovement with outcome constraints (monte_carlo.py:253-330):
    relu(f - best_f) weighted per sample and point by the smoothed feasibility
    of the samples, then max over q and mean over samples."""
    mean, cov = model.posterior(X)
    f = mc_samples(mean, cov, Z)                        # S x b x q
    w = smoothed_feasibility(constraints, f.unsqueeze(-1), eta)
    return ((f - best_f).clamp_min(0) * w).amax(dim=-1).mean(dim=0)


# -- LogEI family (acquisition/logei.py; utils/safe_math.py) -------------------------
TAU_RELU = 1e-6  # logei.py:66
TAU_MAX = 1e-2   # logei.py:67


def _softplus(x):
    """torch.nn.functional.softplus(x), beta = 1, threshold = 20."""
    return torch.where(x > 20, x, torch.log1p(torch.exp(x.clamp_max(20))))


def log_fatplus(z, tau):
    """safe_math.py:293-320: log(tau (softplus(z/tau) + 0.1 / (1 + (z/tau)^2)))."""
    x = z / tau
    return torch.log(tau * (_softplus(x) + 0.1 / (1 + x * x)))


def log_softplus(z, tau):
    """safe_math.py:226-247 (fp64: below z/tau = -35 the asymptote z/tau + log tau;
    above z/tau = 32 softplus is the identity)."""
    x = z / tau
    lo = x <= -35
    hi = x > 32
    mid = torch.log(tau * torch.log1p(torch.exp(x.clamp(-35, 32))))
    return torch.where(lo, x + math.log(tau), torch.where(hi, torch.log(z.abs().clamp_min(1e-300)), mid))


def fatmax(x, tau, dim=-1):
    """safe_math.py:323-352 with alpha = 2 (_pareto at :454-478 reduces to
    2 / (2 + 2y + y^2)), anchored at the maximum as _inf_max_helper (:149-187)."""
    M = x.amax(dim=dim, keepdim=True)
    y = (M - x) / tau
    return (M + tau * torch.log((2.0 / (2.0 + 2.0 * y + y * y)).sum(dim=dim, keepdim=True))).squeeze(dim)


def smooth_amax(x, tau, dim=-1):
    """safe_math.py:250-273: tau logsumexp(x / tau)."""
    return tau * torch.logsumexp(x / tau, dim=dim)


def logmeanexp(x, dim=0):
    """safe_math.py:209-223."""
    return torch.logsumexp(x, dim=dim) - math.log(x.shape[dim])


def qlogei_from_samples(samples, best_f, fat=True, tau_relu=TAU_RELU, tau_max=TAU_MAX):
    """qLogExpectedImprovement / qLogNEI reduction of S x b x q samples;
    best_f is a scalar or per-sample (S) tensor (logei.py:122, 219-234, 509-534)."""
    bf = torch.as_tensor(best_f, dtype=samples.dtype)
    if bf.ndim == 1:
        bf = bf.view(-1, *([1] * (samples.ndim - 1)))
    z = samples - bf
    li = log_fatplus(z, tau_relu) if fat else log_softplus(z, tau_relu)
    u = fatmax(li, tau_max) if fat else smooth_amax(li, tau_max)
    return logmeanexp(u, dim=0)


def qlogei(model: ExactGPOracle, X, Z, best_f, **kw):
    """qLogExpectedImprovement.forward on an exact GP."""
    mean, cov = model.posterior(X)
    return qlogei_from_samples(mc_samples(mean, cov, Z), best_f, **kw)


def qlognei(oracle: "QNEIOracle", X, **kw):
    """qLogNoisyExpectedImprovement (cache_root=True, logei.py:236-507): the
    cached-root qNEI samples against the per-sample baseline best."""
    return qlogei_from_samples(oracle.samples(X), oracle.best_f, **kw)


# -- qEHVI -----------------------------------------------------------------------
def qehvi_from_samples(obj, cell_lower, cell_upper):
    """qExpectedHypervolumeImprovement._compute_qehvi (multi_objective/
    monte_carlo.py:230-317): inclusion-exclusion over all nonempty q-subsets,
    per hypercell; obj is S x b x q x m.  Returns b."""
    S, b, q, m = obj.shape
    total = torch.zeros(S, b, cell_lower.shape[0], dtype=obj.dtype)
    for i in range(1, q + 1):
        idx = torch.tensor(list(itertools.combinations(range(q), i)), dtype=torch.long)
        sub = obj[:, :, idx.view(-1), :].view(S, b, idx.shape[0], i, m)
        ov = sub.min(dim=-2).values  # S x b x C x m
        ov = torch.minimum(ov.unsqueeze(-3), cell_upper.view(1, 1, -1, 1, m))
        lengths = (ov - cell_lower.view(1, 1, -1, 1, m)).clamp_min(0.0)
        areas = lengths.prod(dim=-1).sum(dim=-1)  # S x b x K
        total += (-1) ** (i + 1) * areas
    return total.sum(dim=-1).mean(dim=0)


def qehvi(models, X, Z, cell_lower, cell_upper):
    """ModelListGP posterior (independent outputs) + qEHVI.  Z is S x m x q
    (see sampling.base_samples_multi_output)."""
    samples = []
    for t, mdl in enumerate(models):
        mean, cov = mdl.posterior(X)
        samples.append(mc_samples(mean, cov, Z[:, t, :]))
    obj = torch.stack(samples, dim=-1)  # S x b x q x m
    return qehvi_from_samples(obj, cell_lower, cell_upper)


# -- qNEHVI (multi_objective/monte_carlo.py:325-468; utils/multi_objective/
#    hypervolume.py:507-835) ---------------------------------------------------------
def hypervolume(Y, ref):
    """Exact dominated hypervolume of the points Y (n x m, maximisation) above
    ref, m in {2, 3}, by slicing (an independent restatement of what
    DominatedPartitioning.compute_hypervolume returns, box_decompositions/
    dominated.py; pinned by tests/golden hv_* fixtures)."""
    Y = Y[(Y > ref).all(dim=-1)]
    if Y.shape[0] == 0:
        return Y.new_zeros(())
    m = Y.shape[-1]
    if m == 2:
        order = torch.argsort(Y[:, 0], descending=True)
        P = Y[order]
        best2 = torch.cummax(P[:, 1], dim=0).values
        x_next = torch.cat([P[1:, 0], ref[:1]])
        return ((P[:, 0] - x_next) * (best2 - ref[1])).sum()
    if m == 3:
        order = torch.argsort(Y[:, 2], descending=True)
        P = Y[order]
        z_next = torch.cat([P[1:, 2], ref[2:3]])
        total = Y.new_zeros(())
        for i in range(P.shape[0]):
            total = total + hypervolume(P[: i + 1, :2], ref[:2]) * (P[i, 2] - z_next[i])
        return total
    raise NotImplementedError("hypervolume oracle covers m = 2, 3")


class QNEHVIOracle:
    """qNoisyExpectedHypervolumeImprovement on a list of independent exact GPs
    with the cached baseline root (cache_root=True, incremental, no pending
    points): per MC sample s, the improvement of the new q points over the
    hypervolume dominated by f_s(X_baseline), averaged over samples.

    Base samples: the baseline draw has Sobol dimension r m (point-major,
    output-minor: z[s, i m + t]); the forward draw has dimension (r + q) m with
    its first r m columns replaced by the baseline draw
    (sampling/normal.py:68-131), so the new points use columns r m + p m + t."""

    def __init__(self, models, X_baseline, ref_point, S: int, seed: int):
        self.models = models
        self.Xb = X_baseline
        self.ref = torch.as_tensor(ref_point, dtype=torch.float64)
        self.S, self.seed = S, seed
        r, m = X_baseline.shape[0], len(models)
        self.Zb = draw_sobol_normal_samples(r * m, S, seed).view(S, r, m)
        self.L_rr, base = [], []
        for t, mdl in enumerate(models):
            mean_b, cov_b = mdl.posterior(X_baseline)
            Lb, _ = psd_safe_cholesky(cov_b)
            self.L_rr.append(Lb)
            base.append(mean_b.unsqueeze(0) + self.Zb[:, :, t] @ Lb.mT)
        self.Y_base = torch.stack(base, dim=-1)  # S x r x m
        self.initial_hv = torch.stack([hypervolume(self.Y_base[s], self.ref) for s in range(S)])

    def samples(self, X):
        """S x b x q x m joint samples at the new points."""
        b, q, d = X.shape
        r, m = self.Xb.shape[0], len(self.models)
        Zq = draw_sobol_normal_samples((r + q) * m, self.S, self.seed).view(self.S, r + q, m)[:, r:, :]
        out = []
        Xf = torch.cat([self.Xb.expand(b, r, d), X], dim=-2)
        for t, mdl in enumerate(self.models):
            mean, cov = mdl.posterior(Xf)
            bottom = cov[..., -q:, :]
            bl = torch.linalg.solve_triangular(self.L_rr[t], bottom[..., :r].mT, upper=False).mT
            br_chol, _ = psd_safe_cholesky(bottom[..., r:] - bl @ bl.mT)
            f = (mean[..., -q:].unsqueeze(0) + torch.einsum("bir,sr->sbi", bl, self.Zb[:, :, t])
                 + torch.einsum("bij,sj->sbi", br_chol, Zq[:, :, t]))
            out.append(f)
        return torch.stack(out, dim=-1)

    def samples_joint(self, X):
        """cache_root=False (monte_carlo.py:444-468, cached_cholesky.py:161-165):
        the joint posterior over [X_baseline; X] of each t-batch, its own
        psd_safe_cholesky, base samples with the baseline draw in the leading
        r columns; the new rows.  S x b x q x m."""
        b, q, d = X.shape
        r, m = self.Xb.shape[0], len(self.models)
        Zq = draw_sobol_normal_samples((r + q) * m, self.S, self.seed).view(self.S, r + q, m)[:, r:, :]
        Xf = torch.cat([self.Xb.expand(b, r, d), X], dim=-2)
        out = []
        for t, mdl in enumerate(self.models):
            mean, cov = mdl.posterior(Xf)
            L, _ = psd_safe_cholesky(cov)
            z = torch.cat([self.Zb[:, :, t], Zq[:, :, t]], dim=-1)   # S x (r + q)
            f = mean.unsqueeze(0) + torch.einsum("bij,sj->sbi", L, z)
            out.append(f[..., r:])
        return torch.stack(out, dim=-1)

    def value_cells_joint(self, X, cell_lo, cell_hi):
        f = self.samples_joint(X)
        vals = [qehvi_from_samples(f[s:s + 1], cell_lo[s], cell_hi[s]) for s in range(f.shape[0])]
        return torch.stack(vals, dim=0).mean(dim=0)

    def value_exact(self, X):
        """mean_s [HV(front_s + new points) - HV(front_s)] by exact hypervolumes."""
        f = self.samples(X).detach()
        S, b = f.shape[0], f.shape[1]
        res = torch.zeros(b, dtype=torch.float64)
        for j in range(b):
            acc = 0.0
            for s in range(S):
                acc += (hypervolume(torch.cat([self.Y_base[s], f[s, j]]), self.ref) - self.initial_hv[s]).item()
            res[j] = acc / S
        return res

    def value_cells(self, X, cell_lo, cell_hi):
        """The same quantity through per-sample hypercells (S x K x m; the
        inclusion-exclusion of qehvi_from_samples per sample), differentiable."""
        f = self.samples(X)  # S x b x q x m
        vals = [qehvi_from_samples(f[s:s + 1], cell_lo[s], cell_hi[s]) for s in range(f.shape[0])]
        return torch.stack(vals, dim=0).mean(dim=0)


def saas_members(train_X, train_Y, mcmc_samples, standardize=False):
    """SaasFullyBayesianSingleTaskGP.load_mcmc_samples (models/fully_bayesian.py:
    267-312): one Matern-5/2 x outputscale exact GP per MCMC sample, noise
    clamped at 1e-4."""
    from .gp import MATERN52, GPHyper
    out = []
    for i in range(len(mcmc_samples["mean"])):
        h = GPHyper(mcmc_samples["lengthscale"][i].double().reshape(-1),
                    max(float(mcmc_samples["noise"][i]), 1e-4), float(mcmc_samples["mean"][i]),
                    float(mcmc_samples["outputscale"][i]), MATERN52)
        out.append(ExactGPOracle(train_X, train_Y, h, standardize=standardize))
    return out


def saas_qei(members, X, Z, best_f):
    """qEI on the b x M mixture posterior (fully_bayesian.py:509-546), averaged
    over MCMC_DIM by t_batch_mode_transform (utils/transforms.py:289-293)."""
    return torch.stack([qei(m, X, Z, best_f) for m in members], dim=-1).mean(dim=-1)
