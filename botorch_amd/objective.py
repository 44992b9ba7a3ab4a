"""MC objectives, posterior transforms and outcome-constraint helpers of the
acquisition path (botorch/acquisition/objective.py, botorch/utils/objective.py,
botorch/acquisition/utils.py:90-243).

Constraints are arbitrary Python callables on posterior samples, so they are
applied to device tensors by torch on the generic acquisition route (the
samples themselves come from the gfx950 posterior and sampling kernels).
"""
from __future__ import annotations

from typing import Callable, List, Optional, Union

import torch
from torch import nn

from .safe_math import log_fatmoid, logexpit


class MCAcquisitionObjective(nn.Module):
    """acquisition/objective.py:230-285 (callable on samples, optional X)."""

    _verify_output_shape = True

    def forward(self, samples: torch.Tensor, X: Optional[torch.Tensor] = None) -> torch.Tensor:
        raise NotImplementedError


MCObjective = MCAcquisitionObjective


class IdentityMCObjective(MCAcquisitionObjective):
    """acquisition/objective.py:288-298: drop the (single) output dimension."""

    def forward(self, samples, X=None):
        return samples.squeeze(-1)


class GenericMCObjective(MCAcquisitionObjective):
    """acquisition/objective.py:344-382: ``objective(samples, X=X)``."""

    def __init__(self, objective: Callable[..., torch.Tensor]) -> None:
        super().__init__()
        self.objective = objective

    def forward(self, samples, X=None):
        return self.objective(samples, X=X)


class ConstrainedMCObjective(GenericMCObjective):
    """acquisition/objective.py:385-466 (legacy outcome constraints): the
    objective shifted by ``infeasible_cost``, clamped at 0, weighted by the
    smoothed feasibility indicator, shifted back (utils/objective.py:52-98, 183-232)."""

    def __init__(self, objective, constraints, infeasible_cost=0.0, eta=1e-3) -> None:
        super().__init__(objective=objective)
        self.constraints = constraints
        if type(eta) is not torch.Tensor:
            eta = torch.full((len(constraints),), eta)
        self.register_buffer("eta", eta)
        self.register_buffer("infeasible_cost", torch.as_tensor(infeasible_cost))

    def forward(self, samples, X=None):
        obj = super().forward(samples=samples) + self.infeasible_cost.to(samples)
        w = compute_smoothed_feasibility_indicator(self.constraints, samples, self.eta)
        if obj.dim() == samples.dim():
            w = w.unsqueeze(-1)
        return obj.clamp_min(0).mul(w) - self.infeasible_cost.to(samples)


class LinearMCObjective(MCAcquisitionObjective):
    """acquisition/objective.py:301-341: weights . samples over the outputs."""

    def __init__(self, weights: torch.Tensor) -> None:
        super().__init__()
        if weights.dim() != 1:
            raise ValueError("weights must be a one-dimensional tensor.")
        self.register_buffer("weights", weights)

    def forward(self, samples, X=None):
        if samples.shape[-1] != self.weights.shape[-1]:
            raise RuntimeError("Output shape of samples not equal to that of weights")
        return torch.einsum("...m, m", [samples, self.weights.to(samples)])


class ScalarizedPosteriorTransform(nn.Module):
    """acquisition/objective.py:75-129: w^T f + offset of a (multi-output)
    Gaussian posterior, as a single-output Gaussian posterior.  For a list of
    independent outputs (ModelListGP) the scalarised covariance is
    sum_t w_t^2 Sigma_t (posteriors/posterior_list.py + utils/transforms)."""

    scalarize = True

    def __init__(self, weights: torch.Tensor, offset: float = 0.0) -> None:
        super().__init__()
        if weights.dim() != 1:
            raise ValueError("weights must be a one-dimensional tensor.")
        self.register_buffer("weights", weights)
        self.offset = offset

    def evaluate(self, Y: torch.Tensor) -> torch.Tensor:
        return self.offset + Y @ self.weights.to(Y)

    def forward(self, posterior):
        from .posteriors import GPyTorchPosterior, MultivariateNormal, PosteriorList
        parts = posterior.posteriors if isinstance(posterior, PosteriorList) else [posterior]
        if len(parts) != self.weights.shape[0]:
            raise RuntimeError("Output shape of samples not equal to that of weights")
        mean, cov = None, None
        for w, p in zip(self.weights.tolist(), parts):
            mvn = p.distribution
            m_t = w * mvn.mean
            c_t = (w * w) * mvn.covariance_matrix
            mean = m_t if mean is None else mean + m_t
            cov = c_t if cov is None else cov + c_t
        return GPyTorchPosterior(MultivariateNormal(mean + self.offset, cov),
                                 model=getattr(parts[0], "model", None), X=getattr(parts[0], "X", None))


def repeat_to_match_aug_dim(target_tensor: torch.Tensor, reference_tensor: torch.Tensor):
    """acquisition/utils.py:44-87: repeat along dim 0 to the augmented sample size."""
    aug, rem = divmod(reference_tensor.shape[0], target_tensor.shape[0])
    if rem != 0:
        raise ValueError("The first dimension of the reference tensor must be a multiple "
                         "of that of the target tensor.")
    if aug > 1:
        return target_tensor.repeat(aug, *[1] * (target_tensor.ndim - 1))
    return target_tensor


# -- outcome constraints --------------------------------------------------------------
# The reference's helpers (utils/objective.py:101-180, acquisition/utils.py:
# 90-242) are restated here around one primitive: every constraint evaluated
# once on the samples and stacked on a leading constraint axis.  Hard
# feasibility, the smoothed (log-)indicator and the best feasible objective
# are reductions over that axis.  Pinned by tests/test_objective_cpu.py
# against the reference's own outputs (golden.npz ``feas_*``).
def _constraint_stack(constraints: List[Callable], samples: torch.Tensor) -> torch.Tensor:
    """c x samples.shape[:-1]: constraint i's values in row i (<= 0 feasible)."""
    shape = samples.shape[:-1]
    return torch.stack([torch.as_tensor(c(samples)).to(samples.device).expand(shape)
                        for c in constraints])


def _majority(ind: torch.Tensor, dim: int) -> torch.Tensor:
    """Feasible in at least half of the entries along ``dim`` (rounded mean).
    A negative ``dim`` counts from the first batch dimension, as the
    reference's ``1 + (dim % ndim)`` does."""
    if dim < 0:
        dim = dim % ind.ndim + 1
    return ind.to(torch.float32).mean(dim=dim).round().to(torch.bool)


def compute_feasibility_indicator(constraints: Optional[List[Callable]], samples: torch.Tensor,
                                  marginalize_dim: Optional[int] = None) -> torch.Tensor:
    """utils/objective.py:101-131: True where every constraint is <= 0 (all
    True without constraints); with ``marginalize_dim`` (3+-dim indicators)
    the majority vote along it."""
    if constraints:
        ind = (_constraint_stack(constraints, samples) <= 0).all(dim=0)
    else:
        ind = torch.ones(samples.shape[:-1], dtype=torch.bool, device=samples.device)
    if marginalize_dim is not None and ind.ndim >= 3:
        ind = _majority(ind, marginalize_dim)
    return ind


def _as_etas(eta: Union[torch.Tensor, float], count: int) -> torch.Tensor:
    etas = eta if torch.is_tensor(eta) else torch.full((count,), float(eta))
    if len(etas) != count:
        raise ValueError("Number of provided constraints and number of provided etas do not match.")
    if not bool((etas > 0).all()):
        raise ValueError("eta must be positive.")
    return etas


def compute_smoothed_feasibility_indicator(constraints: List[Callable], samples: torch.Tensor,
                                           eta: Union[torch.Tensor, float], log: bool = False,
                                           fat: bool = False) -> torch.Tensor:
    """utils/objective.py:134-180: the product over constraints of
    sigmoid(-c_i / eta_i) (fatmoid with ``fat``), summed in log space in the
    constraints' order; its log with ``log``."""
    etas = _as_etas(eta, len(constraints))
    log_sig = log_fatmoid if fat else logexpit
    vals = _constraint_stack(constraints, samples)
    total = torch.zeros_like(samples[..., 0])
    for i in range(vals.shape[0]):  # in order: the same rounding as a running sum
        total = total + log_sig(-vals[i] / etas[i].to(samples))
    return total if log else total.exp()


def get_infeasible_cost(X: torch.Tensor, model, objective=None, posterior_transform=None):
    """acquisition/utils.py:203-242: M >= 0 with -M below the objective's
    6-sigma lower bound over X (one entry per output of the objective)."""
    with torch.no_grad():
        post = model.posterior(X, posterior_transform=posterior_transform)
        lower = post.mean - 6.0 * post.variance.clamp_min(0).sqrt()
        lb = lower.squeeze(-1) if objective is None else objective(lower, X=X)
    if lb.ndim < post.mean.ndim:
        lb = lb.unsqueeze(-1)
    lb = lb.reshape(-1, lb.shape[-1]).amin(dim=0) if lb.ndim > 1 else lb
    return lb.clamp_max(0.0).neg()


def _estimate_objective_lower_bound(model, objective, posterior_transform, X: torch.Tensor):
    """acquisition/utils.py:166-200: the lower bound over 32 random convex
    combinations of the rows of X."""
    mix = torch.rand(32, X.shape[-2], dtype=X.dtype, device=X.device)
    mix = mix / mix.sum(dim=0, keepdim=True)
    return get_infeasible_cost(X=mix @ X, model=model, objective=objective,
                               posterior_transform=posterior_transform).neg()


def compute_best_feasible_objective(samples: torch.Tensor, obj: torch.Tensor,
                                    constraints: Optional[List[Callable]], model=None,
                                    objective=None, posterior_transform=None,
                                    X_baseline: Optional[torch.Tensor] = None,
                                    infeasible_obj: Optional[torch.Tensor] = None) -> torch.Tensor:
    """acquisition/utils.py:90-163: the best objective value over the q points
    counting only feasible ones.  An infeasible entry counts as -inf when every
    sample has a feasible point, else as ``infeasible_obj`` or the model's
    lower bound over ``X_baseline``."""
    if constraints is not None:
        feas = compute_feasibility_indicator(constraints=constraints, samples=samples)
        if bool(feas.any(dim=-1).all()):
            fill = -torch.inf
        elif infeasible_obj is not None:
            fill = infeasible_obj.item()
        elif model is None:
            raise ValueError("Must specify `model` when no feasible observation exists.")
        elif X_baseline is None:
            raise ValueError("Must specify `X_baseline` when no feasible observation exists.")
        else:
            fill = _estimate_objective_lower_bound(model=model, objective=objective,
                                                   posterior_transform=posterior_transform,
                                                   X=X_baseline).item()
        obj = obj.where(repeat_to_match_aug_dim(feas, obj), torch.as_tensor(fill, dtype=obj.dtype,
                                                                            device=obj.device))
    with torch.no_grad():
        return obj.amax(dim=-1)
