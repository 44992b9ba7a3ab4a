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
def compute_feasibility_indicator(constraints: Optional[List[Callable]], samples: torch.Tensor,
                                  marginalize_dim: Optional[int] = None) -> torch.Tensor:
    """utils/objective.py:101-131: Boolean feasibility (all constraints <= 0)."""
    ind = torch.ones(samples.shape[:-1], dtype=torch.bool, device=samples.device)
    if constraints is not None:
        for constraint in constraints:
            ind = ind.logical_and(constraint(samples) <= 0)
    if ind.ndim >= 3 and marginalize_dim is not None:
        if marginalize_dim < 0:
            marginalize_dim = 1 + (marginalize_dim % ind.ndim)
        ind = ind.float().mean(dim=marginalize_dim).round().bool()
    return ind


def compute_smoothed_feasibility_indicator(constraints: List[Callable], samples: torch.Tensor,
                                           eta: Union[torch.Tensor, float], log: bool = False,
                                           fat: bool = False) -> torch.Tensor:
    """utils/objective.py:134-180: prod_i sigmoid(-c_i(samples) / eta_i) (or its
    log, or the fat-tailed fatmoid form)."""
    if type(eta) is not torch.Tensor:
        eta = torch.full((len(constraints),), eta)
    if len(eta) != len(constraints):
        raise ValueError("Number of provided constraints and number of provided etas do not match.")
    if not (eta > 0).all():
        raise ValueError("eta must be positive.")
    is_feasible = torch.zeros_like(samples[..., 0])
    log_sigmoid = log_fatmoid if fat else logexpit
    for constraint, e in zip(constraints, eta):
        is_feasible = is_feasible + log_sigmoid(-constraint(samples) / e.to(samples))
    return is_feasible if log else is_feasible.exp()


def get_infeasible_cost(X: torch.Tensor, model, objective=None, posterior_transform=None):
    """acquisition/utils.py:203-242: M with -M < min_x f(x) (6-sigma lower bound)."""
    if objective is None:
        def objective(Y, X=None):
            return Y.squeeze(-1)
    with torch.no_grad():
        posterior = model.posterior(X, posterior_transform=posterior_transform)
        lb = objective(posterior.mean - 6 * posterior.variance.clamp_min(0).sqrt(), X=X)
    if lb.ndim < posterior.mean.ndim:
        lb = lb.unsqueeze(-1)
    while lb.dim() > 1:
        lb = lb.min(dim=-2).values
    return -(lb.clamp_max(0.0))


def _estimate_objective_lower_bound(model, objective, posterior_transform, X: torch.Tensor):
    """acquisition/utils.py:166-200: -M over 32 random convex combinations of X."""
    w = torch.rand(32, X.shape[-2], dtype=X.dtype, device=X.device)
    w = w / w.sum(dim=0, keepdim=True)
    return -get_infeasible_cost(X=w @ X, model=model, objective=objective,
                                posterior_transform=posterior_transform)


def compute_best_feasible_objective(samples: torch.Tensor, obj: torch.Tensor,
                                    constraints: Optional[List[Callable]], model=None,
                                    objective=None, posterior_transform=None,
                                    X_baseline: Optional[torch.Tensor] = None,
                                    infeasible_obj: Optional[torch.Tensor] = None) -> torch.Tensor:
    """acquisition/utils.py:90-163: max over q of the feasible objective values
    (infeasible entries replaced by -inf, or by a model-based lower bound when a
    sample has no feasible point at all)."""
    if constraints is None:
        with torch.no_grad():
            return obj.amax(dim=-1, keepdim=False)
    is_feasible = compute_feasibility_indicator(constraints=constraints, samples=samples)
    if is_feasible.any(dim=-1).all():
        infeasible_value = -torch.inf
    elif infeasible_obj is not None:
        infeasible_value = infeasible_obj.item()
    else:
        if model is None:
            raise ValueError("Must specify `model` when no feasible observation exists.")
        if X_baseline is None:
            raise ValueError("Must specify `X_baseline` when no feasible observation exists.")
        infeasible_value = _estimate_objective_lower_bound(model=model, objective=objective,
                                                           posterior_transform=posterior_transform,
                                                           X=X_baseline).item()
    is_feasible = repeat_to_match_aug_dim(is_feasible, obj)
    obj = torch.where(is_feasible, obj, infeasible_value)
    with torch.no_grad():
        return obj.amax(dim=-1, keepdim=False)
