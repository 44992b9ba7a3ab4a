"""Pareto front and non-dominated box decomposition (setup side of qEHVI).

Restates botorch/utils/multi_objective/pareto.py:16-64 (is_non_dominated) and
box_decompositions/{non_dominated.py:353-457, box_decomposition.py, utils.py}
(FastNondominatedPartitioning: Alg. 1 of Lacour et al. 2017 applied twice, as
in Yang et al. 2019; the direct sweep for m = 2).  Runs once per acquisition
function on the host, like the reference; the hot path consumes only the
resulting hypercell bounds.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch


def is_non_dominated(Y: torch.Tensor, maximize: bool = True, deduplicate: bool = True) -> torch.Tensor:
    """pareto.py:16-64: device fp64 inputs run bo_pareto_mask (any batch
    shape, m <= 8, one launch); host inputs the pairwise torch form (the loop
    form beyond n = 2000, as the reference)."""
    n = Y.shape[-2]
    if n == 0:
        return torch.zeros(Y.shape[:-1], dtype=torch.bool, device=Y.device)
    if Y.is_cuda and Y.dtype == torch.float64 and Y.shape[-1] <= 8:
        from . import kernels
        return kernels.pareto_mask(Y, maximize, deduplicate)
    if n > 2000:
        return _is_non_dominated_loop(Y, maximize, deduplicate)
    Y1 = Y.unsqueeze(-3)
    Y2 = Y.unsqueeze(-2)
    if maximize:
        dominates = (Y1 >= Y2).all(dim=-1) & (Y1 > Y2).any(dim=-1)
    else:
        dominates = (Y1 <= Y2).all(dim=-1) & (Y1 < Y2).any(dim=-1)
    nd_mask = ~(dominates.any(dim=-1))
    if deduplicate:
        indices = (Y1 == Y2).all(dim=-1).long().argmax(dim=-1)
        keep = torch.zeros_like(nd_mask)
        keep.scatter_(dim=-1, index=indices, value=1.0)
        return nd_mask & keep
    return nd_mask


def _is_non_dominated_loop(Y, maximize=True, deduplicate=True):
    is_efficient = torch.ones(Y.shape[:-1], dtype=torch.bool, device=Y.device)
    for i in range(Y.shape[-2]):
        vals = Y[..., i:i + 1, :]
        if maximize:
            update = (Y > vals).any(dim=-1)
        else:
            update = (Y < vals).any(dim=-1)
        if not deduplicate:
            update = update | (Y == vals).all(dim=-1)
        update[..., i] = True
        is_efficient = is_efficient & (update | ~is_efficient[..., i:i + 1])
    return is_efficient


class FastNondominatedPartitioning:
    """box_decompositions/non_dominated.py:353-457 (maximisation)."""

    def __init__(self, ref_point: torch.Tensor, Y: Optional[torch.Tensor] = None):
        self.ref_point = ref_point.to(torch.float64)
        self.num_outcomes = ref_point.shape[-1]
        self.Y = None
        if Y is not None:
            self.update(Y)

    def update(self, Y: torch.Tensor) -> None:
        Y = Y.to(torch.float64).to(self.ref_point.device)
        self.Y = Y if self.Y is None else torch.cat([self.Y, Y], dim=-2)
        mask = is_non_dominated(self.Y) & (self.Y > self.ref_point).all(dim=-1)
        pareto = self.Y[mask]
        if self.num_outcomes == 2:
            pareto = pareto[torch.argsort(pareto[:, 0])]
        self.pareto_Y = pareto
        self._partition()

    def _partition(self) -> None:
        """Lacour17 (utils.py:103-288) in native host code: bo_nd_partition_host."""
        from . import kernels
        lo, hi = kernels.nd_partition_host(self.Y, self.ref_point.cpu())
        dev = self.ref_point.device
        self.hypercell_bounds = torch.stack([lo, hi]).to(dev)

    def get_hypercell_bounds(self) -> torch.Tensor:
        return self.hypercell_bounds

    def compute_hypervolume(self) -> torch.Tensor:
        """non_dominated.py:442-457."""
        if self.pareto_Y.shape[0] == 0:
            return torch.tensor(0.0, dtype=torch.float64)
        ideal = self.pareto_Y.max(dim=-2, keepdim=True).values
        total = (ideal.squeeze(-2) - self.ref_point).clamp_min(0.0).prod(dim=-1)
        finite = torch.min(self.hypercell_bounds, ideal)
        non_dom = (finite[1] - finite[0]).clamp_min(0.0).prod(dim=-1).sum(dim=-1)
        return total - non_dom


NondominatedPartitioning = FastNondominatedPartitioning
