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
    """pareto.py:16-64 (pairwise form; n x m, no batch)."""
    n = Y.shape[-2]
    if n == 0:
        return torch.zeros(Y.shape[:-1], dtype=torch.bool, device=Y.device)
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


def _local_upper_bounds(U, Z, z):
    """utils.py:103-162 (Lacour17 Alg. 1, minimisation): update local upper
    bounds U (k x m) and defining points Z (k x m x m) with the point z."""
    m = U.shape[-1]
    z_dom = (U > z).all(dim=-1)
    if not z_dom.any():
        return U, Z
    A = U[z_dom]
    A_Z = Z[z_dom]
    P, P_Z = [], []
    mask = torch.ones(m, dtype=torch.bool, device=U.device)
    for j in range(m):
        mask[j] = 0
        z_uj_max = A_Z[:, mask, j].max(dim=-1).values.view(-1)
        add_z = z[j] >= z_uj_max
        if add_z.any():
            u_j = A[add_z].clone()
            u_j[:, j] = z[j]
            P.append(u_j)
            Z_ku = A_Z[add_z][:, mask]
            lt_zj = Z_ku[..., j] <= z[j]
            P_uj = torch.zeros(u_j.shape[0], m, m, dtype=U.dtype, device=U.device)
            P_uj[:, mask] = Z_ku[lt_zj].view(P_uj.shape[0], m - 1, -1)
            P_uj[:, ~mask] = z
            P_Z.append(P_uj)
        mask[j] = 1
    keep = ~z_dom
    U, Z = U[keep], Z[keep]
    if P:
        Z = torch.cat([Z, *P_Z], dim=0)
        U = torch.cat([U, *P], dim=-2)
    return U, Z


def _partition_bounds(Z, U, ref_point):
    """utils.py:165-195 (Lacour17 Eq. 2)."""
    k, m = U.shape
    lo = torch.empty(k, m, dtype=U.dtype, device=U.device)
    hi = torch.empty(k, m, dtype=U.dtype, device=U.device)
    lo[:, 0] = Z[:, 0, 0]
    hi[:, 0] = ref_point[0]
    for j in range(1, m):
        lo[:, j] = Z[:, :j, j].max(dim=-1).values
        hi[:, j] = U[:, j]
    empty = (hi <= lo).any(dim=-1)
    return torch.stack([lo[~empty], hi[~empty]])


def _nd_cells_2d(pareto_sorted, ref_point):
    """utils.py:222-288 (m = 2, pareto sorted by objective 0 ascending)."""
    inf = torch.tensor(float("inf"), dtype=pareto_sorted.dtype, device=pareto_sorted.device)
    left = torch.stack([ref_point[0], pareto_sorted[0, 1]]).unsqueeze(0)
    right = torch.stack([pareto_sorted[-1, 0], ref_point[1]]).unsqueeze(0)
    front = torch.cat([left, pareto_sorted, right], dim=0)
    bottom_lefts = torch.stack([front[:-1, 0], front[1:, 1]], dim=-1)
    top_x = torch.cat([front[1:-1, 0], inf.view(1)])
    top_rights = torch.stack([top_x, inf.expand_as(top_x)], dim=-1)
    return torch.stack([bottom_lefts, top_rights])


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
        m = self.num_outcomes
        dev, dt = self.ref_point.device, self.ref_point.dtype
        if self.pareto_Y.shape[0] == 0:
            b = torch.full((2, 1, m), float("inf"), dtype=dt, device=dev)
            b[0] = self.ref_point
            self.hypercell_bounds = b
            return
        if m == 2:
            self.hypercell_bounds = _nd_cells_2d(self.pareto_Y, self.ref_point)
            return
        neg_ref = -self.ref_point
        U = neg_ref.unsqueeze(0).clone()
        Z = torch.zeros(1, m, m, dtype=dt, device=dev)
        for j in range(m):
            Z[0, j] = float("-inf")
            Z[0, j, j] = U[0, j]
        for z in -self.pareto_Y:
            U, Z = _local_upper_bounds(U, Z, z)
        # second pass: -U as a new front for minimisation with reference +inf
        U2 = torch.full((1, m), float("inf"), dtype=dt, device=dev)
        Z2 = self.ref_point.expand(1, m, m).clone()
        for j in range(m):
            Z2[0, j, j] = U2[0, j]
        for z in -U:
            U2, Z2 = _local_upper_bounds(U2, Z2, z)
        self.hypercell_bounds = _partition_bounds(Z2, U2, U2.new_full((m,), float("inf")))

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
