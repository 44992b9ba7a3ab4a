"""Linear parameter constraints for the optimiser callers.

Two pieces of the reference's constrained ``optimize_acqf``:

* scipy constraint records for SLSQP candidate generation
  (botorch/optim/parameter_constraints.py:29-312, 412-471), used by
  ``optim.gen_candidates_scipy`` (generation/gen.py:124-189, 256);
* raw-sample designs drawn uniformly from the feasible polytope by a
  hit-and-run Markov chain (botorch/utils/sampling.py:219-309, 356-704,
  828-985; optim/initializers.py:72-240), used by
  ``optim.gen_batch_initial_conditions`` (initializers.py:365-375).

A constraint is the reference's sparse triple ``(indices, coefficients, rhs)``:
``sum_i X[..., indices[i]] * coefficients[i] >= rhs`` (inequality) or ``== rhs``
(equality).  1-d ``indices`` apply to every point of a q-batch (intra-point);
a ``c x 2`` tensor of (point, feature) pairs couples points of one q-batch
(inter-point).

The chain's steps run in native host code (``bo_hit_and_run_host``): they are
one dependent step after another, a few hundred flops each, which the
reference runs as a Python loop on the CPU.  Every random number it consumes
is drawn here with torch, in the reference's order and under the reference's
seeds, so a seeded draw reproduces the reference's samples (to rounding:
``A y`` is summed in a fixed order instead of by BLAS).
"""
from __future__ import annotations

import ctypes
import warnings
from typing import List, Optional, Tuple

import numpy as np
import scipy.optimize
import torch
from scipy.optimize import Bounds

from .exceptions import BotorchError, CandidateGenerationError, UnsupportedError, UserInputWarning
from .utils_sampling import manual_seed

Constraint = Tuple[torch.Tensor, torch.Tensor, float]


# ---- scipy records (parameter_constraints.py) ----------------------------------------

def _as_numpy(X: torch.Tensor) -> np.ndarray:
    """parameter_constraints.py:168-177: a detached host float64 copy."""
    return X.detach().cpu().contiguous().double().clone().numpy()


def make_scipy_bounds(X: torch.Tensor, lower_bounds=None, upper_bounds=None) -> Optional[Bounds]:
    """parameter_constraints.py:29-65: column bounds broadcast over X and
    flattened; a missing side is -inf / +inf; None when both are missing."""
    if lower_bounds is None and upper_bounds is None:
        return None

    def side(v, fill):
        if v is None:
            full = torch.full_like(X, fill)
        else:
            full = (v if torch.is_tensor(v) else torch.tensor(v)).expand_as(X)
        return _as_numpy(full).reshape(-1)

    return Bounds(lb=side(lower_bounds, float("-inf")), ub=side(upper_bounds, float("inf")),
                  keep_feasible=True)


def _lin_value(x: np.ndarray, flat_idx, coeffs: np.ndarray, rhs: float):
    """parameter_constraints.py:131-145."""
    return np.sum(x[flat_idx] * coeffs, -1) - rhs


def _lin_jacobian(x: np.ndarray, flat_idx, coeffs: np.ndarray, n: int) -> np.ndarray:
    """parameter_constraints.py:148-165 (dense row)."""
    row = np.zeros(n)
    row[flat_idx] = coeffs
    return row


def _bqd(shapeX) -> Tuple[int, int, int]:
    """parameter_constraints.py:180-195: (b) x q x d, b = 1 when absent."""
    if len(shapeX) not in (2, 3):
        raise UnsupportedError(f"`shapeX` must be `(b) x q x d` (at least two-dimensional). It is "
                               f"{shapeX}.")
    return (1, *shapeX) if len(shapeX) == 2 else tuple(shapeX)


def _check_indices(indices: torch.Tensor, q: int, d: int) -> None:
    """parameter_constraints.py:198-213."""
    if indices.dim() > 2:
        raise UnsupportedError("Linear constraints supported only on individual candidates and "
                               "across q-batches, not across general batch shapes.")
    if indices.dim() == 0:
        raise ValueError("`indices` must be at least one-dimensional")
    if indices.dim() == 2 and indices[:, 0].max() > q - 1:
        raise RuntimeError(f"Index out of bounds for {q}-batch")
    feat = indices[:, 1] if indices.dim() == 2 else indices
    if feat.max() > d - 1:
        raise RuntimeError(f"Index out of bounds for {d}-dim parameter tensor")


def _constraint_records(indices, coefficients, rhs, shapeX, eq: bool) -> List[dict]:
    """parameter_constraints.py:216-312: one scipy record per t-batch (2-d
    indices) or per t-batch and q-batch point (1-d indices), in that order;
    x is X flattened row-major, so X[i, j, k] sits at i q d + j d + k."""
    b, q, d = _bqd(shapeX)
    _check_indices(indices, q, d)
    n = b * q * d
    coeffs = _as_numpy(coefficients)
    kind = "eq" if eq else "ineq"
    rhs = float(rhs)
    if indices.dim() == 2:
        within = [int(p) * d + int(f) for p, f in indices.tolist()]
        slots = [[i * q * d + o for o in within] for i in range(b)]
    else:
        feats = indices.tolist()
        slots = [[i * q * d + j * d + f for f in feats] for i in range(b) for j in range(q)]
    recs = []
    for idx in slots:
        recs.append({
            "type": kind,
            "fun": (lambda x, _i=idx: _lin_value(x, _i, coeffs, rhs)),
            "jac": (lambda x, _i=idx: _lin_jacobian(x, _i, coeffs, n)),
        })
    return recs


def make_scipy_linear_constraints(shapeX, inequality_constraints=None,
                                  equality_constraints=None) -> List[dict]:
    """parameter_constraints.py:68-128: the inequality records, then the
    equality records, each constraint broadcast over the t-batches."""
    recs: List[dict] = []
    for group, eq in ((inequality_constraints, False), (equality_constraints, True)):
        for indices, coefficients, rhs in group or []:
            recs += _constraint_records(indices, coefficients, rhs, shapeX, eq)
    return recs


def _generate_unfixed_lin_constraints(constraints, fixed_features: dict, dimension: int,
                                      eq: bool):
    """parameter_constraints.py:412-471: the constraints on the free features
    only.  A fixed feature's term moves to the right-hand side; the remaining
    feature indices are renumbered over the free features; a constraint with no
    free term left must hold as it stands (CandidateGenerationError)."""
    if not constraints:
        return constraints
    free = [k for k in range(dimension) if k not in fixed_features]
    renumber = {k: pos for pos, k in enumerate(free)}
    out = []
    for cid, (indices, coefficients, rhs) in enumerate(constraints):
        rows = indices if indices.ndim == 2 else indices.unsqueeze(-1)
        keep_rows, keep_coefs, rhs_new = [], [], rhs
        for coef, row in zip(coefficients, rows):
            val = fixed_features.get(row[-1].item())
            if val is None:
                keep_rows.append(row)
                keep_coefs.append(coef)
            else:
                rhs_new = rhs_new - coef.item() * val
        if not keep_rows:
            if (eq and rhs_new != 0) or (not eq and rhs_new > 0):
                raise CandidateGenerationError(f"{'Eq' if eq else 'Ineq'}uality constraint {cid} "
                                               "not met with fixed_features.")
            continue
        idx = torch.stack(keep_rows, dim=0)
        idx[:, -1] = torch.tensor([renumber[int(v)] for v in idx[:, -1].tolist()]).to(idx)
        out.append((idx.squeeze(-1), torch.stack(keep_coefs), rhs_new))
    return out


# ---- dense forms and the polytope (utils/sampling.py) ----------------------------------

def sparse_to_dense_constraints(d: int, constraints) -> Tuple[torch.Tensor, torch.Tensor]:
    """sampling.py:957-985: rows A (n_con x d) and right-hand sides b (n_con x 1)."""
    like = constraints[0][1]
    A = torch.zeros(len(constraints), d, dtype=like.dtype, device=like.device)
    b = torch.zeros(len(constraints), 1, dtype=like.dtype, device=like.device)
    for row, (indices, coefficients, rhs) in enumerate(constraints):
        A[row, indices.long()] = coefficients
        b[row] = rhs
    return A, b


def normalize_dense_linear_constraints(bounds: torch.Tensor, constraints):
    """sampling.py:859-879: A x <= b over the box becomes A' z <= b' over the
    unit cube (x = lower + (upper - lower) z)."""
    lower, upper = bounds
    A, b = constraints
    return (upper - lower) * A, b - (A @ lower).unsqueeze(-1)


def normalize_sparse_linear_constraints(bounds: torch.Tensor, constraints):
    """sampling.py:828-856 (intra-point constraints only)."""
    out = []
    for indices, coefficients, rhs in constraints:
        if indices.ndim != 1:
            raise ValueError(
                "`indices` must be a one-dimensional tensor. This method does not support the "
                "kind of 'inter-point constraints' that are supported by `optimize_acqf()`. To "
                "achieve this behavior, you need define the problem on the joint space over `q` "
                "points and impose use constraints, see "
                "https://github.com/pytorch/botorch/issues/2468#issuecomment-2287706461")
        lower, upper = bounds[:, indices]
        out.append((indices, (upper - lower) * coefficients,
                    (rhs - torch.dot(coefficients, lower)).item()))
    return out


def _box_as_inequalities(bounds: torch.Tensor):
    """sampling.py:356-373: -x <= -lower for the finite lower bounds, then
    x <= upper for the finite upper bounds."""
    d = bounds.shape[-1]
    eye = torch.eye(d, dtype=bounds.dtype, device=bounds.device)
    lower, upper = bounds
    fl, fu = bounds.isfinite()
    return (torch.cat([-eye[fl], eye[fu]], dim=0),
            torch.cat([-lower[fl], upper[fu]], dim=0).unsqueeze(-1))


def find_interior_point(A: np.ndarray, b: np.ndarray, A_eq: Optional[np.ndarray] = None,
                        b_eq: Optional[np.ndarray] = None) -> np.ndarray:
    """sampling.py:376-454: the LP  max s  s.t.  A x + 2 s <= b, s >= 0,
    A_eq x = b_eq  (HiGHS); an unbounded LP is re-solved with s <= 1."""
    d = A.shape[-1]
    cost = np.zeros(d + 1)
    cost[-1] = -1.0
    A_ub = np.zeros((A.shape[-2] + 1, d + 1))
    A_ub[:-1, :-1] = A
    A_ub[:-1, -1] = 2.0
    A_ub[-1, -1] = -1.0
    b_ub = np.zeros(A.shape[-2] + 1)
    b_ub[:-1] = b.reshape(-1)

    def solve(Au, bu):
        return scipy.optimize.linprog(c=cost, A_ub=Au, b_ub=bu, A_eq=A_eq, b_eq=b_eq,
                                      bounds=(None, None), method="highs")

    res = solve(A_ub, b_ub)
    if res.status == 3:  # unbounded: cap the slack
        cap = np.zeros((1, d + 1))
        cap[0, -1] = 1.0
        res = solve(np.concatenate([A_ub, cap], axis=0), np.concatenate([b_ub, np.ones(1)]))
    if res.status == 2:
        raise ValueError("No feasible point found. Constraint polytope appears empty. "
                         "Check your constraints.")
    if res.status > 0:
        raise ValueError("Problem checking constraint specification. "
                         f"linprog status: {res.message}")
    return res.x[:-1]


def _unit_directions(d: int, n: int, seed: Optional[int], dtype) -> torch.Tensor:
    """sampling.py:140-175 with qmc=False: n uniform directions on the unit
    sphere of R^d (normalised Gaussians under ``seed``; d = 1: random signs
    from the global generator, unseeded as in the reference)."""
    if d == 1:
        return 2 * torch.randint(0, 2, (n, 1), dtype=dtype) - 1
    with manual_seed(seed=seed):
        g = torch.randn(n, d, dtype=dtype)
    return g / torch.linalg.norm(g, dim=-1, keepdim=True)


def _f64_host(t: torch.Tensor) -> torch.Tensor:
    return t.detach().to(device="cpu", dtype=torch.float64).contiguous()


def sample_polytope(A: torch.Tensor, b: torch.Tensor, x0: torch.Tensor, n: int = 10000,
                    n0: int = 100, n_thinning: int = 1, seed: Optional[int] = None) -> torch.Tensor:
    """sampling.py:219-309: n points of the hit-and-run chain from x0 over
    {x : A x <= b}, after n0 burn-in steps, every n_thinning-th.  The draws
    (uniform step fractions under ``seed``, unit directions under seed + 1, and
    their products with A) are the reference's; the steps run in
    ``bo_hit_and_run_host`` (fp64)."""
    from ._lib import check, lib
    slack = A @ x0 - b
    if not (slack <= 0).all():
        raise ValueError(f"Starting point does not satisfy the constraints. Inputs: A={A},"
                         f"b={b}, x0={x0}, A@x0-b={slack}.")
    rows = torch.any(A != 0, dim=-1)  # all-zero rows carry no constraint
    A, b = A[rows], b[rows]
    n_tot = n0 + n * n_thinning
    if seed is None:
        seed = torch.randint(0, 1000000, (1,)).item()
    with manual_seed(seed=seed):
        u = torch.rand(n_tot, dtype=A.dtype, device=A.device)
    R = _unit_directions(x0.shape[0], n_tot, seed + 1, A.dtype).to(A.device).unsqueeze(-1)
    AR = (A @ R).squeeze(-1)
    k, m = x0.shape[0], A.shape[0]
    hA, hb, hy = _f64_host(A).reshape(m, k), _f64_host(b).reshape(m), _f64_host(x0).reshape(k)
    hR, hAR, hu = _f64_host(R).reshape(n_tot, k), _f64_host(AR).reshape(n_tot, m), _f64_host(u)
    if m == 0:  # no constraint rows: keep the pointers valid
        hA, hb, hAR = torch.zeros(1, k, dtype=torch.float64), torch.zeros(1, dtype=torch.float64), \
            torch.zeros(max(n_tot, 1), dtype=torch.float64)
    out = torch.empty(n, k, dtype=torch.float64)
    P = ctypes.c_void_p
    check(lib().bo_hit_and_run_host(P(hA.data_ptr()), P(hb.data_ptr()), m, k, P(hy.data_ptr()),
                                    P(hR.data_ptr()), P(hAR.data_ptr()), P(hu.data_ptr()), n_tot,
                                    n0, n_thinning, P(out.data_ptr()), n),
          "bo_hit_and_run_host")
    return out.to(dtype=A.dtype, device=A.device)


def _stack_rows(parts, d, like):
    """Concatenate (rows, rhs) blocks of A x <= b; an empty polytope of
    dimension d when there are none."""
    parts = [p for p in parts if p is not None]
    if not parts:
        return like.new_zeros(0, d), like.new_zeros(0, 1)
    return torch.cat([p[0] for p in parts], 0), torch.cat([p[1] for p in parts], 0)


def _equality_chart(C: Optional[torch.Tensor], d: int, like: torch.Tensor) -> torch.Tensor:
    """Orthonormal columns spanning {x : C x = 0}: the right singular vectors
    past C's numerical rank (no equality: the identity).  Moves of the chain
    are taken in these coordinates, so every sample keeps C x = rhs."""
    if C is None:
        return torch.eye(d, dtype=like.dtype, device=like.device)
    _, sv, Vh = torch.linalg.svd(C)
    return Vh[int((sv != 0).sum()):].mT


class PolytopeSampler:
    """sampling.py:457-578.  The region {x : A x <= b, C x = rhs} with the box
    appended as inequalities, the chart of C's null space in which the chain
    moves, and a starting point inside (the one given, if feasible, else the
    Chebyshev-like LP point of ``find_interior_point``)."""

    def __init__(self, inequality_constraints=None, equality_constraints=None, bounds=None,
                 interior_point=None):
        if inequality_constraints is None and bounds is None:
            raise BotorchError("PolytopeSampler requires either inequality constraints or "
                               "bounds.")
        like = bounds if bounds is not None else inequality_constraints[0]
        d = like.shape[-1]
        self.A, self.b = _stack_rows(
            [inequality_constraints, _box_as_inequalities(bounds) if bounds is not None else None],
            d, like)
        self.equality_constraints = equality_constraints
        self.C, self.d = equality_constraints if equality_constraints is not None else (None, None)
        self.nullC = _equality_chart(self.C, d, self.A)
        self.new_A = self.A @ self.nullC  # the inequalities in chart coordinates
        if interior_point is None:
            self.x0 = self.find_interior_point()
        elif not self.feasible(interior_point):
            raise ValueError("The given input point is not feasible.")
        else:
            self.x0 = interior_point

    def feasible(self, x: torch.Tensor) -> bool:
        ok = bool((self.A @ x <= self.b).all())
        if self.C is not None:
            ok = ok and bool((self.C @ x == self.d).all())
        return ok

    def find_interior_point(self) -> torch.Tensor:
        eq = None
        if self.C is not None:  # the LP's slack column is not in the equalities
            eq = (np.pad(self.C.cpu().numpy(), ((0, 0), (0, 1))), self.d.cpu().numpy())
        x = find_interior_point(self.A.cpu().numpy(), self.b.cpu().numpy(),
                                *(eq if eq is not None else (None, None)))
        return torch.from_numpy(x).to(self.A).reshape(-1, 1)

    def draw(self, n: int = 1) -> torch.Tensor:  # pragma: no cover - abstract
        raise NotImplementedError


class HitAndRunPolytopeSampler(PolytopeSampler):
    """sampling.py:581-704.  Given bounds, the problem is posed on the unit
    cube (x = lower + width * z, sampling.py:624-652) and samples are mapped
    back.  Draws continue one chain: the burn-in runs before the first draw
    only, the chain restarts each draw from the previous draw's last sample,
    and a seeded sampler's seed moves on by n per draw."""

    def __init__(self, inequality_constraints=None, equality_constraints=None, bounds=None,
                 interior_point=None, n_burnin: int = 200, n_thinning: int = 20,
                 seed: Optional[int] = None):
        if inequality_constraints is None and bounds is None:
            raise BotorchError("HitAndRunPolytopeSampler requires either inequality constraints "
                               "or bounds.")
        self._to_box = None  # (lower, width) when the chain runs on the unit cube
        if (inequality_constraints or equality_constraints) and bounds is None:
            warnings.warn("HitAndRunPolytopeSampler did not receive `bounds`, which can lead "
                          "to non-uniform sampling if the parameter ranges are very different "
                          "(see https://github.com/pytorch/botorch/issues/1225).",
                          UserInputWarning, stacklevel=3)
        elif inequality_constraints or equality_constraints:
            lower, width = bounds[0], bounds[1] - bounds[0]
            unit = lambda c: normalize_dense_linear_constraints(bounds, c) if c else c  # noqa: E731
            inequality_constraints, equality_constraints = (unit(inequality_constraints),
                                                            unit(equality_constraints))
            if interior_point is not None:
                interior_point = (interior_point - lower.unsqueeze(-1)) / width.unsqueeze(-1)
            bounds = torch.stack([torch.zeros_like(lower), torch.ones_like(lower)])
            self._to_box = (lower, width)
        super().__init__(inequality_constraints, equality_constraints, bounds, interior_point)
        self.n_burnin, self.n_thinning = n_burnin, n_thinning
        self.num_samples_generated = 0
        self._seed = seed

    def draw(self, n: int = 1) -> torch.Tensor:
        # chart coordinates y (x = x0 + nullC y), the chain starting at y = 0
        first = self.num_samples_generated == 0
        y = sample_polytope(A=self.new_A.cpu(), b=(self.b - self.A @ self.x0).cpu(),
                            x0=self.new_A.new_zeros(self.nullC.shape[1], 1).cpu(), n=n,
                            n0=self.n_burnin if first else 0, n_thinning=self.n_thinning,
                            seed=self._seed).to(self.b)
        if self._seed is not None:
            self._seed += n
        pts = self.x0.mT + y @ self.nullC.mT
        self.x0 = pts[-1:].mT.clone()  # the next draw continues from here
        self.num_samples_generated += n
        if self._to_box is None:
            return pts
        lower, width = self._to_box
        return lower + width * pts


def get_polytope_samples(n: int, bounds: torch.Tensor, inequality_constraints=None,
                         equality_constraints=None, seed: Optional[int] = None,
                         n_burnin: int = 10_000, n_thinning: int = 32) -> torch.Tensor:
    """sampling.py:882-954: n hit-and-run samples from the box and the sparse
    (in)equality constraints (``>=`` inequalities, so they enter the sampler
    negated)."""
    ineq = None
    if inequality_constraints:
        A, b = sparse_to_dense_constraints(bounds.shape[-1], inequality_constraints)
        ineq = (-A, -b)
    eq = (sparse_to_dense_constraints(bounds.shape[-1], equality_constraints)
          if equality_constraints else None)
    sampler = HitAndRunPolytopeSampler(bounds=bounds, inequality_constraints=ineq,
                                       equality_constraints=eq, n_burnin=n_burnin,
                                       n_thinning=n_thinning, seed=seed)
    return sampler.draw(n=n)


# ---- q-batches (optim/initializers.py:72-240) ------------------------------------------

def transform_intra_point_constraint(constraint, d: int, q: int):
    """initializers.py:105-140: one copy per point of the q-batch, on the
    flattened q*d coordinates."""
    indices, coefficients, rhs = constraint
    if indices.max() >= d:
        raise ValueError(f"Constraint indices cannot exceed the problem dimension d={d}.")
    feats = indices.tolist()
    return [(torch.tensor([i * d + f for f in feats], dtype=torch.int64, device=indices.device),
             coefficients, rhs) for i in range(q)]


def transform_inter_point_constraint(constraint, d: int):
    """initializers.py:143-175: (point, feature) pairs to flat indices."""
    indices, coefficients, rhs = constraint
    if indices[:, 1].max() >= d:
        raise ValueError(f"Constraint indices cannot exceed the problem dimension d={d}.")
    flat = [int(p) * d + int(f) for p, f in indices.tolist()]
    return (torch.tensor(flat, dtype=torch.int64, device=indices.device), coefficients, rhs)


def transform_constraints(constraints, q: int, d: int):
    """initializers.py:72-102 (list order kept; None stays None)."""
    if constraints is None:
        return None
    out = []
    for c in constraints:
        if len(c[0].shape) == 1:
            out += transform_intra_point_constraint(c, d, q)
        else:
            out.append(transform_inter_point_constraint(c, d))
    return out


def sample_q_batches_from_polytope(n: int, q: int, bounds: torch.Tensor, n_burnin: int,
                                   n_thinning: int, seed: Optional[int],
                                   inequality_constraints=None,
                                   equality_constraints=None) -> torch.Tensor:
    """initializers.py:178-240: n x q x d raw designs (host).  With an
    inter-point constraint the chain runs on the q*d-dimensional space (thinning
    scaled by q); otherwise n q points of the d-dimensional polytope are
    grouped into q-batches."""
    inter = any(len(ix.shape) > 1 for group in (inequality_constraints or [],
                                                equality_constraints or [])
                for ix, _, _ in group)
    if inter:
        d = bounds.shape[1]
        s = get_polytope_samples(n=n, bounds=torch.hstack([bounds] * q),
                                 inequality_constraints=transform_constraints(
                                     inequality_constraints, q, d),
                                 equality_constraints=transform_constraints(
                                     equality_constraints, q, d),
                                 seed=seed, n_burnin=n_burnin, n_thinning=n_thinning * q)
    else:
        s = get_polytope_samples(n=n * q, bounds=bounds,
                                 inequality_constraints=inequality_constraints,
                                 equality_constraints=equality_constraints, seed=seed,
                                 n_burnin=n_burnin, n_thinning=n_thinning)
    return s.view(n, q, -1).cpu()


def has_inter_point(constraints) -> bool:
    return any(len(ix.shape) > 1 for ix, _, _ in constraints or [])
