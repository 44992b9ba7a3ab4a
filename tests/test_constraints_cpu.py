"""Linear parameter constraints on the host (no GPU): the polytope sampler and
the scipy constraint records against the reference's golden outputs
(``tests/golden/golden_polytope.npz``, made by ``make_golden_polytope.py``
from botorch/utils/sampling.py and botorch/optim/parameter_constraints.py),
then SLSQP candidate generation and constrained optimize_acqf on a smooth
host acquisition.

Reference: utils/sampling.py:219-309, 356-704, 828-985;
optim/parameter_constraints.py:29-312, 412-471; optim/initializers.py:72-240,
304-375; generation/gen.py:124-298; optim/optimize.py:162-178, 246-394.
"""
import os
import warnings

import numpy as np
import pytest
import torch
from scipy.optimize import Bounds, minimize

from botorch_amd import constraints as C
from botorch_amd.acquisition import AcquisitionFunction
from botorch_amd.exceptions import CandidateGenerationError, UnsupportedError
from botorch_amd.optim import gen_batch_initial_conditions, gen_candidates_scipy, optimize_acqf

from tests.golden.cases import POLYTOPE_CASES

HERE = os.path.dirname(os.path.abspath(__file__))
D = torch.float64


@pytest.fixture(scope="module")
def gp():
    return np.load(os.path.join(HERE, "golden", "golden_polytope.npz"))


def t(x):
    return torch.tensor(x, dtype=D)


# ---- the polytope sampler against the reference ---------------------------------------

@pytest.mark.parametrize("tag", ["interior", "face"])
@pytest.mark.parametrize("case", POLYTOPE_CASES["sample_polytope"])
def test_sample_polytope_matches_reference(gp, tag, case):
    """sampling.py:219-309: same draws, same chain (bit for bit here; the
    tolerance covers A y summed in another order than BLAS's)."""
    n, n0, thin, seed = case
    A, b = torch.from_numpy(gp["sp_A"]), torch.from_numpy(gp["sp_b"])
    x0 = torch.from_numpy(gp[f"sp_{tag}_x0"]).to(D)
    s = C.sample_polytope(A, b, x0, n=n, n0=n0, n_thinning=thin, seed=seed)
    ref = gp[f"sp_{tag}_n{n}_b{n0}_t{thin}_s{seed}"]
    assert s.shape == ref.shape
    np.testing.assert_allclose(s.numpy(), ref, rtol=0, atol=1e-12)
    assert bool(((A @ s.T - b) <= 1e-12).all())


def test_sample_polytope_rejects_infeasible_start():
    A, b = t([[1.0, 1.0]]), t([[1.0]])
    with pytest.raises(ValueError, match="Starting point does not satisfy"):
        C.sample_polytope(A, b, t([[1.0], [1.0]]), n=2, n0=0, seed=0)


def test_find_interior_point_matches_reference(gp):
    np.testing.assert_allclose(C.find_interior_point(gp["fip_A"], gp["fip_b"]), gp["fip_bounded"],
                               atol=1e-12)
    np.testing.assert_allclose(C.find_interior_point(gp["fip_unb_A"], gp["fip_unb_b"]),
                               gp["fip_unbounded"], atol=1e-12)
    np.testing.assert_allclose(C.find_interior_point(gp["fip_A"], gp["fip_b"],
                                                     A_eq=gp["fip_eq_A_eq"],
                                                     b_eq=gp["fip_eq_b_eq"]),
                               gp["fip_eq"], atol=1e-12)
    with pytest.raises(ValueError, match="polytope appears empty"):
        C.find_interior_point(np.array([[1.0], [-1.0]]), np.array([[0.0], [-1.0]]))


@pytest.mark.parametrize("case", POLYTOPE_CASES["hit_and_run"])
@pytest.mark.parametrize("eq", [False, True])
def test_hit_and_run_sampler_matches_reference(gp, case, eq):
    """sampling.py:581-704: unit-cube normalisation, the null space of the
    equality constraints, burn-in on the first draw only, seed + n per draw,
    the chain continued from the last sample."""
    burn, thin, seed, n1, n2 = case
    bounds = torch.from_numpy(gp["hr_bounds"])
    A, b = torch.from_numpy(gp["hr_A"]), torch.from_numpy(gp["hr_b"])
    Cm, dc = torch.from_numpy(gp["hr_C"]), torch.from_numpy(gp["hr_d"])
    smp = C.HitAndRunPolytopeSampler(inequality_constraints=(A, b),
                                     equality_constraints=(Cm, dc) if eq else None, bounds=bounds,
                                     n_burnin=burn, n_thinning=thin, seed=seed)
    tag = f"hr_eq{int(eq)}_b{burn}_t{thin}_s{seed}"
    np.testing.assert_allclose(smp.x0.numpy(), gp[tag + "_x0"], atol=1e-12)
    d1, d2 = smp.draw(n1), smp.draw(n2)
    np.testing.assert_allclose(d1.numpy(), gp[tag + "_draw1"], atol=1e-10)
    np.testing.assert_allclose(d2.numpy(), gp[tag + "_draw2"], atol=1e-10)
    X = torch.cat([d1, d2])
    assert bool(((X @ A.T - b.T) <= 1e-9).all())
    assert bool((X >= bounds[0] - 1e-9).all() and (X <= bounds[1] + 1e-9).all())
    if eq:
        np.testing.assert_allclose((X @ Cm.T).numpy(), np.broadcast_to(dc.T.numpy(), (len(X), 1)),
                                   atol=1e-9)


@pytest.mark.parametrize("case", POLYTOPE_CASES["get_polytope_samples"])
def test_get_polytope_samples_matches_reference(gp, case):
    n, burn, thin, seed = case
    bnd = torch.from_numpy(gp["gps_bounds"])
    ineq = [(torch.tensor([0, 2]), t([1.0, 1.0]), 0.5),
            (torch.tensor([1, 3, 4]), t([-1.0, -1.0, -1.0]), -2.0)]
    eqc = [(torch.tensor([0, 1]), t([1.0, 1.0]), 1.0)]
    s1 = C.get_polytope_samples(n=n, bounds=bnd, inequality_constraints=ineq, seed=seed,
                                n_burnin=burn, n_thinning=thin)
    s2 = C.get_polytope_samples(n=n, bounds=bnd, inequality_constraints=ineq,
                                equality_constraints=eqc, seed=seed, n_burnin=burn,
                                n_thinning=thin)
    np.testing.assert_allclose(s1.numpy(), gp[f"gps_ineq_n{n}_b{burn}_t{thin}_s{seed}"], atol=1e-10)
    np.testing.assert_allclose(s2.numpy(), gp[f"gps_both_n{n}_b{burn}_t{thin}_s{seed}"], atol=1e-10)


def test_dense_and_normalised_forms_match_reference(gp):
    bnd = torch.from_numpy(gp["gps_bounds"])
    ineq = [(torch.tensor([0, 2]), t([1.0, 1.0]), 0.5),
            (torch.tensor([1, 3, 4]), t([-1.0, -1.0, -1.0]), -2.0)]
    A, b = C.sparse_to_dense_constraints(5, ineq)
    np.testing.assert_array_equal(A.numpy(), gp["s2d_A"])
    np.testing.assert_array_equal(b.numpy(), gp["s2d_b"])
    An, bn = C.normalize_dense_linear_constraints(bnd, (A, b))
    np.testing.assert_array_equal(An.numpy(), gp["ndl_A"])
    np.testing.assert_array_equal(bn.numpy(), gp["ndl_b"])
    for i, (ix, cf, rhs) in enumerate(C.normalize_sparse_linear_constraints(bnd, ineq)):
        np.testing.assert_array_equal(ix.numpy(), gp[f"nsl_{i}_idx"])
        np.testing.assert_array_equal(cf.numpy(), gp[f"nsl_{i}_coef"])
        assert rhs == float(gp[f"nsl_{i}_rhs"])
    with pytest.raises(ValueError, match="one-dimensional"):
        C.normalize_sparse_linear_constraints(bnd, [(torch.tensor([[0, 1]]), t([1.0]), 0.0)])


def test_q_batches_from_polytope_match_reference(gp):
    """initializers.py:178-240: the inter-point draw runs on the q*d space with
    thinning * q; the intra-point draw groups n q samples."""
    q, bq = 3, t([[0.0, 0.0], [1.0, 1.0]])
    inter = [(torch.tensor([[0, 0], [1, 0], [2, 1]]), t([1.0, 1.0, 1.0]), 0.8)]
    intra = [(torch.tensor([0, 1]), t([-1.0, -1.0]), -1.5)]
    n, burn, thin, seed = 6, 50, 2, 5
    s = C.sample_q_batches_from_polytope(n, q, bq, burn, thin, seed, inequality_constraints=inter + intra)
    np.testing.assert_allclose(s.numpy(), gp["qb_inter"], atol=1e-10)
    s = C.sample_q_batches_from_polytope(n, q, bq, burn, thin, seed, inequality_constraints=intra)
    np.testing.assert_allclose(s.numpy(), gp["qb_intra"], atol=1e-10)
    with pytest.raises(ValueError, match="cannot exceed the problem dimension"):
        C.transform_constraints([(torch.tensor([2]), t([1.0]), 0.0)], q=2, d=2)


# ---- scipy records ----------------------------------------------------------------------

def test_scipy_records_match_reference(gp):
    shapeX = torch.Size([3, 2, 4])
    x = gp["msl_x"]
    cons = C.make_scipy_linear_constraints(
        shapeX, inequality_constraints=[(torch.tensor([1, 3]), t([1.0, 0.5]), -0.1)],
        equality_constraints=[(torch.tensor([[0, 1], [1, 3]]), t([1.0, -2.0]), 0.25)])
    np.testing.assert_array_equal([1 if c["type"] == "eq" else 0 for c in cons], gp["msl_type"])
    np.testing.assert_array_equal([c["fun"](x) for c in cons], gp["msl_fun"])
    np.testing.assert_array_equal(np.stack([c["jac"](x) for c in cons]), gp["msl_jac"])
    sb = C.make_scipy_bounds(torch.zeros(shapeX, dtype=D), t([0.0, -1.0, 0.0, 0.5]), 2.0)
    np.testing.assert_array_equal(sb.lb, gp["msb_lb"])
    np.testing.assert_array_equal(sb.ub, gp["msb_ub"])
    assert C.make_scipy_bounds(torch.zeros(shapeX, dtype=D)) is None


def test_scipy_record_validation():
    ok = (torch.tensor([0]), t([1.0]), 0.0)
    with pytest.raises(UnsupportedError, match="at least two-dimensional"):
        C.make_scipy_linear_constraints(torch.Size([4]), [ok])
    with pytest.raises(RuntimeError, match="4-dim parameter tensor"):
        C.make_scipy_linear_constraints(torch.Size([2, 4]), [(torch.tensor([4]), t([1.0]), 0.0)])
    with pytest.raises(RuntimeError, match="2-batch"):
        C.make_scipy_linear_constraints(torch.Size([2, 4]),
                                        [(torch.tensor([[2, 0]]), t([1.0]), 0.0)])
    with pytest.raises(UnsupportedError, match="general batch shapes"):
        C.make_scipy_linear_constraints(torch.Size([2, 4]),
                                        [(torch.zeros(1, 1, 2, dtype=torch.long), t([1.0]), 0.0)])
    with pytest.raises(ValueError, match="at least one-dimensional"):
        C.make_scipy_linear_constraints(torch.Size([2, 4]), [(torch.tensor(0), t([1.0]), 0.0)])
    # a 2-d shape is one t-batch
    assert len(C.make_scipy_linear_constraints(torch.Size([2, 4]), [ok])) == 2


def test_unfixed_constraints_match_reference(gp):
    cl = [(torch.tensor([0, 2, 3]), t([1.0, 2.0, -1.0]), 0.5),
          (torch.tensor([[0, 1], [1, 2]]), t([1.0, 1.0]), 0.3)]
    new = C._generate_unfixed_lin_constraints(cl, {2: 0.25}, dimension=4, eq=False)
    assert len(new) == int(gp["gul_count"])
    for i, (ix, cf, rhs) in enumerate(new):
        np.testing.assert_array_equal(ix.numpy(), gp[f"gul_{i}_idx"])
        np.testing.assert_array_equal(cf.numpy(), gp[f"gul_{i}_coef"])
        assert rhs == float(gp[f"gul_{i}_rhs"])
    # every term fixed: the constraint must hold as it stands
    with pytest.raises(CandidateGenerationError, match="Inequality constraint 0 not met"):
        C._generate_unfixed_lin_constraints([(torch.tensor([1]), t([1.0]), 0.5)], {1: 0.2}, 3,
                                            eq=False)
    assert C._generate_unfixed_lin_constraints([(torch.tensor([1]), t([1.0]), 0.5)], {1: 0.7}, 3,
                                               eq=False) == []


# ---- SLSQP candidate generation and constrained optimize_acqf --------------------------

class _Quad(AcquisitionFunction):
    """-||x - target||^2 summed over the q points."""

    def __init__(self, target):
        super().__init__(model=None)
        self.target = target

    def forward(self, X):
        X = X if X.dim() == 3 else X.unsqueeze(0)
        return -((X - self.target.to(X)) ** 2).sum(dim=(-1, -2))


BOUNDS = torch.stack([torch.zeros(3, dtype=D), torch.ones(3, dtype=D)])
TARGET = t([0.9, 0.9, 0.45])
SUM01 = [(torch.tensor([0, 1]), t([-1.0, -1.0]), -1.0)]        # x0 + x1 <= 1
X2EQ = [(torch.tensor([2]), t([1.0]), 0.3)]                     # x2 == 0.3


def test_slsqp_is_scipy_slsqp_with_the_reference_records():
    """gen.py:182-267: the candidates are exactly what scipy's SLSQP returns
    on the flattened problem with make_scipy_bounds / the constraint records."""
    acq = _Quad(TARGET)
    X0 = t([[[0.1, 0.2, 0.3]], [[0.4, 0.1, 0.9]]])
    cand, val = gen_candidates_scipy(X0, acq, BOUNDS[0], BOUNDS[1], inequality_constraints=SUM01,
                                     equality_constraints=X2EQ)
    shapeX = X0.shape

    def f(x):
        X = torch.from_numpy(x).view(shapeX).requires_grad_(True)
        loss = -acq(X).sum()
        return loss.item(), torch.autograd.grad(loss, X)[0].reshape(-1).numpy()

    cons = C.make_scipy_linear_constraints(shapeX, SUM01, X2EQ)
    res = minimize(f, X0.reshape(-1).numpy(), method="SLSQP", jac=True,
                   bounds=Bounds(np.zeros(6), np.ones(6), keep_feasible=True), constraints=cons,
                   options={"maxiter": 2000})
    np.testing.assert_array_equal(cand.reshape(-1).numpy(), res.x)
    # the projection of the target on {x0 + x1 <= 1, x2 = 0.3}
    np.testing.assert_allclose(cand.numpy(), np.broadcast_to([0.5, 0.5, 0.3], (2, 1, 3)), atol=1e-6)
    np.testing.assert_allclose(val.numpy(), acq(cand).numpy())


@pytest.mark.parametrize("ff", [{1: 0.2}, {1: None}])
def test_slsqp_with_fixed_features(ff):
    """A fixed value moves into the right-hand sides (reduced domain); a None
    value with constraints present keeps the full space, pinned inside the
    objective (gen.py:124-175, 208)."""
    acq = _Quad(TARGET)
    X0 = t([[[0.1, 0.2, 0.3]]])
    cand, _ = gen_candidates_scipy(X0, acq, BOUNDS[0], BOUNDS[1], inequality_constraints=SUM01,
                                   equality_constraints=X2EQ, fixed_features=ff)
    c = cand.reshape(-1).numpy()
    if ff[1] is not None:
        np.testing.assert_allclose(c, [0.8, 0.2, 0.3], atol=1e-6)
    else:
        # the None column is only detached from the objective: SLSQP may still
        # move it to satisfy the constraints (the reference's semantics)
        assert c[0] + c[1] <= 1 + 1e-9 and abs(c[2] - 0.3) < 1e-9
        np.testing.assert_allclose(c[0], 0.9, atol=1e-6)


def test_initial_conditions_come_from_the_polytope():
    """initializers.py:365-375: under constraints the raw designs are the
    hit-and-run q-batches of the seed; all feasible."""
    acq = _Quad(TARGET)
    ineq = SUM01 + [(torch.tensor([[0, 2], [1, 2]]), t([1.0, 1.0]), 0.5)]  # inter-point
    opts = {"seed": 3, "n_burnin": 200, "n_thinning": 4}
    ics = gen_batch_initial_conditions(acq, BOUNDS, q=2, num_restarts=4, raw_samples=16,
                                       options=opts, inequality_constraints=ineq)
    assert ics.shape == (4, 2, 3)
    raw = C.sample_q_batches_from_polytope(16, 2, BOUNDS, 200, 4, 3, inequality_constraints=ineq)
    # every pick is one of the seeded polytope designs
    hits = [(raw == ic).all(-1).all(-1).any().item() for ic in ics]
    assert all(hits)
    assert bool((ics[..., 0] + ics[..., 1] <= 1 + 1e-12).all())
    assert bool((ics[:, 0, 2] + ics[:, 1, 2] >= 0.5 - 1e-12).all())
    with pytest.raises(NotImplementedError, match="finite values in `bounds`"):
        gen_batch_initial_conditions(acq, torch.stack([BOUNDS[0], torch.full((3,), float("inf"),
                                                                             dtype=D)]),
                                     q=1, num_restarts=2, raw_samples=4)


def test_optimize_acqf_with_linear_constraints():
    acq = _Quad(TARGET)
    torch.manual_seed(0)
    with warnings.catch_warnings():
        warnings.simplefilter("error", RuntimeWarning)  # no retry needed
        cand, val = optimize_acqf(acq, BOUNDS, q=2, num_restarts=4, raw_samples=32,
                                  options={"seed": 1, "n_burnin": 500},
                                  inequality_constraints=SUM01, equality_constraints=X2EQ)
    np.testing.assert_allclose(cand.numpy(), [[0.5, 0.5, 0.3]] * 2, atol=1e-6)
    # sequential greedy q keeps intra-point constraints, refuses inter-point ones
    torch.manual_seed(0)
    cs, _ = optimize_acqf(acq, BOUNDS, q=2, num_restarts=4, raw_samples=32, sequential=True,
                          options={"seed": 1, "n_burnin": 500}, inequality_constraints=SUM01)
    assert bool((cs[:, 0] + cs[:, 1] <= 1 + 1e-9).all())
    with pytest.raises(UnsupportedError, match="across the q-dimension"):
        optimize_acqf(acq, BOUNDS, q=2, num_restarts=4, raw_samples=32, sequential=True,
                      inequality_constraints=[(torch.tensor([[0, 0], [1, 0]]), t([1.0, 1.0]),
                                               0.5)])


def test_native_chain_argument_checks():
    from botorch_amd._lib import lib
    import ctypes
    # n_tot must be n0 + n * n_thin
    z = torch.zeros(16, dtype=D)
    P = ctypes.c_void_p(z.data_ptr())
    assert lib().bo_hit_and_run_host(P, P, 1, 1, P, P, P, P, 5, 1, 1, P, 3) != 0
