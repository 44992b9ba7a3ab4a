"""qNEHVI (acquisition/multi_objective/monte_carlo.py:325-468) on the fused
gfx950 path vs. the oracle: exact hypervolume differences per sample (values)
and the per-sample-cell restatement (values and gradients)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _setup(m, n=60, r=15, seed=0):
    from botorch_amd.models import ModelListGP, SingleTaskGP
    from botorch_amd.test_functions import DTLZ2
    from oracle.gp import ExactGPOracle, GPHyper
    g = torch.Generator().manual_seed(seed)
    X = torch.rand(n, 6, generator=g, dtype=torch.float64)
    Y = DTLZ2(dim=6, num_objectives=m).evaluate_true(X)  # positive; maximised above ref 0
    Y = Y + 0.05 * torch.randn(n, m, generator=g, dtype=torch.float64)
    models, oracles = [], []
    for t in range(m):
        mm = SingleTaskGP(X.to(DEV), Y[:, t:t + 1].to(DEV))
        mm.covar_module.lengthscale = torch.full((1, 6), 0.6, dtype=torch.float64)
        mm.likelihood.noise = torch.tensor([1e-2], dtype=torch.float64)
        models.append(mm.eval())
        oracles.append(ExactGPOracle(X, Y[:, t:t + 1],
                                     GPHyper(torch.full((6,), 0.6, dtype=torch.float64), 1e-2, 0.0)))
    return X, Y, ModelListGP(*models), oracles, X[:r]


@pytest.mark.parametrize("m,q,S", [(2, 1, 32), (2, 3, 16), (3, 2, 16)])
def test_qnehvi_value_matches_exact_hv(m, q, S):
    from botorch_amd.acquisition import qNoisyExpectedHypervolumeImprovement
    from botorch_amd.sampling import SobolQMCNormalSampler
    from oracle.acquisition import QNEHVIOracle
    X, Y, model, oracles, Xb = _setup(m)
    ref_point = [0.0] * m
    acqf = qNoisyExpectedHypervolumeImprovement(model, ref_point, Xb.to(DEV),
                                                sampler=SobolQMCNormalSampler(torch.Size([S]), seed=3))
    orc = QNEHVIOracle(oracles, Xb, ref_point, S, seed=3)
    torch.testing.assert_close(acqf.baseline_samples, orc.Y_base, rtol=1e-8, atol=1e-10)
    g = torch.Generator().manual_seed(m * 10 + q)
    Xc = torch.rand(5, q, 6, generator=g, dtype=torch.float64)
    with torch.no_grad():
        v = acqf(Xc.to(DEV)).cpu()
    ref = orc.value_exact(Xc)
    assert (ref > 0).any()
    torch.testing.assert_close(v, ref, rtol=1e-2, atol=1e-6)   # north_star MC bar
    torch.testing.assert_close(v, ref, rtol=1e-7, atol=1e-10)  # observed: same fp64 algebra


@pytest.mark.parametrize("m,q", [(2, 2), (3, 1)])
def test_qnehvi_gradient_matches_oracle(m, q):
    from botorch_amd.acquisition import qNoisyExpectedHypervolumeImprovement
    from botorch_amd.sampling import SobolQMCNormalSampler
    from oracle.acquisition import QNEHVIOracle
    X, Y, model, oracles, Xb = _setup(m, seed=1)
    S = 16
    ref_point = [0.0] * m
    acqf = qNoisyExpectedHypervolumeImprovement(model, ref_point, Xb.to(DEV),
                                                sampler=SobolQMCNormalSampler(torch.Size([S]), seed=7))
    orc = QNEHVIOracle(oracles, Xb, ref_point, S, seed=7)
    g = torch.Generator().manual_seed(5 + m)
    Xc = torch.rand(4, q, 6, generator=g, dtype=torch.float64)
    Xd = Xc.to(DEV).requires_grad_(True)
    v = acqf(Xd)
    (gd,) = torch.autograd.grad(v.sum(), Xd)
    Xo = Xc.clone().requires_grad_(True)
    lo, hi = acqf.cell_lower_bounds.cpu(), acqf.cell_upper_bounds.cpu()
    rv = orc.value_cells(Xo, lo, hi)
    (go,) = torch.autograd.grad(rv.sum(), Xo)
    torch.testing.assert_close(v.detach().cpu(), rv.detach(), rtol=1e-7, atol=1e-10)
    assert go.abs().max() > 0
    torch.testing.assert_close(gd.cpu(), go, rtol=1e-5, atol=1e-8)


def test_qnehvi_empty_front_and_pending():
    """Reference point above every baseline sample: one cell [ref, inf) per
    sample (test/acquisition/multi_objective/test_monte_carlo.py:976-994); pending
    points join the baseline (cache_pending)."""
    from botorch_amd.acquisition import qNoisyExpectedHypervolumeImprovement
    from botorch_amd.exceptions import UnsupportedError
    from botorch_amd.sampling import SobolQMCNormalSampler
    X, Y, model, oracles, Xb = _setup(2)
    acqf = qNoisyExpectedHypervolumeImprovement(model, [15.0, 14.0], Xb.to(DEV),
                                                sampler=SobolQMCNormalSampler(torch.Size([8]), seed=0))
    assert acqf.cell_lower_bounds.shape == (8, 1, 2)
    assert (acqf.cell_lower_bounds[..., 0] == 15).all() and (acqf.cell_lower_bounds[..., 1] == 14).all()
    assert torch.isinf(acqf.cell_upper_bounds).all()
    with pytest.raises(ValueError, match="m>=2"):
        qNoisyExpectedHypervolumeImprovement(model, [0.0], Xb.to(DEV))
    with pytest.raises(UnsupportedError):
        qNoisyExpectedHypervolumeImprovement(model, [0.0, 0.0], Xb.unsqueeze(0).to(DEV))
    acqf = qNoisyExpectedHypervolumeImprovement(model, [0.0, 0.0], Xb.to(DEV),
                                                sampler=SobolQMCNormalSampler(torch.Size([8]), seed=0))
    acqf.set_X_pending(X[20:22].to(DEV))
    assert acqf.X_baseline.shape[0] == Xb.shape[0] + 2 and acqf.X_pending is None


def test_prune_inferior_points_multi_objective():
    from botorch_amd.acquisition import prune_inferior_points_multi_objective
    X, Y, model, oracles, Xb = _setup(2, n=60, r=60)
    kept = prune_inferior_points_multi_objective(model, X.to(DEV), [0.0, 0.0], num_samples=256)
    assert 0 < kept.shape[0] < 60
    # the observed Pareto-optimal points (tiny noise -> posterior mean ~ data) survive
    from botorch_amd.multi_objective import is_non_dominated
    pm = is_non_dominated(Y) & (Y > 0).all(-1)
    kept_c = kept.cpu()
    for x in X[pm]:
        assert (kept_c == x).all(-1).any()
