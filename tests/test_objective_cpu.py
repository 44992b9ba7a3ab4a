"""Outcome-constraint helpers and sampler selection on the host, pinned by the
reference's own functions (tests/golden: utils/objective.py:101-180)."""
import numpy as np
import pytest
import torch


def _cons():
    return [lambda Z: Z[..., 0] - 0.2, lambda Z: 0.5 * Z[..., 1] + Z[..., 0] - 0.4]


def test_feasibility_indicator_hard(golden):
    from botorch_amd.objective import compute_feasibility_indicator
    smp = torch.from_numpy(golden["feas_samples"])
    got = compute_feasibility_indicator(_cons(), smp)
    assert np.array_equal(got.numpy(), golden["feas_hard"])


@pytest.mark.parametrize("log", [False, True])
@pytest.mark.parametrize("fat", [False, True])
@pytest.mark.parametrize("ename", ["e1", "e2"])
def test_smoothed_feasibility_matches_reference(golden, log, fat, ename):
    from botorch_amd.objective import compute_smoothed_feasibility_indicator
    eta = 1e-1 if ename == "e1" else torch.tensor([0.05, 0.3], dtype=torch.float64)
    x = torch.from_numpy(golden["feas_samples"]).clone().requires_grad_(True)
    ind = compute_smoothed_feasibility_indicator(_cons(), x, eta, log=log, fat=fat)
    (gx,) = torch.autograd.grad(ind.sum(), x)
    tag = f"feas_l{int(log)}_f{int(fat)}_{ename}"
    np.testing.assert_allclose(ind.detach().numpy(), golden[tag], rtol=1e-13, atol=1e-300)
    np.testing.assert_allclose(gx.numpy(), golden[tag + "_grad"], rtol=1e-12, atol=1e-300)


def test_smoothed_feasibility_errors():
    from botorch_amd.objective import compute_smoothed_feasibility_indicator
    smp = torch.zeros(2, 3, 1, dtype=torch.float64)
    with pytest.raises(ValueError, match="do not match"):
        compute_smoothed_feasibility_indicator(_cons(), smp, torch.tensor([0.1]))
    with pytest.raises(ValueError, match="positive"):
        compute_smoothed_feasibility_indicator(_cons()[:1], smp, -1.0)


def test_best_feasible_objective_unconstrained_and_constrained():
    from botorch_amd.objective import compute_best_feasible_objective
    samples = torch.tensor([[[1.0], [3.0], [2.0]], [[0.5], [0.1], [4.0]]], dtype=torch.float64)
    obj = samples.squeeze(-1)
    assert torch.equal(compute_best_feasible_objective(samples, obj, None), torch.tensor([3.0, 4.0], dtype=torch.float64))
    cons = [lambda Z: Z[..., 0] - 2.5]  # feasible iff sample <= 2.5
    got = compute_best_feasible_objective(samples, obj, cons)
    assert torch.equal(got, torch.tensor([2.0, 0.5], dtype=torch.float64))


def test_get_sampler_iid_fallback_above_sobol_maxdim():
    """sampling/get_sampler.py:84-89: IID base samples beyond SobolEngine.MAXDIM."""
    from botorch_amd.sampling import (IIDNormalSampler, ShapeOnlyPosterior, SobolQMCNormalSampler,
                                      get_sampler)
    small = ShapeOnlyPosterior(torch.Size([4]), 100, "cpu")
    assert type(get_sampler(small, torch.Size([8]))) is SobolQMCNormalSampler
    big = ShapeOnlyPosterior(torch.Size([4]), 21202, "cpu")
    with pytest.warns(RuntimeWarning, match="too large for the Sobol engine"):
        s = get_sampler(big, torch.Size([8]), seed=3)
    assert type(s) is IIDNormalSampler and s.seed == 3


def test_iid_sampler_reuses_collapsed_base_samples():
    """Base samples installed for one collapsed shape serve another that differs
    only in size-1 batch dims (no redraw); a new dimension redraws."""
    from botorch_amd.sampling import IIDNormalSampler, ShapeOnlyPosterior
    s = IIDNormalSampler(torch.Size([5]), seed=0)
    s._construct_base_samples(ShapeOnlyPosterior(torch.Size([3]), 4, "cpu"))
    mine = torch.arange(20, dtype=torch.float64).view(5, 1, 4)
    s.base_samples = mine
    s._construct_base_samples(ShapeOnlyPosterior(torch.Size([4, 3]), 4, "cpu"))
    assert s.base_samples.shape == (5, 1, 1, 4) and torch.equal(s.base_samples.reshape(5, 4), mine.reshape(5, 4))
    s._construct_base_samples(ShapeOnlyPosterior(torch.Size([3]), 6, "cpu"))
    assert s.base_samples.shape == (5, 1, 6)


def test_update_base_samples_keeps_baseline_columns():
    """sampling/normal.py:68-131: the joint draw's leading columns are the base
    sampler's (single-output)."""
    import copy
    from botorch_amd.sampling import IIDNormalSampler, ShapeOnlyPosterior
    base = IIDNormalSampler(torch.Size([6]), seed=1)
    base._construct_base_samples(ShapeOnlyPosterior(torch.Size(), 3, "cpu"))
    s = copy.deepcopy(base)
    s._update_base_samples(ShapeOnlyPosterior(torch.Size([2]), 5, "cpu"), base)
    assert s.base_samples.shape == (6, 1, 5)
    assert torch.equal(s.base_samples[:, 0, :3], base.base_samples)
