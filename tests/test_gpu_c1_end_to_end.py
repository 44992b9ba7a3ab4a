"""C1 (BASELINE.json configs[0]): SingleTaskGP + analytic EI on Hartmann6,
n = 20, q = 1, on the reference's end-to-end protocol (test/test_end_to_end.py:
36-132): fit_gpytorch_mll with maxiter 5, then optimize_acqf for analytic EI
and qEI (q = 3) with num_restarts = 10, raw_samples = 20.  Checked against the
oracle: the 5-iteration fit against the same L-BFGS-B run over the oracle's MLL,
the acquisition values at the returned candidates against the oracle's EI /
qEI, the candidates in bounds.  Plus the reference test itself (noisy sin, 10
points, d = 1, fp64 and fp32, inferred and fixed noise), and the caller
contract on the device: fixed features, sample_around_best, sequential q.
"""
import math
import warnings

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
EPS = 1e-8


def _c1_data():
    from botorch_amd.test_functions import Hartmann
    from oracle.sampling import draw_sobol_samples
    lo = torch.zeros(6, dtype=torch.float64)
    X = draw_sobol_samples(lo, lo + 1, 20, 1, 0).squeeze(1)
    Y = Hartmann(negate=True)(X).unsqueeze(-1)
    return X, Y


def _fitted_c1():
    from botorch_amd.exceptions import OptimizationWarning
    from botorch_amd.fit import ExactMarginalLogLikelihood, _Layout, fit_gpytorch_mll
    from botorch_amd.models import SingleTaskGP
    X, Y = _c1_data()
    m = SingleTaskGP(X.to(DEV), Y.to(DEV))
    lay = _Layout(m)
    x0, bounds = lay.get(), lay.bounds
    with warnings.catch_warnings():
        warnings.filterwarnings("ignore", category=OptimizationWarning)
        mll = fit_gpytorch_mll(ExactMarginalLogLikelihood(m.likelihood, m),
                               optimizer_kwargs={"options": {"maxiter": 5}}, max_attempts=1)
    assert not mll.training
    return m, X, Y, x0, bounds, lay.get()


def _oracle_of(m, X, Y):
    from oracle.gp import ExactGPOracle, GPHyper
    ls, _, noise, c = m.hyper()
    return ExactGPOracle(X, Y, GPHyper(ls.cpu(), noise, c))


def test_c1_fit_matches_oracle_five_iterations():
    from oracle.gp import fit_scipy, standardize_fit
    m, X, Y, x0, bounds, x_fit = _fitted_c1()
    mu, sd = standardize_fit(Y)
    res = fit_scipy(X, ((Y - mu) / sd).squeeze(-1), x0, bounds, options={"maxiter": 5})
    assert res.nit == 5 or res.success
    np.testing.assert_allclose(x_fit, res.x, rtol=1e-7, atol=1e-9)


def test_c1_analytic_ei_optimize_acqf():
    from botorch_amd.acquisition import ExpectedImprovement
    from botorch_amd.optim import optimize_acqf
    from oracle.acquisition import ei_analytic
    m, X, Y, *_ = _fitted_c1()
    orc = _oracle_of(m, X, Y)
    best_f = float(Y.max())
    ei = ExpectedImprovement(m, best_f=best_f)
    Xt = torch.rand(64, 1, 6, dtype=torch.float64, generator=torch.Generator().manual_seed(3))
    torch.testing.assert_close(ei(Xt.to(DEV)).cpu(), ei_analytic(orc, Xt, best_f),
                               rtol=1e-6, atol=1e-12)
    bounds = torch.stack([torch.zeros(6), torch.ones(6)]).to(DEV, torch.float64)
    torch.manual_seed(0)
    cand, val = optimize_acqf(ei, bounds, q=1, num_restarts=10, raw_samples=20,
                              options={"maxiter": 5})
    assert cand.shape == (1, 6)
    assert torch.all(cand >= -EPS) and torch.all(cand <= 1 + EPS)
    torch.testing.assert_close(val.cpu().reshape(()), ei_analytic(orc, cand.cpu().unsqueeze(0),
                                                                  best_f).reshape(()),
                               rtol=1e-6, atol=1e-12)


@pytest.mark.parametrize("gen", ["scipy", "device"])
def test_c1_qei_optimize_acqf(gen):
    from botorch_amd.acquisition import qExpectedImprovement
    from botorch_amd.optim import gen_candidates_device, gen_candidates_scipy, optimize_acqf
    from botorch_amd.sampling import SobolQMCNormalSampler
    from oracle.acquisition import qei
    from oracle.sampling import draw_sobol_normal_samples
    m, X, Y, *_ = _fitted_c1()
    orc = _oracle_of(m, X, Y)
    best_f = float(Y.max()) - 0.5
    acqf = qExpectedImprovement(m, best_f=best_f,
                                sampler=SobolQMCNormalSampler(torch.Size([512]), seed=0))
    bounds = torch.stack([torch.zeros(6), torch.ones(6)]).to(DEV, torch.float64)
    g = gen_candidates_scipy if gen == "scipy" else gen_candidates_device
    Z = draw_sobol_normal_samples(3, 512, 0)
    for opts in ({"maxiter": 5}, {"maxiter": 5, "batch_limit": 5}):
        torch.manual_seed(0)
        cand, val = optimize_acqf(acqf, bounds, q=3, num_restarts=10, raw_samples=20,
                                  options=opts, gen_candidates=g)
        assert cand.shape == (3, 6)
        assert torch.all(cand >= -EPS) and torch.all(cand <= 1 + EPS)
        ref = qei(orc, cand.cpu().unsqueeze(0), Z, best_f)
        torch.testing.assert_close(val.cpu().reshape(1), ref, rtol=1e-6, atol=1e-12)
        assert float(val) > 0


def test_c1_qei_optimize_acqf_linear_constraints():
    """optimize_acqf under linear constraints with the HIP qEI: polytope raw
    samples (native hit-and-run, initializers.py:365-375) evaluated on the
    device, SLSQP candidates (gen.py:256) through the HIP forward + backward;
    the candidates are feasible and their values are the oracle's qEI."""
    from botorch_amd.acquisition import qExpectedImprovement
    from botorch_amd.optim import optimize_acqf
    from botorch_amd.sampling import SobolQMCNormalSampler
    from oracle.acquisition import qei
    from oracle.sampling import draw_sobol_normal_samples
    m, X, Y, *_ = _fitted_c1()
    orc = _oracle_of(m, X, Y)
    best_f = float(Y.max()) - 0.5
    acqf = qExpectedImprovement(m, best_f=best_f,
                                sampler=SobolQMCNormalSampler(torch.Size([512]), seed=0))
    bounds = torch.stack([torch.zeros(6), torch.ones(6)]).to(DEV, torch.float64)
    f64 = dict(dtype=torch.float64, device=DEV)
    ineq = [(torch.tensor([0, 1], device=DEV), torch.tensor([-1.0, -1.0], **f64), -0.8),
            (torch.tensor([[0, 2], [1, 2]], device=DEV), torch.tensor([1.0, 1.0], **f64), 0.6)]
    eq = [(torch.tensor([3, 4], device=DEV), torch.tensor([1.0, 1.0], **f64), 1.0)]
    torch.manual_seed(0)
    cand, val = optimize_acqf(acqf, bounds, q=2, num_restarts=6, raw_samples=32,
                              options={"maxiter": 50, "seed": 0, "n_burnin": 500},
                              inequality_constraints=ineq, equality_constraints=eq)
    assert cand.shape == (2, 6)
    c = cand.cpu()
    assert torch.all(c >= -EPS) and torch.all(c <= 1 + EPS)
    assert torch.all(c[:, 0] + c[:, 1] <= 0.8 + 1e-6)
    assert float(c[0, 2] + c[1, 2]) >= 0.6 - 1e-6
    torch.testing.assert_close(c[:, 3] + c[:, 4], torch.ones(2, dtype=torch.float64), atol=1e-6,
                               rtol=0)
    Z = draw_sobol_normal_samples(2, 512, 0)
    ref = qei(orc, c.unsqueeze(0), Z, best_f)
    torch.testing.assert_close(val.cpu().reshape(1), ref, rtol=1e-6, atol=1e-12)
    assert float(val) > 0


def _sin_setup(dtype):
    """test/test_end_to_end.py:37-72: 10 noisy sin points in [0, 1]."""
    from botorch_amd.exceptions import OptimizationWarning
    from botorch_amd.fit import ExactMarginalLogLikelihood, fit_gpytorch_mll
    from botorch_amd.models import SingleTaskGP
    noise = torch.tensor([[0.127], [-0.113], [-0.345], [-0.034], [-0.069], [-0.272], [0.013],
                          [0.056], [0.087], [-0.081]], dtype=dtype)
    x = torch.linspace(0, 1, 10, dtype=dtype).view(-1, 1)
    y = torch.sin(x * (2 * math.pi)) + noise
    yvar = torch.tensor(0.1 ** 2, dtype=dtype)
    models = []
    for m in (SingleTaskGP(x.to(DEV), y.to(DEV)),
              SingleTaskGP(x.to(DEV), y.to(DEV), yvar.expand_as(y).to(DEV))):
        with warnings.catch_warnings():
            warnings.filterwarnings("ignore", category=OptimizationWarning)
            fit_gpytorch_mll(ExactMarginalLogLikelihood(m.likelihood, m),
                             optimizer_kwargs={"options": {"maxiter": 5}}, max_attempts=1)
        models.append(m)
    return models, torch.tensor([[0.0], [1.0]], dtype=dtype, device=DEV)


@pytest.mark.parametrize("dtype", [torch.float64, torch.float32])
def test_reference_end_to_end_sin(dtype):
    """test_end_to_end.py:74-132: qEI (q = 3, also batch_limit 5) and analytic
    EI candidates lie in the bounds, for both models and both dtypes."""
    from botorch_amd.acquisition import ExpectedImprovement, qExpectedImprovement
    from botorch_amd.optim import optimize_acqf
    (m_st, m_fn), bounds = _sin_setup(dtype)
    for m in (m_st, m_fn):
        for opts in ({"maxiter": 5}, {"maxiter": 5, "batch_limit": 5}):
            c, _ = optimize_acqf(qExpectedImprovement(m, best_f=0.0), bounds, q=3,
                                 num_restarts=10, raw_samples=20, options=opts)
            assert c.shape == (3, 1)
            assert torch.all(-EPS <= c) and torch.all(c <= 1 + EPS)
        c, _ = optimize_acqf(ExpectedImprovement(m, best_f=0.0), bounds, q=1, num_restarts=10,
                             raw_samples=20, options={"maxiter": 5})
        assert -EPS <= float(c) <= 1 + EPS


@pytest.mark.parametrize("gen", ["scipy", "device"])
def test_fixed_features_on_device(gen):
    """optimize_acqf with fixed_features (optimize.py:289-295 -> gen.py:124-175):
    the fixed column is exact, the value is the base acquisition's at the full
    candidate, and it is the optimum over the free columns (no better than the
    unconstrained optimum)."""
    from botorch_amd.acquisition import qExpectedImprovement
    from botorch_amd.optim import gen_candidates_device, gen_candidates_scipy, optimize_acqf
    from botorch_amd.sampling import SobolQMCNormalSampler
    m, X, Y, *_ = _fitted_c1()
    acqf = qExpectedImprovement(m, best_f=float(Y.max()) - 0.5,
                                sampler=SobolQMCNormalSampler(torch.Size([256]), seed=0))
    bounds = torch.stack([torch.zeros(6), torch.ones(6)]).to(DEV, torch.float64)
    g = gen_candidates_scipy if gen == "scipy" else gen_candidates_device
    torch.manual_seed(0)
    with warnings.catch_warnings(record=True) as ws:
        warnings.simplefilter("always")
        c, v = optimize_acqf(acqf, bounds, q=2, num_restarts=6, raw_samples=64,
                             options={"use_graph": True} if gen == "device" else None,
                             fixed_features={1: 0.25, 4: 0.5}, gen_candidates=g)
    assert not any("Graph is empty" in str(w.message) for w in ws)
    assert torch.all(c[:, 1] == 0.25) and torch.all(c[:, 4] == 0.5)
    torch.testing.assert_close(v.reshape(1), acqf(c.unsqueeze(0)).reshape(1))
    if gen == "device":
        # the fixed-feature wrapper copies nothing from the host, so the
        # evaluation graph is captured and replayed (not a silent eager run),
        # and its candidates are the eager evaluations' bit for bit
        assert gen_candidates_device.last_graph_error is None, gen_candidates_device.last_graph_error
        assert gen_candidates_device.last_graphed_evals > 0
        torch.manual_seed(0)
        c_e, v_e = optimize_acqf(acqf, bounds, q=2, num_restarts=6, raw_samples=64,
                                 options={"use_graph": False},
                                 fixed_features={1: 0.25, 4: 0.5}, gen_candidates=g)
        assert gen_candidates_device.last_graphed_evals == 0
        assert torch.equal(c, c_e) and torch.equal(v, v_e)
    torch.manual_seed(0)
    _, v_free = optimize_acqf(acqf, bounds, q=2, num_restarts=6, raw_samples=64, gen_candidates=g)
    assert float(v) <= float(v_free) + 1e-9


def test_sample_around_best_and_sequential_on_device():
    from botorch_amd.acquisition import qExpectedImprovement
    from botorch_amd.optim import gen_batch_initial_conditions, optimize_acqf
    from botorch_amd.sampling import SobolQMCNormalSampler
    m, X, Y, *_ = _fitted_c1()
    acqf = qExpectedImprovement(m, best_f=float(Y.max()) - 0.5,
                                sampler=SobolQMCNormalSampler(torch.Size([256]), seed=0))
    bounds = torch.stack([torch.zeros(6), torch.ones(6)]).to(DEV, torch.float64)
    torch.manual_seed(0)
    ics = gen_batch_initial_conditions(acqf, bounds, q=2, num_restarts=8, raw_samples=32,
                                       options={"sample_around_best": True, "seed": 0})
    assert ics.shape == (8, 2, 6) and torch.all((ics >= 0) & (ics <= 1))
    torch.manual_seed(1)
    c, v = optimize_acqf(acqf, bounds, q=3, num_restarts=4, raw_samples=32,
                         options={"maxiter": 20}, sequential=True)
    assert c.shape == (3, 6) and v.shape == (3,)
    assert acqf.X_pending is None
    # the i-th value is the q = 1 acquisition given the earlier picks pending
    for i in range(3):
        acqf.set_X_pending(c[:i] if i else None)
        torch.testing.assert_close(acqf(c[i:i + 1].unsqueeze(0)).reshape(()), v[i].reshape(()))
    acqf.set_X_pending(None)
