"""GP fitting (exact MLL + gradient on the device) and the optimize_acqf driver."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _data(n, seed=0):
    from botorch_amd.test_functions import Hartmann
    from oracle.sampling import draw_sobol_samples
    lo = torch.zeros(6, dtype=torch.float64)
    X = draw_sobol_samples(lo, lo + 1, n, 1, seed).squeeze(1)
    Y = Hartmann(negate=True)(X).unsqueeze(-1)
    return X, Y


@pytest.mark.parametrize("n", [50, 300])
def test_mll_value_and_grad_match_oracle(n):
    from botorch_amd.fit import _Layout, mll_value_and_grad
    from botorch_amd.models import SingleTaskGP
    from oracle.gp import neg_mll, standardize_fit
    X, Y = _data(n)
    m = SingleTaskGP(X.to(DEV), Y.to(DEV))
    lay = _Layout(m)
    x = np.array([0.02, 0.3, 0.4, 0.5, 0.6, 0.7, 0.8, 0.9])
    val, grad = mll_value_and_grad(m, x, lay)
    mu, sd = standardize_fit(Y)
    y = ((Y - mu) / sd).squeeze(-1)
    ls = torch.tensor(x[2:], requires_grad=True)
    noise = torch.tensor(x[0], requires_grad=True)
    c = torch.tensor(x[1], requires_grad=True)
    loss = neg_mll(X, y, ls, noise, c)
    loss.backward()
    ref_g = np.concatenate([[noise.grad.item(), c.grad.item()], ls.grad.numpy()])
    assert abs(val - loss.item()) < 1e-9 * max(1.0, abs(loss.item()))
    np.testing.assert_allclose(grad, ref_g, rtol=1e-6, atol=1e-9)


def test_fit_gpytorch_mll_improves_and_matches_oracle_optimum():
    from botorch_amd.fit import ExactMarginalLogLikelihood, _Layout, fit_gpytorch_mll, mll_value_and_grad
    from botorch_amd.models import SingleTaskGP
    X, Y = _data(128)
    m = SingleTaskGP(X.to(DEV), Y.to(DEV))
    lay = _Layout(m)
    x0 = lay.get()
    v0, _ = mll_value_and_grad(m, x0, lay)
    mll = fit_gpytorch_mll(ExactMarginalLogLikelihood(m.likelihood, m))
    assert not mll.training
    x1 = lay.get()
    v1, g1 = mll_value_and_grad(m, x1, lay)
    assert v1 < v0
    # projected gradient ~ 0 at the optimum (bounds active -> zero only inside)
    free = (x1[2:] > 0.0251) 
    assert np.all(np.abs(g1[2:][free]) < 1e-3)


def test_optimize_acqf_qei_end_to_end():
    from botorch_amd.acquisition import qExpectedImprovement
    from botorch_amd.models import SingleTaskGP
    from botorch_amd.optim import optimize_acqf
    from botorch_amd.sampling import SobolQMCNormalSampler
    X, Y = _data(64)
    m = SingleTaskGP(X.to(DEV), Y.to(DEV)).eval()
    acqf = qExpectedImprovement(m, Y.max().item(), sampler=SobolQMCNormalSampler(torch.Size([128]), seed=0))
    bounds = torch.stack([torch.zeros(6), torch.ones(6)]).to(torch.float64).to(DEV)
    from botorch_amd.optim import gen_batch_initial_conditions
    from botorch_amd.utils_sampling import draw_sobol_samples
    # MC qEI is exactly 0 wherever no QMC sample beats best_f: compare with the
    # best raw sample the driver itself starts from.
    raw = draw_sobol_samples(bounds.cpu(), n=256, q=3, seed=0)
    with torch.no_grad():
        base = acqf(raw.to(DEV)).max().item()
    assert base > 0
    cand, val = optimize_acqf(acqf, bounds, q=3, num_restarts=8, raw_samples=256,
                              options={"maxiter": 50, "seed": 0})
    assert cand.shape == (3, 6)
    assert (cand >= 0).all() and (cand <= 1).all()
    assert val.item() >= 0.9 * base
    with torch.no_grad():
        torch.testing.assert_close(acqf(cand.unsqueeze(0)).reshape(()), val.reshape(()))


@pytest.mark.parametrize("n,q,d,seed", [(20, 1, 6, 0), (64, 8, 6, 1), (32, 16, 6, 1)])
def test_device_sobol_box_matches_reference(golden, n, q, d, seed):
    """bo_sobol_box is bit-identical to the reference's draw_sobol_samples."""
    from botorch_amd import kernels
    bounds = torch.stack([torch.zeros(d), torch.ones(d)]).to(torch.float64).to(DEV)
    x = kernels.sobol_box(bounds, n, q, seed).cpu().numpy()
    np.testing.assert_array_equal(x, golden[f"sobol_box_n{n}_q{q}_d{d}_s{seed}"])
    # a non-unit box matches the host restatement bit for bit
    from botorch_amd.utils_sampling import draw_sobol_samples
    b2 = torch.tensor([[-2.0] * d, [3.5] * d], dtype=torch.float64)
    torch.testing.assert_close(kernels.sobol_box(b2.to(DEV), n, q, seed).cpu(),
                               draw_sobol_samples(b2, n, q, seed=seed), rtol=0, atol=0)


def test_device_sobol_box_unseeded_matches_reference():
    """seed=None (gen_batch_initial_conditions without options['seed']): the
    device raw designs equal draw_sobol_samples(seed=None), whose engine draws
    its scramble from the global CPU generator, under the same manual_seed,
    and leave that generator where the reference leaves it."""
    from oracle.sampling import draw_sobol_samples as oracle_draw
    from botorch_amd import kernels
    lo, hi = torch.full((6,), -1.0, dtype=torch.float64), torch.full((6,), 2.0, dtype=torch.float64)
    torch.manual_seed(11)
    x = kernels.sobol_box(torch.stack([lo, hi]).to(DEV), 40, 4, None).cpu()
    after = torch.rand(2)
    torch.manual_seed(11)
    ref = oracle_draw(lo, hi, 40, 4, None)
    assert torch.equal(torch.rand(2), after)
    torch.testing.assert_close(x, ref, rtol=0, atol=0)


def test_gen_batch_initial_conditions_on_device():
    """Raw designs, their forward-only values and the Boltzmann selection stay
    on the device; the picks are raw designs and include the best one."""
    from botorch_amd.acquisition import qExpectedImprovement, qLogExpectedImprovement
    from botorch_amd.models import SingleTaskGP
    from botorch_amd.optim import (evaluate_raw_samples, gen_batch_initial_conditions, initialize_q_batch,
                                   initialize_q_batch_nonneg)
    from botorch_amd.sampling import SobolQMCNormalSampler
    from botorch_amd.utils_sampling import draw_sobol_samples
    X, Y = _data(128)
    m = SingleTaskGP(X.to(DEV), Y.to(DEV)).eval()
    bounds = torch.stack([torch.zeros(6), torch.ones(6)]).to(torch.float64).to(DEV)
    for cls, bf in ((qExpectedImprovement, Y.max().item() - 0.5), (qLogExpectedImprovement, Y.max().item())):
        acqf = cls(m, bf, sampler=SobolQMCNormalSampler(torch.Size([64]), seed=0))
        torch.manual_seed(21)
        ics = gen_batch_initial_conditions(acqf, bounds, q=4, num_restarts=6, raw_samples=96,
                                           options={"seed": 3, "init_batch_limit": 40})
        assert ics.is_cuda and ics.shape == (6, 4, 6)
        raw = draw_sobol_samples(bounds.cpu(), 96, 4, seed=3)
        yr = evaluate_raw_samples(acqf, raw.to(DEV), 40).cpu()
        with torch.no_grad():
            torch.testing.assert_close(yr, acqf(raw.to(DEV)).cpu(), rtol=1e-12, atol=0)
        hits = [(raw == ic).all(-1).all(-1).nonzero().flatten().tolist() for ic in ics.cpu()]
        assert all(len(h) == 1 for h in hits)
        assert int(yr.argmax()) in [h[0] for h in hits]
        # the reference's host selection on the same values and generator state
        init = initialize_q_batch_nonneg if cls is qExpectedImprovement else initialize_q_batch
        torch.manual_seed(21)
        assert torch.equal(ics.cpu(), init(X=raw, Y=yr, n=6))
        torch.manual_seed(21)
        again = gen_batch_initial_conditions(acqf, bounds, q=4, num_restarts=6, raw_samples=96,
                                             options={"seed": 3, "init_batch_limit": 40})
        assert torch.equal(ics, again)


class _Quad(torch.nn.Module):
    """-(sum of squares to a target partly outside the box) per t-batch: the box
    solution is clamp(target)."""

    def __init__(self, target):
        super().__init__()
        self.target = target

    def forward(self, X):
        return -((X - self.target) ** 2).sum((-1, -2))


def test_device_lbfgs_box_quadratic():
    from botorch_amd.optim import gen_candidates_device
    torch.manual_seed(0)
    target = torch.tensor([[0.3, 1.4, -0.2], [0.9, 0.5, 2.0]], dtype=torch.float64, device=DEV)
    X0 = torch.rand(16, 2, 3, dtype=torch.float64, device=DEV)
    lo = torch.zeros(3, dtype=torch.float64, device=DEV)
    hi = torch.ones(3, dtype=torch.float64, device=DEV)
    c, v = gen_candidates_device(X0, _Quad(target), lo, hi, options={"maxiter": 100})
    st = gen_candidates_device.last_state
    assert (st.status.cpu() > 0).all()
    sol = target.clamp(0, 1).expand(16, 2, 3)
    torch.testing.assert_close(c, sol, atol=1e-7, rtol=0)
    assert (c >= 0).all() and (c <= 1).all()


def test_device_lbfgs_rosenbrock_matches_scipy():
    """Unbounded-inside-the-box Rosenbrock per restart: both optimisers reach the
    minimum (1, 1)."""
    from botorch_amd.optim import gen_candidates_device, gen_candidates_scipy

    class _Rosen(torch.nn.Module):
        def forward(self, X):
            x, y = X[..., 0, 0], X[..., 0, 1]
            return -((1 - x) ** 2 + 100 * (y - x * x) ** 2)

    g = torch.Generator().manual_seed(1)
    X0 = (torch.rand(8, 1, 2, generator=g, dtype=torch.float64) * 2 - 1).to(DEV)
    lo = torch.full((2,), -2.0, dtype=torch.float64, device=DEV)
    hi = torch.full((2,), 2.0, dtype=torch.float64, device=DEV)
    c, v = gen_candidates_device(X0, _Rosen(), lo, hi, options={"maxiter": 2000, "gtol": 1e-9,
                                                                 "ftol": 1e-15})
    torch.testing.assert_close(c.cpu(), torch.ones(8, 1, 2, dtype=torch.float64), atol=1e-4, rtol=0)
    cs, vs = gen_candidates_scipy(X0, _Rosen(), lo, hi, options={"maxiter": 2000})
    torch.testing.assert_close(v.cpu(), vs.cpu(), atol=1e-7, rtol=0)


def test_device_lbfgs_qei_reaches_scipy_values():
    """qEI restarts from the same initial conditions: the device optimiser ends at
    a KKT point at least as good as scipy's (per restart, up to 1e-6 relative
    of the best value)."""
    from botorch_amd.acquisition import qExpectedImprovement
    from botorch_amd.models import SingleTaskGP
    from botorch_amd.optim import (gen_batch_initial_conditions, gen_candidates_device,
                                   gen_candidates_scipy)
    from botorch_amd.sampling import SobolQMCNormalSampler
    X, Y = _data(128)
    m = SingleTaskGP(X.to(DEV), Y.to(DEV)).eval()
    acqf = qExpectedImprovement(m, Y.max().item() - 0.2, sampler=SobolQMCNormalSampler(torch.Size([128]), seed=0))
    bounds = torch.stack([torch.zeros(6), torch.ones(6)]).to(torch.float64).to(DEV)
    ics = gen_batch_initial_conditions(acqf, bounds, q=2, num_restarts=8, raw_samples=128,
                                       options={"seed": 1})
    cd, vd = gen_candidates_device(ics, acqf, bounds[0], bounds[1], options={"maxiter": 300})
    cs, vs = gen_candidates_scipy(ics, acqf, bounds[0], bounds[1], options={"maxiter": 300})
    assert cd.shape == cs.shape == (8, 2, 6)
    assert (cd >= 0).all() and (cd <= 1).all()
    # the best restart of each agrees; no device restart ends below its start
    assert vd.max().item() >= vs.max().item() * (1 - 1e-6) - 1e-9
    with torch.no_grad():
        v0 = acqf(ics)
    assert (vd >= v0 - 1e-12).all()
    st = gen_candidates_device.last_state
    assert (st.nit.cpu() > 0).any()


def test_fit_rejects_nan_training_data():
    """NaN inputs raise NanError once, before the first closure (the closure
    itself skips the per-evaluation check)."""
    from botorch_amd.exceptions import NanError
    from botorch_amd.fit import ExactMarginalLogLikelihood, fit_gpytorch_mll_scipy
    from botorch_amd.models import SingleTaskGP
    X = torch.rand(40, 6, dtype=torch.float64)
    Y = X.sum(dim=-1, keepdim=True)
    m = SingleTaskGP(X.to(DEV), Y.to(DEV))
    m.train_inputs[0][3, 2] = float("nan")
    with pytest.raises(NanError):
        fit_gpytorch_mll_scipy(ExactMarginalLogLikelihood(m.likelihood, m))
