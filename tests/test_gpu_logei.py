"""qLogEI / qLogNEI (acquisition/logei.py) on the fused gfx950 path vs. the
oracle restatement (pinned by tests/test_logei_golden.py), values and gradients."""
import pytest
import torch

from tests.test_gpu_acquisition import DEV, _setup

pytestmark = pytest.mark.gpu

CASES = {  # (fat, tau_relu, tau_max)
    "default": (True, 1e-6, 1e-2),
    "nofat": (False, 1e-6, 1e-2),
    "fat_wide": (True, 0.1, 0.5),
}


@pytest.mark.parametrize("tag", list(CASES))
@pytest.mark.parametrize("B,q,S,shift", [(16, 4, 128, 0.0), (9, 16, 256, 0.3), (5, 1, 64, 0.0),
                                         (7, 3, 512, 0.5)])
def test_qlogei_value(tag, B, q, S, shift):
    from botorch_amd.acquisition import qLogExpectedImprovement
    from botorch_amd.sampling import SobolQMCNormalSampler
    from oracle.acquisition import qlogei
    from oracle.sampling import draw_sobol_normal_samples
    fat, tau_relu, tau_max = CASES[tag]
    X, Y, m, orc = _setup()
    best_f = Y.max().item() - shift
    acqf = qLogExpectedImprovement(m, best_f, sampler=SobolQMCNormalSampler(torch.Size([S]), seed=5),
                                   fat=fat, tau_relu=tau_relu, tau_max=tau_max)
    g = torch.Generator().manual_seed(B * 100 + q)
    Xc = torch.rand(B, q, 6, generator=g, dtype=torch.float64)
    with torch.no_grad():
        v = acqf(Xc.to(DEV)).cpu()
    ref = qlogei(orc, Xc, draw_sobol_normal_samples(q, S, 5), best_f, fat=fat, tau_relu=tau_relu,
                 tau_max=tau_max)
    assert torch.isfinite(v).all()
    torch.testing.assert_close(v, ref, rtol=1e-6, atol=1e-8)


@pytest.mark.parametrize("tag", list(CASES))
@pytest.mark.parametrize("B,q", [(8, 4), (3, 16), (4, 1)])
def test_qlogei_gradient(tag, B, q):
    from botorch_amd.acquisition import qLogExpectedImprovement
    from botorch_amd.sampling import SobolQMCNormalSampler
    from oracle.acquisition import qlogei
    from oracle.sampling import draw_sobol_normal_samples
    fat, tau_relu, tau_max = CASES[tag]
    X, Y, m, orc = _setup()
    best_f = Y.max().item() - 0.2
    S = 128
    acqf = qLogExpectedImprovement(m, best_f, sampler=SobolQMCNormalSampler(torch.Size([S]), seed=2),
                                   fat=fat, tau_relu=tau_relu, tau_max=tau_max)
    g = torch.Generator().manual_seed(B * 10 + q)
    Xc = torch.rand(B, q, 6, generator=g, dtype=torch.float64)
    Xd = Xc.to(DEV).requires_grad_(True)
    val = acqf(Xd)
    (gd,) = torch.autograd.grad(val.sum(), Xd)
    Xo = Xc.clone().requires_grad_(True)
    ref = qlogei(orc, Xo, draw_sobol_normal_samples(q, S, 2), best_f, fat=fat, tau_relu=tau_relu,
                 tau_max=tau_max)
    (go,) = torch.autograd.grad(ref.sum(), Xo)
    torch.testing.assert_close(val.detach().cpu(), ref.detach(), rtol=1e-6, atol=1e-8)
    assert go.abs().max() > 0
    torch.testing.assert_close(gd.cpu(), go, rtol=1e-5, atol=1e-8)


def test_qlogei_generic_route_q_gt_16():
    """q > 16 leaves the fused kernel: device posterior + sampler + the torch
    LogEI reductions (botorch_amd/safe_math.py)."""
    from botorch_amd.acquisition import qLogExpectedImprovement
    from botorch_amd.sampling import SobolQMCNormalSampler
    from oracle.acquisition import qlogei
    from oracle.sampling import draw_sobol_normal_samples
    X, Y, m, orc = _setup()
    best_f = Y.max().item()
    S, q = 64, 20
    acqf = qLogExpectedImprovement(m, best_f, sampler=SobolQMCNormalSampler(torch.Size([S]), seed=4))
    Xc = torch.rand(3, q, 6, dtype=torch.float64)
    with torch.no_grad():
        v = acqf(Xc.to(DEV)).cpu()
    ref = qlogei(orc, Xc, draw_sobol_normal_samples(q, S, 4), best_f)
    torch.testing.assert_close(v, ref, rtol=1e-5, atol=1e-8)


@pytest.mark.parametrize("tag", ["default", "nofat"])
@pytest.mark.parametrize("r,B,q,S", [(40, 8, 4, 128), (25, 6, 16, 64), (12, 16, 1, 128)])
def test_qlognei_value_and_gradient(tag, r, B, q, S):
    from botorch_amd.acquisition import qLogNoisyExpectedImprovement
    from botorch_amd.sampling import SobolQMCNormalSampler
    from oracle.acquisition import QNEIOracle, qlognei
    fat, tau_relu, tau_max = CASES[tag]
    X, Y, m, orc = _setup(n=200, noise=1e-2)
    Xb = X[:r]
    acqf = qLogNoisyExpectedImprovement(m, Xb.to(DEV), sampler=SobolQMCNormalSampler(torch.Size([S]), seed=5),
                                        fat=fat, tau_relu=tau_relu, tau_max=tau_max)
    ref = QNEIOracle(orc, Xb, S, seed=5)
    g = torch.Generator().manual_seed(200 + r)
    Xc = torch.rand(B, q, 6, generator=g, dtype=torch.float64)
    Xd = Xc.to(DEV).requires_grad_(True)
    v = acqf(Xd)
    (gd,) = torch.autograd.grad(v.sum(), Xd)
    Xo = Xc.clone().requires_grad_(True)
    rv = qlognei(ref, Xo, fat=fat, tau_relu=tau_relu, tau_max=tau_max)
    (go,) = torch.autograd.grad(rv.sum(), Xo)
    torch.testing.assert_close(v.detach().cpu(), rv.detach(), rtol=1e-6, atol=1e-8)
    assert go.abs().max() > 0
    torch.testing.assert_close(gd.cpu(), go, rtol=1e-5, atol=1e-8)
