"""Public API (models / posteriors / samplers / acquisition) on the GPU vs. the oracle,
values and gradients."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _setup(n=256, d=6, seed=0, ls=0.35, noise=1e-3, const=0.1):
    from botorch_amd.models import SingleTaskGP
    from botorch_amd.test_functions import Hartmann
    from oracle.gp import ExactGPOracle, GPHyper
    from oracle.sampling import draw_sobol_samples
    lo = torch.zeros(d, dtype=torch.float64)
    X = draw_sobol_samples(lo, lo + 1, n, 1, seed).squeeze(1)
    Y = Hartmann(negate=True)(X[:, :6]).unsqueeze(-1)
    m = SingleTaskGP(X.to(DEV), Y.to(DEV))
    m.covar_module.lengthscale = torch.full((1, d), ls, dtype=torch.float64)
    m.likelihood.noise = torch.tensor([noise], dtype=torch.float64)
    m.mean_module.constant = const
    m.eval()
    orc = ExactGPOracle(X, Y, GPHyper(torch.full((d,), ls, dtype=torch.float64), noise, const))
    return X, Y, m, orc


def test_posterior_api_matches_oracle():
    X, Y, m, orc = _setup()
    Xc = torch.rand(7, 5, 6, dtype=torch.float64)
    post = m.posterior(Xc.to(DEV))
    assert post.mean.shape == (7, 5, 1) and post.variance.shape == (7, 5, 1)
    mr, cr = orc.posterior(Xc)
    torch.testing.assert_close(post.mean.squeeze(-1).cpu(), mr, rtol=1e-4, atol=1e-9)
    torch.testing.assert_close(post.variance.squeeze(-1).cpu(), cr.diagonal(dim1=-2, dim2=-1), rtol=1e-4, atol=1e-10)
    # 2-d input (q x d) -> batch shape ()
    p2 = m.posterior(Xc[0].to(DEV))
    assert p2.mean.shape == (5, 1)
    # observation noise adds s^2 sigma^2 (test/models/test_gp_regression.py:131-157)
    pn = m.posterior(Xc.to(DEV), observation_noise=True)
    diff = (pn.variance - post.variance).cpu()
    torch.testing.assert_close(diff, torch.full_like(diff, 1e-3 * orc.ystd.item() ** 2), rtol=1e-9, atol=1e-12)


def test_posterior_gradient_matches_oracle():
    X, Y, m, orc = _setup()
    g = torch.Generator().manual_seed(3)
    Xc = torch.rand(6, 4, 6, generator=g, dtype=torch.float64)
    Xd = Xc.to(DEV).requires_grad_(True)
    post = m.posterior(Xd)
    loss = (post.mean.sum() + 3.0 * post.variance.sum()
            + 0.7 * post.covariance_matrix[..., 0, 1].sum())
    (gd,) = torch.autograd.grad(loss, Xd)
    Xo = Xc.clone().requires_grad_(True)
    mr, cr = orc.posterior(Xo)
    lo = mr.sum() + 3.0 * cr.diagonal(dim1=-2, dim2=-1).sum() + 0.7 * cr[..., 0, 1].sum()
    (go,) = torch.autograd.grad(lo, Xo)
    torch.testing.assert_close(gd.cpu(), go, rtol=1e-5, atol=1e-8)


def test_posterior_general_path_q_gt_16():
    X, Y, m, orc = _setup()
    Xc = torch.rand(2, 20, 6, dtype=torch.float64)
    post = m.posterior(Xc.to(DEV))
    mr, cr = orc.posterior(Xc)
    torch.testing.assert_close(post.mean.squeeze(-1).cpu(), mr, rtol=1e-4, atol=1e-9)
    torch.testing.assert_close(post.covariance_matrix.cpu(), cr, rtol=1e-4, atol=1e-9)


# q = 7 / 9-15: the q x q ladder's 8- and 16-wide entry layouts with rows
# past q masked (qmc.hip ladder_factor); S = 300 / 512 the grouped sampling
@pytest.mark.parametrize("B,q,S", [(16, 4, 128), (40, 8, 256), (9, 16, 64), (5, 1, 32), (3, 3, 16),
                                   (7, 7, 64), (6, 9, 128), (4, 12, 512), (3, 13, 300), (5, 15, 64)])
def test_qei_api_value(B, q, S):
    from botorch_amd.acquisition import qExpectedImprovement
    from botorch_amd.sampling import SobolQMCNormalSampler
    from oracle.acquisition import qei
    from oracle.sampling import draw_sobol_normal_samples
    X, Y, m, orc = _setup()
    best_f = Y.max().item()
    acqf = qExpectedImprovement(m, best_f, sampler=SobolQMCNormalSampler(torch.Size([S]), seed=5))
    Xc = torch.rand(B, q, 6, dtype=torch.float64)
    with torch.no_grad():
        v = acqf(Xc.to(DEV)).cpu()
    ref = qei(orc, Xc, draw_sobol_normal_samples(q, S, 5), best_f)
    torch.testing.assert_close(v, ref, rtol=1e-6, atol=1e-10)


@pytest.mark.parametrize("B,q", [(8, 4), (3, 16), (4, 1), (2, 5), (3, 11)])
def test_qei_gradient_matches_oracle(B, q):
    from botorch_amd.acquisition import qExpectedImprovement
    from botorch_amd.sampling import SobolQMCNormalSampler
    from oracle.acquisition import qei
    from oracle.sampling import draw_sobol_normal_samples
    X, Y, m, orc = _setup()
    best_f = Y.max().item() - 0.3  # plenty of positive improvement
    S = 128
    acqf = qExpectedImprovement(m, best_f, sampler=SobolQMCNormalSampler(torch.Size([S]), seed=2))
    g = torch.Generator().manual_seed(B * 10 + q)
    Xc = torch.rand(B, q, 6, generator=g, dtype=torch.float64)
    Xd = Xc.to(DEV).requires_grad_(True)
    val = acqf(Xd)
    (gd,) = torch.autograd.grad(val.sum(), Xd)
    Xo = Xc.clone().requires_grad_(True)
    ref = qei(orc, Xo, draw_sobol_normal_samples(q, S, 2), best_f)
    (go,) = torch.autograd.grad(ref.sum(), Xo)
    torch.testing.assert_close(val.detach().cpu(), ref.detach(), rtol=1e-6, atol=1e-10)
    torch.testing.assert_close(gd.cpu(), go, rtol=1e-5, atol=1e-8)


def test_analytic_ei_value_and_grad():
    from botorch_amd.acquisition import ExpectedImprovement
    from oracle.acquisition import ei_analytic
    X, Y, m, orc = _setup()
    best_f = Y.max().item()
    Xc = torch.rand(11, 1, 6, dtype=torch.float64)
    Xd = Xc.to(DEV).requires_grad_(True)
    v = ExpectedImprovement(m, best_f)(Xd)
    (gd,) = torch.autograd.grad(v.sum(), Xd)
    Xo = Xc.clone().requires_grad_(True)
    r = ei_analytic(orc, Xo, best_f)
    (go,) = torch.autograd.grad(r.sum(), Xo)
    torch.testing.assert_close(v.detach().cpu(), r.detach(), rtol=1e-5, atol=1e-10)
    torch.testing.assert_close(gd.cpu(), go, rtol=1e-4, atol=1e-8)


def test_sampler_base_samples_match_reference(golden):
    from botorch_amd.sampling import SobolQMCNormalSampler
    X, Y, m, orc = _setup()
    s = SobolQMCNormalSampler(torch.Size([256]), seed=0)
    post = m.posterior(torch.rand(4, 8, 6, dtype=torch.float64, device=DEV))
    samples = s(post)
    assert samples.shape == (256, 4, 8, 1)
    assert s.base_samples.shape == (256, 1, 8)
    np.testing.assert_allclose(s.base_samples.squeeze(1).cpu().numpy(),
                               golden["sobol_normal_d8_n256_s0"], rtol=4e-15, atol=4e-15)


@pytest.mark.parametrize("q", [3, 16, 40, 150])
def test_chol_jitter_batched(q):
    from botorch_amd import kernels
    g = torch.Generator().manual_seed(q)
    M = torch.randn(5, q, q, generator=g, dtype=torch.float64)
    A = M @ M.mT + 0.1 * torch.eye(q, dtype=torch.float64)
    L = kernels.chol_jitter(A.to(DEV)).cpu()
    torch.testing.assert_close(L, torch.linalg.cholesky(A), rtol=1e-9, atol=1e-11)


def test_chol_jitter_ladder_matches_reference_semantics():
    """A singular PSD member gets the smallest sufficient jitter; others none."""
    from botorch_amd import kernels
    from botorch_amd.exceptions import NumericalWarning
    from oracle.gp import psd_safe_cholesky
    v = torch.tensor([[1.0, 2.0, 3.0]], dtype=torch.float64)
    A = torch.stack([v.T @ v, torch.eye(3, dtype=torch.float64)])
    with pytest.warns(NumericalWarning):
        L = kernels.chol_jitter(A.to(DEV)).cpu()
    Lr, jit = psd_safe_cholesky(A)
    torch.testing.assert_close(L, Lr, rtol=1e-7, atol=1e-9)


@pytest.mark.parametrize("r,B,q,S", [(40, 16, 4, 128), (90, 12, 16, 256), (20, 5, 1, 64)])
def test_qnei_cached_root_matches_oracle(r, B, q, S):
    """qNEI (prune_baseline=False, cache_root=True) vs. the oracle's restatement of
    sample_cached_cholesky; tolerance of north_star: 1e-2 on MC values."""
    from botorch_amd.acquisition import qNoisyExpectedImprovement
    from botorch_amd.sampling import SobolQMCNormalSampler
    from oracle.acquisition import QNEIOracle
    X, Y, m, orc = _setup(n=200, noise=1e-2)
    Xb = X[:r]
    acqf = qNoisyExpectedImprovement(m, Xb.to(DEV), sampler=SobolQMCNormalSampler(torch.Size([S]), seed=11),
                                     prune_baseline=False)
    ref = QNEIOracle(orc, Xb, S, seed=11)
    torch.testing.assert_close(acqf._baseline_best_f.cpu(), ref.best_f, rtol=1e-6, atol=1e-8)
    g = torch.Generator().manual_seed(r)
    Xc = torch.rand(B, q, 6, generator=g, dtype=torch.float64)
    with torch.no_grad():
        v = acqf(Xc.to(DEV)).cpu()
    rv = ref(Xc)
    torch.testing.assert_close(v, rv, rtol=1e-2, atol=1e-6)
    torch.testing.assert_close(v, rv, rtol=1e-5, atol=1e-8)


@pytest.mark.parametrize("r,B,q,S", [(40, 8, 4, 128), (25, 6, 16, 64), (12, 16, 2, 128)])
def test_qnei_gradient_matches_oracle(r, B, q, S):
    """d qNEI / dX through the cached-root path (utils/low_rank.py:85-173
    differentiated) vs. torch autograd through the oracle restatement."""
    from botorch_amd.acquisition import qNoisyExpectedImprovement
    from botorch_amd.sampling import SobolQMCNormalSampler
    from oracle.acquisition import QNEIOracle
    X, Y, m, orc = _setup(n=200, noise=1e-2)
    Xb = X[:r]
    acqf = qNoisyExpectedImprovement(m, Xb.to(DEV), sampler=SobolQMCNormalSampler(torch.Size([S]), seed=5),
                                     prune_baseline=False)
    ref = QNEIOracle(orc, Xb, S, seed=5)
    g = torch.Generator().manual_seed(100 + r)
    Xc = torch.rand(B, q, 6, generator=g, dtype=torch.float64)
    Xd = Xc.to(DEV).requires_grad_(True)
    v = acqf(Xd)
    (gd,) = torch.autograd.grad(v.sum(), Xd)
    Xo = Xc.clone().requires_grad_(True)
    rv = ref(Xo)
    (go,) = torch.autograd.grad(rv.sum(), Xo)
    torch.testing.assert_close(v.detach().cpu(), rv.detach(), rtol=1e-5, atol=1e-8)
    assert go.abs().max() > 0
    torch.testing.assert_close(gd.cpu(), go, rtol=1e-5, atol=1e-8)


def test_prune_inferior_points_matches_oracle():
    from botorch_amd.acquisition import prune_inferior_points
    from botorch_amd.sampling import SobolQMCNormalSampler
    from oracle.acquisition import prune_inferior_points as prune_ref
    X, Y, m, orc = _setup(n=300, noise=1e-2)
    kept = prune_inferior_points(m, X.to(DEV), sampler=SobolQMCNormalSampler(torch.Size([512]), seed=3))
    ref = prune_ref(orc, X, num_samples=512, seed=3)
    assert kept.shape == ref.shape
    torch.testing.assert_close(kept.cpu(), ref)


@pytest.mark.parametrize("B,q,S", [(6, 2, 64), (4, 4, 128)])
def test_qehvi_api_matches_oracle(golden, B, q, S):
    from botorch_amd.acquisition import qExpectedHypervolumeImprovement
    from botorch_amd.models import ModelListGP, SingleTaskGP
    from botorch_amd.multi_objective import FastNondominatedPartitioning
    from botorch_amd.sampling import SobolQMCNormalSampler
    from oracle.acquisition import qehvi
    from oracle.gp import ExactGPOracle, GPHyper
    from oracle.sampling import base_samples_multi_output
    X = torch.from_numpy(golden["dtlz2_X"][:96])
    Y = torch.from_numpy(golden["dtlz2_Y"][:96])
    models, oracles = [], []
    for t in range(3):
        mdl = SingleTaskGP(X.to(DEV), Y[:, t:t + 1].to(DEV))
        mdl.covar_module.lengthscale = torch.full((1, 6), 0.6, dtype=torch.float64)
        mdl.likelihood.noise = torch.tensor([1e-3], dtype=torch.float64)
        models.append(mdl.eval())
        oracles.append(ExactGPOracle(X, Y[:, t:t + 1], GPHyper(torch.full((6,), 0.6, dtype=torch.float64), 1e-3, 0.0)))
    ref_point = torch.full((3,), -1.1, dtype=torch.float64)
    part = FastNondominatedPartitioning(ref_point, Y)
    acqf = qExpectedHypervolumeImprovement(ModelListGP(*models), ref_point.tolist(), part,
                                           sampler=SobolQMCNormalSampler(torch.Size([S]), seed=4))
    g = torch.Generator().manual_seed(q)
    Xc = torch.rand(B, q, 6, generator=g, dtype=torch.float64)
    with torch.no_grad():
        v = acqf(Xc.to(DEV)).cpu()
    lo, hi = part.get_hypercell_bounds()
    ref = qehvi(oracles, Xc, base_samples_multi_output(S, q, 3, 4), lo, hi)
    torch.testing.assert_close(v, ref, rtol=1e-2, atol=1e-8)
    torch.testing.assert_close(v, ref, rtol=1e-7, atol=1e-10)


@pytest.mark.parametrize("B,q,S", [(5, 2, 64), (3, 4, 128), (2, 8, 32)])
def test_qehvi_gradient_matches_oracle(golden, B, q, S):
    """d qEHVI / dX (bo_qehvi_backward + bo_chol_backward + bo_post_backward per
    output) vs. torch autograd through the oracle's _compute_qehvi restatement."""
    from botorch_amd.acquisition import qExpectedHypervolumeImprovement
    from botorch_amd.models import ModelListGP, SingleTaskGP
    from botorch_amd.multi_objective import FastNondominatedPartitioning
    from botorch_amd.sampling import SobolQMCNormalSampler
    from oracle.acquisition import qehvi
    from oracle.gp import ExactGPOracle, GPHyper
    from oracle.sampling import base_samples_multi_output
    X = torch.from_numpy(golden["dtlz2_X"][:96])
    Y = torch.from_numpy(golden["dtlz2_Y"][:96])
    models, oracles = [], []
    for t in range(3):
        mdl = SingleTaskGP(X.to(DEV), Y[:, t:t + 1].to(DEV))
        mdl.covar_module.lengthscale = torch.full((1, 6), 0.6, dtype=torch.float64)
        mdl.likelihood.noise = torch.tensor([1e-3], dtype=torch.float64)
        models.append(mdl.eval())
        oracles.append(ExactGPOracle(X, Y[:, t:t + 1], GPHyper(torch.full((6,), 0.6, dtype=torch.float64), 1e-3, 0.0)))
    ref_point = torch.full((3,), -1.1, dtype=torch.float64)
    part = FastNondominatedPartitioning(ref_point, Y)
    acqf = qExpectedHypervolumeImprovement(ModelListGP(*models), ref_point.tolist(), part,
                                           sampler=SobolQMCNormalSampler(torch.Size([S]), seed=9))
    g = torch.Generator().manual_seed(50 + q)
    Xc = torch.rand(B, q, 6, generator=g, dtype=torch.float64)
    Xd = Xc.to(DEV).requires_grad_(True)
    v = acqf(Xd)
    (gd,) = torch.autograd.grad(v.sum(), Xd)
    lo, hi = part.get_hypercell_bounds()
    Xo = Xc.clone().requires_grad_(True)
    ref = qehvi(oracles, Xo, base_samples_multi_output(S, q, 3, 9), lo, hi)
    (go,) = torch.autograd.grad(ref.sum(), Xo)
    torch.testing.assert_close(v.detach().cpu(), ref.detach(), rtol=1e-7, atol=1e-10)
    assert go.abs().max() > 0
    torch.testing.assert_close(gd.cpu(), go, rtol=1e-5, atol=1e-8)
    # the backward reduces per sample in a fixed order: bitwise reproducible
    for _ in range(2):
        (g2,) = torch.autograd.grad(acqf(Xd).sum(), Xd)
        assert torch.equal(g2, gd)


@pytest.mark.parametrize("d,M,q", [(50, 16, 4), (10, 3, 2)])
def test_saas_qei_matches_oracle(d, M, q):
    """C5 shape: SAAS ensemble of M Matern-5/2 GPs, d=50, qEI averaged over MCMC_DIM."""
    from botorch_amd.acquisition import qExpectedImprovement
    from botorch_amd.models import SaasFullyBayesianSingleTaskGP, sample_saas_prior
    from botorch_amd.sampling import SobolQMCNormalSampler
    from botorch_amd.test_functions import Hartmann
    from oracle.acquisition import saas_members, saas_qei
    from oracle.sampling import base_samples_single_output, draw_sobol_samples
    n, S, B = 256, 256, 12
    lo = torch.zeros(d, dtype=torch.float64)
    X = draw_sobol_samples(lo, lo + 1, n, 1, 0).squeeze(1)
    Y = Hartmann(negate=True)(X[:, :6]).unsqueeze(-1)
    Y = (Y - Y.mean()) / Y.std()
    smp = sample_saas_prior(d, M, seed=0)
    m = SaasFullyBayesianSingleTaskGP(X.to(DEV), Y.to(DEV))
    m.load_mcmc_samples({k: v.to(DEV) for k, v in smp.items()})
    m.eval()
    Xc = draw_sobol_samples(lo, lo + 1, B, q, 1)
    post = m.posterior(Xc.to(DEV))
    assert post.mean.shape == (B, M, q, 1)
    members = saas_members(X, Y, smp)
    mr = torch.stack([mm.posterior(Xc)[0] for mm in members], dim=1)
    torch.testing.assert_close(post.mean.squeeze(-1).cpu(), mr, rtol=1e-4, atol=1e-8)
    best_f = float(Y.max())
    acqf = qExpectedImprovement(m, best_f, sampler=SobolQMCNormalSampler(torch.Size([S]), seed=0))
    with torch.no_grad():
        val = acqf(Xc.to(DEV)).cpu()
    assert val.shape == (B,)
    ref = saas_qei(members, Xc, base_samples_single_output(S, q, 0), best_f)
    torch.testing.assert_close(val, ref, rtol=1e-2, atol=1e-6)


@pytest.mark.parametrize("d,M,q", [(50, 4, 3), (10, 3, 2)])
def test_saas_qei_gradient_matches_oracle(d, M, q):
    """d qEI / dX over the SAAS ensemble (generic-d path: bo_kernel_grad) vs. torch
    autograd through the oracle members."""
    from botorch_amd.acquisition import qExpectedImprovement
    from botorch_amd.models import SaasFullyBayesianSingleTaskGP, sample_saas_prior
    from botorch_amd.sampling import SobolQMCNormalSampler
    from botorch_amd.test_functions import Hartmann
    from oracle.acquisition import saas_members, saas_qei
    from oracle.sampling import base_samples_single_output, draw_sobol_samples
    n, S, B = 64, 128, 6
    lo = torch.zeros(d, dtype=torch.float64)
    X = draw_sobol_samples(lo, lo + 1, n, 1, 0).squeeze(1)
    Y = Hartmann(negate=True)(X[:, :6]).unsqueeze(-1)
    Y = (Y - Y.mean()) / Y.std()
    smp = sample_saas_prior(d, M, seed=1)
    m = SaasFullyBayesianSingleTaskGP(X.to(DEV), Y.to(DEV))
    m.load_mcmc_samples({k: v.to(DEV) for k, v in smp.items()})
    m.eval()
    best_f = float(Y.median())
    acqf = qExpectedImprovement(m, best_f, sampler=SobolQMCNormalSampler(torch.Size([S]), seed=2))
    Xc = draw_sobol_samples(lo, lo + 1, B, q, 3)
    Xd = Xc.to(DEV).requires_grad_(True)
    v = acqf(Xd)
    (gd,) = torch.autograd.grad(v.sum(), Xd)
    members = saas_members(X, Y, smp)
    Xo = Xc.clone().requires_grad_(True)
    ref = saas_qei(members, Xo, base_samples_single_output(S, q, 2), best_f)
    (go,) = torch.autograd.grad(ref.sum(), Xo)
    torch.testing.assert_close(v.detach().cpu(), ref.detach(), rtol=1e-6, atol=1e-9)
    assert go.abs().max() > 0
    torch.testing.assert_close(gd.cpu(), go, rtol=1e-5, atol=1e-8)


def test_qei_edge_shapes():
    """Empty t-batch, extra batch dimensions, a ragged n (not a multiple of 128)."""
    from botorch_amd.acquisition import qExpectedImprovement
    from botorch_amd.sampling import SobolQMCNormalSampler
    from oracle.acquisition import qei
    from oracle.sampling import draw_sobol_normal_samples
    X, Y, m, orc = _setup(n=300)
    best_f = Y.max().item()
    acqf = qExpectedImprovement(m, best_f, sampler=SobolQMCNormalSampler(torch.Size([64]), seed=3))
    with torch.no_grad():
        v0 = acqf(torch.empty(0, 4, 6, dtype=torch.float64, device=DEV))
        assert v0.shape == (0,)
        Xc = torch.rand(2, 3, 4, 6, dtype=torch.float64)
        v = acqf(Xc.to(DEV)).cpu()
    assert v.shape == (2, 3)
    ref = qei(orc, Xc.reshape(6, 4, 6), draw_sobol_normal_samples(4, 64, 3), best_f).reshape(2, 3)
    torch.testing.assert_close(v, ref, rtol=1e-6, atol=1e-10)
    post = m.posterior(torch.empty(0, 4, 6, dtype=torch.float64, device=DEV))
    assert post.mean.shape == (0, 4, 1)


def test_empty_batches_all_acquisitions(golden):
    """A zero-size t-batch returns an empty value for every fused acquisition."""
    from botorch_amd.acquisition import (qExpectedHypervolumeImprovement, qLogExpectedImprovement,
                                         qLogNoisyExpectedImprovement, qNoisyExpectedImprovement)
    from botorch_amd.models import ModelListGP, SingleTaskGP
    from botorch_amd.multi_objective import FastNondominatedPartitioning
    from botorch_amd.sampling import SobolQMCNormalSampler
    X, Y, m, orc = _setup(n=200, noise=1e-2)
    empty = torch.empty(0, 3, 6, dtype=torch.float64, device=DEV)
    acqfs = [qLogExpectedImprovement(m, Y.max().item()),
             qNoisyExpectedImprovement(m, X[:20].to(DEV), prune_baseline=False),
             qLogNoisyExpectedImprovement(m, X[:20].to(DEV))]
    Xm = torch.from_numpy(golden["dtlz2_X"][:64])
    Ym = torch.from_numpy(golden["dtlz2_Y"][:64])
    models = [SingleTaskGP(Xm.to(DEV), Ym[:, t:t + 1].to(DEV)).eval() for t in range(3)]
    ref_point = torch.full((3,), -1.1, dtype=torch.float64)
    acqfs.append(qExpectedHypervolumeImprovement(
        ModelListGP(*models), ref_point.tolist(), FastNondominatedPartitioning(ref_point, Ym),
        sampler=SobolQMCNormalSampler(torch.Size([32]), seed=0)))
    with torch.no_grad():
        for a in acqfs:
            v = a(empty)
            assert v.shape == (0,), type(a).__name__


@pytest.mark.parametrize("B,q", [(64, 16), (128, 8)])
def test_qei_gradient_post_w_path(B, q):
    """Grids of 8 x 8 super-tiles (n = 1024, B * Qp = 1024) can take W^T =
    L^{-T} R^T from bo_post_w instead of the GEMM: W (forced) against the GEMM
    route, and the qEI value and gradient through the API (GEMM route at this
    grid size) against the oracle."""
    from botorch_amd import _lib, kernels
    from botorch_amd.acquisition import qExpectedImprovement
    from botorch_amd.sampling import SobolQMCNormalSampler
    from oracle.acquisition import qei
    from oracle.sampling import draw_sobol_normal_samples
    X, Y, m, orc = _setup(n=1024)
    g = torch.Generator().manual_seed(B + q)
    Xc = torch.rand(B, q, 6, generator=g, dtype=torch.float64)
    cache = m.prediction_cache()
    pp = kernels.post_partials(cache, Xc.to(DEV), store_R=True)
    assert pp.nC % 8 == 0 and (pp.nrows_pad // 128) % 8 == 0
    W = kernels.w_matrix(cache, pp, post_w=True)
    assert W.kmajor and W.t.shape == (cache.np, pp.nrows_pad)
    Wg = kernels.gemm(pp.Rt, cache.U, transA=True, transB=True, flags=_lib.GEMM_B_LOWER)
    torch.testing.assert_close(W.t.T.cpu(), Wg.cpu(), rtol=1e-10, atol=1e-11)
    # post_backward reading W^T k-major == reading W row-major
    dmean = torch.randn(B, q, generator=g, dtype=torch.float64).to(DEV)
    dcov = torch.randn(B, q, q, generator=g, dtype=torch.float64).to(DEV)
    dx_k = kernels.post_backward(cache, pp, W, dmean, dcov, 0.7)
    dx_r = kernels.post_backward(cache, pp, kernels.WMat(Wg, False), dmean, dcov, 0.7)
    torch.testing.assert_close(dx_k, dx_r, rtol=1e-10, atol=1e-12)

    best_f = Y.max().item() - 0.3
    S = 64
    acqf = qExpectedImprovement(m, best_f, sampler=SobolQMCNormalSampler(torch.Size([S]), seed=3))
    Xd = Xc.to(DEV).requires_grad_(True)
    val = acqf(Xd)
    (gd,) = torch.autograd.grad(val.sum(), Xd)
    Xo = Xc.clone().requires_grad_(True)
    ref = qei(orc, Xo, draw_sobol_normal_samples(q, S, 3), best_f)
    (go,) = torch.autograd.grad(ref.sum(), Xo)
    torch.testing.assert_close(val.detach().cpu(), ref.detach(), rtol=1e-6, atol=1e-10)
    torch.testing.assert_close(gd.cpu(), go, rtol=1e-5, atol=1e-8)


def test_post_w_full_size_matches_gemm():
    """bo_post_w at the C3 training size (n = 4096, 32 column tiles, the
    mirrored heaviest-first schedule) against the triangular GEMM route."""
    from botorch_amd import _lib, kernels
    X, Y, m, orc = _setup(n=4096)
    g = torch.Generator().manual_seed(7)
    Xc = torch.rand(64, 16, 6, generator=g, dtype=torch.float64)
    cache = m.prediction_cache()
    pp = kernels.post_partials(cache, Xc.to(DEV), store_R=True)
    W = kernels.w_matrix(cache, pp, post_w=True)
    assert W.kmajor
    Wg = kernels.gemm(pp.Rt, cache.U, transA=True, transB=True, flags=_lib.GEMM_B_LOWER)
    torch.testing.assert_close(W.t.T, Wg, rtol=1e-10, atol=1e-10)


def test_qei_forward_only_ladder_status_is_deferred():
    """Forward-only fused qEI: the jitter-ladder status is read one call later
    (or at check_ladder_status / the optimiser's sync), not in the call; the
    warning of a jittered q x q root still reaches the caller."""
    import warnings
    from botorch_amd import kernels
    from botorch_amd.acquisition import qExpectedImprovement
    from botorch_amd.exceptions import NumericalWarning
    from botorch_amd.sampling import SobolQMCNormalSampler
    X, Y, m, orc = _setup(n=64, noise=1e-4)
    m.likelihood.noise = torch.tensor([1e-12], dtype=torch.float64)
    m.eval()
    acqf = qExpectedImprovement(m, Y.max().item(), sampler=SobolQMCNormalSampler(torch.Size([32]), seed=0))
    Xd = X[:3].unsqueeze(1).repeat(1, 2, 1).to(DEV)  # duplicated rows at training points: singular
    kernels.check_ladder_status()
    with warnings.catch_warnings(record=True) as ws:
        warnings.simplefilter("always")
        with torch.no_grad():
            v = acqf(Xd)
        assert not any(issubclass(w.category, NumericalWarning) for w in ws)
        kernels.check_ladder_status()
        assert any(issubclass(w.category, NumericalWarning) for w in ws)
    assert torch.isfinite(v).all()


@pytest.mark.parametrize("n,B,q", [(4096, 64, 16), (1000, 64, 8), (2048, 128, 8)])
def test_post_w_stream_k_matches_gemm(n, B, q):
    """Stream-K W^T = L^{-T} R^T (bo_post_w_split, the default below four tiles
    per slot) against the triangular GEMM route, and post_backward through it
    against the GEMM's W."""
    from botorch_amd import _lib, kernels
    X, Y, m, orc = _setup(n=n)
    g = torch.Generator().manual_seed(n + B)
    Xc = torch.rand(B, q, 6, generator=g, dtype=torch.float64)
    cache = m.prediction_cache()
    pp = kernels.post_partials(cache, Xc.to(DEV), store_R=True)
    W = kernels.w_matrix(cache, pp)
    assert W.kmajor  # the stream-K plan applies at these grids
    Wg = kernels.gemm(pp.Rt, cache.U, transA=True, transB=True, flags=_lib.GEMM_B_LOWER)
    atol = 1e-11 * max(1.0, n / 1024)
    torch.testing.assert_close(W.t.T[:, :n], Wg[:, :n], rtol=1e-10, atol=atol)
    dmean = torch.randn(B, q, generator=g, dtype=torch.float64).to(DEV)
    dcov = torch.randn(B, q, q, generator=g, dtype=torch.float64).to(DEV)
    dx_k = kernels.post_backward(cache, pp, W, dmean, dcov, 0.7)
    dx_r = kernels.post_backward(cache, pp, kernels.WMat(Wg, False), dmean, dcov, 0.7)
    torch.testing.assert_close(dx_k, dx_r, rtol=1e-9, atol=1e-11)


@pytest.mark.parametrize("n,B,q,kind", [(2048, 1024, 16, 0), (2048, 2048, 8, 0), (2048, 2048, 6, 1),
                                        (4096, 256, 16, 0)])
def test_post_w_dx_fused_matches_w_route(n, B, q, kind):
    """bo_post_w_dx (W = R L^-1 reduced into dX inside the W tiles' epilogue,
    W never stored) against W^T from the triangular GEMM + bo_post_backward,
    on one-pass grids (>= 1024 paired tiles): q = 16 (one t-batch per 16-row
    tile), q = 8 (two per tile: the block-diagonal G), q = 6 with Matern-5/2,
    and a rank's b = 256 share of C3."""
    from botorch_amd import _lib, kernels
    g = torch.Generator().manual_seed(n + B + q)
    X = torch.rand(n, 6, generator=g, dtype=torch.float64).to(DEV)
    y = torch.randn(n, generator=g, dtype=torch.float64).to(DEV)
    ls = torch.full((6,), 0.35, dtype=torch.float64, device=DEV)
    cache = kernels.build_gp_cache(X, y, ls, 1e-3, 0.1, kind=kind, outputscale=1.3)
    Xc = torch.rand(B, q, 6, generator=g, dtype=torch.float64).to(DEV)
    pp = kernels.post_partials(cache, Xc, store_R=True)                    # row-major R^T
    ppb = kernels.post_partials(cache, Xc, store_R=True, rt_layout=_lib.RT_BLOCKED)
    assert torch.equal(ppb.Spart, pp.Spart)  # the layout changes nothing else
    # the blocked layout is a permutation of the row-major R^T
    nb = pp.nrows_pad // 16
    blk = ppb.Rt.view(-1, nb, 4, 4, 16)          # [kb][ib][k%16/4][k%4][i%16]
    rm = blk.permute(0, 2, 3, 1, 4).reshape(-1, pp.nrows_pad)
    assert torch.equal(rm, pp.Rt)
    dmean = torch.randn(B, q, generator=g, dtype=torch.float64).to(DEV)
    dcov = torch.randn(B, q, q, generator=g, dtype=torch.float64).to(DEV)
    dx_f = kernels.post_w_dx(cache, ppb, dmean, dcov, 0.7)
    assert dx_f is not None, "the fused one-pass grid should apply here"
    Wg = kernels.gemm(pp.Rt, cache.U, transA=True, transB=True, flags=_lib.GEMM_B_LOWER)
    dx_r = kernels.post_backward(cache, pp, kernels.WMat(Wg, False), dmean, dcov, 0.7)
    torch.testing.assert_close(dx_f, dx_r, rtol=1e-9, atol=1e-10)
    # below the one-pass grid the fused entry declines (the caller falls back)
    pp_s = kernels.post_partials(cache, Xc[:64], store_R=True)
    assert kernels.post_w_dx(cache, pp_s, dmean[:64], dcov[:64], 0.7) is None


@pytest.mark.parametrize("n,B,q,S", [(1024, 64, 8, 256), (768, 100, 4, 128), (1500, 50, 3, 64)])
def test_quad_plan_matches_r_route_and_oracle(n, B, q, S, monkeypatch):
    """Forward-only small grids take the quad plan (64 x 64 block pairs of the
    cached A^{-1}, csrc/quad.hip) with the ladder status fused into the
    finalisation; its qEI equals the R route's (the same posterior through
    L^{-T}) and the oracle's, over repeated calls (the status counter re-arms)."""
    from botorch_amd import kernels
    from botorch_amd.acquisition import qExpectedImprovement
    from botorch_amd.sampling import SobolQMCNormalSampler
    from oracle.acquisition import qei
    from oracle.sampling import draw_sobol_normal_samples
    X, Y, m, orc = _setup(n=n, ls=0.3, noise=1e-3)
    best = float(Y.mean())  # most random t-batches improve on it: non-zero values
    acqf = qExpectedImprovement(m, best, sampler=SobolQMCNormalSampler(torch.Size([S]), seed=0))
    g = torch.Generator().manual_seed(1)
    Xc = torch.rand(B, q, 6, generator=g, dtype=torch.float64)
    Xd = Xc.to(DEV)
    monkeypatch.setenv("BO_POST_QUAD", "auto")  # opt-in plan
    kernels.quad_pairs.cache_clear()
    assert kernels.quad_pairs(B, q, n) > 0
    kernels.check_ladder_status()
    with torch.no_grad():
        vals = [acqf(Xd) for _ in range(3)]
    kernels.check_ladder_status()
    assert getattr(m.prediction_cache(), "_ainv_full", None) is not None
    for v in vals[1:]:
        torch.testing.assert_close(v, vals[0], rtol=0, atol=0)
    monkeypatch.setenv("BO_POST_QUAD", "0")
    kernels.quad_pairs.cache_clear()
    assert kernels.quad_pairs(B, q, n) == 0
    with torch.no_grad():
        v_r = acqf(Xd)
    monkeypatch.delenv("BO_POST_QUAD")
    kernels.quad_pairs.cache_clear()
    assert kernels.quad_pairs(B, q, n) == 0  # the default
    torch.testing.assert_close(vals[0], v_r, rtol=1e-9, atol=1e-13)
    ref = qei(orc, Xc, draw_sobol_normal_samples(q, S, 0), best)
    torch.testing.assert_close(vals[0].cpu(), ref, rtol=1e-7, atol=1e-12)
    assert (ref > 0).sum() >= B // 4
