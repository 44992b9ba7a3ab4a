"""The generic (non-fused) acquisition route on the GPU: q > 16, d > 8, SAAS
qNEI, outcome constraints, qNEI cache_root=False, the NotPSD/NaN fallback of
the cached root, and the reference's cached-vs-uncached self-consistency test
(test/acquisition/test_monte_carlo.py:468-585)."""
import warnings

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(n=40, d=6, seed=0, ls=0.4, noise=2e-3, const=0.05):
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


def test_chol_backward_q_gt_16_matches_torch():
    from botorch_amd import kernels
    g = torch.Generator().manual_seed(0)
    for q in (17, 40, 64):
        A = torch.randn(3, q, q, generator=g, dtype=torch.float64)
        A = A @ A.mT + q * torch.eye(q, dtype=torch.float64)
        A.requires_grad_(True)
        L = torch.linalg.cholesky(A)
        dL = torch.randn(3, q, q, generator=g, dtype=torch.float64).tril()
        (gA,) = torch.autograd.grad(L, A, dL)
        got = kernels.chol_backward(L.detach().to(DEV), dL.to(DEV)).cpu()
        gs = 0.5 * (gA + gA.mT)
        torch.testing.assert_close(0.5 * (got + got.mT), gs, rtol=1e-9, atol=1e-10)


@pytest.mark.parametrize("q,d", [(20, 6), (3, 10), (24, 12)])
def test_general_posterior_gradient_matches_oracle(q, d):
    """_GeneralMoments (q > 16 or d > 8): mean, covariance and their gradient."""
    X, Y, m, orc = _model(n=48, d=d, seed=2)
    g = torch.Generator().manual_seed(q + d)
    Xc = torch.rand(3, q, d, generator=g, dtype=torch.float64)
    Xd = Xc.to(DEV).requires_grad_(True)
    post = m.posterior(Xd)
    loss = post.mean.sum() + 2.0 * post.variance.sum() + 0.5 * post.covariance_matrix[..., 0, -1].sum()
    (gd,) = torch.autograd.grad(loss, Xd)
    Xo = Xc.clone().requires_grad_(True)
    mr, cr = orc.posterior(Xo)
    lo = mr.sum() + 2.0 * cr.diagonal(dim1=-2, dim2=-1).sum() + 0.5 * cr[..., 0, -1].sum()
    (go,) = torch.autograd.grad(lo, Xo)
    torch.testing.assert_close(post.mean.squeeze(-1).detach().cpu(), mr.detach(), rtol=1e-4, atol=1e-9)
    torch.testing.assert_close(post.covariance_matrix.detach().cpu(), cr.detach(), rtol=1e-4, atol=1e-9)
    torch.testing.assert_close(gd.cpu(), go, rtol=1e-5, atol=1e-8)


@pytest.mark.parametrize("q,d", [(20, 6), (4, 10)])
def test_qei_generic_value_and_gradient(q, d):
    from botorch_amd.acquisition import qExpectedImprovement
    from botorch_amd.sampling import SobolQMCNormalSampler
    from oracle.acquisition import qei
    from oracle.sampling import base_samples_single_output
    X, Y, m, orc = _model(n=48, d=d, seed=3)
    S = 128
    best_f = float(Y.median())
    acqf = qExpectedImprovement(m, best_f, sampler=SobolQMCNormalSampler(torch.Size([S]), seed=4))
    g = torch.Generator().manual_seed(1)
    Xc = torch.rand(5, q, d, generator=g, dtype=torch.float64)
    Xd = Xc.to(DEV).requires_grad_(True)
    v = acqf(Xd)
    (gd,) = torch.autograd.grad(v.sum(), Xd)
    Xo = Xc.clone().requires_grad_(True)
    ref = qei(orc, Xo, base_samples_single_output(S, q, 4), best_f)
    (go,) = torch.autograd.grad(ref.sum(), Xo)
    torch.testing.assert_close(v.detach().cpu(), ref.detach(), rtol=1e-6, atol=1e-10)
    torch.testing.assert_close(gd.cpu(), go, rtol=1e-5, atol=1e-8)


def test_qei_constraints_match_oracle():
    """Outcome constraints with eta smoothing (monte_carlo.py:305-330,
    utils/objective.py:134-180): values and gradients vs. the oracle."""
    from botorch_amd.acquisition import qExpectedImprovement
    from botorch_amd.sampling import SobolQMCNormalSampler
    from oracle.acquisition import qei_constrained
    from oracle.sampling import base_samples_single_output
    X, Y, m, orc = _model(n=40, seed=5)
    S, q = 128, 3
    best_f = float(Y.median())
    thr = float(Y.quantile(0.8))
    cons = [lambda Z: Z[..., 0] - thr]
    eta = 0.05
    acqf = qExpectedImprovement(m, best_f, sampler=SobolQMCNormalSampler(torch.Size([S]), seed=1),
                                constraints=cons, eta=eta)
    g = torch.Generator().manual_seed(2)
    Xc = torch.rand(6, q, 6, generator=g, dtype=torch.float64)
    Xd = Xc.to(DEV).requires_grad_(True)
    v = acqf(Xd)
    (gd,) = torch.autograd.grad(v.sum(), Xd)
    Xo = Xc.clone().requires_grad_(True)
    ref = qei_constrained(orc, Xo, base_samples_single_output(S, q, 1), best_f, cons, eta)
    (go,) = torch.autograd.grad(ref.sum(), Xo)
    assert ref.abs().max() > 0
    torch.testing.assert_close(v.detach().cpu(), ref.detach(), rtol=1e-6, atol=1e-10)
    torch.testing.assert_close(gd.cpu(), go, rtol=1e-5, atol=1e-8)
    # without constraints the weights are 1: the constrained value is smaller
    plain = qExpectedImprovement(m, best_f, sampler=SobolQMCNormalSampler(torch.Size([S]), seed=1))
    with torch.no_grad():
        assert (plain(Xc.to(DEV)) >= v.detach() - 1e-12).all()


@pytest.mark.parametrize("q", [2, 5])
def test_qnei_cache_root_false_matches_oracle(q):
    """cache_root=False: the joint (r + q) posterior sampled per forward with the
    Sobol(r + q) base samples; the baseline best comes from those samples."""
    from botorch_amd.acquisition import qNoisyExpectedImprovement
    from botorch_amd.sampling import SobolQMCNormalSampler
    from oracle.acquisition import qnei_full_joint
    from oracle.sampling import draw_sobol_normal_samples
    X, Y, m, orc = _model(n=40, seed=6)
    S = 64
    Xb = X[:12]
    acqf = qNoisyExpectedImprovement(m, Xb.to(DEV), sampler=SobolQMCNormalSampler(torch.Size([S]), seed=7),
                                     prune_baseline=False, cache_root=False)
    g = torch.Generator().manual_seed(q)
    Xc = torch.rand(4, q, 6, generator=g, dtype=torch.float64)
    Xd = Xc.to(DEV).requires_grad_(True)
    v = acqf(Xd)
    (gd,) = torch.autograd.grad(v.sum(), Xd)
    Xo = Xc.clone().requires_grad_(True)
    ref = qnei_full_joint(orc, Xb, Xo, draw_sobol_normal_samples(12 + q, S, 7))
    (go,) = torch.autograd.grad(ref.sum(), Xo)
    torch.testing.assert_close(v.detach().cpu(), ref.detach(), rtol=1e-6, atol=1e-10)
    torch.testing.assert_close(gd.cpu(), go, rtol=1e-5, atol=1e-8)


@pytest.mark.parametrize("q,d", [(20, 6), (3, 10)])
def test_qnei_generic_cached_matches_oracle(q, d):
    """Cached root outside the fused limits (q > 16 or d > 8):
    sample_cached_cholesky over the joint posterior, vs. the oracle."""
    from botorch_amd.acquisition import qNoisyExpectedImprovement
    from botorch_amd.sampling import SobolQMCNormalSampler
    from oracle.acquisition import QNEIOracle
    X, Y, m, orc = _model(n=40, d=d, seed=8)
    S = 64
    Xb = X[:10]
    acqf = qNoisyExpectedImprovement(m, Xb.to(DEV), sampler=SobolQMCNormalSampler(torch.Size([S]), seed=3),
                                     prune_baseline=False)
    g = torch.Generator().manual_seed(4)
    Xc = torch.rand(3, q, d, generator=g, dtype=torch.float64)
    Xd = Xc.to(DEV).requires_grad_(True)
    v = acqf(Xd)
    (gd,) = torch.autograd.grad(v.sum(), Xd)
    ref_acq = QNEIOracle(orc, Xb, S, seed=3)
    Xo = Xc.clone().requires_grad_(True)
    ref = ref_acq(Xo)
    (go,) = torch.autograd.grad(ref.sum(), Xo)
    torch.testing.assert_close(v.detach().cpu(), ref.detach(), rtol=1e-6, atol=1e-10)
    torch.testing.assert_close(gd.cpu(), go, rtol=1e-5, atol=1e-8)


@pytest.mark.parametrize("log", [False, True])
def test_qnei_cache_root_vs_no_cache(log):
    """Port of test/acquisition/test_monte_carlo.py:468-585 (single output): the
    cached-root acquisition (fused path) and cache_root=False agree in values and
    gradients within 1e-4 once the uncached sampler uses the cached one's joint
    base samples; with the cached root zeroed, one BotorchWarning and a
    fall-back to standard sampling."""
    from botorch_amd.acquisition import qLogNoisyExpectedImprovement, qNoisyExpectedImprovement
    from botorch_amd.exceptions import BotorchWarning
    from botorch_amd.models import SingleTaskGP
    from botorch_amd.sampling import IIDNormalSampler
    torch.manual_seed(1234)
    train_X = torch.rand(3, 2, dtype=torch.float64)
    train_Y = torch.sin(train_X * 2 * torch.pi)[:, :1] + torch.randn(3, 1, dtype=torch.float64)
    train_Y = (train_Y - train_Y.mean()) / train_Y.std()
    model = SingleTaskGP(train_X.to(DEV), train_Y.to(DEV))
    model.likelihood.noise = torch.tensor([0.0895], dtype=torch.float64)
    model.mean_module.constant = -0.4545
    model.covar_module.lengthscale = torch.tensor([[0.72, 0.29]], dtype=torch.float64)
    model.eval()
    cls = qLogNoisyExpectedImprovement if log else qNoisyExpectedImprovement
    sampler = IIDNormalSampler(sample_shape=torch.Size([5]), seed=0)
    acqf = cls(model=model, X_baseline=train_X.to(DEV), sampler=sampler, prune_baseline=False,
               cache_root=True)
    orig_base_samples = acqf.base_sampler.base_samples.detach().clone()
    sampler2 = IIDNormalSampler(sample_shape=torch.Size([5]), seed=0)
    sampler2.base_samples = orig_base_samples
    acqf_no_cache = cls(model=model, X_baseline=train_X.to(DEV), sampler=sampler2,
                        prune_baseline=False, cache_root=False)
    for q, batch_shape in [(1, ()), (3, ()), (1, (3,)), (3, (3,)), (1, (4, 3)), (3, (4, 3))]:
        acqf.q_in = -1
        acqf_no_cache.q_in = -1
        test_X = (0.3 + 0.05 * torch.randn(*batch_shape, q, 2, dtype=torch.float64)).to(DEV)
        test_X.requires_grad_(True)
        val = acqf(test_X)
        val.sum().backward()
        base_samples = acqf.sampler.base_samples.detach().clone()
        X_grad = test_X.grad.clone()
        test_X2 = test_X.detach().clone().requires_grad_(True)
        acqf_no_cache.sampler.base_samples = base_samples
        val2 = acqf_no_cache(test_X2)
        torch.testing.assert_close(val, val2, atol=1e-4, rtol=0)
        val2.sum().backward()
        torch.testing.assert_close(X_grad, test_X2.grad, atol=1e-4, rtol=0)
    # ill-conditioned cached root -> standard sampling, one BotorchWarning
    acqf._baseline_L = torch.zeros_like(acqf._baseline_L)
    with warnings.catch_warnings(record=True) as ws:
        warnings.simplefilter("always")
        with torch.no_grad():
            out = acqf(test_X)
    assert sum(issubclass(w.category, BotorchWarning) for w in ws) == 1
    assert torch.isfinite(out).all()


def test_qnei_fused_notpsd_falls_back():
    """The fused cached-root path: a joint covariance the q x q ladder cannot
    factor (duplicated candidate rows with zero noise left over) takes the
    reference fallback with one BotorchWarning instead of raising."""
    from botorch_amd.acquisition import qNoisyExpectedImprovement
    from botorch_amd.exceptions import BotorchWarning
    from botorch_amd.sampling import SobolQMCNormalSampler
    X, Y, m, orc = _model(n=40, seed=9)
    acqf = qNoisyExpectedImprovement(m, X[:8].to(DEV), sampler=SobolQMCNormalSampler(torch.Size([32]), seed=1),
                                     prune_baseline=False)
    assert acqf._fused_ready
    # poison the fused cross term: the conditional covariance becomes NaN
    acqf._root.Linv.fill_(float("nan"))
    Xc = torch.rand(4, 2, 6, dtype=torch.float64).to(DEV)
    with warnings.catch_warnings(record=True) as ws:
        warnings.simplefilter("always")
        with torch.no_grad():
            out = acqf(Xc)
    assert sum(issubclass(w.category, BotorchWarning) for w in ws) == 1
    assert torch.isfinite(out).all() and out.shape == (4,)


def test_saas_qnei_generic_matches_member_oracle():
    """qNEI over the SAAS ensemble (cached root over M members, generic route):
    values vs. the per-member oracle averaged over MCMC_DIM."""
    from botorch_amd.acquisition import qNoisyExpectedImprovement
    from botorch_amd.models import SaasFullyBayesianSingleTaskGP, sample_saas_prior
    from botorch_amd.sampling import SobolQMCNormalSampler
    from botorch_amd.test_functions import Hartmann
    from oracle.acquisition import QNEIOracle, saas_members
    from oracle.sampling import draw_sobol_samples
    d, M, n, S, q = 10, 3, 48, 64, 2
    lo = torch.zeros(d, dtype=torch.float64)
    X = draw_sobol_samples(lo, lo + 1, n, 1, 0).squeeze(1)
    Y = Hartmann(negate=True)(X[:, :6]).unsqueeze(-1)
    Y = (Y - Y.mean()) / Y.std()
    smp = sample_saas_prior(d, M, seed=3)
    m = SaasFullyBayesianSingleTaskGP(X.to(DEV), Y.to(DEV))
    m.load_mcmc_samples({k: v.to(DEV) for k, v in smp.items()})
    m.eval()
    Xb = X[:6]
    acqf = qNoisyExpectedImprovement(m, Xb.to(DEV), sampler=SobolQMCNormalSampler(torch.Size([S]), seed=2),
                                     prune_baseline=False)
    Xc = draw_sobol_samples(lo, lo + 1, 4, q, 5)
    with torch.no_grad():
        v = acqf(Xc.to(DEV)).cpu()
    # the reference's joint draw: one Sobol(r + q) set shared by the members, the
    # baseline columns from one Sobol(r) set
    members = saas_members(X, Y, smp)
    refs = [QNEIOracle(mm, Xb, S, seed=2)(Xc) for mm in members]
    torch.testing.assert_close(v, torch.stack(refs, dim=-1).mean(dim=-1), rtol=1e-6, atol=1e-10)


def test_saas_observation_noise_scaled_by_outcome_transform():
    """observation noise joins before the Standardize untransform."""
    from botorch_amd.models import SaasFullyBayesianSingleTaskGP, Standardize, sample_saas_prior
    from oracle.sampling import draw_sobol_samples
    d, M, n = 8, 2, 32
    lo = torch.zeros(d, dtype=torch.float64)
    X = draw_sobol_samples(lo, lo + 1, n, 1, 0).squeeze(1)
    Y = 3.0 + 5.0 * torch.sin(X.sum(-1, keepdim=True))
    m = SaasFullyBayesianSingleTaskGP(X.to(DEV), Y.to(DEV), outcome_transform=Standardize(m=1))
    smp = sample_saas_prior(d, M, seed=0)
    m.load_mcmc_samples({k: v.to(DEV) for k, v in smp.items()})
    m.eval()
    Xc = torch.rand(3, 2, d, dtype=torch.float64).to(DEV)
    p0 = m.posterior(Xc)
    p1 = m.posterior(Xc, observation_noise=True)
    s2 = float(Y.std()) ** 2
    noise = torch.tensor([float(mm.likelihood.noise.detach()) for mm in m._members], dtype=torch.float64)
    diff = (p1.variance - p0.variance).squeeze(-1).cpu()                 # 3 x M x 2
    torch.testing.assert_close(diff, (noise * s2).view(1, M, 1).expand_as(diff), rtol=1e-9, atol=1e-12)
