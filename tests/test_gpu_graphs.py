"""HIP-graph capture of the fused acquisition (botorch_amd.graphs): replays
equal the eager path bit for bit, forward and forward + backward."""
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _model(n, seed=0):
    from botorch_amd.models import SingleTaskGP
    from botorch_amd.test_functions import Hartmann
    g = torch.Generator().manual_seed(seed)
    X = torch.rand(n, 6, generator=g, dtype=torch.float64)
    Y = Hartmann(dim=6, negate=True)(X).unsqueeze(-1)
    m = SingleTaskGP(X.to(DEV), Y.to(DEV))
    m.covar_module.lengthscale = torch.full((1, 6), 0.4, dtype=torch.float64)
    return m.eval(), Y


@pytest.mark.parametrize("cls,n,B,q,S", [("qExpectedImprovement", 1024, 64, 8, 256),
                                         ("qLogExpectedImprovement", 512, 33, 4, 128),
                                         ("qExpectedImprovement", 4096, 64, 16, 512)])
def test_graphed_forward_equals_eager(cls, n, B, q, S):
    from botorch_amd import acquisition
    from botorch_amd.graphs import GraphedAcquisition
    from botorch_amd.sampling import SobolQMCNormalSampler
    m, Y = _model(n)
    acqf = getattr(acquisition, cls)(m, best_f=Y.max().item() - 0.2,
                                     sampler=SobolQMCNormalSampler(torch.Size([S]), seed=1))
    g = torch.Generator().manual_seed(B)
    X1 = torch.rand(B, q, 6, generator=g, dtype=torch.float64).to(DEV)
    X2 = torch.rand(B, q, 6, generator=g, dtype=torch.float64).to(DEV)
    ga = GraphedAcquisition(acqf, X1)
    for X in (X1, X2, X1):
        with torch.no_grad():
            ref = acqf(X)
        out = ga(X).clone()
        assert torch.equal(out, ref)
    ga.check_status()


def test_graphed_forward_backward_equals_eager():
    from botorch_amd.acquisition import qExpectedImprovement
    from botorch_amd.graphs import GraphedAcquisition
    from botorch_amd.sampling import SobolQMCNormalSampler
    m, Y = _model(1024, seed=3)
    acqf = qExpectedImprovement(m, best_f=Y.max().item() - 0.2,
                                sampler=SobolQMCNormalSampler(torch.Size([256]), seed=2))
    g = torch.Generator().manual_seed(5)
    X1 = torch.rand(64, 8, 6, generator=g, dtype=torch.float64).to(DEV)
    X2 = torch.rand(64, 8, 6, generator=g, dtype=torch.float64).to(DEV)
    ga = GraphedAcquisition(acqf, X1, with_grad=True)
    for X in (X2, X1):
        Xg = X.clone().requires_grad_(True)
        ref = acqf(Xg)
        (gref,) = torch.autograd.grad(ref.sum(), Xg)
        v, gr = ga(X)
        assert torch.equal(v, ref.detach()) and torch.equal(gr, gref)
    ga.check_status()


def test_graphed_rejects_changed_model_and_shape():
    from botorch_amd.acquisition import qExpectedImprovement
    from botorch_amd.graphs import GraphedAcquisition
    from botorch_amd.sampling import SobolQMCNormalSampler
    m, Y = _model(256, seed=4)
    acqf = qExpectedImprovement(m, best_f=Y.max().item(), sampler=SobolQMCNormalSampler(torch.Size([64]), seed=0))
    X = torch.rand(8, 2, 6, dtype=torch.float64).to(DEV)
    ga = GraphedAcquisition(acqf, X)
    with pytest.raises(ValueError):
        ga(torch.rand(4, 2, 6, dtype=torch.float64).to(DEV))
    m.likelihood.noise = torch.tensor([2e-3], dtype=torch.float64)
    with pytest.raises(RuntimeError):
        ga(X)


def test_graphed_forward_status_without_stalls():
    """A replay never waits on the previous one's ladder status: a call acts
    on it once a finished replay has published it to pinned memory (event
    query), check_status() waits.  A jittered q x q root (duplicated rows at
    training points of a noiseless model) still reaches the caller as the
    NumericalWarning [G] psd_safe_cholesky gives, and a clean batch after the
    warning re-arms silently."""
    import warnings
    from botorch_amd import kernels
    from botorch_amd.acquisition import qExpectedImprovement
    from botorch_amd.exceptions import NumericalWarning
    from botorch_amd.graphs import GraphedAcquisition
    from botorch_amd.sampling import SobolQMCNormalSampler
    from tests.test_gpu_acquisition import _setup
    X, Y, m, orc = _setup(n=64, noise=1e-4)
    m.likelihood.noise = torch.tensor([1e-12], dtype=torch.float64)
    m.eval()
    acqf = qExpectedImprovement(m, Y.max().item(), sampler=SobolQMCNormalSampler(torch.Size([32]), seed=0))
    bad = X[:3].unsqueeze(1).repeat(1, 2, 1).to(DEV)   # singular 2 x 2 covariances
    good = torch.rand(3, 2, 6, dtype=torch.float64).to(DEV)
    kernels.check_ladder_status()
    ga = GraphedAcquisition(acqf, good)
    with warnings.catch_warnings(record=True) as ws:
        warnings.simplefilter("always")
        ga(good)
        ga.check_status()
        assert not any(issubclass(w.category, NumericalWarning) for w in ws)
        ga(bad)
        torch.cuda.synchronize()
        ga(good)  # the finished bad replay is seen here, without a wait
        assert any(issubclass(w.category, NumericalWarning) for w in ws)
        n_warn = sum(issubclass(w.category, NumericalWarning) for w in ws)
        ga.check_status()  # the good replay after the re-arm: nothing new
        for _ in range(3):
            ga(good)
        ga.check_status()
        assert sum(issubclass(w.category, NumericalWarning) for w in ws) == n_warn


def test_graphed_mixed_routes_keep_both_statuses():
    """A forward-only capture whose body mixes a route that records a device
    ladder status (qEHVI's members, _FusedQEHVI under capture) with the native
    fused qEI (its finalisation folds into the graph's pinned words): the
    device status is kept beside the native one (kernels.
    record_capture_status, a second pinned pair), so a jittered qEHVI root in
    a replay still reaches the caller as NumericalWarning, and the replay
    equals the eager body."""
    import warnings
    from botorch_amd import kernels
    from botorch_amd.acquisition import qExpectedHypervolumeImprovement, qExpectedImprovement
    from botorch_amd.exceptions import NumericalWarning
    from botorch_amd.graphs import GraphedAcquisition
    from botorch_amd.models import ModelListGP
    from botorch_amd.multi_objective import FastNondominatedPartitioning
    from botorch_amd.sampling import SobolQMCNormalSampler
    from tests.test_gpu_acquisition import _setup
    members = []
    for _ in range(2):   # noiseless members: duplicated training rows give singular roots
        X, Y, mm, _ = _setup(n=64, noise=1e-4)
        mm.likelihood.noise = torch.tensor([1e-12], dtype=torch.float64)
        members.append(mm.eval())
    Ym = torch.cat([Y, 0.5 * Y], dim=-1)
    ref_point = Ym.min(dim=0).values - 0.1
    part = FastNondominatedPartitioning(ref_point, Ym)
    qehvi = qExpectedHypervolumeImprovement(ModelListGP(*members), ref_point.tolist(), part,
                                            sampler=SobolQMCNormalSampler(torch.Size([16]), seed=0))
    m2, Y2 = _model(256, seed=6)   # noisy: clean roots everywhere
    qei = qExpectedImprovement(m2, Y2.max().item() - 0.2,
                               sampler=SobolQMCNormalSampler(torch.Size([32]), seed=0))

    class Mixed(torch.nn.Module):
        def forward(self, X):   # the device-status route first, then the native one
            return qehvi(X) + qei(X)

    body = Mixed()
    bad = X[:3].unsqueeze(1).repeat(1, 2, 1).to(DEV)
    good = torch.rand(3, 2, 6, dtype=torch.float64).to(DEV)
    kernels.check_ladder_status()
    ga = GraphedAcquisition(body, good)
    with warnings.catch_warnings(record=True) as ws:
        warnings.simplefilter("always")
        for Xc in (good,):
            with torch.no_grad():
                ref = body(Xc)
            kernels.check_ladder_status()
            assert torch.equal(ga(Xc).clone(), ref)
        ga.check_status()
        assert not any(issubclass(w.category, NumericalWarning) for w in ws)
        ga(bad)
        ga.check_status()
        assert any(issubclass(w.category, NumericalWarning) for w in ws), \
            "the qEHVI root's jitter was dropped by the mixed capture"
