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
