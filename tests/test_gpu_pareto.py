"""bo_pareto_mask against the host restatement of pareto.py:16-64."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _host(Y, maximize, dedup):
    from botorch_amd.multi_objective import is_non_dominated
    return torch.stack([is_non_dominated(y, maximize=maximize, deduplicate=dedup) for y in Y])


@pytest.mark.parametrize("S,n,m", [(3, 50, 2), (4, 300, 3), (2, 2100, 3), (5, 17, 8), (3, 700, 1),
                                   (2, 513, 4), (3, 257, 5), (2, 300, 6), (2, 129, 7)])
@pytest.mark.parametrize("maximize", [True, False])
@pytest.mark.parametrize("dedup", [True, False])
def test_pareto_mask_matches_host(S, n, m, maximize, dedup):
    from botorch_amd import kernels
    g = torch.Generator().manual_seed(S * n + m)
    Y = torch.rand(S, n, m, generator=g, dtype=torch.float64)
    Y[:, 1] = Y[:, 0]                       # exact duplicates
    Y = torch.round(Y * 20) / 20            # ties in single objectives
    dev = kernels.pareto_mask(Y.cuda(), maximize, dedup).cpu()
    torch.testing.assert_close(dev, _host(Y, maximize, dedup))


def test_is_non_dominated_routes_to_device():
    from botorch_amd.multi_objective import is_non_dominated
    Y = torch.tensor([[1.0, 2.0], [2.0, 1.0], [0.5, 0.5], [2.0, 1.0]], dtype=torch.float64)
    out = is_non_dominated(Y.cuda())
    assert out.is_cuda and out.tolist() == [True, True, False, False]
