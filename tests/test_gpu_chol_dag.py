"""The persistent task-DAG Cholesky + inverse (csrc/chol_dag.hip) behind
bo_cholesky_inverse: L and L^{-1} against torch.linalg on the CPU for padded
orders 128 .. 4096 (one tile row to the C3 size), ragged n inside the padding,
and the info convention of a failing leading minor (torch cholesky_ex)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _spd(n, seed, noise=1e-3, ls=0.3):
    from oracle.gp import covar
    g = torch.Generator().manual_seed(seed)
    X = torch.rand(n, 6, generator=g, dtype=torch.float64)
    K = covar(X, X, torch.full((6,), ls, dtype=torch.float64), x1_eq_x2=True)
    return K + noise * torch.eye(n, dtype=torch.float64)


@pytest.mark.parametrize("n", [128, 200, 640, 1024, 2048, 4096])
def test_cholesky_inverse_matches_torch(n):
    from botorch_amd import kernels
    torch.set_num_threads(16)
    A = _spd(n, n)
    L, Linv, info = kernels.cholesky_inverse(A.to(DEV))
    assert info == 0
    Lr = torch.linalg.cholesky(A)
    Lg = L.cpu()
    assert torch.equal(Lg.triu(1), torch.zeros_like(Lg))
    err = (Lg - Lr).abs().max() / Lr.abs().max()
    assert err < 1e-10, float(err)
    Xg = Linv.cpu()
    assert torch.equal(Xg.triu(1), torch.zeros_like(Xg))
    # residual of the inverse: X L = I (conditioning-aware bound)
    I = torch.eye(n, dtype=torch.float64)
    res = (Xg @ Lr - I).abs().max()
    Xr = torch.linalg.solve_triangular(Lr, I, upper=False)
    res_ref = (Xr @ Lr - I).abs().max()
    assert res < max(100 * res_ref, 1e-9), (float(res), float(res_ref))
    rel = (Xg - Xr).abs().max() / Xr.abs().max()
    assert rel < 1e-8, float(rel)


@pytest.mark.parametrize("n,p", [(128, 0), (256, 70), (1024, 1000), (4096, 2900)])
def test_cholesky_info_first_failing_minor(n, p):
    from botorch_amd import kernels
    A = torch.eye(n, dtype=torch.float64)
    A[p, p] = -1.0
    _, _, info = kernels.cholesky_inverse(A.to(DEV))
    assert info == p + 1
    _, info_ref = torch.linalg.cholesky_ex(A)
    assert info == int(info_ref)


def test_cholesky_repeated_calls_are_deterministic():
    """The DAG's counters are re-zeroed every call and every tile sum runs in a
    fixed order: two calls give bit-identical factors."""
    from botorch_amd import kernels
    A = _spd(1024, 5).to(DEV)
    L1, X1, i1 = kernels.cholesky_inverse(A)
    L1, X1 = L1.clone(), X1.clone()
    L2, X2, i2 = kernels.cholesky_inverse(A)
    assert i1 == i2 == 0
    assert torch.equal(L1, L2) and torch.equal(X1, X2)


@pytest.mark.parametrize("n", [300, 2048, 4096])
def test_ainv_in_the_factorisation_launch(n):
    """bo_cholesky_inverse_ainv: L, L^{-1} bit-identical to bo_cholesky_inverse
    (the added A^{-1} tasks change no factorisation task), and the lower
    64 x 64 tiles of A^{-1} equal bo_ainv's (L^{-T} L^{-1}) and torch's
    inverse of A."""
    import ctypes
    from botorch_amd import kernels
    from botorch_amd._lib import check, lib
    g = torch.Generator().manual_seed(n)
    X = torch.rand(n, 6, generator=g, dtype=torch.float64)
    K = torch.exp(-0.5 * torch.cdist(X / 0.5, X / 0.5) ** 2) + 1e-2 * torch.eye(n, dtype=torch.float64)
    np_ = kernels.padded_order(n)
    base = torch.eye(np_, dtype=torch.float64)
    base[:n, :n] = torch.tril(K)
    T = np_ // 64
    P = kernels._p
    st = kernels._stream(torch.device(DEV))
    outs = []
    for with_ainv in (False, True):
        W = base.to(DEV)
        Li = torch.empty(np_, np_, dtype=torch.float64, device=DEV)
        work = torch.empty((16 + 5 * T * T + 1) // 2, dtype=torch.float64, device=DEV)
        info = torch.zeros(1, dtype=torch.int32, device=DEV)
        if with_ainv:
            Ai = torch.full((np_, np_), float("nan"), dtype=torch.float64, device=DEV)
            check(lib().bo_cholesky_inverse_ainv(P(W), P(Li), P(Ai), P(work), np_, P(info), st),
                  "chol_ainv")
        else:
            Ai = None
            check(lib().bo_cholesky_inverse(P(W), P(Li), P(work), np_, P(info), st), "chol")
        torch.cuda.synchronize()
        assert int(info.item()) == 0
        outs.append((W, Li, Ai))
    (W0, L0, _), (W1, L1, Ai) = outs
    assert torch.equal(torch.tril(W0), torch.tril(W1)) and torch.equal(L0, L1)
    # the lower 64-tiles (diagonal tiles whole) are written, nothing else read
    tile = torch.arange(np_, device=DEV) // 64
    low = tile.view(-1, 1) >= tile.view(1, -1)
    assert not torch.isnan(Ai[low]).any()
    cache = kernels.GPCache(0, n, 6, np_, X, X, X, 1.0, 0.0, 0.0, W1, L1, L1, X, X, 0.0)
    ref = kernels.ainv(cache)  # bo_ainv: the 128-tile lower part
    m = low & (torch.arange(np_, device=DEV).view(-1, 1) >= torch.arange(np_, device=DEV).view(1, -1))
    m[n:, :] = False  # bo_ainv stops at n; the identity pad's inverse (1) is not its business
    m[:, n:] = False
    torch.testing.assert_close(Ai[m], ref[m], rtol=1e-11, atol=1e-9)
    inv = torch.linalg.inv(K)
    Ain = Ai[:n, :n].cpu()
    mm = torch.tril(torch.ones(n, n, dtype=torch.bool))
    torch.testing.assert_close(Ain[mm], inv[mm], rtol=1e-7, atol=1e-6 * inv.abs().max().item())
