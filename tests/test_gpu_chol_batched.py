"""Batched DAG Cholesky (bo_cholesky_inverse_batched): nb independent
factorisations + inverses in one persistent launch, bit-identical to nb single
launches; the batched GP-cache build behind multi-output / ModelListGP / SAAS
members and the multi-output MLL closure."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _spd(n, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    X = torch.rand(n, 6, generator=g, dtype=torch.float64)
    K = torch.exp(-0.5 * torch.cdist(X, X) ** 2 / 0.3 ** 2) * scale
    return K + 1e-3 * torch.eye(n, dtype=torch.float64)


@pytest.mark.parametrize("nb,n", [(3, 1000), (4, 4096), (5, 200)])
def test_batched_equals_single_launches(nb, n):
    from botorch_amd import kernels
    As = torch.stack([_spd(n, s, 1.0 + s) for s in range(nb)]).to(DEV)
    L, Li, info = kernels.cholesky_inverse_batched(As)
    assert info == [0] * nb
    for m in range(nb):
        L1, Li1, i1 = kernels.cholesky_inverse(As[m])
        assert i1 == 0
        assert torch.equal(L[m], L1) and torch.equal(Li[m], Li1)
    # against torch (fp64): the factor and the inverse
    Lt = torch.linalg.cholesky(As[0].cpu())
    torch.testing.assert_close(L[0].cpu(), Lt, rtol=1e-9, atol=1e-11)
    eye = torch.eye(n, dtype=torch.float64)
    torch.testing.assert_close((Li[0] @ L[0]).cpu(), eye, rtol=0, atol=1e-8)


def test_batched_reports_each_member_not_pd():
    from botorch_amd import kernels
    n = 300
    A0, A2 = _spd(n, 0), _spd(n, 2)
    A1 = _spd(n, 1)
    A1[150, 150] = -5.0  # leading minor 151 is not p.d.
    L, Li, info = kernels.cholesky_inverse_batched(torch.stack([A0, A1, A2]).to(DEV))
    _, _, i1 = kernels.cholesky_inverse(A1.to(DEV))
    assert info[0] == 0 and info[2] == 0 and info[1] == i1 and i1 > 0
    L0, _, _ = kernels.cholesky_inverse(A0.to(DEV))
    assert torch.equal(L[0], L0)


def test_build_gp_caches_bit_identical():
    from botorch_amd import kernels
    from botorch_amd.test_functions import Hartmann
    g = torch.Generator().manual_seed(0)
    X = torch.rand(500, 6, generator=g, dtype=torch.float64).to(DEV)
    Y = Hartmann(negate=True)(X.cpu()).to(DEV)
    specs = [dict(Xt=X, y=(Y * (1 + t)).contiguous(),
                  lengthscale=torch.full((6,), 0.3 + 0.1 * t, dtype=torch.float64, device=DEV),
                  noise=1e-3 * (t + 1), constant=0.1 * t, outputscale=1.0 + t) for t in range(3)]
    batched = kernels.build_gp_caches(specs)
    for sp, cb in zip(specs, batched):
        c1 = kernels.build_gp_cache(**sp)
        for f in ("L", "Linv", "U", "beta", "alpha", "Xt_scaled"):
            assert torch.equal(getattr(cb, f), getattr(c1, f)), f
        assert cb.jitter == c1.jitter == 0.0


def test_multi_output_closure_and_posterior_use_the_batched_caches():
    """The batched multi-output MLL closure equals the per-member closures
    summed, and the members' primed caches equal their own builds."""
    import numpy as np
    from botorch_amd.fit import _Layout, _MultiLayout, mll_value_and_grad
    from botorch_amd.models import SingleTaskGP
    from botorch_amd.test_functions import Hartmann
    g = torch.Generator().manual_seed(1)
    X = torch.rand(256, 6, generator=g, dtype=torch.float64)
    Y = torch.stack([Hartmann(negate=True)(X), (X ** 2).sum(-1), X[:, 0] - X[:, 1]], -1)
    m = SingleTaskGP(X.to(DEV), Y.to(DEV))
    lay = _MultiLayout(m)
    x = lay.get()
    loss, grad = lay.value_and_grad(x)
    tot, grads = 0.0, []
    for p, v in zip(lay.parts, lay._split(x)):
        lt, gt = mll_value_and_grad(p.model, v, p)
        tot += lt
        grads.append(gt)
    assert abs(loss - tot) <= 1e-12 * abs(tot)
    np.testing.assert_allclose(grad, np.concatenate(grads)[lay.perm], rtol=1e-12, atol=1e-14)
    m.eval()
    Xc = torch.rand(4, 2, 6, generator=g, dtype=torch.float64).to(DEV)
    post = m.posterior(Xc)  # primes all three caches in one launch
    for mm in m.models:
        c = mm._cache
        ls, os_, noise, cst = mm.hyper()
        ref = __import__("botorch_amd.kernels", fromlist=["x"]).build_gp_cache(
            mm.train_inputs[0], mm.train_targets, ls, noise, cst, kind=mm.kind, outputscale=os_)
        assert torch.equal(c.U, ref.U) and torch.equal(c.alpha, ref.alpha)
    assert post.mean.shape[-1] == 3


@pytest.mark.parametrize("singular", [False, True])
def test_optimistic_mll_closure_matches_the_ladder_path(singular):
    """fit.mll_terms enqueues the jitter-free factorisation and reads its status
    with the MLL sums; a K + s2 I that is not p.d. without jitter falls back to
    build_gp_cache's ladder and must give exactly the ladder path's terms."""
    import numpy as np
    from botorch_amd import kernels
    from botorch_amd.fit import mll_terms
    g = torch.Generator().manual_seed(3)
    X = torch.rand(300, 6, generator=g, dtype=torch.float64)
    if singular:
        X[150:] = X[:150]  # duplicated points
    y = torch.sin(X.sum(-1))
    Xd, yd = X.to(DEV), y.to(DEV)
    ls = torch.full((6,), 0.4, dtype=torch.float64, device=DEV)
    noise = 0.0 if singular else 1e-3
    ll, grad = mll_terms(Xd, yd, ls, noise, 0.1, 1.3, 0)
    with pytest.warns(Warning) if singular else _nullcontext():
        ref_cache = kernels.build_gp_cache(Xd, yd, ls, noise, 0.1, outputscale=1.3)
    assert (ref_cache.jitter > 0) == singular
    ll2, grad2 = mll_terms(Xd, yd, ls, noise, 0.1, 1.3, 0, cache=ref_cache)
    if singular or not kernels.AINV_IN_DAG:
        # both from the ladder's caches: the same bits
        assert ll == ll2
        np.testing.assert_array_equal(grad, grad2)
    else:
        # the optimistic closure's A^{-1} comes from the factorisation's launch
        # (64-tile sums in K order), the ladder path's from bo_ainv (128-tile
        # stream-K): the same sums in another order
        assert abs(ll - ll2) <= 1e-10 * abs(ll2)
        np.testing.assert_allclose(grad, grad2, rtol=1e-9, atol=1e-9)


class _nullcontext:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


@pytest.mark.parametrize("uplo", [1, 2])
def test_gemv_tri_bit_identical_to_gemv(uplo):
    from botorch_amd import kernels
    from botorch_amd._lib import lib
    g = torch.Generator().manual_seed(5)
    n, ld = 1000, 1024
    M = torch.randn(ld, ld, generator=g, dtype=torch.float64)
    M = (torch.tril(M) if uplo == 1 else torch.triu(M)).to(DEV)
    x = torch.randn(ld, generator=g, dtype=torch.float64).to(DEV)
    y0 = torch.empty(n, dtype=torch.float64, device=DEV)
    y1 = torch.empty_like(y0)
    st = kernels._stream(DEV)
    assert lib().bo_gemv(kernels._p(M), ld, n, kernels._p(x), 0.25, kernels._p(y0), st) == 0
    assert lib().bo_gemv_tri(kernels._p(M), ld, n, kernels._p(x), 0.25, kernels._p(y1), uplo,
                             st) == 0
    assert torch.equal(y0, y1)
    torch.testing.assert_close(y1.cpu(), (M[:n, :n] @ (x[:n] - 0.25)).cpu(), rtol=1e-12,
                               atol=1e-12)


def test_covar_matrix_against_torch():
    from botorch_amd import kernels
    from botorch_amd._lib import lib
    g = torch.Generator().manual_seed(6)
    n, d, np_ = 700, 6, 768
    X = torch.rand(n, d, generator=g, dtype=torch.float64)
    ls = torch.rand(d, generator=g, dtype=torch.float64) + 0.2
    K = torch.empty(np_, np_, dtype=torch.float64, device=DEV)
    Xd, lsd = X.to(DEV), ls.to(DEV)
    assert lib().bo_covar_matrix(0, kernels._p(Xd), n, kernels._p(Xd), n, d, kernels._p(lsd), 1.7,
                                 0.01, 1, kernels._p(K), np_, np_, np_, kernels._stream(DEV)) == 0
    Xs = X / ls
    ref = 1.7 * torch.exp(-0.5 * torch.cdist(Xs, Xs) ** 2) + 0.01 * torch.eye(n, dtype=torch.float64)
    Kc = K.cpu()
    torch.testing.assert_close(Kc[:n, :n], torch.tril(ref), rtol=1e-12, atol=1e-13)
    torch.testing.assert_close(Kc[n:, n:], torch.eye(np_ - n, dtype=torch.float64))
    assert float(Kc[:n, n:].abs().max()) == 0.0


@pytest.mark.parametrize("n,ld", [(1000, 1024), (4096, 4096), (37, 128)])
def test_gemv_lt_matches_transposed_product(n, ld):
    """bo_gemv_lt: y = M^T (x - s) for a lower-triangular M read column-wise
    (alpha = L^{-T} beta without forming L^{-T}), against torch in fp64; entries
    above the diagonal are never read (filled with NaN here)."""
    import ctypes
    from botorch_amd import kernels
    from botorch_amd._lib import check, lib
    g = torch.Generator().manual_seed(n)
    M = torch.tril(torch.randn(ld, ld, generator=g, dtype=torch.float64))
    x = torch.randn(ld, generator=g, dtype=torch.float64)
    Mn = M.clone()
    Mn[torch.triu(torch.ones(ld, ld, dtype=torch.bool), 1)] = float("nan")
    we = ctypes.c_int64()
    check(lib().bo_gemv_lt_work(n, ctypes.byref(we)), "gemv_lt_work")
    work = torch.empty(we.value, dtype=torch.float64, device=DEV)
    y = torch.empty(n, dtype=torch.float64, device=DEV)
    Md, xd = Mn.to(DEV), x.to(DEV)
    check(lib().bo_gemv_lt(kernels._p(Md), ld, n, kernels._p(xd), 0.25, kernels._p(y),
                           kernels._p(work), kernels._stream(y.device)), "gemv_lt")
    ref = M[:n, :n].T @ (x[:n] - 0.25)
    torch.testing.assert_close(y.cpu(), ref, rtol=1e-12, atol=1e-12)
