"""The small-grid forward posterior (bo_post_small, round 5): 32-row units
over pairs of 32-column tiles whose triangular k-ranges sum to a constant, so
every unit emits finished R R^T / R beta partials -- no split-k workspace and
no reduction launch (acquisition/monte_carlo.py:405-414 through [G] exact
prediction, botorch/models/gpytorch.py:446).  The forward-only acquisition
takes it where the 128-tile plan would be stream-K; the gradient path keeps
the 128-tile route (it stores R^T).  Both are compared with each other (the
same sums in another order: 1e-12) and with the oracle (1e-7)."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _plan(B, q, n):
    from botorch_amd._lib import check, lib
    v = ctypes.c_int()
    check(lib().bo_post_small_plan(B, q, n, ctypes.byref(v)), "post_small_plan")
    return v.value


def _route_128(acqf, m, X):
    """The same qEI on the 128-tile route: the bo::post_partials op (its schema
    keeps the 128-tile partials) + bo::qmc_finalize."""
    from botorch_amd import _lib
    c = m.prediction_cache()
    ymean, ystd = m.outcome_stats()
    q = X.shape[1]
    Z = acqf._ensure_sampler().base_samples_2d(q, X.device)
    Sp, mp, Xq, _ = torch.ops.bo.post_partials(X, c.Xt, c.Xt_scaled, c.U, c.beta, c.lengthscale,
                                               int(c.kind), float(c.outputscale), False)
    out = torch.ops.bo.qmc_finalize(Sp, mp, Xq, Z, None, X.shape[0], q, int(c.n), int(c.kind),
                                    _lib.QMC_QEI, float(c.outputscale), float(c.constant),
                                    float(ymean), float(ystd), float(acqf.best_f), True, 1.0, 1.0)
    return out[0]


@pytest.mark.parametrize("n,B,q,S", [(1024, 64, 8, 256),    # C2
                                     (1024, 1, 8, 256),     # one t-batch
                                     (300, 33, 5, 128),     # ragged n, odd q and b
                                     (4096, 1, 16, 512)])   # one C3-sized t-batch
def test_small_route_matches_128_route_and_oracle(n, B, q, S):
    from botorch_amd.acquisition import qExpectedImprovement
    from botorch_amd.sampling import SobolQMCNormalSampler
    from oracle.acquisition import qei
    from oracle.sampling import draw_sobol_normal_samples
    from tests.test_gpu_acquisition import _setup
    X, Y, m, orc = _setup(n=n, ls=0.4, noise=1e-3)
    assert _plan(B, q, n) == kernels_np(n) // 64  # these grids take the small route
    bf = float(Y.mean())  # most t-batches improve on it: values and gradients are non-zero
    acqf = qExpectedImprovement(m, bf, sampler=SobolQMCNormalSampler(torch.Size([S]), seed=3))
    Xc = torch.rand(B, q, 6, dtype=torch.float64, generator=torch.Generator().manual_seed(B + q))
    with torch.no_grad():
        v_small = acqf(Xc.to(DEV)).cpu()
        v_128 = _route_128(acqf, m, Xc.to(DEV)).cpu()
    torch.testing.assert_close(v_small, v_128, rtol=1e-12, atol=1e-15)
    # the gradient path (R^T stored row-major by the small kernel)
    Xg = Xc.to(DEV).requires_grad_(True)
    v_grad = acqf(Xg)
    (dx,) = torch.autograd.grad(v_grad.sum(), Xg)
    assert torch.equal(v_grad.detach().cpu(), v_small)
    ref = qei(orc, Xc, draw_sobol_normal_samples(q, S, 3), bf)
    assert int((ref > 0).sum()) > 0
    torch.testing.assert_close(v_small, ref, rtol=1e-7, atol=1e-12)
    Xo = Xc.clone().requires_grad_(True)
    (dref,) = torch.autograd.grad(qei(orc, Xo, draw_sobol_normal_samples(q, S, 3), bf).sum(), Xo)
    torch.testing.assert_close(dx.cpu(), dref, rtol=1e-5, atol=1e-8)


def kernels_np(n):
    from botorch_amd import kernels
    return kernels.padded_order(n)


def test_small_kernel_partials_match_dense_algebra():
    """bo_post_small through the C ABI on a random upper-triangular U and
    K*x^T: the pair partials summed equal R R^T's 16 x 16 diagonal blocks and
    R beta, R = K U, computed densely in torch (fp64)."""
    from botorch_amd._lib import check, lib
    g = torch.Generator().manual_seed(0)
    n, B, q = 320, 24, 8
    Qp, rows = 8, 24 * 8
    np_, nrows_pad = 384, 256
    U = torch.triu(torch.randn(np_, np_, generator=g, dtype=torch.float64))
    U[n:, :] = 0
    U[:, n:] = 0
    U[range(n, np_), range(n, np_)] = 1.0
    K = torch.zeros(np_, nrows_pad, dtype=torch.float64)
    K[:n, :rows] = torch.randn(n, rows, generator=g, dtype=torch.float64)
    beta = torch.randn(n, generator=g, dtype=torch.float64)
    nparts = _plan(B, q, n)
    if nparts == 0:
        pytest.skip("small route off (BO_POST_SMALL=0)")
    assert nparts == np_ // 64
    Ud, Kd, bd = U.to(DEV), K.to(DEV), beta.to(DEV)
    Sp = torch.zeros(nparts, nrows_pad // 16, 16, 16, dtype=torch.float64, device=DEV)
    mp = torch.zeros(nparts, nrows_pad, dtype=torch.float64, device=DEV)
    P = ctypes.c_void_p
    st = torch.cuda.current_stream().cuda_stream
    check(lib().bo_post_small(P(Kd.data_ptr()), B, q, n, P(Ud.data_ptr()), np_, P(bd.data_ptr()),
                              P(Sp.data_ptr()), P(mp.data_ptr()), None, P(st)), "post_small")
    torch.cuda.synchronize()
    R = K[:, :rows].T @ U            # rows x np
    S = Sp.sum(0).cpu()[: rows // 16]
    for t in range(rows // 16):
        blk = R[16 * t:16 * t + 16]
        torch.testing.assert_close(S[t], blk @ blk.T, rtol=1e-12, atol=1e-9)
    torch.testing.assert_close(mp.sum(0).cpu()[:rows], R[:, :n] @ beta, rtol=1e-12, atol=1e-9)
