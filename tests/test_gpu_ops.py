"""The torch.library custom ops (botorch_amd/ops.py): torch.library.opcheck
(schema, fake/meta implementation, autograd registration, AOT dispatch) for
every op on small device inputs, and the ops against the direct C-ABI calls."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
F64 = torch.float64


def _model(n=96, d=6, seed=0):
    from botorch_amd.models import SingleTaskGP
    from botorch_amd.test_functions import Hartmann
    from oracle.sampling import draw_sobol_samples
    lo = torch.zeros(d, dtype=F64)
    X = draw_sobol_samples(lo, lo + 1, n, 1, seed).squeeze(1)
    Y = Hartmann(negate=True)(X[:, :6]).unsqueeze(-1)
    m = SingleTaskGP(X.to(DEV), Y.to(DEV))
    m.covar_module.lengthscale = torch.full((1, d), 0.4, dtype=F64)
    m.likelihood.noise = torch.tensor([1e-3], dtype=F64)
    return m.eval(), X, Y


def _check(op, args, grad=False):
    from botorch_amd import ops  # noqa: F401
    utils = ["test_schema", "test_faketensor"]
    if grad:
        utils.append("test_autograd_registration")
    torch.library.opcheck(op, args, test_utils=utils)


def test_opcheck_sobol_and_cache():
    from botorch_amd import kernels, ops  # noqa: F401  (registers torch.ops.bo)
    state, shift = kernels.sobol_engine_state(5, 3)
    _check(torch.ops.bo.sobol_normal.default, (state.to(DEV), shift.to(DEV), 64, 0, False))
    m, X, Y = _model()
    c = m.prediction_cache()
    _check(torch.ops.bo.gp_cache.default, (c.Xt, m.train_targets.contiguous(), c.lengthscale, 1.0,
                                           1e-3, 0.0, 0))
    _check(torch.ops.bo.mll.default, (c.Xt, m.train_targets.contiguous(), c.lengthscale, 1e-3, 0.0,
                                      1.0, 0))


@pytest.mark.parametrize("dim,seed", [(1, 0), (5, 3), (30, 1234), (96, 7), (1000, 2**31 - 1),
                                      (4096, 99), (21201, 5)])
def test_sobol_scramble_equals_sobol_engine(dim, seed):
    """bo_sobol_scramble's state and shift are SobolEngine(dim, scramble=True,
    seed)'s, bit for bit, up to the engine's largest dimension."""
    from torch.quasirandom import SobolEngine
    from botorch_amd import kernels
    state, shift = kernels.sobol_engine_state(dim, seed, DEV)
    assert state.device.type == "cuda" and shift.device.type == "cuda"
    eng = SobolEngine(dimension=dim, scramble=True, seed=seed)
    assert torch.equal(state.cpu(), eng.sobolstate)
    assert torch.equal(shift.cpu(), eng.shift)


def test_sobol_scramble_dimension_range():
    from botorch_amd import kernels
    with pytest.raises(ValueError, match="dimensionality"):
        kernels.sobol_engine_state(21202, 0, DEV)


@pytest.mark.parametrize("dim", [1, 8, 6144])
def test_sobol_scramble_unseeded_is_a_scrambled_net(dim):
    """seed=None: the engine's draws from the global CPU generator -- the
    state equals SobolEngine(dim, scramble=True) after the same manual_seed,
    and the global stream is left where the engine leaves it -- and the state
    is a scrambled Sobol sequence: in every dimension the first 2^k points
    fall one in each interval [i 2^-k, (i + 1) 2^-k); two draws differ."""
    import numpy as np
    from torch.quasirandom import SobolEngine
    from botorch_amd import kernels
    torch.manual_seed(123)
    s1, sh1 = kernels.sobol_engine_state(dim, None, DEV)
    after = torch.rand(3)
    torch.manual_seed(123)
    eng = SobolEngine(dimension=dim, scramble=True)
    assert torch.equal(s1.cpu(), eng.sobolstate) and torch.equal(sh1.cpu(), eng.shift)
    assert torch.equal(torch.rand(3), after)
    s2, _ = kernels.sobol_engine_state(dim, None, DEV)
    assert s1.shape == (dim, 30) and sh1.shape == (dim,)
    assert dim == 1 or not torch.equal(s1, s2)
    st, sh = s1.cpu().numpy(), sh1.cpu().numpy()
    assert (st >= 0).all() and (st < 2**30).all() and (sh >= 0).all() and (sh < 2**30).all()
    k = 10
    idx = np.arange(2**k)
    gray = idx ^ (idx >> 1)
    for j in range(0, dim, max(1, dim // 64)):
        u = np.full(2**k, sh[j], dtype=np.int64)
        for b in range(k):
            u ^= np.where((gray >> b) & 1, st[j, b], 0)
        assert np.array_equal(np.sort(u >> (30 - k)), idx)


def test_opcheck_chol_jitter():
    g = torch.Generator().manual_seed(0)
    M = torch.randn(4, 6, 6, generator=g, dtype=F64)
    A = (M @ M.mT + 6 * torch.eye(6, dtype=F64)).to(DEV).requires_grad_(True)
    _check(torch.ops.bo.chol_jitter.default, (A,), grad=True)
    L = torch.ops.bo.chol_jitter(A)
    torch.testing.assert_close(L.detach().cpu(), torch.linalg.cholesky(A.detach().cpu()))
    (gA,) = torch.autograd.grad(L.sum(), A)
    Ar = A.detach().cpu().requires_grad_(True)
    (gr,) = torch.autograd.grad(torch.linalg.cholesky(Ar).sum(), Ar)
    torch.testing.assert_close(0.5 * (gA + gA.mT).cpu(), 0.5 * (gr + gr.mT), rtol=1e-9, atol=1e-10)


def test_opcheck_posterior_ops():
    m, X, Y = _model()
    c = m.prediction_cache()
    ymean, ystd = m.outcome_stats()
    g = torch.Generator().manual_seed(1)
    Xc = torch.rand(5, 4, 6, generator=g, dtype=F64).to(DEV)
    _check(torch.ops.bo.post_partials.default, (Xc, c.Xt, c.Xt_scaled, c.U, c.beta, c.lengthscale,
                                                0, 1.0, True))
    Sp, mp, Xq, Rt = torch.ops.bo.post_partials(Xc, c.Xt, c.Xt_scaled, c.U, c.beta, c.lengthscale,
                                                0, 1.0, False)
    Z = torch.randn(32, 4, generator=g, dtype=F64).to(DEV)
    _check(torch.ops.bo.qmc_finalize.default, (Sp, mp, Xq, Z, None, 5, 4, c.n, 0, 1, 1.0,
                                               c.constant, ymean, ystd, 0.5, True, 1.0, 1.0))
    Xg = Xc.clone().requires_grad_(True)
    args = (Xg, c.Xt, c.Xt_scaled, c.U, c.Linv, c.beta, c.alpha, c.lengthscale, 0, 1.0, c.constant,
            ymean, ystd, True)
    _check(torch.ops.bo.gp_posterior.default, args, grad=True)
    # the op's gradient equals the direct kernels' (posterior_moments' former path)
    mean, cov, _, _, _ = torch.ops.bo.gp_posterior(*args)
    (gx,) = torch.autograd.grad(mean.sum() + cov.diagonal(dim1=-2, dim2=-1).sum(), Xg)
    from oracle.gp import ExactGPOracle, GPHyper
    orc = ExactGPOracle(X, Y, GPHyper(torch.full((6,), 0.4, dtype=F64), 1e-3, 0.0))
    Xo = Xc.cpu().requires_grad_(True)
    mr, cr = orc.posterior(Xo)
    (go,) = torch.autograd.grad(mr.sum() + cr.diagonal(dim1=-2, dim2=-1).sum(), Xo)
    torch.testing.assert_close(gx.cpu(), go, rtol=1e-5, atol=1e-8)


@pytest.mark.parametrize("mode", [1, 4])
def test_opcheck_qmc_acq(mode):
    m, X, Y = _model()
    c = m.prediction_cache()
    ymean, ystd = m.outcome_stats()
    g = torch.Generator().manual_seed(2)
    Xc = torch.rand(6, 3, 6, generator=g, dtype=F64).to(DEV).requires_grad_(True)
    Z = torch.randn(64, 3, generator=g, dtype=F64).to(DEV)
    args = (Xc, c.Xt, c.Xt_scaled, c.U, c.Linv, c.beta, c.alpha, c.lengthscale, Z, None, 0, mode,
            1.0, c.constant, ymean, ystd, float(Y.max()) - 0.5, True, 1e-6, 1e-2, True)
    _check(torch.ops.bo.qmc_acq.default, args, grad=True)


def test_opcheck_qehvi():
    g = torch.Generator().manual_seed(3)
    m_, B, q, S = 2, 4, 3, 32
    mean = torch.randn(m_, B, q, generator=g, dtype=F64).to(DEV).requires_grad_(True)
    Lm = torch.randn(m_, B, q, q, generator=g, dtype=F64).tril()
    Lm = (Lm + 2 * torch.eye(q, dtype=F64)).to(DEV).requires_grad_(True)
    Z = torch.randn(S, q * m_, generator=g, dtype=F64).to(DEV)
    lo = torch.tensor([[-3.0, -3.0], [0.0, -3.0]], dtype=F64).to(DEV)
    hi = torch.tensor([[0.0, 5.0], [5.0, 0.0]], dtype=F64).to(DEV)
    _check(torch.ops.bo.qehvi.default, (mean, Lm, Z, lo, hi), grad=True)
