"""Oracle parity at the full BASELINE configurations:

* C3 qEI: all 512 t-batches x q=16 x S=512 through the public API at n=4096,
  64 spread t-batches compared with the oracle;
* C3 qNEI: prune_baseline=True on the n=4096 training set (2048 Sobol samples
  of dimension 4096), the kept set against the oracle's pruning, then the
  cached-root values of b=512, S=512 against the oracle at r=1 (the bench's
  hyperparameters) and at r=32 (a noisier fit, so the cross term is wide);
* C4 qEHVI: ModelListGP(3) on the reference's DTLZ2 draw (n=2048), q=8,
  S=128, b=128, the 294 reference cells;
* the MLL value and gradient at n=4096 (default and fitted hyperparameters)
  and fit_gpytorch_mll's optimum at n=1024 against an oracle scipy fit.

Tolerances: north_star's 1e-4 relative on posterior moments and 1e-2 on MC
values, plus the tighter bound the fp64 kernels actually reach."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
# bench.py: C3 on BoTorch's default-prior modes (lengthscale 0.5016 at d = 6, noise e^-5)
N3, Q3, S3, B3 = 4096, 16, 512, 512
LS3, NOISE3 = 0.5016, 6.737947e-3


def _c3_data():
    from botorch_amd.test_functions import Hartmann
    from oracle.sampling import draw_sobol_samples
    lo = torch.zeros(6, dtype=torch.float64)
    Xtr = draw_sobol_samples(lo, lo + 1, N3, 1, 0).squeeze(1)
    Ytr = Hartmann(negate=True)(Xtr).unsqueeze(-1)
    Xc = draw_sobol_samples(lo, lo + 1, B3, Q3, 1)
    return Xtr, Ytr, Xc


def _stgp(X, Y, ls, noise, const=0.0):
    from botorch_amd.models import SingleTaskGP
    from oracle.gp import ExactGPOracle, GPHyper
    d = X.shape[-1]
    m = SingleTaskGP(X.to(DEV), Y.to(DEV))
    m.covar_module.lengthscale = torch.full((1, d), ls, dtype=torch.float64)
    m.likelihood.noise = torch.tensor([noise], dtype=torch.float64)
    m.mean_module.constant = const
    m.eval()
    return m, ExactGPOracle(X, Y, GPHyper(torch.full((d,), ls, dtype=torch.float64), noise, const))


@pytest.fixture(scope="module")
def c3():
    torch.set_num_threads(16)
    Xtr, Ytr, Xc = _c3_data()
    m, orc = _stgp(Xtr, Ytr, LS3, NOISE3)
    return Xtr, Ytr, Xc, m, orc


def test_c3_qei_full_batch_matches_oracle(c3):
    from botorch_amd.acquisition import qExpectedImprovement
    from botorch_amd.sampling import SobolQMCNormalSampler
    from oracle.acquisition import qei
    from oracle.sampling import draw_sobol_normal_samples
    Xtr, Ytr, Xc, m, orc = c3
    idx = torch.arange(0, B3, B3 // 64)                      # 64 t-batches, first to last
    Z = draw_sobol_normal_samples(Q3, S3, 0)
    # best_f = max Y (the bench's): no Sobol candidate improves on the data at
    # n = 4096, every value is exactly 0 on both sides; best_f 1.5 lower gives
    # non-zero improvements to compare
    for off, min_pos in ((0.0, 0), (1.5, 16)):
        best_f = Ytr.max().item() - off
        acqf = qExpectedImprovement(m, best_f, sampler=SobolQMCNormalSampler(torch.Size([S3]), seed=0))
        with torch.no_grad():
            v = acqf(Xc.to(DEV)).cpu()
        assert v.shape == (B3,) and torch.isfinite(v).all()
        ref = qei(orc, Xc[idx], Z, best_f)
        assert (ref > 0).sum() >= min_pos, "degenerate check: too few non-zero improvements"
        torch.testing.assert_close(v[idx], ref, rtol=1e-2, atol=1e-8)
        torch.testing.assert_close(v[idx], ref, rtol=1e-7, atol=1e-12)
    # the posterior moments of the same t-batches (north_star: 1e-4 relative)
    post = m.posterior(Xc[idx].to(DEV))
    mr, cr = orc.posterior(Xc[idx])
    torch.testing.assert_close(post.mean.squeeze(-1).cpu(), mr, rtol=1e-4, atol=1e-10)
    torch.testing.assert_close(post.variance.squeeze(-1).cpu(), cr.diagonal(dim1=-2, dim2=-1),
                               rtol=1e-4, atol=1e-12)


def _prune_seed(k):
    """The seed the reference's unseeded pruning sampler draws after
    torch.manual_seed(k) (sampling/base.py:64)."""
    torch.manual_seed(k)
    return torch.randint(0, 1000000, (1,)).item()


def _near_best(Xtr, Ytr, b, q, scale, seed):
    """b t-batches of q points scattered around the q best training points (so
    the MC improvements over the baseline are not all zero)."""
    g = torch.Generator().manual_seed(seed)
    top = Xtr[Ytr.squeeze(-1).topk(q).indices]
    return (top.unsqueeze(0) + scale * torch.randn(b, q, Xtr.shape[-1], generator=g,
                                                   dtype=torch.float64)).clamp(0, 1)


@pytest.mark.parametrize("ls,noise,r_expect", [(LS3, NOISE3, 1), (0.15, 0.5, 31)])
def test_c3_qnei_pruned_full_batch_matches_oracle(ls, noise, r_expect):
    from botorch_amd.acquisition import qNoisyExpectedImprovement
    from botorch_amd.sampling import SobolQMCNormalSampler
    from oracle.acquisition import QNEIOracle, prune_inferior_points
    torch.set_num_threads(16)
    Xtr, Ytr, Xc = _c3_data()
    m, orc = _stgp(Xtr, Ytr, ls, noise)
    seed = _prune_seed(7)
    torch.manual_seed(7)
    acqf = qNoisyExpectedImprovement(m, Xtr.to(DEV), sampler=SobolQMCNormalSampler(torch.Size([S3]), seed=0),
                                     prune_baseline=True)
    kept = acqf.X_baseline.cpu()
    kept_ref = prune_inferior_points(orc, Xtr, num_samples=2048, seed=seed)
    assert kept.shape[0] == kept_ref.shape[0] == r_expect
    torch.testing.assert_close(kept, kept_ref, rtol=0, atol=0)
    assert acqf._fused_ready
    with torch.no_grad():
        v = acqf(Xc.to(DEV)).cpu()
    assert v.shape == (B3,) and torch.isfinite(v).all()
    ref_acq = QNEIOracle(orc, kept_ref, S3, seed=0)
    torch.testing.assert_close(acqf._baseline_best_f.cpu(), ref_acq.best_f, rtol=1e-9, atol=1e-10)
    idx = torch.arange(0, B3, B3 // 32)
    # Sobol candidates (the bench's: nearly all values 0), then t-batches around
    # the best training points (non-zero improvements)
    Xn = _near_best(Xtr, Ytr, B3, Q3, 0.03, 1)
    with torch.no_grad():
        vn = acqf(Xn.to(DEV)).cpu()
    for got, X in ((v, Xc), (vn, Xn)):
        ref = ref_acq(X[idx])
        torch.testing.assert_close(got[idx], ref, rtol=1e-2, atol=1e-8)
        torch.testing.assert_close(got[idx], ref, rtol=1e-6, atol=1e-10)
    assert (ref > 0).sum() >= 8


def test_c4_qehvi_full_config_matches_oracle(golden):
    from botorch_amd.acquisition import qExpectedHypervolumeImprovement
    from botorch_amd.models import ModelListGP
    from botorch_amd.multi_objective import FastNondominatedPartitioning
    from botorch_amd.sampling import SobolQMCNormalSampler
    from oracle.acquisition import qehvi
    from oracle.sampling import base_samples_multi_output, draw_sobol_samples
    torch.set_num_threads(16)
    X = torch.from_numpy(golden["dtlz2_X"])
    Y = torch.from_numpy(golden["dtlz2_Y"])
    assert X.shape == (2048, 6)
    pairs = [_stgp(X, Y[:, t:t + 1], 0.6, 1e-3) for t in range(3)]
    ref_point = torch.full((3,), -1.1, dtype=torch.float64)
    part = FastNondominatedPartitioning(ref_point, Y)
    lo, hi = part.get_hypercell_bounds()
    np.testing.assert_array_equal(lo.cpu().numpy(), golden["dtlz2_cells_lower"])
    np.testing.assert_array_equal(hi.cpu().numpy(), golden["dtlz2_cells_upper"])
    S, q, b = 128, 8, 128
    acqf = qExpectedHypervolumeImprovement(ModelListGP(*[p[0] for p in pairs]), ref_point.tolist(), part,
                                           sampler=SobolQMCNormalSampler(torch.Size([S]), seed=0))
    u = torch.zeros(6, dtype=torch.float64)
    Xc = draw_sobol_samples(u, u + 1, b, q, 1)
    # Sobol candidates (most values 0 against 2048 points) and t-batches around
    # the Pareto set (non-zero improvements)
    g = torch.Generator().manual_seed(2)
    P = X[torch.from_numpy(golden["dtlz2_pareto_mask"])]
    pick = torch.randint(0, P.shape[0], (b, q), generator=g)
    Xn = (P[pick] + 0.05 * torch.randn(b, q, 6, generator=g, dtype=torch.float64)).clamp(0, 1)
    idx = torch.tensor([0, 17, 40, 63, 64, 99, 111, 127])
    cl = torch.from_numpy(golden["dtlz2_cells_lower"])
    cu = torch.from_numpy(golden["dtlz2_cells_upper"])
    Zm = base_samples_multi_output(S, q, 3, 0)
    for Xt in (Xc, Xn):
        with torch.no_grad():
            v = acqf(Xt.to(DEV)).cpu()
        assert v.shape == (b,) and torch.isfinite(v).all()
        ref = torch.cat([qehvi([p[1] for p in pairs], Xt[i:i + 1], Zm, cl, cu) for i in idx.tolist()])
        torch.testing.assert_close(v[idx], ref, rtol=1e-2, atol=1e-8)
        torch.testing.assert_close(v[idx], ref, rtol=1e-7, atol=1e-10)
    assert (ref > 0).sum() >= 6


def _oracle_loss_grad(X, Y, x):
    from oracle.gp import neg_mll, standardize_fit
    mu, sd = standardize_fit(Y)
    y = ((Y - mu) / sd).squeeze(-1)
    noise = torch.tensor(float(x[0]), dtype=torch.float64, requires_grad=True)
    c = torch.tensor(float(x[1]), dtype=torch.float64, requires_grad=True)
    ls = torch.tensor(np.asarray(x[2:]), dtype=torch.float64, requires_grad=True)
    loss = neg_mll(X, y, ls, noise, c)
    loss.backward()
    return loss.item(), np.concatenate([[noise.grad.item(), c.grad.item()], ls.grad.numpy()])


def test_mll_full_size_value_and_grad_match_oracle():
    """The MLL closure at the size the bench fits (n = 4096, d = 6), at the
    default initialisation and at the fitted hyperparameters."""
    from botorch_amd.fit import ExactMarginalLogLikelihood, _Layout, fit_gpytorch_mll, mll_value_and_grad
    from botorch_amd.models import SingleTaskGP
    torch.set_num_threads(16)
    Xtr, Ytr, _ = _c3_data()
    m = SingleTaskGP(Xtr.to(DEV), Ytr.to(DEV))
    lay = _Layout(m)
    x0 = lay.get()
    v0, g0 = mll_value_and_grad(m, x0, lay)
    rv0, rg0 = _oracle_loss_grad(Xtr, Ytr, x0)
    assert abs(v0 - rv0) <= 1e-9 * max(1.0, abs(rv0))
    np.testing.assert_allclose(g0, rg0, rtol=1e-6, atol=1e-9)
    fit_gpytorch_mll(ExactMarginalLogLikelihood(m.likelihood, m))
    x1 = lay.get()
    assert not np.allclose(x1, x0)
    v1, g1 = mll_value_and_grad(m, x1, lay)
    rv1, rg1 = _oracle_loss_grad(Xtr, Ytr, x1)
    assert v1 < v0
    assert abs(v1 - rv1) <= 1e-9 * max(1.0, abs(rv1))
    np.testing.assert_allclose(g1, rg1, rtol=1e-5, atol=1e-8)


def test_fit_matches_oracle_scipy_fit():
    """fit_gpytorch_mll at n = 1024 against the same L-BFGS-B run over the
    oracle's closure (oracle.gp.fit_scipy): the same optimum."""
    from botorch_amd.fit import ExactMarginalLogLikelihood, _Layout, fit_gpytorch_mll
    from botorch_amd.models import SingleTaskGP
    from botorch_amd.test_functions import Hartmann
    from oracle.gp import fit_scipy, standardize_fit
    from oracle.sampling import draw_sobol_samples
    torch.set_num_threads(16)
    lo = torch.zeros(6, dtype=torch.float64)
    X = draw_sobol_samples(lo, lo + 1, 1024, 1, 0).squeeze(1)
    Y = Hartmann(negate=True)(X).unsqueeze(-1)
    m = SingleTaskGP(X.to(DEV), Y.to(DEV))
    lay = _Layout(m)
    x0, bounds = lay.get(), lay.bounds
    fit_gpytorch_mll(ExactMarginalLogLikelihood(m.likelihood, m))
    x_gpu = lay.get()
    mu, sd = standardize_fit(Y)
    res = fit_scipy(X, ((Y - mu) / sd).squeeze(-1), x0, bounds)
    assert res.success
    np.testing.assert_allclose(x_gpu, res.x, rtol=1e-3, atol=1e-5)
    lg, _ = _oracle_loss_grad(X, Y, x_gpu)
    assert abs(lg - res.fun) <= 1e-7 * max(1.0, abs(res.fun))


def _spread_nonzero(v, k):
    """k t-batch indices spread over the batch among those with a non-zero
    value (so their gradients are not trivially zero)."""
    nz = (v != 0).nonzero().flatten()
    assert nz.numel() >= k, f"only {nz.numel()} non-zero values"
    return nz[torch.linspace(0, nz.numel() - 1, k).round().long()]


@pytest.mark.parametrize("b,acq", [(512, "qei"), (256, "qei"), (512, "qlogei")])
def test_c3_gradient_fused_route_matches_oracle(c3, b, acq):
    """The gradient every C3 optimiser evaluation takes (generation/gen.py:
    194-222): forward + backward at the config size (n = 4096, q = 16, S = 512;
    b = 512 restarts, and a 2-rank shard's 256) goes through the fused
    W = R L^-1 -> dX pass (bo_post_w_dx, asserted), and dX at 16 spread t-batches
    equals torch.autograd through the oracle's qEI / qLogEI on those t-batches
    (rtol 1e-5).  best_f = max Y - 1.5 so the improvements are non-zero."""
    from botorch_amd.acquisition import qExpectedImprovement, qLogExpectedImprovement
    from botorch_amd.sampling import SobolQMCNormalSampler
    from oracle.acquisition import qei, qlogei
    from oracle.sampling import draw_sobol_normal_samples
    Xtr, Ytr, Xc, m, orc = c3
    best_f = Ytr.max().item() - 1.5
    cls, ref_fn = ((qExpectedImprovement, qei) if acq == "qei"
                   else (qLogExpectedImprovement, qlogei))
    acqf = cls(m, best_f, sampler=SobolQMCNormalSampler(torch.Size([S3]), seed=0))
    Xd = Xc[:b].to(DEV).requires_grad_(True)
    torch.ops.bo.last_backward_route()  # registers the op library
    v = acqf(Xd)
    (gd,) = torch.autograd.grad(v.sum(), Xd)
    assert torch.ops.bo.last_backward_route() == 1, "config-size gradient left the fused W -> dX pass"
    v, gd = v.detach().cpu(), gd.cpu()
    assert torch.isfinite(gd).all()
    idx = _spread_nonzero(v if acq == "qei" else v.exp(), 16)
    Z = draw_sobol_normal_samples(Q3, S3, 0)
    Xo = Xc[idx].clone().requires_grad_(True)
    ref = ref_fn(orc, Xo, Z, best_f)
    (go,) = torch.autograd.grad(ref.sum(), Xo)
    torch.testing.assert_close(v[idx], ref.detach(), rtol=1e-6, atol=1e-10)
    assert go.abs().amax(dim=(1, 2)).min() > 0
    torch.testing.assert_close(gd[idx], go, rtol=1e-5, atol=1e-8)


def _c4_models(golden):
    X = torch.from_numpy(golden["dtlz2_X"])
    Y = torch.from_numpy(golden["dtlz2_Y"])
    assert X.shape == (2048, 6)
    return X, Y, [_stgp(X, Y[:, t:t + 1], 0.6, 1e-3) for t in range(3)]


def _spy_member_routes(monkeypatch):
    """Counts of the ModelListGP gradient routes taken: the members' W in one
    launch (kernels.w_matrix_members -> bo_post_w_split_members), the per-member
    W (kernels.w_matrix), and the members' posterior backward passes in one
    launch (kernels.post_backward_jobs)."""
    from botorch_amd import kernels
    calls = {"w_members": 0, "w_single": 0, "pb_jobs": 0}

    def spy(name, key):
        orig = getattr(kernels, name)

        def f(*a, **k):
            calls[key] += 1
            return orig(*a, **k)
        monkeypatch.setattr(kernels, name, f)
    spy("w_matrix_members", "w_members")
    spy("w_matrix", "w_single")
    spy("post_backward_jobs", "pb_jobs")
    return calls


def test_c4_qehvi_gradient_member_routes_match_oracle(golden, monkeypatch):
    """C4 forward + backward at the config size (ModelListGP(3), n = 2048,
    q = 8, S = 128, b = 128) through the round-5 member-batched gradient routes
    -- the members' W = R L^-1 in one stream-K launch (bo_post_w_split_members,
    asserted: no per-member W) and the members' posterior backward passes in
    one launch (bo_post_backward_jobs, asserted) -- dX at 8 spread t-batches
    with non-zero values against torch.autograd through the oracle's qEHVI on
    the reference's 294 cells (multi_objective/monte_carlo.py:230-322,
    generation/gen.py:194-222), rtol 1e-5."""
    from botorch_amd import kernels
    from botorch_amd.acquisition import qExpectedHypervolumeImprovement
    from botorch_amd.models import ModelListGP
    from botorch_amd.multi_objective import FastNondominatedPartitioning
    from botorch_amd.sampling import SobolQMCNormalSampler
    from oracle.acquisition import qehvi
    from oracle.sampling import base_samples_multi_output
    torch.set_num_threads(16)
    X, Y, pairs = _c4_models(golden)
    ref_point = torch.full((3,), -1.1, dtype=torch.float64)
    part = FastNondominatedPartitioning(ref_point, Y)
    S, q, b = 128, 8, 128
    acqf = qExpectedHypervolumeImprovement(ModelListGP(*[p[0] for p in pairs]), ref_point.tolist(), part,
                                           sampler=SobolQMCNormalSampler(torch.Size([S]), seed=0))
    g = torch.Generator().manual_seed(2)
    P = X[torch.from_numpy(golden["dtlz2_pareto_mask"])]
    pick = torch.randint(0, P.shape[0], (b, q), generator=g)
    Xn = (P[pick] + 0.05 * torch.randn(b, q, 6, generator=g, dtype=torch.float64)).clamp(0, 1)
    calls = _spy_member_routes(monkeypatch)
    Xd = Xn.to(DEV).requires_grad_(True)
    v = acqf(Xd)
    (gd,) = torch.autograd.grad(v.sum(), Xd)
    kernels.check_ladder_status(DEV)
    assert calls["w_members"] >= 1 and calls["w_single"] == 0, \
        f"the members' W did not go as one launch: {calls}"
    assert calls["pb_jobs"] >= 1, f"the members' posterior backward was not one launch: {calls}"
    v, gd = v.detach().cpu(), gd.cpu()
    assert torch.isfinite(gd).all()
    idx = _spread_nonzero(v, 8)
    cl = torch.from_numpy(golden["dtlz2_cells_lower"])
    cu = torch.from_numpy(golden["dtlz2_cells_upper"])
    Zm = base_samples_multi_output(S, q, 3, 0)
    orcs = [p[1] for p in pairs]
    for i in idx.tolist():   # one t-batch at a time: the oracle's subset x cell tensors are large
        Xo = Xn[i:i + 1].clone().requires_grad_(True)
        ref = qehvi(orcs, Xo, Zm, cl, cu)
        (go,) = torch.autograd.grad(ref.sum(), Xo)
        torch.testing.assert_close(v[i:i + 1], ref.detach(), rtol=1e-7, atol=1e-10)
        assert go.abs().max() > 0
        torch.testing.assert_close(gd[i:i + 1], go, rtol=1e-5, atol=1e-8)


def test_c4_qnehvi_config_size_matches_oracle(golden, monkeypatch):
    """qNEHVI (section 8(f) rank 4) at the C4 shape: ModelListGP(3) on the
    reference's DTLZ2 draw (n = 2048), X_baseline = the training inputs pruned
    on the device (prune_baseline=True), S = 128 per-sample box decompositions,
    q = 8, b = 128 through the cached baseline roots and the member-batched
    routes (asserted).  Against QNEHVIOracle on the kept baseline: the baseline
    samples, the values of 4 spread t-batches by exact hypervolume differences
    (north_star's 1e-2 and the observed 1e-7), and value + dX through the
    per-sample cells (rtol 1e-7 / 1e-5) -- multi_objective/monte_carlo.py:
    325-468, utils/multi_objective/hypervolume.py:507-835."""
    from botorch_amd import kernels
    from botorch_amd.acquisition import qNoisyExpectedHypervolumeImprovement
    from botorch_amd.models import ModelListGP
    from botorch_amd.sampling import SobolQMCNormalSampler
    from oracle.acquisition import QNEHVIOracle
    torch.set_num_threads(16)
    X, Y, pairs = _c4_models(golden)
    ref_point = [-1.1] * 3
    S, q, b = 128, 8, 128
    torch.manual_seed(0)
    acqf = qNoisyExpectedHypervolumeImprovement(ModelListGP(*[p[0] for p in pairs]), ref_point,
                                                X.to(DEV), prune_baseline=True,
                                                sampler=SobolQMCNormalSampler(torch.Size([S]), seed=0))
    Xb = acqf.X_baseline.cpu()
    r = Xb.shape[0]
    assert 100 < r < 2048, f"pruned baseline size {r}"
    orc = QNEHVIOracle([p[1] for p in pairs], Xb, ref_point, S, seed=0)
    torch.testing.assert_close(acqf.baseline_samples, orc.Y_base, rtol=1e-8, atol=1e-10)
    g = torch.Generator().manual_seed(4)
    P = X[torch.from_numpy(golden["dtlz2_pareto_mask"])]
    pick = torch.randint(0, P.shape[0], (b, q), generator=g)
    Xn = (P[pick] + 0.05 * torch.randn(b, q, 6, generator=g, dtype=torch.float64)).clamp(0, 1)
    calls = _spy_member_routes(monkeypatch)
    from botorch_amd import acquisition
    orig_rf = acquisition._roots_forward_batched

    def spy_rf(*a, **k):
        calls["roots_batched"] = calls.get("roots_batched", 0) + 1
        return orig_rf(*a, **k)
    monkeypatch.setattr(acquisition, "_roots_forward_batched", spy_rf)
    Xd = Xn.to(DEV).requires_grad_(True)
    v = acqf(Xd)
    (gd,) = torch.autograd.grad(v.sum(), Xd)
    assert calls.get("roots_batched", 0) >= 1, f"the members' batched roots did not run: {calls}"
    with torch.no_grad():
        v_fwd = acqf(Xn.to(DEV)).cpu()
    kernels.check_ladder_status(DEV)
    assert calls["w_single"] == 0 and calls["w_members"] >= 1, calls
    v, gd = v.detach().cpu(), gd.cpu()
    torch.testing.assert_close(v_fwd, v, rtol=1e-10, atol=1e-13)
    idx = _spread_nonzero(v, 4)
    ref_exact = orc.value_exact(Xn[idx[:2]])
    torch.testing.assert_close(v[idx[:2]], ref_exact, rtol=1e-2, atol=1e-6)   # north_star MC bar
    torch.testing.assert_close(v[idx[:2]], ref_exact, rtol=1e-7, atol=1e-10)
    lo, hi = acqf.cell_lower_bounds.cpu(), acqf.cell_upper_bounds.cpu()
    for i in idx.tolist():
        Xo = Xn[i:i + 1].clone().requires_grad_(True)
        rv = orc.value_cells(Xo, lo, hi)
        (go,) = torch.autograd.grad(rv.sum(), Xo)
        torch.testing.assert_close(v[i:i + 1], rv.detach(), rtol=1e-7, atol=1e-10)
        assert go.abs().max() > 0
        torch.testing.assert_close(gd[i:i + 1], go, rtol=1e-5, atol=1e-8)
