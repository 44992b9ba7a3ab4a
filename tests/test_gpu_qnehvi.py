"""qNEHVI (acquisition/multi_objective/monte_carlo.py:325-468) on the fused
gfx950 path vs. the oracle: exact hypervolume differences per sample (values)
and the per-sample-cell restatement (values and gradients)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _setup(m, n=60, r=15, seed=0):
    from botorch_amd.models import ModelListGP, SingleTaskGP
    from botorch_amd.test_functions import DTLZ2
    from oracle.gp import ExactGPOracle, GPHyper
    g = torch.Generator().manual_seed(seed)
    X = torch.rand(n, 6, generator=g, dtype=torch.float64)
    Y = DTLZ2(dim=6, num_objectives=m).evaluate_true(X)  # positive; maximised above ref 0
    Y = Y + 0.05 * torch.randn(n, m, generator=g, dtype=torch.float64)
    models, oracles = [], []
    for t in range(m):
        mm = SingleTaskGP(X.to(DEV), Y[:, t:t + 1].to(DEV))
        mm.covar_module.lengthscale = torch.full((1, 6), 0.6, dtype=torch.float64)
        mm.likelihood.noise = torch.tensor([1e-2], dtype=torch.float64)
        models.append(mm.eval())
        oracles.append(ExactGPOracle(X, Y[:, t:t + 1],
                                     GPHyper(torch.full((6,), 0.6, dtype=torch.float64), 1e-2, 0.0)))
    return X, Y, ModelListGP(*models), oracles, X[:r]


@pytest.mark.parametrize("m,q,S", [(2, 1, 32), (2, 3, 16), (3, 2, 16)])
def test_qnehvi_value_matches_exact_hv(m, q, S):
    from botorch_amd.acquisition import qNoisyExpectedHypervolumeImprovement
    from botorch_amd.sampling import SobolQMCNormalSampler
    from oracle.acquisition import QNEHVIOracle
    X, Y, model, oracles, Xb = _setup(m)
    ref_point = [0.0] * m
    acqf = qNoisyExpectedHypervolumeImprovement(model, ref_point, Xb.to(DEV),
                                                sampler=SobolQMCNormalSampler(torch.Size([S]), seed=3))
    orc = QNEHVIOracle(oracles, Xb, ref_point, S, seed=3)
    torch.testing.assert_close(acqf.baseline_samples, orc.Y_base, rtol=1e-8, atol=1e-10)
    g = torch.Generator().manual_seed(m * 10 + q)
    Xc = torch.rand(5, q, 6, generator=g, dtype=torch.float64)
    with torch.no_grad():
        v = acqf(Xc.to(DEV)).cpu()
    ref = orc.value_exact(Xc)
    assert (ref > 0).any()
    torch.testing.assert_close(v, ref, rtol=1e-2, atol=1e-6)   # north_star MC bar
    torch.testing.assert_close(v, ref, rtol=1e-7, atol=1e-10)  # observed: same fp64 algebra


@pytest.mark.parametrize("m,q", [(2, 2), (3, 1)])
def test_qnehvi_gradient_matches_oracle(m, q):
    from botorch_amd.acquisition import qNoisyExpectedHypervolumeImprovement
    from botorch_amd.sampling import SobolQMCNormalSampler
    from oracle.acquisition import QNEHVIOracle
    X, Y, model, oracles, Xb = _setup(m, seed=1)
    S = 16
    ref_point = [0.0] * m
    acqf = qNoisyExpectedHypervolumeImprovement(model, ref_point, Xb.to(DEV),
                                                sampler=SobolQMCNormalSampler(torch.Size([S]), seed=7))
    orc = QNEHVIOracle(oracles, Xb, ref_point, S, seed=7)
    g = torch.Generator().manual_seed(5 + m)
    Xc = torch.rand(4, q, 6, generator=g, dtype=torch.float64)
    Xd = Xc.to(DEV).requires_grad_(True)
    v = acqf(Xd)
    (gd,) = torch.autograd.grad(v.sum(), Xd)
    Xo = Xc.clone().requires_grad_(True)
    lo, hi = acqf.cell_lower_bounds.cpu(), acqf.cell_upper_bounds.cpu()
    rv = orc.value_cells(Xo, lo, hi)
    (go,) = torch.autograd.grad(rv.sum(), Xo)
    torch.testing.assert_close(v.detach().cpu(), rv.detach(), rtol=1e-7, atol=1e-10)
    assert go.abs().max() > 0
    torch.testing.assert_close(gd.cpu(), go, rtol=1e-5, atol=1e-8)


def test_qnehvi_empty_front_and_pending():
    """Reference point above every baseline sample: one cell [ref, inf) per
    sample (test/acquisition/multi_objective/test_monte_carlo.py:976-994); pending
    points join the baseline (cache_pending)."""
    from botorch_amd.acquisition import qNoisyExpectedHypervolumeImprovement
    from botorch_amd.exceptions import UnsupportedError
    from botorch_amd.sampling import SobolQMCNormalSampler
    X, Y, model, oracles, Xb = _setup(2)
    acqf = qNoisyExpectedHypervolumeImprovement(model, [15.0, 14.0], Xb.to(DEV),
                                                sampler=SobolQMCNormalSampler(torch.Size([8]), seed=0))
    assert acqf.cell_lower_bounds.shape == (8, 1, 2)
    assert (acqf.cell_lower_bounds[..., 0] == 15).all() and (acqf.cell_lower_bounds[..., 1] == 14).all()
    assert torch.isinf(acqf.cell_upper_bounds).all()
    with pytest.raises(ValueError, match="m>=2"):
        qNoisyExpectedHypervolumeImprovement(model, [0.0], Xb.to(DEV))
    with pytest.raises(UnsupportedError):
        qNoisyExpectedHypervolumeImprovement(model, [0.0, 0.0], Xb.unsqueeze(0).to(DEV))
    acqf = qNoisyExpectedHypervolumeImprovement(model, [0.0, 0.0], Xb.to(DEV),
                                                sampler=SobolQMCNormalSampler(torch.Size([8]), seed=0))
    acqf.set_X_pending(X[20:22].to(DEV))
    assert acqf.X_baseline.shape[0] == Xb.shape[0] + 2 and acqf.X_pending is None


def test_prune_inferior_points_multi_objective():
    from botorch_amd.acquisition import prune_inferior_points_multi_objective
    X, Y, model, oracles, Xb = _setup(2, n=60, r=60)
    kept = prune_inferior_points_multi_objective(model, X.to(DEV), [0.0, 0.0], num_samples=256)
    assert 0 < kept.shape[0] < 60
    # the observed Pareto-optimal points (tiny noise -> posterior mean ~ data) survive
    from botorch_amd.multi_objective import is_non_dominated
    pm = is_non_dominated(Y) & (Y > 0).all(-1)
    kept_c = kept.cpu()
    for x in X[pm]:
        assert (kept_c == x).all(-1).any()


@pytest.mark.parametrize("m", [2, 3])
def test_prune_inferior_points_multi_objective_matches_oracle(m):
    """The kept baseline equals the oracle's restatement of the reference
    (multi_objective/utils.py:77-161) under the same global seed: the sampler
    seed is the reference's one torch.randint draw, the base samples its
    point-major / output-minor Sobol draw, the masks pareto.py's."""
    from botorch_amd.acquisition import prune_inferior_points_multi_objective
    from oracle.acquisition import prune_inferior_points_multi_objective as oracle_prune
    X, Y, model, oracles, _ = _setup(m, n=60)
    torch.manual_seed(7 + m)
    kept = prune_inferior_points_multi_objective(model, X.to(DEV), [0.0] * m, num_samples=256)
    after = torch.rand(2)  # the global stream continues where the reference's would
    torch.manual_seed(7 + m)
    seed = int(torch.randint(0, 1000000, (1,)).item())
    ref = oracle_prune(oracles, X, [0.0] * m, num_samples=256, seed=seed)
    assert torch.equal(torch.rand(2), after)
    assert 0 < ref.shape[0] < 60
    assert torch.equal(kept.cpu(), ref)


def _qnehvi(model, Xb, S, seed, m, **kw):
    from botorch_amd.acquisition import qNoisyExpectedHypervolumeImprovement
    from botorch_amd.sampling import SobolQMCNormalSampler
    return qNoisyExpectedHypervolumeImprovement(model, [0.0] * m, Xb.to(DEV),
                                                sampler=SobolQMCNormalSampler(torch.Size([S]),
                                                                              seed=seed), **kw)


def _value_and_grad(acqf, Xc):
    Xd = Xc.to(DEV).requires_grad_(True)
    v = acqf(Xd)
    (g,) = torch.autograd.grad(v.sum(), Xd)
    return v.detach().cpu(), g.cpu()


def test_qnehvi_pending_appended_without_cache():
    """cache_pending=False (hypervolume.py:821-822): the pending points are
    appended to every q-batch (concatenate_pending_points) -- the same value
    as the pending-free acquisition on [X, X_pending], gradient on X only."""
    from oracle.acquisition import QNEHVIOracle
    m, S, seed = 2, 16, 5
    X, Y, model, oracles, Xb = _setup(m, seed=2)
    Xp = X[40:42]
    acq_p = _qnehvi(model, Xb, S, seed, m, cache_pending=False, X_pending=Xp.to(DEV))
    acq_0 = _qnehvi(model, Xb, S, seed, m)
    assert acq_p.X_baseline.shape[0] == Xb.shape[0] and acq_p.X_pending.shape[0] == 2
    g = torch.Generator().manual_seed(11)
    Xc = torch.rand(4, 2, 6, generator=g, dtype=torch.float64)
    Xcat = torch.cat([Xc, Xp.expand(4, 2, 6)], dim=-2)
    v, gx = _value_and_grad(acq_p, Xc)
    v0, g0 = _value_and_grad(acq_0, Xcat)
    torch.testing.assert_close(v, v0, rtol=0, atol=0)
    torch.testing.assert_close(gx, g0[:, :2], rtol=0, atol=0)
    orc = QNEHVIOracle(oracles, Xb, [0.0] * m, S, seed=seed)
    torch.testing.assert_close(v, orc.value_exact(Xcat), rtol=1e-7, atol=1e-10)


def test_qnehvi_max_iep():
    """max_iep (hypervolume.py:795-820): up to max_iep new pending points ride
    along with the q-batch; more join the baseline (decompositions rebuilt)."""
    m, S, seed = 2, 16, 3
    X, Y, model, oracles, Xb = _setup(m, seed=4)
    acqf = _qnehvi(model, Xb, S, seed, m, max_iep=2)
    g = torch.Generator().manual_seed(7)
    Xc = torch.rand(3, 1, 6, generator=g, dtype=torch.float64)
    acqf.set_X_pending(X[50:52].to(DEV))  # 2 <= max_iep: appended
    assert acqf.X_baseline.shape[0] == Xb.shape[0] and acqf.X_pending.shape[0] == 2
    ref = _qnehvi(model, Xb, S, seed, m, cache_pending=False, X_pending=X[50:52].to(DEV))
    with torch.no_grad():
        torch.testing.assert_close(acqf(Xc.to(DEV)), ref(Xc.to(DEV)), rtol=0, atol=0)
    acqf.set_X_pending(X[50:53].to(DEV))  # 3 new > max_iep: joins the baseline
    assert acqf.X_baseline.shape[0] == Xb.shape[0] + 3 and acqf.X_pending is None
    fresh = _qnehvi(model, torch.cat([Xb, X[50:53]]), S, seed, m)
    with torch.no_grad():
        torch.testing.assert_close(acqf(Xc.to(DEV)), fresh(Xc.to(DEV)), rtol=0, atol=0)


@pytest.mark.parametrize("m", [2, 3])
def test_qnehvi_not_incremental(m):
    """incremental_nehvi=False (hypervolume.py:741-742, 807-812): absorbing
    pending points carries mean_s (HV_s(baseline + pending) - HV_s(baseline))+
    in prev_nehvi; checked against exact hypervolumes of the oracle's samples."""
    from oracle.acquisition import QNEHVIOracle
    S, seed = 16, 9
    X, Y, model, oracles, Xb = _setup(m, seed=6)
    Xp = X[45:48]
    acqf = _qnehvi(model, Xb, S, seed, m, incremental_nehvi=False)
    init = QNEHVIOracle(oracles, Xb, [0.0] * m, S, seed=seed).initial_hv
    torch.testing.assert_close(acqf._initial_hvs.cpu(), init, rtol=1e-9, atol=1e-12)
    acqf.set_X_pending(Xp.to(DEV))
    after = QNEHVIOracle(oracles, torch.cat([Xb, Xp]), [0.0] * m, S, seed=seed).initial_hv
    prev = (after - init).clamp_min(0.0).mean()
    assert prev > 0
    torch.testing.assert_close(acqf._prev_nehvi.cpu(), prev, rtol=1e-9, atol=1e-12)
    fresh = _qnehvi(model, torch.cat([Xb, Xp]), S, seed, m)
    g = torch.Generator().manual_seed(3)
    Xc = torch.rand(3, 2, 6, generator=g, dtype=torch.float64)
    with torch.no_grad():
        torch.testing.assert_close(acqf(Xc.to(DEV)), fresh(Xc.to(DEV)) + acqf._prev_nehvi,
                                   rtol=0, atol=0)


def test_qnehvi_approximate_partitioning():
    """alpha > 0, m = 3: the per-sample cells are NondominatedPartitioning's
    approximate binary partitioning (bo_nd_partition_alpha_host); the value is
    the inclusion-exclusion over those cells (oracle restatement), and can only
    fall below the exact one (dropped cells are non-dominated space)."""
    from botorch_amd import kernels
    from oracle.acquisition import QNEHVIOracle
    m, S, seed = 3, 8, 2
    X, Y, model, oracles, Xb = _setup(m, seed=8)
    acqf = _qnehvi(model, Xb, S, seed, m, alpha=0.01)
    lo, hi = kernels.nd_partition_host(acqf.baseline_samples, torch.zeros(m, dtype=torch.float64),
                                       alpha=0.01)
    assert torch.equal(acqf.cell_lower_bounds.cpu(), lo) and torch.equal(acqf.cell_upper_bounds.cpu(), hi)
    g = torch.Generator().manual_seed(1)
    Xc = torch.rand(4, 2, 6, generator=g, dtype=torch.float64)
    orc = QNEHVIOracle(oracles, Xb, [0.0] * m, S, seed=seed)
    v, gx = _value_and_grad(acqf, Xc)
    Xo = Xc.clone().requires_grad_(True)
    rv = orc.value_cells(Xo, lo, hi)
    (go,) = torch.autograd.grad(rv.sum(), Xo)
    torch.testing.assert_close(v, rv.detach(), rtol=1e-7, atol=1e-10)
    torch.testing.assert_close(gx, go, rtol=1e-5, atol=1e-8)
    assert (v <= orc.value_exact(Xc) + 1e-10).all()


@pytest.mark.parametrize("m,q", [(2, 2), (3, 1)])
def test_qnehvi_without_cached_root(m, q):
    """cache_root=False: the joint (r + q) root of every t-batch per forward;
    value and gradient against the oracle's joint sampling over the same cells,
    and the cached-root value (the same quantity without jitter)."""
    from oracle.acquisition import QNEHVIOracle
    S, seed = 16, 4
    X, Y, model, oracles, Xb = _setup(m, seed=3)
    acq_j = _qnehvi(model, Xb, S, seed, m, cache_root=False)
    acq_c = _qnehvi(model, Xb, S, seed, m)
    assert torch.equal(acq_j.cell_lower_bounds, acq_c.cell_lower_bounds)
    g = torch.Generator().manual_seed(2 + m)
    Xc = torch.rand(4, q, 6, generator=g, dtype=torch.float64)
    v, gx = _value_and_grad(acq_j, Xc)
    vc, gc = _value_and_grad(acq_c, Xc)
    orc = QNEHVIOracle(oracles, Xb, [0.0] * m, S, seed=seed)
    Xo = Xc.clone().requires_grad_(True)
    lo, hi = acq_j.cell_lower_bounds.cpu(), acq_j.cell_upper_bounds.cpu()
    rv = orc.value_cells_joint(Xo, lo, hi)
    (go,) = torch.autograd.grad(rv.sum(), Xo)
    assert (rv > 0).any()
    torch.testing.assert_close(v, rv.detach(), rtol=1e-7, atol=1e-10)
    torch.testing.assert_close(gx, go, rtol=1e-5, atol=1e-8)
    torch.testing.assert_close(v, vc, rtol=1e-6, atol=1e-9)
    torch.testing.assert_close(gx, gc, rtol=1e-4, atol=1e-7)


def test_qnehvi_members_batched_roots_match_per_member(monkeypatch):
    """At a size whose one-model plan splits k (n = 1024: the members' route
    stores R^T stacked), the members' cached-root terms go as batched GEMMs
    over the members (acquisition._roots_forward_batched); values and
    gradients equal the per-member route (s^2 folded into the operands:
    rounding only)."""
    import torch
    from botorch_amd import acquisition, kernels
    from botorch_amd.acquisition import qNoisyExpectedHypervolumeImprovement
    from botorch_amd.sampling import SobolQMCNormalSampler
    X, Y, model, _, _ = _setup(3, n=1024, r=40, seed=3)
    assert kernels.split_plan(32, 4, 1024)[0] != 0  # stream-K: the members' route applies
    acqf = qNoisyExpectedHypervolumeImprovement(model, [-1.1] * 3, X[:40].to(DEV),
                                                sampler=SobolQMCNormalSampler(torch.Size([64]), seed=0),
                                                prune_baseline=False)
    Xc = torch.rand(32, 4, 6, dtype=torch.float64, generator=torch.Generator().manual_seed(1)).to(DEV)
    calls = []
    orig = acquisition._roots_forward_batched

    def spy(*a, **k):
        calls.append(1)
        return orig(*a, **k)

    monkeypatch.setattr(acquisition, "_roots_forward_batched", spy)

    def run():
        Xg = Xc.clone().requires_grad_(True)
        v = acqf(Xg)
        (g,) = torch.autograd.grad(v.sum(), Xg)
        with torch.no_grad():
            v2 = acqf(Xc)
        kernels.check_ladder_status(DEV)
        return v.detach().cpu(), g.cpu(), v2.cpu()

    v1, g1, w1 = run()
    assert calls, "the batched roots route did not run"
    monkeypatch.setattr(acquisition, "_roots_batched", lambda *a, **k: False)
    v0, g0, w0 = run()
    assert (v0 > 0).sum() > 5
    torch.testing.assert_close(v1, v0, rtol=1e-10, atol=1e-13)
    torch.testing.assert_close(w1, w0, rtol=1e-10, atol=1e-13)
    torch.testing.assert_close(g1, g0, rtol=1e-8, atol=1e-11)


def test_qnehvi_batched_roots_rebuilt_after_pending_join(monkeypatch):
    """The members' stacked root operands (_roots_forward_batched's L_rr^-1 /
    P_b / Z_base stacks, the backward's Q_b stack) belong to the roots they were
    built from: after set_X_pending grows the baseline past max_iep (the roots
    rebuilt with a larger r, hypervolume.py:795-820) the batched route must
    rebuild them.  On the n = 1024 batched route: values and gradients after
    the join equal a fresh acquisition on [X_baseline; X_pending]."""
    from botorch_amd import acquisition, kernels
    X, Y, model, _, _ = _setup(3, n=1024, r=40, seed=3)
    assert kernels.split_plan(32, 4, 1024)[0] != 0
    calls = []
    orig = acquisition._roots_forward_batched

    def spy(*a, **k):
        calls.append(1)
        return orig(*a, **k)

    monkeypatch.setattr(acquisition, "_roots_forward_batched", spy)
    acqf = _qnehvi(model, X[:40], 32, 0, 3)
    Xc = torch.rand(32, 4, 6, dtype=torch.float64, generator=torch.Generator().manual_seed(1))
    _value_and_grad(acqf, Xc)              # builds the stacks for r = 40
    assert calls
    Xp = X[600:603]
    acqf.set_X_pending(Xp.to(DEV))         # 3 > max_iep = 0: joins the baseline
    assert acqf.X_baseline.shape[0] == 43 and acqf.X_pending is None
    n0 = len(calls)
    v, g = _value_and_grad(acqf, Xc)
    with torch.no_grad():
        w = acqf(Xc.to(DEV)).cpu()
    assert len(calls) > n0, "the batched roots route did not run after the join"
    fresh = _qnehvi(model, torch.cat([X[:40], Xp]), 32, 0, 3)
    v0, g0 = _value_and_grad(fresh, Xc)
    kernels.check_ladder_status(DEV)
    assert (v0 > 0).sum() > 5
    torch.testing.assert_close(v, v0, rtol=0, atol=0)
    torch.testing.assert_close(w, v0, rtol=1e-12, atol=1e-14)
    torch.testing.assert_close(g, g0, rtol=0, atol=0)
