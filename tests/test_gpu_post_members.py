"""Member-batched stream-K posterior (bo_post_partials_members, round 5): the
posterior partials of a ModelListGP's members (models/model_list_gp.py ->
[G] ModelListGP.posterior, one posterior per member) in ONE stream-K launch
over all members' 128 x 128 tiles and one split-k reduction, where the
one-model plan is stream-K.  Compared member by member with the one-model
128-tile route (the same sums cut at other k positions: 1e-12 relative, 1e-11 absolute), R^T
included, and end to end through qEHVI values and gradients (C4's shape)."""
import ctypes

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _models(n, m=3, seed=0):
    from botorch_amd.models import SingleTaskGP
    from botorch_amd.test_functions import DTLZ2
    g = torch.Generator().manual_seed(seed)
    X = torch.rand(n, 6, generator=g, dtype=torch.float64)
    Y = -DTLZ2(dim=6, num_objectives=m, negate=True).evaluate_true(X)
    out = []
    for t in range(m):
        mm = SingleTaskGP(X.to(DEV), Y[:, t:t + 1].to(DEV))
        mm.covar_module.lengthscale = torch.full((1, 6), 0.5 + 0.1 * t, dtype=torch.float64)
        mm.likelihood.noise = torch.tensor([1e-3], dtype=torch.float64)
        out.append(mm.eval())
    return X, Y, out


def _members_work(nm, B, q, n):
    from botorch_amd._lib import check, lib
    we = ctypes.c_int64()
    check(lib().bo_post_members_work(nm, B, q, n, ctypes.byref(we)), "post_members_work")
    return we.value


@pytest.mark.parametrize("n,B,q,store_R", [(2048, 128, 8, False),   # C4
                                           (2048, 128, 8, True),
                                           (1500, 40, 5, True)])    # ragged n, odd q
def test_members_route_matches_one_model_route(n, B, q, store_R):
    from botorch_amd import kernels
    _, _, models = _models(n)
    if _members_work(len(models), B, q, n) < 0:
        pytest.skip("one-model plan not stream-K at this shape")
    caches = [mm.prediction_cache() for mm in models]
    X = torch.rand(B, q, 6, dtype=torch.float64, generator=torch.Generator().manual_seed(7)).to(DEV)
    pps = kernels._post_members_streamk(caches, X, store_R,
                                        _members_work(len(models), B, q, n))
    for c, pp in zip(caches, pps):
        ref = kernels.post_partials(c, X, store_R=store_R, small=False)
        assert pp.Spart.shape == ref.Spart.shape
        # per-tile partials summed: the same R R^T / R beta as the one-model route
        # (k-sums cut at other positions: rounding of O(1e-16) x the terms'
        # magnitude, so an absolute floor for the entries that cancel)
        torch.testing.assert_close(pp.Spart.sum(0), ref.Spart.sum(0), rtol=1e-12, atol=1e-11)
        torch.testing.assert_close(pp.mpart.sum(0), ref.mpart.sum(0), rtol=1e-12, atol=1e-11)
        if store_R:
            torch.testing.assert_close(pp.Rt, ref.Rt, rtol=1e-12, atol=1e-11)


def test_qehvi_members_route_values_and_gradients(monkeypatch):
    """C4-shaped qEHVI through the members route and through one launch per
    member (BO_POST_MEMBERS off): values 1e-12, gradients 1e-10."""
    from botorch_amd import kernels
    from botorch_amd.acquisition import qExpectedHypervolumeImprovement
    from botorch_amd.models import ModelListGP
    from botorch_amd.multi_objective import FastNondominatedPartitioning
    from botorch_amd.sampling import SobolQMCNormalSampler
    _, Y, models = _models(2048)
    ref = torch.full((3,), -1.1, dtype=torch.float64)
    part = FastNondominatedPartitioning(ref, Y)
    acqf = qExpectedHypervolumeImprovement(ModelListGP(*models), ref.tolist(), part,
                                           sampler=SobolQMCNormalSampler(torch.Size([128]), seed=0))
    X = torch.rand(128, 8, 6, dtype=torch.float64, generator=torch.Generator().manual_seed(3)).to(DEV)
    assert _members_work(3, 128, 8, 2048) >= 0  # C4 takes the members route

    def run():
        Xg = X.clone().requires_grad_(True)
        v = acqf(Xg)
        (g,) = torch.autograd.grad(v.sum(), Xg)
        return v.detach().cpu(), g.cpu()

    v1, g1 = run()
    monkeypatch.setattr(kernels, "MEMBERS_STREAMK", False)
    v0, g0 = run()
    assert (v0 > 0).sum() > 10
    torch.testing.assert_close(v1, v0, rtol=1e-12, atol=1e-14)
    torch.testing.assert_close(g1, g0, rtol=1e-10, atol=1e-12)


def test_qehvi_member_status_words(monkeypatch):
    """The members' ladder outcomes reach the host through the pinned words
    their finalisation launches fold into (sticky max): a word seeded with a
    jitter warns, one seeded with a failure raises NotPSDError, clean calls
    neither (the reference's per-member psd_safe_cholesky outcomes)."""
    import warnings
    from botorch_amd import kernels
    from botorch_amd.acquisition import qExpectedHypervolumeImprovement
    from botorch_amd.exceptions import NotPSDError, NumericalWarning
    from botorch_amd.models import ModelListGP
    from botorch_amd.multi_objective import FastNondominatedPartitioning
    from botorch_amd.sampling import SobolQMCNormalSampler
    _, Y, models = _models(512)
    ref = torch.full((3,), -1.1, dtype=torch.float64)
    acqf = qExpectedHypervolumeImprovement(ModelListGP(*models), ref.tolist(),
                                           FastNondominatedPartitioning(ref, Y),
                                           sampler=SobolQMCNormalSampler(torch.Size([64]), seed=0))
    X = torch.rand(16, 4, 6, dtype=torch.float64, generator=torch.Generator().manual_seed(2)).to(DEV)
    with warnings.catch_warnings():
        warnings.simplefilter("error", NumericalWarning)
        acqf(X)  # clean: no warning, no error (the native forward-only call)
        kernels.check_ladder_status(X.device)  # its deferred outcome: clean
        acqf(X.clone().requires_grad_(True))  # the autograd path
    # a t-batch with a repeated point: its q x q posterior covariance is
    # singular, the ladder adds the first jitter (psd_safe_cholesky's
    # warning); the native call's outcome is deferred (as the eager qEI's) to
    # the next call or the end-of-loop poll
    Xd = X.clone()
    Xd[3, 1] = Xd[3, 0]
    with pytest.warns(NumericalWarning, match="1.0e-08"):
        v_native = acqf(Xd)
        kernels.check_ladder_status(X.device)
    # the gradient path: the outcome is read at the end of the backward
    # (kernels._LadderRing) -- within the forward + backward call -- or, for a
    # forward whose backward never runs, at check_ladder_status
    Xg = Xd.clone().requires_grad_(True)
    with pytest.warns(NumericalWarning, match="1.0e-08"):
        v_grad = acqf(Xg)
        torch.autograd.grad(v_grad.sum(), Xg)
    torch.testing.assert_close(v_native, v_grad.detach(), rtol=1e-12, atol=1e-14)
    with warnings.catch_warnings():
        warnings.simplefilter("error", NumericalWarning)
        acqf(Xd.clone().requires_grad_(True))  # not read in the forward
    with pytest.warns(NumericalWarning, match="1.0e-08"):
        kernels.check_ladder_status(X.device)
    # seeded words (the autograd path's pinned status pairs)
    X = X.clone().requires_grad_(True)
    orig = kernels._PinnedStatus.arm
    seed = {}

    def arm(self, m):
        out = orig(self, m)
        for i, v in seed.items():
            self.words[i] = v
        return out

    monkeypatch.setattr(kernels._PinnedStatus, "arm", arm)
    seed.update({3: 1e-6})  # member 1 added jitter
    with pytest.warns(NumericalWarning, match="1.0e-06"):
        torch.autograd.grad(acqf(X).sum(), X)
    seed.clear()
    seed.update({4: 1.0})  # member 2 failed
    with pytest.raises(NotPSDError):
        torch.autograd.grad(acqf(X).sum(), X)
    with pytest.raises(NotPSDError):  # a forward alone: at the poll
        acqf(X)
        kernels.check_ladder_status(X.device)
    seed.clear()
    with warnings.catch_warnings():
        warnings.simplefilter("error", NumericalWarning)
        torch.autograd.grad(acqf(X).sum(), X)
        kernels.check_ladder_status(X.device)


def test_kxt_rows_members_bit_equal_to_per_member():
    """bo_post_kxt_rows_members (one launch, grid z = model) writes exactly
    what bo_post_kxt_rows writes per model: the rows and K*x^T."""
    from botorch_amd import kernels
    from botorch_amd._lib import check, lib
    _, _, models = _models(1500)
    caches = [mm.prediction_cache() for mm in models]
    X = torch.rand(40, 5, 6, dtype=torch.float64, generator=torch.Generator().manual_seed(9)).to(DEV)
    _, nrows_pad, _ = kernels.geometry(40, 5, 1500)
    Xqs, Kts = kernels._kxt_rows_members(caches, X, nrows_pad)
    st = kernels._stream(X.device)
    for c, Xq, Kt in zip(caches, Xqs, Kts):
        Xq1 = torch.empty_like(Xq)
        Kt1 = torch.empty_like(Kt)
        check(lib().bo_post_kxt_rows(c.kind, kernels._p(X), 40, 5, 6, kernels._p(c.lengthscale),
                                     kernels._p(c.Xt_scaled), c.n, c.outputscale, kernels._p(Xq1),
                                     kernels._p(Kt1), st), "post_kxt_rows")
        assert torch.equal(Xq, Xq1)
        assert torch.equal(Kt, Kt1)


def test_qmc_finalize_members_bit_equal_to_per_member():
    """bo_qmc_finalize_members (one launch, grid B x models, root-only mode)
    writes exactly what bo_qmc_finalize does per member: means, q x q roots,
    ladder info and jitter, and the fused status words."""
    import ctypes
    from botorch_amd import _lib, kernels
    from botorch_amd._lib import check, lib
    _, _, models = _models(1500)
    caches = [mm.prediction_cache() for mm in models]
    X = torch.rand(40, 5, 6, dtype=torch.float64, generator=torch.Generator().manual_seed(4)).to(DEV)
    X[7, 1] = X[7, 0]  # one t-batch needs the jitter ladder
    pps = kernels.post_partials_members(caches, X)
    stats = [mm.outcome_stats() for mm in models]
    refs = []
    for c, pp, (ym, ys) in zip(caches, pps, stats):
        refs.append(kernels.qmc_finalize(c, pp, _lib.QMC_CHOL, ym, ys, want_mean=True, want_cov=False,
                                         want_L=True))
    M, B, q = len(models), 40, 5
    f64 = dict(dtype=torch.float64, device=DEV)
    mean = torch.empty(M, B, q, **f64)
    L = torch.empty(M, B, q, q, **f64)
    info = torch.empty(M, B, dtype=torch.int32, device=DEV)
    jit = torch.empty(M, B, **f64)
    status = torch.zeros(M, 2, **f64)
    count = torch.zeros(M, dtype=torch.int32, device=DEV)
    P = ctypes.c_void_p * M
    D = ctypes.c_double * M
    nparts = int(pps[0].Spart.shape[0]) if pps[0].Spart.shape[0] != pps[0].nC else 0
    check(lib().bo_qmc_finalize_members(
        M, caches[0].kind, B, q, P(*[p.Xq.data_ptr() for p in pps]),
        P(*[p.Spart.data_ptr() for p in pps]), P(*[p.mpart.data_ptr() for p in pps]), caches[0].n,
        D(*[c.outputscale for c in caches]), D(*[c.constant for c in caches]),
        D(*[s[0] for s in stats]), D(*[s[1] for s in stats]), kernels.CHOLESKY_MAX_TRIES,
        kernels.CHOLESKY_JITTER_F64, P(*[mean[m].data_ptr() for m in range(M)]),
        P(*[L[m].data_ptr() for m in range(M)]), P(*[info[m].data_ptr() for m in range(M)]),
        P(*[jit[m].data_ptr() for m in range(M)]), nparts,
        P(*[status[m].data_ptr() for m in range(M)]),
        P(*[count[m:].data_ptr() for m in range(M)]), None, 0, 0, None, 0,
        kernels._stream(X.device)),
        "qmc_finalize_members")
    for m, r in enumerate(refs):
        assert torch.equal(mean[m], r["mean"])
        assert torch.equal(L[m], r["L"])
        assert torch.equal(info[m], r["info"])
        assert torch.equal(jit[m], r["jitter"])
        assert float(status[m, 0]) == float(r["info"].max())
        assert float(status[m, 1]) == float(r["jitter"].max())
    assert float(jit.max()) > 0  # the repeated point did take the ladder


@pytest.mark.parametrize("n,B,q", [(2048, 128, 8),    # C4
                                   (1500, 40, 5)])    # ragged n, odd q
def test_w_matrix_members_matches_per_member(n, B, q):
    """bo_post_w_split_members (all members' W^T = L^{-T} R^T in one
    stream-K launch) against w_matrix per member; the members' plan cuts the
    k-sums at other positions (1e-12 relative, 1e-11 absolute)."""
    from botorch_amd import kernels
    from botorch_amd._lib import check, lib
    _, _, models = _models(n)
    nm = len(models)
    we = ctypes.c_int64()
    check(lib().bo_post_w_members_work(nm, B, q, n, ctypes.byref(we)), "post_w_members_work")
    if we.value < 0:
        pytest.skip("one-model W plan not stream-K at this shape")
    caches = [mm.prediction_cache() for mm in models]
    X = torch.rand(B, q, 6, dtype=torch.float64, generator=torch.Generator().manual_seed(9)).to(DEV)
    pps = [kernels.post_partials(c, X, store_R=True, small=False) for c in caches]
    Ws = kernels.w_matrix_members(caches, pps)
    for c, pp, W in zip(caches, pps, Ws):
        ref = kernels.w_matrix(c, pp)
        assert W.kmajor == ref.kmajor and W.t.shape == ref.t.shape
        torch.testing.assert_close(W.t, ref.t, rtol=1e-12, atol=1e-11)


def test_post_backward_jobs_matches_sequential_passes():
    """bo_post_backward_jobs (the members' training + baseline passes in one
    launch, per-job dX slices summed) against post_backward accumulated pass by
    pass (the same per-pass sums, added in another order: 1e-12)."""
    from botorch_amd import kernels
    n, B, q, r = 1500, 40, 5, 37
    _, _, models = _models(n)
    caches = [mm.prediction_cache() for mm in models]
    g = torch.Generator().manual_seed(11)
    X = torch.rand(B, q, 6, dtype=torch.float64, generator=g).to(DEV)
    jobs = []
    for c in caches:
        pp = kernels.post_partials(c, X, store_R=True, small=False)
        W = kernels.w_matrix(c, pp)
        dmean = torch.randn(B, q, dtype=torch.float64, generator=g).to(DEV)
        dcov = torch.randn(B, q, q, dtype=torch.float64, generator=g).to(DEV)
        E = torch.randn(pp.nrows_pad, c.np, dtype=torch.float64, generator=g).to(DEV)
        Xb = torch.zeros(r, kernels.DP, dtype=torch.float64)
        Xb[:, :6] = torch.rand(r, 6, dtype=torch.float64, generator=g)
        Eb = torch.randn(pp.nrows_pad, r, dtype=torch.float64, generator=g).to(DEV)
        jobs.append(dict(cache=c, pp=pp, W=W, dmean=dmean, dcov=dcov, ystd=0.7, E=E))
        jobs.append(dict(cache=c, pp=pp, ystd=0.7, E=Eb, Xt_scaled=Xb.to(DEV), n=r))
    got = kernels.post_backward_jobs(jobs)
    ref = None
    for j in jobs:
        ref = kernels.post_backward(j["cache"], j["pp"], j.get("W"), j.get("dmean"), j.get("dcov"),
                                    j["ystd"], E=j["E"], Xt_scaled=j.get("Xt_scaled"), n=j.get("n"),
                                    dX=ref)
    torch.testing.assert_close(got, ref, rtol=1e-12, atol=1e-12)
