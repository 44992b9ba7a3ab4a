"""Device L-BFGS-B (bo_lbfgsb_step, csrc/lbfgsb.hip) against scipy 1.15's
L-BFGS-B, the optimiser of gen_candidates_scipy (botorch/generation/gen.py:
252-267).

* The kernel driven directly: 16 restarts in one launch per evaluation, f and g
  computed on the host by the same function scipy sees, so the only difference
  left is the 64-lane summation order of the kernel's dot products.  Every
  restart must request scipy's trial points in scipy's order.
* gen_candidates_device at b = 1 on qEI equals gen_candidates_scipy (the
  reference's joint problem is the restart's own problem there).
* b = 8 restarts at once equal scipy run on each restart alone.
"""
import ctypes

import numpy as np
import pytest
import torch

from tests.lbfgsb_harness import scipy_trials
from tests.test_lbfgsb_cpu import _hartmann_batch, _rosen

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def _drive(fgs, x0s, lo, hi, m=10, maxiter=15000, max_evals=3000):
    """Run the kernel on B restarts (objective i = fgs[i], evaluated on the host)."""
    from botorch_amd import _lib
    from botorch_amd.optim import _LBFGSBState
    B, n = x0s.shape
    X0 = torch.from_numpy(np.clip(x0s, lo, hi)).to(DEV)
    st = _LBFGSBState(X0.view(B, 1, n), m)
    lo_d = torch.from_numpy(np.ascontiguousarray(lo)).to(DEV)
    hi_d = torch.from_numpy(np.ascontiguousarray(hi)).to(DEV)
    trials = [[] for _ in range(B)]
    done = [False] * B
    for _ in range(max_evals):
        xt = st.xt.cpu().numpy()
        fs, gs = np.zeros(B), np.zeros((B, n))
        for b in range(B):
            if not done[b]:
                trials[b].append(xt[b].copy())
            fs[b], gs[b] = fgs[b](xt[b].copy())
        ft = torch.from_numpy(fs).to(DEV)
        gt = torch.from_numpy(gs).to(DEV)
        a = _lib.LbfgsbArgs(B=B, n=n, m=m, maxls=20, maxiter=maxiter, maxfun=15000,
                            ftol=2.2204460492503131e-09, pgtol=1e-5, lower=lo_d, upper=hi_d,
                            xt=st.xt, ft=ft, gt=gt, v=st.v, iv=st.iv, ws=st.ws, wy=st.wy,
                            mat=st.mat, ds=st.ds, is_=st.is_)
        _lib.check(_lib.lib().bo_lbfgsb_step_v(ctypes.byref(a), None), "lbfgsb")
        torch.cuda.synchronize()
        status = st.status.cpu().numpy()
        done = [bool(s > 0) for s in status]
        if all(done):
            break
    return trials, st.x.cpu().numpy(), st.f.cpu().numpy(), st.status.cpu().numpy(), st.nit.cpu().numpy()


@pytest.mark.parametrize("q,m,maxiter", [(2, 10, 15000), (3, 5, 40), (1, 3, 15000)])
def test_kernel_trial_points_equal_scipy(q, m, maxiter):
    n = 6 * q
    rng = np.random.default_rng(7 + q)
    B = 16
    x0s = rng.uniform(0, 1, (B, n))
    lo, hi = np.zeros(n), np.ones(n)
    fg = _hartmann_batch(q)
    trials, x, f, status, nit = _drive([fg] * B, x0s, lo, hi, m=m, maxiter=maxiter)
    exact = 0
    for b in range(B):
        sp, res = scipy_trials(fg, x0s[b], list(zip(lo, hi)), maxcor=m, maxiter=maxiter)
        k = min(25, len(sp))
        assert len(trials[b]) >= k
        for i in range(k):  # the opening of every run: scipy's points in scipy's order
            np.testing.assert_allclose(trials[b][i], sp[i], atol=1e-9, rtol=0,
                                       err_msg=f"restart {b} trial {i}")
        np.testing.assert_allclose(f[b], res.fun, rtol=1e-7, atol=1e-9)
        if len(trials[b]) == len(sp) and nit[b] == res.nit and np.abs(x[b] - res.x).max() < 1e-8:
            exact += 1
    # whole runs: summation order may show only near convergence of a few runs
    assert exact >= B - 2, exact


def test_kernel_box_rosenbrock_long_run():
    """44 evaluations, active upper bounds, history wrap-around (34 iterations, m = 10)."""
    rng = np.random.default_rng(0)
    n = 10
    x0 = rng.uniform(-1, 1, n)
    lo, hi = np.full(n, -1.5), np.full(n, 0.8)
    trials, x, f, status, nit = _drive([_rosen], x0[None], lo, hi)
    sp, res = scipy_trials(_rosen, x0, list(zip(lo, hi)))
    assert len(trials[0]) == len(sp) and nit[0] == res.nit and status[0] == 2
    for a, b in zip(sp, trials[0]):
        np.testing.assert_allclose(b, a, atol=1e-9, rtol=0)
    np.testing.assert_allclose(x[0], res.x, atol=1e-10, rtol=0)


def _qei_setup():
    from botorch_amd.acquisition import qExpectedImprovement
    from botorch_amd.models import SingleTaskGP
    from botorch_amd.optim import gen_batch_initial_conditions
    from botorch_amd.sampling import SobolQMCNormalSampler
    from tests.test_gpu_fit_optim import _data
    X, Y = _data(128)
    m = SingleTaskGP(X.to(DEV), Y.to(DEV)).eval()
    acqf = qExpectedImprovement(m, Y.max().item() - 0.2,
                                sampler=SobolQMCNormalSampler(torch.Size([128]), seed=0))
    bounds = torch.stack([torch.zeros(6), torch.ones(6)]).to(torch.float64).to(DEV)
    ics = gen_batch_initial_conditions(acqf, bounds, q=2, num_restarts=8, raw_samples=128,
                                       options={"seed": 1})
    return acqf, bounds, ics


def test_gen_candidates_device_b1_equals_scipy():
    """One restart: the reference's L-BFGS-B problem is the restart's own, so
    the device optimiser returns scipy's candidate."""
    from botorch_amd.optim import gen_candidates_device, gen_candidates_scipy
    acqf, bounds, ics = _qei_setup()
    for i in range(4):
        ic = ics[i:i + 1]
        cd, vd = gen_candidates_device(ic, acqf, bounds[0], bounds[1])
        cs, vs = gen_candidates_scipy(ic, acqf, bounds[0], bounds[1])
        torch.testing.assert_close(cd, cs, atol=1e-7, rtol=0)
        torch.testing.assert_close(vd, vs, atol=1e-10, rtol=1e-8)


@pytest.mark.parametrize("opts", [{}, {"compact": True, "compact_min": 1}, {"maxiter": 2}])
def test_gen_candidates_device_values_are_the_candidates_values(opts):
    """Converged restarts return -f from their L-BFGS-B state instead of a
    final forward: equal to the acquisition at the returned candidates (also
    after compaction, whose evaluations sum in another order); a run that
    stops on maxiter evaluates the candidates."""
    from botorch_amd.optim import gen_candidates_device
    acqf, bounds, ics = _qei_setup()
    cd, vd = gen_candidates_device(ics, acqf, bounds[0], bounds[1], options=opts)
    st = gen_candidates_device.last_state
    converged = set(st.status.cpu().tolist()) <= {1, 2}
    assert converged == ("maxiter" not in opts)
    with torch.no_grad():
        ve = acqf(cd)
    assert vd.shape == ve.shape and vd.dtype == ve.dtype
    torch.testing.assert_close(vd, ve, rtol=1e-10, atol=1e-13)


def test_gen_candidates_device_early_checks_same_result():
    """The early status reads (after evaluations 1 and 2 where the batch can
    shrink) move the shrink earlier, not the result: the same candidates and
    values as reading every 4 evaluations, to the rounding of the smaller
    batch's evaluation order."""
    from botorch_amd.optim import gen_candidates_device
    acqf, bounds, ics = _qei_setup()
    opts = {"compact": True, "compact_min": 1}
    c1, v1 = gen_candidates_device(ics, acqf, bounds[0], bounds[1], options=opts)
    s1 = list(gen_candidates_device.last_shrinks)
    c0, v0 = gen_candidates_device(ics, acqf, bounds[0], bounds[1],
                                   options={**opts, "early_checks": False})
    s0 = list(gen_candidates_device.last_shrinks)
    assert all(e % 4 == 0 for e, _ in s0)
    if s1:
        assert s1[0][0] <= (s0[0][0] if s0 else 4)
    torch.testing.assert_close(c1, c0, atol=1e-9, rtol=0)
    torch.testing.assert_close(v1, v0, atol=1e-12, rtol=1e-9)


def test_gen_candidates_device_restarts_equal_scipy_per_restart():
    from botorch_amd.optim import gen_candidates_device, gen_candidates_scipy
    acqf, bounds, ics = _qei_setup()
    cd, vd = gen_candidates_device(ics, acqf, bounds[0], bounds[1])
    st = gen_candidates_device.last_state
    assert set(st.status.cpu().tolist()) <= {1, 2}
    close = 0
    for i in range(ics.shape[0]):
        cs, vs = gen_candidates_scipy(ics[i:i + 1], acqf, bounds[0], bounds[1])
        assert vd[i].item() >= vs.item() - 1e-7 * max(1.0, abs(vs.item()))
        close += int(torch.allclose(cd[i:i + 1], cs, atol=1e-6, rtol=0))
    assert close >= ics.shape[0] - 1, close


def test_projected_algorithm_still_available():
    from botorch_amd.optim import gen_candidates_device
    acqf, bounds, ics = _qei_setup()
    c, v = gen_candidates_device(ics, acqf, bounds[0], bounds[1],
                                 options={"algorithm": "projected", "maxiter": 200})
    assert c.shape == ics.shape and (c >= 0).all() and (c <= 1).all()
    with torch.no_grad():
        assert (v >= acqf(ics) - 1e-12).all()


def test_restart_shards_reproduce_the_whole_batch():
    """Per-restart L-BFGS-B makes the restart sharding of
    distributed.optimize_acqf_sharded exact: the halves a 2-rank job optimises
    return the candidates of the whole batch (the reference's joint L-BFGS-B
    couples the restarts through one line search, so sharding it would change
    its iterates)."""
    from botorch_amd.optim import gen_candidates_device
    acqf, bounds, ics = _qei_setup()
    c_all, v_all = gen_candidates_device(ics, acqf, bounds[0], bounds[1])
    halves = [gen_candidates_device(ics[s], acqf, bounds[0], bounds[1])
              for s in (slice(0, 4), slice(4, 8))]
    c_sh = torch.cat([h[0] for h in halves])
    v_sh = torch.cat([h[1] for h in halves])
    torch.testing.assert_close(c_sh, c_all, atol=1e-8, rtol=0)
    torch.testing.assert_close(v_sh, v_all, atol=1e-12, rtol=1e-10)


def test_restart_compaction_matches_and_is_deterministic():
    """Stopped restarts leave the batch (their states set aside, the graph
    re-captured for the smaller shape): every restart ends where it ends
    without compaction, to rounding (the smaller batch's evaluations take
    another split plan, so f and g are summed in another order); a compacted
    run repeats bit for bit, and "auto" decides from the deterministic cost
    estimate (C3-sized qEI shrinks, a small one does not)."""
    from botorch_amd.optim import _eval_flops, gen_candidates_device
    acqf, bounds, ics = _qei_setup()
    c0, v0 = gen_candidates_device(ics, acqf, bounds[0], bounds[1], options={"compact": False})
    s0 = gen_candidates_device.last_state.status.clone()
    opts = {"compact": True, "compact_min": 1, "check_every": 2}
    c1, v1 = gen_candidates_device(ics, acqf, bounds[0], bounds[1], options=opts)
    sh = list(gen_candidates_device.last_shrinks)
    assert sh, "no compaction happened"
    assert torch.equal(gen_candidates_device.last_state.status, s0)
    torch.testing.assert_close(c1, c0, atol=1e-8, rtol=0)
    torch.testing.assert_close(v1, v0, atol=1e-12, rtol=1e-10)
    c2, v2 = gen_candidates_device(ics, acqf, bounds[0], bounds[1], options=opts)
    assert gen_candidates_device.last_shrinks == sh
    assert torch.equal(c2, c1) and torch.equal(v2, v1)
    n = acqf.model.train_inputs[0].shape[0]
    q = ics.shape[-2]
    assert _eval_flops(acqf, ics.shape[0], q) == 2.0 * ics.shape[0] * q * n * n
    gen_candidates_device(ics, acqf, bounds[0], bounds[1], options={"compact_flops": 1.0,
                                                                     "compact_min": 1})
    assert gen_candidates_device.last_shrinks  # "auto" with a tiny threshold shrinks
    gen_candidates_device(ics, acqf, bounds[0], bounds[1], options={"compact_flops": 1e30,
                                                                     "compact_min": 1})
    assert not gen_candidates_device.last_shrinks


def test_kernel_unconstrained_and_fixed_variables():
    """The kernel on the unconstrained branch (no bounds: the Cauchy search is
    skipped once memory exists) and on fixed variables (l == u)."""
    from tests.test_lbfgsb_cpu import _quad
    rng = np.random.default_rng(0)
    x0 = rng.uniform(-1, 1, 10)
    inf = np.full(10, np.inf)
    trials, x, f, status, nit = _drive([_rosen], x0[None], -inf, inf)
    sp, res = scipy_trials(_rosen, x0, None)
    assert len(trials[0]) == len(sp) and nit[0] == res.nit
    for a, b in zip(sp[:50], trials[0][:50]):
        np.testing.assert_allclose(b, a, atol=1e-9, rtol=0)
    np.testing.assert_allclose(x[0], res.x, atol=1e-8, rtol=0)
    rng = np.random.default_rng(11)
    n = 10
    M = rng.standard_normal((n, n))
    A = M @ M.T + np.eye(n)
    bb = rng.standard_normal(n) * 4
    lo = np.array([0.3, 0.3, 0, 0, -np.inf, -np.inf, 0, -1, -np.inf, 0.5])
    hi = np.array([0.3, 0.3, 1, 1, np.inf, 0.0, np.inf, 1, np.inf, 0.5])
    x0 = np.clip(rng.uniform(-0.5, 0.5, n), lo, hi)
    fg = _quad(A, bb)
    trials, x, f, status, nit = _drive([fg], x0[None], lo, hi)
    sp, res = scipy_trials(fg, x0, list(zip(lo, hi)))
    assert len(trials[0]) == len(sp) and nit[0] == res.nit
    np.testing.assert_allclose(x[0], res.x, atol=1e-10, rtol=0)
    assert x[0][0] == 0.3 and x[0][1] == 0.3 and x[0][9] == 0.5


@pytest.mark.parametrize("q", [200, 300])
def test_kernel_joint_width_trial_points_equal_scipy(q):
    """A restart wider than one wave's working set (n = 6 q = 1200 / 1800 > 1024:
    the 4-wave workgroup the joint problem runs on, block-wide reductions) on
    one Hartmann q-batch: scipy's trial points in scipy's order (the opening 25),
    its final value."""
    n = 6 * q
    x0 = np.random.default_rng(q).uniform(0, 1, n)
    lo, hi = np.zeros(n), np.ones(n)
    fg = _hartmann_batch(q)
    trials, x, f, status, nit = _drive([fg], x0[None], lo, hi, maxiter=60)
    sp, res = scipy_trials(fg, x0, list(zip(lo, hi)), maxiter=60)
    k = min(25, len(sp))
    assert len(trials[0]) >= k
    for i in range(k):
        np.testing.assert_allclose(trials[0][i], sp[i], atol=1e-9, rtol=0, err_msg=f"trial {i}")
    np.testing.assert_allclose(f[0], res.fun, rtol=1e-7, atol=1e-9)


@pytest.mark.parametrize("b", [8, 32])
def test_gen_candidates_device_joint_equals_scipy(b):
    """joint=True is the reference's problem (generation/gen.py:252-267: one
    L-BFGS-B over the b q d stacked variables and -sum_b acq): at C2 size
    (n = 1024, q = 8, S = 256) its candidates and values equal
    gen_candidates_scipy's on the same initial conditions -- b = 8 (384
    variables, one wave) and b = 32 (1536, the 4-wave workgroup)."""
    from botorch_amd.acquisition import qExpectedImprovement
    from botorch_amd.models import SingleTaskGP
    from botorch_amd.optim import (gen_batch_initial_conditions, gen_candidates_device,
                                   gen_candidates_scipy)
    from botorch_amd.sampling import SobolQMCNormalSampler
    from botorch_amd.test_functions import Hartmann
    from botorch_amd.utils_sampling import draw_sobol_samples
    box = torch.stack([torch.zeros(6), torch.ones(6)]).to(torch.float64)
    X = draw_sobol_samples(box, 1024, 1, seed=0).squeeze(1)
    Y = Hartmann(negate=True)(X).unsqueeze(-1)
    m = SingleTaskGP(X.to(DEV), Y.to(DEV))
    m.covar_module.lengthscale = torch.full((1, 6), 0.5016, dtype=torch.float64)
    m.likelihood.noise = torch.tensor([6.737947e-3], dtype=torch.float64)
    m.eval()
    acqf = qExpectedImprovement(m, float(Y.max()) - 0.3,
                                sampler=SobolQMCNormalSampler(torch.Size([256]), seed=0))
    bounds = box.to(DEV)
    ics = gen_batch_initial_conditions(acqf, bounds, q=8, num_restarts=b, raw_samples=4 * b,
                                       options={"seed": 3})
    opts = {"maxiter": 100}
    cs, vs = gen_candidates_scipy(ics, acqf, bounds[0], bounds[1], options=opts)
    cd, vd = gen_candidates_device(ics, acqf, bounds[0], bounds[1], options={**opts, "joint": True})
    st = gen_candidates_device.last_state
    assert st.B == 1 and st.n == b * 8 * 6
    assert gen_candidates_device.last_graph_error is None
    torch.testing.assert_close(cd, cs, atol=1e-6, rtol=0)
    torch.testing.assert_close(vd, vs, atol=1e-10, rtol=1e-7)
    assert float(vs.max()) > 0


# ---- the grid-wide kernel of a single restart (csrc/lbfgsb_grid.hip) --------
class _grid:
    """bo_lbfgsb_set_grid(mode) for the block; asserts the grid route ran
    (mode 1) or did not (mode -1)."""

    def __init__(self, mode):
        self.mode = mode

    def __enter__(self):
        from botorch_amd._lib import lib
        lib().bo_lbfgsb_set_grid(self.mode)
        self.before = lib().bo_lbfgsb_grid_launches()
        return self

    def __exit__(self, *exc):
        from botorch_amd._lib import lib
        self.launches = lib().bo_lbfgsb_grid_launches() - self.before
        lib().bo_lbfgsb_set_grid(0)
        if exc[0] is None and self.mode != 0:
            assert (self.launches > 0) == (self.mode == 1), (self.mode, self.launches)


@pytest.mark.parametrize("q", [50, 200, 300, 700])
def test_grid_kernel_trial_points_equal_scipy(q):
    """The grid route (one workgroup per 256 variables: n = 300 / 1200 / 1800 /
    4200 on 2 / 5 / 8 / 17 workgroups) on one Hartmann q-batch: scipy's trial
    points in scipy's order (the opening 25), its final value."""
    n = 6 * q
    x0 = np.random.default_rng(q).uniform(0, 1, n)
    lo, hi = np.zeros(n), np.ones(n)
    fg = _hartmann_batch(q)
    with _grid(1):
        trials, x, f, status, nit = _drive([fg], x0[None], lo, hi, maxiter=60)
    sp, res = scipy_trials(fg, x0, list(zip(lo, hi)), maxiter=60)
    k = min(25, len(sp))
    assert len(trials[0]) >= k
    for i in range(k):
        np.testing.assert_allclose(trials[0][i], sp[i], atol=1e-9, rtol=0, err_msg=f"trial {i}")
    np.testing.assert_allclose(f[0], res.fun, rtol=1e-7, atol=1e-9)


def test_grid_kernel_long_runs_equal_scipy():
    """The grid route on one workgroup: the box Rosenbrock run (active upper
    bounds, history wrap-around, 44 evaluations), the unconstrained branch and
    fixed variables -- whole runs equal scipy's."""
    from tests.test_lbfgsb_cpu import _quad
    rng = np.random.default_rng(0)
    n = 10
    x0 = rng.uniform(-1, 1, n)
    lo, hi = np.full(n, -1.5), np.full(n, 0.8)
    with _grid(1):
        trials, x, f, status, nit = _drive([_rosen], x0[None], lo, hi)
    sp, res = scipy_trials(_rosen, x0, list(zip(lo, hi)))
    assert len(trials[0]) == len(sp) and nit[0] == res.nit and status[0] == 2
    for a, b in zip(sp, trials[0]):
        np.testing.assert_allclose(b, a, atol=1e-9, rtol=0)
    np.testing.assert_allclose(x[0], res.x, atol=1e-10, rtol=0)
    inf = np.full(10, np.inf)
    x0 = rng.uniform(-1, 1, 10)
    with _grid(1):
        trials, x, f, status, nit = _drive([_rosen], x0[None], -inf, inf)
    sp, res = scipy_trials(_rosen, x0, None)
    assert len(trials[0]) == len(sp) and nit[0] == res.nit
    for a, b in zip(sp[:50], trials[0][:50]):
        np.testing.assert_allclose(b, a, atol=1e-9, rtol=0)
    rng = np.random.default_rng(11)
    M = rng.standard_normal((n, n))
    A = M @ M.T + np.eye(n)
    bb = rng.standard_normal(n) * 4
    lo = np.array([0.3, 0.3, 0, 0, -np.inf, -np.inf, 0, -1, -np.inf, 0.5])
    hi = np.array([0.3, 0.3, 1, 1, np.inf, 0.0, np.inf, 1, np.inf, 0.5])
    x0 = np.clip(rng.uniform(-0.5, 0.5, n), lo, hi)
    fg = _quad(A, bb)
    with _grid(1):
        trials, x, f, status, nit = _drive([fg], x0[None], lo, hi)
    sp, res = scipy_trials(fg, x0, list(zip(lo, hi)))
    assert len(trials[0]) == len(sp) and nit[0] == res.nit
    np.testing.assert_allclose(x[0], res.x, atol=1e-10, rtol=0)
    assert x[0][0] == 0.3 and x[0][1] == 0.3 and x[0][9] == 0.5


def test_grid_kernel_maxcor_and_wide_multi_round_cauchy():
    """maxcor 3 and 17 (ring wrap-around, the LDS limit) on a 2-workgroup
    problem whose first Cauchy search walks many breakpoints (a linear
    objective pushing every variable to a bound: more than one round of
    published breakpoints), trial points and values equal scipy's."""
    n = 400
    rng = np.random.default_rng(5)
    c = rng.standard_normal(n)
    D = np.abs(rng.standard_normal(n)) * 0.05

    def fg(x):
        return float(c @ x + 0.5 * np.sum(D * x * x) + 0.25 * np.sum(x ** 4)), c + D * x + x ** 3

    x0 = rng.uniform(-0.5, 0.5, n)
    lo, hi = np.full(n, -0.6), np.full(n, 0.6)
    for m in (3, 17):
        with _grid(1):
            trials, x, f, status, nit = _drive([fg], x0[None], lo, hi, m=m, maxiter=80)
        sp, res = scipy_trials(fg, x0, list(zip(lo, hi)), maxcor=m, maxiter=80)
        k = min(30, len(sp))
        assert len(trials[0]) >= k
        for i in range(k):
            np.testing.assert_allclose(trials[0][i], sp[i], atol=1e-9, rtol=0,
                                       err_msg=f"m={m} trial {i}")
        np.testing.assert_allclose(f[0], res.fun, rtol=1e-9, atol=1e-10)


@pytest.mark.parametrize("b,mode", [(32, 1), (64, 0)])
def test_gen_candidates_device_joint_grid_equals_scipy(b, mode):
    """joint=True on the grid route: b = 32 forced (1536 variables, 6
    workgroups), b = 64 by default (3072 >= 2048: 12 workgroups) -- the
    candidates and values of gen_candidates_scipy on the same initial
    conditions."""
    from botorch_amd.acquisition import qExpectedImprovement
    from botorch_amd.models import SingleTaskGP
    from botorch_amd.optim import (gen_batch_initial_conditions, gen_candidates_device,
                                   gen_candidates_scipy)
    from botorch_amd.sampling import SobolQMCNormalSampler
    from botorch_amd.test_functions import Hartmann
    from botorch_amd.utils_sampling import draw_sobol_samples
    box = torch.stack([torch.zeros(6), torch.ones(6)]).to(torch.float64)
    X = draw_sobol_samples(box, 1024, 1, seed=0).squeeze(1)
    Y = Hartmann(negate=True)(X).unsqueeze(-1)
    m = SingleTaskGP(X.to(DEV), Y.to(DEV))
    m.covar_module.lengthscale = torch.full((1, 6), 0.5016, dtype=torch.float64)
    m.likelihood.noise = torch.tensor([6.737947e-3], dtype=torch.float64)
    m.eval()
    acqf = qExpectedImprovement(m, float(Y.max()) - 0.3,
                                sampler=SobolQMCNormalSampler(torch.Size([256]), seed=0))
    bounds = box.to(DEV)
    ics = gen_batch_initial_conditions(acqf, bounds, q=8, num_restarts=b, raw_samples=4 * b,
                                       options={"seed": 3})
    opts = {"maxiter": 100}
    cs, vs = gen_candidates_scipy(ics, acqf, bounds[0], bounds[1], options=opts)
    with _grid(1 if mode == 1 else 0) as gr:
        cd, vd = gen_candidates_device(ics, acqf, bounds[0], bounds[1],
                                       options={**opts, "joint": True})
    assert gr.launches == gen_candidates_device.last_evals
    torch.testing.assert_close(cd, cs, atol=1e-6, rtol=0)
    torch.testing.assert_close(vd, vs, atol=1e-10, rtol=1e-7)
