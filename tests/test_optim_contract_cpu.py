"""The caller contract of optimize_acqf / gen_candidates_scipy / fit_gpytorch_mll
on the host (no GPU): fixed features, timeouts, the scipy exit handling, the
rejected nonlinear constraints, sequential greedy q, post-processing, and the
failure / retry / pick-best policy of _fit_fallback with scripted optimisers.

Reference: optim/optimize.py:140-564, generation/gen.py:46-298, 458-493,
generation/utils.py:102-196, optim/utils/timeout.py:19-108, botorch/fit.py:
116-283, optim/utils/model_utils.py:153-193.
"""
import math
import time
import warnings

import numpy as np
import pytest
import torch

from botorch_amd.acquisition import AcquisitionFunction, FixedFeatureAcquisitionFunction
from botorch_amd.exceptions import (ModelFittingError, NotPSDError, OptimizationWarning,
                                    UnsupportedError)
from botorch_amd.optim import (_process_scipy_result, fix_features, gen_candidates_scipy,
                               minimize_with_timeout, optimize_acqf)

TARGET = torch.tensor([0.2, 0.7, 0.45], dtype=torch.float64)


class _Quad(AcquisitionFunction):
    """-||x - target||^2 summed over the q points (+ pending points counted as
    fixed penalties): a smooth, separable test acquisition on the host."""

    def __init__(self, target=TARGET, sleep=0.0):
        super().__init__(model=None)
        self.target = target
        self.sleep = sleep
        self.calls = 0

    def forward(self, X):
        self.calls += 1
        if self.sleep:
            time.sleep(self.sleep)
        X = X if X.dim() == 3 else X.unsqueeze(0)
        val = -((X - self.target.to(X)) ** 2).sum(dim=(-1, -2))
        if self.X_pending is not None:
            # the pending points repel: the greedy picks must move apart
            P = self.X_pending.to(X)
            d2 = ((X.unsqueeze(-2) - P) ** 2).sum(-1)
            val = val - 0.05 * torch.exp(-d2 / 0.01).sum(dim=(-1, -2))
        return val


BOUNDS = torch.stack([torch.zeros(3, dtype=torch.float64), torch.ones(3, dtype=torch.float64)])


def test_fix_features_sets_values_and_detaches_none():
    X = torch.rand(4, 2, 3, dtype=torch.float64, requires_grad=True)
    Y = fix_features(X, {0: 0.5, 2: None})
    assert torch.all(Y[..., 0] == 0.5)
    assert torch.equal(Y[..., 2], X[..., 2])
    Y.sum().backward()
    assert torch.all(X.grad[..., 0] == 0) and torch.all(X.grad[..., 2] == 0)
    assert torch.all(X.grad[..., 1] == 1)


def test_fixed_feature_acqf_column_order():
    acq = _Quad()
    ff = FixedFeatureAcquisitionFunction(acq, d=3, columns=[1], values=[0.9])
    X = torch.rand(5, 2, 2, dtype=torch.float64)
    full = ff._construct_X_full(X)
    assert full.shape == (5, 2, 3)
    assert torch.equal(full[..., 0], X[..., 0]) and torch.equal(full[..., 2], X[..., 1])
    assert torch.all(full[..., 1] == 0.9)
    torch.testing.assert_close(ff(X), acq(full))
    with pytest.raises(ValueError):
        ff._construct_X_full(torch.rand(2, 3, dtype=torch.float64))


def test_gen_candidates_scipy_fixed_features():
    """gen.py:124-175: the fixed columns leave the search space; the others
    reach the optimum; a None value keeps the clamped initial column."""
    acq = _Quad()
    x0 = torch.full((3, 2, 3), 0.5, dtype=torch.float64)
    x0[..., 2] = torch.tensor([0.1, 0.2, 0.3], dtype=torch.float64).view(3, 1)
    c, v = gen_candidates_scipy(x0, acq, BOUNDS[0], BOUNDS[1],
                                fixed_features={1: 0.3, 2: None})
    assert c.shape == x0.shape
    assert torch.all(c[..., 1] == 0.3)
    assert torch.equal(c[..., 2], x0[..., 2])
    torch.testing.assert_close(c[..., 0], torch.full((3, 2), 0.2, dtype=torch.float64),
                               atol=1e-5, rtol=0)
    torch.testing.assert_close(v, acq(c))


def test_minimize_with_timeout_returns_iterate():
    from scipy.optimize import rosen, rosen_der
    calls = []

    def f(x):
        calls.append(1)
        time.sleep(0.002)
        return rosen(x), rosen_der(x)
    res = minimize_with_timeout(f, np.full(6, -1.0), method="L-BFGS-B", jac=True,
                                timeout_sec=0.05)
    assert not res.success and res.status == 1
    assert res.message.startswith("Optimization timed out after")
    assert np.isfinite(res.fun) and res.x.shape == (6,)
    full = minimize_with_timeout(f, np.full(6, -1.0), method="L-BFGS-B", jac=True)
    assert full.success and full.nit > res.nit


def test_gen_candidates_scipy_timeout_is_logged_not_warned():
    acq = _Quad(sleep=0.01)
    x0 = torch.full((2, 1, 3), 0.9, dtype=torch.float64)
    t0 = time.monotonic()
    with warnings.catch_warnings(record=True) as ws:
        warnings.simplefilter("always")
        c, _ = gen_candidates_scipy(x0, acq, BOUNDS[0], BOUNDS[1],
                                    options={"ftol": 0.0, "gtol": 0.0}, timeout_sec=0.03)
    assert time.monotonic() - t0 < 2.0
    assert not [w for w in ws if issubclass(w.category, OptimizationWarning)]
    assert torch.all((c >= 0) & (c <= 1))


def test_process_scipy_result_policy():
    from scipy.optimize import OptimizeResult
    quiet = ["STOP: TOTAL NO. OF ITERATIONS REACHED LIMIT",
             "STOP: TOTAL NO. of ITERATIONS REACHED LIMIT",
             "STOP: TOTAL NO. OF F,G EVALUATIONS EXCEEDS LIMIT",
             "Optimization timed out after 1.0 seconds."]
    for msg in quiet:
        with warnings.catch_warnings(record=True) as ws:
            warnings.simplefilter("always")
            _process_scipy_result(OptimizeResult(success=False, status=1, message=msg), {})
        assert not ws, msg
    for res in (OptimizeResult(success=False, status=2, message="ABNORMAL: LINE SEARCH FAILED"),
                OptimizeResult(x=0)):
        with pytest.warns(OptimizationWarning):
            _process_scipy_result(res, {})
    with warnings.catch_warnings(record=True) as ws:
        warnings.simplefilter("always")
        _process_scipy_result(OptimizeResult(success=True, status=0, message="CONVERGENCE"), {})
    assert not ws


def test_nonlinear_constraints_are_rejected_not_dropped():
    acq = _Quad()
    kw = {"nonlinear_inequality_constraints": [(lambda x: x.sum() - 1, True)]}
    with pytest.raises(UnsupportedError):
        optimize_acqf(acq, BOUNDS, q=1, num_restarts=2, raw_samples=8, **kw)
    with pytest.raises(UnsupportedError):
        gen_candidates_scipy(torch.full((1, 1, 3), 0.5, dtype=torch.float64), acq,
                             BOUNDS[0], BOUNDS[1], **kw)


@pytest.mark.parametrize("kw", [
    {"inequality_constraints": [(torch.tensor([0, 1]), torch.tensor([1.0, 1.0]), 0.5)]},
    {"equality_constraints": [(torch.tensor([0]), torch.tensor([1.0]), 0.5)]},
])
def test_device_optimizer_rejects_linear_constraints(kw):
    """The device L-BFGS-B handles boxes only: it refuses linear constraints
    (before touching the GPU) instead of dropping them."""
    from botorch_amd.optim import gen_candidates_device
    with pytest.raises(UnsupportedError, match="gen_candidates_scipy"):
        gen_candidates_device(torch.full((1, 1, 3), 0.5, dtype=torch.float64), _Quad(),
                              BOUNDS[0], BOUNDS[1], **kw)


def test_optimize_acqf_input_validation():
    acq = _Quad()
    with pytest.raises(ValueError, match="bounds should be"):
        optimize_acqf(acq, BOUNDS[0], q=1, num_restarts=2, raw_samples=8)
    with pytest.raises(ValueError, match="raw_samples"):
        optimize_acqf(acq, BOUNDS, q=1, num_restarts=2)
    with pytest.raises(ValueError, match="must be 2-dimensional or 3-dimensional"):
        optimize_acqf(acq, BOUNDS, q=1, num_restarts=2,
                      batch_initial_conditions=torch.rand(2, 2, 2, 3, dtype=torch.float64))
    with pytest.raises(ValueError, match="shape\\[-1\\] must be 3"):
        optimize_acqf(acq, BOUNDS, q=1, num_restarts=2,
                      batch_initial_conditions=torch.rand(2, 1, 2, dtype=torch.float64))


def test_optimize_acqf_fixed_features_and_post_processing():
    torch.manual_seed(0)
    acq = _Quad()
    c, v = optimize_acqf(acq, BOUNDS, q=2, num_restarts=3, raw_samples=16,
                         fixed_features={2: 0.8}, options={"seed": 1})
    assert c.shape == (2, 3) and torch.all(c[:, 2] == 0.8)
    torch.testing.assert_close(c[:, :2], TARGET[:2].expand(2, 2), atol=1e-5, rtol=0)

    def snap(X):
        return (X * 10).round() / 10
    c, v = optimize_acqf(acq, BOUNDS, q=1, num_restarts=3, raw_samples=16, options={"seed": 1},
                         post_processing_func=snap, return_best_only=False)
    assert c.shape == (3, 1, 3)
    torch.testing.assert_close(c, snap(c))
    torch.testing.assert_close(v, acq(c))


def test_optimize_acqf_all_features_fixed():
    acq = _Quad()
    c, v = optimize_acqf(acq, BOUNDS, q=2, num_restarts=3, raw_samples=16,
                         fixed_features={0: 0.1, 1: 0.2, 2: 0.3})
    assert c.shape == (2, 3)
    torch.testing.assert_close(c, torch.tensor([[0.1, 0.2, 0.3]] * 2, dtype=torch.float64))
    torch.testing.assert_close(v, acq(c))


def test_optimize_acqf_sequential_is_greedy_over_pending_points():
    """optimize.py:202-243: q picks of q = 1, each added to X_pending; the
    caller's pending points are restored afterwards."""
    acq = _Quad()
    base = torch.tensor([[0.9, 0.9, 0.9]], dtype=torch.float64)
    acq.set_X_pending(base)
    opts = {"seed": 3}
    torch.manual_seed(5)
    c, v = optimize_acqf(acq, BOUNDS, q=3, num_restarts=4, raw_samples=32, options=opts,
                         sequential=True)
    assert c.shape == (3, 3) and v.shape == (3,)
    assert torch.equal(acq.X_pending, base)
    # the same greedy loop by hand
    torch.manual_seed(5)
    picks = []
    for _ in range(3):
        cc, _ = optimize_acqf(acq, BOUNDS, q=1, num_restarts=4, raw_samples=32, options=opts)
        picks.append(cc)
        acq.set_X_pending(torch.cat([base] + picks, dim=-2))
    acq.set_X_pending(base)
    torch.testing.assert_close(c, torch.cat(picks, dim=-2))
    with pytest.raises(UnsupportedError):
        optimize_acqf(acq, BOUNDS, q=2, num_restarts=2, sequential=True,
                      batch_initial_conditions=torch.rand(2, 2, 3, dtype=torch.float64))


def test_optimize_acqf_retry_warning_texts():
    """optimize.py:330-373: a chunk's OptimizationWarning triggers one retry
    with new initial conditions (or none when they were given)."""
    acq = _Quad()
    calls = []

    def gen(ics, acqf, **kw):
        calls.append(kw)
        warnings.warn("Optimization failed within `scipy.optimize.minimize` with status 2",
                      OptimizationWarning)
        return ics, acqf(ics)
    with pytest.warns(RuntimeWarning, match="Trying again"):
        optimize_acqf(acq, BOUNDS, q=1, num_restarts=4, raw_samples=16, gen_candidates=gen,
                      options={"batch_limit": 2}, timeout_sec=4.0)
    assert len(calls) == 4  # 2 chunks, twice
    assert all(k["timeout_sec"] == 2.0 for k in calls)
    assert all(k["fixed_features"] is None for k in calls)
    calls.clear()
    with pytest.warns(RuntimeWarning, match="will not be retried"):
        optimize_acqf(acq, BOUNDS, q=1, num_restarts=4, gen_candidates=gen,
                      batch_initial_conditions=torch.rand(4, 1, 3, dtype=torch.float64))
    assert len(calls) == 1


# -- fit_gpytorch_mll's failure contract (fit.py:116-259) ---------------------
def _model():
    from botorch_amd.models import SingleTaskGP
    X = torch.rand(12, 3, dtype=torch.float64, generator=torch.Generator().manual_seed(0))
    Y = X.sum(-1, keepdim=True).sin()
    return SingleTaskGP(X, Y)


def _mll(model):
    from botorch_amd.fit import ExactMarginalLogLikelihood
    return ExactMarginalLogLikelihood(model.likelihood, model)


class _Scripted:
    """An optimizer (mll, closure, **kw) -> OptimizationResult that plays a
    script: ("warn", msg) / ("raise", exc) / ("ok", fval); it records the
    hyperparameters each attempt started from and writes a marker."""

    def __init__(self, script):
        self.script = list(script)
        self.starts = []

    def __call__(self, mll, closure=None, **kw):
        from botorch_amd.fit import OptimizationResult, OptimizationStatus, _layout
        lay = _layout(mll.model)
        self.starts.append(lay.get())
        kind, arg = self.script.pop(0)
        x = lay.get()
        x[1] = float(len(self.starts))   # the constant: which attempt wrote it
        lay.set(x)
        if kind == "raise":
            raise arg
        if kind == "warn":
            warnings.warn(arg, OptimizationWarning)
            return OptimizationResult(step=1, fval=0.0, status=OptimizationStatus.FAILURE)
        return OptimizationResult(step=1, fval=arg, status=OptimizationStatus.SUCCESS)


def test_fit_all_attempts_fail_raises_and_rolls_back():
    from botorch_amd.fit import _layout, fit_gpytorch_mll
    m = _model()
    x0 = _layout(m).get()
    opt = _Scripted([("warn", "ABNORMAL: LINE SEARCH FAILED")] * 3)
    with warnings.catch_warnings(record=True):
        warnings.simplefilter("always")
        with pytest.raises(ModelFittingError, match="All attempts to fit the model have failed"):
            fit_gpytorch_mll(_mll(m), optimizer=opt, max_attempts=3)
    assert len(opt.starts) == 3
    np.testing.assert_array_equal(_layout(m).get(), x0)
    assert m.training


def test_fit_limit_and_timeout_warnings_are_resolved():
    from botorch_amd.fit import fit_gpytorch_mll
    for msg, rethrown in (("`scipy_minimize` terminated with status 4, displaying original "
                           "message from `scipy.optimize.minimize`: STOP: TOTAL NO. OF "
                           "ITERATIONS REACHED LIMIT", False),
                          ("Optimization timed out after 0.1 seconds.", True)):
        m = _model()
        opt = _Scripted([("warn", msg)])
        with warnings.catch_warnings(record=True) as ws:
            warnings.simplefilter("always")
            mll = fit_gpytorch_mll(_mll(m), optimizer=opt)
        assert not mll.training and len(opt.starts) == 1
        assert any(msg in str(w.message) for w in ws) == rethrown


def test_fit_retry_resamples_priors_from_global_rng():
    """Attempt 2 starts from the checkpoint with its priors resampled from the
    global generator: exp(N(loc, scale)) for the noise (1,) and the
    lengthscales (1, d), in that order (named_priors)."""
    from botorch_amd.fit import _layout, fit_gpytorch_mll
    m = _model()
    x0 = _layout(m).get()
    opt = _Scripted([("raise", NotPSDError("not p.d.")), ("ok", 1.0)])
    torch.manual_seed(1234)
    fit_gpytorch_mll(_mll(m), optimizer=opt)
    assert len(opt.starts) == 2
    np.testing.assert_array_equal(opt.starts[0], x0)
    torch.manual_seed(1234)
    npri, lpri = m.likelihood.noise_prior, m.covar_module.lengthscale_prior
    noise = torch.normal(torch.full((1,), npri.loc, dtype=torch.float64),
                         torch.full((1,), npri.scale, dtype=torch.float64)).exp()
    ls = torch.normal(torch.full((1, 3), lpri.loc, dtype=torch.float64),
                      torch.full((1, 3), lpri.scale, dtype=torch.float64)).exp()
    s = opt.starts[1]
    assert s[0] == noise.item() and s[1] == x0[1]
    np.testing.assert_array_equal(s[2:], ls.reshape(-1).numpy())


def test_fit_uncaught_exception_propagates():
    from botorch_amd.fit import fit_gpytorch_mll
    m = _model()
    with pytest.raises(KeyError):
        fit_gpytorch_mll(_mll(m), optimizer=_Scripted([("raise", KeyError("x"))]))
    m = _model()
    opt = _Scripted([("raise", KeyError("x")), ("ok", 0.0)])
    fit_gpytorch_mll(_mll(m), optimizer=opt, caught_exception_types=(KeyError,))
    assert len(opt.starts) == 2


def test_fit_pick_best_of_all_attempts():
    from botorch_amd.fit import _layout, fit_gpytorch_mll
    m = _model()
    opt = _Scripted([("ok", 3.0), ("warn", "ABNORMAL"), ("ok", -2.0), ("ok", 1.0)])
    with warnings.catch_warnings(record=True):
        warnings.simplefilter("always")
        mll = fit_gpytorch_mll(_mll(m), optimizer=opt, max_attempts=4,
                               pick_best_of_all_attempts=True)
    assert len(opt.starts) == 4 and not mll.training
    assert _layout(m).get()[1] == 3.0  # the third attempt's parameters (fval -2 = best MLL)


def test_fit_custom_closure_rejected():
    from botorch_amd.fit import fit_gpytorch_mll
    with pytest.raises(UnsupportedError):
        fit_gpytorch_mll(_mll(_model()), closure=lambda: None)
