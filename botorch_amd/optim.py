"""Multi-start acquisition optimisation: the callers of the hot path.

Restates the call protocol of optimize_acqf (botorch/optim/optimize.py:246-543),
gen_batch_initial_conditions (optim/initializers.py:243-438),
initialize_q_batch[_nonneg] (:968-1037) and gen_candidates_scipy
(generation/gen.py:46-298): scipy L-BFGS-B on the host over the flattened
b x q x d restarts, one forward + autograd.grad of -acqf(X).sum() per function
evaluation (the only host<->device boundary of the loop).

Multi-GPU (``botorch_amd.distributed``): restarts are sharded over ranks and
the final argmax/gather is one all-reduce.
"""
from __future__ import annotations

import ctypes
import math
import time
import warnings
from typing import Any, Callable, Dict, Optional, Tuple

import numpy as np
import torch
from scipy.optimize import minimize

from .exceptions import OptimizationWarning
from .utils_sampling import draw_sobol_samples, manual_seed

INIT_OPTION_KEYS = {"alpha", "batch_limit", "eta", "init_batch_limit", "nonnegative", "n_burnin",
                    "sample_around_best", "sample_around_best_sigma",
                    "sample_around_best_prob_perturb", "seed", "thinning"}


class BadInitialCandidatesWarning(RuntimeWarning):
    pass


def columnwise_clamp(X, lower=None, upper=None, raise_on_violation=False):
    """utils/transforms (optim/utils): clamp each column to [lower, upper]."""
    Xout = X
    if lower is not None:
        Xout = torch.maximum(Xout, torch.as_tensor(lower).to(X))
    if upper is not None:
        Xout = torch.minimum(Xout, torch.as_tensor(upper).to(X))
    if raise_on_violation and not torch.allclose(Xout, X):
        raise RuntimeError("Original value(s) are out of bounds.")
    return Xout


def initialize_q_batch_nonneg(X, Y, n, eta=1.0, alpha=1e-4):
    """optim/initializers.py:1041-1112 (device-agnostic: runs where X and Y live)."""
    n_samples = X.shape[0]
    if n > n_samples:
        raise RuntimeError("n cannot be larger than the number of provided samples")
    elif n == n_samples:
        return X
    max_val, max_idx = torch.max(Y, dim=0)
    if torch.any(max_val <= 0):
        warnings.warn("All acquisition values for raw sampled points are nonpositive, so "
                      "initial conditions are being selected randomly.", BadInitialCandidatesWarning)
        return X[torch.randperm(n=n_samples, device=X.device)][:n]
    pos = Y > 0
    num_pos = pos.sum().item()
    if num_pos < n:
        remaining = (~pos).nonzero(as_tuple=False).view(-1)
        rand = torch.randperm(remaining.shape[0], device=Y.device)
        pos[remaining[rand[: n - num_pos]]] = 1
        return X[pos]
    alpha_pos = Y >= alpha * max_val
    while alpha_pos.sum() < n:
        alpha = 0.1 * alpha
        alpha_pos = Y >= alpha * max_val
    idx_pos = torch.arange(len(Y), device=Y.device)[alpha_pos]
    weights = torch.exp(eta * (Y[alpha_pos] / max_val - 1))
    idcs = idx_pos[torch.multinomial(weights, n)]
    if max_idx not in idcs:
        idcs[-1] = max_idx
    return X[idcs]


def _batched_multinomial(weights, num_samples):
    """utils/sampling.py batched_multinomial: one multinomial per leading row."""
    flat = weights.reshape(-1, weights.shape[-1])
    out = torch.multinomial(flat, num_samples)
    return out.view(*weights.shape[:-1], num_samples)


def initialize_q_batch(X, Y, n, eta=1.0):
    """optim/initializers.py:968-1038: Boltzmann sampling on the standardized
    values, per batch_shape entry (X: b x batch_shape x q x d, Y: b x batch_shape)."""
    n_samples = X.shape[0]
    batch_shape = X.shape[1:-2] or torch.Size()
    if n > n_samples:
        raise RuntimeError(f"n ({n}) cannot be larger than the number of provided samples ({n_samples})")
    elif n == n_samples:
        return X
    Ystd = Y.std(dim=0)
    if torch.any(Ystd == 0):
        warnings.warn("All acquisition values for raw samples points are the same for "
                      "at least one batch. Choosing initial conditions at random.",
                      BadInitialCandidatesWarning)
        return X[torch.randperm(n=n_samples, device=X.device)][:n]
    max_val, max_idx = torch.max(Y, dim=0)
    Z = (Y - Y.mean(dim=0)) / Ystd
    etaZ = eta * Z
    weights = torch.exp(etaZ)
    while torch.isinf(weights).any():
        etaZ *= 0.5
        weights = torch.exp(etaZ)
    if batch_shape == torch.Size():
        idcs = torch.multinomial(weights, n)
    else:
        idcs = _batched_multinomial(weights.permute(*range(1, len(batch_shape) + 1), 0),
                                    n).permute(-1, *range(len(batch_shape)))
    if max_idx not in idcs:
        idcs[-1] = max_idx
    if batch_shape == torch.Size():
        return X[idcs]
    return X.gather(dim=0, index=idcs.view(*idcs.shape, 1, 1).expand(n, *X.shape[1:]))


_NONNEGATIVE = ("ExpectedImprovement", "ConstrainedExpectedImprovement", "ProbabilityOfImprovement",
                "NoisyExpectedImprovement", "qExpectedImprovement", "qNoisyExpectedImprovement",
                "qProbabilityOfImprovement", "ExpectedHypervolumeImprovement",
                "qExpectedHypervolumeImprovement", "qNoisyExpectedHypervolumeImprovement")


def is_nonnegative(acq_function) -> bool:
    """optim/initializers.py:1272-1300 (by class: the LogEI family is not
    non-negative even where it derives from the qEI classes here)."""
    return type(acq_function).__name__ in _NONNEGATIVE


_is_nonnegative = is_nonnegative


def _check_deferred(X) -> None:
    """Surface a deferred jitter-ladder failure of the fused forward-only path
    at the driver's own synchronisation point (kernels.raise_not_psd_deferred)."""
    if X.is_cuda:
        from . import kernels
        kernels.check_ladder_status(X.device)


def draw_raw_samples(bounds, n, q, seed=None):
    """Raw q-batch designs for the initialiser: on the device (bo_sobol_box,
    bit-identical to draw_sobol_samples) when ``bounds`` lives there, on the
    host (the reference's own path) otherwise."""
    if bounds.is_cuda:
        from . import kernels
        return kernels.sobol_box(bounds.to(torch.float64), n, q, seed).to(bounds.dtype)
    return draw_sobol_samples(bounds=bounds.cpu(), n=n, q=q, seed=seed)


def evaluate_raw_samples(acq_function, X_rnd, batch_limit=None):
    """Forward-only acquisition values of the raw designs in chunks of
    ``batch_limit`` (initializers.py:411-423), kept where they are computed: on
    the GPU path the values stay on the device (no per-chunk ``.cpu()``)."""
    if batch_limit is None:
        batch_limit = X_rnd.shape[0]
    if X_rnd.shape[0] == 0:
        return X_rnd.new_empty(0)
    with torch.no_grad():
        ys = [acq_function(X_rnd[s:s + batch_limit]) for s in range(0, X_rnd.shape[0], batch_limit)]
    return torch.cat([y.reshape(-1) for y in ys])


def init_options(acq_function, bounds, options):
    """The option handling of gen_batch_initial_conditions (initializers.py:
    305-345): (seed, init_batch_limit, init_func, init_kwargs)."""
    if bounds.isinf().any():
        raise NotImplementedError("Currently only finite values in `bounds` are supported for "
                                  "generating initial conditions for optimization.")
    options = options or {}
    if options.get("sample_around_best", False):
        raise NotImplementedError("sample_around_best is out of scope")
    seed = options.get("seed")
    batch_limit = options.get("init_batch_limit", options.get("batch_limit"))
    init_kwargs = {}
    if "eta" in options:
        init_kwargs["eta"] = options.get("eta")
    if options.get("nonnegative") or is_nonnegative(acq_function):
        init_func = initialize_q_batch_nonneg
        if "alpha" in options:
            init_kwargs["alpha"] = options.get("alpha")
    else:
        init_func = initialize_q_batch
    return seed, batch_limit, init_func, init_kwargs


def select_initial_indices(init_func, Y_rnd: torch.Tensor, num_restarts: int, init_kwargs) -> Tuple[torch.Tensor, bool]:
    """The Boltzmann selection of initializers.py:424-426 on the host values
    (one 8 B-per-design copy, where the reference copies each chunk with
    ``.cpu()``), drawing from the global CPU generator exactly as the reference
    does.  ``init_func`` gets an index column in place of X: it reads only
    X's shape and indexes it, so the generator calls and the picks are the
    reference's.  Returns (indices into the raw designs, warned)."""
    Yh = Y_rnd.detach().cpu()
    _check_deferred(Y_rnd)
    n = Yh.shape[0]
    with warnings.catch_warnings(record=True) as ws:
        warnings.simplefilter("always", category=BadInitialCandidatesWarning)
        idx = init_func(X=torch.arange(n).view(n, 1, 1), Y=Yh, n=num_restarts, **init_kwargs)
    # recorded, not re-emitted: the reference only uses them to decide the retry
    return idx.reshape(-1), any(issubclass(w.category, BadInitialCandidatesWarning) for w in ws)


def gen_batch_initial_conditions(acq_function, bounds, q, num_restarts, raw_samples,
                                 fixed_features=None, options=None, inequality_constraints=None,
                                 equality_constraints=None, generator=None, fixed_X_fantasies=None,
                                 **kwargs):
    """optim/initializers.py:243-438: Sobol raw samples, forward-only evaluation
    in chunks of init_batch_limit, Boltzmann selection; retried with up to 5x
    the raw samples (seed + 1 each time) while the selection warns.

    MI355X path (bounds on the GPU): the raw designs are generated on the
    device (bo_sobol_box, bit-identical to draw_sobol_samples) and evaluated
    there chunk by chunk; only the values cross to the host, once, for the
    selection, which draws from the global CPU generator as the reference does
    (so the picks are the reference's)."""
    if inequality_constraints or equality_constraints or generator is not None \
            or fixed_X_fantasies is not None:
        raise NotImplementedError("constrained / custom-generator initialisation is out of scope")
    seed, batch_limit, init_func, init_kwargs = init_options(acq_function, bounds, options)
    q = 1 if q is None else q
    factor, max_factor = 1, 5
    while factor < max_factor:
        n = raw_samples * factor
        X_rnd = draw_raw_samples(bounds, n, q, seed)
        if fixed_features:
            for k, v in fixed_features.items():
                X_rnd[..., k] = v
        Y_rnd = evaluate_raw_samples(acq_function, X_rnd.to(bounds.device), batch_limit)
        idx, warned = select_initial_indices(init_func, Y_rnd, num_restarts, init_kwargs)
        ics = X_rnd[idx.to(X_rnd.device)].to(device=bounds.device)
        if not warned:
            return ics
        if factor < max_factor:
            factor += 1
            if seed is not None:
                seed += 1
    warnings.warn("Unable to find non-zero acquisition function values - initial conditions "
                  "are being selected randomly.", BadInitialCandidatesWarning)
    return ics


def gen_candidates_scipy(initial_conditions, acquisition_function, lower_bounds=None,
                         upper_bounds=None, options=None, fixed_features=None,
                         timeout_sec=None, **kwargs):
    """generation/gen.py:46-298 (box constraints, L-BFGS-B, with_grad)."""
    options = dict(options or {})
    options = {**options, "maxiter": options.get("maxiter", 2000)}
    clamped = columnwise_clamp(initial_conditions, lower_bounds, upper_bounds)
    shapeX = clamped.shape
    x0 = clamped.detach().reshape(-1).cpu().numpy()
    d = shapeX[-1]
    lb = (torch.as_tensor(lower_bounds).expand(shapeX).reshape(-1).cpu().numpy()
          if lower_bounds is not None else np.full(x0.shape, -np.inf))
    ub = (torch.as_tensor(upper_bounds).expand(shapeX).reshape(-1).cpu().numpy()
          if upper_bounds is not None else np.full(x0.shape, np.inf))
    scipy_bounds = list(zip(lb, ub))
    with_grad = options.pop("with_grad", True)
    method = options.pop("method", "L-BFGS-B")
    callback = options.pop("callback", None)

    def f_np_wrapper(x: np.ndarray):
        if np.isnan(x).any():
            raise RuntimeError(f"{np.isnan(x).sum()} elements of the {x.size} element array `x` are NaN.")
        X = torch.from_numpy(x).to(initial_conditions).view(shapeX).contiguous().requires_grad_(True)
        loss = -acquisition_function(X).sum()
        grad = torch.autograd.grad(loss, X)[0].contiguous().view(-1).cpu().numpy()
        _check_deferred(X)
        if np.isnan(grad).any():
            raise RuntimeError(f"{np.isnan(grad).sum()} elements of the {x.size} element gradient "
                               "array `gradf` are NaN. This often indicates numerical issues.")
        return loss.item(), grad

    def f_only(x):
        X = torch.from_numpy(x).to(initial_conditions).view(shapeX).contiguous()
        with torch.no_grad():
            val = -acquisition_function(X).sum().item()
        _check_deferred(X)
        return val

    t0 = time.monotonic()
    res = minimize(f_np_wrapper if with_grad else f_only, x0, method=method, jac=with_grad,
                   bounds=scipy_bounds, callback=callback, options=options)
    if not res.success and "ITERATIONS REACHED LIMIT" not in str(res.message):
        warnings.warn(f"Optimization failed within `scipy.optimize.minimize` with status "
                      f"{res.status} and message {res.message}.", OptimizationWarning)
    candidates = torch.from_numpy(res.x).to(initial_conditions).reshape(shapeX)
    clamped = columnwise_clamp(candidates, lower_bounds, upper_bounds, raise_on_violation=True)
    with torch.no_grad():
        acq = acquisition_function(clamped)
    return clamped, acq


class _LBFGSState:
    """Device buffers of the multi-start projected L-BFGS (bo_lbfgs_step)."""

    def __init__(self, X0: torch.Tensor, m: int):
        B, n = X0.shape[0], X0[0].numel()
        f64 = dict(dtype=torch.float64, device=X0.device)
        i32 = dict(dtype=torch.int32, device=X0.device)
        self.B, self.n, self.m = B, n, m
        self.x = torch.empty(B, n, **f64)
        self.g = torch.empty(B, n, **f64)
        self.xt = X0.reshape(B, n).to(torch.float64).clone()
        self.d = torch.zeros(B, n, **f64)
        self.f = torch.empty(B, **f64)
        self.alpha = torch.ones(B, **f64)
        self.S = torch.empty(B, m, n, **f64)
        self.Y = torch.empty(B, m, n, **f64)
        self.rho = torch.zeros(B, m, **f64)
        self.hcount = torch.zeros(B, **i32)
        self.hhead = torch.zeros(B, **i32)
        self.status = torch.full((B,), -1, **i32)
        self.nacc = torch.zeros(B, **i32)


class _LBFGSBState:
    """Device buffers of the multi-start L-BFGS-B (bo_lbfgsb_step): zeroed
    state = "start at xt"."""

    def __init__(self, X0: torch.Tensor, m: int):
        from ._lib import lib
        lay = (ctypes.c_int * 6)()
        lib().bo_lbfgsb_layout(lay)
        nv, niv, nmat, nd, ni, mmax = list(lay)
        if not 1 <= m <= mmax:
            raise ValueError(f"maxcor={m}: the device L-BFGS-B keeps at most {mmax} pairs")
        B, n = X0.shape[0], X0[0].numel()
        f64 = dict(dtype=torch.float64, device=X0.device)
        i32 = dict(dtype=torch.int32, device=X0.device)
        self.B, self.n, self.m = B, n, m
        self.xt = X0.reshape(B, n).to(torch.float64).clone()
        self.v = torch.zeros(B, nv, n, **f64)
        self.iv = torch.zeros(B, niv, n, **i32)
        self.ws = torch.zeros(B, m, n, **f64)
        self.wy = torch.zeros(B, m, n, **f64)
        self.mat = torch.zeros(B, nmat, **f64)
        self.ds = torch.zeros(B, nd, **f64)
        self.is_ = torch.zeros(B, ni, **i32)

    _FIELDS = ("xt", "v", "iv", "ws", "wy", "mat", "ds", "is_")

    def take(self, idx: torch.Tensor) -> "_LBFGSBState":
        """The restarts idx as a compact state (copies; each restart's state is
        self-contained, so the compact batch continues exactly)."""
        sub = object.__new__(_LBFGSBState)
        sub.B, sub.n, sub.m = int(idx.numel()), self.n, self.m
        for f in self._FIELDS:
            setattr(sub, f, getattr(self, f).index_select(0, idx).contiguous())
        return sub

    def put(self, idx: torch.Tensor, sub: "_LBFGSBState") -> None:
        for f in self._FIELDS:
            getattr(self, f).index_copy_(0, idx, getattr(sub, f))

    @property
    def x(self):
        return self.v[:, 0]

    @property
    def status(self):
        return self.is_[:, 1]

    @property
    def nit(self):
        return self.is_[:, 10]

    @property
    def f(self):
        return self.ds[:, 0]


LBFGSB_STATUS = {0: "running", 1: "CONVERGENCE: NORM OF PROJECTED GRADIENT <= PGTOL",
                 2: "CONVERGENCE: RELATIVE REDUCTION OF F <= FACTR*EPSMCH",
                 3: "ABNORMAL: LINE SEARCH FAILED",
                 4: "STOP: TOTAL NO. OF ITERATIONS REACHED LIMIT",
                 5: "STOP: TOTAL NO. OF F,G EVALUATIONS EXCEEDS LIMIT",
                 6: "ERROR: NON-FINITE VALUE OR LINE-SEARCH INPUT"}


def gen_candidates_device(initial_conditions, acquisition_function, lower_bounds=None,
                          upper_bounds=None, options=None, fixed_features=None, timeout_sec=None,
                          **kwargs):
    """Device-resident replacement of gen_candidates_scipy (generation/gen.py:
    46-298).

    ``algorithm="lbfgsb"`` (default): every restart runs scipy 1.15's L-BFGS-B
    (generalized Cauchy point, subspace minimisation, More-Thuente line search;
    csrc/lbfgsb_core.h) on the GPU with scipy's options ``maxcor`` / ``ftol`` /
    ``gtol`` / ``maxls`` / ``maxiter`` / ``maxfun`` and their defaults.  A
    restart's trial points are scipy's on the same objective; the reference
    runs ONE L-BFGS-B over the sum of the restarts' objectives, so its
    iterates equal these at b = 1 and differ (same stationary points) at b > 1.
    ``algorithm="projected"``: the round-1 projected L-BFGS with Armijo
    backtracking (``maxiter`` bounds its evaluations).

    One evaluation = one batched forward + backward of the acquisition at all
    trial points + one step launch; iterates, gradients and histories never
    leave HBM and the host reads the status vector every ``check_every``
    evaluations.  ``use_graph`` (default True): the evaluation is captured once
    as a HIP graph and replayed (botorch_amd.graphs) where the acquisition
    allows capture.  ``compact`` (L-BFGS-B; True, False or "auto", the
    default): at a status read where at most half of the batch is still
    running (and at least ``compact_min`` restarts have stopped), the running
    restarts continue as a smaller batch (their states gathered, the graph
    re-captured for the new shape), so stopped restarts no longer take slots
    in the evaluations; "auto" does so only when an evaluation has cost at
    least ``compact_eval_ms`` (2 ms) on average, and then also defers the
    first graph capture to the first status read.
    Returns (candidates b x q x d, acq values b); an
    OptimizationWarning is raised for restarts that end abnormally, as
    gen_candidates_scipy does for scipy's failures."""
    from . import _lib, kernels
    from ._lib import check, lib
    if fixed_features:
        raise NotImplementedError("fixed_features is not supported by the device optimiser")
    options = dict(options or {})
    algorithm = options.get("algorithm", "lbfgsb")
    if algorithm not in ("lbfgsb", "projected"):
        raise ValueError(f"algorithm={algorithm!r}: 'lbfgsb' or 'projected'")
    m = int(options.get("maxcor", 10))
    ftol = float(options.get("ftol", 1e7 * np.finfo(float).eps))  # scipy factr 1e7
    pgtol = float(options.get("gtol", 1e-5))
    check_every = int(options.get("check_every", 4 if algorithm == "lbfgsb" else 8))
    X0 = columnwise_clamp(initial_conditions, lower_bounds, upper_bounds).detach()
    if not X0.is_cuda:
        raise RuntimeError("gen_candidates_device runs on ROCm device tensors")
    shapeX = X0.shape
    lbfgsb = algorithm == "lbfgsb"
    if lbfgsb:
        maxiter = int(options.get("maxiter", 2000))  # gen_candidates_scipy's default
        maxfun = int(options.get("maxfun", 15000))
        maxls = int(options.get("maxls", 20))
        max_evals = maxfun + maxls + 1
        st = _LBFGSBState(X0, m)
    else:
        maxiter = int(options.get("maxiter", 200))
        max_evals = maxiter + 1
        st = _LBFGSState(X0, m)
    lo = (torch.as_tensor(lower_bounds, dtype=torch.float64, device=X0.device).expand(shapeX[-2:])
          .reshape(-1).contiguous() if lower_bounds is not None
          else torch.full((st.n,), -math.inf, dtype=torch.float64, device=X0.device))
    hi = (torch.as_tensor(upper_bounds, dtype=torch.float64, device=X0.device).expand(shapeX[-2:])
          .reshape(-1).contiguous() if upper_bounds is not None
          else torch.full((st.n,), math.inf, dtype=torch.float64, device=X0.device))
    stream = kernels._stream(X0.device)
    # one evaluation (forward + backward at all trial points) as a HIP graph
    # replay where the acquisition allows capture (the fused qEI / qLogEI
    # paths); the eager autograd evaluation otherwise
    use_graph = bool(options.get("use_graph", True))
    compact = options.get("compact", "auto") if lbfgsb else False
    compact_min = int(options.get("compact_min", 8))
    # "auto": shrink only when an evaluation costs at least this much (the
    # re-capture of the graph costs a few evaluations' worth: measured C3
    # 55 -> 35 ms, C2 9.1 -> 14.5 ms with an unconditional shrink; eager C3
    # evaluations take 2.5-3 ms, C2 ones 0.7-1.2 ms)
    compact_eval_ms = float(options.get("compact_eval_ms", 2.0))

    def _graph(state, shape):
        if not use_graph:
            return None
        from .graphs import GraphedAcquisition
        try:
            return GraphedAcquisition(acquisition_function, state.xt.view(shape), with_grad=True,
                                      warmup=1, check_each_call=False)
        except RuntimeError:  # capture refused (e.g. a generic route with host reads)
            torch.cuda.synchronize(X0.device)
            return None

    # expensive evaluations (the auto-compaction regime): the first capture
    # waits for the first status read, where the batch usually shrinks and is
    # captured at its new shape anyway; cheap ones are captured at once
    defer = use_graph and compact == "auto"
    expensive = False  # the first evaluation took >= compact_eval_ms
    ga = None if defer else _graph(st, shapeX)
    full, active = st, None   # the whole batch; rows of `full` that `st` holds
    shrinks = []
    t0 = time.monotonic()
    it = 0
    for it in range(max_evals):
        if ga is not None:
            v, g = ga(st.xt.view(shapeX))
            ft = (-v).reshape(-1).to(torch.float64).contiguous()
            gt = (-g).reshape(st.B, st.n).to(torch.float64).contiguous()
        else:
            Xt = st.xt.view(shapeX).detach().requires_grad_(True)
            ft = -acquisition_function(Xt)
            (gt,) = torch.autograd.grad(ft.sum(), Xt)
            ft = ft.detach().reshape(-1).to(torch.float64).contiguous()
            gt = gt.reshape(st.B, st.n).to(torch.float64).contiguous()
        if lbfgsb:
            a = _lib.LbfgsbArgs(B=st.B, n=st.n, m=m, maxls=maxls, maxiter=maxiter, maxfun=maxfun,
                                ftol=ftol, pgtol=pgtol, lower=lo, upper=hi, xt=st.xt, ft=ft, gt=gt,
                                v=st.v, iv=st.iv, ws=st.ws, wy=st.wy, mat=st.mat, ds=st.ds,
                                is_=st.is_)
            check(lib().bo_lbfgsb_step_v(ctypes.byref(a), stream), "lbfgsb_step")
        else:
            a = _lib.LbfgsStepArgs(B=st.B, n=st.n, m=m, x=st.x, f=st.f, g=st.g, xt=st.xt, ft=ft,
                                   gt=gt, d=st.d, alpha=st.alpha, S=st.S, Y=st.Y, rho=st.rho,
                                   hcount=st.hcount, hhead=st.hhead, status=st.status,
                                   nacc=st.nacc, lower=lo, upper=hi, c1=1e-4, ftol=ftol,
                                   pgtol=pgtol, min_alpha=1e-12)
            check(lib().bo_lbfgs_step_v(ctypes.byref(a), stream), "lbfgs_step")
        if defer and it == 0:
            torch.cuda.synchronize(X0.device)  # one eager evaluation timed
            expensive = 1e3 * (time.monotonic() - t0) >= compact_eval_ms
            if not expensive:
                defer = False
                ga = _graph(st, shapeX)
        if (it + 1) % check_every == 0 or it == max_evals - 1:
            if ga is not None:
                ga.check_status()
            running = st.status <= 0  # 0 running; -1: the projected path's first call
            n_run = int(running.sum())
            if n_run == 0:
                break
            if timeout_sec is not None and time.monotonic() - t0 > timeout_sec:
                break
            shrink = compact is True or (compact == "auto" and (
                expensive or 1e3 * (time.monotonic() - t0) / (it + 1) >= compact_eval_ms))
            if shrink and 2 * n_run <= st.B and st.B - n_run >= compact_min:
                keep = running.nonzero().flatten()
                if active is None:
                    rows, sub = keep, st.take(keep)
                else:
                    rows = active.index_select(0, keep)
                    full.put(active, st)
                    sub = full.take(rows)
                active, st = rows, sub
                shrinks.append((it + 1, st.B))
                shapeX = torch.Size((st.B,) + tuple(shapeX[1:]))
                ga = _graph(st, shapeX)
                defer = False
            elif defer:
                defer = False
                ga = _graph(st, shapeX)
    if active is not None:
        full.put(active, st)
        st = full
        shapeX = X0.shape
    cands = st.x.view(shapeX).to(initial_conditions.dtype)
    cands = columnwise_clamp(cands, lower_bounds, upper_bounds)
    with torch.no_grad():
        acq = acquisition_function(cands)
    if lbfgsb:
        bad = (st.status == 3) | (st.status == 6)
        if bool(bad.any()):
            codes = sorted({int(s) for s in st.status[bad].tolist()})
            warnings.warn(f"Optimization failed on the device for {int(bad.sum())} restart(s): "
                          + "; ".join(LBFGSB_STATUS[c_] for c_ in codes), OptimizationWarning)
    gen_candidates_device.last_state = st
    gen_candidates_device.last_evals = it + 1
    gen_candidates_device.last_shrinks = shrinks  # (evaluation, restarts kept)
    return cands, acq


def generate_in_chunks(acq_function, ics, bounds, batch_limit, options, gen_candidates):
    """_optimize_acqf_batch's loop over batch_limit chunks of the initial
    conditions (optimize.py:335-365): (candidates, values, any
    OptimizationWarning)."""
    gen_options = {k: v for k, v in (options or {}).items() if k not in INIT_OPTION_KEYS}
    cands, vals, warned = [], [], False
    for chunk in ics.split(max(1, batch_limit)):
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always", category=OptimizationWarning)
            c, v = gen_candidates(chunk, acq_function, lower_bounds=bounds[0],
                                  upper_bounds=bounds[1], options=gen_options)
        warned |= any(issubclass(x.category, OptimizationWarning) for x in w)
        cands.append(c)
        vals.append(v.reshape(-1))
    if not cands:
        return ics.clone(), ics.new_empty(0), False
    return torch.cat(cands), torch.cat(vals), warned


def optimize_acqf(acq_function, bounds, q, num_restarts, raw_samples=None, options=None,
                  batch_initial_conditions=None, return_best_only=True, gen_candidates=None,
                  sequential=False, retry_on_optimization_warning=True, **kwargs):
    """optim/optimize.py:397-543 -> _optimize_acqf_batch (:246-394): raw-sample
    initialisation, batch_limit chunks through gen_candidates_scipy, one retry
    on OptimizationWarning, argmax over restarts."""
    if sequential:
        raise NotImplementedError("sequential greedy optimisation is out of scope")
    options = options or {}
    gen_candidates = gen_candidates or gen_candidates_scipy
    if batch_initial_conditions is None:
        if raw_samples is None:
            raise ValueError("Must specify `raw_samples` when `batch_initial_conditions` is None`.")
        batch_initial_conditions = gen_batch_initial_conditions(
            acq_function, bounds, q, num_restarts, raw_samples, options=options)
    batch_limit = options.get("batch_limit", num_restarts)

    def _run(ics):
        return generate_in_chunks(acq_function, ics, bounds, batch_limit, options, gen_candidates)

    cands, vals, warned = _run(batch_initial_conditions)
    if retry_on_optimization_warning and warned:
        new_ics = gen_batch_initial_conditions(acq_function, bounds, q, num_restarts,
                                               raw_samples or num_restarts, options=options)
        cands, vals, warned = _run(new_ics)
    _check_deferred(cands)
    if return_best_only:
        best = torch.argmax(vals.view(-1), dim=0)
        return cands[best], vals[best]
    return cands, vals
