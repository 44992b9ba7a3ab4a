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
import logging
import math
import time
import warnings
from typing import Any, Callable, Dict, Optional, Tuple

import numpy as np
import torch
from scipy.optimize import minimize

from .exceptions import BadInitialCandidatesWarning, OptimizationWarning
from .utils_sampling import draw_sobol_samples, manual_seed

logger = logging.getLogger("botorch_amd")  # botorch/logging.py: quiet unless configured

INIT_OPTION_KEYS = {"alpha", "batch_limit", "eta", "init_batch_limit", "nonnegative", "n_burnin",
                    "sample_around_best", "sample_around_best_sigma",
                    "sample_around_best_prob_perturb", "seed", "thinning"}


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


def fix_features(X: torch.Tensor, fixed_features=None) -> torch.Tensor:
    """optim/utils/acquisition_utils.py:66-93: columns with a value are set to
    it (zero gradient); columns mapped to None are detached."""
    if fixed_features is None:
        return X
    cols = list(X.unbind(dim=-1))
    for k, v in fixed_features.items():
        cols[k] = cols[k].detach() if v is None else torch.full_like(cols[k], v)
    return torch.stack(cols, dim=-1)


def _normalize(X, bounds):
    return (X - bounds[0]) / (bounds[1] - bounds[0])


def _unnormalize(X, bounds):
    return X * (bounds[1] - bounds[0]) + bounds[0]


def _std_normal_cdf(x):
    return 0.5 * (1 + torch.erf(x / math.sqrt(2)))


def _std_normal_icdf(p):
    return torch.erfinv(2 * p - 1) * math.sqrt(2)


def sample_truncated_normal_perturbations(X, n_discrete_points, sigma, bounds, qmc=True):
    """optim/initializers.py:1145-1193: N(X, sigma^2 I) truncated to the unit
    cube by the inverse CDF, in normalised coordinates."""
    X = _normalize(X, bounds)
    d = X.shape[1]
    if X.shape[0] > 1:
        X = X[torch.randint(X.shape[0], (n_discrete_points,), device=X.device)]
    if qmc:
        unit = torch.zeros(2, d, dtype=X.dtype, device=X.device)
        unit[1] = 1
        u = draw_sobol_samples(bounds=unit, n=n_discrete_points, q=1).squeeze(1)
    else:
        u = torch.rand((n_discrete_points, d), dtype=X.dtype, device=X.device)
    lo_cdf = _std_normal_cdf(-X / sigma)
    hi_cdf = _std_normal_cdf((1 - X) / sigma)
    pert = _std_normal_icdf(lo_cdf + u * (hi_cdf - lo_cdf)) * sigma
    return _unnormalize((X + pert).clamp(0.0, 1.0), bounds)


def sample_perturbed_subset_dims(X, bounds, n_discrete_points, sigma=1e-1, qmc=True,
                                 prob_perturb=None):
    """optim/initializers.py:1196-1269: perturb a random subset of the
    dimensions (each with probability min(20/d, 1); a row that drew none gets
    ceil(d p) of them)."""
    if bounds.ndim != 2 or X.ndim != 2:
        raise ValueError("bounds must be 2 x d and X must be n x d")
    d = bounds.shape[-1]
    if prob_perturb is None:
        prob_perturb = min(20.0 / d, 1.0)
    if X.shape[0] == 1:
        X_cand = X.repeat(n_discrete_points, 1)
    else:
        X_cand = X[torch.randint(X.shape[0], (n_discrete_points,), device=X.device)]
    pert = sample_truncated_normal_perturbations(X_cand, n_discrete_points, sigma, bounds, qmc)
    mask = torch.rand(n_discrete_points, d, dtype=bounds.dtype, device=bounds.device) <= prob_perturb
    none = (~mask).all(dim=-1).nonzero()
    template = torch.zeros(d, dtype=mask.dtype, device=mask.device)
    template[:math.ceil(d * prob_perturb)] = True
    for row in none:
        mask[row] = template[torch.randperm(d, device=bounds.device)]
    X_cand[mask] = pert[mask]
    return X_cand


def get_X_baseline(acq_function):
    """optim/utils/acquisition_utils.py:96-135: the acquisition's X_baseline,
    else the model's training inputs (None if neither)."""
    Xb = getattr(acq_function, "X_baseline", None)
    if Xb is None:
        model = getattr(acq_function, "model", None)
        if model is None:
            return None
        ti = getattr(model, "train_inputs", None)
        if ti is None and hasattr(model, "models"):
            ti = getattr(model.models[0], "train_inputs", None)
        if ti is None:
            return None
        Xb = ti[0]
    while Xb is not None and Xb.ndim > 2:
        Xb = Xb[0]
    return Xb if Xb is not None and Xb.shape[0] > 0 else None


def sample_points_around_best(acq_function, n_discrete_points, sigma, bounds, best_pct=5.0,
                              subset_sigma=1e-1, prob_perturb=None):
    """optim/initializers.py:1040-1142: the best_pct % best baseline points by
    posterior mean (or the Pareto set of a multi-output objective), perturbed;
    None without baseline points."""
    from .exceptions import BotorchWarning
    X = get_X_baseline(acq_function)
    if X is None:
        return None
    with torch.no_grad():
        try:
            mean = acq_function.model.posterior(X).mean
        except AttributeError:
            warnings.warn("Failed to sample around previous best points.", BotorchWarning)
            return None
        while mean.ndim > 2:
            mean = mean.mean(dim=0)
        try:
            f_pred = acq_function.objective(mean)
        except (AttributeError, TypeError):
            f_pred = mean
        if hasattr(acq_function, "maximize") and not acq_function.maximize:
            f_pred = -f_pred
        constraints = getattr(acq_function, "constraints", None)
        if constraints is not None:
            neg_violation = -torch.stack([c(mean).clamp_min(0.0) for c in constraints],
                                         dim=-1).sum(dim=-1)
            feas = neg_violation == 0
            if feas.any():
                f_pred[~feas] = float("-inf")
            else:
                f_pred = neg_violation
        if f_pred.ndim == mean.ndim and f_pred.shape[-1] > 1:
            from .multi_objective import is_non_dominated
            best_X = X[is_non_dominated(f_pred)]
        else:
            if f_pred.shape[-1] == 1:
                f_pred = f_pred.squeeze(-1)
            n_best = max(1, round(X.shape[0] * best_pct / 100))
            best_X = X[torch.topk(f_pred, n_best).indices.view(-1)]
    subset = best_X.shape[-1] >= 20 or prob_perturb is not None
    n_tn = n_discrete_points // 2 if subset else n_discrete_points
    out = sample_truncated_normal_perturbations(best_X, n_tn, sigma, bounds)
    if subset:
        sub = sample_perturbed_subset_dims(best_X, bounds, n_discrete_points - n_tn, sigma,
                                           prob_perturb=prob_perturb)
        out = torch.cat([out, sub], dim=0)
        out = out[torch.randperm(out.shape[0], device=X.device)]
    return out


SOBOL_MAXDIM = 21201  # torch.quasirandom.SobolEngine.MAXDIM


def check_init_inputs(bounds, options, equality_constraints=None, generator=None) -> None:
    """The argument checks of gen_batch_initial_conditions (initializers.py:
    305-330)."""
    from .exceptions import UnsupportedError
    if bounds.isinf().any():
        raise NotImplementedError("Currently only finite values in `bounds` are supported for "
                                  "generating initial conditions for optimization.")
    sample_around_best = (options or {}).get("sample_around_best", False)
    if sample_around_best and equality_constraints:
        raise UnsupportedError("Option 'sample_around_best' is not supported when equality"
                               "constraints are present.")
    if sample_around_best and generator:
        raise UnsupportedError("Option 'sample_around_best' is not supported when custom "
                               "generator is be used.")


def raw_designs_use_global_rng(options, seed, generator=None, constrained=False) -> bool:
    """Whether raw_designs may draw from the global torch generator (so that
    replicas of it on several ranks could differ): points around the
    incumbents, a caller's generator, an unseeded draw, or the polytope chain
    (its d = 1 directions are random signs from the global generator)."""
    return bool((options or {}).get("sample_around_best", False)) or generator is not None \
        or seed is None or bool(constrained)


def raw_designs(acq_function, bounds, q, n, seed, options, fixed_features=None,
                inequality_constraints=None, equality_constraints=None, generator=None,
                fixed_X_fantasies=None) -> torch.Tensor:
    """The n raw q-batch designs of one round of gen_batch_initial_conditions
    (initializers.py:350-410): ``generator(n, q, seed)``, or polytope q-batches
    under linear constraints, or the Sobol draw (uniform past
    SobolEngine.MAXDIM); joined by points around the incumbents
    (``sample_around_best``), features fixed, ``fixed_X_fantasies`` appended."""
    options = options or {}
    d = bounds.shape[-1]
    if generator is not None:
        X_rnd = generator(n, q, seed)
    elif inequality_constraints or equality_constraints:
        from .constraints import sample_q_batches_from_polytope
        X_rnd = sample_q_batches_from_polytope(
            n=n, q=q, bounds=bounds, n_burnin=options.get("n_burnin", 10000),
            n_thinning=options.get("n_thinning", 32), seed=seed,
            equality_constraints=equality_constraints,
            inequality_constraints=inequality_constraints)
    elif d * q <= SOBOL_MAXDIM:
        X_rnd = draw_raw_samples(bounds, n, q, seed)
    else:
        b_cpu = bounds.cpu()
        with manual_seed(seed):
            u = torch.rand(n, q, d, dtype=bounds.dtype)
        X_rnd = b_cpu[0] + (b_cpu[1] - b_cpu[0]) * u
    if options.get("sample_around_best", False):
        X_best = sample_points_around_best(
            acq_function, n_discrete_points=n * q,
            sigma=options.get("sample_around_best_sigma", 1e-3), bounds=bounds,
            subset_sigma=options.get("sample_around_best_subset_sigma", 1e-1),
            prob_perturb=options.get("sample_around_best_prob_perturb"))
        if X_best is not None:
            X_rnd = torch.cat([X_rnd, X_best.view(n, q, d).to(X_rnd)], dim=0)
    X_rnd = fix_features(X_rnd, fixed_features)
    if fixed_X_fantasies is not None:
        if fixed_X_fantasies.shape[-1] != X_rnd.shape[-1]:
            raise ValueError("`fixed_X_fantasies` and `bounds` must both have the same "
                             f"trailing dimension `d`, but have {fixed_X_fantasies.shape[-1]} "
                             f"and {X_rnd.shape[-1]}, respectively.")
        fx = fixed_X_fantasies.to(X_rnd)
        X_rnd = torch.cat([X_rnd, fx.unsqueeze(0).expand(X_rnd.shape[0], *fx.shape)], dim=-2)
    return X_rnd


def gen_batch_initial_conditions(acq_function, bounds, q, num_restarts, raw_samples,
                                 fixed_features=None, options=None, inequality_constraints=None,
                                 equality_constraints=None, generator=None, fixed_X_fantasies=None):
    """optim/initializers.py:243-438: Sobol raw samples (or ``generator(n, q,
    seed)``; uniform draws past SobolEngine.MAXDIM), optionally joined by
    points sampled around the incumbents, features fixed, forward-only
    evaluation in chunks of init_batch_limit, Boltzmann selection; retried with
    up to 5x the raw samples (seed + 1 each time) while the selection warns.

    MI355X path (bounds on the GPU): the raw designs are generated on the
    device (bo_sobol_box, bit-identical to draw_sobol_samples) and evaluated
    there chunk by chunk; only the values cross to the host, once, for the
    selection, which draws from the global CPU generator as the reference does
    (so the picks are the reference's).  Under linear constraints the raw
    designs are q-batches of the hit-and-run chain over the feasible polytope
    (constraints.sample_q_batches_from_polytope, initializers.py:365-375; the
    chain's steps in native host code), evaluated on the device the same way."""
    options = options or {}
    check_init_inputs(bounds, options, equality_constraints, generator)
    seed, batch_limit, init_func, init_kwargs = init_options(acq_function, bounds, options)
    q = 1 if q is None else q
    factor, max_factor = 1, 5
    while factor < max_factor:
        n = raw_samples * factor
        X_rnd = raw_designs(acq_function, bounds, q, n, seed, options, fixed_features,
                            inequality_constraints, equality_constraints, generator,
                            fixed_X_fantasies)
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


def minimize_with_timeout(fun, x0, args=(), method=None, jac=None, bounds=None, constraints=(),
                          tol=None, callback=None, options=None, timeout_sec=None):
    """optim/utils/timeout.py:19-108: scipy.optimize.minimize whose callback
    raises once ``timeout_sec`` has passed; the iterate it held is returned as
    an unsuccessful result with the message "Optimization timed out after
    <s> seconds." (status 1, as L-BFGS-B's maxiter stop)."""
    from scipy.optimize import OptimizeResult
    from .exceptions import OptimizationTimeoutError
    wrapped = callback
    if timeout_sec is not None:
        t0 = time.monotonic()
        n_it = [0]

        def wrapped(xk, *extra):
            runtime = time.monotonic() - t0
            n_it[0] += 1
            if runtime > timeout_sec:
                raise OptimizationTimeoutError(current_x=xk, runtime=runtime)
            if callback is not None:
                return callback(xk, *extra)
            return False
    try:
        kw = dict(method=method, jac=jac, bounds=bounds, tol=tol, callback=wrapped,
                  options=options)
        if constraints:
            kw["constraints"] = constraints
        return minimize(fun, x0, args=args, **kw)
    except OptimizationTimeoutError as e:
        fval = fun(e.current_x, *args)
        fval = fval[0] if isinstance(fval, tuple) else fval
        return OptimizeResult(fun=fval, x=e.current_x, nit=n_it[0], success=False, status=1,
                              message=f"Optimization timed out after {e.runtime} seconds.")


def _process_scipy_result(res, options) -> None:
    """generation/gen.py:458-493: the iteration limit, the evaluation limit and
    a timeout are logged, not warned; any other unsuccessful exit warns
    OptimizationWarning (which makes optimize_acqf retry)."""
    if "success" not in res.keys() or "status" not in res.keys():
        warnings.warn("Optimization failed within `scipy.optimize.minimize` with no status "
                      "returned to `res.`", OptimizationWarning)
    elif not res.success:
        msg = str(res.message)
        if ("ITERATIONS REACHED LIMIT" in msg or "Iteration limit reached" in msg
                or "EVALUATIONS EXCEEDS LIMIT" in msg or "Optimization timed out after" in msg):
            logger.info("`scipy.minimize` exited: %s (maxiter %s, maxfun %s)", msg,
                        options.get("maxiter"), options.get("maxfun"))
        else:
            warnings.warn(f"Optimization failed within `scipy.optimize.minimize` with status "
                          f"{res.status} and message {msg}.", OptimizationWarning)


def _without_fixed_features(fixed_features, acquisition_function, initial_conditions,
                            lower_bounds, upper_bounds):
    """generation/utils.py:102-196 without constraints: the base acquisition
    wrapped so that it takes only the free columns, and the initial conditions
    and bounds restricted to them."""
    from .acquisition import FixedFeatureAcquisitionFunction
    keys = sorted(fixed_features)
    vals = [initial_conditions[..., [k]] if fixed_features[k] is None else fixed_features[k]
            for k in keys]
    d = initial_conditions.shape[-1]
    ff = FixedFeatureAcquisitionFunction(acquisition_function, d=d, columns=keys, values=vals)
    free = sorted(set(range(d)) - set(keys))
    ics = initial_conditions[..., free]
    if torch.is_tensor(lower_bounds):
        lower_bounds = lower_bounds[..., free]
    if torch.is_tensor(upper_bounds):
        upper_bounds = upper_bounds[..., free]
    return ff, ics, lower_bounds, upper_bounds


def _reject_constraints(inequality_constraints, equality_constraints,
                        nonlinear_inequality_constraints, where: str = "this path") -> None:
    """Nonlinear constraints are out of scope; linear
    ones are refused only by the device-resident L-BFGS-B."""
    from .exceptions import UnsupportedError
    if nonlinear_inequality_constraints:
        raise UnsupportedError("nonlinear inequality constraints are not supported on "
                               f"{where}")
    if inequality_constraints or equality_constraints:
        raise UnsupportedError(f"linear parameter constraints are not supported by {where}: "
                               "use gen_candidates_scipy (SLSQP, generation/gen.py:256)")


def gen_candidates_scipy(initial_conditions, acquisition_function, lower_bounds=None,
                         upper_bounds=None, inequality_constraints=None, equality_constraints=None,
                         nonlinear_inequality_constraints=None, options=None, fixed_features=None,
                         timeout_sec=None):
    """generation/gen.py:46-298: scipy.optimize.minimize over the flattened
    t-batch -- L-BFGS-B on the box, SLSQP (the reference's default there)
    when linear constraints are given (make_scipy_linear_constraints records,
    gen.py:182-189, 256).  Fixed features are removed from the search space
    (gen.py:124-175; the constraints rewritten on the free features) unless a
    constraint is present and some fixed value is None, in which case the
    full space is searched with the features pinned inside the objective
    (gen.py:208).  The run is bounded by ``timeout_sec`` (minimize_with_timeout,
    gen.py:252-267), its exit resolved by _process_scipy_result (gen.py:268),
    the result clamped with raise_on_violation.  Nonlinear constraints raise
    UnsupportedError."""
    from .constraints import (_generate_unfixed_lin_constraints, make_scipy_bounds,
                              make_scipy_linear_constraints)
    _reject_constraints(None, None, nonlinear_inequality_constraints, "gen_candidates_scipy")
    options = dict(options or {})
    options = {**options, "maxiter": options.get("maxiter", 2000)}
    linear = bool(inequality_constraints or equality_constraints)
    if fixed_features and (not linear or None not in fixed_features.values()):
        d = initial_conditions.shape[-1]
        ff, ics, lo, hi = _without_fixed_features(fixed_features, acquisition_function,
                                                  initial_conditions, lower_bounds, upper_bounds)
        ineq = _generate_unfixed_lin_constraints(inequality_constraints, fixed_features, d, False)
        eq = _generate_unfixed_lin_constraints(equality_constraints, fixed_features, d, True)
        c, acq = gen_candidates_scipy(ics, ff, lo, hi, inequality_constraints=ineq,
                                      equality_constraints=eq, options=options,
                                      timeout_sec=timeout_sec)
        return ff._construct_X_full(c), acq
    pinned = fixed_features or None  # only reached with constraints and a None value
    clamped = columnwise_clamp(initial_conditions, lower_bounds, upper_bounds)
    shapeX = clamped.shape
    x0 = clamped.detach().reshape(-1).cpu().numpy()
    if linear:
        scipy_bounds = make_scipy_bounds(initial_conditions, lower_bounds, upper_bounds)
        cons = make_scipy_linear_constraints(shapeX, inequality_constraints, equality_constraints)
    else:
        lb = (torch.as_tensor(lower_bounds).expand(shapeX).reshape(-1).cpu().numpy()
              if lower_bounds is not None else np.full(x0.shape, -np.inf))
        ub = (torch.as_tensor(upper_bounds).expand(shapeX).reshape(-1).cpu().numpy()
              if upper_bounds is not None else np.full(x0.shape, np.inf))
        scipy_bounds = list(zip(lb, ub))
        cons = []
    with_grad = options.get("with_grad", True)

    def f_np_wrapper(x: np.ndarray):
        if np.isnan(x).any():
            raise RuntimeError(f"{np.isnan(x).sum()} elements of the {x.size} element array `x` are NaN.")
        X = torch.from_numpy(x).to(initial_conditions).view(shapeX).contiguous().requires_grad_(True)
        loss = -acquisition_function(fix_features(X, pinned)).sum()
        grad = torch.autograd.grad(loss, X)[0].contiguous().view(-1).cpu().numpy()
        _check_deferred(X)
        if np.isnan(grad).any():
            raise RuntimeError(f"{np.isnan(grad).sum()} elements of the {x.size} element gradient "
                               "array `gradf` are NaN. This often indicates numerical issues.")
        return loss.item(), grad

    def f_only(x):
        X = torch.from_numpy(x).to(initial_conditions).view(shapeX).contiguous()
        with torch.no_grad():
            val = -acquisition_function(fix_features(X, pinned)).sum().item()
        _check_deferred(X)
        return val

    res = minimize_with_timeout(f_np_wrapper if with_grad else f_only, x0,
                                method=options.get("method", "SLSQP" if cons else "L-BFGS-B"),
                                jac=with_grad, bounds=scipy_bounds, constraints=cons,
                                callback=options.get("callback", None),
                                options={k: v for k, v in options.items()
                                         if k not in ("method", "callback", "with_grad")},
                                timeout_sec=timeout_sec)
    _process_scipy_result(res, options)
    candidates = fix_features(torch.from_numpy(res.x).to(initial_conditions).reshape(shapeX),
                              pinned)
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


def _eval_flops(acquisition_function, B: int, q: int):
    """Deterministic cost of one forward + backward of a GP acquisition at B
    t-batches of q points: 2 x B q' n^2 (the two triangular n x n contractions,
    R = K*x L^-T and its backward W), summed over the GP members (a
    ModelListGP's outputs, a SAAS ensemble), q' = q + pending (+ r baseline
    rows for the cached-root qNEI).  None when there is no GP to estimate."""
    acq = acquisition_function
    while hasattr(acq, "acq_func"):  # FixedFeatureAcquisitionFunction
        acq = acq.acq_func
    model = getattr(acq, "model", None)
    if model is None:
        return None
    members = list(getattr(model, "models", None) or [model])
    qq = q + (0 if getattr(acq, "X_pending", None) is None else int(acq.X_pending.shape[-2]))
    total = 0.0
    for mm in members:
        ti = getattr(mm, "train_inputs", None)
        if ti is None:
            return None
        n = int(ti[0].shape[-2])
        total += 2.0 * B * qq * n * n * max(1, int(getattr(mm, "num_mcmc_samples", 1) or 1))
    return total


def _fused_qei(acquisition_function, X: torch.Tensor) -> bool:
    """The evaluation runs the fused qEI / qLogEI forward and backward (two
    native calls, acquisition._fused_mc)."""
    from .acquisition import qExpectedImprovement
    acq = acquisition_function
    while hasattr(acq, "acq_func"):  # FixedFeatureAcquisitionFunction
        acq = acq.acq_func
    return isinstance(acq, qExpectedImprovement) and bool(acq._fused_eligible(X))


def gen_candidates_device(initial_conditions, acquisition_function, lower_bounds=None,
                          upper_bounds=None, inequality_constraints=None,
                          equality_constraints=None, nonlinear_inequality_constraints=None,
                          options=None, fixed_features=None, timeout_sec=None):
    """Device-resident replacement of gen_candidates_scipy (generation/gen.py:
    46-298).

    ``algorithm="lbfgsb"`` (default): every restart runs scipy 1.15's L-BFGS-B
    (generalized Cauchy point, subspace minimisation, More-Thuente line search;
    csrc/lbfgsb_core.h) on the GPU with scipy's options ``maxcor`` / ``ftol`` /
    ``gtol`` / ``maxls`` / ``maxiter`` / ``maxfun`` and their defaults.  A
    restart's trial points are scipy's on the same objective; the reference
    runs ONE L-BFGS-B over the sum of the restarts' objectives, so its
    iterates equal these at b = 1 and differ (same stationary points) at b > 1.
    ``joint=True``: the reference's problem itself -- one L-BFGS-B over all
    b q d variables of the batch and the summed objective (one line search,
    one memory; a single device "restart" on a 4-wave workgroup), whose
    iterates are scipy's on gen_candidates_scipy's objective.
    ``algorithm="projected"``: the round-1 projected L-BFGS with Armijo
    backtracking (``maxiter`` bounds its evaluations).

    One evaluation = one batched forward + backward of the acquisition at all
    trial points + one step launch; iterates, gradients and histories never
    leave HBM and the host reads the status vector every ``check_every``
    evaluations (and, where the batch can shrink, after evaluations 1 and 2:
    ``early_checks``).  ``use_graph`` (True, False or "auto", the default): the
    evaluation is captured once as a HIP graph and replayed
    (botorch_amd.graphs) where the acquisition allows capture; "auto" keeps
    the fused qEI / qLogEI evaluation eager (a replay saves it no host work and
    is slower on the device).  ``compact`` (L-BFGS-B; True, False or "auto", the
    default): at a status read where at most half of the batch is still
    running (and at least ``compact_min`` restarts have stopped), the running
    restarts continue as a smaller batch (their states gathered; the graph
    is re-captured for the new shape only after ``recapture_after`` (16)
    more evaluations -- the tail after a shrink is usually short and a
    capture costs more than its replays save there), so stopped restarts no
    longer take slots
    in the evaluations; "auto" does so only for expensive evaluations --
    decided once, before the first evaluation, from the acquisition's
    deterministic cost estimate (forward + backward GP flops 2 B q' n^2 against
    ``compact_flops``, default 1e10: C3's 128 restarts shrink, C2's 64 do not;
    the minimum of two timed evaluations against ``compact_eval_ms`` only when
    the acquisition has no GP model to estimate) -- and then also defers the
    first graph capture to the first status read.  The shrunken batch runs the
    same per-restart L-BFGS-B, but its evaluations take the split plan of the
    smaller batch, so f and g are summed in another order (equal to ~1e-15
    relative, not bit for bit): a compacted run is deterministic from run to
    run and box to box, and equal to the uncompacted one to rounding.
    Returns (candidates b x q x d, acq values b); an
    OptimizationWarning is raised for restarts that end abnormally, as
    gen_candidates_scipy does for scipy's failures."""
    from . import _lib, kernels
    from ._lib import check, lib
    _reject_constraints(inequality_constraints, equality_constraints,
                        nonlinear_inequality_constraints, "gen_candidates_device")
    if fixed_features:  # the search space without them (generation/utils.py:102-196)
        ff, ics, lo_b, hi_b = _without_fixed_features(fixed_features, acquisition_function,
                                                      initial_conditions, lower_bounds,
                                                      upper_bounds)
        c, acq = gen_candidates_device(ics, ff, lo_b, hi_b, options=options,
                                       timeout_sec=timeout_sec)
        return ff._construct_X_full(c), acq
    options = dict(options or {})
    algorithm = options.get("algorithm", "lbfgsb")
    if algorithm not in ("lbfgsb", "projected"):
        raise ValueError(f"algorithm={algorithm!r}: 'lbfgsb' or 'projected'")
    m = int(options.get("maxcor", 10))
    ftol = float(options.get("ftol", 1e7 * np.finfo(float).eps))  # scipy factr 1e7
    pgtol = float(options.get("gtol", 1e-5))
    check_every = int(options.get("check_every", 4 if algorithm == "lbfgsb" else 8))
    # where the batch can shrink, the status is also read after evaluations 1
    # and 2: restarts that start at a stationary point (qEI's flat zero
    # region) stop at their first evaluation -- C3: 126 of 128 -- and the
    # shrink then spares the full-batch evaluations up to the regular read
    # (optimize_acqf 18.7 -> 16.2 ms, tools/check_every.py)
    early_checks = (1, 2) if options.get("early_checks", True) else ()
    X0 = columnwise_clamp(initial_conditions, lower_bounds, upper_bounds).detach()
    if not X0.is_cuda:
        raise RuntimeError("gen_candidates_device runs on ROCm device tensors")
    shapeX = X0.shape
    lbfgsb = algorithm == "lbfgsb"
    # joint: the reference's own problem (gen.py:252-267) -- ONE L-BFGS-B over
    # all b q d variables with f = -sum_b acq(X_b), one line search and one
    # memory for the whole batch (a single device "restart" of n = b q d)
    joint = bool(options.get("joint", False))
    if joint and not lbfgsb:
        raise ValueError("joint=True runs scipy's L-BFGS-B (algorithm='lbfgsb')")
    if lbfgsb:
        maxiter = int(options.get("maxiter", 2000))  # gen_candidates_scipy's default
        maxfun = int(options.get("maxfun", 15000))
        maxls = int(options.get("maxls", 20))
        max_evals = maxfun + maxls + 1
        st = _LBFGSBState(X0.reshape(1, -1) if joint else X0, m)
    else:
        maxiter = int(options.get("maxiter", 200))
        max_evals = maxiter + 1
        st = _LBFGSState(X0, m)
    bshape = shapeX if joint else shapeX[-2:]  # the bounds of one device restart
    lo = (torch.as_tensor(lower_bounds, dtype=torch.float64, device=X0.device).expand(bshape)
          .reshape(-1).contiguous() if lower_bounds is not None
          else torch.full((st.n,), -math.inf, dtype=torch.float64, device=X0.device))
    hi = (torch.as_tensor(upper_bounds, dtype=torch.float64, device=X0.device).expand(bshape)
          .reshape(-1).contiguous() if upper_bounds is not None
          else torch.full((st.n,), math.inf, dtype=torch.float64, device=X0.device))
    stream = kernels._stream(X0.device)
    # one evaluation (forward + backward at all trial points) as a HIP graph
    # replay where the acquisition allows capture; the eager autograd
    # evaluation otherwise.  "auto" (default): eager for the fused qEI /
    # qLogEI evaluation -- one native call per forward and per backward, so a
    # replay saves no host work: measured inside optimize_acqf, C2 eager 6.6
    # against 7.0 ms with the capture, and at C3 a replay is slower than the
    # eager call (0.29 against 0.27 ms at b = 2, 1.49 against 1.38 ms at
    # b = 128; tools/c2_opt_graph.py, tools/capture_cost.py) -- and a
    # captured graph for the other routes
    ug = options.get("use_graph", "auto")
    use_graph = not _fused_qei(acquisition_function, X0) if ug == "auto" else bool(ug)
    compact = options.get("compact", "auto") if lbfgsb and not joint else False
    compact_min = int(options.get("compact_min", 8))
    # after a shrink the evaluation graph is re-captured only once the smaller
    # batch has run ``recapture_after`` more evaluations: a capture costs ~6
    # ms at C3 against ~0.25 ms of host time saved per replay, and the
    # restarts left at a shrink usually stop soon (C3: 2 of 128 running after
    # 4 evaluations, 16 more; re-captured at once 18.0 ms, eager 15.3 ms)
    recapture_after = int(options.get("recapture_after", 16))
    recapture_at = None  # evaluation count at which the deferred re-capture is due
    # "auto": shrink only expensive evaluations (the re-capture of the graph
    # costs a few evaluations' worth: measured C3 55 -> 35 ms, C2 9.1 -> 14.5 ms
    # with an unconditional shrink; eager C3 evaluations take 2.5-3 ms, C2 ones
    # 0.7-1.2 ms)
    compact_eval_ms = float(options.get("compact_eval_ms", 2.0))
    est = _eval_flops(acquisition_function, shapeX[0], shapeX[-2])
    expensive = (compact == "auto" and est is not None
                 and est >= float(options.get("compact_flops", 1e10)))
    timed = compact == "auto" and est is None  # no estimate: time two evaluations
    eval_ms = []

    graph_errors = []  # why capture was refused, recorded (not swallowed)

    def _graph(state, shape):
        if not use_graph:
            return None
        from .graphs import GraphedAcquisition
        try:
            return GraphedAcquisition(acquisition_function, state.xt.view(shape), with_grad=True,
                                      warmup=1, check_each_call=False, share_input=True)
        except RuntimeError as e:  # capture refused (e.g. a generic route with host reads)
            torch.cuda.synchronize(X0.device)
            graph_errors.append(f"{type(e).__name__}: {e}")
            logger.info("gen_candidates_device: evaluation graph not captured, eager "
                        "evaluations instead (%s)", graph_errors[-1])
            return None

    # expensive evaluations (the auto-compaction regime): the first capture
    # waits for the first status read, where the batch usually shrinks and is
    # captured at its new shape anyway; cheap ones are captured at once
    defer = use_graph and (expensive or timed)
    ga = None if defer else _graph(st, shapeX)
    full, active = st, None   # the whole batch; rows of `full` that `st` holds
    shrinks = []
    graphed_evals = 0
    t0 = time.monotonic()
    it = 0
    for it in range(max_evals):
        if ga is not None:
            graphed_evals += 1
            v, g = ga(st.xt.view(shapeX))
            ft, gt = -v, -g
        else:
            Xt = st.xt.view(shapeX).detach().requires_grad_(True)
            ft = -acquisition_function(Xt)
            (gt,) = torch.autograd.grad(ft.sum(), Xt)
            ft = ft.detach()
        if joint:  # gen.py's loss: -acq(X).sum() over the whole batch
            ft = ft.sum()
        ft = ft.reshape(-1).to(torch.float64).contiguous()
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
        if timed and it < 2:
            torch.cuda.synchronize(X0.device)  # two eager evaluations timed, the min kept
            eval_ms.append(1e3 * (time.monotonic() - (t0 if it == 0 else t_prev)))
            t_prev = time.monotonic()
            if it == 1:
                timed = False
                expensive = min(eval_ms) >= compact_eval_ms
                if not expensive and defer:
                    defer = False
                    ga = _graph(st, shapeX)
        shrink = compact is True or (compact == "auto" and expensive)
        if ((it + 1) % check_every == 0 or it == max_evals - 1
                or (shrink and it + 1 in early_checks)):
            if ga is not None:
                ga.check_status()
            running = st.status <= 0  # 0 running; -1: the projected path's first call
            n_run = int(running.sum())
            if n_run == 0:
                break
            if timeout_sec is not None and time.monotonic() - t0 > timeout_sec:
                break
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
                ga = None
                defer = False
                recapture_at = it + 1 + recapture_after if use_graph else None
            elif recapture_at is not None and it + 1 >= recapture_at:
                recapture_at = None
                ga = _graph(st, shapeX)
            elif defer:
                defer = False
                ga = _graph(st, shapeX)
    if active is not None:
        full.put(active, st)
        st = full
        shapeX = X0.shape
    cands = st.x.view(shapeX).to(initial_conditions.dtype)
    cands = columnwise_clamp(cands, lower_bounds, upper_bounds)
    # every restart converged (status 1 / 2): each x is an accepted iterate,
    # inside the box, and the state holds its objective f = -acq(x) from the
    # evaluation that accepted it -- the values gen_candidates_scipy computes
    # by evaluating the candidates once more (gen.py:292-296), without that
    # forward (C3: 0.71 ms at b = 128).  Joint runs (f is the batch sum) and
    # any other stop evaluate the candidates.
    if lbfgsb and not joint and bool(((st.status == 1) | (st.status == 2)).all()):
        acq = (-st.f).to(cands.dtype).reshape(shapeX[:-2])
    else:
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
    # evaluations replayed from a captured graph, and why a capture was refused
    gen_candidates_device.last_graphed_evals = graphed_evals
    gen_candidates_device.last_graph_error = graph_errors[-1] if graph_errors else None
    kernels.drop_keepalive()
    return cands, acq


def generate_in_chunks(acq_function, ics, bounds, batch_limit, options, gen_candidates,
                       fixed_features=None, timeout_sec=None, **constraints):
    """_optimize_acqf_batch's loop over batch_limit chunks of the initial
    conditions (optimize.py:277-326): ``timeout_sec`` is shared evenly by the
    chunks, an all-infinite bound is passed as None.  Returns (candidates,
    values, the OptimizationWarnings the chunks raised)."""
    gen_options = {k: v for k, v in (options or {}).items() if k not in INIT_OPTION_KEYS}
    chunks = ics.split(max(1, batch_limit))
    t_chunk = timeout_sec / len(chunks) if timeout_sec is not None and len(chunks) else None
    lo = None if bounds[0].isinf().all() else bounds[0]
    hi = None if bounds[1].isinf().all() else bounds[1]
    cands, vals, opt_ws = [], [], []
    for chunk in chunks:
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always", category=OptimizationWarning)
            c, v = gen_candidates(chunk, acq_function, lower_bounds=lo, upper_bounds=hi,
                                  options=gen_options, fixed_features=fixed_features,
                                  timeout_sec=t_chunk, **constraints)
        opt_ws += [x for x in w if issubclass(x.category, OptimizationWarning)]
        for x in w:  # everything else is passed on, as the reference's recorder does not
            if not issubclass(x.category, OptimizationWarning):
                warnings.warn_explicit(x.message, x.category, x.filename, x.lineno)
        cands.append(c)
        vals.append(v)
    if not cands:
        return ics.clone(), ics.new_empty(0), opt_ws
    if vals[0].ndim == 0:
        return torch.cat(cands), torch.stack(vals), opt_ws
    return torch.cat(cands), torch.cat(vals).flatten(), opt_ws


def _validate_optimize_inputs(bounds, raw_samples, batch_initial_conditions, ic_generator,
                              inequality_constraints) -> None:
    """OptimizeAcqfInputs.__post_init__ (optimize.py:94-128)."""
    if inequality_constraints is None and not (bounds.ndim == 2 and bounds.shape[0] == 2):
        raise ValueError(f"bounds should be a `2 x d` tensor, current shape: {list(bounds.shape)}.")
    d = bounds.shape[1]
    if batch_initial_conditions is not None:
        shp = batch_initial_conditions.shape
        if len(shp) not in (2, 3):
            raise ValueError("batch_initial_conditions must be 2-dimensional or 3-dimensional. "
                             f"Its shape is {shp}.")
        if shp[-1] != d:
            raise ValueError(f"batch_initial_conditions.shape[-1] must be {d}. The shape is {shp}.")
    elif ic_generator is None and raw_samples is None:
        raise ValueError("Must specify `raw_samples` when `batch_initial_conditions` is None`.")


def _optimize_acqf_batch(acq_function, bounds, q, num_restarts, raw_samples, options,
                         fixed_features, post_processing_func, batch_initial_conditions,
                         return_best_only, gen_candidates, ic_generator, timeout_sec,
                         retry_on_optimization_warning, ic_gen_kwargs,
                         inequality_constraints=None, equality_constraints=None):
    """optimize.py:246-394 (the linear constraints go to the initial-condition
    generator always and to ``gen_candidates`` when given, :255-303)."""
    options = options or {}
    provided = batch_initial_conditions is not None
    ic_gen = ic_generator or gen_batch_initial_conditions

    def _ics():
        return ic_gen(acq_function=acq_function, bounds=bounds, q=q, num_restarts=num_restarts,
                      raw_samples=raw_samples, fixed_features=fixed_features, options=options,
                      inequality_constraints=inequality_constraints,
                      equality_constraints=equality_constraints, **ic_gen_kwargs)

    ics = batch_initial_conditions if provided else _ics()
    batch_limit = options.get("batch_limit", num_restarts)
    linear = {k: v for k, v in (("inequality_constraints", inequality_constraints),
                                ("equality_constraints", equality_constraints)) if v is not None}

    def _run(x0):
        return generate_in_chunks(acq_function, x0, bounds, batch_limit, options, gen_candidates,
                                  fixed_features=fixed_features, timeout_sec=timeout_sec,
                                  **linear)

    cands, vals, ws = _run(ics)
    if ws and retry_on_optimization_warning:
        msgs = [str(w.message) for w in ws]
        if provided:
            warnings.warn(f"Optimization failed in `gen_candidates_scipy` with the following "
                          f"warning(s):\n{msgs}\nBecause you specified `batch_initial_conditions`, "
                          "optimization will not be retried with new initial conditions and will "
                          "proceed with the current solution. Suggested remediation: Try again "
                          "with different `batch_initial_conditions`, or don't provide "
                          "`batch_initial_conditions.`", RuntimeWarning)
        else:
            warnings.warn(f"Optimization failed in `gen_candidates_scipy` with the following "
                          f"warning(s):\n{msgs}\nTrying again with a new set of initial "
                          "conditions.", RuntimeWarning)
            cands, vals, ws = _run(_ics())
            if ws:
                warnings.warn("Optimization failed on the second try, after generating a new set "
                              "of initial conditions.", RuntimeWarning)
    if post_processing_func is not None:
        cands = post_processing_func(cands)
        with torch.no_grad():
            vals = torch.cat([acq_function(c) for c in cands.split(batch_limit, dim=0)], dim=0)
    _check_deferred(cands)
    if return_best_only:
        best = torch.argmax(vals.view(-1), dim=0)
        return cands[best], vals[best]
    return cands, vals


def optimize_acqf(acq_function, bounds, q, num_restarts, raw_samples=None, options=None,
                  inequality_constraints=None, equality_constraints=None,
                  nonlinear_inequality_constraints=None, fixed_features=None,
                  post_processing_func=None, batch_initial_conditions=None,
                  return_best_only=True, gen_candidates=None, sequential=False, *,
                  ic_generator=None, timeout_sec=None, return_full_tree=False,
                  retry_on_optimization_warning=True, **ic_gen_kwargs):
    """optim/optimize.py:397-564: the all-fixed shortcut (:140-159), sequential
    greedy q (:202-243) or the joint batch (:246-394) -- raw-sample
    initialisation, batch_limit chunks through ``gen_candidates`` (default
    gen_candidates_scipy; gen_candidates_device is the device-resident one)
    with fixed features and the timeout split over the chunks, one retry on
    OptimizationWarning, post-processing, argmax over restarts.

    Linear (in)equality constraints take the reference's route: polytope raw
    samples (hit-and-run) for the initial conditions and SLSQP in
    gen_candidates_scipy (the device L-BFGS-B refuses them).  Nonlinear
    constraints raise UnsupportedError (out of scope); every other argument has
    the reference's meaning.  ``return_full_tree`` only matters for one-shot
    acquisitions, which are not on this path."""
    return optimize_acqf_driver(
        _optimize_acqf_batch, acq_function, bounds, q, num_restarts, raw_samples, options,
        inequality_constraints, equality_constraints, nonlinear_inequality_constraints,
        fixed_features, post_processing_func, batch_initial_conditions, return_best_only,
        gen_candidates, sequential, ic_generator=ic_generator, timeout_sec=timeout_sec,
        return_full_tree=return_full_tree,
        retry_on_optimization_warning=retry_on_optimization_warning, **ic_gen_kwargs)


def optimize_acqf_driver(batch_fn, acq_function, bounds, q, num_restarts, raw_samples=None,
                         options=None, inequality_constraints=None, equality_constraints=None,
                         nonlinear_inequality_constraints=None, fixed_features=None,
                         post_processing_func=None, batch_initial_conditions=None,
                         return_best_only=True, gen_candidates=None, sequential=False, *,
                         ic_generator=None, timeout_sec=None, return_full_tree=False,
                         retry_on_optimization_warning=True, **ic_gen_kwargs):
    """optimize_acqf's control flow (optimize.py:397-564) around the joint
    batch problem ``batch_fn`` (_optimize_acqf_batch here, its restart-sharded
    twin in distributed.py): input validation, the all-fixed shortcut, the
    sequential greedy loop over q."""
    from .exceptions import UnsupportedError
    _reject_constraints(None, None, nonlinear_inequality_constraints, "optimize_acqf")
    gen_candidates = gen_candidates or gen_candidates_scipy
    _validate_optimize_inputs(bounds, raw_samples, batch_initial_conditions, ic_generator,
                              inequality_constraints)
    if fixed_features is not None and len(fixed_features) == bounds.shape[-1]:
        X = torch.tensor([fixed_features[i] for i in range(bounds.shape[-1])],
                         device=bounds.device, dtype=bounds.dtype)
        X = X.expand(q, *X.shape)
        with torch.no_grad():
            return X, acq_function(X)
    args = dict(acq_function=acq_function, bounds=bounds, q=q, num_restarts=num_restarts,
                raw_samples=raw_samples, options=options, fixed_features=fixed_features,
                post_processing_func=post_processing_func,
                batch_initial_conditions=batch_initial_conditions,
                return_best_only=return_best_only, gen_candidates=gen_candidates,
                ic_generator=ic_generator, timeout_sec=timeout_sec,
                retry_on_optimization_warning=retry_on_optimization_warning,
                ic_gen_kwargs=ic_gen_kwargs, inequality_constraints=inequality_constraints,
                equality_constraints=equality_constraints)
    if not (sequential and q > 1):
        return batch_fn(**args)
    # _validate_sequential_inputs (optimize.py:162-199), then q greedy picks
    for group, kind in ((inequality_constraints, "inequality"), (equality_constraints, "equality")):
        if any(len(c[0].shape) > 1 for c in group or []):
            raise UnsupportedError(f"Linear {kind} constraints across the q-dimension are not "
                                   "supported for sequential optimization.")
    if batch_initial_conditions is not None:
        raise UnsupportedError("`batch_initial_conditions` is not supported for sequential "
                               "optimization. Either avoid specifying `batch_initial_conditions` "
                               "to use the custom initializer or use the `ic_generator` kwarg to "
                               "generate initial conditions for the case of nonlinear inequality "
                               "constraints.")
    if not return_best_only:
        raise NotImplementedError("`return_best_only=False` only supported for joint optimization.")
    args.update(q=1, batch_initial_conditions=None, return_best_only=True,
                timeout_sec=timeout_sec / q if timeout_sec is not None else None)
    base_pending = acq_function.X_pending
    picks, values = [], []
    for _ in range(q):
        c, v = batch_fn(**args)
        picks.append(c)
        values.append(v)
        cands = torch.cat(picks, dim=-2)
        acq_function.set_X_pending(torch.cat([base_pending, cands], dim=-2)
                                   if base_pending is not None else cands)
    acq_function.set_X_pending(base_pending)
    return cands, torch.stack(values)
