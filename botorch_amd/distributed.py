"""Multi-GPU sharding of optimize_acqf's candidate batch (one process per GPU).

The reference evaluates all ``raw_samples`` designs, picks ``num_restarts``
starting points from the whole set (optim/initializers.py:411-426), optimises
them in ``batch_limit`` chunks (optim/optimize.py:335-365) and takes one argmax
over all restarts (:384-387).  The sharded version keeps every one of those
decisions global, so W ranks return what one process returns:

* every rank draws the same global raw designs (the seeded Sobol draw is
  deterministic; an unseeded call takes rank 0's seed) and evaluates the
  contiguous slice ``shard_range(raw, W, rank)`` of them;
* one all-reduce(SUM) of a zeroed length-``raw`` buffer, each rank writing its
  slice, gives every rank all raw values;
* rank 0 runs the Boltzmann selection on the host values from its global CPU
  generator -- the reference's own call -- and broadcasts the picked indices;
* each rank optimises the contiguous restart slice ``shard_range(num_restarts,
  W, rank)`` in ``batch_limit`` chunks;
* one all-reduce(SUM) of a zeroed ``num_restarts x (1 + q d)`` buffer of
  ``[value, candidate]`` rows gives every rank all restarts; the argmax over
  them is the reference's (ties to the lowest restart index).

Every option of ``optimize_acqf`` keeps its meaning (the control flow is
optim.optimize_acqf_driver, shared with the single process): fixed features,
linear constraints (polytope raw samples, SLSQP), ``post_processing_func``,
``timeout_sec``, ``sequential``, ``ic_generator``.

W ranks reproduce one process bit for bit when the single process runs the
same chunks: ``init_batch_limit = raw / W`` and ``batch_limit =
num_restarts / W`` (each scipy L-BFGS-B run is over one chunk, so the chunk
boundaries are part of the reference's semantics).

Process groups come from ``torch.distributed`` (``nccl`` = RCCL over xGMI on
the GPU node, ``gloo`` in the CPU tests); buffers live on the acquisition's
device, so RCCL moves device memory.
"""
from __future__ import annotations

import functools
import warnings
from typing import Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from .optim import (BadInitialCandidatesWarning, _check_deferred, check_init_inputs,
                    evaluate_raw_samples, generate_in_chunks, init_options, optimize_acqf_driver,
                    raw_designs, raw_designs_use_global_rng, select_initial_indices)


def world(group=None) -> Tuple[int, int]:
    """(world_size, rank) of ``group``, (1, 0) when not initialised."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def shard_range(total: int, world_size: int, rank: int) -> Tuple[int, int]:
    """Contiguous [start, stop) of ``total`` units owned by ``rank`` (the first
    ``total % world_size`` ranks get one extra)."""
    if world_size < 1 or not 0 <= rank < world_size:
        raise ValueError(f"bad rank {rank} for world size {world_size}")
    base, extra = divmod(total, world_size)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def allgather_rows(local: torch.Tensor, total: int, group=None) -> torch.Tensor:
    """Rows [start, stop) of a ``total``-row table from each rank -> the whole
    table on every rank, with ONE all-reduce(SUM) of a zeroed buffer (adding
    zeros is exact in fp64)."""
    ws, rank = world(group)
    s0, s1 = shard_range(total, ws, rank)
    if local.shape[0] != s1 - s0:
        raise ValueError(f"rank {rank} holds {local.shape[0]} rows, owns {s1 - s0}")
    if ws == 1:
        return local
    buf = local.new_zeros((total,) + tuple(local.shape[1:]))
    buf[s0:s1] = local
    dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=group)
    return buf


def _broadcast_from_rank0(t: torch.Tensor, group=None) -> torch.Tensor:
    if world(group)[0] > 1:
        dist.broadcast(t, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
    return t


def gather_argmax(value: torch.Tensor, candidate: torch.Tensor, group=None
                  ) -> Tuple[torch.Tensor, torch.Tensor, int]:
    """Global argmax of one (value, candidate) per rank with one all-reduce;
    ties go to the lowest rank, as ``torch.argmax`` over the concatenation."""
    ws, rank = world(group)
    if ws == 1:
        return candidate, value.reshape(()), 0
    row = torch.cat([value.reshape(1).to(torch.float64), candidate.reshape(-1).to(torch.float64)])
    table = torch.zeros(ws, row.numel(), dtype=torch.float64, device=row.device)
    table[rank] = row
    dist.all_reduce(table, op=dist.ReduceOp.SUM, group=group)
    owner = int(torch.argmax(table[:, 0]).item())
    best = table[owner]
    return best[1:].reshape(candidate.shape).to(candidate.dtype), best[0].to(value.dtype), owner


def _broadcast_tensor_from_rank0(t: Optional[torch.Tensor], group, dtype, device) -> torch.Tensor:
    """A tensor of any shape that only rank 0 holds -> every rank (its shape
    first, then its data)."""
    ws, rank = world(group)
    if ws == 1:
        return t
    hdr = torch.zeros(9, dtype=torch.int64, device=device)
    if rank == 0:
        hdr[0] = t.dim()
        hdr[1:1 + t.dim()] = torch.tensor(t.shape, dtype=torch.int64)
    hdr = _broadcast_from_rank0(hdr, group).cpu()
    shape = tuple(int(v) for v in hdr[1:1 + int(hdr[0])])
    buf = t.to(device=device, dtype=dtype).contiguous() if rank == 0 else \
        torch.empty(shape, dtype=dtype, device=device)
    return _broadcast_from_rank0(buf, group)


def gen_batch_initial_conditions_sharded(acq_function, bounds, q, num_restarts, raw_samples,
                                         fixed_features=None, options=None,
                                         inequality_constraints=None, equality_constraints=None,
                                         generator=None, fixed_X_fantasies=None, group=None):
    """gen_batch_initial_conditions (initializers.py:243-438) with the raw-sample
    evaluation sharded over the ranks; returns all ``num_restarts`` initial
    conditions (identical on every rank).  Every option of the single-process
    initialiser applies (optim.raw_designs: fixed features, the polytope
    q-batches under linear constraints, a caller's ``generator``, points
    around the incumbents, ``fixed_X_fantasies``).  The seeded Sobol and
    polytope draws are replicated on every rank; a draw from the global
    generator (``sample_around_best``, a ``generator``) is made on rank 0 and
    broadcast, so the designs are rank 0's -- one process's."""
    ws, rank = world(group)
    options = options or {}
    check_init_inputs(bounds, options, equality_constraints, generator)
    seed, batch_limit, init_func, init_kwargs = init_options(acq_function, bounds, options)
    dev = bounds.device
    if seed is None and ws > 1:   # one seed for the global draw: rank 0's
        s = torch.randint(0, 2 ** 31 - 1, (1,), dtype=torch.int64).to(dev)
        seed = int(_broadcast_from_rank0(s, group).item())
    q = 1 if q is None else q
    factor, max_factor = 1, 5
    while factor < max_factor:
        n = raw_samples * factor
        if ws > 1 and raw_designs_use_global_rng(options, seed, generator,
                                                 inequality_constraints or equality_constraints):
            X_rnd = raw_designs(acq_function, bounds, q, n, seed, options, fixed_features,
                                inequality_constraints, equality_constraints, generator,
                                fixed_X_fantasies) if rank == 0 else None
            X_rnd = _broadcast_tensor_from_rank0(X_rnd, group, bounds.dtype, dev)
        else:
            X_rnd = raw_designs(acq_function, bounds, q, n, seed, options, fixed_features,
                                inequality_constraints, equality_constraints, generator,
                                fixed_X_fantasies)
        n_all = X_rnd.shape[0]            # n, or 2n with the points around the incumbents
        s0, s1 = shard_range(n_all, ws, rank)
        y = evaluate_raw_samples(acq_function, X_rnd[s0:s1].to(dev), batch_limit)
        Y_rnd = allgather_rows(y.to(torch.float64), n_all, group)
        # [warned, picks...] from rank 0's selection
        msg = torch.zeros(1 + num_restarts, dtype=torch.int64)
        if rank == 0:
            idx, warned = select_initial_indices(init_func, Y_rnd, num_restarts, init_kwargs)
            msg[0] = int(warned)
            msg[1:] = idx
        msg = _broadcast_from_rank0(msg.to(Y_rnd.device), group).cpu()
        ics = X_rnd[msg[1:].to(X_rnd.device)].to(dev)
        if not bool(msg[0]):
            return ics
        if factor < max_factor:
            factor += 1
            if seed is not None:
                seed += 1
    warnings.warn("Unable to find non-zero acquisition function values - initial conditions "
                  "are being selected randomly.", BadInitialCandidatesWarning)
    return ics


def _optimize_acqf_batch_sharded(acq_function, bounds, q, num_restarts, raw_samples, options,
                                 fixed_features, post_processing_func, batch_initial_conditions,
                                 return_best_only, gen_candidates, ic_generator, timeout_sec,
                                 retry_on_optimization_warning, ic_gen_kwargs,
                                 inequality_constraints=None, equality_constraints=None,
                                 group=None):
    """optim._optimize_acqf_batch (optimize.py:246-394) with the restarts
    partitioned over the ranks: each rank runs the batch_limit chunks of its
    contiguous restart slice (fixed features, linear constraints and its share
    of ``timeout_sec`` passed to ``gen_candidates`` exactly as one process
    passes them to each chunk), the retry on OptimizationWarning is decided
    globally (all-reduce MAX of the ranks' flags), one all-reduce gathers every
    restart's [value, candidate], and ``post_processing_func`` + the
    re-evaluation run on the whole gathered batch on every rank (as one
    process runs them)."""
    ws, rank = world(group)
    options = options or {}
    provided = batch_initial_conditions is not None
    dev = bounds.device

    def _ics():
        kw = dict(acq_function=acq_function, bounds=bounds, q=q, num_restarts=num_restarts,
                  raw_samples=raw_samples, fixed_features=fixed_features, options=options,
                  inequality_constraints=inequality_constraints,
                  equality_constraints=equality_constraints, **ic_gen_kwargs)
        if ic_generator is None:
            return gen_batch_initial_conditions_sharded(group=group, **kw)
        # a caller's initial-condition generator runs once, on rank 0; its
        # initial conditions are broadcast
        ics = ic_generator(**kw) if rank == 0 else None
        return _broadcast_tensor_from_rank0(ics, group, bounds.dtype, dev)

    ics = batch_initial_conditions if provided else _ics()
    b = ics.shape[0]
    batch_limit = options.get("batch_limit", num_restarts)
    linear = {k: v for k, v in (("inequality_constraints", inequality_constraints),
                                ("equality_constraints", equality_constraints)) if v is not None}

    def _run(x0):
        r0, r1 = shard_range(x0.shape[0], ws, rank)
        # one process gives each of its ceil(b / batch_limit) chunks
        # timeout_sec / chunks; this rank's chunks get the same share each
        n_all = -(-x0.shape[0] // max(1, batch_limit))
        n_mine = -(-(r1 - r0) // max(1, batch_limit))
        t_mine = timeout_sec * n_mine / n_all if timeout_sec is not None and n_all else None
        c, v, w = generate_in_chunks(acq_function, x0[r0:r1], bounds, batch_limit, options,
                                     gen_candidates, fixed_features=fixed_features,
                                     timeout_sec=t_mine, **linear)
        flag = torch.tensor([float(bool(w))], dtype=torch.float64, device=x0.device)
        if ws > 1:
            dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
        return c, v, w, bool(flag.item())

    cands, vals, ws_local, warned = _run(ics)
    if warned and retry_on_optimization_warning:
        msgs = [str(w.message) for w in ws_local]
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
            ics = _ics()
            cands, vals, ws_local, warned = _run(ics)
            if warned:
                warnings.warn("Optimization failed on the second try, after generating a new set "
                              "of initial conditions.", RuntimeWarning)
    b = ics.shape[0]
    shape = tuple(ics.shape[1:])
    width = 1 + int(np.prod(shape))
    rows = torch.cat([vals.reshape(-1, 1).to(torch.float64),
                      cands.reshape(vals.numel(), width - 1).to(torch.float64)], dim=1) \
        if vals.numel() else torch.zeros(0, width, dtype=torch.float64, device=ics.device)
    table = allgather_rows(rows.to(ics.device), b, group)
    all_vals = table[:, 0].to(vals.dtype)
    all_cands = table[:, 1:].reshape(b, *shape).to(ics.dtype)
    if post_processing_func is not None:
        all_cands = post_processing_func(all_cands)
        with torch.no_grad():
            all_vals = torch.cat([acq_function(c) for c in all_cands.split(batch_limit, dim=0)],
                                 dim=0)
    _check_deferred(all_cands)
    if return_best_only:
        best = torch.argmax(all_vals.view(-1), dim=0)
        return all_cands[best], all_vals[best]
    return all_cands, all_vals


def optimize_acqf_sharded(acq_function, bounds, q: int, num_restarts: int,
                          raw_samples: Optional[int] = None, options=None,
                          inequality_constraints=None, equality_constraints=None,
                          nonlinear_inequality_constraints=None, fixed_features=None,
                          post_processing_func=None, batch_initial_conditions=None,
                          return_best_only: bool = True, gen_candidates=None,
                          sequential: bool = False, *, ic_generator=None, timeout_sec=None,
                          return_full_tree: bool = False,
                          retry_on_optimization_warning: bool = True, group=None,
                          **ic_gen_kwargs):
    """``optimize_acqf`` (optimize.py:397-543) with the raw samples and the
    restarts partitioned over the ranks of ``group``; returns the global
    (candidate q x d, value) -- or all restarts with ``return_best_only=False``
    -- on every rank.  Each rank holds the same replicated model and
    acquisition function (its caches are built locally).

    Every argument of optim.optimize_acqf has its meaning there (the same
    control flow, optim.optimize_acqf_driver): fixed features, linear
    (in)equality constraints (polytope raw samples, SLSQP in
    gen_candidates_scipy), ``post_processing_func``, ``timeout_sec``,
    ``sequential`` greedy q (each pick a sharded batch problem, pending points
    set on every rank's replica), ``ic_generator`` (run on rank 0, its initial
    conditions broadcast), the all-fixed shortcut; nonlinear constraints raise
    UnsupportedError as in the single process."""
    batch_fn = functools.partial(_optimize_acqf_batch_sharded, group=group)
    return optimize_acqf_driver(
        batch_fn, acq_function, bounds, q, num_restarts, raw_samples, options,
        inequality_constraints, equality_constraints, nonlinear_inequality_constraints,
        fixed_features, post_processing_func, batch_initial_conditions, return_best_only,
        gen_candidates, sequential, ic_generator=ic_generator, timeout_sec=timeout_sec,
        return_full_tree=return_full_tree,
        retry_on_optimization_warning=retry_on_optimization_warning, **ic_gen_kwargs)


def _fit_layouts(mll):
    """The flat hyperparameter layouts a fit writes: one per exact GP (a
    ModelListGP's SumMarginalLogLikelihood fits its members one by one,
    fit.py:262-283)."""
    from .fit import SumMarginalLogLikelihood, _layout
    if isinstance(mll, SumMarginalLogLikelihood):
        return [_layout(sub.model) for sub in mll.mlls]
    return [_layout(mll.model)]


def fit_gpytorch_mll_replicated(mll, group=None, fit=None, **kwargs):
    """``fit_gpytorch_mll`` (fit.py:75-113) for replicated models (SURVEY.md
    8(e): the GP fit is one O(n^3) problem, so it is not sharded).  Rank 0
    runs the fit -- retries, prior resampling and rollback included -- and
    broadcasts ``[ok, x]``, x the fitted hyperparameter vector in the layout
    order of get_parameters_and_bounds (8 numbers at d = 6); every other rank
    writes x into its own model.  Every rank then holds bit-identical
    hyperparameters and ends in eval mode, and builds its prediction caches
    locally on first use (cheaper than moving L, L^-1: 2 x 134 MB at C3).  A
    ModelFittingError on rank 0 is raised on every rank, with every model left
    at its starting state in train mode (the reference's failure contract).
    ``fit`` replaces the fit routine (default fit.fit_gpytorch_mll)."""
    from .exceptions import ModelFittingError
    from .fit import fit_gpytorch_mll
    fit = fit or fit_gpytorch_mll
    ws, rank = world(group)
    if ws == 1:
        return fit(mll, **kwargs)
    layouts = _fit_layouts(mll)
    sizes = [lay.size for lay in layouts]
    dev = mll.model.train_inputs[0].device if hasattr(mll.model, "train_inputs") else \
        mll.mlls[0].model.train_inputs[0].device
    # msg[0]: 1 fitted, 0 ModelFittingError, -1 any other exception on rank 0.
    # Rank 0 catches everything (BaseException: a kernel's RuntimeError, bad
    # kwargs, KeyboardInterrupt) so that the broadcast every other rank is
    # waiting in always happens -- a distributed job fails instead of hanging.
    msg = torch.zeros(1 + sum(sizes), dtype=torch.float64)
    err = None
    if rank == 0:
        try:
            fit(mll, **kwargs)
            msg[0] = 1.0
            msg[1:] = torch.from_numpy(np.concatenate([lay.get() for lay in layouts]))
        except ModelFittingError as e:
            err = e
        except BaseException as e:  # noqa: B902 -- re-raised below, after the broadcast
            err = e
            msg[0] = -1.0
    msg = _broadcast_from_rank0(msg.to(dev), group).cpu()
    status = float(msg[0])
    if status != 1.0:
        if err is not None:
            raise err
        mll.train()
        if status < 0:
            raise RuntimeError("rank 0's replicated fit raised an exception (see rank 0's "
                               "traceback); the hyperparameters were not broadcast")
        raise ModelFittingError("All attempts to fit the model have failed (rank 0 of the "
                                "replicated fit).")
    if rank != 0:
        off = 1
        for lay, k in zip(layouts, sizes):
            lay.set(msg[off:off + k].numpy().astype(np.float64))
            off += k
    return mll.eval()
