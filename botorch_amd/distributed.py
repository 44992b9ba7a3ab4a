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

W ranks reproduce one process bit for bit when the single process runs the
same chunks: ``init_batch_limit = raw / W`` and ``batch_limit =
num_restarts / W`` (each scipy L-BFGS-B run is over one chunk, so the chunk
boundaries are part of the reference's semantics).

Process groups come from ``torch.distributed`` (``nccl`` = RCCL over xGMI on
the GPU node, ``gloo`` in the CPU tests); buffers live on the acquisition's
device, so RCCL moves device memory.
"""
from __future__ import annotations

import warnings
from typing import Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from .optim import (BadInitialCandidatesWarning, draw_raw_samples, evaluate_raw_samples,
                    gen_candidates_scipy, generate_in_chunks, init_options, select_initial_indices)


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


def gen_batch_initial_conditions_sharded(acq_function, bounds, q, num_restarts, raw_samples,
                                         options=None, group=None):
    """gen_batch_initial_conditions (initializers.py:243-438) with the raw-sample
    evaluation sharded over the ranks; returns all ``num_restarts`` initial
    conditions (identical on every rank)."""
    ws, rank = world(group)
    seed, batch_limit, init_func, init_kwargs = init_options(acq_function, bounds, options)
    dev = bounds.device
    if seed is None and ws > 1:   # one seed for the global draw: rank 0's
        s = torch.randint(0, 2 ** 31 - 1, (1,), dtype=torch.int64).to(dev)
        seed = int(_broadcast_from_rank0(s, group).item())
    q = 1 if q is None else q
    factor, max_factor = 1, 5
    while factor < max_factor:
        n = raw_samples * factor
        X_rnd = draw_raw_samples(bounds, n, q, seed)
        s0, s1 = shard_range(n, ws, rank)
        y = evaluate_raw_samples(acq_function, X_rnd[s0:s1].to(dev), batch_limit)
        Y_rnd = allgather_rows(y.to(torch.float64), n, group)
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


def optimize_acqf_sharded(acq_function, bounds, q: int, num_restarts: int,
                          raw_samples: Optional[int] = None, options=None, group=None,
                          batch_initial_conditions=None, return_best_only: bool = True,
                          gen_candidates=None, retry_on_optimization_warning: bool = True,
                          **kwargs):
    """``optimize_acqf`` (optimize.py:397-543) with the raw samples and the
    restarts partitioned over the ranks of ``group``; returns the global
    (candidate q x d, value) -- or all restarts with ``return_best_only=False``
    -- on every rank.  Each rank holds the same replicated model and
    acquisition function (its caches are built locally)."""
    ws, rank = world(group)
    options = dict(options or {})
    gen_candidates = gen_candidates or gen_candidates_scipy
    if batch_initial_conditions is None:
        if raw_samples is None:
            raise ValueError("Must specify `raw_samples` when `batch_initial_conditions` is None`.")
        batch_initial_conditions = gen_batch_initial_conditions_sharded(
            acq_function, bounds, q, num_restarts, raw_samples, options=options, group=group)
    b = batch_initial_conditions.shape[0]
    batch_limit = options.get("batch_limit", b)
    r0, r1 = shard_range(b, ws, rank)

    def _run(ics):
        c, v, warned = generate_in_chunks(acq_function, ics[r0:r1], bounds, batch_limit, options,
                                          gen_candidates)
        flag = torch.tensor([float(bool(warned))], dtype=torch.float64, device=ics.device)
        if ws > 1:
            dist.all_reduce(flag, op=dist.ReduceOp.MAX, group=group)
        return c, v, bool(flag.item())

    cands, vals, warned = _run(batch_initial_conditions)
    if retry_on_optimization_warning and warned:
        new_ics = gen_batch_initial_conditions_sharded(acq_function, bounds, q, num_restarts,
                                                       raw_samples or num_restarts, options=options,
                                                       group=group)
        cands, vals, warned = _run(new_ics)
    shape = batch_initial_conditions.shape[1:]
    rows = torch.cat([vals.reshape(-1, 1).to(torch.float64),
                      cands.reshape(vals.numel(), -1).to(torch.float64)], dim=1)
    table = allgather_rows(rows.to(batch_initial_conditions.device), b, group)
    all_vals = table[:, 0].to(vals.dtype)
    all_cands = table[:, 1:].reshape(b, *shape).to(batch_initial_conditions.dtype)
    if return_best_only:
        best = torch.argmax(all_vals, dim=0)
        return all_cands[best], all_vals[best]
    return all_cands, all_vals


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
    msg = torch.zeros(1 + sum(sizes), dtype=torch.float64)
    err = None
    if rank == 0:
        try:
            fit(mll, **kwargs)
            msg[0] = 1.0
            msg[1:] = torch.from_numpy(np.concatenate([lay.get() for lay in layouts]))
        except ModelFittingError as e:
            err = e
    msg = _broadcast_from_rank0(msg.to(dev), group).cpu()
    if not bool(msg[0]):
        if err is not None:
            raise err
        mll.train()
        raise ModelFittingError("All attempts to fit the model have failed (rank 0 of the "
                                "replicated fit).")
    if rank != 0:
        off = 1
        for lay, k in zip(layouts, sizes):
            lay.set(msg[off:off + k].numpy().astype(np.float64))
            off += k
    return mll.eval()
