"""Multi-GPU sharding of the candidate batch (one process per GPU).

The reference optimises all ``num_restarts`` starting points of
``optimize_acqf`` (optim/optimize.py:246-394) jointly on one device and then
takes ``argmax`` over restarts.  Restarts are independent L-BFGS-B problems
(gen_candidates_scipy sums their acquisition values, so their gradients never
mix), so the batch partitions across ranks with no data-path exchange:

* rank r draws its own ``raw_samples / W`` Sobol raw points (seed + r),
  picks ``num_restarts / W`` starting points from them with the same
  Boltzmann rule as ``initialize_q_batch`` (optim/initializers.py:1116-1190),
  and runs the local optimisation on its own GPU;
* the only collective is ONE all-gather of a packed ``[value, candidate]``
  row per rank at the end (the "argmax/gather" of the north star), after
  which every rank holds the global best candidate.

With W = 1 this is exactly :func:`botorch_amd.optim.optimize_acqf`.
Process groups come from ``torch.distributed`` (``nccl`` = RCCL over xGMI on
the GPU node, ``gloo`` in the CPU tests).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.distributed as dist

from .optim import optimize_acqf


def world() -> Tuple[int, int]:
    """(world_size, rank) of the default group, (1, 0) when not initialised."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(), dist.get_rank()
    return 1, 0


def shard_range(total: int, world_size: int, rank: int) -> Tuple[int, int]:
    """Contiguous [start, stop) of ``total`` units owned by ``rank`` (the first
    ``total % world_size`` ranks get one extra)."""
    if world_size < 1 or not 0 <= rank < world_size:
        raise ValueError(f"bad rank {rank} for world size {world_size}")
    base, extra = divmod(total, world_size)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def gather_argmax(value: torch.Tensor, candidate: torch.Tensor, group=None
                  ) -> Tuple[torch.Tensor, torch.Tensor, int]:
    """Global argmax of per-rank (value, candidate) with ONE all-gather.

    ``value`` is a scalar, ``candidate`` any shape (identical across ranks).
    Returns (best_candidate, best_value, owner_rank) on every rank; ties go to
    the lowest rank, as ``torch.argmax`` over the concatenated restarts would.
    """
    ws = dist.get_world_size(group) if dist.is_initialized() else 1
    if ws == 1:
        return candidate, value.reshape(()), 0
    packed = torch.cat([value.reshape(1).to(torch.float64),
                        candidate.reshape(-1).to(torch.float64)])
    rows = [torch.empty_like(packed) for _ in range(ws)]
    dist.all_gather(rows, packed, group=group)
    table = torch.stack(rows)
    owner = int(torch.argmax(table[:, 0]).item())
    best = table[owner]
    return (best[1:].reshape(candidate.shape).to(candidate.dtype), best[0].to(value.dtype), owner)


def optimize_acqf_sharded(acq_function, bounds, q: int, num_restarts: int,
                          raw_samples: Optional[int] = None, options=None, group=None,
                          **kwargs):
    """``optimize_acqf`` with restarts and raw samples partitioned over the
    ranks of ``group``; returns the global (candidate q x d, value) on every rank.

    Each rank must hold the same model / acquisition function (they are
    replicated: the caches are O(n^2) and built once per rank)."""
    ws = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    if num_restarts < ws:
        raise ValueError(f"num_restarts={num_restarts} < world size {ws}")
    options = dict(options or {})
    r0, r1 = shard_range(num_restarts, ws, rank)
    raw_local = None
    if raw_samples is not None:
        s0, s1 = shard_range(raw_samples, ws, rank)
        raw_local = max(s1 - s0, r1 - r0)
    if options.get("seed") is not None:
        options["seed"] = int(options["seed"]) + rank
    cand, val = optimize_acqf(acq_function, bounds, q, r1 - r0, raw_local, options=options,
                              **kwargs)
    best, best_val, _ = gather_argmax(val, cand, group)
    return best, best_val
