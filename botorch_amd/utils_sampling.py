"""Quasi-random design helpers (botorch/utils/sampling.py:40-137)."""
from __future__ import annotations

from contextlib import contextmanager
from typing import Optional

import torch
from torch.quasirandom import SobolEngine


@contextmanager
def manual_seed(seed: Optional[int] = None):
    """botorch/utils/sampling.py:40-63."""
    old = torch.random.get_rng_state()
    try:
        if seed is not None:
            torch.random.manual_seed(seed)
        yield
    finally:
        if seed is not None:
            torch.random.set_rng_state(old)


def draw_sobol_samples(bounds: torch.Tensor, n: int, q: int, batch_shape=None,
                       seed: Optional[int] = None) -> torch.Tensor:
    """n x (batch_shape) x q x d scrambled-Sobol points in the box
    (botorch/utils/sampling.py:66-105).  Drawn on the host (as the reference
    does) -- these are the raw-sample designs, not the hot path."""
    batch_shape = torch.Size(batch_shape or [])
    batch_size = int(torch.prod(torch.tensor(batch_shape))) if len(batch_shape) else 1
    d = bounds.shape[-1]
    lower = bounds[0]
    rng = bounds[1] - bounds[0]
    eng = SobolEngine(q * d, scramble=True, seed=seed)
    raw = eng.draw(batch_size * n, dtype=lower.dtype)
    raw = raw.view(*batch_shape, n, q, d).to(device=lower.device)
    if len(batch_shape):
        raw = raw.permute(-3, *range(len(batch_shape)), -2, -1)
    return lower + rng * raw
