"""CPU restatement of the Sobol QMC base-sample path.

TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).
"""
from __future__ import annotations

import math

import torch
from torch.quasirandom import SobolEngine


def draw_sobol_normal_samples(d: int, n: int, seed: int) -> torch.Tensor:
    """botorch/utils/sampling.py:108-137 -> NormalQMCEngine(d, seed,
    inv_transform=True).draw(n, dtype=float64) (botorch/sampling/qmc.py:60-98):
    v = 1/2 + (1 - eps)(u - 1/2);  z = sqrt(2) erfinv(2v - 1)."""
    eng = SobolEngine(dimension=d, scramble=True, seed=seed)
    u = eng.draw(n, dtype=torch.float64)
    v = 0.5 + (1 - torch.finfo(u.dtype).eps) * (u - 0.5)
    return torch.erfinv(2 * v - 1) * math.sqrt(2)


def draw_sobol_samples(lower, upper, n: int, q: int, seed: int) -> torch.Tensor:
    """botorch/utils/sampling.py:66-105 (no batch_shape): n x q x d."""
    d = lower.shape[-1]
    eng = SobolEngine(q * d, scramble=True, seed=seed)
    raw = eng.draw(n, dtype=lower.dtype).view(n, q, d)
    return lower + (upper - lower) * raw


def base_samples_single_output(S: int, q: int, seed: int) -> torch.Tensor:
    """SobolQMCNormalSampler._construct_base_samples for a single-output
    posterior (botorch/sampling/normal.py:178-209): collapsed shape S x 1 x q,
    Sobol dimension q.  Returned as S x q."""
    return draw_sobol_normal_samples(q, S, seed)


def base_samples_multi_output(S: int, q: int, m: int, seed: int) -> torch.Tensor:
    """Multi-output (non-interleaved MTMVN) base samples as seen by output t at
    point i: Z[s, t, i] = sobol[s, i*m + t]  (Sobol dim q*m; the reshape in
    botorch/posteriors/base_samples.py:16-45 followed by [G]
    MultitaskMultivariateNormal.rsample).  Returned as S x m x q."""
    z = draw_sobol_normal_samples(q * m, S, seed).view(S, q, m)
    return z.transpose(1, 2).contiguous()
