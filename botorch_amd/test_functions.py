"""Synthetic problems that generate the configs' training data.

Hartmann: botorch/test_functions/synthetic.py:359-455; DTLZ2:
botorch/test_functions/multi_objective.py:420-450.  The constants are stored
as float32 and promoted, exactly as the reference's registered buffers are
(``torch.tensor([...])`` then ``self.to(dtype=X.dtype)``), so values agree
bit-for-bit with the golden fixtures.
"""
from __future__ import annotations

import math

import torch

_H6_A = [[10, 3, 17, 3.5, 1.7, 8], [0.05, 10, 17, 0.1, 8, 14],
         [3, 3.5, 1.7, 10, 17, 8], [17, 8, 0.05, 10, 0.1, 14]]
_H6_P = [[1312, 1696, 5569, 124, 8283, 5886], [2329, 4135, 8307, 3736, 1004, 9991],
         [2348, 1451, 3522, 2883, 3047, 6650], [4047, 8828, 8732, 5743, 1091, 381.0]]
_H_ALPHA = [1.0, 1.2, 3.0, 3.2]


class Hartmann:
    """Hartmann-6: H(x) = -sum_i ALPHA_i exp(-sum_j A_ij (x_j - 1e-4 P_ij)^2)."""

    def __init__(self, dim: int = 6, noise_std=None, negate: bool = False):
        if dim != 6:
            raise ValueError("only the 6-dimensional Hartmann function is provided")
        self.dim = dim
        self.noise_std = noise_std
        self.negate = negate
        self.bounds = torch.tensor([[0.0] * dim, [1.0] * dim])
        self._optimal_value = -3.32237

    def evaluate_true(self, X: torch.Tensor) -> torch.Tensor:
        A = torch.tensor(_H6_A).to(X)
        P = torch.tensor(_H6_P).to(X)
        alpha = torch.tensor(_H_ALPHA).to(X)
        inner = torch.sum(A * (X.unsqueeze(-2) - 0.0001 * P).pow(2), dim=-1)
        return -(torch.sum(alpha * torch.exp(-inner), dim=-1))

    def __call__(self, X: torch.Tensor, noise: bool = True) -> torch.Tensor:
        batch = X.ndimension() > 1
        X = X if batch else X.unsqueeze(0)
        f = self.evaluate_true(X)
        if noise and self.noise_std is not None:
            f = f + self.noise_std * torch.randn_like(f)
        if self.negate:
            f = -f
        return f if batch else f.squeeze(0)


class DTLZ2:
    """DTLZ2 (minimisation problem; negate=True for maximisation)."""

    _ref_val = 1.1

    def __init__(self, dim: int, num_objectives: int = 2, noise_std=None, negate: bool = False):
        if dim <= num_objectives:
            raise ValueError(f"dim must be > num_objectives, got {dim} and {num_objectives}")
        self.dim = dim
        self.num_objectives = num_objectives
        self.k = dim - num_objectives + 1
        self.noise_std = noise_std
        self.negate = negate
        self.bounds = torch.tensor([[0.0] * dim, [1.0] * dim])
        self.ref_point = torch.full((num_objectives,), self._ref_val)
        if negate:
            self.ref_point = -self.ref_point

    def evaluate_true(self, X: torch.Tensor) -> torch.Tensor:
        X_m = X[..., -self.k:]
        g_plus1 = 1 + (X_m - 0.5).pow(2).sum(dim=-1)
        fs = []
        half_pi = math.pi / 2
        for i in range(self.num_objectives):
            idx = self.num_objectives - 1 - i
            f_i = g_plus1.clone()
            f_i *= torch.cos(X[..., :idx] * half_pi).prod(dim=-1)
            if i > 0:
                f_i *= torch.sin(X[..., idx] * half_pi)
            fs.append(f_i)
        return torch.stack(fs, dim=-1)

    def __call__(self, X: torch.Tensor, noise: bool = True) -> torch.Tensor:
        f = self.evaluate_true(X)
        if noise and self.noise_std is not None:
            f = f + self.noise_std * torch.randn_like(f)
        return -f if self.negate else f
