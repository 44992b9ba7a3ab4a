"""MC samplers with BoTorch's interface (botorch/sampling/base.py, normal.py).

SobolQMCNormalSampler generates its base samples on the GPU
(``bo_sobol_normal``) from the scrambled direction numbers of the same
torch SobolEngine(dim, scramble=True, seed) the reference draws from; the
points agree bit for bit in u and to ~1 ulp in z (tests/test_gpu_kernels.py).
"""
from __future__ import annotations

from typing import Optional

import torch
from torch import nn

from . import kernels
from .exceptions import InputDataError, UnsupportedError
from .utils_sampling import manual_seed

SOBOL_MAXDIM = 21201  # torch.quasirandom.SobolEngine.MAXDIM


class MCSampler(nn.Module):
    """sampling/base.py:33-114."""

    def __init__(self, sample_shape: torch.Size, seed: Optional[int] = None):
        super().__init__()
        if not isinstance(sample_shape, torch.Size):
            raise InputDataError(f"Expected `sample_shape` to be a `torch.Size` object, got {sample_shape}.")
        self.sample_shape = sample_shape
        self.seed = seed if seed is not None else torch.randint(0, 1000000, (1,)).item()
        self.register_buffer("base_samples", None)

    def _get_batch_range(self, posterior):
        return getattr(self, "batch_range_override", posterior.batch_range)

    def _get_collapsed_shape(self, posterior) -> torch.Size:
        bss = posterior.base_sample_shape
        b0, b1 = self._get_batch_range(posterior)
        b1 = len(bss) + b1 if b1 <= 0 else b1
        return self.sample_shape + bss[:b0] + torch.Size([1] * (b1 - b0)) + bss[b1:]

    def _get_extended_base_sample_shape(self, posterior) -> torch.Size:
        return self.sample_shape + posterior.base_sample_shape

    def forward(self, posterior):
        self._construct_base_samples(posterior)
        return posterior.rsample_from_base_samples(
            self.sample_shape,
            self.base_samples.expand(self._get_extended_base_sample_shape(posterior)))


class SobolQMCNormalSampler(MCSampler):
    """sampling/normal.py:169-209."""

    def _construct_base_samples(self, posterior) -> None:
        target = self._get_collapsed_shape(posterior)
        if self.base_samples is None or self.base_samples.shape != target:
            dim = target[len(self.sample_shape):].numel()
            if dim > SOBOL_MAXDIM:
                raise UnsupportedError(
                    f"SobolQMCSampler only supports dimensions `q * o <= {SOBOL_MAXDIM}`. Requested: {dim}")
            Z = kernels.sobol_normal(dim, self.sample_shape.numel(), self.seed, posterior.device)
            self.register_buffer("base_samples", Z.view(target))

    def base_samples_2d(self, dim: int, device) -> torch.Tensor:
        """S x dim base samples (shape-keyed cache) for the fused acquisition path,
        identical to what _construct_base_samples produces for a single-output
        posterior of `dim` points."""
        target = self.sample_shape + torch.Size([1, dim])
        if self.base_samples is None or self.base_samples.shape != target:
            Z = kernels.sobol_normal(dim, self.sample_shape.numel(), self.seed, device)
            self.register_buffer("base_samples", Z.view(target))
        return self.base_samples.reshape(-1, dim)


class IIDNormalSampler(MCSampler):
    """sampling/normal.py:137-166 (torch.randn under manual_seed, on the device)."""

    def _construct_base_samples(self, posterior) -> None:
        target = self._get_collapsed_shape(posterior)
        if self.base_samples is None or self.base_samples.shape != target:
            with manual_seed(self.seed):
                Z = torch.randn(target, device=posterior.device, dtype=posterior.dtype)
            self.register_buffer("base_samples", Z)

    def base_samples_2d(self, dim: int, device) -> torch.Tensor:
        target = self.sample_shape + torch.Size([1, dim])
        if self.base_samples is None or self.base_samples.shape != target:
            with manual_seed(self.seed):
                Z = torch.randn(target, device=device, dtype=torch.float64)
            self.register_buffer("base_samples", Z)
        return self.base_samples.reshape(-1, dim)


def get_sampler(posterior=None, sample_shape: torch.Size = torch.Size([512]),
                seed: Optional[int] = None) -> MCSampler:
    """sampling/get_sampler.py:70-90 for Gaussian posteriors."""
    return SobolQMCNormalSampler(sample_shape=sample_shape, seed=seed)
