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

    def _reuse_base_samples(self, target: torch.Size) -> bool:
        """Keep the current base samples when ``target`` differs from their shape
        only in collapsed (size-1) batch dimensions: a fresh draw would give the
        same values (same seed, same dimension), and base samples installed by
        _update_base_samples or by the caller are kept."""
        bs = self.base_samples
        if bs is None:
            return False
        if bs.shape == target:
            return True
        strip = lambda sh: [v for v in sh[len(self.sample_shape):] if v != 1]  # noqa: E731
        if bs.shape[: len(self.sample_shape)] == target[: len(self.sample_shape)] \
                and strip(bs.shape) == strip(target) and bs.numel() == target.numel():
            self.register_buffer("base_samples", bs.reshape(target))
            return True
        return False

    def _instance_check(self, base_sampler):
        """sampling/base.py:142-148."""
        if not isinstance(base_sampler, self.__class__):
            raise RuntimeError("Expected `base_sampler` to be an instance of "
                               f"{self.__class__.__name__}. Got {base_sampler}.")

    def _update_base_samples(self, posterior, base_sampler) -> None:
        """sampling/normal.py:68-131 (single-output posteriors): construct the
        base samples of ``posterior`` and overwrite their leading columns with
        ``base_sampler``'s (the cached X_baseline samples), so the joint
        (X_baseline, X) draw reuses them."""
        self._instance_check(base_sampler)
        self._construct_base_samples(posterior)
        if base_sampler.base_samples is not None:
            cur = base_sampler.base_samples.detach().clone()
            nd = cur.dim() - 1
            target = self._get_collapsed_shape(posterior)
            view_shape = (self.sample_shape + torch.Size([1] * (len(target) - cur.dim()))
                          + cur.shape[-nd:])
            expanded = cur.view(view_shape).expand(target[:-nd] + cur.shape[-nd:])
            base = self.base_samples.clone()
            base[..., : cur.shape[-1]] = expanded
            self.register_buffer("base_samples", base)

    def forward(self, posterior):
        self._construct_base_samples(posterior)
        return posterior.rsample_from_base_samples(
            self.sample_shape,
            self.base_samples.expand(self._get_extended_base_sample_shape(posterior)))


class ShapeOnlyPosterior:
    """The shape attributes the samplers read from a single-output posterior,
    for the fused paths that never build the posterior object."""

    def __init__(self, batch_shape: torch.Size, q: int, device, dtype=torch.float64):
        self.base_sample_shape = torch.Size(batch_shape) + torch.Size([q])
        self.batch_range = (0, -1)
        self.device = device
        self.dtype = dtype


class SobolQMCNormalSampler(MCSampler):
    """sampling/normal.py:169-209."""

    def _construct_base_samples(self, posterior) -> None:
        target = self._get_collapsed_shape(posterior)
        if not self._reuse_base_samples(target):
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
        if not self._reuse_base_samples(target):
            Z = kernels.sobol_normal(dim, self.sample_shape.numel(), self.seed, device)
            self.register_buffer("base_samples", Z.view(target))
        return self.base_samples.reshape(-1, dim)


class IIDNormalSampler(MCSampler):
    """sampling/normal.py:137-166 (torch.randn under manual_seed, on the device)."""

    def _construct_base_samples(self, posterior) -> None:
        target = self._get_collapsed_shape(posterior)
        if not self._reuse_base_samples(target):
            with manual_seed(self.seed):
                Z = torch.randn(target, device=posterior.device, dtype=posterior.dtype)
            self.register_buffer("base_samples", Z)

    def base_samples_2d(self, dim: int, device) -> torch.Tensor:
        target = self.sample_shape + torch.Size([1, dim])
        if not self._reuse_base_samples(target):
            with manual_seed(self.seed):
                Z = torch.randn(target, device=device, dtype=torch.float64)
            self.register_buffer("base_samples", Z)
        return self.base_samples.reshape(-1, dim)


class ListSampler(MCSampler):
    """sampling/list_sampler.py: one sampler per posterior of a PosteriorList,
    samples concatenated along the output dimension."""

    def __init__(self, *samplers: MCSampler) -> None:
        nn.Module.__init__(self)
        self.samplers = nn.ModuleList(samplers)
        self._validate_samplers()

    def _validate_samplers(self) -> None:
        shapes = [s.sample_shape for s in self.samplers]
        if not all(shapes[0] == ss for ss in shapes):
            raise UnsupportedError("ListSampler requires all samplers to have the same sample shape.")

    @property
    def sample_shape(self) -> torch.Size:
        self._validate_samplers()
        return self.samplers[0].sample_shape

    def forward(self, posterior):
        samples = [s(p) for s, p in zip(self.samplers, posterior.posteriors)]
        return posterior._reshape_and_cat(samples)


def get_sampler(posterior=None, sample_shape: torch.Size = torch.Size([512]),
                seed: Optional[int] = None) -> MCSampler:
    """sampling/get_sampler.py:70-131: Sobol QMC for Gaussian posteriors, falling
    back to IID normal base samples when the collapsed base-sample dimension
    exceeds SobolEngine.MAXDIM (:84-89); a ListSampler for a PosteriorList."""
    from .posteriors import PosteriorList
    if isinstance(posterior, PosteriorList):
        return ListSampler(*[get_sampler(p, sample_shape=sample_shape, seed=seed)
                             for p in posterior.posteriors])
    sampler = SobolQMCNormalSampler(sample_shape=sample_shape, seed=seed)
    if posterior is not None:
        collapsed = sampler._get_collapsed_shape(posterior)
        if collapsed[len(sample_shape):].numel() > SOBOL_MAXDIM:
            import warnings
            warnings.warn(f"Output dim {collapsed[len(sample_shape):].numel()} is too large for "
                          "the Sobol engine. Using IIDNormalSampler instead.", RuntimeWarning)
            sampler = IIDNormalSampler(sample_shape=sample_shape, seed=seed)
    return sampler
