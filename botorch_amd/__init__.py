"""botorch_amd: MI355X-native batched GP posterior + Monte-Carlo acquisition.

A drop-in for BoTorch's hot path (SingleTaskGP / GPyTorchPosterior /
MCAcquisitionFunction.forward / optimize_acqf / fit_gpytorch_mll) whose
numerics run as hand-written gfx950 HIP kernels behind the C ABI in
``include/botorch_amd.h`` (``libbotorch_amd.so``, loaded by ``_lib.py``).
"""
__version__ = "0.1.0"
