#!/usr/bin/env python3
"""The rank-local b = 64 shard of C3 (n = 4096, q = 16): 20 stream-K
posterior calls, for a rocprofv3 kernel-trace breakdown."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from botorch_amd import kernels  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
X = torch.rand(4096, 6, generator=g, dtype=torch.float64).to(dev)
y = torch.randn(4096, generator=g, dtype=torch.float64).to(dev)
cache = kernels.build_gp_cache(X, y, torch.full((6,), 0.4, dtype=torch.float64, device=dev), 1e-3, 0.0)
Xc = torch.rand(64, 16, 6, generator=g, dtype=torch.float64).to(dev)
for _ in range(20):
    kernels.post_partials(cache, Xc)
torch.cuda.synchronize()
print("done")
