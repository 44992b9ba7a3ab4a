#!/usr/bin/env python3
"""C3's model (n = 4096) evaluated forward + backward at a tiny batch (b
t-batches of q = 16, default 2 -- the tail of a compacted optimize_acqf run),
``steps`` times after warm-ups, for rocprofv3 kernel traces: is the call
bound by its kernels or by the host?  argv: steps [b]."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from botorch_amd.acquisition import qExpectedImprovement  # noqa: E402
from botorch_amd.models import SingleTaskGP  # noqa: E402
from botorch_amd.sampling import SobolQMCNormalSampler  # noqa: E402
from botorch_amd.test_functions import Hartmann  # noqa: E402
from botorch_amd.utils_sampling import draw_sobol_samples  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 50
b = int(sys.argv[2]) if len(sys.argv) > 2 else 2
dev = torch.device("cuda", 0)
f64 = torch.float64
unit = torch.stack([torch.zeros(6, dtype=f64), torch.ones(6, dtype=f64)])
X = draw_sobol_samples(unit, 4096, 1, seed=0).squeeze(1)
Y = Hartmann(negate=True)(X).unsqueeze(-1)
m = SingleTaskGP(X.to(dev), Y.to(dev))
m.covar_module.lengthscale = torch.full((1, 6), bench.LENGTHSCALE, dtype=f64)
m.likelihood.noise = torch.tensor([bench.NOISE], dtype=f64)
m.eval()
acqf = qExpectedImprovement(m, float(Y.max()) - 0.3, sampler=SobolQMCNormalSampler(torch.Size([512]), seed=0))
Xc = draw_sobol_samples(unit, b, 16, seed=1).to(dev).requires_grad_(True)
for _ in range(5):
    torch.autograd.grad(acqf(Xc).sum(), Xc)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(steps):
    torch.autograd.grad(acqf(Xc).sum(), Xc)
torch.cuda.synchronize()
print(f"b={b}: {1e3 * (time.perf_counter() - t0) / steps:.3f} ms per forward + backward (wall)")
