#!/usr/bin/env python3
"""The bench's C4 qEHVI (ModelListGP of 3 on DTLZ2, n = 2048, b = 128, q = 8)
forward + backward, ``steps`` times after a warm-up (development tool; A/B of
the gradient path).  argv: steps."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from botorch_amd.utils_sampling import draw_sobol_samples  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda", 0)
f64 = torch.float64
w = bench.make_workload("qehvi", dev)
acqf = w.acqf
unit = torch.stack([torch.zeros(6, dtype=f64), torch.ones(6, dtype=f64)])
Xg = draw_sobol_samples(unit, 128, 8, seed=1).to(dev).requires_grad_(True)
for _ in range(3):
    (gx,) = torch.autograd.grad(acqf(Xg).sum(), Xg)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(steps):
    (gx,) = torch.autograd.grad(acqf(Xg).sum(), Xg)
torch.cuda.synchronize()
ms = 1e3 * (time.perf_counter() - t0) / steps
print("done fwd_bwd_ms", round(ms, 4), "grad_abs", float(gx.abs().sum()))
