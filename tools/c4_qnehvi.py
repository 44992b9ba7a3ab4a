#!/usr/bin/env python3
"""The bench's C4 qNEHVI forward alone (ModelListGP of 3 on DTLZ2, n = 2048,
pruned baseline, S = 128, b = 128), ``steps`` times after a warm-up, for
rocprofv3 kernel traces (development tool).  argv: steps."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from botorch_amd.acquisition import qNoisyExpectedHypervolumeImprovement  # noqa: E402
from botorch_amd.models import ModelListGP  # noqa: E402
from botorch_amd.sampling import SobolQMCNormalSampler  # noqa: E402
from botorch_amd.utils_sampling import draw_sobol_samples  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
dev = torch.device("cuda", 0)
f64 = torch.float64
w = bench.make_workload("qehvi", dev)
models = w.acqf.model.models
X = w.Xtr
acqf = qNoisyExpectedHypervolumeImprovement(ModelListGP(*models), w.ref.tolist(), X.to(dev),
                                            sampler=SobolQMCNormalSampler(torch.Size([128]), seed=0),
                                            prune_baseline=True)
unit = torch.stack([torch.zeros(6, dtype=f64), torch.ones(6, dtype=f64)])
Xd = draw_sobol_samples(unit, 128, 8, seed=1).to(dev)
import time  # noqa: E402
with torch.no_grad():
    for _ in range(3):
        v = acqf(Xd)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        v = acqf(Xd)
    torch.cuda.synchronize()
    ms = 1e3 * (time.perf_counter() - t0) / steps
Xg = Xd.clone().requires_grad_(True)
for _ in range(2):
    (gx,) = torch.autograd.grad(acqf(Xg).sum(), Xg)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(steps // 2):
    (gx,) = torch.autograd.grad(acqf(Xg).sum(), Xg)
torch.cuda.synchronize()
ms_fb = 1e3 * (time.perf_counter() - t0) / (steps // 2)
print("done", float(v.sum()), "r", int(acqf.X_baseline.shape[0]), "ms_per_call", round(ms, 4),
      "fwd_bwd_ms", round(ms_fb, 4), "grad_abs", float(gx.abs().sum()))
