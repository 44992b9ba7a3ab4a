#!/usr/bin/env python3
"""C3 qEI forward + backward loop (the optimize_acqf call pattern,
gen.py:194-222), for rocprofv3 --kernel-trace: where does the gradient
path's time go?"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from botorch_amd.acquisition import qExpectedImprovement  # noqa: E402
from botorch_amd.models import SingleTaskGP  # noqa: E402
from botorch_amd.sampling import SobolQMCNormalSampler  # noqa: E402

dev = torch.device("cuda", 0)
f64 = torch.float64
Xtr, Ytr, Xc = bench.build_problem(dev, bench.RESTARTS)
m = SingleTaskGP(Xtr.to(dev), Ytr.to(dev))
m.covar_module.lengthscale = torch.full((1, bench.D), bench.LENGTHSCALE, dtype=f64)
m.likelihood.noise = torch.tensor([bench.NOISE], dtype=f64)
m.mean_module.constant = torch.tensor(bench.CONSTANT, dtype=f64)
m.eval()
m.prediction_cache()
acqf = qExpectedImprovement(m, float(Ytr.max()) - 1.5, sampler=SobolQMCNormalSampler(torch.Size([bench.MC]), seed=0))
Xg = Xc.to(dev).clone().requires_grad_(True)
for it in range(8):
    v = acqf(Xg)
    g, = torch.autograd.grad(v.sum(), Xg)
torch.cuda.synchronize()
print("fwd+bwd ok", float(g.abs().sum()))
