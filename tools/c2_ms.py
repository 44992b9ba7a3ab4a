#!/usr/bin/env python3
"""The bench's C2 qEI forward (n = 1024, d = 6, q = 8, S = 256, b = 64), eager
and graphed, HIP events around 200 back-to-back calls (median of 3), one line
for tools/ab.sh A/B runs; the values' sum as a same-result check."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from botorch_amd.acquisition import qExpectedImprovement  # noqa: E402
from botorch_amd.graphs import GraphedAcquisition  # noqa: E402
from botorch_amd.models import SingleTaskGP  # noqa: E402
from botorch_amd.sampling import SobolQMCNormalSampler  # noqa: E402
from botorch_amd.test_functions import Hartmann  # noqa: E402
from botorch_amd.utils_sampling import draw_sobol_samples  # noqa: E402

dev = torch.device("cuda", 0)
f64 = torch.float64
unit = torch.stack([torch.zeros(6, dtype=f64), torch.ones(6, dtype=f64)])
X = draw_sobol_samples(unit, 1024, 1, seed=0).squeeze(1)
Y = Hartmann(negate=True)(X).unsqueeze(-1)
Xc = draw_sobol_samples(unit, 64, 8, seed=1).to(dev)
m = SingleTaskGP(X.to(dev), Y.to(dev))
m.covar_module.lengthscale = torch.full((1, 6), bench.LENGTHSCALE, dtype=f64)
m.likelihood.noise = torch.tensor([bench.NOISE], dtype=f64)
m.eval()
acqf = qExpectedImprovement(m, float(Y.max()) - 0.3, sampler=SobolQMCNormalSampler(torch.Size([256]), seed=0))
with torch.no_grad():
    v = acqf(Xc)
    eager = bench._gpu_time(lambda: acqf(Xc), steps=200, warmup=20)
    g = GraphedAcquisition(acqf, Xc, share_input=True)
    graphed = bench._gpu_time(lambda: g(Xc), steps=200, warmup=20)
print(f"eager_ms {1e3 * eager:.4f} graphed_ms {1e3 * graphed:.4f} value_sum {float(v.sum()):.15e}")
