#!/usr/bin/env python3
"""The bench's C4 qEHVI forward alone (ModelListGP of 3 on DTLZ2, n = 2048,
d = 6, q = 8, S = 128, b = 128; FastNondominatedPartitioning cells), ``steps``
times after a warm-up, then ``steps`` forward + backward calls, for rocprofv3
kernel-trace / PMC passes over qehvi_kernel.  argv: steps."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from botorch_amd.acquisition import qExpectedHypervolumeImprovement  # noqa: E402
from botorch_amd.models import ModelListGP, SingleTaskGP  # noqa: E402
from botorch_amd.multi_objective import FastNondominatedPartitioning  # noqa: E402
from botorch_amd.sampling import SobolQMCNormalSampler  # noqa: E402
from botorch_amd.test_functions import DTLZ2  # noqa: E402
from botorch_amd.utils_sampling import draw_sobol_samples  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
dev = torch.device("cuda", 0)
f64 = torch.float64
n, q, S, b, mo = 2048, 8, 128, 128, 3
g = torch.Generator().manual_seed(0)
X = torch.rand(n, 6, generator=g, dtype=f64)
Y = -DTLZ2(dim=6, num_objectives=mo, negate=True).evaluate_true(X)
models = []
for t in range(mo):
    m = SingleTaskGP(X.to(dev), Y[:, t:t + 1].to(dev))
    m.covar_module.lengthscale = torch.full((1, 6), 0.6, dtype=f64)
    m.likelihood.noise = torch.tensor([1e-3], dtype=f64)
    models.append(m.eval())
ref_point = torch.full((mo,), -1.1, dtype=f64)
part = FastNondominatedPartitioning(ref_point, Y)
acqf = qExpectedHypervolumeImprovement(ModelListGP(*models), ref_point.tolist(), part,
                                       sampler=SobolQMCNormalSampler(torch.Size([S]), seed=0))
lo, _ = part.get_hypercell_bounds()
Xd = draw_sobol_samples(torch.stack([torch.zeros(6, dtype=f64), torch.ones(6, dtype=f64)]),
                        b, q, seed=1).to(dev)
with torch.no_grad():
    for _ in range(1 + steps):
        v = acqf(Xd)
Xg = Xd.clone().requires_grad_(True)
for _ in range(steps):
    (gx,) = torch.autograd.grad(acqf(Xg).sum(), Xg)
torch.cuda.synchronize()
print("done", steps, "cells", int(lo.shape[0]), "value_sum", float(v.sum()), "grad_abs",
      float(gx.abs().sum()))
