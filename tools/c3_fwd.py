#!/usr/bin/env python3
"""The bench's C3 qEI forward alone (n = 4096, q = 16, S = 512, b = 512 by
default), ``steps`` times after a warm-up, for rocprofv3 kernel-trace / PMC
passes that should see nothing but the timed kernels.  argv: steps [b]."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from botorch_amd.acquisition import qExpectedImprovement  # noqa: E402
from botorch_amd.models import SingleTaskGP  # noqa: E402
from botorch_amd.sampling import SobolQMCNormalSampler  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
b = int(sys.argv[2]) if len(sys.argv) > 2 else bench.RESTARTS
dev = torch.device("cuda", 0)
Xtr, Ytr, Xc = bench.build_problem(dev, max(b, bench.RESTARTS))
m = SingleTaskGP(Xtr.to(dev), Ytr.to(dev))
m.covar_module.lengthscale = torch.full((1, bench.D), bench.LENGTHSCALE, dtype=torch.float64)
m.likelihood.noise = torch.tensor([bench.NOISE], dtype=torch.float64)
m.eval()
acq = qExpectedImprovement(m, Ytr.max().item() - 1.5,
                           sampler=SobolQMCNormalSampler(torch.Size([bench.MC]), seed=0))
Xd = Xc[:b].to(dev)
with torch.no_grad():
    for _ in range(2 + steps):
        acq(Xd)
torch.cuda.synchronize()
print("done", steps, b)
