#!/usr/bin/env python3
"""Spread of C2 optimize_acqf with the device joint L-BFGS-B against scipy:
wall ms of 7 runs each (after one warm-up), and the graph capture alone."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from botorch_amd.acquisition import qExpectedImprovement  # noqa: E402
from botorch_amd.graphs import GraphedAcquisition  # noqa: E402
from botorch_amd.models import SingleTaskGP  # noqa: E402
from botorch_amd.optim import gen_candidates_device, gen_candidates_scipy, optimize_acqf  # noqa: E402
from botorch_amd.sampling import SobolQMCNormalSampler  # noqa: E402
from botorch_amd.test_functions import Hartmann  # noqa: E402
from botorch_amd.utils_sampling import draw_sobol_samples  # noqa: E402

dev = torch.device("cuda", 0)
unit = torch.stack([torch.zeros(6), torch.ones(6)]).to(torch.float64)
X = draw_sobol_samples(unit, 1024, 1, seed=0).squeeze(1)
Y = Hartmann(negate=True)(X).unsqueeze(-1)
m = SingleTaskGP(X.to(dev), Y.to(dev))
m.covar_module.lengthscale = torch.full((1, 6), bench.LENGTHSCALE, dtype=torch.float64)
m.likelihood.noise = torch.tensor([bench.NOISE], dtype=torch.float64)
m.eval()
acq = qExpectedImprovement(m, float(Y.max()), sampler=SobolQMCNormalSampler(torch.Size([256]), seed=0))
bnd = unit.to(dev)
for name, gen, extra in (("scipy", gen_candidates_scipy, {}),
                         ("device_joint", gen_candidates_device, {"algorithm": "lbfgsb", "joint": True})):
    opts = {"seed": 0, "maxiter": 100, **extra}
    optimize_acqf(acq, bnd, 8, 64, 512, options=opts, gen_candidates=gen)
    torch.cuda.synchronize()
    ts = []
    for _ in range(7):
        t0 = time.perf_counter()
        optimize_acqf(acq, bnd, 8, 64, 512, options=opts, gen_candidates=gen)
        torch.cuda.synchronize()
        ts.append(round(1e3 * (time.perf_counter() - t0), 2))
    print(name, "ms", ts, "median", sorted(ts)[3], flush=True)
Xg = draw_sobol_samples(bnd.cpu(), 64, 8, seed=1).to(dev)
for _ in range(3):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ga = GraphedAcquisition(acq, Xg, with_grad=True, warmup=1, check_each_call=False)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for _ in range(20):
        ga(Xg)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"capture {1e3 * (t1 - t0):.2f} ms, 20 replays {1e3 * (t2 - t1):.2f} ms", flush=True)
