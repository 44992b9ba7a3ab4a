#!/usr/bin/env python3
"""Phases of C2 optimize_acqf (n = 1024, q = 8, S = 256, 64 restarts, 512 raw
samples, maxiter 100) on one GPU: raw-sample initialisation, the device
L-BFGS-B (graph capture + evaluations), scipy; wall ms per phase."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from botorch_amd.acquisition import qExpectedImprovement  # noqa: E402
from botorch_amd.models import SingleTaskGP  # noqa: E402
from botorch_amd.optim import (gen_batch_initial_conditions, gen_candidates_device,  # noqa: E402
                               gen_candidates_scipy, optimize_acqf)
from botorch_amd.sampling import SobolQMCNormalSampler  # noqa: E402
from botorch_amd.test_functions import Hartmann  # noqa: E402
from botorch_amd.utils_sampling import draw_sobol_samples  # noqa: E402

dev = torch.device("cuda", 0)
unit = torch.stack([torch.zeros(6), torch.ones(6)]).to(torch.float64)
X = draw_sobol_samples(unit, 1024, 1, seed=0).squeeze(1)
Y = Hartmann(negate=True)(X).unsqueeze(-1)
m = SingleTaskGP(X.to(dev), Y.to(dev))
m.covar_module.lengthscale = torch.full((1, 6), 0.5016, dtype=torch.float64)
m.likelihood.noise = torch.tensor([6.737947e-3], dtype=torch.float64)
m.eval()
acq = qExpectedImprovement(m, float(Y.max()) - 0.3, sampler=SobolQMCNormalSampler(torch.Size([256]), seed=0))
bnd = unit.to(dev)


def t(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        ts.append(1e3 * (time.perf_counter() - t0))
    return sorted(ts)[len(ts) // 2], out


ti, ics = t(lambda: gen_batch_initial_conditions(acq, bnd, 8, 64, 512, options={"seed": 0}))
print(f"init {ti:.2f} ms")
for opts in ({"maxiter": 100}, {"maxiter": 100, "use_graph": False}, {"maxiter": 100, "compact": False}):
    td, _ = t(lambda: gen_candidates_device(ics, acq, bnd[0], bnd[1], options=opts))
    print(f"device {opts}: {td:.2f} ms, evals {gen_candidates_device.last_evals}")
ts_, _ = t(lambda: gen_candidates_scipy(ics, acq, bnd[0], bnd[1], options={"maxiter": 100}), reps=3)
print(f"scipy {ts_:.2f} ms")
to, _ = t(lambda: optimize_acqf(acq, bnd, 8, 64, 512, options={"seed": 0, "maxiter": 100},
                                gen_candidates=gen_candidates_device))
print(f"optimize_acqf device {to:.2f} ms")
from botorch_amd.graphs import GraphedAcquisition  # noqa: E402
Xg = ics.clone()
tg, _ = t(lambda: GraphedAcquisition(acq, Xg, with_grad=True, warmup=1, check_each_call=False))
print(f"graph capture {tg:.2f} ms")
ga = GraphedAcquisition(acq, Xg, with_grad=True, warmup=1, check_each_call=False)
tr, _ = t(lambda: [ga(Xg) for _ in range(16)])
print(f"16 replays {tr:.2f} ms")
