#!/usr/bin/env python3
"""C3 optimize_acqf (qEI, q = 16, S = 512, 128 restarts, 1024 raw samples,
maxiter 100) with the per-restart device L-BFGS-B at several status-read
schedules (gen_candidates_device's check_every), median of 3 after a warm-up,
with the evaluation counts, shrinks and best value (development tool)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from botorch_amd.acquisition import qExpectedImprovement  # noqa: E402
from botorch_amd.models import SingleTaskGP  # noqa: E402
from botorch_amd.optim import gen_candidates_device, optimize_acqf  # noqa: E402
from botorch_amd.sampling import SobolQMCNormalSampler  # noqa: E402
from botorch_amd.test_functions import Hartmann  # noqa: E402
from botorch_amd.utils_sampling import draw_sobol_samples  # noqa: E402

dev = torch.device("cuda", 0)
f64 = torch.float64
unit = torch.stack([torch.zeros(6, dtype=f64), torch.ones(6, dtype=f64)]).to(dev)
X = draw_sobol_samples(unit.cpu(), 4096, 1, seed=0).squeeze(1)
Y = Hartmann(negate=True)(X).unsqueeze(-1)
m = SingleTaskGP(X.to(dev), Y.to(dev))
m.covar_module.lengthscale = torch.full((1, 6), bench.LENGTHSCALE, dtype=f64)
m.likelihood.noise = torch.tensor([bench.NOISE], dtype=f64)
m.eval()
acqf = qExpectedImprovement(m, float(Y.max()) - 0.3, sampler=SobolQMCNormalSampler(torch.Size([512]), seed=0))
for opts in ({}, {"check_every": 1}, {"early_checks": False}, {}, {"check_every": 1}):
    def run():
        return optimize_acqf(acqf, unit, 16, 128, 1024, options={"seed": 0, "maxiter": 100, **opts},
                             gen_candidates=gen_candidates_device)
    run()
    ts = []
    for _ in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        c, v = run()
        torch.cuda.synchronize()
        ts.append(1e3 * (time.perf_counter() - t0))
    g = gen_candidates_device
    st = g.last_state
    print(f"{opts}: {sorted(ts)[1]:.2f} ms ({', '.join(f'{t:.2f}' for t in ts)}), evals {g.last_evals}, "
          f"shrinks {g.last_shrinks}, max nit {int(st.nit.max())}, best {float(v):.12f}", flush=True)
