#!/usr/bin/env python3
"""C2 optimize_acqf (qEI, n = 1024, q = 8, S = 256, 64 restarts, 512 raw
samples, maxiter 100) with the per-restart device L-BFGS-B, its evaluations
replayed from a captured graph (default) or eager, median of 5 after a
warm-up; and the C3 tail's capture cost (tools/capture_cost.py has the
detail).  Development tool."""
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
unit = torch.stack([torch.zeros(6, dtype=f64), torch.ones(6, dtype=f64)])
X = draw_sobol_samples(unit, 1024, 1, seed=0).squeeze(1)
Y = Hartmann(negate=True)(X).unsqueeze(-1)
m = SingleTaskGP(X.to(dev), Y.to(dev))
m.covar_module.lengthscale = torch.full((1, 6), bench.LENGTHSCALE, dtype=f64)
m.likelihood.noise = torch.tensor([bench.NOISE], dtype=f64)
m.eval()
acqf = qExpectedImprovement(m, float(Y.max()) - 0.3, sampler=SobolQMCNormalSampler(torch.Size([256]), seed=0))
for joint in (False, True):
    for use_graph in (True, False, True, False):
        def run():
            return optimize_acqf(acqf, unit.to(dev), 8, 64, 512,
                                 options={"seed": 0, "maxiter": 100, "use_graph": use_graph,
                                          "joint": joint},
                                 gen_candidates=gen_candidates_device)
        run()
        ts = []
        for _ in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            c, v = run()
            torch.cuda.synchronize()
            ts.append(1e3 * (time.perf_counter() - t0))
        g = gen_candidates_device
        print(f"joint={joint} use_graph={use_graph}: {sorted(ts)[2]:.2f} ms "
              f"({', '.join(f'{t:.2f}' for t in ts)}), evals {g.last_evals}, "
              f"graphed {g.last_graphed_evals}, best {float(v):.12f}", flush=True)
