#!/usr/bin/env python3
"""Host profile of C2's eager forward + backward (the per-iteration cost of
gen_candidates_scipy): wall us per call and the top cProfile entries."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from botorch_amd.acquisition import qExpectedImprovement  # noqa: E402
from botorch_amd.models import SingleTaskGP  # noqa: E402
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
Xd = draw_sobol_samples(unit, 64, 8, seed=1).to(dev)


def step():
    Xt = Xd.detach().requires_grad_(True)
    v = acq(Xt)
    (g,) = torch.autograd.grad(v.sum(), Xt)
    return v, g


for _ in range(5):
    step()
torch.cuda.synchronize()
for sync in (True, False):
    t0 = time.perf_counter()
    for _ in range(100):
        v, g = step()
        if sync:
            g.cpu()
    torch.cuda.synchronize()
    print(f"eager fwd+bwd {'with g.cpu()' if sync else 'no sync'}: {1e4 * (time.perf_counter() - t0):.1f} us/call",
          flush=True)
pr = cProfile.Profile()
pr.enable()
for _ in range(100):
    v, g = step()
    g.cpu()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
