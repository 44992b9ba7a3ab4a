#!/usr/bin/env python3
"""Cost of capturing C3's forward + backward evaluation as a HIP graph
(GraphedAcquisition(with_grad=True), the device optimiser's capture) at b = 2
and b = 128, and of the first eager evaluation after it, with torch's
torch.cuda.graph entry as is and with its empty_cache() made a no-op
(development tool).  argv: "noempty" to patch."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from botorch_amd.acquisition import qExpectedImprovement  # noqa: E402
from botorch_amd.graphs import GraphedAcquisition  # noqa: E402
from botorch_amd.models import SingleTaskGP  # noqa: E402
from botorch_amd.sampling import SobolQMCNormalSampler  # noqa: E402
from botorch_amd.test_functions import Hartmann  # noqa: E402
from botorch_amd.utils_sampling import draw_sobol_samples  # noqa: E402

if len(sys.argv) > 1 and sys.argv[1] == "noempty":
    torch.cuda.empty_cache = lambda: None
dev = torch.device("cuda", 0)
f64 = torch.float64
unit = torch.stack([torch.zeros(6, dtype=f64), torch.ones(6, dtype=f64)])
X = draw_sobol_samples(unit, 4096, 1, seed=0).squeeze(1)
Y = Hartmann(negate=True)(X).unsqueeze(-1)
m = SingleTaskGP(X.to(dev), Y.to(dev))
m.covar_module.lengthscale = torch.full((1, 6), bench.LENGTHSCALE, dtype=f64)
m.likelihood.noise = torch.tensor([bench.NOISE], dtype=f64)
m.eval()
acqf = qExpectedImprovement(m, float(Y.max()) - 0.3, sampler=SobolQMCNormalSampler(torch.Size([512]), seed=0))


def fb(Xb):
    Xg = Xb.detach().requires_grad_(True)
    v = acqf(Xg)
    return torch.autograd.grad(v.sum(), Xg)[0]


for b in (2, 128, 2):
    Xb = draw_sobol_samples(unit, b, 16, seed=3).to(dev)
    for _ in range(3):
        fb(Xb)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ga = GraphedAcquisition(acqf, Xb, with_grad=True, warmup=1, check_each_call=False, share_input=True)
    torch.cuda.synchronize()
    t_cap = 1e3 * (time.perf_counter() - t0)
    t0 = time.perf_counter()
    fb(Xb)
    torch.cuda.synchronize()
    t_eager_after = 1e3 * (time.perf_counter() - t0)
    t0 = time.perf_counter()
    for _ in range(10):
        ga(Xb)
    torch.cuda.synchronize()
    t_rep = 1e3 * (time.perf_counter() - t0) / 10
    t0 = time.perf_counter()
    for _ in range(10):
        fb(Xb)
    torch.cuda.synchronize()
    t_eager = 1e3 * (time.perf_counter() - t0) / 10
    print(f"b={b}: capture {t_cap:.2f} ms, first eager after {t_eager_after:.2f} ms, replay {t_rep:.3f} ms, "
          f"eager {t_eager:.3f} ms", flush=True)
