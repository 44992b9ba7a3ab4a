#!/usr/bin/env python3
"""C3 optimize_acqf's raw-sample initialisation (qEI, q = 16, S = 512, 128
restarts, 1024 raw samples): median of 5 timed runs and a cProfile of one,
by cumulative and internal time (development tool; run under rocprofv3
--kernel-trace for the device side)."""
import cProfile
import io
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from botorch_amd.acquisition import qExpectedImprovement  # noqa: E402
from botorch_amd.models import SingleTaskGP  # noqa: E402
from botorch_amd.optim import gen_batch_initial_conditions  # noqa: E402
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


def init():
    return gen_batch_initial_conditions(acqf, unit, q=16, num_restarts=128, raw_samples=1024,
                                        options={"seed": 0})


init()
ts = []
for _ in range(5):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    init()
    torch.cuda.synchronize()
    ts.append(1e3 * (time.perf_counter() - t0))
print("init ms", [round(t, 2) for t in ts], "median", round(sorted(ts)[2], 2), flush=True)
raw = draw_sobol_samples(unit, 1024, 16, seed=0)
with torch.no_grad():
    acqf(raw)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        acqf(raw)
    torch.cuda.synchronize()
print("forward b=1024 ms", round(1e3 * (time.perf_counter() - t0) / 5, 3), flush=True)
pr = cProfile.Profile()
pr.enable()
init()
torch.cuda.synchronize()
pr.disable()
for key in ("cumulative", "tottime"):
    st = io.StringIO()
    pstats.Stats(pr, stream=st).sort_stats(key).print_stats(25)
    print(st.getvalue())
