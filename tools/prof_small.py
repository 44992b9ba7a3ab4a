#!/usr/bin/env python3
"""C2 qEI, C5 SAAS qEI and C3 qNEI forward loops (for rocprofv3
--kernel-trace): where does the time of the non-headline configurations go?"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda", 0)
from botorch_amd.acquisition import qExpectedImprovement  # noqa: E402
from botorch_amd.models import SaasFullyBayesianSingleTaskGP, SingleTaskGP, sample_saas_prior  # noqa: E402
from botorch_amd.sampling import SobolQMCNormalSampler  # noqa: E402
from botorch_amd.test_functions import Hartmann  # noqa: E402
from botorch_amd.utils_sampling import draw_sobol_samples  # noqa: E402

f64 = torch.float64


def unit(d):
    return torch.stack([torch.zeros(d, dtype=f64), torch.ones(d, dtype=f64)])


which = sys.argv[1] if len(sys.argv) > 1 else "both"
if which in ("c2", "both"):
    X = draw_sobol_samples(unit(6), 1024, 1, seed=0).squeeze(1)
    Y = Hartmann(negate=True)(X).unsqueeze(-1)
    m = SingleTaskGP(X.to(dev), Y.to(dev))
    m.covar_module.lengthscale = torch.full((1, 6), bench.LENGTHSCALE, dtype=f64)
    m.likelihood.noise = torch.tensor([bench.NOISE], dtype=f64)
    m.eval()
    acqf = qExpectedImprovement(m, float(Y.max()), sampler=SobolQMCNormalSampler(torch.Size([256]), seed=0))
    Xd = draw_sobol_samples(unit(6), 64, 8, seed=1).to(dev)
    with torch.no_grad():
        for _ in range(3):
            acqf(Xd)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(50):
            acqf(Xd)
        torch.cuda.synchronize()
    print("C2 ms", 1e3 * (time.perf_counter() - t0) / 50)
if which in ("c5", "both"):
    d, n, M, q, S, b = 50, 256, 16, 4, 256, 64
    X = draw_sobol_samples(unit(d), n, 1, seed=0).squeeze(1)
    Y = Hartmann(negate=True)(X[:, :6]).unsqueeze(-1)
    Y = (Y - Y.mean()) / Y.std()
    smp = sample_saas_prior(d, M, seed=0)
    m = SaasFullyBayesianSingleTaskGP(X.to(dev), Y.to(dev))
    m.load_mcmc_samples({k: v.to(dev) for k, v in smp.items()})
    m.eval()
    acqf = qExpectedImprovement(m, float(Y.max()), sampler=SobolQMCNormalSampler(torch.Size([S]), seed=0))
    Xd = draw_sobol_samples(unit(d), b, q, seed=1).to(dev)
    with torch.no_grad():
        for _ in range(3):
            acqf(Xd)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(20):
            acqf(Xd)
        torch.cuda.synchronize()
    print("C5 ms", 1e3 * (time.perf_counter() - t0) / 20)
if which in ("c3nei",):
    from botorch_amd.acquisition import qNoisyExpectedImprovement
    X = draw_sobol_samples(unit(6), 4096, 1, seed=0).squeeze(1)
    Y = Hartmann(negate=True)(X).unsqueeze(-1)
    m = SingleTaskGP(X.to(dev), Y.to(dev))
    m.covar_module.lengthscale = torch.full((1, 6), bench.LENGTHSCALE, dtype=f64)
    m.likelihood.noise = torch.tensor([bench.NOISE], dtype=f64)
    m.eval()
    acqf = qNoisyExpectedImprovement(m, X.to(dev), sampler=SobolQMCNormalSampler(torch.Size([512]), seed=0),
                                     prune_baseline=True)
    Xd = draw_sobol_samples(unit(6), 512, 16, seed=1).to(dev)
    with torch.no_grad():
        for _ in range(2):
            acqf(Xd)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(10):
            acqf(Xd)
        torch.cuda.synchronize()
    print("C3 qNEI ms", 1e3 * (time.perf_counter() - t0) / 10, "r", acqf.X_baseline.shape[0])
