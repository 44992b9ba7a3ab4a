#!/usr/bin/env python3
"""C2 eager qEI forward (n = 1024, b = 64, q = 8, S = 256) with K*x^T built by
its own launch (kxt_cap = default) against the posterior kernel evaluating
K*x between its MFMAs (kxt_cap = 0): per-call time over 2000 calls (issue and
with the final drain), interleaved 3 times, and the values compared."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from botorch_amd import _lib, kernels  # noqa: E402
from botorch_amd.acquisition import qExpectedImprovement  # noqa: E402
from botorch_amd.models import SingleTaskGP  # noqa: E402
from botorch_amd.sampling import SobolQMCNormalSampler  # noqa: E402
from botorch_amd.test_functions import Hartmann  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
X = torch.rand(1024, 6, generator=g, dtype=torch.float64)
Y = Hartmann(negate=True)(X).unsqueeze(-1)
m = SingleTaskGP(X.to(dev), Y.to(dev)).eval()
acqf = qExpectedImprovement(m, float(Y.mean()), sampler=SobolQMCNormalSampler(torch.Size([256]), seed=0))
Xc = torch.rand(64, 8, 6, generator=g, dtype=torch.float64).to(dev)
ops = _lib.torch_ops()
c = m.prediction_cache()
Z = acqf.sampler.base_samples_2d(8, dev)
cap = kernels.kxt_cap(dev)


def call(kcap):
    return ops.qmc_acq_eager(Xc, c.Xt_scaled, c.U, c.beta, c.lengthscale, Z, None, 0, 1, 1024, 1.0,
                             0.0, 0.0, 1.0, 0.5, True, 1.0, 1.0, kcap, None, c.alpha)


def rate(fn, n=2000):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t_issue = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    return round(1e6 * t_issue / n, 2), round(1e6 * t_all / n, 2)


out = {"kxt": [], "in_kernel": []}
with torch.no_grad():
    a = call(cap)[0].clone()
    b = call(0)[0].clone()
    torch.cuda.synchronize()
    out["max_abs_diff"] = float((a - b).abs().max())
    for _ in range(3):
        out["kxt"].append(rate(lambda: call(cap)))
        out["in_kernel"].append(rate(lambda: call(0)))
    ops.ladder_poll(0)
print(json.dumps(out))
