#!/usr/bin/env python3
"""Host cost of the pieces of an eager C2 qEI call (n = 1024, q = 8, S = 256):
per-call time over 3000 calls without syncs of acqf(X) and of the native op
at b = 64 (GPU-bound when the GPU is slower) and at b = 1 (host-bound: the
kernels are short), and of the Python pieces of the fused path alone."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from botorch_amd import _lib, kernels  # noqa: E402
from botorch_amd.acquisition import qExpectedImprovement, t_batch_mode  # noqa: E402
from botorch_amd.models import SingleTaskGP  # noqa: E402
from botorch_amd.sampling import SobolQMCNormalSampler  # noqa: E402
from botorch_amd.test_functions import Hartmann  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
X = torch.rand(1024, 6, generator=g, dtype=torch.float64)
Y = Hartmann(negate=True)(X).unsqueeze(-1)
m = SingleTaskGP(X.to(dev), Y.to(dev)).eval()
acqf = qExpectedImprovement(m, float(Y.mean()), sampler=SobolQMCNormalSampler(torch.Size([256]), seed=0))
ops = _lib.torch_ops()


def rate(fn, n=3000):
    for _ in range(100):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t_issue = time.perf_counter() - t0
    torch.cuda.synchronize()
    return round(1e6 * t_issue / n, 2), round(1e6 * (time.perf_counter() - t0) / n, 2)


out = {}
with torch.no_grad():
    for b in (64, 1):
        Xc = torch.rand(b, 8, 6, generator=g, dtype=torch.float64).to(dev)
        c = m.prediction_cache()
        Z = acqf.sampler.base_samples_2d(8, dev)
        cap = kernels.kxt_cap(dev)
        out[f"acqf_b{b}"] = rate(lambda: acqf(Xc))
        out[f"op_b{b}"] = rate(lambda: ops.qmc_acq_eager(
            Xc, c.Xt_scaled, c.U, c.beta, c.lengthscale, Z, None, 0, 1, 1024, 1.0, 0.0, 0.0, 1.0,
            0.5, True, 1.0, 1.0, cap, None, c.alpha))
    Xc = torch.rand(64, 8, 6, generator=g, dtype=torch.float64).to(dev)
    out["prediction_cache"] = rate(lambda: m.prediction_cache())
    out["model_key"] = rate(lambda: m._key())
    out["outcome_stats"] = rate(lambda: m.outcome_stats())
    out["base_samples_2d"] = rate(lambda: acqf.sampler.base_samples_2d(8, dev))
    out["quad_ainv"] = rate(lambda: kernels.quad_ainv(m.prediction_cache(), 64, 8))
    out["kxt_cap"] = rate(lambda: kernels.kxt_cap(dev))
    out["fused_eligible"] = rate(lambda: acqf._fused_eligible(Xc))
    out["t_batch_mode"] = rate(lambda: t_batch_mode(Xc))
    out["float_best_f"] = rate(lambda: float(acqf.best_f))
    st = torch.zeros(3, dtype=torch.float64)
    out["ladder_prev_outcome"] = rate(lambda: kernels.ladder_prev_outcome(st, 0, "x"))
    ops.ladder_poll(0)
print(json.dumps(out))
