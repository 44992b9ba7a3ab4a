#!/usr/bin/env python3
"""Host cost per call of the pieces of an eager C2 qEI forward (n = 1024,
b = 64, q = 8, S = 256), each timed over 2000 calls without syncs (issue
rate): the whole acqf(X), the native ops alone (bo::qmc_acq_eager and
bo::qmc_acq_native), model.prediction_cache(), and an empty torch.ops call
for scale.  Device time per call from the kernel trace is ~45 us, so a
number above that is host-bound."""
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
A = kernels.quad_ainv(c, 64, 8)
cap = kernels.kxt_cap(dev)


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
    return round(1e6 * t_issue / n, 1), round(1e6 * t_all / n, 1)


out = {}
with torch.no_grad():
    out["acqf_call"] = rate(lambda: acqf(Xc))
    out["qmc_acq_eager"] = rate(lambda: ops.qmc_acq_eager(
        Xc, c.Xt_scaled, c.U, c.beta, c.lengthscale, Z, None, 0, 1, 1024, 1.0, 0.0, 0.0, 1.0, 0.5,
        True, 1.0, 1.0, cap, A, c.alpha))
    out["qmc_acq_native_defer"] = rate(lambda: ops.qmc_acq_native(
        Xc, c.Xt_scaled, c.U, c.Linv, c.beta, c.lengthscale, Z, None, 0, 1, 1024, 1.0, 0.0, 0.0,
        1.0, 0.5, True, 1.0, 1.0, False, cap, True, A, c.alpha))
    out["prediction_cache"] = rate(lambda: m.prediction_cache())
    out["ladder_poll"] = rate(lambda: ops.ladder_poll(0))
    t = torch.zeros(4, device=dev)
    out["torch_add_inplace"] = rate(lambda: t.add_(1.0))
    out["torch_empty"] = rate(lambda: torch.empty(4096, device=dev))
print(json.dumps({k: {"issue_us": v[0], "with_drain_us": v[1]} for k, v in out.items()}))
