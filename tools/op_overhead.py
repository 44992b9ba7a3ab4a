#!/usr/bin/env python3
"""Host overhead of the torch.ops.bo dispatcher path against the direct
implementation call, on a tiny fused qEI (device time negligible)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from botorch_amd import kernels, ops  # noqa: E402
from botorch_amd.models import SingleTaskGP  # noqa: E402

dev = torch.device("cuda", 0)
X = torch.rand(64, 6, dtype=torch.float64, device=dev)
Y = X.sum(-1, keepdim=True)
m = SingleTaskGP(X, Y).eval()
c = m.prediction_cache()
Xc = torch.rand(4, 3, 6, dtype=torch.float64, device=dev)
Z = torch.randn(16, 3, dtype=torch.float64, device=dev)
args = (Xc, c.Xt, c.Xt_scaled, c.U, c.Linv, c.beta, c.alpha, c.lengthscale, Z, None, 0, 1, 1.0,
        0.0, 0.0, 1.0, 0.5, True, 1.0, 1.0, False)


def run(fn, n=2000):
    for _ in range(50):
        fn(*args)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn(*args)
    torch.cuda.synchronize()
    return 1e6 * (time.perf_counter() - t0) / n


with torch.no_grad():
    out = {"op_us": run(torch.ops.bo.qmc_acq), "direct_us": run(ops.qmc_acq._init_fn if hasattr(ops.qmc_acq, "_init_fn") else ops._qmc_acq_impl)}
print(json.dumps(out))
