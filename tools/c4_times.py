#!/usr/bin/env python3
"""C4 acquisition timings for A/B runs (development tool): qEHVI and qNEHVI
(ModelListGP of 3 on DTLZ2, n = 2048, b = 128, q = 8, S = 128; qNEHVI on the
pruned baseline) forward-only and forward + backward, HIP events around
``steps`` back-to-back calls after warm-ups, one JSON line.  argv: steps."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from botorch_amd.utils_sampling import draw_sobol_samples  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda", 0)
f64 = torch.float64
unit = torch.stack([torch.zeros(6, dtype=f64), torch.ones(6, dtype=f64)])
X = draw_sobol_samples(unit, 128, 8, seed=1).to(dev)
out = {}
w = bench.make_workload("qehvi", dev)
for acq in ("qehvi", "qnehvi"):
    if acq == "qehvi":
        acqf = w.acqf
    else:
        from botorch_amd.acquisition import qNoisyExpectedHypervolumeImprovement
        from botorch_amd.sampling import SobolQMCNormalSampler
        torch.manual_seed(0)
        acqf = qNoisyExpectedHypervolumeImprovement(
            w.acqf.model, w.ref.tolist(), w.Xtr.to(dev), prune_baseline=True,
            sampler=SobolQMCNormalSampler(torch.Size([128]), seed=0))
    Xg = X.clone().requires_grad_(True)

    def fwd():
        with torch.no_grad():
            return acqf(X)

    def fb():
        (gx,) = torch.autograd.grad(acqf(Xg).sum(), Xg)
        return gx

    res = {}
    for name, fn in (("fwd_ms", fwd), ("fwd_bwd_ms", fb)):
        res[name] = 1e3 * bench._gpu_time(fn, steps=steps, warmup=3, reps=3)
    res["value_sum"] = float(fwd().sum())
    res["grad_abs_sum"] = float(fb().abs().sum())
    out[acq] = res
print(json.dumps(out))
