#!/usr/bin/env python3
"""C2 / C3 optimize_acqf with the device L-BFGS-B (for rocprofv3
--kernel-trace --stats): what one bo_lbfgsb_step launch costs next to the
evaluation kernels it sits between."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from botorch_amd._lib import lib  # noqa: E402
from botorch_amd.acquisition import qExpectedImprovement  # noqa: E402
from botorch_amd.models import SingleTaskGP  # noqa: E402
from botorch_amd.optim import gen_candidates_device, optimize_acqf  # noqa: E402
from botorch_amd.sampling import SobolQMCNormalSampler  # noqa: E402
from botorch_amd.test_functions import Hartmann  # noqa: E402
from botorch_amd.utils_sampling import draw_sobol_samples  # noqa: E402

dev = torch.device("cuda", 0)
f64 = torch.float64
unit = torch.stack([torch.zeros(6, dtype=f64), torch.ones(6, dtype=f64)])
for n, q, S, b, raw in ((1024, 8, 256, 64, 512), (4096, 16, 512, 128, 1024)):
    X = draw_sobol_samples(unit, n, 1, seed=0).squeeze(1)
    Y = Hartmann(negate=True)(X).unsqueeze(-1)
    m = SingleTaskGP(X.to(dev), Y.to(dev))
    m.covar_module.lengthscale = torch.full((1, 6), bench.LENGTHSCALE, dtype=f64)
    m.likelihood.noise = torch.tensor([bench.NOISE], dtype=f64)
    m.eval()
    acqf = qExpectedImprovement(m, float(Y.max()) - 0.3,
                                sampler=SobolQMCNormalSampler(torch.Size([S]), seed=0))
    for staged in (1, 0, 1):
        lib().bo_lbfgsb_set_staging(staged)
        prof = torch.zeros(b, 8, dtype=torch.int64, device=dev)
        for it in range(2):
            if it == 1:  # phase clocks of the second run (100 MHz wall clock)
                torch.cuda.synchronize()
                lib().bo_lbfgsb_set_profile(prof.data_ptr(), b)
                t0 = time.perf_counter()
            c, v = optimize_acqf(acqf, unit.to(dev), q, b, raw, options={"seed": 0, "maxiter": 100},
                                 gen_candidates=gen_candidates_device)
        torch.cuda.synchronize()
        wall = 1e3 * (time.perf_counter() - t0)
        lib().bo_lbfgsb_set_profile(None, 0)
        ev = gen_candidates_device.last_evals
        tot = prof.double().cpu() * 0.01 / ev  # 100 MHz wall clock -> us per launch, per restart
        names = ["load", "cauchy", "freev", "formk", "cmprlb", "subsm", "linesearch+update",
                 "store"]
        worst = int(tot.sum(1).argmax())
        print(f"n={n} q={q} b={b} staged={staged}: optimize_acqf {wall:.1f} ms, best {float(v):.8f},"
              f" evals {ev}; us per launch, restart mean: "
              + ", ".join(f"{k} {x:.2f}" for k, x in zip(names, tot.mean(0).tolist()))
              + f"; total mean {tot.sum(1).mean():.2f}, slowest restart {tot.sum(1).max():.2f} ("
              + ", ".join(f"{k} {x:.2f}" for k, x in zip(names, tot[worst].tolist())) + ")",
              flush=True)
