#!/usr/bin/env python3
"""Phase clocks of the joint device L-BFGS-B (gen_candidates_device(joint=True):
ONE restart of n = b q d on a 4-wave workgroup) inside C2 / C3 optimize_acqf,
next to the per-restart run and scipy: where one bo_lbfgsb_step launch spends
its time (us per launch; load, cauchy, freev, formk, cmprlb, subsm, line
search + update, store).  On the grid route (n >= 2048) the freev column is
the number of Cauchy breakpoints walked per launch and the store column adds
the breakpoint rounds per launch to its ~1 us."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from botorch_amd._lib import lib  # noqa: E402
from botorch_amd.acquisition import qExpectedImprovement  # noqa: E402
from botorch_amd.models import SingleTaskGP  # noqa: E402
from botorch_amd.optim import gen_candidates_device, gen_candidates_scipy, optimize_acqf  # noqa: E402
from botorch_amd.sampling import SobolQMCNormalSampler  # noqa: E402
from botorch_amd.test_functions import Hartmann  # noqa: E402
from botorch_amd.utils_sampling import draw_sobol_samples  # noqa: E402

dev = torch.device("cuda", 0)
f64 = torch.float64
unit = torch.stack([torch.zeros(6, dtype=f64), torch.ones(6, dtype=f64)])
names = ["load", "cauchy", "freev", "formk", "cmprlb", "subsm", "linesearch+update", "store"]
for n, q, S, b, raw in ((1024, 8, 256, 64, 512), (4096, 16, 512, 128, 1024)):
    X = draw_sobol_samples(unit, n, 1, seed=0).squeeze(1)
    Y = Hartmann(negate=True)(X).unsqueeze(-1)
    m = SingleTaskGP(X.to(dev), Y.to(dev))
    m.covar_module.lengthscale = torch.full((1, 6), bench.LENGTHSCALE, dtype=f64)
    m.likelihood.noise = torch.tensor([bench.NOISE], dtype=f64)
    m.eval()
    acqf = qExpectedImprovement(m, float(Y.max()) - 0.3,
                                sampler=SobolQMCNormalSampler(torch.Size([S]), seed=0))
    for label, gen, extra in (("scipy", gen_candidates_scipy, {}),
                              ("joint", gen_candidates_device, {"joint": True}),
                              ("joint_1wg", gen_candidates_device, {"joint": True})):
        # joint: the default route (the grid kernel for n >= 2048); joint_1wg:
        # the one-workgroup kernel (bo_lbfgsb_set_grid(-1))
        lib().bo_lbfgsb_set_grid(-1 if label == "joint_1wg" else 0)
        prof = torch.zeros(1, 8, dtype=torch.int64, device=dev)
        walls = []
        for it in range(5):  # a warm-up, three timed runs, one profiled run
            if it == 4 and label != "scipy":
                lib().bo_lbfgsb_set_profile(prof.data_ptr(), 1)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            c, v = optimize_acqf(acqf, unit.to(dev), q, b, raw,
                                 options={"seed": 0, "maxiter": 100, **extra}, gen_candidates=gen)
            torch.cuda.synchronize()
            if 1 <= it <= 3:
                walls.append(1e3 * (time.perf_counter() - t0))
        lib().bo_lbfgsb_set_profile(None, 0)
        wall = sorted(walls)[1]
        line = (f"n={n} q={q} b={b} {label}: optimize_acqf {wall:.1f} ms (runs "
                + " ".join(f"{w:.1f}" for w in walls) + f"), best {float(v):.10f}")
        if label != "scipy":
            ev = gen_candidates_device.last_evals
            st = gen_candidates_device.last_state
            tot = prof.double().cpu()[0] * 0.01 / ev
            line += (f", evals {ev}, nit {int(st.nit[0])}, status {int(st.status[0])}; us per launch: "
                     + ", ".join(f"{k} {x:.1f}" for k, x in zip(names, tot.tolist()))
                     + f"; total {tot.sum():.1f}")
        print(line, flush=True)
    lib().bo_lbfgsb_set_grid(0)
