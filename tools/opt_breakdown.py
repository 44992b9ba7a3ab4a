#!/usr/bin/env python3
"""Where C3's optimize_acqf (qEI, q = 16, S = 512, 128 restarts, 1024 raw
samples, maxiter 100) spends its time with the per-restart device L-BFGS-B:
the raw-sample initialisation alone, gen_candidates_device alone on its
initial conditions (default options, without graphs, without compaction),
each the median of 3 runs after a warm-up, with the evaluation counts."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from botorch_amd.acquisition import qExpectedImprovement  # noqa: E402
from botorch_amd.models import SingleTaskGP  # noqa: E402
from botorch_amd.optim import gen_batch_initial_conditions, gen_candidates_device, optimize_acqf  # noqa: E402
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


def timed(fn, reps=3):
    fn()
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        ts.append(1e3 * (time.perf_counter() - t0))
    return sorted(ts)[len(ts) // 2], out


t_all, _ = timed(lambda: optimize_acqf(acqf, unit, 16, 128, 1024, options={"seed": 0, "maxiter": 100},
                                       gen_candidates=gen_candidates_device))
t_init, ics = timed(lambda: gen_batch_initial_conditions(acqf, unit, q=16, num_restarts=128,
                                                         raw_samples=1024, options={"seed": 0}))
print(f"optimize_acqf {t_all:.1f} ms; init {t_init:.1f} ms", flush=True)
for label, opts in (("default", {}), ("no_graph", {"use_graph": False}), ("no_compact", {"compact": False}),
                    ("compact_min1", {"compact_min": 1})):
    t, _ = timed(lambda: gen_candidates_device(ics, acqf, unit[0], unit[1], options={"maxiter": 100, **opts}))
    g = gen_candidates_device
    print(f"gen {label}: {t:.1f} ms, evals {g.last_evals}, graphed {g.last_graphed_evals}, "
          f"shrinks {g.last_shrinks}", flush=True)
with torch.no_grad():
    t_f, _ = timed(lambda: acqf(ics))
Xg = ics.detach().clone().requires_grad_(True)


def fb():
    v = acqf(Xg)
    return torch.autograd.grad(v.sum(), Xg)


t_fb, _ = timed(fb)
x2 = ics[:2].detach().clone().requires_grad_(True)


def fb2():
    v = acqf(x2)
    return torch.autograd.grad(v.sum(), x2)


t_fb2, _ = timed(fb2)
print(f"eval b=128 fwd {t_f:.2f} ms, fwd+bwd {t_fb:.2f} ms; b=2 fwd+bwd {t_fb2:.2f} ms", flush=True)
