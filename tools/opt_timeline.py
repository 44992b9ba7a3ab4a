#!/usr/bin/env python3
"""One warm C3 optimize_acqf (qEI, q = 16, S = 512, 128 restarts, 1024 raw
samples, per-restart device L-BFGS-B) between two cumsum marker kernels, for
rocprofv3 --kernel-trace: argv[1] = the kernel_trace.csv of a previous run to
analyse instead (device busy time, idle gaps, top kernels inside the window)."""
import csv
import os
import sys
import time
from collections import defaultdict

if len(sys.argv) > 1:
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [i for i, r in enumerate(rows) if "cumsum" in r["Kernel_Name"].lower()
             or "scan" in r["Kernel_Name"].lower()]
    a, b = marks[-2], marks[-1]
    win = rows[a + 1:b]
    t0 = int(win[0]["Start_Timestamp"])
    t1 = int(win[-1]["End_Timestamp"])
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in win)
    gaps = []
    for p, r in zip(win, win[1:]):
        g = int(r["Start_Timestamp"]) - int(p["End_Timestamp"])
        if g > 20000:
            gaps.append((g, p["Kernel_Name"][:60], r["Kernel_Name"][:60]))
    print(f"window {(t1 - t0) / 1e6:.2f} ms, kernels {len(win)}, busy {busy / 1e6:.2f} ms, "
          f"idle {(t1 - t0 - busy) / 1e6:.2f} ms")
    print("gaps > 20 us:", len(gaps), "total", round(sum(g for g, _, _ in gaps) / 1e6, 2), "ms")
    for g, p, r in sorted(gaps, reverse=True)[:15]:
        print(f"  {g / 1e3:8.1f} us  after {p}  before {r}")
    tot = defaultdict(lambda: [0, 0])
    for r in win:
        k = r["Kernel_Name"][:70]
        tot[k][0] += 1
        tot[k][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    for k, (c, t) in sorted(tot.items(), key=lambda kv: -kv[1][1])[:15]:
        print(f"  {t / 1e6:7.3f} ms {c:5d}  {k}")
    sys.exit(0)

import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from botorch_amd.acquisition import qExpectedImprovement  # noqa: E402
from botorch_amd.models import SingleTaskGP  # noqa: E402
from botorch_amd.optim import gen_candidates_device, optimize_acqf  # noqa: E402
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


def run():
    return optimize_acqf(acqf, unit, 16, 128, 1024, options={"seed": 0, "maxiter": 100},
                         gen_candidates=gen_candidates_device)


for _ in range(2):
    run()
mark = torch.ones(7, device=dev)
torch.cuda.synchronize()
mark.cumsum(0)
t0 = time.perf_counter()
run()
torch.cuda.synchronize()
ms = 1e3 * (time.perf_counter() - t0)
mark.cumsum(0)
torch.cuda.synchronize()
g = gen_candidates_device
print(f"optimize_acqf {ms:.2f} ms, evals {g.last_evals}, graphed {g.last_graphed_evals}, "
      f"shrinks {g.last_shrinks}", flush=True)
