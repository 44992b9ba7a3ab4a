#!/usr/bin/env python3
"""Host side of the C4 qEHVI forward + backward (ModelListGP of 3, n = 2048,
b = 128, q = 8): per-call issue time (no sync) against wall time, and a
cProfile of 20 calls by internal time (development tool)."""
import cProfile
import io
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from botorch_amd.utils_sampling import draw_sobol_samples  # noqa: E402

dev = torch.device("cuda", 0)
f64 = torch.float64
acqf = bench.make_workload("qehvi", dev).acqf
unit = torch.stack([torch.zeros(6, dtype=f64), torch.ones(6, dtype=f64)])
Xg = draw_sobol_samples(unit, 128, 8, seed=1).to(dev).requires_grad_(True)


def fb():
    return torch.autograd.grad(acqf(Xg).sum(), Xg)[0]


for _ in range(5):
    fb()
torch.cuda.synchronize()
n = 40
t0 = time.perf_counter()
for _ in range(n):
    fb()
t_issue = time.perf_counter() - t0
torch.cuda.synchronize()
t_wall = time.perf_counter() - t0
print(f"fwd_bwd issue {1e3 * t_issue / n:.4f} ms, wall {1e3 * t_wall / n:.4f} ms", flush=True)
pr = cProfile.Profile()
pr.enable()
for _ in range(20):
    fb()
torch.cuda.synchronize()
pr.disable()
st = io.StringIO()
pstats.Stats(pr, stream=st).sort_stats("tottime").print_stats(30)
print(st.getvalue())
