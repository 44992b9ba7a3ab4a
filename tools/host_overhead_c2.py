#!/usr/bin/env python3
"""Host-side cost of one eager C2 qEI forward (n = 1024, b = 64, q = 8,
S = 256): wall time per call over 200 calls without per-call syncs, and the
top cumulative Python costs from cProfile."""
import cProfile
import io
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from botorch_amd.acquisition import qExpectedImprovement  # noqa: E402
from botorch_amd.models import SingleTaskGP  # noqa: E402
from botorch_amd.sampling import SobolQMCNormalSampler  # noqa: E402
from botorch_amd.test_functions import Hartmann  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
X = torch.rand(1024, 6, generator=g, dtype=torch.float64)
Y = Hartmann(negate=True)(X).unsqueeze(-1)
m = SingleTaskGP(X.to(dev), Y.to(dev)).eval()
acqf = qExpectedImprovement(m, float(Y.max()), sampler=SobolQMCNormalSampler(torch.Size([256]), seed=0))
Xc = torch.rand(64, 8, 6, generator=g, dtype=torch.float64).to(dev)
with torch.no_grad():
    for _ in range(10):
        acqf(Xc)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        acqf(Xc)
    t_host = (time.perf_counter() - t0) / 200
    torch.cuda.synchronize()
    t_all = (time.perf_counter() - t0) / 200
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(500):
        acqf(Xc)
    pr.disable()
    torch.cuda.synchronize()
buf = io.StringIO()
st = pstats.Stats(pr, stream=buf)
st.sort_stats("tottime").print_stats(25)
st.sort_stats("cumulative").print_stats(25)
print(f"host issue {1e6 * t_host:.1f} us/call, with drain {1e6 * t_all:.1f} us/call")
print(buf.getvalue()[:12000])
