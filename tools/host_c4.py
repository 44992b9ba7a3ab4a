"""Host cost of the C4 qEHVI forward: wall time per call with a device sync,
the host issue time per call without one, and a cProfile of the issue path
(development tool)."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda", 0)
w = bench.make_workload("qehvi", dev)
acqf = w.acqf
X = w.Xc[: w.restarts].to(dev)
with torch.no_grad():
    for _ in range(5):
        acqf(X)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(50):
        acqf(X)
        torch.cuda.synchronize()
    print("wall per call (sync each)", (time.perf_counter() - t) / 50 * 1e3, "ms")
    p = cProfile.Profile()
    p.enable()
    for _ in range(50):
        acqf(X)
    p.disable()
    torch.cuda.synchronize()
pstats.Stats(p).sort_stats("tottime").print_stats(30)
