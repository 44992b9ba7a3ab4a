"""Host cost of the native C4 qEHVI forward: wall per call with the sync,
the split between the Python prologue and the op call (perf_counter around
each, device work excluded by a sync before each call), and a cProfile of the
prologue (development tool)."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from botorch_amd import _lib, acquisition, kernels  # noqa: E402

dev = torch.device("cuda", 0)
w = bench.make_workload("qehvi", dev)
acqf = w.acqf
X = w.Xc[: w.restarts].to(dev)
ops = _lib.torch_ops()
orig = ops.qehvi_members_eager
t_op = []


class Wrap:
    def __getattr__(self, k):
        return getattr(ops, k)

    def qehvi_members_eager(self, *a):
        t = time.perf_counter()
        r = orig(*a)
        t_op.append(time.perf_counter() - t)
        return r


acquisition._lib.torch_ops = lambda: Wrap()
orig_sync = kernels._stream_sync
t_sync = []


def sync(d):
    t = time.perf_counter()
    orig_sync(d)
    t_sync.append(time.perf_counter() - t)


kernels._stream_sync = sync
with torch.no_grad():
    for _ in range(10):
        acqf(X)
    t_op.clear()
    t_sync.clear()
    tot = []
    for _ in range(200):
        torch.cuda.synchronize()
        t = time.perf_counter()
        acqf(X)
        tot.append(time.perf_counter() - t)
    n = len(tot)
    print(f"per call: wall {1e6 * sum(tot) / n:.1f} us, op call {1e6 * sum(t_op) / n:.1f} us, "
          f"sync wait {1e6 * sum(t_sync) / n:.1f} us, rest (python) "
          f"{1e6 * (sum(tot) - sum(t_op) - sum(t_sync)) / n:.1f} us")
    p = cProfile.Profile()
    p.enable()
    for _ in range(200):
        acqf(X)
    p.disable()
pstats.Stats(p).sort_stats("tottime").print_stats(25)
