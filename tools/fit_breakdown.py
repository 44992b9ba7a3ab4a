"""Where the bench's GP fit spends its wall time outside the MLL closures:
total fit time against the summed closure wall times (each ends in the
closure's device-to-host read), then a cProfile pass (development tool)."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from botorch_amd import fit as fitmod  # noqa: E402
from botorch_amd.models import SingleTaskGP  # noqa: E402


def run(dev, Xtr, Ytr, prof=None):
    model = SingleTaskGP(Xtr.to(dev), Ytr.to(dev))
    mll = fitmod.ExactMarginalLogLikelihood(model.likelihood, model)
    ts = []
    orig = fitmod.mll_value_and_grad

    def timed(*a, **k):
        t = time.perf_counter()
        r = orig(*a, **k)
        ts.append(time.perf_counter() - t)
        return r

    fitmod.mll_value_and_grad = timed
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    if prof:
        prof.enable()
    fitmod.fit_gpytorch_mll(mll)
    if prof:
        prof.disable()
    torch.cuda.synchronize(dev)
    tot = time.perf_counter() - t0
    fitmod.mll_value_and_grad = orig
    return tot * 1e3, sum(ts) * 1e3, len(ts)


if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    Xtr, Ytr, _ = bench.build_problem(dev, 1)
    mode = sys.argv[1] if len(sys.argv) > 1 else ""
    if mode == "busy":  # 1 s of device work first (clock ramp?)
        a = torch.randn(4096, 4096, dtype=torch.float64, device=dev)
        t = time.perf_counter()
        while time.perf_counter() - t < 1.0:
            a = (a @ a).clamp_(-1, 1)
            torch.cuda.synchronize(dev)
    elif mode == "one":  # one closure first (allocations, tables)
        model = SingleTaskGP(Xtr.to(dev), Ytr.to(dev))
        lay = fitmod._layout(model)
        fitmod.mll_value_and_grad(model, lay.get(), lay, sync_model=False)
        torch.cuda.synchronize(dev)
    for r in range(3):
        tot, cl, n = run(dev, Xtr, Ytr)
        print(f"rep {r}: fit {tot:.1f} ms, closures {n} summing {cl:.1f} ms ({cl / n:.3f} ms each), "
              f"outside {tot - cl:.1f} ms")
    p = cProfile.Profile()
    run(dev, Xtr, Ytr, p)
    pstats.Stats(p).sort_stats("cumulative").print_stats(35)
