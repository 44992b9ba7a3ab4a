#!/usr/bin/env python3
"""C4 qNEHVI construction (ModelListGP(3) on DTLZ2, n = 2048, X_baseline = the
training points, prune_baseline, S = 128) timed cold and warm -- the bench's
C4_qNEHVI init_ms -- and a cProfile of a warm construction's top entries."""
import cProfile
import io
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from botorch_amd.acquisition import qNoisyExpectedHypervolumeImprovement  # noqa: E402
from botorch_amd.models import ModelListGP, SingleTaskGP  # noqa: E402
from botorch_amd.sampling import SobolQMCNormalSampler  # noqa: E402
from botorch_amd.test_functions import DTLZ2  # noqa: E402

dev = torch.device("cuda", 0)
f64 = torch.float64
g = torch.Generator().manual_seed(0)
X = torch.rand(2048, 6, generator=g, dtype=f64)
Y = -DTLZ2(dim=6, num_objectives=3, negate=True).evaluate_true(X)
ref = torch.full((3,), -1.1, dtype=f64)


def stgp(t):
    m = SingleTaskGP(X.to(dev), Y[:, t:t + 1].to(dev))
    m.covar_module.lengthscale = torch.full((1, 6), 0.6, dtype=f64)
    m.likelihood.noise = torch.tensor([1e-3], dtype=f64)
    return m.eval()


def build():
    models = [stgp(t) for t in range(3)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    a = qNoisyExpectedHypervolumeImprovement(ModelListGP(*models), ref.tolist(), X.to(dev),
                                             sampler=SobolQMCNormalSampler(torch.Size([128]), seed=0),
                                             prune_baseline=True)
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0), a


t_cold, a = build()
t_warm, _ = build()
t_warm2, _ = build()
print(f"qNEHVI init cold {t_cold:.1f} ms, warm {t_warm:.1f} / {t_warm2:.1f} ms, "
      f"r = {a.X_baseline.shape[0]}, cells/sample {a.cell_lower_bounds.shape[1]}", flush=True)
pr = cProfile.Profile()
pr.enable()
build()
pr.disable()
st = io.StringIO()
pstats.Stats(pr, stream=st).sort_stats("cumulative").print_stats(40)
print(st.getvalue())
st = io.StringIO()
pstats.Stats(pr, stream=st).sort_stats("tottime").print_stats(15)
print(st.getvalue())
