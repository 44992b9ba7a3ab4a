#!/usr/bin/env python3
"""C3 qNEI construction (n = 4096, X_baseline = the 4096 training points,
prune_baseline, S = 512) timed cold (first in the process) and warm (new
model object, same data) -- the bench's C3_qNEI init_ms -- and a cProfile of
a warm construction's top entries."""
import cProfile
import io
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from botorch_amd.acquisition import qNoisyExpectedImprovement  # noqa: E402
from botorch_amd.models import SingleTaskGP  # noqa: E402
from botorch_amd.sampling import SobolQMCNormalSampler  # noqa: E402
from botorch_amd.test_functions import Hartmann  # noqa: E402
from botorch_amd.utils_sampling import draw_sobol_samples  # noqa: E402

dev = torch.device("cuda", 0)
f64 = torch.float64
unit = torch.stack([torch.zeros(6, dtype=f64), torch.ones(6, dtype=f64)])
X = draw_sobol_samples(unit, 4096, 1, seed=0).squeeze(1)
Y = Hartmann(negate=True)(X).unsqueeze(-1)


def build():
    m = SingleTaskGP(X.to(dev), Y.to(dev))
    m.covar_module.lengthscale = torch.full((1, 6), bench.LENGTHSCALE, dtype=f64)
    m.likelihood.noise = torch.tensor([bench.NOISE], dtype=f64)
    m.eval()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    a = qNoisyExpectedImprovement(m, X.to(dev), sampler=SobolQMCNormalSampler(torch.Size([512]), seed=0),
                                  prune_baseline=True)
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0), a


t_cold, a = build()
t_warm, _ = build()
t_warm2, _ = build()
print(f"qNEI init cold {t_cold:.1f} ms, warm {t_warm:.1f} / {t_warm2:.1f} ms, r = {a.X_baseline.shape[0]}",
      flush=True)
pr = cProfile.Profile()
pr.enable()
build()
pr.disable()
st = io.StringIO()
pstats.Stats(pr, stream=st).sort_stats("cumulative").print_stats(30)
print(st.getvalue())
