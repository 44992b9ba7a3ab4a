#!/usr/bin/env python3
"""Phase clocks of qmc_kernel (tools-only build with -DBO_QMC_PHASES swapped in
for libbotorch_amd.so by tools/qmc_phases.sh): per workgroup the 100 MHz wall
clock at entry, covariance finalised, factor done, value reduced, exit -- for
the C2 and C3 qEI eager forwards."""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from botorch_amd import _lib  # noqa: E402
from botorch_amd.acquisition import qExpectedImprovement  # noqa: E402
from botorch_amd.models import SingleTaskGP  # noqa: E402
from botorch_amd.sampling import SobolQMCNormalSampler  # noqa: E402
from botorch_amd.test_functions import Hartmann  # noqa: E402
from botorch_amd.utils_sampling import draw_sobol_samples  # noqa: E402

dev = torch.device("cuda", 0)
f64 = torch.float64
PH_N, PH_WG = 5, 1024
so = ctypes.CDLL(_lib.LIB_PATH)
so.bo_qmc_phase_dump.argtypes = [ctypes.c_void_p, ctypes.c_int]


def unit(d):
    return torch.stack([torch.zeros(d, dtype=f64), torch.ones(d, dtype=f64)])


def run(tag, n, q, S, b):
    X = draw_sobol_samples(unit(6), n, 1, seed=0).squeeze(1)
    Y = Hartmann(negate=True)(X).unsqueeze(-1)
    m = SingleTaskGP(X.to(dev), Y.to(dev))
    m.covar_module.lengthscale = torch.full((1, 6), bench.LENGTHSCALE, dtype=f64)
    m.likelihood.noise = torch.tensor([bench.NOISE], dtype=f64)
    m.eval()
    acqf = qExpectedImprovement(m, float(Y.max()), sampler=SobolQMCNormalSampler(torch.Size([S]), seed=0))
    Xd = draw_sobol_samples(unit(6), b, q, seed=1).to(dev)
    spans = []
    per = []
    with torch.no_grad():
        for it in range(12):
            acqf(Xd)
            torch.cuda.synchronize()
            if it < 2:
                continue
            buf = np.zeros(PH_WG * PH_N, dtype=np.uint64)
            assert so.bo_qmc_phase_dump(buf.ctypes.data, buf.size) == 0
            t = buf.reshape(PH_WG, PH_N)[: min(b, PH_WG)].astype(np.int64)
            t = (t - t[:, 0].min()) * 0.01  # us
            spans.append(t[:, 4].max())
            per.append(t)
    t = per[-1]
    print(f"{tag}: B={b} kernel span (first entry -> last exit) median {np.median(spans):.2f} us "
          f"(min {min(spans):.2f}, max {max(spans):.2f})")
    for k, name in enumerate(["entry", "cov", "factor", "value", "exit"]):
        c = t[:, k]
        print(f"   {name:7s} min {c.min():7.2f}  med {np.median(c):7.2f}  max {c.max():7.2f} us")
    d = np.diff(t, axis=1)
    for k, name in enumerate(["load+finalise", "factor", "samples+reduce", "status"]):
        print(f"   d[{name:15s}] med {np.median(d[:, k]):6.2f}  max {d[:, k].max():6.2f} us")
    last = int(np.argmax(t[:, 4]))
    print("   last WG", last, "phases", np.round(t[last], 2).tolist())


run("C2", 1024, 8, 256, 64)
run("C3", 4096, 16, 512, 512)
