#!/usr/bin/env python3
"""Split-k chunk length sweep of bo_post_partials (C2 and other small grids):
device time of post_partials (+ reduction) per chunk length, HIP events on the
launch stream."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from botorch_amd import kernels  # noqa: E402
from botorch_amd.test_functions import Hartmann  # noqa: E402
from botorch_amd.utils_sampling import draw_sobol_samples  # noqa: E402

dev = torch.device("cuda", 0)
f64 = torch.float64


def unit(d):
    return torch.stack([torch.zeros(d, dtype=f64), torch.ones(d, dtype=f64)])


def timed(fn, reps=50):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return 1e3 * s.elapsed_time(e) / reps  # us


out = {}
for (n, B, q) in [(1024, 64, 8), (2048, 128, 8), (4096, 1, 1), (4096, 64, 16), (256, 64, 4)]:
    X = draw_sobol_samples(unit(6), n, 1, seed=0).squeeze(1)
    Y = Hartmann(negate=True)(X)
    y = (Y - Y.mean()) / Y.std()
    cache = kernels.build_gp_cache(X.to(dev), y.to(dev), torch.full((6,), 0.5, dtype=f64, device=dev),
                                   1e-3, 0.0)
    Xc = draw_sobol_samples(unit(6), B, q, seed=1).to(dev)
    row = {"plan": kernels.split_plan(B, q, n)[0]}
    for split in (0, 64, 128, 256, 512, 1024):
        if split and split >= n:
            continue
        row[str(split)] = round(timed(lambda: kernels.post_partials(cache, Xc, split=split)), 1)
    out[f"n{n}_B{B}_q{q}"] = row
    print(f"n={n} B={B} q={q}", row, flush=True)
print(json.dumps(out))
