#!/usr/bin/env python3
"""The n = 4096 DAG Cholesky + inverse alone on the C3 kernel matrix (12
single launches, no batched shapes): the program the Cholesky PMC passes of
tools/prof_r03_final.sh count.  BO_CHOL_SHAPES="3x2048" times batched shapes
instead of nothing."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from botorch_amd.utils_sampling import draw_sobol_samples  # noqa: E402

f64 = torch.float64
unit = torch.stack([torch.zeros(6, dtype=f64), torch.ones(6, dtype=f64)])
X = draw_sobol_samples(unit, 4096, 1, seed=0).squeeze(1)
shapes = tuple(tuple(int(v) for v in s.split("x")) for s in os.environ.get("BO_CHOL_SHAPES", "").split(",") if s)
print(json.dumps(bench.time_cholesky(X, torch.device("cuda", 0), shapes=shapes)))
