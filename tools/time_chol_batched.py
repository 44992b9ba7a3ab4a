#!/usr/bin/env python3
"""bench.time_cholesky (single n = 4096 and the batched shapes) on the C3
kernel matrix; BO_CHOL_BATCH_STAGGER selects the batched queue's stagger."""
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
r = bench.time_cholesky(X, torch.device("cuda", 0))
print(json.dumps({"stagger": os.environ.get("BO_CHOL_BATCH_STAGGER", "0"), **r}))
