#!/usr/bin/env python3
"""bench.time_cholesky alone (n = 4096 single, 3 x 2048, 4 x 4096): one JSON
line; the environment picks the variant (BO_CHOL_* knobs are read once per
process, so A/B runs alternate processes)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda", 0)
Xtr, Ytr, _ = bench.build_problem(dev, 8)
out = bench.time_cholesky(Xtr, dev, reps=20, shapes=((3, 2048), (4, 4096)))
print(json.dumps({"env": {k: v for k, v in os.environ.items() if k.startswith("BO_CHOL")},
                  "ms": out["ms"], "frac": out["frac_of_spec"],
                  "batched": [(b["nb"], b["n"], b["ms"], b["frac_of_spec"]) for b in out["batched"]]}),
      flush=True)
