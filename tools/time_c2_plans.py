#!/usr/bin/env python3
"""C2 (n = 1024, q = 8, b = 64) posterior plans: HIP-event time of
bo_post_partials (+ its split reduction) per plan -- one pass, stream-K over
the default slots, uniform chunks of kc training rows -- median of 30."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from botorch_amd import kernels  # noqa: E402

dev = torch.device("cuda", 0)
g = torch.Generator().manual_seed(0)
out = {}
for n, B, q in ((1024, 64, 8), (4096, 64, 16)):
    X = torch.rand(n, 6, generator=g, dtype=torch.float64).to(dev)
    y = torch.randn(n, generator=g, dtype=torch.float64).to(dev)
    cache = kernels.build_gp_cache(X, y, torch.full((6,), 0.4, dtype=torch.float64, device=dev),
                                   1e-3, 0.0)
    Xc = torch.rand(B, q, 6, generator=g, dtype=torch.float64).to(dev)
    row = {}
    for name, split in (("auto", None), ("one_pass", 0), ("stream_k", -1), ("kc32", 32),
                        ("kc64", 64), ("kc128", 128), ("kc256", 256), ("kc512", 512)):
        if split is not None and split > n:
            continue
        ts = []
        for rep in range(33):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            kernels.post_partials(cache, Xc, split=split)
            e1.record()
            torch.cuda.synchronize()
            if rep >= 3:
                ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        row[name] = round(ts[len(ts) // 2], 1)
    out[f"n{n}_b{B}_q{q}"] = row
print(json.dumps(out))
