#!/usr/bin/env python3
"""HIP-event timing of bo_post_partials (+ K*x^T build) at n = 4096, q = 16
for b = 64 / 128 / 256 / 512 t-batches (the per-rank shares of C3 over
8 / 4 / 2 / 1 GPUs) under the library's plan and under forced one-pass /
stream-K plans; prints one JSON line (microseconds, median of 20)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from botorch_amd import kernels  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    n, d, q = 4096, 6, 16
    X = torch.rand(n, d, generator=g, dtype=torch.float64).to(dev)
    y = torch.randn(n, generator=g, dtype=torch.float64).to(dev)
    ls = torch.full((d,), 0.4, dtype=torch.float64, device=dev)
    cache = kernels.build_gp_cache(X, y, ls, 1e-3, 0.0)
    out = {}
    Xs = torch.rand(1024, d, generator=g, dtype=torch.float64).to(dev)
    ys = torch.randn(1024, generator=g, dtype=torch.float64).to(dev)
    c2 = kernels.build_gp_cache(Xs, ys, ls, 1e-3, 0.0)
    for B, q, cache in ((64, 16, cache), (128, 16, cache), (256, 16, cache), (512, 16, cache),
                        (64, 8, c2)):
        n = cache.n
        Xc = torch.rand(B, q, d, generator=g, dtype=torch.float64).to(dev)
        plan = kernels.split_plan(B, q, n)[0]
        row = {"plan": plan}
        for name, split in (("auto", None), ("one_pass", 0), ("stream_k", -1), ("kc64", 64)):
            ts = []
            for rep in range(23):
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


if __name__ == "__main__":
    main()
