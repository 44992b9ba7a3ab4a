#!/usr/bin/env python3
"""Quad plan (csrc/quad.hip) vs the R route on forward-only geometries: per
call of bo::qmc_acq_native, the posterior launch's HIP-event time (post_quad
or post_partials + split reduction, bo::post_timing) and the whole call's
device time and host wall time, median of 40.  argv: [force] -- also time the
quad plan where its default rule declines (BO_POST_QUAD=1)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from botorch_amd import _lib, kernels  # noqa: E402
from botorch_amd.sampling import SobolQMCNormalSampler  # noqa: E402

force = len(sys.argv) > 1 and sys.argv[1] == "force"
if force:
    os.environ["BO_POST_QUAD"] = "1"
dev = torch.device("cuda", 0)
ops = _lib.torch_ops()
g = torch.Generator().manual_seed(0)
out = {}
geoms = [(1024, 64, 8, 256), (2048, 128, 8, 128), (2048, 33, 16, 128), (1024, 256, 8, 256)]
if force:
    geoms += [(4096, 64, 16, 512), (4096, 128, 16, 512), (4096, 512, 16, 512)]
for n, B, q, S in geoms:
    X = torch.rand(n, 6, generator=g, dtype=torch.float64).to(dev)
    y = torch.randn(n, generator=g, dtype=torch.float64).to(dev)
    cache = kernels.build_gp_cache(X, y, torch.full((6,), 0.4, dtype=torch.float64, device=dev),
                                   1e-3, 0.0)
    Xc = torch.rand(B, q, 6, generator=g, dtype=torch.float64).to(dev)
    Z = SobolQMCNormalSampler(torch.Size([S]), seed=0).base_samples_2d(q, dev).contiguous()
    kernels.quad_pairs.cache_clear()
    A = kernels.quad_ainv(cache, B, q)
    row = {"npairs": kernels.quad_pairs(B, q, n)}
    vals = {}
    for name, Ainv in (("quad", A), ("r_route", None)):
        if name == "quad" and Ainv is None:
            continue

        def call():
            return ops.qmc_acq_native(Xc, cache.Xt_scaled, cache.U, cache.Linv, cache.beta,
                                      cache.lengthscale, Z, None, int(cache.kind), 1, n, 1.0, 0.0,
                                      0.0, 1.0, 0.5, True, 1.0, 1.0, False, kernels.kxt_cap(dev),
                                      True, Ainv, cache.alpha)
        for _ in range(3):
            call()
        torch.cuda.synchronize()
        ops.post_timing(True)
        dts, walls = [], []
        for _ in range(40):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = time.perf_counter()
            e0.record()
            o = call()
            e1.record()
            torch.cuda.synchronize()
            walls.append(1e6 * (time.perf_counter() - t0))
            dts.append(1e3 * e0.elapsed_time(e1))
        ops.post_timing(False)
        post = sorted(1e3 * float(v) for v in ops.post_timing_read())
        dts.sort()
        walls.sort()
        vals[name] = o[0]
        row[name] = {"post_us": round(post[len(post) // 2], 1), "call_device_us": round(dts[20], 1),
                     "call_wall_us": round(walls[20], 1)}
    if "quad" in vals:
        rel = ((vals["quad"] - vals["r_route"]).abs() / vals["r_route"].abs().clamp_min(1e-300)).max()
        row["max_rel_diff"] = float(rel)
    out[f"n{n}_b{B}_q{q}"] = row
    print(json.dumps({f"n{n}_b{B}_q{q}": row}), flush=True)
print(json.dumps(out))
