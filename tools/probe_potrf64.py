#!/usr/bin/env python3
"""The DAG Cholesky's 64 x 64 diagonal-tile factor + inverse alone on one
workgroup (bo_probe_potrf64): microseconds per call and per phase for the
column-owner form (variants 1-4: pivots from the column, on a reciprocal
chain, one Newton step on 1/sqrt, the chain without the LDS-fed updates) and
the four-panel form (0), and the result
against torch."""
import json
import os
import sys

import torch
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _toolslib  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from botorch_amd import kernels  # noqa: E402
from botorch_amd._lib import check  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator().manual_seed(0)
    B = torch.randn(64, 64, generator=g, dtype=torch.float64)
    A = (B @ B.T + 64 * torch.eye(64, dtype=torch.float64)).to(dev)
    L = torch.linalg.cholesky(A)
    D = torch.linalg.inv(L)
    res = {}
    for var in (1, 2, 3, 4, 0):
        out = torch.zeros(2 * 4096, dtype=torch.float64, device=dev)
        ct = torch.zeros(9, dtype=torch.int64, device=dev)
        info = torch.zeros(1, dtype=torch.int32, device=dev)
        reps = 200
        check(_toolslib.tools().bo_probe_potrf64(kernels._p(A), kernels._p(out), kernels._p(ct),
                                                 kernels._p(info), var, reps, kernels._stream(dev)),
              "probe_potrf64")
        torch.cuda.synchronize()
        c = ct.cpu().tolist()
        Lg, Dg = out[:4096].view(64, 64), out[4096:].view(64, 64)
        res[f"variant{var}"] = {
            "us_per_call": c[8] / 100.0 / reps,
            "last_call_us": (c[1] - c[0]) / 100.0,
            "to_ct4_us": (c[4] - c[0]) / 100.0, "to_ct5_us": (c[5] - c[0]) / 100.0,
            "ct6_us": (c[6] - c[0]) / 100.0 if c[6] else None,
            "ct7_us": (c[7] - c[0]) / 100.0 if c[7] else None,
            "L_err": float((Lg - L).abs().max()), "D_err": float((Dg - D).abs().max()),
            "info": int(info.item())}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
