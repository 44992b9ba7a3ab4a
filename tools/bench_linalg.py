#!/usr/bin/env python3
"""Micro-benchmarks of the dense fp64 building blocks on the GPU: the MFMA GEMM
on the shapes the Cholesky / inverse / MLL use, the full n x n Cholesky +
inverse, and one exact-MLL closure.  Prints one JSON line."""
import ctypes
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from botorch_amd import _lib, kernels  # noqa: E402

dev = torch.device("cuda", 0)


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def gemm_case(M, N, K, ta, tb, flags, fl, name, batch=1):
    A = torch.randn(batch, K if ta else M, M if ta else K, dtype=torch.float64, device=dev)
    B = torch.randn(batch, N if tb else K, K if tb else N, dtype=torch.float64, device=dev)
    C = torch.zeros(batch, M, N, dtype=torch.float64, device=dev)
    ms = timed(lambda: kernels.gemm(A, B, ta, tb, C=C, flags=flags, beta=1.0))
    ref = None
    if batch == 1 and flags == 0 and M * N * K <= 2048 ** 3:
        C.zero_()
        kernels.gemm(A, B, ta, tb, C=C)
        a = A[0].mT if ta else A[0]
        b = B[0].mT if tb else B[0]
        ref = float((C[0] - a @ b).abs().max() / (a @ b).abs().max())
    return {"case": name, "ms": ms, "tflops": fl / ms / 1e9, "relerr": ref}


def main():
    n = int(os.environ.get("BO_N", "4096"))
    out = {"n": n, "gemm": []}
    g = out["gemm"]
    only = os.environ.get("BO_ONLY", "")
    if only != "chol":
        gemm_suite(g, n)
    chol_suite(out, n)
    if only != "chol":
        fit_suite(out, n)
    print(json.dumps(out))


def gemm_suite(g, n):
    g.append(gemm_case(n, n, n, False, False, 0, 2 * n ** 3, f"NN {n}^3"))
    g.append(gemm_case(n, n, n, False, True, 0, 2 * n ** 3, f"NT {n}^3"))
    g.append(gemm_case(n, n, n, True, False, 0, 2 * n ** 3, f"TN {n}^3"))
    g.append(gemm_case(2048, 2048, 2048, False, False, 0, 2 * 2048 ** 3, "NN 2048^3"))
    g.append(gemm_case(n, n, 128, False, True, _lib.GEMM_LOWER_C, n * n * 128,
                       f"SYRK {n}x{n}x128 lower"))
    g.append(gemm_case(n, n, 64, False, True, _lib.GEMM_LOWER_C, n * n * 64,
                       f"SYRK {n}x{n}x64 lower"))
    g.append(gemm_case(n, 64, 64, False, True, 0, 2 * n * 64 * 64, f"TRSM-like {n}x64x64"))
    g.append(gemm_case(n, 32, 32, False, True, 0, 2 * n * 32 * 32, f"TRSM-like {n}x32x32"))
    g.append(gemm_case(512, 16, n, False, False, 0, 2 * 512 * 16 * n, f"skinny 512x16x{n}"))
    g.append(gemm_case(n, n, n, False, False,
                       _lib.GEMM_LOWER_C | _lib.GEMM_A_UPPER | _lib.GEMM_B_LOWER, n ** 3 / 3,
                       f"U U^T {n} (lower, triangular operands)"))



def chol_suite(out, n):
    # full Cholesky + inverse of an RBF kernel matrix
    X = torch.rand(n, 6, dtype=torch.float64, device=dev)
    ls = torch.full((6,), 0.5, dtype=torch.float64, device=dev)
    K = kernels.covar_matrix(X, X, ls, diag_add=1e-2)
    ms = timed(lambda: kernels.cholesky_inverse(K), reps=5)
    L, Linv, info = kernels.cholesky_inverse(K)
    Kc = K.cpu()
    err = float((L.cpu() @ L.cpu().mT - Kc).abs().max() / Kc.abs().max())
    eye_err = float((Linv.cpu() @ L.cpu() - torch.eye(n, dtype=torch.float64)).abs().max())
    out["cholesky_inverse"] = {"ms": ms, "tflops_chol_plus_inv": (2 * n ** 3 / 3) / ms / 1e9,
                               "info": info, "rel_err_LLT": err, "err_LinvL": eye_err}
    y = torch.randn(n, dtype=torch.float64, device=dev)
    ms = timed(lambda: kernels.build_gp_cache(X, y, ls, 1e-2, 0.0), reps=5)
    out["gp_cache_build_ms"] = ms


def fit_suite(out, n):
    X = torch.rand(n, 6, dtype=torch.float64, device=dev)
    from botorch_amd import fit as fitmod
    from botorch_amd.models import SingleTaskGP
    Y = torch.sin(6 * X.sum(-1, keepdim=True))
    model = SingleTaskGP(X, Y)
    lay = fitmod._Layout(model)
    x0 = lay.get()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reps = 5
    for _ in range(reps):
        fitmod.mll_value_and_grad(model, x0, lay)
    torch.cuda.synchronize()
    out["mll_closure_ms"] = 1e3 * (time.perf_counter() - t0) / reps


if __name__ == "__main__":
    main()
