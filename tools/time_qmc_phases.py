#!/usr/bin/env python3
"""Where qmc_kernel's time goes at C2 / C3: the finalisation launched alone on
real posterior partials (HIP events over 100 launches each) in its modes --
POSTERIOR (the partial sums and K** only), CHOL (+ the q x q jitter ladder),
QEI (+ the Sobol samples and the reduction) -- each with and without the fused
ladder status, and the split-k reduction it follows (C2)."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from botorch_amd import _lib, kernels  # noqa: E402
from botorch_amd._lib import check, lib  # noqa: E402
from botorch_amd.models import SingleTaskGP  # noqa: E402
from botorch_amd.test_functions import Hartmann  # noqa: E402
from botorch_amd.utils_sampling import draw_sobol_samples  # noqa: E402

dev = torch.device("cuda", 0)
f64 = torch.float64
unit = torch.stack([torch.zeros(6, dtype=f64), torch.ones(6, dtype=f64)])
out = {}
for tag, (n, q, S, b) in {"C2": (1024, 8, 256, 64), "C3": (4096, 16, 512, 512)}.items():
    X = draw_sobol_samples(unit, n, 1, seed=0).squeeze(1)
    Y = Hartmann(negate=True)(X).unsqueeze(-1)
    m = SingleTaskGP(X.to(dev), Y.to(dev))
    m.covar_module.lengthscale = torch.full((1, 6), bench.LENGTHSCALE, dtype=f64)
    m.likelihood.noise = torch.tensor([bench.NOISE], dtype=f64)
    m.eval()
    cache = m.prediction_cache()
    Xc = draw_sobol_samples(unit, b, q, seed=1).to(dev)
    pp = kernels.post_partials(cache, Xc)
    Z = kernels.sobol_normal(q, S, 0, dev)
    acq = torch.empty(b, dtype=f64, device=dev)
    info = torch.empty(b, dtype=torch.int32, device=dev)
    jit = torch.empty(b, dtype=f64, device=dev)
    mean = torch.empty(b, q, dtype=f64, device=dev)
    status = torch.zeros(2, dtype=f64, device=dev)
    count = torch.zeros(1, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev)
    res = {}
    for mode_name, mode in (("posterior", _lib.QMC_POSTERIOR), ("chol", _lib.QMC_CHOL),
                            ("qei", _lib.QMC_QEI)):
        for fused in (False, True):
            if fused and mode == _lib.QMC_POSTERIOR:
                continue
            a = _lib.QmcFinalizeArgs(kind=cache.kind, mode=mode, B=b, q=q, Xq=pp.Xq, Spart=pp.Spart,
                                     mpart=pp.mpart, n=cache.n, outputscale=cache.outputscale,
                                     constant=cache.constant, ymean=0.0, ystd=1.0, Z=Z, S=S,
                                     max_tries=6, best_f=0.0, best_f_s=None, jitter0=1e-8,
                                     acq=acq, mean_out=mean, cov_out=None, L_out=None,
                                     info_out=info if mode else None,
                                     jitter_out=jit if mode else None, Tm=None, r=0, fat=1, ldT=0,
                                     F=None, ldF=0, tau_relu=1.0, tau_max=1.0, nparts=0,
                                     sym_parts=0, status_out=status if fused else None,
                                     status_count=count if fused else None)
            for _ in range(5):
                check(lib().bo_qmc_finalize_v(ctypes.byref(a), ctypes.c_void_p(st.cuda_stream)), "q")
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(100):
                check(lib().bo_qmc_finalize_v(ctypes.byref(a), ctypes.c_void_p(st.cuda_stream)), "q")
            e1.record(st)
            torch.cuda.synchronize()
            res[f"{mode_name}{'_status' if fused else ''}_us"] = 1e3 * e0.elapsed_time(e1) / 100
    out[tag] = res
    print(tag, json.dumps(res), flush=True)
