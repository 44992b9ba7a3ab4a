"""Drivers for the L-BFGS-B parity tests (test infrastructure).

* ``scipy_trials``: scipy.optimize.minimize(method="L-BFGS-B") -- the call
  botorch's gen_candidates_scipy makes (botorch/generation/gen.py:252-267) --
  with the objective wrapped so that every point scipy evaluates is recorded,
  in order.  That sequence (start point, then every line-search trial point)
  is what the reverse-communication state machine of
  botorch_amd/csrc/lbfgsb_core.h must reproduce.
* ``HostLbfgsb``: the single-lane host build of that state machine
  (tests/host/lbfgsb_host.cpp, compiled here with g++), driven one restart at
  a time.
"""
import ctypes
import os
import subprocess

import numpy as np
from scipy.optimize import minimize

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOST_SO = os.path.join(ROOT, "build", "lbfgsb_host.so")
_SRC = [os.path.join(ROOT, "tests", "host", "lbfgsb_host.cpp"),
        os.path.join(ROOT, "botorch_amd", "csrc", "lbfgsb_core.h")]

ST_NAMES = {1: "pgtol", 2: "ftol", 3: "abnormal", 4: "maxiter", 5: "maxfun", 6: "error"}


def build_host():
    if not os.path.exists(HOST_SO) or any(os.path.getmtime(s) > os.path.getmtime(HOST_SO)
                                          for s in _SRC):
        os.makedirs(os.path.dirname(HOST_SO), exist_ok=True)
        subprocess.run(["g++", "-O2", "-std=c++20", "-fPIC", "-shared", "-pthread", "-o", HOST_SO,
                        _SRC[0]], check=True)
    lib = ctypes.CDLL(HOST_SO)
    P = ctypes.c_void_p
    for fn in (lib.bo_lbfgsb_host_step, lib.bo_lbfgsb_host_step_lanes, lib.bo_lbfgsb_host_step_wide):
        fn.restype = ctypes.c_int
        fn.argtypes = ([ctypes.c_int] * 5 + [ctypes.c_double] * 2 + [P, P, P, ctypes.c_double]
                       + [P] * 8)
    return lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def scipy_trials(fun_and_grad, x0, bounds, maxiter=15000, maxcor=10, ftol=2.2204460492503131e-09,
                 gtol=1e-05, maxls=20, maxfun=15000):
    """(trial points evaluated by scipy in order, OptimizeResult)."""
    pts = []

    def f(x):
        pts.append(np.array(x, dtype=np.float64))
        return fun_and_grad(x)

    res = minimize(f, np.asarray(x0, dtype=np.float64), jac=True, method="L-BFGS-B",
                   bounds=bounds,
                   options=dict(maxiter=maxiter, maxcor=maxcor, ftol=ftol, gtol=gtol, maxls=maxls,
                                maxfun=maxfun))
    return pts, res


class HostLbfgsb:
    """One restart of the host build; ``run`` returns (trial points, x, f, status, nit).
    ``lanes=True``: the 64-thread emulation of the kernel's wave; ``lanes="wide"``:
    128 threads as two waves, the kernel's workgroup-wide (joint-problem) paths."""

    def __init__(self, n, m=10, maxls=20, maxiter=15000, maxfun=15000,
                 ftol=2.2204460492503131e-09, gtol=1e-05, lower=None, upper=None, lanes=False):
        self.lib = build_host()
        self._step = (self.lib.bo_lbfgsb_host_step_wide if lanes == "wide" else
                      self.lib.bo_lbfgsb_host_step_lanes if lanes else self.lib.bo_lbfgsb_host_step)
        lay = (ctypes.c_int * 6)()
        self.lib.bo_lbfgsb_host_layout(lay)
        nv, niv, nmat, nd, ni, _ = list(lay)
        self.n, self.m = n, m
        self.cfg = (maxls, maxiter, maxfun, ftol, gtol)
        self.lower = np.full(n, -np.inf) if lower is None else np.ascontiguousarray(lower, np.float64)
        self.upper = np.full(n, np.inf) if upper is None else np.ascontiguousarray(upper, np.float64)
        self.v = np.zeros(nv * n)
        self.iv = np.zeros(niv * n, dtype=np.int32)
        self.ws = np.zeros(m * n)
        self.wy = np.zeros(m * n)
        self.mat = np.zeros(nmat)
        self.ds = np.zeros(nd)
        self.is_ = np.zeros(ni, dtype=np.int32)

    def step(self, xt, f, g):
        maxls, maxiter, maxfun, ftol, gtol = self.cfg
        g = np.ascontiguousarray(g, np.float64)
        return self._step(
            self.n, self.m, maxls, maxiter, maxfun, ftol, gtol, _p(self.lower), _p(self.upper),
            _p(xt), float(f), _p(g), _p(self.v), _p(self.iv), _p(self.ws), _p(self.wy),
            _p(self.mat), _p(self.ds), _p(self.is_))

    def run(self, fun_and_grad, x0, max_evals=100000):
        xt = np.clip(np.array(x0, dtype=np.float64), self.lower, self.upper)
        pts = []
        status = 0
        for _ in range(max_evals):
            pts.append(xt.copy())
            f, g = fun_and_grad(xt.copy())
            status = self.step(xt, f, g)
            if status:
                break
        x = self.v[: self.n].copy()  # V_X
        return pts, x, self.ds[0], status, int(self.is_[10])  # D_F, I_NITER
