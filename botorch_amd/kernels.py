"""Tensor-level wrappers of the C ABI (device buffers in, device buffers out).

Every function here enqueues HIP kernels from ``libbotorch_amd.so`` on the
current torch stream of the tensors' device.  There is no CPU path: inputs
must be fp64 tensors on a ROCm device, and a missing library raises.
"""
from __future__ import annotations

import collections
import ctypes
import functools
import math
import os
from dataclasses import dataclass
from typing import Optional

import torch
from torch.quasirandom import SobolEngine

from . import _lib
from ._lib import check, lib

DP = 8  # padded input dimension of the fused posterior kernel
# Largest K*x^T workspace built per posterior call: 4 GiB, at most 1/16 of the
# device's memory, overridable with BO_KXT_MAX_BYTES (above it the posterior
# kernel evaluates the kernel rows between its MFMAs instead).
KXT_MAX_BYTES = int(os.environ.get("BO_KXT_MAX_BYTES", 4 << 30))
_KXT_CAP = {}


def kxt_cap(device: torch.device) -> int:
    """KXT_MAX_BYTES bounded by 1/16 of the device's total memory (cached per
    device; no synchronisation)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    if idx not in _KXT_CAP:
        _KXT_CAP[idx] = min(KXT_MAX_BYTES, torch.cuda.get_device_properties(idx).total_memory // 16)
    return _KXT_CAP[idx]
CHOLESKY_MAX_TRIES = 6  # botorch/__init__.py:47
CHOLESKY_JITTER_F64 = 1e-8  # [G] linear_operator.settings.cholesky_jitter (double)

# Optional callable(tag) invoked around the bo_post_partials launch (bench.py
# records HIP events on the current stream through it).
TIMING_HOOK = None
# the MLL closure's A^{-1} inside the factorisation's launch (round 5, opt-in:
# BO_MLL_AINV_DAG=1).  Measured slower than the separate bo_ainv pass: n = 4096
# factor + inverse + A^{-1} 2.25-2.28 ms in one launch against 2.11 ms as two
# (profiles/r05/ainv_fold/), so the closure keeps the two launches
AINV_IN_DAG = os.environ.get("BO_MLL_AINV_DAG", "0") == "1"


# Tensors whose pointers were handed to the C ABI most recently.  A call such as
# lib().bo_x(_p(a.contiguous()), _p(b.to(dev))) would otherwise drop each
# temporary as soon as _p returns -- before the launch is enqueued -- and the
# caching allocator could hand the same block to the next temporary of the same
# argument list.  Holding the last few references spans any one call.
_KEEPALIVE = collections.deque(maxlen=64)


def drop_keepalive() -> None:
    """Release the held references once every launch that used them is
    enqueued (or captured): the caching allocator is stream-ordered, so a
    block freed after its launch is queued is reused only behind it.  Called
    where a caller is done issuing (the end of a graph capture, of the device
    optimiser), so the deque does not pin graph-pool or large blocks."""
    _KEEPALIVE.clear()


def _p(t: Optional[torch.Tensor]):
    if t is None:
        return ctypes.c_void_p(0)
    _KEEPALIVE.append(t)
    return ctypes.c_void_p(t.data_ptr())


def _stream(device: torch.device):
    """The caller's current HIP stream on ``device`` (raw handle; the same
    stream torch.cuda.current_stream(device) wraps, without building the
    Python stream object on every launch)."""
    idx = device.index if device.index is not None else torch.cuda.current_device()
    return ctypes.c_void_p(torch._C._cuda_getCurrentRawStream(idx))


def _dev(*tensors: torch.Tensor) -> torch.device:
    dev = tensors[0].device
    for t in tensors:
        if t is None:
            continue
        if t.device.type != "cuda":
            raise RuntimeError("botorch_amd kernels need ROCm device tensors (no CPU fallback)")
        if t.dtype not in (torch.float64, torch.int64, torch.int32):
            raise TypeError(f"expected fp64 tensors, got {t.dtype}")
    return dev


def gemm(A, B, transA=False, transB=False, alpha=1.0, beta=0.0, C=None, flags=0):
    """C = alpha op(A) op(B) + beta C (2-D or batched 3-D row-major fp64)."""
    dev = _dev(A, B)
    batched = A.dim() == 3
    A3 = A if batched else A.unsqueeze(0)
    B3 = B if batched else B.unsqueeze(0)
    A3, B3 = A3.contiguous(), B3.contiguous()
    M = A3.shape[2] if transA else A3.shape[1]
    K = A3.shape[1] if transA else A3.shape[2]
    N = B3.shape[1] if transB else B3.shape[2]
    batch = A3.shape[0]
    if C is None:
        # every element is written when beta = 0 (no fill launch); a lower-
        # triangular result leaves the upper part to the zeros
        alloc = torch.zeros if flags & _lib.GEMM_LOWER_C else torch.empty
        C3 = alloc(batch, M, N, dtype=torch.float64, device=dev)
        beta = 0.0
    else:
        C3 = C if batched else C.unsqueeze(0)
    check(lib().bo_gemm_f64(int(transA), int(transB), M, N, K, alpha, _p(A3), A3.shape[2],
                            A3.stride(0), _p(B3), B3.shape[2], B3.stride(0), beta, _p(C3),
                            C3.shape[2], C3.stride(0), batch, flags, _stream(dev)), "gemm")
    return C3 if batched else C3.squeeze(0)


def gemm_strided(M, N, K, A, lda, sA, B, ldb, sB, C, ldc, sC, batch, alpha=1.0, beta=0.0,
                 transA=False, transB=False, flags=0):
    """Raw strided batched GEMM on tensors' storage (views with custom strides,
    e.g. per-t-batch column blocks of a padded matrix)."""
    dev = _dev(A, B, C)
    check(lib().bo_gemm_f64(int(transA), int(transB), M, N, K, alpha, _p(A), lda, sA, _p(B), ldb,
                            sB, beta, _p(C), ldc, sC, batch, flags, _stream(dev)), "gemm_strided")
    return C


def covar_matrix(X1, X2, lengthscale, kind=_lib.RBF, outputscale=1.0, diag_add=0.0, out=None):
    dev = _dev(X1, X2, lengthscale)
    n1, d = X1.shape
    n2 = X2.shape[0]
    K = out if out is not None else torch.empty(n1, n2, dtype=torch.float64, device=dev)
    if tuple(K.shape) != (n1, n2) or not K.is_contiguous():
        raise ValueError("covar_matrix: out must be a contiguous n1 x n2 fp64 tensor")
    check(lib().bo_covar_matrix(kind, _p(X1.contiguous()), n1, _p(X2.contiguous()), n2, d,
                                _p(lengthscale.contiguous()), outputscale, diag_add, 0, _p(K),
                                n2, n1, n2, _stream(dev)), "covar_matrix")
    return K


def covar_batched(kind, X1, s1, n1, X2, s2, n2, d, ls, sl, os_, so, K, sK, ldk, outer, inner):
    """bo_covar_batched on raw storage: every stride argument is an (outer, inner)
    pair of element strides."""
    dev = _dev(X1, X2, ls, os_, K)
    check(lib().bo_covar_batched(kind, _p(X1), s1[0], s1[1], n1, _p(X2), s2[0], s2[1], n2, d,
                                 _p(ls), sl[0], sl[1], _p(os_), so[0], so[1], _p(K), sK[0], sK[1],
                                 ldk, outer, inner, _stream(dev)), "covar_batched")
    return K


def padded_order(n: int) -> int:
    return int(lib().bo_padded_order(n))


def cholesky_inverse(A: torch.Tensor):
    """Lower Cholesky factor and its inverse of an SPD matrix (np x np, np % 128 == 0
    handled by padding with identity).  Returns (L, Linv, info)."""
    dev = _dev(A)
    n = A.shape[0]
    np_ = padded_order(n)
    W = torch.eye(np_, dtype=torch.float64, device=dev)
    W[:n, :n] = torch.tril(A)
    Linv = torch.empty_like(W)
    work = torch.empty_like(W)
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    check(lib().bo_cholesky_inverse(_p(W), _p(Linv), _p(work), np_, _p(info), _stream(dev)),
          "cholesky_inverse")
    status = int(info.item())
    if status < 0:
        raise RuntimeError("bo_cholesky_inverse: the Cholesky task DAG timed out")
    return W[:n, :n], Linv[:n, :n], status


@dataclass
class GPCache:
    """Device-resident exact-GP prediction caches ([G] DefaultPredictionStrategy)."""
    kind: int
    n: int
    d: int
    np: int
    Xt: torch.Tensor           # n x d raw training inputs
    Xt_scaled: torch.Tensor    # n x 8, divided by the lengthscale (zero padded)
    lengthscale: torch.Tensor  # d
    outputscale: float
    noise: float
    constant: float
    L: torch.Tensor            # np x np lower Cholesky factor of K + s2 I (+ jitter)
    Linv: torch.Tensor         # np x np
    U: torch.Tensor            # np x np = L^{-T}  (covar_cache)
    beta: torch.Tensor         # n  = L^{-1} (y - c)
    alpha: torch.Tensor        # n  = (K + s2 I)^{-1} (y - c)  (mean_cache)
    jitter: float
    # A^{-1} lower 64 x 64 tiles when the factorisation's launch formed it (the
    # MLL closure, bo_cholesky_inverse_ainv), else None (kernels.ainv forms it)
    Ainv: Optional[torch.Tensor] = None


def build_gp_cache(Xt, y, lengthscale, noise, constant, kind=_lib.RBF, outputscale=1.0,
                   max_tries=CHOLESKY_MAX_TRIES, jitter0=CHOLESKY_JITTER_F64,
                   check_nan: bool = True) -> GPCache:
    """``check_nan=False``: the caller has already checked Xt and y (the MLL
    closure checks once per fit, not once per evaluation: each check is a
    device-to-host sync)."""
    dev = _dev(Xt, y, lengthscale)
    Xt = Xt.contiguous()
    n, d = Xt.shape
    if check_nan and (torch.isnan(Xt).any() or torch.isnan(y).any()):
        from .exceptions import NanError
        raise NanError("training data contains NaN")
    np_ = padded_order(n)
    f64 = dict(dtype=torch.float64, device=dev)
    L = torch.empty(np_, np_, **f64)
    Linv = torch.empty(np_, np_, **f64)
    U = torch.empty(np_, np_, **f64)
    beta = torch.empty(n, **f64)
    alpha = torch.empty(n, **f64)
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    jit = ctypes.c_double(0.0)
    ls = lengthscale.detach().reshape(-1).contiguous()
    st = _stream(dev)
    if torch.is_tensor(noise) and noise.numel() > 1:
        # fixed-noise likelihood: one observed variance per training point
        nv = noise.detach().reshape(-1).to(**f64).contiguous()
        if nv.numel() != n:
            raise ValueError(f"fixed noise has {nv.numel()} entries for {n} training points")
        check(lib().bo_gp_cache_build_fixed(kind, _p(Xt), n, d, _p(ls), float(outputscale),
                                            _p(nv), float(constant), _p(y.contiguous()), _p(L),
                                            _p(Linv), _p(U), _p(beta), _p(alpha), max_tries,
                                            jitter0, ctypes.byref(jit), _p(info), st),
              "gp_cache_build_fixed")
        noise = float(nv.mean())
    else:
        check(lib().bo_gp_cache_build(kind, _p(Xt), n, d, _p(ls), float(outputscale),
                                      float(noise), float(constant), _p(y.contiguous()), _p(L),
                                      _p(Linv), _p(U), _p(beta), _p(alpha), max_tries, jitter0,
                                      ctypes.byref(jit), _p(info), st), "gp_cache_build")
    if jit.value > 0:
        import warnings
        from .exceptions import NumericalWarning
        warnings.warn(f"A not p.d., added jitter of {jit.value:.1e} to the diagonal",
                      NumericalWarning)
    Xs = torch.empty(n, DP, **f64)
    if d <= DP:
        check(lib().bo_scale_inputs(_p(Xt), n, d, _p(ls), ctypes.c_void_p(0), DP, _p(Xs), st),
              "scale_inputs")
    return GPCache(kind, n, d, np_, Xt, Xs, ls, float(outputscale), float(noise),
                   float(constant), L, Linv, U, beta, alpha, jit.value)


def cholesky_inverse_batched(As: torch.Tensor):
    """L = chol(A_m), Linv = L^{-1} of nb SPD matrices (nb x n x n) in ONE
    persistent DAG launch (bo_cholesky_inverse_batched; bit-identical to nb
    cholesky_inverse calls).  Returns (L, Linv, info list)."""
    dev = _dev(As)
    nb, n = As.shape[0], As.shape[-1]
    np_ = padded_order(n)
    W = torch.eye(np_, dtype=torch.float64, device=dev).repeat(nb, 1, 1)
    W[:, :n, :n] = torch.tril(As)
    Linv = torch.empty_like(W)
    T = np_ // 64
    work = torch.empty((16 + 4 * nb * T * T + 3) // 4 * 2, dtype=torch.float64, device=dev)
    info = torch.zeros(nb, dtype=torch.int32, device=dev)
    check(lib().bo_cholesky_inverse_batched(_p(W), _p(Linv), _p(work), nb, np_, _p(info),
                                            _stream(dev)), "cholesky_inverse_batched")
    status = info.cpu().tolist()
    if any(s_ < 0 for s_ in status):
        raise RuntimeError("bo_cholesky_inverse_batched: the Cholesky task DAG timed out")
    return W[:, :n, :n], Linv[:, :n, :n], status


def build_gp_cache_optimistic(Xt, y, lengthscale, noise: float, constant: float, kind=_lib.RBF,
                              outputscale=1.0):
    """The first (jitter-free) attempt of build_gp_cache, enqueued without a
    status read-back: returns (cache, info) with info a device int that the
    caller reads together with its own results (the MLL closure: one
    device-to-host transfer per evaluation).  info != 0 means K + s2 I was not
    p.d. without jitter and the cache is invalid: the caller then reruns
    build_gp_cache, whose ladder starts from jitter 0 as the reference's
    psd_safe_cholesky does."""
    dev = _dev(Xt, y, lengthscale)
    Xt = Xt.contiguous()
    y = y.contiguous()
    n, d = Xt.shape
    np_ = padded_order(n)
    f64 = dict(dtype=torch.float64, device=dev)
    L = torch.empty(np_, np_, **f64)
    Linv = torch.empty(np_, np_, **f64)
    # A^{-1} in the factorisation's own launch with BO_MLL_AINV_DAG=1 (opt-in,
    # see AINV_IN_DAG); by default the separate bo_ainv pass in mll_terms
    Ainv = torch.empty(np_, np_, **f64) if AINV_IN_DAG else None
    # the DAG's tile counters (5 (np/64)^2 + 16 ints) and alpha's chunk partials;
    # the MLL closure forms no U = L^{-T} (alpha from L^{-1}'s columns)
    T = np_ // 64
    we = ctypes.c_int64()
    check(lib().bo_gemv_lt_work(n, ctypes.byref(we)), "gemv_lt_work")
    work = torch.empty(max((16 + 5 * T * T + 1) // 2, we.value), **f64)
    beta = torch.empty(n, **f64)
    alpha = torch.empty(n, **f64)
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    ls = lengthscale.detach().reshape(-1).to(**f64).contiguous()
    st = _stream(dev)
    check(lib().bo_covar_matrix(kind, _p(Xt), n, _p(Xt), n, d, _p(ls), float(outputscale),
                                float(noise), 1, _p(L), np_, np_, np_, st), "covar_matrix")
    if Ainv is not None:
        check(lib().bo_cholesky_inverse_ainv(_p(L), _p(Linv), _p(Ainv), _p(work), np_, _p(info),
                                             st), "cholesky_inverse_ainv")
    else:
        check(lib().bo_cholesky_inverse(_p(L), _p(Linv), _p(work), np_, _p(info), st),
              "cholesky_inverse")
    check(lib().bo_gemv_tri(_p(Linv), np_, n, _p(y), float(constant), _p(beta), 1, st),
          "gemv_tri")
    check(lib().bo_gemv_lt(_p(Linv), np_, n, _p(beta), 0.0, _p(alpha), _p(work), st), "gemv_lt")
    U = Linv.new_empty(0)  # not formed (no posterior is taken from this cache)
    Xs = torch.empty(n, DP, **f64)
    if d <= DP:
        check(lib().bo_scale_inputs(_p(Xt), n, d, _p(ls), ctypes.c_void_p(0), DP, _p(Xs), st),
              "scale_inputs")
    cache = GPCache(kind, n, d, np_, Xt, Xs, ls, float(outputscale), float(noise),
                    float(constant), L, Linv, U, beta, alpha, 0.0, Ainv)
    return cache, info


def build_gp_caches(specs, check_nan: bool = True):
    """GPCaches of several exact GPs whose training sets pad to one order (the
    outputs of a batched multi-output SingleTaskGP, a ModelListGP's members):
    their covariances are built side by side and factorised in ONE
    bo_cholesky_inverse_batched launch, with one status read-back for all.  A
    member whose first factorisation fails runs the jitter ladder on its own
    (build_gp_cache: the reference's psd_safe_cholesky sequence from jitter 0).
    Results are bit-identical to build_gp_cache per member.  specs: dicts of
    build_gp_cache's arguments (Xt, y, lengthscale, noise, constant, kind,
    outputscale); fixed-noise members, unequal orders or members on different
    devices fall back to build_gp_cache per member."""
    specs = list(specs)
    if not specs:
        return []
    nps = {padded_order(sp["Xt"].shape[0]) for sp in specs}
    devs = {sp["Xt"].device for sp in specs}
    fixed = any(torch.is_tensor(sp["noise"]) and sp["noise"].numel() > 1 for sp in specs)
    if len(specs) == 1 or len(nps) != 1 or len(devs) != 1 or fixed or len(specs) > 128:
        return [build_gp_cache(check_nan=check_nan, **sp) for sp in specs]
    dev = _dev(specs[0]["Xt"])
    np_ = nps.pop()
    nb = len(specs)
    f64 = dict(dtype=torch.float64, device=dev)
    Lb = torch.empty(nb, np_, np_, **f64)
    Linvb = torch.empty(nb, np_, np_, **f64)
    T = np_ // 64
    work = torch.empty((16 + 4 * nb * T * T + 3) // 4 * 2, **f64)
    info = torch.zeros(nb, dtype=torch.int32, device=dev)
    st = _stream(dev)
    prep = []
    for m, sp in enumerate(specs):
        Xt = sp["Xt"].contiguous()
        y = sp["y"].contiguous()
        n, d = Xt.shape
        if check_nan and (torch.isnan(Xt).any() or torch.isnan(y).any()):
            from .exceptions import NanError
            raise NanError("training data contains NaN")
        ls = sp["lengthscale"].detach().reshape(-1).to(**f64).contiguous()
        kind = sp.get("kind", _lib.RBF)
        os_ = float(sp.get("outputscale", 1.0))
        check(lib().bo_covar_matrix(kind, _p(Xt), n, _p(Xt), n, d, _p(ls), os_, float(sp["noise"]),
                                    1, _p(Lb[m]), np_, np_, np_, st), "covar_matrix")
        prep.append((Xt, y, ls, kind, os_, n, d))
    check(lib().bo_cholesky_inverse_batched(_p(Lb), _p(Linvb), _p(work), nb, np_, _p(info), st),
          "cholesky_inverse_batched")
    status = info.cpu().tolist()  # the one read-back for all members
    if any(s_ < 0 for s_ in status):
        raise RuntimeError("bo_cholesky_inverse_batched: the Cholesky task DAG timed out")
    out = []
    for m, (sp, (Xt, y, ls, kind, os_, n, d)) in enumerate(zip(specs, prep)):
        if status[m] != 0:  # not p.d. without jitter: the member's own ladder
            out.append(build_gp_cache(check_nan=False, **sp))
            continue
        L, Linv = Lb[m], Linvb[m]
        U = torch.empty(np_, np_, **f64)
        beta = torch.empty(n, **f64)
        alpha = torch.empty(n, **f64)
        c = float(sp["constant"])
        check(lib().bo_transpose(_p(Linv), _p(U), np_, np_, st), "transpose")
        check(lib().bo_gemv_tri(_p(Linv), np_, n, _p(y), c, _p(beta), 1, st), "gemv_tri")
        we = ctypes.c_int64()
        check(lib().bo_gemv_lt_work(n, ctypes.byref(we)), "gemv_lt_work")
        wlt = torch.empty(max(1, we.value), **f64)
        check(lib().bo_gemv_lt(_p(Linv), np_, n, _p(beta), 0.0, _p(alpha), _p(wlt), st),
              "gemv_lt")  # alpha = L^{-T} beta, as bo_gp_cache_build
        Xs = torch.empty(n, DP, **f64)
        if d <= DP:
            check(lib().bo_scale_inputs(_p(Xt), n, d, _p(ls), ctypes.c_void_p(0), DP, _p(Xs), st),
                  "scale_inputs")
        out.append(GPCache(kind, n, d, np_, Xt, Xs, ls, os_, float(sp["noise"]), c, L, Linv, U,
                           beta, alpha, 0.0))
    return out


@dataclass
class PostPartials:
    B: int
    q: int
    Qp: int
    nrows_pad: int
    nC: int
    Xq: torch.Tensor
    Spart: torch.Tensor
    mpart: torch.Tensor
    # R^T on the gradient path: nC*128 x nrows_pad row-major, or blocked
    # (nC*8 x nrows_pad/16 x 256, rt_layout=RT_BLOCKED) for the fused W -> dX pass
    Rt: Optional[torch.Tensor] = None
    Cx: Optional[torch.Tensor] = None  # cross K*x^T (rq x nrows_pad), fused cross term


@functools.lru_cache(maxsize=256)
def geometry(B: int, q: int, n: int):
    Qp, nrows, nC = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
    check(lib().bo_post_geometry(B, q, n, ctypes.byref(Qp), ctypes.byref(nrows),
                                 ctypes.byref(nC)), "post_geometry")
    return Qp.value, nrows.value, nC.value


def ainv(cache: "GPCache") -> torch.Tensor:
    """A^{-1} = L^{-T} L^{-1} (np x np; the lower tiles -- tile row >= tile
    column, diagonal tiles whole -- are written) by bo_ainv."""
    dev = cache.Linv.device
    out = torch.empty(cache.np, cache.np, dtype=torch.float64, device=dev)
    we = ctypes.c_int64()
    check(lib().bo_ainv_work(cache.n, ctypes.byref(we)), "ainv_work")
    work = torch.empty(max(1, we.value), dtype=torch.float64, device=dev)
    check(lib().bo_ainv(_p(cache.Linv), cache.np, cache.n, _p(out), _p(work), _stream(dev)), "ainv")
    return out


@functools.lru_cache(maxsize=256)
def quad_pairs(B: int, q: int, n: int) -> int:
    """Partials of the quad plan (bo_post_quad_plan: chunks of A^{-1} block
    pairs) at this geometry; 0 where the posterior keeps the R route."""
    npairs = ctypes.c_int()
    check(lib().bo_post_quad_plan(B, q, n, ctypes.byref(npairs)), "post_quad_plan")
    return npairs.value


def quad_ainv(cache: "GPCache", B: int, q: int) -> Optional[torch.Tensor]:
    """The full symmetric A^{-1} (np x np) of ``cache`` when the quad plan
    applies to (B, q, n) -- built once per cache (bo_ainv + bo_sym_lower) --
    else None."""
    if B == 0 or quad_pairs(B, q, cache.n) == 0:
        return None
    A = getattr(cache, "_ainv_full", None)
    if A is None:
        A = ainv(cache)
        check(lib().bo_sym_lower(_p(A), cache.np, cache.np, _stream(A.device)), "sym_lower")
        cache._ainv_full = A
    return A


@functools.lru_cache(maxsize=256)
def split_plan(B: int, q: int, n: int, slots: int = 0):
    """(kc_len, workspace doubles) of the posterior plan; kc_len = 0: one pass,
    -1: stream-K."""
    kc, we = ctypes.c_int(), ctypes.c_int64()
    check(lib().bo_post_split_plan(B, q, n, slots, ctypes.byref(kc), ctypes.byref(we)),
          "post_split_plan")
    return kc.value, we.value


@functools.lru_cache(maxsize=256)
def rt_blocked_plan(B: int, q: int, n: int) -> bool:
    """Whether the fused forward (bo::qmc_acq_native) stores R^T blocked for
    (B, q, n): the one-pass grid of the fused W -> dX backward.  Shape metadata
    only (the op's fake): the real layout travels with the tensor's shape."""
    we = ctypes.c_int64()
    check(lib().bo_post_w_dx_work(B, q, n, ctypes.byref(we)), "post_w_dx_work")
    return we.value > 0 and split_plan(B, q, n)[0] == 0


def small_plan(B: int, q: int, n: int) -> int:
    """Pair partials per 16-row tile of the small-grid posterior
    (bo_post_small_plan), 0 where the 128-tile plan is kept."""
    v = ctypes.c_int()
    check(lib().bo_post_small_plan(B, q, n, ctypes.byref(v)), "post_small_plan")
    return v.value


def post_partials_members(caches, X: torch.Tensor, store_R: bool = False) -> list:
    """post_partials of one X under several models of one shape (a
    ModelListGP's members, models/gpytorch.py:629-726): every member's K*x^T
    in one launch, then ONE launch for all members' partials -- the
    small-grid kernel where its plan applies, the member-batched stream-K
    128-tile kernel where the one-model plan is stream-K (C4: three outputs);
    elsewhere one post_partials per member."""
    c0 = caches[0]
    B, q, d = X.shape
    same = all(c.n == c0.n and c.np == c0.np and c.d == c0.d for c in caches)
    nparts = small_plan(B, q, c0.n) if same and 1 < len(caches) <= 8 else 0
    fits = c0.np * geometry(B, q, c0.n)[1] * 8 <= kxt_cap(_dev(X))
    if nparts == 0 and same and 1 < len(caches) <= 8 and fits and MEMBERS_STREAMK:
        we = ctypes.c_int64()
        check(lib().bo_post_members_work(len(caches), B, q, c0.n, ctypes.byref(we)),
              "post_members_work")
        if we.value >= 0:
            return _post_members_streamk(caches, X, store_R, we.value)
    if nparts == 0 or not fits:
        return [post_partials(c, X, store_R=store_R) for c in caches]
    dev = _dev(X)
    Qp, nrows_pad, nC = geometry(B, q, c0.n)
    f64 = dict(dtype=torch.float64, device=dev)
    st = _stream(dev)
    Xc = X.contiguous()
    pps, ptrs = [], {k: [] for k in ("Kt", "U", "beta", "S", "m", "Rt")}
    Xqs, Kts = _kxt_rows_members(caches, Xc, nrows_pad)
    Rt_all = torch.empty(len(caches), nC * 128, nrows_pad, **f64) if store_R else None
    for m_, (c, Xq, Kt) in enumerate(zip(caches, Xqs, Kts)):
        Sp = torch.empty(nparts, nrows_pad // 16, 16, 16, **f64)
        mp = torch.empty(nparts, nrows_pad, **f64)
        Rt = Rt_all[m_] if store_R else None
        pps.append(PostPartials(B, q, Qp, nrows_pad, nC, Xq, Sp, mp, Rt))
        for k, t in (("Kt", Kt), ("U", c.U), ("beta", c.beta), ("S", Sp), ("m", mp), ("Rt", Rt)):
            ptrs[k].append(_p(t).value if t is not None else None)
    nm = len(caches)
    arr = {k: (ctypes.c_void_p * nm)(*v) for k, v in ptrs.items()}
    if TIMING_HOOK is not None:
        TIMING_HOOK("post_partials_begin")
    check(lib().bo_post_small_batched(nm, arr["Kt"], arr["U"], arr["beta"], arr["S"], arr["m"],
                                      arr["Rt"], B, q, c0.n, c0.np, st), "post_small_batched")
    if TIMING_HOOK is not None:
        TIMING_HOOK("post_partials_end")
    return pps


def _kxt_rows_members(caches, Xc: torch.Tensor, nrows_pad: int):
    """Every member's padded rows and K*x^T from one X: one launch where the
    members share the kernel kind (bo_post_kxt_rows_members), else one each."""
    dev = _dev(Xc)
    B, q, d = Xc.shape
    f64 = dict(dtype=torch.float64, device=dev)
    st = _stream(dev)
    Xqs = [torch.empty(nrows_pad, DP, **f64) for _ in caches]
    Kts = [torch.empty(c.np, nrows_pad, **f64) for c in caches]
    nm = len(caches)
    if nm <= 8 and all(c.kind == caches[0].kind for c in caches):
        P = ctypes.c_void_p * nm
        os_ = (ctypes.c_double * nm)(*[float(c.outputscale) for c in caches])
        check(lib().bo_post_kxt_rows_members(nm, caches[0].kind, _p(Xc), B, q, d,
                                             P(*[_p(c.lengthscale).value for c in caches]),
                                             P(*[_p(c.Xt_scaled).value for c in caches]), os_,
                                             caches[0].n, P(*[_p(t).value for t in Xqs]),
                                             P(*[_p(t).value for t in Kts]), st),
              "post_kxt_rows_members")
    else:
        for c, Xq, Kt in zip(caches, Xqs, Kts):
            check(lib().bo_post_kxt_rows(c.kind, _p(Xc), B, q, d, _p(c.lengthscale),
                                         _p(c.Xt_scaled), c.n, c.outputscale, _p(Xq), _p(Kt), st),
                  "post_kxt_rows")
    return Xqs, Kts


# BO_POST_MEMBERS=0: one stream-K launch per member instead (A/B knob)
MEMBERS_STREAMK = os.environ.get("BO_POST_MEMBERS", "1") != "0"


def _post_members_streamk(caches, X: torch.Tensor, store_R: bool, work_elems: int) -> list:
    """post_partials_members on the 128-tile kernel: every member's K*x^T,
    then ONE member-batched stream-K launch + one reduction
    (bo_post_partials_members); nC column-tile partials per member."""
    c0 = caches[0]
    dev = _dev(X)
    B, q, d = X.shape
    Qp, nrows_pad, nC = geometry(B, q, c0.n)
    f64 = dict(dtype=torch.float64, device=dev)
    st = _stream(dev)
    Xc = X.contiguous()
    pps, ptrs = [], {k: [] for k in ("Kt", "U", "beta", "S", "m", "Rt")}
    Xqs, Kts = _kxt_rows_members(caches, Xc, nrows_pad)
    # the members' R^T stacked (M x np x nrows_pad): slices per member, and
    # batched GEMMs over all members read it as one operand (qNEHVI)
    Rt_all = torch.empty(len(caches), nC * 128, nrows_pad, **f64) if store_R else None
    for m_, (c, Xq, Kt) in enumerate(zip(caches, Xqs, Kts)):
        Sp = torch.empty(nC, nrows_pad // 16, 16, 16, **f64)
        mp = torch.empty(nC, nrows_pad, **f64)
        Rt = Rt_all[m_] if store_R else None
        pps.append(PostPartials(B, q, Qp, nrows_pad, nC, Xq, Sp, mp, Rt))
        for k, t in (("Kt", Kt), ("U", c.U), ("beta", c.beta), ("S", Sp), ("m", mp), ("Rt", Rt)):
            ptrs[k].append(_p(t).value if t is not None else None)
    nm = len(caches)
    arr = {k: (ctypes.c_void_p * nm)(*v) for k, v in ptrs.items()}
    work = torch.empty(max(1, work_elems), **f64)
    if TIMING_HOOK is not None:
        TIMING_HOOK("post_partials_begin")
    check(lib().bo_post_partials_members(nm, arr["Kt"], arr["U"], arr["beta"], arr["S"], arr["m"],
                                         arr["Rt"] if store_R else None, _p(pps[0].Xq), B, q, c0.n,
                                         c0.np, _p(work), st), "post_partials_members")
    if TIMING_HOOK is not None:
        TIMING_HOOK("post_partials_end")
    return pps


def _post_small_one(cache: GPCache, X: torch.Tensor, store_R: bool) -> PostPartials:
    """post_partials on the small-grid kernel, one model."""
    dev = _dev(X)
    B, q, d = X.shape
    Qp, nrows_pad, nC = geometry(B, q, cache.n)
    nparts = small_plan(B, q, cache.n)
    f64 = dict(dtype=torch.float64, device=dev)
    st = _stream(dev)
    Xq = torch.empty(nrows_pad, DP, **f64)
    Kt = torch.empty(cache.np, nrows_pad, **f64)
    check(lib().bo_post_kxt_rows(cache.kind, _p(X.contiguous()), B, q, d, _p(cache.lengthscale),
                                 _p(cache.Xt_scaled), cache.n, cache.outputscale, _p(Xq), _p(Kt),
                                 st), "post_kxt_rows")
    Sp = torch.empty(nparts, nrows_pad // 16, 16, 16, **f64)
    mp = torch.empty(nparts, nrows_pad, **f64)
    Rt = torch.empty(nC * 128, nrows_pad, **f64) if store_R else None
    if TIMING_HOOK is not None:
        TIMING_HOOK("post_partials_begin")
    check(lib().bo_post_small(_p(Kt), B, q, cache.n, _p(cache.U), cache.np, _p(cache.beta), _p(Sp),
                              _p(mp), _p(Rt), st), "post_small")
    if TIMING_HOOK is not None:
        TIMING_HOOK("post_partials_end")
    return PostPartials(B, q, Qp, nrows_pad, nC, Xq, Sp, mp, Rt)


def post_partials(cache: GPCache, X: torch.Tensor, store_R: bool = False,
                  split: Optional[int] = None, cross: Optional[torch.Tensor] = None,
                  kxt: Optional[bool] = None, rt_layout: int = 0,
                  small: Optional[bool] = None) -> PostPartials:
    """Column-tile partials of R R^T and R beta for X (B x q x d).  ``split``:
    None = the library's plan, 0 = one pass, k > 0 = chunks of k rows,
    -1 = stream-K (equal k-step shares over the resident slots).
    ``cross`` (rq <= 16 rows x >= n): also return pp.Cx = cross K*x^T
    (rq x nrows_pad) from the same pass -- on one-pass plans only; under a
    split-k plan pp.Cx is None and R^T is stored instead.  ``kxt``: build
    K*x^T first and read it in the posterior kernel (None: when it fits
    kxt_cap).  ``rt_layout``: _lib.RT_BLOCKED stores R^T in the blocked
    layout bo_post_w_dx reads (one-pass plans only).  ``small``: None = the
    small-grid plan (bo_post_small) where the library takes it and nothing
    above asks for the 128-tile kernel (no cross term, library split plan,
    row-major R^T, K*x^T within the cap); False = never (the bo::post_partials
    op, whose schema has nC partials)."""
    dev = _dev(X)
    B, q, d = X.shape
    if d != cache.d:
        raise ValueError(f"X has d={d}, model has d={cache.d}")
    Qp, nrows_pad, nC = geometry(B, q, cache.n)
    f64 = dict(dtype=torch.float64, device=dev)
    if (small is not False and cross is None and split is None and rt_layout == 0
            and kxt is not False and cache.np * nrows_pad * 8 <= kxt_cap(dev)
            and small_plan(B, q, cache.n) > 0):
        return _post_small_one(cache, X, store_R)
    Xq = torch.empty(nrows_pad, DP, **f64)
    Spart = torch.empty(nC, nrows_pad // 16, 16, 16, **f64)
    mpart = torch.empty(nC, nrows_pad, **f64)
    st = _stream(dev)
    check(lib().bo_prepare_rows(_p(X.contiguous()), B, q, d, _p(cache.lengthscale), _p(Xq), st),
          "prepare_rows")
    Rt = torch.empty(nC * 128, nrows_pad, **f64) if store_R else None
    if split is None:
        kc_len, work_elems = split_plan(B, q, cache.n)
    elif split != 0:
        kc_len = int(split)
        we = ctypes.c_int64()
        check(lib().bo_post_split_work(B, q, cache.n, kc_len, ctypes.byref(we)), "post_split_work")
        work_elems = we.value
    else:
        kc_len, work_elems = 0, 0
    work = torch.empty(work_elems, **f64) if kc_len else None
    # K*x^T built once and read by every column tile (instead of re-evaluating
    # the kernel there), within a memory cap
    Kt = None
    if kxt is None:
        kxt = cache.np * nrows_pad * 8 <= kxt_cap(dev)
    if kxt:
        Kt = torch.empty(cache.np, nrows_pad, **f64)
        check(lib().bo_post_kxt(cache.kind, _p(Xq), B, q, d, _p(cache.Xt_scaled), cache.n,
                                cache.outputscale, _p(Kt), st), "post_kxt")
    Cx = None
    if cross is not None and cross.shape[0] <= 16 and kc_len == 0:
        cross = cross.contiguous()
        Cx = torch.empty(nC, cross.shape[0], nrows_pad, **f64)  # column-tile partials
    elif cross is not None and Rt is None:
        Rt = torch.empty(nC * 128, nrows_pad, **f64)  # the caller forms the cross term from R^T
    if TIMING_HOOK is not None:
        TIMING_HOOK("post_partials_begin")
    a = _lib.PostPartialsArgs(kind=cache.kind, B=B, q=q, d=d, Xq=Xq, Xt_scaled=cache.Xt_scaled,
                              n=cache.n, U=cache.U, ldu=cache.np, beta=cache.beta,
                              outputscale=cache.outputscale, Spart=Spart, mpart=mpart, Rt=Rt,
                              kc_len=kc_len, work=work, Qc=cross if Cx is not None else None,
                              rq=cross.shape[0] if Cx is not None else 0,
                              ldq=cross.shape[1] if Cx is not None else 0, Cx=Cx, Kt=Kt,
                              rt_layout=int(rt_layout))
    check(lib().bo_post_partials_v(ctypes.byref(a), st), "post_partials")
    if TIMING_HOOK is not None:
        TIMING_HOOK("post_partials_end")
    if Rt is not None and rt_layout == _lib.RT_BLOCKED:
        Rt = Rt.view(nC * 8, nrows_pad // 16, 256)  # the layout travels with the shape
    return PostPartials(B, q, Qp, nrows_pad, nC, Xq, Spart, mpart, Rt,
                        Cx.sum(dim=0) if Cx is not None else None)


def qmc_finalize(cache: GPCache, pp: PostPartials, mode: int, ymean: float, ystd: float,
                 Z: Optional[torch.Tensor] = None, best_f: float = 0.0,
                 best_f_s: Optional[torch.Tensor] = None, want_mean=True, want_cov=True,
                 want_L=False, max_tries=CHOLESKY_MAX_TRIES, jitter0=CHOLESKY_JITTER_F64,
                 T: Optional[torch.Tensor] = None, F: Optional[torch.Tensor] = None,
                 log_params: Optional[tuple] = None, mean_out: Optional[torch.Tensor] = None,
                 L_out: Optional[torch.Tensor] = None, status=None):
    """log_params = (fat, tau_relu, tau_max) for the qLogEI / qLogNEI modes.
    mean_out / L_out: contiguous B x q / B x q x q buffers to write instead of
    fresh ones (a ModelListGP's members straight into their stacked slices).
    status: (status_out, status_count) device pointers the launch folds the
    ladder's [max info, max jitter] into (pinned_status().arm)."""
    dev = pp.Xq.device
    B, q = pp.B, pp.q
    f64 = dict(dtype=torch.float64, device=dev)
    for t, shp in ((mean_out, (B, q)), (L_out, (B, q, q))):
        if t is not None and (tuple(t.shape) != shp or not t.is_contiguous() or t.dtype != torch.float64):
            raise ValueError(f"qmc_finalize: output buffer must be contiguous fp64 {shp}")
    mean = (mean_out if mean_out is not None else torch.empty(B, q, **f64)) if want_mean else None
    cov = torch.empty(B, q, q, **f64) if want_cov else None
    L = (L_out if L_out is not None else torch.empty(B, q, q, **f64)) if want_L else None
    need_mc = mode in (_lib.QMC_QEI, _lib.QMC_QNEI) + _lib.LOG_MODES
    fat, tau_relu, tau_max = log_params if log_params is not None else (1, 1.0, 1.0)
    acq = torch.empty(B, **f64) if need_mc else None
    info = torch.empty(B, dtype=torch.int32, device=dev) if mode != _lib.QMC_POSTERIOR else None
    jit = torch.empty(B, **f64) if mode != _lib.QMC_POSTERIOR else None
    S = Z.shape[0] if Z is not None else 0
    if Z is not None:
        Z = Z.reshape(S, q).contiguous()
    a = _lib.QmcFinalizeArgs(kind=cache.kind, mode=mode, B=B, q=q, Xq=pp.Xq, Spart=pp.Spart,
                             mpart=pp.mpart, n=cache.n, outputscale=cache.outputscale,
                             constant=cache.constant, ymean=float(ymean), ystd=float(ystd), Z=Z,
                             S=S, max_tries=max_tries, best_f=float(best_f), best_f_s=best_f_s,
                             jitter0=jitter0, acq=acq, mean_out=mean, cov_out=cov, L_out=L,
                             info_out=info, jitter_out=jit, Tm=T,
                             r=T.shape[0] if T is not None else 0, fat=int(bool(fat)),
                             ldT=T.shape[1] if T is not None else 0, F=F,
                             ldF=F.shape[1] if F is not None else 0, tau_relu=float(tau_relu),
                             tau_max=float(tau_max), nparts=int(pp.Spart.shape[0]),
                             status_out=status[0] if status else None,
                             status_count=status[1] if status else None)
    check(lib().bo_qmc_finalize_v(ctypes.byref(a), _stream(dev)), "qmc_finalize")
    return dict(acq=acq, mean=mean, cov=cov, L=L, info=info, jitter=jit)


def qmc_finalize_members(caches, pps, stats, mean: torch.Tensor, L: torch.Tensor, status=None,
                         Ts=None, F: Optional[torch.Tensor] = None):
    """Root-only finalisation (QMC_CHOL: mean + jittered q x q root) of a
    ModelListGP's members in ONE launch (bo_qmc_finalize_members): member t's
    mean / root into mean[t] / L[t] (M x B x q / M x B x q x q, contiguous);
    ``status``: per member (status_out, status_count) pointers
    (pinned_status().arm); ``Ts`` / ``F``: the cached-root qNEHVI terms (T_t
    r x nrows_pad, F[t] S x nrows_pad).  Returns (info, jitter), M x B."""
    M = len(caches)
    c0, p0 = caches[0], pps[0]
    B, q = p0.B, p0.q
    dev = mean.device
    info = torch.empty(M, B, dtype=torch.int32, device=dev)
    jit = torch.empty(M, B, dtype=torch.float64, device=dev)
    P = ctypes.c_void_p * M
    D = ctypes.c_double * M
    nparts = int(p0.Spart.shape[0]) if p0.Spart.shape[0] != p0.nC else 0
    st_out = P(*[w[0] for w in status]) if status is not None else None
    st_cnt = P(*[w[1] for w in status]) if status is not None else None
    Tp = P(*[t.data_ptr() for t in Ts]) if Ts is not None else None
    Fp = P(*[F[t].data_ptr() for t in range(M)]) if F is not None else None
    r = int(Ts[0].shape[0]) if Ts is not None else 0
    ldT = int(Ts[0].shape[1]) if Ts is not None else 0
    ldF = int(F.shape[2]) if F is not None else 0
    check(lib().bo_qmc_finalize_members(
        M, c0.kind, B, q, P(*[p.Xq.data_ptr() for p in pps]), P(*[p.Spart.data_ptr() for p in pps]),
        P(*[p.mpart.data_ptr() for p in pps]), c0.n, D(*[float(c.outputscale) for c in caches]),
        D(*[float(c.constant) for c in caches]), D(*[float(sv[0]) for sv in stats]),
        D(*[float(sv[1]) for sv in stats]), CHOLESKY_MAX_TRIES, CHOLESKY_JITTER_F64,
        P(*[mean[t].data_ptr() for t in range(M)]), P(*[L[t].data_ptr() for t in range(M)]),
        P(*[info[t].data_ptr() for t in range(M)]), P(*[jit[t].data_ptr() for t in range(M)]),
        nparts, st_out, st_cnt, Tp, r, ldT, Fp, ldF, _stream(dev)), "qmc_finalize_members")
    return info, jit


SOBOL_MAXBIT = 30  # torch.quasirandom.SobolEngine.MAXBIT


@functools.lru_cache(maxsize=16)
def _sobol_state0(dim: int, device: torch.device) -> torch.Tensor:
    """Unscrambled direction numbers (dim x 30) on the device, once per dim."""
    st = torch.zeros(dim, SOBOL_MAXBIT, dtype=torch.long)
    torch._sobol_engine_initialize_state_(st, dim)
    return st.to(device)


def sobol_engine_state(dim: int, seed: Optional[int], device=None):
    """Scrambled direction numbers + digital shift of torch's SobolEngine
    (the engine the reference's NormalQMCEngine wraps, sampling/qmc.py:56).

    On a ROCm device the state is built there (bo_sobol_scramble): the
    engine's own two draws from its seeded CPU generator -- shift bits, then the
    lower-triangular matrix bits, drawn as uint8 (the same stream as the int64
    draws) into one pinned buffer -- go over in one copy, and the scramble,
    the engine's 30 x 30 bit-matrix products per dimension, runs in one launch
    with the unscrambled direction numbers cached on the device.  Bit-identical
    to SobolEngine(dim, scramble=True, seed) (tests/test_gpu_ops.py); the
    engine itself spends ~30 ms of host time at dim 4096 (the baseline pruning
    of every qNEI / qNEHVI construction).  seed=None: the global CPU
    generator's draws, as the engine's."""
    if device is None or torch.device(device).type != "cuda":
        eng = SobolEngine(dimension=dim, scramble=True, seed=seed)
        return eng.sobolstate.clone(), eng.shift.clone()
    if not 1 <= dim <= SobolEngine.MAXDIM:
        raise ValueError(f"Supported range of dimensionality for SobolEngine is "
                         f"[1, {SobolEngine.MAXDIM}]")
    dev = torch.device(device)
    if dev.index is None:
        dev = torch.device("cuda", torch.cuda.current_device())
    nb = dim * SOBOL_MAXBIT
    # unseeded, the engine draws from torch's global CPU generator (as
    # SobolEngine._scramble does with seed=None): the same stream, consumed
    # by the same amount, so later global draws see the reference's state
    g = None
    if seed is not None:
        g = torch.Generator()
        g.manual_seed(seed)
    host = torch.empty(nb * (1 + SOBOL_MAXBIT), dtype=torch.uint8, pin_memory=True)
    torch.randint(2, (dim, SOBOL_MAXBIT), generator=g, dtype=torch.uint8,
                  out=host[:nb].view(dim, SOBOL_MAXBIT))
    torch.randint(2, (dim, SOBOL_MAXBIT, SOBOL_MAXBIT), generator=g, dtype=torch.uint8,
                  out=host[nb:].view(dim, SOBOL_MAXBIT, SOBOL_MAXBIT))
    bits = host.to(dev, non_blocking=True)
    state0 = _sobol_state0(dim, dev)
    state = torch.empty(dim, SOBOL_MAXBIT, dtype=torch.long, device=dev)
    shift = torch.empty(dim, dtype=torch.long, device=dev)
    check(lib().bo_sobol_scramble(dim, _p(state0), _p(bits), _p(state), _p(shift), _stream(dev)),
          "sobol_scramble")
    return state, shift


def sobol_normal(dim: int, n: int, seed: int, device, skip: int = 0) -> torch.Tensor:
    """n x dim scrambled-Sobol N(0,1) samples generated on the device."""
    from . import ops  # noqa: F401  (torch.ops.bo registration)
    state, shift = sobol_engine_state(dim, seed, device)
    first_f32 = torch.get_default_dtype() == torch.float32
    return torch.ops.bo.sobol_normal(state.to(device), shift.to(device), n, skip, first_f32)


def sobol_box(bounds: torch.Tensor, n: int, q: int, seed: Optional[int]) -> torch.Tensor:
    """n x q x d scrambled-Sobol raw designs in the box ``bounds`` (2 x d, on the
    device), bit-identical to draw_sobol_samples (botorch/utils/sampling.py:66-105)."""
    dev = bounds.device
    d = bounds.shape[-1]
    state, shift = sobol_engine_state(q * d, seed, dev)  # kept alive across the launch
    lower = bounds[0].to(torch.float64).contiguous()
    rng = (bounds[1] - bounds[0]).to(torch.float64).contiguous()
    out = torch.empty(n, q, d, dtype=torch.float64, device=dev)
    first_f32 = int(torch.get_default_dtype() == torch.float32)
    check(lib().bo_sobol_box(_p(state), _p(shift), q * d, n, 0, first_f32,
                             _p(lower), _p(rng), d, _p(out), _stream(dev)), "sobol_box")
    return out


def probe_mfma_layout(device) -> torch.Tensor:
    out = torch.empty(64, 8, dtype=torch.float64, device=device)
    check(lib().bo_probe_mfma_f64_layout(_p(out), _stream(torch.device(device))), "probe")
    return out


@dataclass
class WMat:
    """W = R L^{-1} for post_backward: ``t`` is W (nrows_pad x np) or, with
    ``kmajor``, W^T (np x nrows_pad) as bo_post_w writes it."""
    t: torch.Tensor
    kmajor: bool


def w_matrix(cache: GPCache, pp: PostPartials, post_w: Optional[bool] = None) -> WMat:
    """W = R L^{-1} = K*x (K + s2 I)^{-1}, from the stored R^T, as W^T =
    L^{-T} R^T on the posterior kernel's MFMA tiles: under a stream-K plan
    below four tiles per slot (bo_post_w_split), one pass on grids of 8 x 8
    super-tiles (bo_post_w); otherwise the GEMM W[i][k] = sum_c R[i][c] U[k][c]
    (U = L^{-T} upper -> op(B) zero below c < k).  ``post_w``: None = the plan
    above, True = bo_post_w whenever the grid allows it, False = the GEMM."""
    if pp.Rt is None:
        raise RuntimeError("post_partials(store_R=True) is required for gradients")
    if pp.Rt.dim() != 2:
        raise ValueError("w_matrix reads the row-major R^T; this one is blocked (use post_w_dx)")
    dev = pp.Rt.device
    nI = pp.nrows_pad // 128
    kc, we = ctypes.c_int(), ctypes.c_int64()
    check(lib().bo_post_w_work(pp.B, pp.q, cache.n, ctypes.byref(kc), ctypes.byref(we)), "post_w_work")
    if post_w is None and kc.value == -1:
        # stream-K W^T: grids below four tiles per slot (b <= 256 at n = 4096, C4)
        Wt = torch.empty(cache.np, pp.nrows_pad, dtype=torch.float64, device=dev)
        work = torch.empty(max(1, we.value), dtype=torch.float64, device=dev)
        check(lib().bo_post_w_split(_p(cache.Linv), cache.np, _p(pp.Rt), pp.B, pp.q, cache.n, _p(Wt),
                                    _p(work), _stream(dev)), "post_w_split")
        return WMat(Wt, True)
    if post_w is None:
        post_w = pp.nC * nI >= 512
    if post_w and pp.nC % 8 == 0 and nI % 8 == 0:
        Wt = torch.empty(cache.np, pp.nrows_pad, dtype=torch.float64, device=dev)
        check(lib().bo_post_w(_p(cache.Linv), cache.np, _p(pp.Rt), pp.B, pp.q, cache.n, _p(Wt),
                              _stream(dev)), "post_w")
        return WMat(Wt, True)
    W = torch.empty(pp.nrows_pad, cache.np, dtype=torch.float64, device=dev)
    K = pp.nC * 128
    check(lib().bo_gemm_f64(1, 1, pp.nrows_pad, cache.np, K, 1.0, _p(pp.Rt), pp.nrows_pad, 0,
                            _p(cache.U), cache.np, 0, 0.0, _p(W), cache.np, 0, 1,
                            _lib.GEMM_B_LOWER, _stream(dev)), "w_matrix")
    return WMat(W, False)


# BO_W_MEMBERS=0: w_matrix per member in w_matrix_members (A/B)
W_MEMBERS = os.environ.get("BO_W_MEMBERS", "1") != "0"


def w_matrix_members(caches, pps) -> list:
    """w_matrix of every member (a ModelListGP's, one shape): where the
    one-model plan is stream-K, all members' W^T = L^{-T} R^T in ONE
    member-batched launch + one reduction (bo_post_w_split_members), else
    per member."""
    nm = len(caches)
    p0, c0 = pps[0], caches[0]
    same = all(c.n == c0.n and c.np == c0.np for c in caches) and all(
        p_.Rt is not None and p_.Rt.dim() == 2 and p_.Rt.is_contiguous() and p_.B == p0.B
        and p_.q == p0.q for p_ in pps)
    we = ctypes.c_int64(-1)
    if W_MEMBERS and 1 < nm <= 8 and same:
        check(lib().bo_post_w_members_work(nm, p0.B, p0.q, c0.n, ctypes.byref(we)), "post_w_members_work")
    if we.value < 0:
        return [w_matrix(c, p_) for c, p_ in zip(caches, pps)]
    dev = p0.Rt.device
    Wt = torch.empty(nm, c0.np, p0.nrows_pad, dtype=torch.float64, device=dev)
    work = torch.empty(max(1, we.value), dtype=torch.float64, device=dev)
    arr = lambda ts: (ctypes.c_void_p * nm)(*[_p(t).value for t in ts])  # noqa: E731
    check(lib().bo_post_w_split_members(nm, arr([c.Linv for c in caches]), c0.np,
                                        arr([p_.Rt for p_ in pps]), p0.B, p0.q, c0.n,
                                        arr([Wt[m] for m in range(nm)]), _p(work), _stream(dev)),
          "post_w_split_members")
    return [WMat(Wt[m], True) for m in range(nm)]


def post_w_dx(cache: GPCache, pp: PostPartials, dmean: torch.Tensor, dcov: torch.Tensor,
              ystd: float) -> Optional[torch.Tensor]:
    """dX of the posterior moments' cotangents with W = R L^{-1} reduced into
    dX tile by tile (bo_post_w_dx; W never stored); None where the one-pass
    grid does not apply or R^T was stored row-major (then w_matrix +
    post_backward): the fused pass reads only the blocked R^T
    (post_partials(rt_layout=RT_BLOCKED), 3-d)."""
    if pp.Rt is None:
        raise RuntimeError("post_partials(store_R=True) is required for gradients")
    dev = pp.Rt.device
    we = ctypes.c_int64()
    check(lib().bo_post_w_dx_work(pp.B, pp.q, cache.n, ctypes.byref(we)), "post_w_dx_work")
    if we.value == 0 or pp.Rt.dim() != 3:
        return None
    work = torch.empty(we.value, dtype=torch.float64, device=dev)
    dX = torch.empty(pp.B, pp.q, cache.d, dtype=torch.float64, device=dev)
    check(lib().bo_post_w_dx(cache.kind, _p(cache.Linv), cache.np, _p(pp.Rt), pp.B, pp.q, cache.d,
                             cache.n, _p(pp.Xq), _p(cache.Xt_scaled), _p(cache.alpha),
                             _p(dmean.contiguous()), _p(dcov.contiguous()), _p(cache.lengthscale),
                             cache.outputscale, float(ystd), _p(work), _p(dX), _stream(dev)),
          "post_w_dx")
    return dX


def qmc_backward(mode: int, mean: torch.Tensor, L: torch.Tensor, Z: torch.Tensor,
                 dacq: torch.Tensor, best_f: float = 0.0,
                 best_f_s: Optional[torch.Tensor] = None, F: Optional[torch.Tensor] = None,
                 acq_fwd: Optional[torch.Tensor] = None, log_params: Optional[tuple] = None):
    """dacq -> (dmean, dcov[, dF]).  qNEI passes F = Z_base T (S x nrows_pad) and
    gets its cotangent dF back as a third output.  The log modes also take the
    forward values acq_fwd and log_params = (fat, tau_relu, tau_max)."""
    dev = mean.device
    B, q = mean.shape
    S = Z.shape[0]
    dmean = torch.empty(B, q, dtype=torch.float64, device=dev)
    dcov = torch.empty(B, q, q, dtype=torch.float64, device=dev)
    dF = torch.zeros_like(F) if F is not None else None
    fat, tau_relu, tau_max = log_params if log_params is not None else (1, 1.0, 1.0)
    if acq_fwd is not None:
        acq_fwd = acq_fwd.contiguous()
    a = _lib.QmcBackwardArgs(mode=mode, B=B, q=q, S=S, mean=mean, Lq=L,
                             Z=Z.reshape(S, q).contiguous(), best_f=float(best_f),
                             best_f_s=best_f_s, F=F, ldF=F.shape[1] if F is not None else 0,
                             dacq=dacq.contiguous(), dmean=dmean, dcov=dcov, dF=dF,
                             acq_fwd=acq_fwd, fat=int(bool(fat)), tau_relu=float(tau_relu),
                             tau_max=float(tau_max))
    check(lib().bo_qmc_backward_v(ctypes.byref(a), _stream(dev)), "qmc_backward")
    if F is not None:
        return dmean, dcov, dF
    return dmean, dcov


def post_backward(cache: GPCache, pp: PostPartials, W: Optional[WMat],
                  dmean: Optional[torch.Tensor], dcov: Optional[torch.Tensor], ystd: float,
                  E: Optional[torch.Tensor] = None, Xt_scaled: Optional[torch.Tensor] = None,
                  n: Optional[int] = None, dX: Optional[torch.Tensor] = None) -> torch.Tensor:
    """dX of the batched posterior: dK*x = ystd dmean alpha^T - G W (+ E), through
    dk/dx over the training points.  With ``Xt_scaled``/``n`` (other points, e.g.
    the qNEI baseline) and only ``E``, the gradient through K(points, X); ``dX``
    given -> accumulated into it."""
    dev = pp.Xq.device
    acc = dX is not None
    if dX is None:
        dX = torch.empty(pp.B, pp.q, cache.d, dtype=torch.float64, device=dev)
    other = Xt_scaled is not None
    cont = lambda t: t.contiguous() if t is not None else None  # noqa: E731
    if isinstance(W, torch.Tensor):
        W = WMat(W, False)
    kmajor = W is not None and W.kmajor
    W = cont(W.t) if W is not None else None
    E, dmean, dcov = cont(E), cont(dmean), cont(dcov)
    a = _lib.PostBackwardArgs(kind=cache.kind, B=pp.B, q=pp.q, d=cache.d, Xq=pp.Xq,
                              Xt_scaled=Xt_scaled if other else cache.Xt_scaled,
                              n=n if other else cache.n, W=W,
                              ldw=W.shape[1] if W is not None else 0,
                              alpha=None if other else cache.alpha, dmean=dmean, dcov=dcov, E=E,
                              lde=E.shape[1] if E is not None else 0,
                              lengthscale=cache.lengthscale, outputscale=cache.outputscale,
                              ystd=float(ystd), accumulate=int(acc), w_kmajor=int(kmajor), dX=dX)
    check(lib().bo_post_backward_v(ctypes.byref(a), _stream(dev)), "post_backward")
    return dX


def post_backward_jobs(jobs: list) -> torch.Tensor:
    """Several post_backward passes of one (B, q, d, kind) -- each job a dict
    of post_backward's arguments (cache, pp, W, dmean, dcov, ystd, E,
    Xt_scaled, n) -- in ONE launch (bo_post_backward_jobs, grid B x jobs),
    every job's dX into its own slice; returns their sum (B x q x d)."""
    nj = len(jobs)
    c0, p0 = jobs[0]["cache"], jobs[0]["pp"]
    dev = p0.Xq.device
    parts = torch.empty(nj, p0.B, p0.q, c0.d, dtype=torch.float64, device=dev)
    recs, keep = [], []
    cont = lambda t: t.contiguous() if t is not None else None  # noqa: E731
    for j in jobs:
        cache, pp = j["cache"], j["pp"]
        W = j.get("W")
        if isinstance(W, torch.Tensor):
            W = WMat(W, False)
        kmajor = W is not None and W.kmajor
        Wt = cont(W.t) if W is not None else None
        E, dmean, dcov = cont(j.get("E")), cont(j.get("dmean")), cont(j.get("dcov"))
        other = j.get("Xt_scaled") is not None
        keep += [Wt, E, dmean, dcov]
        recs.append(_lib.PostBackwardArgs(
            kind=cache.kind, B=pp.B, q=pp.q, d=cache.d, Xq=pp.Xq,
            Xt_scaled=j["Xt_scaled"] if other else cache.Xt_scaled,
            n=j["n"] if other else cache.n, W=Wt, ldw=Wt.shape[1] if Wt is not None else 0,
            alpha=None if other else cache.alpha, dmean=dmean, dcov=dcov, E=E,
            lde=E.shape[1] if E is not None else 0, lengthscale=cache.lengthscale,
            outputscale=cache.outputscale, ystd=float(j["ystd"]), accumulate=0,
            w_kmajor=int(kmajor), dX=parts))
    arr = (ctypes.POINTER(_lib.PostBackwardArgs) * nj)(*[ctypes.pointer(r) for r in recs])
    check(lib().bo_post_backward_jobs(nj, arr, _p(parts), _stream(dev)), "post_backward_jobs")
    return parts.sum(0)


# Deferred ladder status (forward-only fused acquisitions): the status of call t
# is copied to pinned host memory behind an event and checked at call t + 1, at
# the driver's own synchronisation points (gen_candidates_scipy's loss.item(),
# the raw-sample selection, optimize_acqf's return) or by check_ladder_status().
# The host thus runs at most one forward ahead of the device instead of
# draining the queue every call.  Failed t-batches carry NaN values meanwhile.
# BO_SYNC_LADDER=1 restores the per-call check.
SYNC_LADDER = os.environ.get("BO_SYNC_LADDER", "0") == "1"
# The deferred status itself lives in the native operators (bo::ladder_defer /
# bo::ladder_poll, csrc/torch/bo_torch.cpp: two pinned slots + events per
# device); here only the name of the acquisition whose status is pending.
_LADDER_WHAT = {}


def _dev_index(device) -> int:
    d = torch.device(device)
    return d.index if d.index is not None else torch.cuda.current_device()


def ladder_prev_outcome(status: torch.Tensor, idx: int, what: str) -> None:
    """Act on the previous deferred status [has, info_max, jitter_max] that a
    native call returned, and record ``what`` as the name of the new pending
    one."""
    prev_what = _LADDER_WHAT.get(idx, what)
    _LADDER_WHAT[idx] = what
    has, info_max, jitter_max = status.tolist()
    if has:
        _ladder_outcome(info_max, jitter_max, prev_what)


def check_ladder_status(device=None) -> None:
    """Raise NotPSDError / warn NumericalWarning for a deferred ladder status
    (waits for the forward that produced it); no-op when none is pending."""
    ops = _lib.torch_ops()
    keys = list(_LADDER_WHAT) if device is None else [_dev_index(device)]
    for idx in keys:
        has, info_max, jitter_max = ops.ladder_poll(idx).tolist()
        what = _LADDER_WHAT.pop(idx, "acquisition")
        if has:
            _ladder_outcome(info_max, jitter_max, what)
    # the gradient path's outcomes whose backward has not run (_LadderRing)
    for idx in (list(_RINGS) if device is None else [_dev_index(device)]):
        if idx in _RINGS:
            _RINGS[idx].settle_all()


def _ladder_outcome(info_max: float, jitter_max: float, what: str) -> None:
    if info_max > 0:
        from .exceptions import NotPSDError
        raise NotPSDError(f"{what}: matrix not positive definite after repeatedly adding "
                          f"jitter up to {CHOLESKY_JITTER_F64 * 10 ** (CHOLESKY_MAX_TRIES - 1):.1e}")
    if jitter_max > 0:
        import warnings
        from .exceptions import NumericalWarning
        warnings.warn(f"A not p.d., added jitter of {jitter_max:.1e} to the diagonal", NumericalWarning)


# Graph capture (graphs.GraphedAcquisition): inside capturing(dev) the ladder
# status is reduced into a device buffer that the graph owns and is read by
# the wrapper after a replay -- no host read, pinned copy or event in the graph.
# A forward-only capture registers (pinned status words, device counter) in
# _CAPTURE_STATUS: the fused forward's finalisation kernel then folds the
# status into those words itself and the capture records ("native", what).
_CAPTURE = {}
_CAPTURE_STATUS = {}


class capturing:
    """Context of a HIP-graph capture on ``device`` (see _CAPTURE)."""

    def __init__(self, device):
        d = torch.device(device)
        self.idx = d.index if d.index is not None else torch.cuda.current_device()

    def __enter__(self):
        _CAPTURE[self.idx] = None
        return self

    def __exit__(self, *exc):
        return False


def take_captured_status(device):
    """(packed status tensor, what) written by the captured forward, or None."""
    d = torch.device(device)
    idx = d.index if d.index is not None else torch.cuda.current_device()
    return _CAPTURE.pop(idx, None)


def _capture_status(info: torch.Tensor, jitter: torch.Tensor, what: str) -> bool:
    dev = info.device
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    if idx not in _CAPTURE:
        return False
    packed = torch.zeros(2, dtype=torch.float64, device=dev)
    if info.numel():
        check(lib().bo_ladder_status(_p(info.contiguous()), _p(jitter.contiguous()), info.numel(),
                                     _p(packed), _stream(dev)), "ladder_status")
    record_capture_status(idx, packed, what)
    return True


def record_capture_status(idx: int, packed, what: str) -> None:
    """Record one route's ladder status in the running capture, merging with
    what earlier routes of the same body recorded: device statuses combine by
    a captured max; a device status beside the native route (whose
    finalisation folds into the graph's pinned words) is kept as
    ("native+", what, packed) so the graph copies it to a second pinned pair
    -- neither kind ever overwrites the other.  ``packed`` None: the native
    route."""
    prev = _CAPTURE.get(idx)
    if packed is None:                                   # the native route
        if prev is None or prev[0] == "native":
            _CAPTURE[idx] = ("native", what)
        elif prev[0] == "native+":
            pass
        else:                                            # a device status came first
            _CAPTURE[idx] = ("native+", what, prev[0])
        return
    if prev is None:
        _CAPTURE[idx] = (packed, what)
    elif prev[0] == "native":
        _CAPTURE[idx] = ("native+", prev[1], packed)
    elif prev[0] == "native+":
        _CAPTURE[idx] = ("native+", prev[1], torch.maximum(prev[2], packed))
    else:
        _CAPTURE[idx] = (torch.maximum(prev[0], packed), prev[1])


def raise_not_psd_deferred(info: torch.Tensor, jitter: torch.Tensor, what: str) -> None:
    """_raise_not_psd without the per-call device-to-host synchronisation."""
    if _capture_status(info, jitter, what):
        return
    if SYNC_LADDER or info.numel() == 0:
        return _raise_not_psd(info, jitter, what)
    # this call's status is enqueued, the previous call's read (one forward behind)
    prev = _lib.torch_ops().ladder_defer(info.contiguous(), jitter.contiguous())
    ladder_prev_outcome(prev, _dev_index(info.device), what)


class _PinnedStatus:
    """Per device: 8 pairs of pinned, device-mapped status words and 8 device
    arrival counters -- where bo_qmc_finalize folds each member's ladder
    outcome (status_out / status_count) for raise_not_psd_members."""

    def __init__(self, dev):
        h, d = ctypes.c_void_p(), ctypes.c_void_p()
        check(lib().bo_pinned_alloc(16 * 8, ctypes.byref(h), ctypes.byref(d)), "pinned_alloc")
        self.host_ptr, self.dev_ptr = h.value, d.value
        self.words = (ctypes.c_double * 16).from_address(self.host_ptr)
        self.count = torch.zeros(8, dtype=torch.int32, device=dev)  # kernels re-zero them

    def arm(self, m: int):
        """Zero the first m pairs; (status_out, status_count) pointers of each."""
        ctypes.memset(self.host_ptr, 0, 16 * m)
        base = self.count.data_ptr()
        return [(self.dev_ptr + 16 * t, base + 4 * t) for t in range(m)]

    def __del__(self):
        try:
            lib().bo_pinned_free(ctypes.c_void_p(self.host_ptr))
        except Exception:  # interpreter shutdown
            pass


_PINNED = {}


def pinned_status(dev) -> "_PinnedStatus":
    idx = _dev_index(dev)
    if idx not in _PINNED:
        _PINNED[idx] = _PinnedStatus(torch.device("cuda", idx))
    return _PINNED[idx]


class _LadderRing:
    """Per device: a few _PinnedStatus blocks for the gradient path of the
    ModelListGP acquisitions (qEHVI / qNEHVI).  A forward takes a block, its
    finalisation launch folds the members' ladder outcomes into it, and an
    event is recorded behind the forward; the outcome is read at the end of the
    backward (``settle``: waits for that event only, once the backward's
    launches are queued) -- not in the forward, whose stream drain kept the
    device idle while the host issued the backward (C4 forward + backward
    0.92-1.07 -> 0.84 ms).  A forward whose backward never runs is read when
    its block comes round again (one ring behind) or at check_ladder_status,
    as the eager qEI's deferred status is.  Outcomes raise / warn in member
    order, as raise_not_psd_members."""

    N = 4

    def __init__(self, dev):
        self.dev = dev
        self.blocks = [_PinnedStatus(dev) for _ in range(self.N)]
        self.events = [torch.cuda.Event() for _ in range(self.N)]
        self.pending = [None] * self.N  # (generation, members, what)
        self.next = 0
        self.gen = 0

    def take(self, m: int, what: str):
        """(token, per-member (status_out, status_count) pointers) of a block."""
        i = self.next
        self.next = (i + 1) % self.N
        if self.pending[i] is not None:
            self._settle_slot(i)
        self.gen += 1
        self.pending[i] = (self.gen, m, what)
        return (i, self.gen), self.blocks[i].arm(m)

    def record(self, token) -> None:
        self.events[token[0]].record(torch.cuda.current_stream(self.dev))

    def settle(self, token) -> None:
        i, g = token
        p = self.pending[i]
        if p is not None and p[0] == g:
            self._settle_slot(i)

    def settle_all(self) -> None:
        for k in range(self.N):  # oldest first
            i = (self.next + k) % self.N
            if self.pending[i] is not None:
                self._settle_slot(i)

    def _settle_slot(self, i: int) -> None:
        _, m, what = self.pending[i]
        self.pending[i] = None
        self.events[i].synchronize()
        w = self.blocks[i].words
        raise_status_words([(w[2 * t], w[2 * t + 1]) for t in range(m)], what)


_RINGS = {}


def ladder_ring(dev) -> "_LadderRing":
    idx = _dev_index(dev)
    if idx not in _RINGS:
        _RINGS[idx] = _LadderRing(torch.device("cuda", idx))
    return _RINGS[idx]


def raise_not_psd_members(ps: "_PinnedStatus", m: int, dev, what: str) -> None:
    """The members' ladder outcomes folded into ps's pinned words by their
    finalisation launches: one stream sync, then raised / warned in member
    order as per-member checks would (no status launch, no copy)."""
    _stream_sync(dev)
    w = ps.words
    raise_status_words([(w[2 * t], w[2 * t + 1]) for t in range(m)], what)


def raise_status_words(pairs, what: str) -> None:
    """[max info, max jitter] per member, in member order: NotPSDError for a
    failed ladder, the reference's NumericalWarning for added jitter."""
    for info_max, jit_max in pairs:
        if info_max > 0:
            from .exceptions import NotPSDError
            raise NotPSDError(f"{what}: matrix not positive definite after repeatedly adding "
                              f"jitter up to {CHOLESKY_JITTER_F64 * 10 ** (CHOLESKY_MAX_TRIES - 1):.1e}")
        if jit_max > 0:
            import warnings
            from .exceptions import NumericalWarning
            warnings.warn(f"A not p.d., added jitter of {float(jit_max):.1e} to the diagonal",
                          NumericalWarning)


def _stream_sync(dev):
    torch.cuda.current_stream(torch.device("cuda", _dev_index(dev))).synchronize()


def raise_not_psd_many(pairs, what: str) -> None:
    """_raise_not_psd over several ladders (a ModelListGP's members) with ONE
    device-to-host read, issued after the caller has enqueued its remaining
    work: the members' statuses are packed side by side, then raised / warned
    in member order, as the per-member checks would.  Under graph capture,
    the per-member path (its capture slot)."""
    pairs = [(i, j) for i, j in pairs if i.numel()]
    if not pairs:
        return
    dev = pairs[0][0].device
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    if idx in _CAPTURE or len(pairs) == 1:
        for info, jitter in pairs:
            _raise_not_psd(info, jitter, what)
        return
    packed = torch.empty(len(pairs), 2, dtype=torch.float64, device=dev)
    for m, (info, jitter) in enumerate(pairs):
        check(lib().bo_ladder_status(_p(info.contiguous()), _p(jitter.contiguous()), info.numel(),
                                     _p(packed[m]), _stream(dev)), "ladder_status")
    packed = packed.cpu()
    for m in range(len(pairs)):
        if packed[m, 0] > 0:
            from .exceptions import NotPSDError
            raise NotPSDError(f"{what}: matrix not positive definite after repeatedly adding "
                              f"jitter up to {CHOLESKY_JITTER_F64 * 10 ** (CHOLESKY_MAX_TRIES - 1):.1e}")
        if packed[m, 1] > 0:
            import warnings
            from .exceptions import NumericalWarning
            warnings.warn(f"A not p.d., added jitter of {float(packed[m, 1]):.1e} to the diagonal",
                          NumericalWarning)


def _raise_not_psd(info: torch.Tensor, jitter: torch.Tensor, what: str):
    """Host check of a batched ladder (one D2H read, as [G] psd_safe_cholesky's
    torch.any(info)); warns like [G] when jitter was added."""
    if info.numel() == 0 or _capture_status(info, jitter, what):
        return
    packed = torch.empty(2, dtype=torch.float64, device=info.device)
    check(lib().bo_ladder_status(_p(info.contiguous()), _p(jitter.contiguous()), info.numel(),
                                 _p(packed), _stream(info.device)), "ladder_status")
    packed = packed.cpu()
    if packed[0] > 0:
        from .exceptions import NotPSDError
        raise NotPSDError(f"{what}: matrix not positive definite after repeatedly adding "
                          f"jitter up to {CHOLESKY_JITTER_F64 * 10 ** (CHOLESKY_MAX_TRIES - 1):.1e}")
    if packed[1] > 0:
        import warnings
        from .exceptions import NumericalWarning
        warnings.warn(f"A not p.d., added jitter of {float(packed[1]):.1e} to the diagonal",
                      NumericalWarning)


def chol_jitter(A: torch.Tensor, max_tries=CHOLESKY_MAX_TRIES,
                jitter0=CHOLESKY_JITTER_F64) -> torch.Tensor:
    """psd_safe_cholesky of (..., q, q) on the device (batched kernel for q <= 64,
    blocked MFMA Cholesky per matrix beyond)."""
    dev = _dev(A)
    q = A.shape[-1]
    batch = A.shape[:-2]
    A3 = A.reshape(-1, q, q).contiguous()
    B = A3.shape[0]
    if q <= 64:
        L = torch.empty_like(A3)
        info = torch.empty(B, dtype=torch.int32, device=dev)
        jit = torch.empty(B, dtype=torch.float64, device=dev)
        check(lib().bo_chol_small(_p(A3), B, q, max_tries, jitter0, _p(L), _p(info), _p(jit),
                                  _stream(dev)), "chol_small")
        _raise_not_psd(info, jit, "psd_safe_cholesky")
        return L.reshape(*batch, q, q)
    out = []
    np_ = padded_order(q)
    for b in range(B):
        L = torch.empty(np_, np_, dtype=torch.float64, device=dev)
        Linv = torch.empty_like(L)
        work = torch.empty_like(L)
        info = torch.zeros(1, dtype=torch.int32, device=dev)
        jit = ctypes.c_double(0.0)
        check(lib().bo_cholesky_jitter(_p(A3[b]), q, _p(L), _p(Linv), _p(work), max_tries, jitter0,
                                       ctypes.byref(jit), _p(info), _stream(dev)), "cholesky_jitter")
        if jit.value > 0:
            import warnings
            from .exceptions import NumericalWarning
            warnings.warn(f"A not p.d., added jitter of {jit.value:.1e} to the diagonal",
                          NumericalWarning)
        out.append(L[:q, :q])
    return torch.stack(out).reshape(*batch, q, q)


def covar_blocks(X3: torch.Tensor, lengthscale, kind=_lib.RBF, outputscale=1.0, diag_add=0.0):
    dev = _dev(X3)
    B, q, d = X3.shape
    K = torch.empty(B, q, q, dtype=torch.float64, device=dev)
    check(lib().bo_covar_blocks(kind, _p(X3.contiguous()), B, q, d,
                                _p(lengthscale.reshape(-1).contiguous()), outputscale, diag_add,
                                _p(K), _stream(dev)), "covar_blocks")
    return K


def posterior_general(model, X3: torch.Tensor):
    """Exact posterior of B t-batches of any q / d through the generic kernels:
    K*x (covar_matrix), R = K*x L^{-T} (triangular MFMA GEMM), R R^T blocks
    (batched GEMM), mean = c + K*x alpha.  Outcome space."""
    cache = model.prediction_cache()
    ymean, ystd = model.outcome_stats()
    B, q, d = X3.shape
    n = cache.n
    X2 = X3.reshape(B * q, d).contiguous()
    Kx = covar_matrix(X2, cache.Xt, cache.lengthscale, cache.kind, cache.outputscale)
    R = gemm(Kx, cache.U[:n, :n], flags=_lib.GEMM_B_UPPER)
    mean = gemm(Kx, cache.alpha.reshape(n, 1)).reshape(B, q)
    RR = gemm(R.reshape(B, q, n), R.reshape(B, q, n), transB=True)
    Kxx = covar_blocks(X3, cache.lengthscale, cache.kind, cache.outputscale)
    cov = (Kxx - RR) * (ystd * ystd)
    mean = ymean + ystd * (mean + cache.constant)
    return mean, cov


def cholesky_with_inverse(A: torch.Tensor, max_tries=CHOLESKY_MAX_TRIES,
                          jitter0=CHOLESKY_JITTER_F64):
    """psd_safe_cholesky of one n x n matrix on the device, with L^{-1}:
    returns (L, Linv, jitter) as n x n views of np x np buffers."""
    dev = _dev(A)
    n = A.shape[-1]
    np_ = padded_order(n)
    L = torch.empty(np_, np_, dtype=torch.float64, device=dev)
    Linv = torch.empty_like(L)
    work = torch.empty_like(L)
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    jit = ctypes.c_double(0.0)
    check(lib().bo_cholesky_jitter(_p(A.contiguous()), n, _p(L), _p(Linv), _p(work), max_tries,
                                   jitter0, ctypes.byref(jit), _p(info), _stream(dev)),
          "cholesky_jitter")
    if jit.value > 0:
        import warnings
        from .exceptions import NumericalWarning
        warnings.warn(f"A not p.d., added jitter of {jit.value:.1e} to the diagonal",
                      NumericalWarning)
    return L[:n, :n], Linv[:n, :n], jit.value


def sample_mvn(mean: torch.Tensor, L: torch.Tensor, Z: torch.Tensor) -> torch.Tensor:
    """f[s, b, i] = mean[b, i] + sum_j L[b, i, j] Z[s, j]  (S x B x q), as one
    batched MFMA GEMM with the shared base samples broadcast (stride 0)."""
    dev = _dev(mean, L, Z)
    B, q = mean.shape
    S = Z.shape[0]
    Z = Z.reshape(S, q).contiguous()
    L = L.contiguous()
    out = torch.empty(B, S, q, dtype=torch.float64, device=dev)
    check(lib().bo_gemm_f64(0, 1, S, q, q, 1.0, _p(Z), q, 0, _p(L), q, q * q, 0.0, _p(out), q,
                            S * q, B, 0, _stream(dev)), "sample_mvn")
    return out.permute(1, 0, 2) + mean.unsqueeze(0)


def nd_partition_host(Y: torch.Tensor, ref_point: torch.Tensor, nthreads: int = 0,
                      alpha=None):
    """Non-dominated box decompositions of S point sets (host, native threads):
    Y (S x n x m, or n x m) -> (lo, hi) each S x K x m (K x m for a single
    set), padded with empty cells as BoxDecompositionList does.  alpha None:
    the exact FastNondominatedPartitioning cells (bo_nd_partition_host); a
    number: NondominatedPartitioning's binary partitioning with that
    approximation threshold (bo_nd_partition_alpha_host)."""
    single = Y.dim() == 2
    Yc = Y.detach().to("cpu", torch.float64).contiguous()
    if single:
        Yc = Yc.unsqueeze(0)
    S, n, m = Yc.shape
    ref = ref_point.detach().to("cpu", torch.float64).contiguous()
    nthreads = nthreads or min(16, os.cpu_count() or 1)
    K = ctypes.c_int64(0)
    cap = max(64, 8 * n)
    while True:
        lo = torch.empty(S, cap, m, dtype=torch.float64)
        hi = torch.empty(S, cap, m, dtype=torch.float64)
        if alpha is None:
            st = lib().bo_nd_partition_host(_p(Yc), S, n, m, _p(ref), cap, ctypes.byref(K),
                                            _p(lo), _p(hi), nthreads)
        else:
            st = lib().bo_nd_partition_alpha_host(_p(Yc), S, n, m, _p(ref), float(alpha), cap,
                                                  ctypes.byref(K), _p(lo), _p(hi), nthreads)
        if st == _lib.BO_ERR_ARG and K.value > cap:
            cap = int(K.value)  # one retry with the exact size
            continue
        check(st, "nd_partition_host")
        break
    Kc = max(int(K.value), 1)
    lo, hi = lo[:, :Kc].contiguous(), hi[:, :Kc].contiguous()
    return (lo[0], hi[0]) if single else (lo, hi)


def _cells_layout(cell_lo: torch.Tensor, S: int):
    """(K, cell_stride): shared K x m cells, or per-sample S x K x m cells."""
    if cell_lo.dim() == 3:
        if cell_lo.shape[0] != S:
            raise ValueError(f"per-sample cells for {cell_lo.shape[0]} samples, expected {S}")
        return cell_lo.shape[1], cell_lo.shape[1] * cell_lo.shape[2]
    return cell_lo.shape[0], 0


def qehvi(mean: torch.Tensor, L: torch.Tensor, Z: torch.Tensor, cell_lo: torch.Tensor,
          cell_hi: torch.Tensor, F: Optional[torch.Tensor] = None, Qp: int = 0) -> torch.Tensor:
    """mean: m x B x q, L: m x B x q x q, Z: S x (q m) -> acq (B).  Cells K x m
    (shared) or S x K x m (per sample, qNEHVI); F: m x S x ldF cached-root
    baseline term (rows b * Qp + p)."""
    dev = _dev(mean, L, Z, cell_lo, cell_hi)
    m, B, q = mean.shape
    S = Z.shape[0]
    K, cstride = _cells_layout(cell_lo, S)
    acq = torch.empty(B, dtype=torch.float64, device=dev)
    work = torch.empty(8 * B, dtype=torch.float64, device=dev)  # sample split (B < 256)
    Fc = F.contiguous() if F is not None else None
    a = _lib.QehviArgs(B=B, q=q, m=m, S=S, mean=mean.contiguous(), L=L.contiguous(),
                       Z=Z.reshape(S, q * m).contiguous(), cell_lo=cell_lo.contiguous(),
                       cell_hi=cell_hi.contiguous(), K=K, Qp=Qp, cell_stride=cstride, F=Fc,
                       ldF=Fc.shape[-1] if Fc is not None else 0,
                       sF=Fc.shape[-1] * S if Fc is not None else 0, acq=acq, work=work,
                       work_elems=work.numel())
    check(lib().bo_qehvi_v(ctypes.byref(a), _stream(dev)), "qehvi")
    return acq


def qehvi_backward(mean: torch.Tensor, L: torch.Tensor, Z: torch.Tensor, cell_lo: torch.Tensor,
                   cell_hi: torch.Tensor, dacq: torch.Tensor, F: Optional[torch.Tensor] = None,
                   Qp: int = 0):
    """Backward of :func:`qehvi`: -> dmean (m x B x q), dL (m x B x q x q)[, dF]."""
    dev = _dev(mean, L, Z, cell_lo, cell_hi)
    m, B, q = mean.shape
    S = Z.shape[0]
    K, cstride = _cells_layout(cell_lo, S)
    dmean = torch.empty(m, B, q, dtype=torch.float64, device=dev)
    dL = torch.empty(m, B, q, q, dtype=torch.float64, device=dev)
    Fc = F.contiguous() if F is not None else None
    dF = torch.zeros_like(Fc) if Fc is not None else None
    work = torch.empty(8 * B * m * q * (q + 3) // 2, dtype=torch.float64, device=dev)
    a = _lib.QehviArgs(B=B, q=q, m=m, S=S, mean=mean.contiguous(), L=L.contiguous(),
                       Z=Z.reshape(S, q * m).contiguous(), cell_lo=cell_lo.contiguous(),
                       cell_hi=cell_hi.contiguous(), K=K, Qp=Qp, cell_stride=cstride, F=Fc,
                       ldF=Fc.shape[-1] if Fc is not None else 0,
                       sF=Fc.shape[-1] * S if Fc is not None else 0, dacq=dacq.contiguous(),
                       dmean=dmean, dL=dL, dF=dF, work=work, work_elems=work.numel())
    check(lib().bo_qehvi_backward_v(ctypes.byref(a), _stream(dev)), "qehvi_backward")
    if F is not None:
        return dmean, dL, dF
    return dmean, dL


def kernel_grad(X: torch.Tensor, Y: torch.Tensor, dK: torch.Tensor, lengthscale: torch.Tensor,
                kind: int, outputscale: float = 1.0, group: int = 0,
                dX: Optional[torch.Tensor] = None) -> torch.Tensor:
    """dX (+)= sum_k dK[i, k] d k(X_i, Y_k)/dX_i for any d <= 128 (original scale)."""
    dev = _dev(X, Y, dK)
    rows, d = X.shape
    acc = dX is not None
    if dX is None:
        dX = torch.empty(rows, d, dtype=torch.float64, device=dev)
    dK = dK.contiguous()
    check(lib().bo_kernel_grad(kind, _p(X.contiguous()), rows, _p(Y.contiguous()), Y.shape[0], d,
                               _p(lengthscale.reshape(-1).contiguous()), float(outputscale),
                               _p(dK), dK.shape[-1], group, int(acc), _p(dX), _stream(dev)),
          "kernel_grad")
    return dX


def chol_backward(L: torch.Tensor, dL: torch.Tensor) -> torch.Tensor:
    """Batched Cholesky backward (B x q x q) -> dA (torch linalg.cholesky semantics)."""
    dev = _dev(L, dL)
    B, q, _ = L.shape
    dA = torch.empty(B, q, q, dtype=torch.float64, device=dev)
    check(lib().bo_chol_backward(B, q, _p(L.contiguous()), _p(dL.contiguous()), _p(dA),
                                 _stream(dev)), "chol_backward")
    return dA


def mc_reduce(samples: torch.Tensor, best_f: float = 0.0,
              best_f_s: Optional[torch.Tensor] = None) -> torch.Tensor:
    """samples: S x B x q -> qEI/qNEI value per t-batch."""
    dev = _dev(samples)
    S, B, q = samples.shape
    acq = torch.empty(B, dtype=torch.float64, device=dev)
    check(lib().bo_mc_reduce(S, B, q, _p(samples.contiguous()), float(best_f), _p(best_f_s),
                             _p(acq), _stream(dev)), "mc_reduce")
    return acq


def pareto_mask(Y: torch.Tensor, maximize: bool = True, deduplicate: bool = True) -> torch.Tensor:
    """Non-dominated mask of (..., n, m) point sets on the device (bool, ... x n)."""
    dev = _dev(Y)
    n, m = Y.shape[-2], Y.shape[-1]
    Y3 = Y.reshape(-1, n, m).contiguous()
    S = Y3.shape[0]
    out = torch.empty(S, n, dtype=torch.uint8, device=dev)
    for s0 in range(0, S, 65535):
        s1 = min(S, s0 + 65535)
        check(lib().bo_pareto_mask(_p(Y3[s0:s1]), s1 - s0, n, m, int(maximize), int(deduplicate),
                                   _p(out[s0:s1]), _stream(dev)), "pareto_mask")
    return out.bool().reshape(Y.shape[:-1])
