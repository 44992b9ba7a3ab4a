"""ctypes binding of the C ABI in ``include/botorch_amd.h``.

This is the "reference-side FFI" of the drop-in boundary: plain pointers and
sizes go in, status codes come out.  The library is built in-tree
(``make`` -> ``botorch_amd/libbotorch_amd.so``) and there is deliberately no
fallback: if it is missing, every GPU entry point raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_double, c_int, c_int64, c_void_p

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "libbotorch_amd.so")

BO_OK, BO_ERR_ARG, BO_ERR_HIP, BO_ERR_NOT_PSD, BO_ERR_NAN = 0, 1, 2, 3, 4
RBF, MATERN52 = 0, 1
GEMM_LOWER_C, GEMM_A_LOWER, GEMM_B_UPPER, GEMM_A_UPPER, GEMM_B_LOWER = 1, 2, 4, 8, 16
QMC_POSTERIOR, QMC_QEI, QMC_QNEI, QMC_CHOL, QMC_QLOGEI, QMC_QLOGNEI = 0, 1, 2, 3, 4, 5
LOG_MODES = (QMC_QLOGEI, QMC_QLOGNEI)
ABI_VERSION = 8

_P = c_void_p  # device pointers travel as void*

# name -> (restype, argtypes)
_SIGNATURES = {
    "bo_last_error": (ctypes.c_char_p, []),
    "bo_version": (c_int, []),
    "bo_probe_mfma_f64_layout": (c_int, [_P, _P]),
    "bo_probe_mfma_f64_rate": (c_int, [c_int, c_int, _P, _P]),
    "bo_probe_valu_f64": (c_int, [c_int, _P, _P]),
    "bo_gemm_f64": (c_int, [c_int, c_int, c_int, c_int, c_int, c_double, _P, c_int64, c_int64,
                            _P, c_int64, c_int64, c_double, _P, c_int64, c_int64, c_int, c_int,
                            _P]),
    "bo_covar_matrix": (c_int, [c_int, _P, c_int64, _P, c_int64, c_int, _P, c_double, c_double,
                                c_int, _P, c_int64, c_int64, c_int64, _P]),
    "bo_padded_order": (c_int64, [c_int64]),
    "bo_covar_batched": (c_int, [c_int, _P, c_int64, c_int64, c_int, _P, c_int64, c_int64, c_int,
                                 c_int, _P, c_int64, c_int64, _P, c_int64, c_int64, _P, c_int64,
                                 c_int64, c_int64, c_int, c_int, _P]),
    "bo_cholesky_inverse": (c_int, [_P, _P, _P, c_int64, _P, _P]),
    "bo_transpose": (c_int, [_P, _P, c_int64, c_int64, _P]),
    "bo_cholesky_jitter": (c_int, [_P, c_int64, _P, _P, _P, c_int, c_double, POINTER(c_double),
                                   _P, _P]),
    "bo_chol_small": (c_int, [_P, c_int64, c_int, c_int, c_double, _P, _P, _P, _P]),
    "bo_ladder_status": (c_int, [_P, _P, c_int64, _P, _P]),
    "bo_pareto_mask": (c_int, [_P, c_int64, c_int, c_int, c_int, c_int, _P, _P]),
    "bo_covar_blocks": (c_int, [c_int, _P, c_int64, c_int, c_int, _P, c_double, c_double, _P,
                                _P]),
    "bo_gemv": (c_int, [_P, c_int64, c_int64, _P, c_double, _P, _P]),
    "bo_scale_inputs": (c_int, [_P, c_int64, c_int, _P, _P, c_int, _P, _P]),
    "bo_gp_cache_build": (c_int, [c_int, _P, c_int64, c_int, _P, c_double, c_double, c_double,
                                  _P, _P, _P, _P, _P, _P, c_int, c_double, POINTER(c_double),
                                  _P, _P]),
    "bo_post_geometry": (c_int, [c_int64, c_int, c_int64, POINTER(c_int), POINTER(c_int),
                                 POINTER(c_int)]),
    "bo_prepare_rows": (c_int, [_P, c_int, c_int, c_int, _P, _P, _P]),
    "bo_post_partials": (c_int, [c_int, _P, c_int, c_int, c_int, _P, c_int64, _P, c_int64, _P,
                                 c_double, _P, _P, _P, c_int, _P, _P, c_int, c_int64, _P, _P,
                                 _P]),
    "bo_post_kxt": (c_int, [c_int, _P, c_int, c_int, c_int, _P, c_int64, c_double, _P, _P]),
    "bo_post_w": (c_int, [_P, c_int64, _P, c_int, c_int, c_int64, _P, _P]),
    "bo_post_split_plan": (c_int, [c_int64, c_int, c_int64, c_int, POINTER(c_int),
                                   POINTER(c_int64)]),
    "bo_qmc_finalize": (c_int, [c_int, c_int, c_int, c_int, _P, _P, _P, c_int64, c_double,
                                c_double, c_double, c_double, _P, c_int, c_double, _P, c_int,
                                c_double, _P, _P, _P, _P, _P, _P, _P, c_int, c_int64, _P,
                                c_int64, c_int, c_double, c_double, _P]),
    "bo_qehvi": (c_int, [c_int, c_int, c_int, _P, _P, _P, c_int, _P, _P, c_int, c_int64, _P,
                         c_int64, c_int64, c_int, _P, _P]),
    "bo_qehvi_backward": (c_int, [c_int, c_int, c_int, _P, _P, _P, c_int, _P, _P, c_int, c_int64,
                                  _P, c_int64, c_int64, c_int, _P, _P, _P, _P, _P]),
    "bo_chol_backward": (c_int, [c_int, c_int, _P, _P, _P, _P]),
    "bo_probe_potrf_phases": (c_int, [_P, c_int64, _P, _P, _P, _P]),
    "bo_probe_chol_dag": (c_int, [_P, _P, c_int64, _P, _P, _P, _P, _P]),
    "bo_chol_dag_tasks": (c_int, [c_int, _P, c_int]),
    "bo_kernel_grad": (c_int, [c_int, _P, c_int64, _P, c_int64, c_int, _P, c_double, _P, c_int64,
                               c_int, c_int, _P, _P]),
    "bo_mc_reduce": (c_int, [c_int, c_int, c_int, _P, c_double, _P, _P, _P]),
    "bo_sobol_normal": (c_int, [_P, _P, c_int, c_int64, c_int64, c_int, _P, _P]),
    "bo_lbfgs_step": (c_int, [c_int, c_int, c_int, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                              _P, _P, _P, _P, _P, _P, c_double, c_double, c_double, c_double, _P]),
    "bo_nd_partition_host": (c_int, [_P, c_int64, c_int64, c_int, _P, c_int64, POINTER(c_int64), _P,
                                     _P, c_int]),
    "bo_sobol_box": (c_int, [_P, _P, c_int, c_int64, c_int64, c_int, _P, _P, c_int, _P, _P]),
    "bo_mll_terms": (c_int, [c_int, _P, c_int64, c_int, _P, c_double, _P, _P, c_int64, _P, _P, _P,
                             _P]),
    "bo_qmc_backward": (c_int, [c_int, c_int, c_int, _P, _P, _P, c_int, c_double, _P, _P,
                                c_int64, _P, _P, _P, _P, _P, c_int, c_double, c_double, _P]),
    "bo_post_backward": (c_int, [c_int, c_int, c_int, c_int, _P, _P, c_int64, _P, c_int64, _P,
                                 _P, _P, _P, c_int64, _P, c_double, c_double, c_int, _P, c_int,
                                 _P]),
}

_lib = None


class NativeLibraryMissing(RuntimeError):
    pass


def lib():
    """Load (once) and return the native library; raise loudly if absent."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeLibraryMissing(
                f"{LIB_PATH} not found: build it with `make` (or __graft_entry__.build()). "
                "botorch_amd has no CPU fallback.")
        handle = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGNATURES.items():
            fn = getattr(handle, name)
            fn.restype = res
            fn.argtypes = args
        if handle.bo_version() != ABI_VERSION:
            raise NativeLibraryMissing(
                f"{LIB_PATH} has ABI {handle.bo_version()}, expected {ABI_VERSION}: rebuild with `make`")
        _lib = handle
    return _lib


def exported_symbols():
    return list(_SIGNATURES)


def check(status: int, what: str = "") -> None:
    """Map a C-ABI status to the reference's exception taxonomy."""
    if status == BO_OK:
        return
    from .exceptions import NanError, NotPSDError
    msg = lib().bo_last_error().decode(errors="replace")
    if status == BO_ERR_NOT_PSD:
        raise NotPSDError(msg)
    if status == BO_ERR_NAN:
        raise NanError(msg)
    if status == BO_ERR_ARG:
        raise ValueError(f"{what}: {msg}")
    raise RuntimeError(f"{what}: HIP error: {msg}")
