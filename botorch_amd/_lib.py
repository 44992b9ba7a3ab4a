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
ABI_VERSION = 11
RT_ROWMAJOR, RT_BLOCKED = 0, 1  # BoPostPartialsArgs.rt_layout (include/botorch_amd.h)

_P = c_void_p  # device pointers travel as void*

# name -> (restype, argtypes)
_SIGNATURES = {
    "bo_last_error": (ctypes.c_char_p, []),
    "bo_version": (c_int, []),
    "bo_probe_mfma_f64_layout": (c_int, [_P, _P]),
    "bo_probe_mfma_f64_rate": (c_int, [c_int, c_int, _P, _P]),
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
    "bo_cholesky_inverse_ainv": (c_int, [_P, _P, _P, _P, c_int64, _P, _P]),
    "bo_chol_dag_tasks_ainv": (c_int, [c_int, _P, c_int]),
    "bo_cholesky_inverse_batched": (c_int, [_P, _P, _P, c_int, c_int64, _P, _P]),
    "bo_transpose": (c_int, [_P, _P, c_int64, c_int64, _P]),
    "bo_cholesky_jitter": (c_int, [_P, c_int64, _P, _P, _P, c_int, c_double, POINTER(c_double),
                                   _P, _P]),
    "bo_chol_small": (c_int, [_P, c_int64, c_int, c_int, c_double, _P, _P, _P, _P]),
    "bo_ladder_status": (c_int, [_P, _P, c_int64, _P, _P]),
    "bo_pareto_mask": (c_int, [_P, c_int64, c_int, c_int, c_int, c_int, _P, _P]),
    "bo_covar_blocks": (c_int, [c_int, _P, c_int64, c_int, c_int, _P, c_double, c_double, _P,
                                _P]),
    "bo_gemv": (c_int, [_P, c_int64, c_int64, _P, c_double, _P, _P]),
    "bo_gemv_tri": (c_int, [_P, c_int64, c_int64, _P, c_double, _P, c_int, _P]),
    "bo_gemv_lt_work": (c_int, [c_int64, POINTER(c_int64)]),
    "bo_gemv_lt": (c_int, [_P, c_int64, c_int64, _P, c_double, _P, _P, _P]),
    "bo_scale_inputs": (c_int, [_P, c_int64, c_int, _P, _P, c_int, _P, _P]),
    "bo_gp_cache_build": (c_int, [c_int, _P, c_int64, c_int, _P, c_double, c_double, c_double,
                                  _P, _P, _P, _P, _P, _P, c_int, c_double, POINTER(c_double),
                                  _P, _P]),
    "bo_gp_cache_build_fixed": (c_int, [c_int, _P, c_int64, c_int, _P, c_double, _P, c_double,
                                        _P, _P, _P, _P, _P, _P, c_int, c_double,
                                        POINTER(c_double), _P, _P]),
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
    "bo_post_split_work": (c_int, [c_int64, c_int, c_int64, c_int, POINTER(c_int64)]),
    "bo_ainv_work": (c_int, [c_int64, POINTER(c_int64)]),
    "bo_post_w_work": (c_int, [c_int, c_int, c_int64, POINTER(c_int), POINTER(c_int64)]),
    "bo_post_w_split": (c_int, [_P, c_int64, _P, c_int, c_int, c_int64, _P, _P, _P]),
    "bo_post_w_members_work": (c_int, [c_int, c_int, c_int, c_int64, POINTER(c_int64)]),
    "bo_post_w_split_members": (c_int, [c_int, _P, c_int64, _P, c_int, c_int, c_int64, _P, _P, _P]),
    "bo_post_w_dx_work": (c_int, [c_int, c_int, c_int64, POINTER(c_int64)]),
    "bo_post_w_dx": (c_int, [c_int, _P, c_int64, _P, c_int, c_int, c_int, c_int64, _P, _P, _P, _P,
                             _P, _P, c_double, c_double, _P, _P, _P]),
    "bo_ainv": (c_int, [_P, c_int64, c_int64, _P, _P, _P]),
    "bo_sym_lower": (c_int, [_P, c_int64, c_int64, _P]),
    "bo_post_kxt_rows": (c_int, [c_int, _P, c_int, c_int, c_int, _P, _P, c_int64, c_double, _P,
                                 _P, _P]),
    "bo_post_quad_plan": (c_int, [c_int64, c_int, c_int64, POINTER(c_int)]),
    "bo_post_small_plan": (c_int, [c_int64, c_int, c_int64, POINTER(c_int)]),
    "bo_post_small": (c_int, [_P, c_int64, c_int, c_int64, _P, c_int64, _P, _P, _P, _P, _P]),
    "bo_post_small_batched": (c_int, [c_int, _P, _P, _P, _P, _P, _P, c_int64, c_int, c_int64,
                                      c_int64, _P]),
    "bo_pinned_alloc": (c_int, [c_int64, POINTER(c_void_p), POINTER(c_void_p)]),
    "bo_pinned_free": (c_int, [c_void_p]),
    "bo_qmc_finalize_members": (c_int, [c_int, c_int, c_int, c_int, _P, _P, _P, c_int64, _P, _P, _P,
                                        _P, c_int, c_double, _P, _P, _P, _P, c_int, _P, _P, _P,
                                        c_int, c_int64, _P, c_int64, _P]),
    "bo_post_kxt_rows_members": (c_int, [c_int, c_int, _P, c_int, c_int, c_int, _P, _P, _P, c_int64,
                                         _P, _P, _P]),
    "bo_post_members_work": (c_int, [c_int, c_int64, c_int, c_int64, POINTER(c_int64)]),
    "bo_post_partials_members": (c_int, [c_int, _P, _P, _P, _P, _P, _P, _P, c_int64, c_int,
                                         c_int64, c_int64, _P, _P]),
    "bo_post_quad": (c_int, [_P, _P, c_int64, _P, c_int64, c_int, c_int64, _P, _P, _P]),
    "bo_post_split_table": (c_int, [c_int64, c_int, c_int64, c_int, _P, c_int, _P, c_int,
                                    POINTER(c_int), POINTER(c_int)]),
    "bo_qmc_finalize": (c_int, [c_int, c_int, c_int, c_int, _P, _P, _P, c_int64, c_double,
                                c_double, c_double, c_double, _P, c_int, c_double, _P, c_int,
                                c_double, _P, _P, _P, _P, _P, _P, _P, c_int, c_int64, _P,
                                c_int64, c_int, c_double, c_double, _P]),
    "bo_qehvi": (c_int, [c_int, c_int, c_int, _P, _P, _P, c_int, _P, _P, c_int, c_int64, _P,
                         c_int64, c_int64, c_int, _P, _P]),
    "bo_qehvi_backward": (c_int, [c_int, c_int, c_int, _P, _P, _P, c_int, _P, _P, c_int, c_int64,
                                  _P, c_int64, c_int64, c_int, _P, _P, _P, _P, _P]),
    "bo_chol_backward": (c_int, [c_int, c_int, _P, _P, _P, _P]),
    "bo_chol_dag_tasks": (c_int, [c_int, _P, c_int]),
    "bo_kernel_grad": (c_int, [c_int, _P, c_int64, _P, c_int64, c_int, _P, c_double, _P, c_int64,
                               c_int, c_int, _P, _P]),
    "bo_mc_reduce": (c_int, [c_int, c_int, c_int, _P, c_double, _P, _P, _P]),
    "bo_sobol_normal": (c_int, [_P, _P, c_int, c_int64, c_int64, c_int, _P, _P]),
    "bo_sobol_scramble": (c_int, [c_int, _P, _P, _P, _P, _P]),
    "bo_lbfgs_step": (c_int, [c_int, c_int, c_int, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                              _P, _P, _P, _P, _P, _P, c_double, c_double, c_double, c_double, _P]),
    "bo_lbfgsb_step": (c_int, [c_int, c_int, c_int, c_int, c_int, c_int, c_double, c_double, _P,
                               _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P]),
    "bo_lbfgsb_layout": (c_int, [_P]),
    "bo_lbfgsb_set_profile": (c_int, [_P, c_int]),
    "bo_lbfgsb_set_staging": (c_int, [c_int]),
    "bo_lbfgsb_set_grid": (c_int, [c_int]),
    "bo_lbfgsb_grid_launches": (c_int64, []),
    "bo_nd_partition_host": (c_int, [_P, c_int64, c_int64, c_int, _P, c_int64, POINTER(c_int64), _P,
                                     _P, c_int]),
    "bo_nd_partition_alpha_host": (c_int, [_P, c_int64, c_int64, c_int, _P, c_double, c_int64,
                                           POINTER(c_int64), _P, _P, c_int]),
    "bo_hit_and_run_host": (c_int, [_P, _P, c_int64, c_int64, _P, _P, _P, _P, c_int64, c_int64,
                                    c_int64, _P, c_int64]),
    "bo_sobol_box": (c_int, [_P, _P, c_int, c_int64, c_int64, c_int, _P, _P, c_int, _P, _P]),
    "bo_mll_terms": (c_int, [c_int, _P, c_int64, c_int, _P, c_double, _P, _P, c_int64, _P, _P, _P,
                             _P]),
    "bo_qmc_backward": (c_int, [c_int, c_int, c_int, _P, _P, _P, c_int, c_double, _P, _P,
                                c_int64, _P, _P, _P, _P, _P, c_int, c_double, c_double, _P]),
    "bo_post_backward": (c_int, [c_int, c_int, c_int, c_int, _P, _P, c_int64, _P, c_int64, _P,
                                 _P, _P, _P, c_int64, _P, c_double, c_double, c_int, _P, c_int,
                                 _P]),
}



# ---- parameter-struct entry points (ABI 9): ctypes mirrors of the C records ----------
from ctypes import Structure, c_uint32, sizeof  # noqa: E402

c_int32 = ctypes.c_int32
_D = ctypes.c_void_p  # device pointer field


class _Args(Structure):
    """Base of the ABI-9 argument records: fills struct_size / abi_version and
    maps torch tensors (or None) of pointer fields to their data pointers."""

    def __init__(self, **kw):
        super().__init__()
        self.struct_size = sizeof(self)
        self.abi_version = ABI_VERSION
        self._keep = []
        for k, v in kw.items():
            if hasattr(v, "data_ptr"):
                self._keep.append(v)
                v = v.data_ptr()
            setattr(self, k, v)


_HDR = [("struct_size", c_uint32), ("abi_version", c_uint32)]


class PostPartialsArgs(_Args):
    _fields_ = _HDR + [("kind", c_int32), ("B", c_int32), ("q", c_int32), ("d", c_int32),
                       ("Xq", _D), ("Xt_scaled", _D), ("n", c_int64), ("U", _D), ("ldu", c_int64),
                       ("beta", _D), ("outputscale", c_double), ("Spart", _D), ("mpart", _D),
                       ("Rt", _D), ("kc_len", c_int32), ("rq", c_int32), ("work", _D),
                       ("Qc", _D), ("ldq", c_int64), ("Cx", _D), ("Kt", _D),
                       ("rt_layout", c_int32), ("_pad", c_int32)]


class QmcFinalizeArgs(_Args):
    _fields_ = _HDR + [("kind", c_int32), ("mode", c_int32), ("B", c_int32), ("q", c_int32),
                       ("Xq", _D), ("Spart", _D), ("mpart", _D), ("n", c_int64),
                       ("outputscale", c_double), ("constant", c_double), ("ymean", c_double),
                       ("ystd", c_double), ("Z", _D), ("S", c_int32), ("max_tries", c_int32),
                       ("best_f", c_double), ("best_f_s", _D), ("jitter0", c_double),
                       ("acq", _D), ("mean_out", _D), ("cov_out", _D), ("L_out", _D),
                       ("info_out", _D), ("jitter_out", _D), ("Tm", _D), ("r", c_int32),
                       ("fat", c_int32), ("ldT", c_int64), ("F", _D), ("ldF", c_int64),
                       ("tau_relu", c_double), ("tau_max", c_double),
                       ("nparts", c_int32), ("sym_parts", c_int32), ("status_out", _D),
                       ("status_count", _D)]


class QmcBackwardArgs(_Args):
    _fields_ = _HDR + [("mode", c_int32), ("B", c_int32), ("q", c_int32), ("S", c_int32),
                       ("mean", _D), ("Lq", _D), ("Z", _D), ("best_f", c_double),
                       ("best_f_s", _D), ("F", _D), ("ldF", c_int64), ("dacq", _D),
                       ("dmean", _D), ("dcov", _D), ("dF", _D), ("acq_fwd", _D),
                       ("fat", c_int32), ("_pad", c_int32), ("tau_relu", c_double),
                       ("tau_max", c_double)]


class PostBackwardArgs(_Args):
    _fields_ = _HDR + [("kind", c_int32), ("B", c_int32), ("q", c_int32), ("d", c_int32),
                       ("Xq", _D), ("Xt_scaled", _D), ("n", c_int64), ("W", _D), ("ldw", c_int64),
                       ("alpha", _D), ("dmean", _D), ("dcov", _D), ("E", _D), ("lde", c_int64),
                       ("lengthscale", _D), ("outputscale", c_double), ("ystd", c_double),
                       ("accumulate", c_int32), ("w_kmajor", c_int32), ("dX", _D)]


class QehviArgs(_Args):
    _fields_ = _HDR + [("B", c_int32), ("q", c_int32), ("m", c_int32), ("S", c_int32),
                       ("mean", _D), ("L", _D), ("Z", _D), ("cell_lo", _D), ("cell_hi", _D),
                       ("K", c_int32), ("Qp", c_int32), ("cell_stride", c_int64), ("F", _D),
                       ("ldF", c_int64), ("sF", c_int64), ("acq", _D), ("dacq", _D),
                       ("dmean", _D), ("dL", _D), ("dF", _D), ("work", _D),
                       ("work_elems", c_int64)]


class LbfgsStepArgs(_Args):
    _fields_ = _HDR + [("B", c_int32), ("n", c_int32), ("m", c_int32), ("_pad", c_int32),
                       ("x", _D), ("f", _D), ("g", _D), ("xt", _D), ("ft", _D), ("gt", _D),
                       ("d", _D), ("alpha", _D), ("S", _D), ("Y", _D), ("rho", _D),
                       ("hcount", _D), ("hhead", _D), ("status", _D), ("nacc", _D),
                       ("lower", _D), ("upper", _D), ("c1", c_double), ("ftol", c_double),
                       ("pgtol", c_double), ("min_alpha", c_double)]


class LbfgsbArgs(_Args):
    _fields_ = _HDR + [("B", c_int32), ("n", c_int32), ("m", c_int32), ("maxls", c_int32),
                       ("maxiter", c_int32), ("maxfun", c_int32), ("ftol", c_double),
                       ("pgtol", c_double), ("lower", _D), ("upper", _D), ("xt", _D), ("ft", _D),
                       ("gt", _D), ("v", _D), ("iv", _D), ("ws", _D), ("wy", _D), ("mat", _D),
                       ("ds", _D), ("is_", _D)]


for _name, _cls in (("bo_post_partials_v", PostPartialsArgs), ("bo_qmc_finalize_v", QmcFinalizeArgs),
                    ("bo_qmc_backward_v", QmcBackwardArgs), ("bo_post_backward_v", PostBackwardArgs),
                    ("bo_qehvi_v", QehviArgs), ("bo_qehvi_backward_v", QehviArgs),
                    ("bo_lbfgs_step_v", LbfgsStepArgs), ("bo_lbfgsb_step_v", LbfgsbArgs)):
    _SIGNATURES[_name] = (c_int, [POINTER(_cls), _P])
_SIGNATURES["bo_struct_size"] = (c_int64, [ctypes.c_char_p])
_SIGNATURES["bo_post_backward_jobs"] = (c_int, [c_int, POINTER(POINTER(PostBackwardArgs)), _P, _P])
ARG_RECORDS = {"BoPostPartialsArgs": PostPartialsArgs, "BoQmcFinalizeArgs": QmcFinalizeArgs,
               "BoQmcBackwardArgs": QmcBackwardArgs, "BoPostBackwardArgs": PostBackwardArgs,
               "BoQehviArgs": QehviArgs, "BoLbfgsStepArgs": LbfgsStepArgs,
               "BoLbfgsbArgs": LbfgsbArgs}

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
        for cname, rec in ARG_RECORDS.items():  # record layouts agree with the C header
            if handle.bo_struct_size(cname.encode()) != sizeof(rec):
                raise NativeLibraryMissing(f"{cname}: ctypes layout differs from the library's")
        _lib = handle
    return _lib


TORCH_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libbotorch_amd_torch.so")
_torch_ops_loaded = False


def torch_ops():
    """Load (once) the TORCH_LIBRARY operators of csrc/torch/bo_torch.cpp
    (libbotorch_amd_torch.so: torch.ops.bo.qmc_acq_native, ladder_defer,
    ladder_poll, post_timing[_read]); raise loudly if absent."""
    global _torch_ops_loaded
    if not _torch_ops_loaded:
        lib()  # the kernel library it links against (and its ABI check)
        if not os.path.exists(TORCH_LIB_PATH):
            raise NativeLibraryMissing(
                f"{TORCH_LIB_PATH} not found: build it with `make` (or __graft_entry__.build()).")
        import torch
        torch.ops.load_library(TORCH_LIB_PATH)
        _torch_ops_loaded = True
    import torch
    return torch.ops.bo


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
