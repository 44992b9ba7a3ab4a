"""ctypes loader of tools/libbotorch_amd_tools.so (`make tools`): the
development probes of tools/bo_tools.h, which the product library does not
export."""
import ctypes
import os

PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libbotorch_amd_tools.so")
_P, _I, _I64 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64
_SIG = {"bo_probe_valu_f64": [_I, _P, _P],
        "bo_probe_chol_dag": [_P, _P, _I64, _P, _P, _P, _P, _P],
        "bo_probe_diag16": [_P, _P, _P],
        "bo_probe_potrf64": [_P, _P, _P, _P, _I, _I, _P]}
_h = None


def tools():
    global _h
    if _h is None:
        if not os.path.exists(PATH):
            raise RuntimeError(f"{PATH} not found: build it with `make tools`")
        _h = ctypes.CDLL(PATH)
        for name, args in _SIG.items():
            fn = getattr(_h, name)
            fn.restype = ctypes.c_int
            fn.argtypes = args
    return _h
