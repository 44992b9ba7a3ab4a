#!/usr/bin/env python3
"""s_memtime ticks per 16 x 16 diagonal factor (+ inverse) step of the DAG
Cholesky's potrf_trtri64 on one wave, for the broadcast variants of
bo_probe_diag16 (DPP row broadcast / readlane to SGPR / DPP factor only)."""
import ctypes
import json
import os
import sys

import torch
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _toolslib  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from botorch_amd import _lib  # noqa: E402

dev = torch.device("cuda", 0)
out = torch.zeros(4, dtype=torch.int64, device=dev)
sink = torch.zeros(1, dtype=torch.float64, device=dev)
st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
for _ in range(2):
    _lib.check(_toolslib.tools().bo_probe_diag16(ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(sink.data_ptr()), st))
torch.cuda.synchronize()
o = out.cpu().tolist()
print(json.dumps({"dpp_factor_inverse": o[0], "readlane_factor_inverse": o[1], "dpp_factor_only": o[2]}))
