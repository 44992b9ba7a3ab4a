"""Measure the fp64 MFMA issue rate of this MI355X (sets roofline.peak sanity)."""
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
out = torch.zeros(1, dtype=torch.float64, device=dev)
st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
res = {}
for blocks in (256, 512, 1024, 2048):
    iters = 2000
    _lib.check(_lib.lib().bo_probe_mfma_f64_rate(blocks, 10, ctypes.c_void_p(out.data_ptr()), st))
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    _lib.check(_lib.lib().bo_probe_mfma_f64_rate(blocks, iters, ctypes.c_void_p(out.data_ptr()), st))
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1)
    fl = blocks * 4 * iters * 8 * 2048
    res[blocks] = fl / (ms * 1e-3) / 1e12
valu = {}
for waves in (1, 4, 8):
    o = torch.zeros(8, dtype=torch.int64, device=dev)
    for _ in range(2):
        _lib.check(_toolslib.tools().bo_probe_valu_f64(waves, ctypes.c_void_p(o.data_ptr()), st))
    torch.cuda.synchronize()
    t = o.cpu().tolist()
    valu[waves] = {"dep_fma_cyc": t[0] / 256, "indep_fma_cyc": t[1] / 2048,
                   "rsq2nr_chain_cyc": t[2] / 64, "lds_dep_read_cyc": t[3] / 256}
print(json.dumps({"fp64_mfma_tflops": res, "valu_f64": valu}))
