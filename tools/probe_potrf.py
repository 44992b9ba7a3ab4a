"""Phase timing of the 128-block Cholesky kernel (s_memtime ticks)."""
import ctypes
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from botorch_amd import _lib, kernels  # noqa: E402

dev = torch.device("cuda", 0)
X = torch.rand(128, 6, dtype=torch.float64, device=dev)
ls = torch.full((6,), 0.5, dtype=torch.float64, device=dev)
K = kernels.covar_matrix(X, X, ls, diag_add=1e-2)
names = ["start", "load", "F1 s0", "F2 s0", "F3 s0", "F1 s1", "F2 s1", "F3 s1", "F1 s2", "F2 s2",
         "F3 s2", "F1 s3", "L store + dinv copy", "merge64", "merge128", "Linv store"]
p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
st = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
res = []
for rep in range(3):
    A = K.clone()
    Linv = torch.zeros_like(A)
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    tsc = torch.zeros(16, dtype=torch.int64, device=dev)
    _lib.check(_lib.lib().bo_probe_potrf_phases(p(A), 128, p(Linv), p(info), p(tsc), st))
    torch.cuda.synchronize()
    t = tsc.cpu().tolist()
    res.append({names[i]: t[i] - t[i - 1] for i in range(1, 16) if t[i] and t[i - 1]})
L = torch.linalg.cholesky(K.cpu())
err = float((A.cpu().tril() - L).abs().max())
ierr = float((Linv.cpu().tril() @ L - torch.eye(128, dtype=torch.float64)).abs().max())
print(json.dumps({"phases_ticks": res[-1], "total": sum(res[-1].values()), "info": int(info.item()),
                  "chol_err": err, "inv_err": ierr}))
