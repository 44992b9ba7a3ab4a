"""Which device blocks survive a gen_candidates_device run with gc off, and
what refers to them (development diagnostic)."""
import gc, sys, types
import torch
sys.path.insert(0, '.')
from tests.test_gpu_memory import _acqf, DEV
from botorch_amd.optim import gen_candidates_device

acqf = _acqf(1024, 256, seed=2)
g = torch.Generator().manual_seed(3)
ics = torch.rand(64, 8, 6, generator=g, dtype=torch.float64).to(DEV)
lo = torch.zeros(6, dtype=torch.float64, device=DEV)
hi = torch.ones(6, dtype=torch.float64, device=DEV)
c, v = gen_candidates_device(ics, acqf, lo, hi, options={"maxiter": 30}); del c, v
gen_candidates_device.last_state = None
torch.cuda.synchronize(); gc.collect(); gc.disable()
snap0 = torch.cuda.memory._snapshot()
addr0 = {b["address"] for seg in snap0["segments"] for b in seg["blocks"] if b["state"] == "active_allocated"}
c, v = gen_candidates_device(ics, acqf, lo, hi, options={"maxiter": 30}); del c, v
gen_candidates_device.last_state = None
torch.cuda.synchronize()
snap = torch.cuda.memory._snapshot()
new = {b["address"]: b["size"] for seg in snap["segments"] for b in seg["blocks"]
       if b["state"] == "active_allocated" and b["address"] not in addr0}
print("new blocks", new)
def desc(o):
    if isinstance(o, dict):
        return "dict keys=" + str(list(o.keys())[:12])
    if isinstance(o, (list, tuple)):
        return f"{type(o).__name__} len={len(o)}"
    if isinstance(o, types.FrameType):
        return f"frame {o.f_code.co_filename}:{o.f_lineno} {o.f_code.co_name}"
    return repr(type(o))
hits = [o for o in gc.get_objects() if isinstance(o, torch.Tensor) and o.is_cuda
        and o.untyped_storage().data_ptr() in new]
print("tensors found", len(hits))
for t in hits:
    print("TENSOR", t.shape, t.dtype)
    for r in gc.get_referrers(t):
        if r is hits: continue
        print("   <-", desc(r))
        for r2 in gc.get_referrers(r):
            if r2 is hits: continue
            print("       <-", desc(r2))
            for r3 in gc.get_referrers(r2)[:6]:
                print("           <-", desc(r3))
