"""C2 qEI forward: eager call vs HIP-graph replay (forward only and forward +
backward), back-to-back calls timed on the host clock (development tool)."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from botorch_amd.acquisition import qExpectedImprovement
    from botorch_amd.graphs import GraphedAcquisition
    from botorch_amd.models import SingleTaskGP
    from botorch_amd.sampling import SobolQMCNormalSampler
    from botorch_amd.test_functions import Hartmann
    from botorch_amd.utils_sampling import draw_sobol_samples
    dev = torch.device("cuda", 0)
    unit = torch.stack([torch.zeros(6), torch.ones(6)]).to(torch.float64)
    X = draw_sobol_samples(unit, 1024, 1, seed=0).squeeze(1)
    Y = Hartmann(negate=True)(X).unsqueeze(-1)
    m = SingleTaskGP(X.to(dev), Y.to(dev))
    m.covar_module.lengthscale = torch.full((1, 6), 0.5016, dtype=torch.float64)
    m.likelihood.noise = torch.tensor([6.737947e-3], dtype=torch.float64)
    m.eval()
    acqf = qExpectedImprovement(m, float(Y.max()), sampler=SobolQMCNormalSampler(torch.Size([256]), seed=0))
    Xd = draw_sobol_samples(unit, 64, 8, seed=1).to(dev)

    def t(fn, n=300):
        for _ in range(30):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        return 1e3 * (time.perf_counter() - t0) / n

    out = {}
    with torch.no_grad():
        out["eager_ms"] = t(lambda: acqf(Xd))
    ga = GraphedAcquisition(acqf, Xd, share_input=True)
    out["graph_ms"] = t(lambda: ga(Xd))
    ga.check_status()
    gc = GraphedAcquisition(acqf, Xd)
    Xo = Xd.clone()
    out["graph_copy_ms"] = t(lambda: gc(Xo))
    with torch.no_grad():
        ref = acqf(Xd)
    out["graph_equal"] = bool(torch.equal(ga(Xd).clone(), ref))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
