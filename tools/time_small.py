"""A/B of the small-grid forward posterior (BO_POST_SMALL=0 / 1 / auto, set by
the caller; read once per process): eager forward ms per call of qEI at C2 and
at the strong split's per-rank C3 shards, HIP events over back-to-back calls."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from botorch_amd.acquisition import qExpectedImprovement
    from botorch_amd.models import SingleTaskGP
    from botorch_amd.sampling import SobolQMCNormalSampler
    from botorch_amd.test_functions import Hartmann
    from botorch_amd.utils_sampling import draw_sobol_samples
    dev = torch.device("cuda", 0)
    out = {"BO_POST_SMALL": os.environ.get("BO_POST_SMALL", "auto")}
    unit = torch.stack([torch.zeros(6), torch.ones(6)]).to(torch.float64)
    for n, q, S, bs in ((1024, 8, 256, (1, 16, 64)), (2048, 8, 128, (32, 128)),
                       (2048, 16, 512, (64,)), (4096, 16, 512, (1, 64, 128, 256))):
        X = draw_sobol_samples(unit, n, 1, seed=0).squeeze(1)
        Y = Hartmann(negate=True)(X).unsqueeze(-1)
        m = SingleTaskGP(X.to(dev), Y.to(dev))
        m.covar_module.lengthscale = torch.full((1, 6), 0.5016, dtype=torch.float64)
        m.likelihood.noise = torch.tensor([6.737947e-3], dtype=torch.float64)
        m.eval()
        acqf = qExpectedImprovement(m, float(Y.max()) - 0.3,
                                    sampler=SobolQMCNormalSampler(torch.Size([S]), seed=0))
        for b in bs:
            Xc = draw_sobol_samples(unit, b, q, seed=1).to(dev)
            calls = 400 if n == 1024 else 40
            with torch.no_grad():
                for _ in range(10):
                    acqf(Xc)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(calls):
                    v = acqf(Xc)
                e1.record()
                torch.cuda.synchronize()
            out[f"n{n}_q{q}_b{b}"] = {"ms": e0.elapsed_time(e1) / calls,
                                      "checksum": float(v.sum())}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
