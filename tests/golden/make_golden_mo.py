"""Golden fixtures of the approximate box decompositions (``golden_mo.npz``).

Runs ONLY in the development container, where ``/root/reference`` exists: it
imports the gpytorch-free box-decomposition modules of the reference through
``_refload`` and records inputs and outputs as plain arrays.

Usage:  python tests/golden/make_golden_mo.py

Sources (reference file:line):
  * NondominatedPartitioning(alpha)      box_decompositions/non_dominated.py:30-350
  * FastNondominatedPartitioning.compute_hypervolume  non_dominated.py:445-457
  * DominatedPartitioning.compute_hypervolume         dominated.py:51-62
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import _refload  # noqa: E402

from cases import MO_ALPHA_CASES  # noqa: E402


def main():
    nd = _refload.load("botorch.utils.multi_objective.box_decompositions.non_dominated")
    dom = _refload.load("botorch.utils.multi_objective.box_decompositions.dominated")
    out = {}
    for m, n, seed, alphas in MO_ALPHA_CASES:
        g = torch.Generator().manual_seed(seed)
        # points near a concave front plus dominated ones
        Y = torch.rand(n, m, generator=g, dtype=torch.float64)
        Y = Y / Y.norm(dim=-1, keepdim=True) * (0.7 + 0.3 * torch.rand(n, 1, generator=g,
                                                                         dtype=torch.float64))
        ref = torch.full((m,), 0.05, dtype=torch.float64)
        tag = f"m{m}_n{n}_s{seed}"
        out[f"{tag}_Y"], out[f"{tag}_ref"] = Y.numpy(), ref.numpy()
        for a in alphas:
            cb = nd.NondominatedPartitioning(ref_point=ref, Y=Y, alpha=a).get_hypercell_bounds()
            out[f"{tag}_a{a}_lo"], out[f"{tag}_a{a}_hi"] = cb[0].numpy(), cb[1].numpy()
        out[f"{tag}_hv_fast"] = np.asarray(
            nd.FastNondominatedPartitioning(ref_point=ref, Y=Y).compute_hypervolume().item())
        out[f"{tag}_hv_dom"] = np.asarray(
            dom.DominatedPartitioning(ref_point=ref, Y=Y).compute_hypervolume().item())
    path = os.path.join(HERE, "golden_mo.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {len(out)} arrays to {path}")


if __name__ == "__main__":
    main()
