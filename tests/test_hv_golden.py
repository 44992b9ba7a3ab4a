"""The oracle's exact hypervolume against the reference's DominatedPartitioning
(tests/golden hv_* fixtures), and hypercell sums of the host partitioning."""
import numpy as np
import pytest
import torch

from tests.golden.cases import HV_CASES


@pytest.mark.parametrize("m,n", HV_CASES)
def test_oracle_hypervolume_matches_reference(golden, m, n):
    from oracle.acquisition import hypervolume
    Y = torch.from_numpy(golden[f"hv_m{m}_n{n}_Y"])
    ref = torch.from_numpy(golden[f"hv_m{m}_n{n}_ref"])
    assert abs(hypervolume(Y, ref).item() - float(golden[f"hv_m{m}_n{n}_hv"])) < 1e-12
    for e, hv in zip(torch.from_numpy(golden[f"hv_m{m}_n{n}_extra"]), golden[f"hv_m{m}_n{n}_hv_plus"]):
        assert abs(hypervolume(torch.cat([Y, e.view(1, -1)]), ref).item() - hv) < 1e-12


@pytest.mark.parametrize("m,n", HV_CASES)
def test_partition_cells_give_reference_improvements(golden, m, n):
    """HVI of one extra point = sum over the non-dominated cells of the box
    clipped by the point (the per-sample quantity the qNEHVI kernel sums)."""
    from botorch_amd.multi_objective import FastNondominatedPartitioning
    Y = torch.from_numpy(golden[f"hv_m{m}_n{n}_Y"])
    ref = torch.from_numpy(golden[f"hv_m{m}_n{n}_ref"])
    lo, hi = FastNondominatedPartitioning(ref, Y).get_hypercell_bounds()
    hv0 = float(golden[f"hv_m{m}_n{n}_hv"])
    for e, hv in zip(torch.from_numpy(golden[f"hv_m{m}_n{n}_extra"]), golden[f"hv_m{m}_n{n}_hv_plus"]):
        hvi = (torch.minimum(hi, e) - lo).clamp_min(0).prod(dim=-1).sum().item()
        assert abs(hvi - (hv - hv0)) < 1e-12
