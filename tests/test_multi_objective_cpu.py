"""Box decomposition (host side of qEHVI) and the oracle's qEHVI known answers."""
import numpy as np
import pytest
import torch

from botorch_amd.multi_objective import FastNondominatedPartitioning, is_non_dominated


def _rows_sorted(a):
    a = np.asarray(a)
    return a[np.lexsort(a.T[::-1])]


@pytest.mark.parametrize("prefix,Ykey,ref", [
    ("dtlz2_small", "dtlz2_small_Y", -1.1),
    ("dtlz2", "dtlz2_Y", -1.1),
])
def test_fast_partitioning_matches_reference(golden, prefix, Ykey, ref):
    Y = torch.from_numpy(golden[Ykey])
    p = FastNondominatedPartitioning(torch.full((3,), ref, dtype=torch.float64), Y)
    lo, hi = p.get_hypercell_bounds()
    glo, ghi = golden[f"{prefix}_cells_lower"], golden[f"{prefix}_cells_upper"]
    mine = _rows_sorted(np.concatenate([lo.numpy(), hi.numpy()], axis=1))
    ref_ = _rows_sorted(np.concatenate([glo, ghi], axis=1))
    np.testing.assert_array_equal(mine, ref_)
    np.testing.assert_allclose(p.compute_hypervolume().item(), float(golden[f"{prefix}_hv"]), rtol=1e-12)


def test_pareto_mask_matches_reference(golden):
    Y = torch.from_numpy(golden["dtlz2_Y"])
    np.testing.assert_array_equal(is_non_dominated(Y).numpy(), golden["dtlz2_pareto_mask"])


@pytest.mark.parametrize("name", ["m2", "m3a_refm1", "m3a_ref0", "m3a_ref1", "m3b_refm1"])
def test_partitioning_known_cases(golden, name):
    Y = torch.from_numpy(golden[f"ehvi_{name}_pareto_Y"])
    rp = torch.from_numpy(golden[f"ehvi_{name}_ref_point"])
    p = FastNondominatedPartitioning(rp, Y)
    lo, hi = p.get_hypercell_bounds()
    mine = _rows_sorted(np.concatenate([lo.numpy(), hi.numpy()], axis=1))
    ref_ = _rows_sorted(np.concatenate([golden[f"ehvi_{name}_fnd_lower"], golden[f"ehvi_{name}_fnd_upper"]], axis=1))
    np.testing.assert_array_equal(mine, ref_)
