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


def test_native_batched_partitions_match_single_sets():
    """bo_nd_partition_host over a batch of point sets: each set's cells equal
    its own single-set decomposition, padded with empty (zero) cells to the
    common count (BoxDecompositionList, box_decomposition_list.py:62-94)."""
    import torch
    from botorch_amd import kernels
    g = torch.Generator().manual_seed(4)
    for m in (2, 3):
        Y = torch.rand(6, 25, m, generator=g, dtype=torch.float64)
        Y[3] = -1.0  # an empty front -> the single cell [ref, inf)
        ref = torch.zeros(m, dtype=torch.float64)
        lo, hi = kernels.nd_partition_host(Y, ref)
        for s in range(6):
            l1, h1 = kernels.nd_partition_host(Y[s], ref)
            k = l1.shape[0]
            assert torch.equal(lo[s, :k], l1) and torch.equal(hi[s, :k], h1)
            assert (lo[s, k:] == 0).all() and (hi[s, k:] == 0).all()
        l3, h3 = kernels.nd_partition_host(Y[3], ref)
        assert torch.equal(l3, ref.view(1, m)) and torch.isinf(h3).all()
