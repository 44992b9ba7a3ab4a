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


# ---- approximate decompositions and hypervolumes (golden_mo.npz) -----------------------

@pytest.fixture(scope="module")
def golden_mo():
    import os
    return np.load(os.path.join(os.path.dirname(__file__), "golden", "golden_mo.npz"))


def _mo_cases():
    from tests.golden.cases import MO_ALPHA_CASES
    return [(m, n, s, a) for m, n, s, alphas in MO_ALPHA_CASES for a in alphas]


@pytest.mark.parametrize("m,n,seed,alpha", _mo_cases())
def test_binary_partitioning_matches_reference(golden_mo, m, n, seed, alpha):
    """NondominatedPartitioning(ref, Y, alpha) (non_dominated.py:30-335): the
    binary partitioning with the alpha approximation, m > 2, cell for cell and
    in the reference's order (bo_nd_partition_alpha_host); for m = 2 the
    reference's direct 2-d partition ignores alpha and gives the exact cells
    (FastNondominatedPartitioning's, in reverse order)."""
    from botorch_amd import kernels
    tag = f"m{m}_n{n}_s{seed}"
    Y, ref = torch.from_numpy(golden_mo[tag + "_Y"]), torch.from_numpy(golden_mo[tag + "_ref"])
    rlo, rhi = golden_mo[f"{tag}_a{alpha}_lo"], golden_mo[f"{tag}_a{alpha}_hi"]
    if m == 2:
        lo, hi = kernels.nd_partition_host(Y, ref)
        np.testing.assert_array_equal(lo.numpy()[::-1], rlo)
        np.testing.assert_array_equal(hi.numpy()[::-1], rhi)
        return
    lo, hi = kernels.nd_partition_host(Y, ref, alpha=alpha)
    np.testing.assert_array_equal(lo.numpy(), rlo)
    np.testing.assert_array_equal(hi.numpy(), rhi)
    # batched over samples: every set padded to the common count with empty cells
    Y2 = 0.9 * Y
    lo2, hi2 = kernels.nd_partition_host(torch.stack([Y, Y2]), ref, alpha=alpha)
    for s, Ys in enumerate((Y, Y2)):
        one_lo, one_hi = kernels.nd_partition_host(Ys, ref, alpha=alpha)
        k = one_lo.shape[0]
        assert torch.equal(lo2[s, :k], one_lo) and torch.equal(hi2[s, :k], one_hi)
        assert (lo2[s, k:] == 0).all() and (hi2[s, k:] == 0).all()


@pytest.mark.parametrize("m,n,seed", sorted({(m, n, s) for m, n, s, _ in _mo_cases()}))
def test_hypervolumes_match_reference(golden_mo, m, n, seed):
    """FastNondominatedPartitioning.compute_hypervolume (non_dominated.py:
    445-457) from the cells, and DominatedPartitioning's (dominated.py:51-62)."""
    from botorch_amd import kernels
    from botorch_amd.acquisition import cells_hypervolume, dominated_hypervolume
    tag = f"m{m}_n{n}_s{seed}"
    Y, ref = torch.from_numpy(golden_mo[tag + "_Y"]), torch.from_numpy(golden_mo[tag + "_ref"])
    lo, hi = kernels.nd_partition_host(Y.unsqueeze(0), ref)
    hv = cells_hypervolume(Y.unsqueeze(0), ref, lo, hi)
    assert hv.item() == float(golden_mo[tag + "_hv_fast"])
    np.testing.assert_allclose(dominated_hypervolume(Y.unsqueeze(0), ref).item(),
                               float(golden_mo[tag + "_hv_dom"]), rtol=1e-13)
    # no point above the reference point: zero
    below = torch.full((1, 3, m), -1.0, dtype=torch.float64)
    assert dominated_hypervolume(below, ref).item() == 0.0
