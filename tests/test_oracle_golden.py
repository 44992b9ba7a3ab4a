"""Pin the CPU oracle against the reference's own outputs (tests/golden)."""
import numpy as np
import pytest
import torch

from oracle.sampling import draw_sobol_normal_samples, draw_sobol_samples
from tests.golden.cases import SOBOL_NORMAL_CASES, SOBOL_BOX_CASES


@pytest.mark.parametrize("d,n,seed", SOBOL_NORMAL_CASES)
def test_sobol_normal_matches_reference(golden, d, n, seed):
    z = draw_sobol_normal_samples(d, n, seed).numpy()
    ref = golden[f"sobol_normal_d{d}_n{n}_s{seed}"]
    assert z.shape == ref.shape
    np.testing.assert_array_equal(z, ref)


@pytest.mark.parametrize("n,q,d,seed", SOBOL_BOX_CASES)
def test_sobol_box_matches_reference(golden, n, q, d, seed):
    lo = torch.zeros(d, dtype=torch.float64)
    hi = torch.ones(d, dtype=torch.float64)
    x = draw_sobol_samples(lo, hi, n, q, seed).numpy()
    np.testing.assert_array_equal(x, golden[f"sobol_box_n{n}_q{q}_d{d}_s{seed}"])
