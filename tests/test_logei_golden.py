"""LogEI reductions (acquisition/logei.py, utils/safe_math.py): the oracle's
restatement and the product's generic-route torch module against the
reference's own outputs (tests/golden, made by make_golden.py from the
reference safe_math), values and gradients w.r.t. the samples."""
import pytest
import torch

from tests.golden.cases import LOGEI_CASES


def _ref(golden, tag, bname):
    return (torch.from_numpy(golden[f"logei_{tag}_{bname}_acq"]),
            torch.from_numpy(golden[f"logei_{tag}_{bname}_grad"]))


def _inputs(golden, bname):
    obj = torch.from_numpy(golden["logei_obj"]).clone()
    bf = (torch.from_numpy(golden["logei_best_f_s"]) if bname == "persample"
          else torch.full((obj.shape[0],), 0.2, dtype=torch.float64))
    return obj, bf


@pytest.mark.parametrize("tag", list(LOGEI_CASES))
@pytest.mark.parametrize("bname", ["scalar", "persample"])
def test_oracle_logei_matches_reference(golden, tag, bname):
    from oracle.acquisition import qlogei_from_samples
    fat, tau_relu, tau_max = LOGEI_CASES[tag]
    obj, bf = _inputs(golden, bname)
    x = obj.requires_grad_(True)
    acq = qlogei_from_samples(x, bf, fat=fat, tau_relu=tau_relu, tau_max=tau_max)
    (gx,) = torch.autograd.grad(acq.sum(), x)
    ref_acq, ref_g = _ref(golden, tag, bname)
    torch.testing.assert_close(acq.detach(), ref_acq, rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(gx, ref_g, rtol=1e-9, atol=1e-12)


@pytest.mark.parametrize("tag", list(LOGEI_CASES))
@pytest.mark.parametrize("bname", ["scalar", "persample"])
def test_generic_route_logei_matches_reference(golden, tag, bname):
    from botorch_amd.safe_math import fatmax, log_improvement, logmeanexp, smooth_amax
    fat, tau_relu, tau_max = LOGEI_CASES[tag]
    obj, bf = _inputs(golden, bname)
    x = obj.requires_grad_(True)
    li = log_improvement(x, bf.view(-1, 1), tau=tau_relu, fat=fat)
    acq = logmeanexp((fatmax if fat else smooth_amax)(li, dim=-1, tau=tau_max), dim=0)
    (gx,) = torch.autograd.grad(acq.sum(), x)
    ref_acq, ref_g = _ref(golden, tag, bname)
    torch.testing.assert_close(acq.detach(), ref_acq, rtol=1e-12, atol=1e-12)
    torch.testing.assert_close(gx, ref_g, rtol=1e-9, atol=1e-12)


def test_check_tau_rejects_bad_temperatures():
    from botorch_amd.acquisition import _check_tau
    with pytest.raises(ValueError):
        _check_tau(0.0, "tau_max")
    with pytest.raises(ValueError):
        _check_tau(torch.tensor([1.0, 2.0]), "tau_relu")
    assert _check_tau(1e-2, "tau_max") == 1e-2
