"""acquisition._host_scalar: the host value of a scalar buffer (qEI's best_f)
is read once per tensor and version -- an in-place change or a replacement
tensor (even one the allocator places where the old one was) is read again."""
import torch

from botorch_amd.acquisition import _host_scalar


class _M(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.register_buffer("best_f", torch.tensor(1.5, dtype=torch.float64))


def test_host_scalar_follows_in_place_changes_and_replacements():
    m = _M()
    assert _host_scalar(m, "best_f") == 1.5
    assert _host_scalar(m, "best_f") == 1.5
    m.best_f.fill_(2.5)
    assert _host_scalar(m, "best_f") == 2.5
    for x in (3.0, 4.0, 5.0, 6.0):  # replacements, old tensors freed in between
        m.best_f = torch.tensor(x, dtype=torch.float64)
        assert _host_scalar(m, "best_f") == x
