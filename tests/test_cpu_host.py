"""CPU-side checks: test functions vs. golden, the C ABI library loads and exports."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_hartmann_matches_reference(golden):
    from botorch_amd.test_functions import Hartmann
    h = Hartmann(negate=True)
    for xk, yk in (("hartmann6_X", "hartmann6_Y"), ("hartmann6_rand_X", "hartmann6_rand_Y")):
        y = h(torch.from_numpy(golden[xk])).numpy()
        np.testing.assert_array_equal(y, golden[yk])


def test_dtlz2_matches_reference(golden):
    from botorch_amd.test_functions import DTLZ2
    f = DTLZ2(dim=6, num_objectives=3, negate=True)
    y = f(torch.from_numpy(golden["dtlz2_X"])).numpy()
    np.testing.assert_array_equal(y, golden["dtlz2_Y"])


def _header_symbols():
    src = open(os.path.join(ROOT, "include", "botorch_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[a-z0-9_]+\*?\s+\*?(bo_[a-z0-9_]+)\(", src, flags=re.M)))


def test_library_exports_every_header_symbol():
    from botorch_amd import _lib
    syms = _header_symbols()
    assert len(syms) >= 10
    handle = ctypes.CDLL(_lib.LIB_PATH)
    for s in syms:
        assert hasattr(handle, s), s
    assert set(syms) == set(_lib.exported_symbols()), set(syms) ^ set(_lib.exported_symbols())
    lib = _lib.lib()
    assert lib.bo_version() == _lib.ABI_VERSION == 11
    assert lib.bo_padded_order(4096) == 4096 and lib.bo_padded_order(20) == 128


def test_split_plan_geometry():
    """Host-side plan of bo_post_partials (no GPU call): one pass where the
    tile grid fills the slots, stream-K where the triangular tiles are too few
    or too unequal."""
    from botorch_amd import kernels
    assert kernels.split_plan(512, 16, 4096)[0] == 0      # C3: 2048 tiles, one pass
    assert kernels.split_plan(64, 8, 1024)[0] == -1       # C2: 8 x 4 tiles
    assert kernels.split_plan(64, 16, 4096)[0] == -1      # a rank's b = 64 share of C3
    assert kernels.split_plan(1, 1, 4096)[0] == -1
    assert kernels.split_plan(64, 8, 100)[0] == 0         # nothing to split


def _split_table(B, q, n, kc):
    import ctypes
    import numpy as np
    from botorch_amd import _lib
    ns, nw = ctypes.c_int(), ctypes.c_int()
    _lib.check(_lib.lib().bo_post_split_table(B, q, n, kc, None, 0, None, -1, ctypes.byref(ns),
                                              ctypes.byref(nw)), "split_table")
    segs = np.zeros((ns.value, 4), dtype=np.int32)
    off = np.zeros(nw.value + 1, dtype=np.int32)
    _lib.check(_lib.lib().bo_post_split_table(B, q, n, kc, segs.ctypes.data, ns.value,
                                              off.ctypes.data, nw.value, ctypes.byref(ns),
                                              ctypes.byref(nw)), "split_table")
    return segs, off


@pytest.mark.parametrize("B,q,n,kc", [(64, 16, 4096, -1), (64, 8, 1024, -1), (9, 5, 513, -1),
                                      (64, 8, 1024, 64), (20, 3, 1000, 128), (1, 1, 4096, -1)])
def test_split_table_covers_every_tile_once(B, q, n, kc):
    """Every (column tile, row tile) k-range [0, min(n, 128 (ci + 1))) is
    covered exactly once by the segments; chunk numbers are dense, in k order
    within a tile, -1 exactly for whole-tile segments; stream-K shares differ
    by at most one tile boundary's rounding."""
    import numpy as np
    from botorch_amd import kernels
    Qp, nrows_pad, nC = kernels.geometry(B, q, n)
    nI = nrows_pad // 128
    segs, off = _split_table(B, q, n, kc)
    tiles = {}
    for ci_ii, kb, ke, ch in segs.tolist():
        tiles.setdefault((ci_ii & 0xffff, ci_ii >> 16), []).append((kb, ke, ch))
    assert len(tiles) == nC * nI
    chunks = []
    for (ci, ii), lst in tiles.items():
        lst.sort()
        assert lst[0][0] == 0 and lst[-1][1] == min(n, 128 * (ci + 1))
        assert all(a[1] == b[0] for a, b in zip(lst, lst[1:]))
        assert all(kb % 16 == 0 and ke > kb for kb, ke, _ in lst)
        if len(lst) == 1:
            assert lst[0][2] == -1
        else:
            cs = [c for _, _, c in lst]
            assert cs == list(range(cs[0], cs[0] + len(cs)))
            chunks += cs
    assert sorted(chunks) == list(range(len(chunks)))
    assert off[0] == 0 and off[-1] == len(segs) and np.all(np.diff(off) >= 0)
    if kc == -1:
        # one lane of equal shares per row tile: every non-empty workgroup but
        # the last of each lane has the same k-step count
        steps = [sum(-(-(ke - kb) // 16) for _, kb, ke, _ in segs[off[w]:off[w + 1]].tolist())
                 for w in range(len(off) - 1)]
        busy = sorted(s for s in steps if s > 0)
        assert len(steps) <= 512 + 8 * nI
        assert sum(1 for s in busy if s != busy[-1]) <= nI


def test_custom_ops_registered_with_meta_shapes():
    """torch.ops.bo.* exist and their fake (meta) implementations give the
    shapes the device kernels produce -- no device needed."""
    import torch
    from botorch_amd import ops
    for name in ops.OPS:
        assert hasattr(torch.ops.bo, name), name
    meta = dict(device="meta", dtype=torch.float64)
    n, d, B, q = 300, 6, 5, 4
    Xt, y, ls = torch.empty(n, d, **meta), torch.empty(n, **meta), torch.empty(d, **meta)
    L, Linv, U, beta, alpha, Xs, jit = torch.ops.bo.gp_cache(Xt, y, ls, 1.0, 1e-3, 0.0, 0)
    assert L.shape == U.shape == (384, 384) and Xs.shape == (n, 8) and jit.shape == (1,)
    X = torch.empty(B, q, d, **meta)
    mean, cov, Xq, Rt, Wt = torch.ops.bo.gp_posterior(X, Xt, Xs, U, Linv, beta, alpha, ls, 0, 1.0,
                                                      0.0, 0.0, 1.0, True)
    assert mean.shape == (B, q) and cov.shape == (B, q, q)
    assert Xq.shape == (128, 8) and Rt.shape == (384, 128) and Wt.shape == (384, 128)
    Z = torch.empty(64, q, **meta)
    outs = torch.ops.bo.qmc_acq(X, Xt, Xs, U, Linv, beta, alpha, ls, Z, None, 0, 1, 1.0, 0.0, 0.0,
                                1.0, 0.5, True, 1.0, 1.0, False)
    assert outs[0].shape == (B,) and outs[7].dtype == torch.int32
    Sp, mp, Xq2, Rt2 = torch.ops.bo.post_partials(X, Xt, Xs, U, beta, ls, 0, 1.0, False)
    assert Sp.shape == (3, 8, 16, 16) and mp.shape == (3, 128) and Rt2.numel() == 0


def test_arg_records_match_c_layout():
    """ABI-9 parameter records: the ctypes layouts equal the C header's sizeof,
    the header fields are filled, and a wrong abi_version / struct_size is
    refused with an error code before anything is launched."""
    import ctypes
    from botorch_amd import _lib
    lib = _lib.lib()
    for cname, rec in _lib.ARG_RECORDS.items():
        assert lib.bo_struct_size(cname.encode()) == ctypes.sizeof(rec), cname
        r = rec()
        assert r.struct_size == ctypes.sizeof(rec) and r.abi_version == _lib.ABI_VERSION
    assert lib.bo_struct_size(b"NoSuchStruct") < 0
    a = _lib.PostPartialsArgs(B=1, q=1, d=1)
    a.abi_version = 8
    assert lib.bo_post_partials_v(ctypes.byref(a), None) != 0
    a = _lib.LbfgsStepArgs(B=1, n=1, m=1)
    a.struct_size = 8
    assert lib.bo_lbfgs_step_v(ctypes.byref(a), None) != 0


def test_settings_flags_mirror_reference():
    """settings.py:16-77 switch semantics; propagate_grads with training data
    that require grad raises (no silent detach) before any device work."""
    from botorch_amd import settings
    from botorch_amd.exceptions import UnsupportedError
    from botorch_amd.models import SingleTaskGP
    assert settings.propagate_grads.off() and settings.validate_input_scaling.on()
    with settings.propagate_grads(True):
        assert settings.propagate_grads.on()
        with settings.propagate_grads(False):
            assert settings.propagate_grads.off()
        assert settings.propagate_grads.on()
    assert settings.propagate_grads.off()
    X = torch.rand(8, 2, dtype=torch.float64, requires_grad=True)
    m = SingleTaskGP(X, torch.rand(8, 1, dtype=torch.float64)).eval()
    with settings.propagate_grads(True):
        with pytest.raises(UnsupportedError):
            m.prediction_cache()


def test_native_torch_operators_load():
    """The TORCH_LIBRARY operators (csrc/torch/bo_torch.cpp) load on the host
    and declare their schemas; the ladder poll of a device that never
    deferred anything reports no status (no device needed)."""
    import torch
    from botorch_amd import _lib
    ops = _lib.torch_ops()
    for name in ("qmc_acq_native", "qmc_acq_eager", "ladder_defer", "ladder_poll", "post_timing",
                 "post_timing_read"):
        assert hasattr(ops, name), name
    schema = str(torch.ops.bo.qmc_acq_native.default._schema)
    assert "bool need_grad" in schema and "Tensor[]" in schema
    assert torch.ops.bo.ladder_poll(7).tolist() == [0.0, 0.0, 0.0]
    torch.ops.bo.post_timing(False)
    assert torch.ops.bo.post_timing_read().numel() == 0


def test_quad_plan_geometries(monkeypatch):
    """bo_post_quad_plan (host): opt-in (BO_POST_QUAD=auto), the quad plan
    takes the stream-K geometries with n <= 2048 and <= 1024 units (C2), not
    the C3 one-pass grid, large n or many units; BO_POST_QUAD=0
    disables and =1 forces it; the partial count is that of the chunks (of 1
    by default) of block pairs (64 x 64 blocks of A^{-1}) sharing a block row."""
    import ctypes
    from botorch_amd import _lib
    lib = _lib.lib()

    def pairs(B, q, n):
        out = ctypes.c_int()
        assert lib.bo_post_quad_plan(B, q, n, ctypes.byref(out)) == 0
        return out.value

    monkeypatch.delenv("BO_POST_QUAD", raising=False)
    def chunks(nb, g=1):  # partials per row tile: sum_kb ceil((nb - kb) / g)
        return sum(-(-(nb - kb) // g) for kb in range(nb))

    assert pairs(64, 8, 1024) == 0                  # opt-in: the R route by default
    monkeypatch.setenv("BO_POST_QUAD", "auto")
    assert pairs(64, 8, 1024) == chunks(16) == 136  # C2: 136 pairs, 544 pair units
    assert pairs(50, 3, 1500) == chunks(24)         # 600 pair units, ragged n
    assert pairs(33, 16, 2048) == 0                 # 2640 pair units: the R route
    assert pairs(512, 16, 4096) == 0 and pairs(64, 16, 4096) == 0 and pairs(0, 8, 1024) == 0
    monkeypatch.setenv("BO_POST_QUAD", "0")
    assert pairs(64, 8, 1024) == 0
    monkeypatch.setenv("BO_POST_QUAD", "1")
    assert pairs(512, 16, 4096) == chunks(64)


def test_capture_status_merge_never_overwrites():
    """kernels.record_capture_status: inside one graph capture, the native
    route (its finalisation folds the ladder status into the graph's pinned
    words) and any device-side status of another route are both kept --
    device statuses combine by max, a device status beside the native route
    becomes ("native+", what, packed) in either order (graphs.py copies it to
    a second pinned pair)."""
    from botorch_amd import kernels
    idx = 7
    t = lambda a, b: torch.tensor([a, b], dtype=torch.float64)  # noqa: E731
    try:
        for order in ("native_first", "device_first"):
            kernels._CAPTURE[idx] = None
            if order == "native_first":
                kernels.record_capture_status(idx, None, "qEI")
                kernels.record_capture_status(idx, t(0.0, 1e-8), "qEHVI")
                kernels.record_capture_status(idx, t(2.0, 0.0), "qEHVI")
            else:
                kernels.record_capture_status(idx, t(0.0, 1e-8), "qEHVI")
                kernels.record_capture_status(idx, None, "qEI")
                kernels.record_capture_status(idx, t(2.0, 0.0), "qEHVI")
                kernels.record_capture_status(idx, None, "qEI")
            st = kernels._CAPTURE[idx]
            assert st[0] == "native+"
            assert torch.equal(st[2], t(2.0, 1e-8))
        kernels._CAPTURE[idx] = None
        kernels.record_capture_status(idx, t(1.0, 0.0), "a")
        kernels.record_capture_status(idx, t(0.0, 1e-6), "b")
        assert torch.equal(kernels._CAPTURE[idx][0], t(1.0, 1e-6))
        kernels._CAPTURE[idx] = None
        kernels.record_capture_status(idx, None, "qEI")
        kernels.record_capture_status(idx, None, "qEI")
        assert kernels._CAPTURE[idx] == ("native", "qEI")
    finally:
        kernels._CAPTURE.pop(idx, None)
