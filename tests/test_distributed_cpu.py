"""Restart sharding over ranks (botorch_amd/distributed.py) with the gloo backend
on CPU, driving a GP-shaped acquisition (qEI on an exact GP, the oracle's CPU
restatement standing in for the device path): W ranks return what one process
returns, bit for bit, when the single process runs the same chunks."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from botorch_amd.distributed import shard_range


class _GPqEI(torch.nn.Module):
    """qExpectedImprovement on a 48-point exact GP over Hartmann6 (fixed Sobol
    base samples), differentiable in X on the CPU."""

    def __init__(self, q=2, S=64):
        super().__init__()
        from botorch_amd.test_functions import Hartmann
        from oracle.gp import ExactGPOracle, GPHyper
        from oracle.sampling import draw_sobol_normal_samples, draw_sobol_samples
        lo = torch.zeros(6, dtype=torch.float64)
        X = draw_sobol_samples(lo, lo + 1, 48, 1, 0).squeeze(1)
        Y = Hartmann(negate=True)(X).unsqueeze(-1)
        self.orc = ExactGPOracle(X, Y, GPHyper(torch.full((6,), 0.35, dtype=torch.float64), 1e-3, 0.0))
        self.Z = draw_sobol_normal_samples(q, S, 3)
        self.best_f = float(Y.max()) - 0.2

    def forward(self, X):
        from oracle.acquisition import qei
        return qei(self.orc, X, self.Z, self.best_f)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


OPTS = {"seed": 5, "maxiter": 30}
B, RAW, Q = 8, 64, 2


def _worker(rank, ws, port, outdir, mode):
    import torch.distributed as dist
    from botorch_amd.distributed import (gather_argmax, gen_batch_initial_conditions_sharded,
                                         optimize_acqf_sharded)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        if mode == "argmax":
            # rank 0 and 1 tie on value 2.0; rank 2.. lower -> lowest tied rank wins
            val = torch.tensor([2.0, 2.0, 1.0, 0.5][rank], dtype=torch.float64)
            cand = torch.full((3, 2), float(rank), dtype=torch.float64)
            best, bv, owner = gather_argmax(val, cand)
            out = {"best": best, "val": bv, "owner": owner}
        else:
            acqf = _GPqEI(q=Q)
            bounds = torch.stack([torch.zeros(6), torch.ones(6)]).to(torch.float64)
            opts = dict(OPTS, batch_limit=B // ws, init_batch_limit=RAW // ws)
            torch.manual_seed(123)
            ics = gen_batch_initial_conditions_sharded(acqf, bounds, Q, B, RAW, options=opts)
            torch.manual_seed(123)
            cand, val = optimize_acqf_sharded(acqf, bounds, q=Q, num_restarts=B, raw_samples=RAW,
                                              options=opts)
            torch.manual_seed(123)
            cands, vals = optimize_acqf_sharded(acqf, bounds, q=Q, num_restarts=B, raw_samples=RAW,
                                                options=opts, return_best_only=False)
            out = {"ics": ics, "cand": cand, "val": val, "cands": cands, "vals": vals}
        torch.save(out, os.path.join(outdir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


def _run(ws, mode, tmp_path):
    port = _free_port()
    mp.spawn(_worker, args=(ws, port, str(tmp_path), mode), nprocs=ws, join=True)
    return [torch.load(os.path.join(tmp_path, f"r{r}.pt"), weights_only=True) for r in range(ws)]


@pytest.mark.parametrize("total,ws", [(512, 8), (10, 3), (3, 4), (0, 2), (7, 1)])
def test_shard_range_partitions(total, ws):
    spans = [shard_range(total, ws, r) for r in range(ws)]
    assert spans[0][0] == 0 and spans[-1][1] == total
    for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
        assert a1 == b0 and a1 >= a0
    sizes = [b - a for a, b in spans]
    assert max(sizes) - min(sizes) <= 1


def test_gather_argmax_ties_lowest_rank(tmp_path):
    outs = _run(2, "argmax", tmp_path)
    for o in outs:
        assert o["owner"] == 0 and float(o["val"]) == 2.0
        assert torch.equal(o["best"], torch.zeros(3, 2, dtype=torch.float64))


@pytest.mark.parametrize("ws", [2, 4])
def test_sharded_optimize_acqf_equals_single_process(tmp_path, ws):
    """W ranks vs one process running the same chunks (init_batch_limit =
    raw / W, batch_limit = restarts / W): identical initial conditions, all
    restarts' candidates and values, and the same argmax, bit for bit."""
    from botorch_amd.optim import gen_batch_initial_conditions, optimize_acqf
    outs = _run(ws, "opt", tmp_path)
    acqf = _GPqEI(q=Q)
    bounds = torch.stack([torch.zeros(6), torch.ones(6)]).to(torch.float64)
    opts = dict(OPTS, batch_limit=B // ws, init_batch_limit=RAW // ws)
    torch.manual_seed(123)
    ics = gen_batch_initial_conditions(acqf, bounds, Q, B, RAW, options=opts)
    torch.manual_seed(123)
    cand, val = optimize_acqf(acqf, bounds, q=Q, num_restarts=B, raw_samples=RAW, options=opts)
    torch.manual_seed(123)
    cands, vals = optimize_acqf(acqf, bounds, q=Q, num_restarts=B, raw_samples=RAW, options=opts,
                                return_best_only=False)
    assert float(val) > 0
    for o in outs:
        assert torch.equal(o["ics"], ics)
        assert torch.equal(o["cands"], cands) and torch.equal(o["vals"], vals)
        assert torch.equal(o["cand"], cand) and torch.equal(o["val"].reshape(()), val.reshape(()))


def _fit_worker(rank, ws, port, outdir, mode):
    """fit_gpytorch_mll_replicated over gloo with a stand-in fit routine (the
    device MLL needs a GPU; tests/test_gpu_distributed.py runs the real one):
    rank 0's fitted hyperparameters reach every rank bit for bit, a failure on
    rank 0 raises on every rank, and a ModelListGP's members all travel."""
    import torch.distributed as dist
    from botorch_amd.distributed import fit_gpytorch_mll_replicated
    from botorch_amd.exceptions import ModelFittingError
    from botorch_amd.fit import ExactMarginalLogLikelihood, SumMarginalLogLikelihood
    from botorch_amd.models import ModelListGP, SingleTaskGP
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        g = torch.Generator().manual_seed(0)
        X = torch.rand(32, 6, generator=g, dtype=torch.float64)
        Y = torch.rand(32, 2, generator=g, dtype=torch.float64)
        calls = []

        def fake_fit(mll, **kw):  # "fits" to rank-specific values: only rank 0's may survive
            calls.append(rank)
            mods = [s.model for s in mll.mlls] if isinstance(mll, SumMarginalLogLikelihood) \
                else [mll.model]
            if mode == "fail":
                raise ModelFittingError("All attempts to fit the model have failed.")
            for t, mm in enumerate(mods):
                mm.covar_module.lengthscale = torch.linspace(0.1, 0.7, 6, dtype=torch.float64
                                                             ).reshape(1, 6) * (1 + t) / 3 + rank
                mm.likelihood.noise = torch.tensor([1e-3 * (t + 1) / 7 + rank], dtype=torch.float64)
                mm.mean_module.constant = 0.1 / 3 * (t + 1) + rank
            return mll.eval()

        if mode == "list":
            model = ModelListGP(SingleTaskGP(X, Y[:, :1]), SingleTaskGP(X, Y[:, 1:]))
            mll = SumMarginalLogLikelihood(None, model)
            mods = list(model.models)
        else:
            model = SingleTaskGP(X, Y[:, :1])
            mll = ExactMarginalLogLikelihood(model.likelihood, model)
            mods = [model]
        out = {"calls": calls}
        try:
            fit_gpytorch_mll_replicated(mll, fit=fake_fit)
            out["state"] = [torch.cat([mm.covar_module.lengthscale.detach().reshape(-1),
                                       mm.likelihood.noise.detach().reshape(-1),
                                       mm.mean_module.constant.detach().reshape(-1)])
                            for mm in mods]
            out["training"] = any(mm.training for mm in mods)
        except ModelFittingError as e:
            out["error"] = str(e)
        torch.save(out, os.path.join(outdir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode,ws", [("single", 2), ("single", 3), ("list", 2), ("fail", 2)])
def test_replicated_fit_broadcasts_rank0(tmp_path, mode, ws):
    port = _free_port()
    mp.spawn(_fit_worker, args=(ws, port, str(tmp_path), mode), nprocs=ws, join=True)
    outs = [torch.load(os.path.join(tmp_path, f"r{r}.pt"), weights_only=True) for r in range(ws)]
    assert outs[0]["calls"] == [0] and all(o["calls"] == [] for o in outs[1:])
    if mode == "fail":
        assert all("failed" in o["error"] for o in outs)
        return
    for o in outs:
        assert not o["training"]
        for a, b in zip(o["state"], outs[0]["state"]):
            assert torch.equal(a, b)
    # rank 0's values, not any other rank's
    assert float(outs[0]["state"][0][0]) < 1.0
