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
        self.S = S
        self.Z = {q: draw_sobol_normal_samples(q, S, 3)}
        self.best_f = float(Y.max()) - 0.2
        self.X_pending = None

    def set_X_pending(self, X_pending=None):
        self.X_pending = None if X_pending is None else X_pending.detach().clone()

    def forward(self, X):
        from oracle.acquisition import qei
        from oracle.sampling import draw_sobol_normal_samples
        if self.X_pending is not None:   # concatenate_pending_points
            X = torch.cat([X, self.X_pending.expand(*X.shape[:-2], *self.X_pending.shape)], dim=-2)
        q = X.shape[-2]
        if q not in self.Z:
            self.Z[q] = draw_sobol_normal_samples(q, self.S, 3)
        return qei(self.orc, X, self.Z[q], self.best_f)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


OPTS = {"seed": 5, "maxiter": 30}
B, RAW, Q = 8, 64, 2
# x0 + x1 <= 1.2 (Σ coeff x >= rhs form, optimize.py:417-421), feature 5 fixed
INEQ = [(torch.tensor([0, 1]), torch.tensor([-1.0, -1.0], dtype=torch.float64), -1.2)]
FIXED = {5: 0.3}


def _round2(X):
    """A post_processing_func (optimize.py:371-376): rounds every coordinate."""
    return torch.round(X * 100) / 100


def _ics_generator(acq_function, bounds, q, num_restarts, raw_samples, **kw):
    """A caller's ic_generator: draws from the global generator (so only rank
    0's draw may be used)."""
    return bounds[0] + (bounds[1] - bounds[0]) * torch.rand(num_restarts, q, bounds.shape[-1],
                                                            dtype=bounds.dtype)


def _opt_calls(optimize, ics_fn, acqf, bounds, mode, ws):
    """The calls the sharded and the single-process runs make (same order,
    same global RNG state before each)."""
    opts = dict(OPTS, batch_limit=B // ws, init_batch_limit=RAW // ws)
    out = {}
    if mode == "opt":
        torch.manual_seed(123)
        out["ics"] = ics_fn(acqf, bounds, Q, B, RAW, options=opts)
        torch.manual_seed(123)
        out["cand"], out["val"] = optimize(acqf, bounds, q=Q, num_restarts=B, raw_samples=RAW,
                                           options=opts)
        torch.manual_seed(123)
        out["cands"], out["vals"] = optimize(acqf, bounds, q=Q, num_restarts=B, raw_samples=RAW,
                                             options=opts, return_best_only=False)
    elif mode == "constrained":
        copts = dict(opts, n_burnin=200, n_thinning=4, maxiter=20)
        torch.manual_seed(7)
        out["ics"] = ics_fn(acqf, bounds, Q, B, RAW, fixed_features=FIXED, options=copts,
                            inequality_constraints=INEQ)
        torch.manual_seed(7)
        out["cands"], out["vals"] = optimize(acqf, bounds, q=Q, num_restarts=B, raw_samples=RAW,
                                             options=copts, fixed_features=FIXED,
                                             inequality_constraints=INEQ, return_best_only=False)
        torch.manual_seed(7)
        out["cand"], out["val"] = optimize(acqf, bounds, q=Q, num_restarts=B, raw_samples=RAW,
                                           options=copts, fixed_features=FIXED,
                                           inequality_constraints=INEQ)
    elif mode == "misc":
        torch.manual_seed(11)
        out["cands"], out["vals"] = optimize(acqf, bounds, q=Q, num_restarts=B, raw_samples=RAW,
                                             options=opts, post_processing_func=_round2,
                                             timeout_sec=60.0, return_best_only=False)
        torch.manual_seed(11)
        out["cand"], out["val"] = optimize(acqf, bounds, q=Q, num_restarts=B, raw_samples=RAW,
                                           options=opts, sequential=True)
        torch.manual_seed(11)
        out["cands_icg"], out["vals_icg"] = optimize(acqf, bounds, q=Q, num_restarts=B,
                                                     options=opts, ic_generator=_ics_generator,
                                                     return_best_only=False)
        out["all_fixed"], out["all_fixed_val"] = optimize(
            acqf, bounds, q=Q, num_restarts=B, raw_samples=RAW, options=opts,
            fixed_features={i: 0.1 * (i + 1) for i in range(6)})
    return out


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
            out = _opt_calls(optimize_acqf_sharded, gen_batch_initial_conditions_sharded, acqf,
                             bounds, mode, ws)
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


@pytest.mark.parametrize("ws,mode", [(2, "opt"), (4, "opt"), (2, "constrained"), (2, "misc")])
def test_sharded_optimize_acqf_equals_single_process(tmp_path, ws, mode):
    """W ranks vs one process running the same chunks (init_batch_limit =
    raw / W, batch_limit = restarts / W): identical initial conditions, all
    restarts' candidates and values, and the same argmax, bit for bit -- also
    with fixed features + a linear inequality constraint (polytope raw samples,
    SLSQP), a post_processing_func, timeout_sec, sequential greedy q, a
    caller's ic_generator and the all-fixed shortcut (optimize.py:397-419)."""
    from botorch_amd.optim import gen_batch_initial_conditions, optimize_acqf
    outs = _run(ws, mode, tmp_path)
    acqf = _GPqEI(q=Q)
    bounds = torch.stack([torch.zeros(6), torch.ones(6)]).to(torch.float64)
    ref = _opt_calls(optimize_acqf, gen_batch_initial_conditions, acqf, bounds, mode, ws)
    assert float(ref["val"].reshape(-1)[0]) > 0
    if mode == "constrained":
        for X in (ref["ics"], ref["cands"]):
            assert (X[..., 5] == 0.3).all()
            assert (X[..., 0] + X[..., 1] <= 1.2 + 1e-6).all()
    if mode == "misc":
        assert torch.equal(ref["cands"], _round2(ref["cands"]))
        assert ref["cand"].shape == (Q, 6) and ref["val"].shape == (Q,)
        assert torch.equal(ref["all_fixed"][0], torch.tensor([0.1 * (i + 1) for i in range(6)],
                                                             dtype=torch.float64))
    for o in outs:
        assert set(o) == set(ref)
        for k in ref:
            a, b = o[k], ref[k]
            if torch.is_tensor(b):
                assert torch.equal(a.reshape(b.shape), b), k


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
            if mode == "crash":   # not a fitting failure: a kernel error, bad kwargs, ...
                raise RuntimeError("device fault in the MLL closure")
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
        except (ModelFittingError, RuntimeError) as e:
            out["error"] = str(e)
            out["error_type"] = type(e).__name__
        torch.save(out, os.path.join(outdir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode,ws", [("single", 2), ("single", 3), ("list", 2), ("fail", 2),
                                     ("crash", 2), ("crash", 3)])
def test_replicated_fit_broadcasts_rank0(tmp_path, mode, ws):
    port = _free_port()
    mp.spawn(_fit_worker, args=(ws, port, str(tmp_path), mode), nprocs=ws, join=True)
    outs = [torch.load(os.path.join(tmp_path, f"r{r}.pt"), weights_only=True) for r in range(ws)]
    assert outs[0]["calls"] == [0] and all(o["calls"] == [] for o in outs[1:])
    if mode == "fail":
        assert all("failed" in o["error"] for o in outs)
        return
    if mode == "crash":   # raised on every rank (no rank left waiting in the broadcast)
        assert outs[0]["error_type"] == "RuntimeError" and "device fault" in outs[0]["error"]
        assert all(o["error_type"] == "RuntimeError" and "rank 0" in o["error"] for o in outs[1:])
        return
    for o in outs:
        assert not o["training"]
        for a, b in zip(o["state"], outs[0]["state"]):
            assert torch.equal(a, b)
    # rank 0's values, not any other rank's
    assert float(outs[0]["state"][0][0]) < 1.0
