"""Restart sharding over ranks (botorch_amd/distributed.py) with the gloo backend,
world_size 2, on CPU: the only collective is the final argmax all-gather."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from botorch_amd.distributed import shard_range


class _Bumps(torch.nn.Module):
    """Multimodal CPU acquisition surrogate (sum over t-batches is separable,
    like every acquisition function optimize_acqf drives)."""

    def forward(self, X):
        X = X if X.dim() > 2 else X.unsqueeze(0)
        c1 = torch.tensor([0.2, 0.7], dtype=X.dtype)
        c2 = torch.tensor([0.8, 0.3], dtype=X.dtype)
        f = (torch.exp(-20 * ((X - c1) ** 2).sum(-1)) + 1.3 * torch.exp(-30 * ((X - c2) ** 2).sum(-1)))
        return f.sum(-1)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, ws, port, outdir, mode):
    import torch.distributed as dist
    from botorch_amd.distributed import gather_argmax, optimize_acqf_sharded
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        if mode == "argmax":
            # rank 0 and 1 tie on value 2.0; rank 2.. lower -> lowest tied rank wins
            val = torch.tensor([2.0, 2.0, 1.0, 0.5][rank], dtype=torch.float64)
            cand = torch.full((3, 2), float(rank), dtype=torch.float64)
            best, bv, owner = gather_argmax(val, cand)
            torch.save({"best": best, "val": bv, "owner": owner}, os.path.join(outdir, f"r{rank}.pt"))
        else:
            bounds = torch.tensor([[0.0, 0.0], [1.0, 1.0]], dtype=torch.float64)
            cand, val = optimize_acqf_sharded(_Bumps(), bounds, q=1, num_restarts=4, raw_samples=32,
                                              options={"seed": 5, "maxiter": 50})
            torch.save({"cand": cand, "val": val}, os.path.join(outdir, f"r{rank}.pt"))
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


def test_optimize_acqf_sharded_matches_local_shards(tmp_path):
    from botorch_amd.optim import optimize_acqf
    outs = _run(2, "opt", tmp_path)
    # every rank ends with the same global answer
    assert torch.equal(outs[0]["cand"], outs[1]["cand"])
    # ... which is the best of the two per-shard runs (seed + rank, half the work each)
    bounds = torch.tensor([[0.0, 0.0], [1.0, 1.0]], dtype=torch.float64)
    local = [optimize_acqf(_Bumps(), bounds, q=1, num_restarts=2, raw_samples=16,
                           options={"seed": 5 + r, "maxiter": 50}) for r in range(2)]
    best = max(range(2), key=lambda r: float(local[r][1]))
    torch.testing.assert_close(outs[0]["cand"], local[best][0])
    torch.testing.assert_close(outs[0]["val"].reshape(()), local[best][1].reshape(()))
    # the global optimum of the surrogate is the taller bump
    torch.testing.assert_close(outs[0]["cand"].reshape(-1), torch.tensor([0.8, 0.3], dtype=torch.float64),
                               atol=1e-3, rtol=0)
