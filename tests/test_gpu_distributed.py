"""optimize_acqf_sharded on the device: 2 ranks, fresh
processes started with mp.spawn, both on cuda:0 over gloo, each running the
real HIP qExpectedImprovement at C2 size (n = 1024, d = 6, q = 8, S = 256),
and (round 5) C3's qNoisyExpectedImprovement with its pruning replicated on
every rank and C4's qExpectedHypervolumeImprovement over a ModelListGP(3)
with its box decomposition replicated, at reduced n; plus the replicated GP
fit (rank 0 fits, the hyperparameters are broadcast).
The sharded raw-sample evaluation, rank 0's Boltzmann selection, the restart
slices and the final gather must reproduce one process running the same
chunks (init_batch_limit = raw / W, batch_limit = restarts / W), bit for bit
(optim/optimize.py:384-387, optim/initializers.py:411-423) -- the CPU twin is
tests/test_distributed_cpu.py.  Two ranks on one GPU measure nothing; the
8-GPU runs use RCCL."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
WS, B, RAW, Q, S, N = 2, 8, 64, 8, 256, 1024


def _c2_acqf(dev):
    from botorch_amd.acquisition import qExpectedImprovement
    from botorch_amd.models import SingleTaskGP
    from botorch_amd.sampling import SobolQMCNormalSampler
    from botorch_amd.test_functions import Hartmann
    from botorch_amd.utils_sampling import draw_sobol_samples
    b = torch.stack([torch.zeros(6), torch.ones(6)]).to(torch.float64)
    X = draw_sobol_samples(b, N, 1, seed=0).squeeze(1)
    Y = Hartmann(negate=True)(X).unsqueeze(-1)
    m = SingleTaskGP(X.to(dev), Y.to(dev))
    m.covar_module.lengthscale = torch.full((1, 6), 0.5016, dtype=torch.float64)
    m.likelihood.noise = torch.tensor([6.737947e-3], dtype=torch.float64)
    m.eval()
    acqf = qExpectedImprovement(m, float(Y.max()) - 0.3,
                                sampler=SobolQMCNormalSampler(torch.Size([S]), seed=0))
    return acqf, b.to(dev)


def _qnei_acqf(dev):
    """C3's acquisition at reduced size: qNEI over the training inputs with
    prune_baseline (the pruning's Sobol draw is seeded from the global RNG,
    reseeded identically on every rank, so every rank keeps the same r)."""
    from botorch_amd.acquisition import qNoisyExpectedImprovement
    from botorch_amd.models import SingleTaskGP
    from botorch_amd.sampling import SobolQMCNormalSampler
    from botorch_amd.test_functions import Hartmann
    from botorch_amd.utils_sampling import draw_sobol_samples
    b = torch.stack([torch.zeros(6), torch.ones(6)]).to(torch.float64)
    X = draw_sobol_samples(b, 512, 1, seed=0).squeeze(1)
    Y = Hartmann(negate=True)(X).unsqueeze(-1)
    m = SingleTaskGP(X.to(dev), Y.to(dev))
    m.covar_module.lengthscale = torch.full((1, 6), 0.15, dtype=torch.float64)
    m.likelihood.noise = torch.tensor([0.5], dtype=torch.float64)
    m.eval()
    torch.manual_seed(7)
    acqf = qNoisyExpectedImprovement(m, X.to(dev), prune_baseline=True,
                                     sampler=SobolQMCNormalSampler(torch.Size([128]), seed=0))
    assert acqf.X_baseline.shape[0] > 1
    return acqf, b.to(dev)


def _qehvi_acqf(dev):
    """C4's acquisition at reduced size: qEHVI over a ModelListGP of 3 on
    DTLZ2, the FastNondominatedPartitioning built on every rank."""
    from botorch_amd.acquisition import qExpectedHypervolumeImprovement
    from botorch_amd.models import ModelListGP, SingleTaskGP
    from botorch_amd.multi_objective import FastNondominatedPartitioning
    from botorch_amd.sampling import SobolQMCNormalSampler
    from botorch_amd.test_functions import DTLZ2
    g = torch.Generator().manual_seed(0)
    X = torch.rand(256, 6, generator=g, dtype=torch.float64)
    Y = -DTLZ2(dim=6, num_objectives=3, negate=True).evaluate_true(X)
    ms = []
    for t in range(3):
        mm = SingleTaskGP(X.to(dev), Y[:, t:t + 1].to(dev))
        mm.covar_module.lengthscale = torch.full((1, 6), 0.6, dtype=torch.float64)
        mm.likelihood.noise = torch.tensor([1e-3], dtype=torch.float64)
        ms.append(mm.eval())
    ref = torch.full((3,), -1.1, dtype=torch.float64)
    part = FastNondominatedPartitioning(ref, Y)
    acqf = qExpectedHypervolumeImprovement(ModelListGP(*ms), ref.tolist(), part,
                                           sampler=SobolQMCNormalSampler(torch.Size([64]), seed=0))
    return acqf, torch.stack([torch.zeros(6), torch.ones(6)]).to(torch.float64).to(dev)


ACQ = {"qei": (_c2_acqf, Q), "qnei": (_qnei_acqf, 4), "qehvi": (_qehvi_acqf, 3)}


def _opts(gen="scipy"):
    o = {"seed": 5, "maxiter": 25, "batch_limit": B // WS, "init_batch_limit": RAW // WS}
    if gen == "device_joint":
        o["joint"] = True
    return o


def _gen(name):
    from botorch_amd.optim import gen_candidates_device, gen_candidates_scipy
    return gen_candidates_scipy if name == "scipy" else gen_candidates_device


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, port, outdir, gen, acq):
    import torch.distributed as dist
    from botorch_amd.distributed import optimize_acqf_sharded
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(2)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=WS)
    try:
        make, q = ACQ[acq]
        acqf, bounds = make(torch.device("cuda", 0))
        torch.manual_seed(123)
        cands, vals = optimize_acqf_sharded(acqf, bounds, q=q, num_restarts=B, raw_samples=RAW,
                                            options=_opts(gen), gen_candidates=_gen(gen),
                                            return_best_only=False)
        torch.save({"cands": cands.cpu(), "vals": vals.cpu()}, os.path.join(outdir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("acq,gen", [("qei", "scipy"), ("qei", "device"), ("qei", "device_joint"),
                                     ("qnei", "scipy"), ("qnei", "device"),
                                     ("qehvi", "scipy"), ("qehvi", "device")])
def test_sharded_optimize_acqf_on_device_equals_single_process(tmp_path, acq, gen):
    from botorch_amd.optim import optimize_acqf
    mp.spawn(_worker, args=(_port(), str(tmp_path), gen, acq), nprocs=WS, join=True)
    outs = [torch.load(os.path.join(tmp_path, f"r{r}.pt"), weights_only=True) for r in range(WS)]
    make, q = ACQ[acq]
    acqf, bounds = make(torch.device("cuda", 0))
    torch.manual_seed(123)
    cands, vals = optimize_acqf(acqf, bounds, q=q, num_restarts=B, raw_samples=RAW,
                                options=_opts(gen), gen_candidates=_gen(gen), return_best_only=False)
    cands, vals = cands.cpu(), vals.cpu()
    assert vals.shape == (B,) and float(vals.max()) > 0
    for o in outs:
        assert torch.equal(o["cands"], cands) and torch.equal(o["vals"], vals)


def _fit_model(dev):
    from botorch_amd.fit import ExactMarginalLogLikelihood
    from botorch_amd.models import SingleTaskGP
    from botorch_amd.test_functions import Hartmann
    from botorch_amd.utils_sampling import draw_sobol_samples
    b = torch.stack([torch.zeros(6), torch.ones(6)]).to(torch.float64)
    X = draw_sobol_samples(b, 384, 1, seed=0).squeeze(1)
    Y = Hartmann(negate=True)(X).unsqueeze(-1)
    m = SingleTaskGP(X.to(dev), Y.to(dev))
    return m, ExactMarginalLogLikelihood(m.likelihood, m)


def _state(m):
    return torch.cat([m.covar_module.lengthscale.detach().reshape(-1).cpu(),
                      m.likelihood.noise.detach().reshape(-1).cpu(),
                      m.mean_module.constant.detach().reshape(-1).cpu()])


def _fit_worker(rank, port, outdir):
    import torch.distributed as dist
    from botorch_amd.distributed import fit_gpytorch_mll_replicated
    from botorch_amd.fit import fit_gpytorch_mll
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(2)
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=WS)
    try:
        dev = torch.device("cuda", 0)
        m, mll = _fit_model(dev)
        torch.manual_seed(0)
        fit_gpytorch_mll_replicated(mll)
        rep = _state(m)
        # every rank fitting on its own: the DAG Cholesky's dynamic task order
        # must not change the fit (bit-identical closures on every rank)
        m2, mll2 = _fit_model(dev)
        torch.manual_seed(0)
        fit_gpytorch_mll(mll2)
        with torch.no_grad():
            post = m.posterior(torch.rand(5, 6, dtype=torch.float64,
                                          generator=torch.Generator().manual_seed(1)).to(dev))
        torch.save({"rep": rep, "own": _state(m2), "training": m.training,
                    "mean": post.mean.cpu(), "var": post.variance.cpu()},
                   os.path.join(outdir, f"r{rank}.pt"))
    finally:
        dist.destroy_process_group()


def test_replicated_fit_on_device_equals_single_process(tmp_path):
    """fit_gpytorch_mll_replicated (fit.py:75-113): every rank's
    hyperparameters and posterior equal one process's fit bit for bit; an
    independent fit on every rank gives the same bits too."""
    from botorch_amd.fit import fit_gpytorch_mll
    mp.spawn(_fit_worker, args=(_port(), str(tmp_path)), nprocs=WS, join=True)
    outs = [torch.load(os.path.join(tmp_path, f"r{r}.pt"), weights_only=True) for r in range(WS)]
    m, mll = _fit_model(torch.device("cuda", 0))
    torch.manual_seed(0)
    fit_gpytorch_mll(mll)
    ref = _state(m)
    assert float(ref[0]) != 0.5016  # the fit moved the lengthscales
    for o in outs:
        assert not o["training"]
        assert torch.equal(o["rep"], ref) and torch.equal(o["own"], ref)
        assert torch.equal(o["mean"], outs[0]["mean"]) and torch.equal(o["var"], outs[0]["var"])
