#!/usr/bin/env python3
"""Headline benchmark: batched qEI forward (q x restarts x MC evals/s) on MI355X.

Workload (BASELINE.json metric, SURVEY.md section 8 config C3 at N=1):
SingleTaskGP on Hartmann6, n=4096, d=6, fp64, Standardize; qExpectedImprovement
with q=16, 512 restarts (t-batches) per GPU, 512 Sobol-QMC samples.  A "step" is
one acquisition forward over the whole batch: the kernel rows K*x^T (bo_post_kxt),
the R = K*x L^{-T} GEMM + R R^T epilogue (post_partials), then per-t-batch finalisation,
jittered q x q Cholesky, reparameterised sampling and the MC reduction
(qmc_finalize), then the cross-rank argmax (one all-reduce).  Model caches
(Cholesky, L^{-T}) are built once before timing, as the reference builds them
on the first eval-mode call.

Multi-GPU: one process per GPU (torchrun; ``--gpus N`` without torchrun's
environment starts the ranks itself).  N > 1 default (strong scaling): the 512
restarts of ONE global candidate draw are sharded over the ranks
(distributed.shard_range, north_star's "512 restarts sharded over 8 GPUs"),
and the step ends with the values gathered by one all-reduce of a zeroed
512-entry buffer (distributed.allgather_rows) and the global argmax (the
argmax/gather of optimize_acqf, botorch/optim/optimize.py:384-387).
``--weak``: each rank evaluates its own 512 restarts, no data-path
collective, one all-reduce(MAX) of the best value per step.  N = 1 is labelled
"single".  On one GPU the line also carries the projected strong-scaling
curve: the same step at b = 512/W restarts for W = 2, 4, 8 (a projection from
single-GPU timings, collectives excluded).

``--acq qnei`` times C3's qNEI instead (X_baseline = X_tr, pruned on every
rank from the same seed: replicated, not sharded) and ``--acq qehvi`` C4's
qEHVI (ModelListGP(3) on DTLZ2, n = 2048, q = 8, S = 128, 128 restarts; the
box decomposition replicated); both shard their restarts exactly as qEI does.
At N > 1 the default qEI line also carries both as ``sharded_other_acqs``.

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import subprocess
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

N_TRAIN, D, Q, RESTARTS, MC = 4096, 6, 16, 512, 512
# Fixed hyperparameters for acquisition timing (the BoTorch defaults' modes:
# lengthscale LogNormal mode 0.5016 at d=6, noise exp(-5)) -- see DESIGN.md.
LENGTHSCALE, NOISE, CONSTANT = 0.5016, 6.737947e-3, 0.0


def _dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return ws, rank, local


def flops_post_partials(B, q, n):
    """Algorithmic flops of one post_partials launch:
    triangular R = K*x L^{-T}: (B q) n^2; R R^T diagonal blocks: 2 B q^2 n;
    R beta: 2 B q n.  The kernel rows K*x (B q n (3 d + 3) flops plus one exp
    each) are built beforehand by bo_post_kxt and are not counted here."""
    return B * q * n * n + 2 * B * q * q * n + 2 * B * q * n


def post_partials_bytes(B, q, n):
    """Algorithmic HBM bytes of one post_partials launch: K*x^T read once
    (B q n doubles), the upper triangle of U = L^{-T} read once (n^2/2
    doubles), the per-strip partials written (n/128 strips x B x 16 x 16 +
    B q doubles)."""
    return 8 * (B * q * n + n * n // 2 + (n // 128) * (B * 256 + B * q))


def _pmc_rank(path):
    """Sort key of a PMC summary: its round (profiles/rNN/...), then its own
    creation stamp (tools/pmc_summary.py writes ``_meta.created``), then the
    path -- so the newest round's newest summary wins at any depth."""
    import re
    rel = os.path.relpath(path, os.path.join(ROOT, "profiles"))
    m = re.match(r"r(\d+)", rel)
    try:
        created = float(json.load(open(path)).get("_meta", {}).get("created", 0.0))
    except Exception:
        created = 0.0
    return (int(m.group(1)) if m else -1, created, rel)


def pmc_traffic(restarts, kernel="post_partials_kernel<0, 6, false, false, true, false>"):
    """HBM bytes per launch of ``kernel`` at ``restarts`` t-batches, from the
    newest committed rocprofv3 PMC summary under profiles/ at any depth
    (``BO_PMC_SUMMARY`` names one explicitly), written by tools/pmc_summary.py
    from separate --pmc FETCH_SIZE / WRITE_SIZE passes of the bench command,
    FETCH_SIZE doubled per the gfx950 correction.  A summary collected at a
    different restart count (``_meta.restarts``; 512 when absent) is scaled by
    restarts / its count and says so.  (None, None, None) if absent."""
    import glob
    env = os.environ.get("BO_PMC_SUMMARY")
    files = ([env] if env else
             glob.glob(os.path.join(ROOT, "profiles", "r*", "**", "pmc_summary.json"), recursive=True))
    if not files:
        return None, None, None
    path = max(files, key=_pmc_rank)
    summ = json.load(open(path))
    # the template argument list grows between rounds: match the named prefix
    keys = [k for k in summ if k == kernel or k.startswith(kernel.rstrip(">") + ",")]
    e = summ[keys[0]] if keys else {}
    hbm = e.get("hbm_bytes")
    at = int(summ.get("_meta", {}).get("restarts", RESTARTS))
    note = None
    if hbm is not None and at != restarts:
        hbm = hbm * restarts / at
        note = f"scaled from the PMC pass at {at} restarts to {restarts}"
    return hbm, os.path.relpath(path, ROOT), note


def mfma_f64_ceiling(dev):
    """On-box fp64 MFMA ceiling, TFLOP/s: bo_probe_mfma_f64_rate (8 independent
    v_mfma_f64_16x16x4f64 chains per wave, 2048 workgroups = 8 waves per SIMD,
    operands in registers) timed with HIP events on its launch stream."""
    import ctypes
    from botorch_amd import _lib
    out = torch.zeros(1, dtype=torch.float64, device=dev)
    st = torch.cuda.current_stream(dev)
    blocks, iters = 2048, 2000
    _lib.check(_lib.lib().bo_probe_mfma_f64_rate(blocks, 10, ctypes.c_void_p(out.data_ptr()),
                                                 ctypes.c_void_p(st.cuda_stream)), "probe")
    best = 0.0
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        _lib.check(_lib.lib().bo_probe_mfma_f64_rate(blocks, iters, ctypes.c_void_p(out.data_ptr()),
                                                     ctypes.c_void_p(st.cuda_stream)), "probe")
        e1.record(st)
        torch.cuda.synchronize(dev)
        best = max(best, blocks * 4 * iters * 8 * 2048 / (e0.elapsed_time(e1) * 1e-3) / 1e12)
    return best


def cpu_cores():
    """Host cores this process may use: the affinity mask, capped by
    OMP_NUM_THREADS (the GPU box grants a 16-core share of a larger host)."""
    try:
        n = len(os.sched_getaffinity(0))
    except Exception:
        n = os.cpu_count() or 1
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit():
        n = min(n, int(omp))
    return n


def cpu_model():
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            if line.startswith("Model name"):
                return line.split(":", 1)[1].strip()
    except Exception:
        pass
    return platform.processor()


def build_problem(device, restarts, seed_offset=0):
    from botorch_amd.test_functions import Hartmann
    from botorch_amd.utils_sampling import draw_sobol_samples
    lo = torch.zeros(D, dtype=torch.float64)
    hi = torch.ones(D, dtype=torch.float64)
    Xtr = draw_sobol_samples(torch.stack([lo, hi]), N_TRAIN, 1, seed=0).squeeze(1)
    Ytr = Hartmann(dim=6, negate=True)(Xtr).unsqueeze(-1)
    Xc = draw_sobol_samples(torch.stack([lo, hi]), restarts, Q, seed=1 + seed_offset)
    return Xtr, Ytr, Xc


def cpu_baseline(Xtr, Ytr, Xc, best_f, budget_s=20.0):
    """The reference-equivalent CPU restatement (oracle/, torch fp64 on the host
    cores) timed on a bounded sample of the same workload."""
    from oracle.acquisition import qei
    from oracle.gp import ExactGPOracle, GPHyper
    from oracle.sampling import draw_sobol_normal_samples
    torch.set_num_threads(cpu_cores())
    h = GPHyper(torch.full((D,), LENGTHSCALE, dtype=torch.float64), NOISE, CONSTANT)
    model = ExactGPOracle(Xtr, Ytr, h)
    Z = draw_sobol_normal_samples(Q, MC, 0)
    b = 64
    Xs = Xc[:b]
    qei(model, Xs, Z, best_f)  # warm-up
    times = []
    t_start = time.perf_counter()
    while len(times) < 5 or (time.perf_counter() - t_start < budget_s and len(times) < 50):
        t0 = time.perf_counter()
        qei(model, Xs, Z, best_f)
        times.append(time.perf_counter() - t0)
        if time.perf_counter() - t_start > budget_s and len(times) >= 2:
            break
    times.sort()
    med = times[len(times) // 2]
    return {
        "value": b * Q * MC / med,
        "unit": "acq-evals/s",
        "cores": torch.get_num_threads(),
        "kind": "port",
        "sample": f"qEI forward, {b} of the {RESTARTS} restarts (q={Q}, S={MC}, n={N_TRAIN}, "
                  f"fp64), median of {len(times)} runs; torch fp64 CPU restatement (oracle/), "
                  f"{cpu_model()}",
    }


def _gpu_time(fn, steps=5, warmup=2, reps=3):
    """Seconds per call of ``fn``: HIP events on torch's current stream (the
    stream every op here launches on) around ``steps`` back-to-back calls,
    after ``warmup`` untimed calls; the median of ``reps`` such runs.  A call
    that waits on the host in between still shows as idle device time between
    the events, so host-bound calls are timed as they run."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(steps):
            fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e-3 / steps)
    ts.sort()
    return ts[len(ts) // 2]


def _cpu_time(fn, budget_s=4.0, max_runs=5):
    fn()
    times = []
    t_start = time.perf_counter()
    while len(times) < max_runs and (len(times) < 2 or time.perf_counter() - t_start < budget_s):
        t0 = time.perf_counter()
        fn()
        times.append(time.perf_counter() - t0)
    times.sort()
    return times[len(times) // 2], len(times)


def _check_qnehvi(acqf, Xd, X, Y, models, ref_point, S, k=4):
    """Outside the timed region: the timed qNEHVI forward (and dX) at k spread
    t-batches against the CPU restatement (oracle.QNEHVIOracle, the checker) on
    the same pruned baseline and per-sample cells -- values by the per-sample
    cell inclusion-exclusion (rtol 1e-7) and by exact hypervolume differences
    on two of them (north_star's 1e-2), dX by autograd through the oracle
    (rtol 1e-5).  Where the timed Sobol t-batches improve on too few samples,
    t-batches scattered around the Pareto set are checked as well."""
    from oracle.acquisition import QNEHVIOracle
    from oracle.gp import ExactGPOracle, GPHyper
    f64 = torch.float64
    orcs = [ExactGPOracle(X, Y[:, t:t + 1], GPHyper(torch.full((6,), 0.6, dtype=f64), 1e-3, 0.0))
            for t in range(Y.shape[-1])]
    orc = QNEHVIOracle(orcs, acqf.X_baseline.cpu(), ref_point.tolist(), S, seed=0)
    base_err = float((acqf.baseline_samples - orc.Y_base).abs().max())
    lo, hi = acqf.cell_lower_bounds.cpu(), acqf.cell_upper_bounds.cpu()
    g = torch.Generator().manual_seed(4)
    from botorch_amd.multi_objective import is_non_dominated
    P = X[is_non_dominated(Y)]
    b, q = Xd.shape[0], Xd.shape[1]
    pick = torch.randint(0, P.shape[0], (b, q), generator=g)
    Xn = (P[pick] + 0.05 * torch.randn(b, q, X.shape[-1], generator=g, dtype=f64)).clamp(0, 1)
    res = {"baseline_samples_max_abs_err": base_err, "rtol_cells": 1e-7, "rtol_exact": 1e-2,
           "rtol_grad": 1e-5}
    worst_v, worst_g, worst_x, checked = 0.0, 0.0, 0.0, []
    for tag, Xs in (("timed", Xd.detach().cpu()), ("near_pareto", Xn)):
        Xg = Xs.to(Xd.device).requires_grad_(True)
        v = acqf(Xg)
        (gd,) = torch.autograd.grad(v.sum(), Xg)
        v, gd = v.detach().cpu(), gd.cpu()
        nz = (v != 0).nonzero().flatten()
        res[f"{tag}_nonzero"] = int(nz.numel())
        if nz.numel() < k:
            continue
        idx = nz[torch.linspace(0, nz.numel() - 1, k).round().long()]
        for i in idx.tolist():
            Xo = Xs[i:i + 1].clone().requires_grad_(True)
            rv = orc.value_cells(Xo, lo, hi)
            (go,) = torch.autograd.grad(rv.sum(), Xo)
            worst_v = max(worst_v, float(((v[i] - rv.detach()[0]).abs() / rv.detach().abs()[0])))
            worst_g = max(worst_g, float(((gd[i] - go[0]).abs() / go[0].abs().clamp_min(1e-8)).max()))
            ok = torch.allclose(v[i:i + 1], rv.detach(), rtol=1e-7, atol=1e-10) and \
                torch.allclose(gd[i:i + 1], go, rtol=1e-5, atol=1e-8)
            if not ok:
                raise SystemExit(f"bench: C4 qNEHVI disagrees with the oracle at t-batch {i} ({tag})")
        ex = orc.value_exact(Xs[idx[:2]])
        worst_x = max(worst_x, float(((v[idx[:2]] - ex).abs() / ex.abs()).max()))
        if not torch.allclose(v[idx[:2]], ex, rtol=1e-2, atol=1e-6):
            raise SystemExit(f"bench: C4 qNEHVI disagrees with the exact hypervolumes ({tag})")
        checked += [f"{tag}:{i}" for i in idx.tolist()]
    if not checked:
        raise SystemExit("bench: C4 qNEHVI check degenerate (no non-zero values)")
    res.update(t_batches=checked, max_rel_err_cells=worst_v, max_rel_err_grad=worst_g,
               max_rel_err_exact_hv=worst_x)
    return res


def other_configs(dev, cpu=True):
    """The other SURVEY.md section 8 configurations, forward-only acq-evals/s on
    this GPU beside the torch-fp64 CPU restatement (oracle/) on a bounded sample
    of the same workload (C2 qEI, C3 qNEI with pruned baseline, C4 qEHVI over a
    ModelListGP on DTLZ2, C5 SAAS qEI at d = 50)."""
    from botorch_amd.acquisition import (qExpectedHypervolumeImprovement, qExpectedImprovement,
                                         qNoisyExpectedImprovement)
    from botorch_amd.models import (ModelListGP, SaasFullyBayesianSingleTaskGP, SingleTaskGP,
                                    sample_saas_prior)
    from botorch_amd.multi_objective import FastNondominatedPartitioning
    from botorch_amd.sampling import SobolQMCNormalSampler
    from botorch_amd.test_functions import DTLZ2, Hartmann
    from botorch_amd.utils_sampling import draw_sobol_samples
    from oracle import acquisition as oacq
    from oracle.gp import MATERN52, ExactGPOracle, GPHyper
    from oracle.sampling import base_samples_multi_output, base_samples_single_output
    torch.set_num_threads(cpu_cores())
    out = {}
    f64 = torch.float64

    def unit(d):
        return torch.stack([torch.zeros(d, dtype=f64), torch.ones(d, dtype=f64)])

    def stgp(X, Y, ls, noise, kind_matern=False):
        m = SingleTaskGP(X.to(dev), Y.to(dev))
        m.covar_module.lengthscale = torch.full((1, X.shape[-1]), ls, dtype=f64)
        m.likelihood.noise = torch.tensor([noise], dtype=f64)
        return m.eval()

    # C2: qEI n=1024 d=6 q=8 S=256 b=64
    n, q, S, b = 1024, 8, 256, 64
    X = draw_sobol_samples(unit(6), n, 1, seed=0).squeeze(1)
    Y = Hartmann(negate=True)(X).unsqueeze(-1)
    Xc = draw_sobol_samples(unit(6), b, q, seed=1)
    m = stgp(X, Y, LENGTHSCALE, NOISE)
    m_c2, bf_c2 = m, float(Y.max()) - 0.3
    acqf = qExpectedImprovement(m, float(Y.max()), sampler=SobolQMCNormalSampler(torch.Size([S]), seed=0))
    Xd = Xc.to(dev)
    # a call is ~0.07 ms: 200 back-to-back calls give the steady per-call rate
    # (20 of them were dominated by the first call's latency)
    with torch.no_grad():
        t = _gpu_time(lambda: acqf(Xd), steps=200, warmup=20)
    e = {"config": "C2 qEI n=1024 d=6 q=8 S=256 b=64", "gpu_evals_per_s": q * S * b / t,
         "gpu_ms": 1e3 * t, "calls_timed": 200}
    # the same forward (and forward + backward) captured once as a HIP graph and
    # replayed (botorch_amd.graphs; values bit-equal to the eager call)
    from botorch_amd.graphs import GraphedAcquisition
    ga = GraphedAcquisition(acqf, Xd, share_input=True)
    tg = _gpu_time(lambda: ga(Xd), steps=200, warmup=20)
    Xg = Xd.clone().requires_grad_(True)

    def c2_fb():
        v = acqf(Xg)
        torch.autograd.grad(v.sum(), Xg)

    tfb = _gpu_time(c2_fb, steps=20, warmup=3)
    gab = GraphedAcquisition(acqf, Xd, with_grad=True, share_input=True)
    tgb = _gpu_time(lambda: gab(Xd), steps=50, warmup=5)
    e.update(graphed_ms=1e3 * tg, graphed_evals_per_s=q * S * b / tg, fwd_bwd_ms=1e3 * tfb,
             graphed_fwd_bwd_ms=1e3 * tgb)
    if cpu:
        orc = ExactGPOracle(X, Y, GPHyper(torch.full((6,), LENGTHSCALE, dtype=f64), NOISE, 0.0))
        Z = base_samples_single_output(S, q, 0)
        tc, runs = _cpu_time(lambda: oacq.qei(orc, Xc, Z, float(Y.max())))
        e.update(cpu_evals_per_s=q * S * b / tc, cpu_sample=f"all {b} restarts, median of {runs}")
    out["C2"] = e

    # C3 qNEI: n=4096 d=6 q=16 S=512 b=512, X_baseline = X_tr pruned (2048 samples)
    n, q, S, b = N_TRAIN, Q, MC, RESTARTS
    X = draw_sobol_samples(unit(6), n, 1, seed=0).squeeze(1)
    Y = Hartmann(negate=True)(X).unsqueeze(-1)
    Xc = draw_sobol_samples(unit(6), b, q, seed=1)
    m = stgp(X, Y, LENGTHSCALE, NOISE)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    acqf = qNoisyExpectedImprovement(m, X.to(dev), sampler=SobolQMCNormalSampler(torch.Size([S]), seed=0),
                                     prune_baseline=True)
    torch.cuda.synchronize()
    init_ms = 1e3 * (time.perf_counter() - t0)
    r = int(acqf.X_baseline.shape[0])
    Xd = Xc.to(dev)
    with torch.no_grad():
        t = _gpu_time(lambda: acqf(Xd), steps=10, warmup=2)
    e = {"config": "C3 qNEI n=4096 d=6 q=16 S=512 b=512, pruned baseline (cache_root)",
         "r": r, "init_ms": init_ms, "gpu_evals_per_s": q * S * b / t, "gpu_ms": 1e3 * t}
    if cpu:
        orc = ExactGPOracle(X, Y, GPHyper(torch.full((6,), LENGTHSCALE, dtype=f64), NOISE, 0.0))
        Xb = acqf.X_baseline.cpu()
        ref = oacq.QNEIOracle(orc, Xb, S, seed=0)
        bs = 8
        tc, runs = _cpu_time(lambda: ref(Xc[:bs]))
        e.update(cpu_evals_per_s=q * S * bs / tc,
                 cpu_sample=f"{bs} of {b} restarts (full (r+q) posterior as the reference), median of {runs}")
    out["C3_qNEI"] = e

    # The same qNEI on a rougher model (lengthscale 0.15, noise 0.5): pruning
    # keeps r = 31 baseline points, so the cached-root cross term
    # T = L_rr^-1 Sigma'(X_b, X) carries 31 rows through the fused pass
    # (tests/test_gpu_full_configs.py pins this setting against the oracle).
    m31 = stgp(X, Y, 0.15, 0.5)
    torch.manual_seed(7)  # the pruning's sample draw (the test's seed)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    acqf31 = qNoisyExpectedImprovement(m31, X.to(dev), sampler=SobolQMCNormalSampler(torch.Size([S]), seed=0),
                                       prune_baseline=True)
    torch.cuda.synchronize()
    init31 = 1e3 * (time.perf_counter() - t0)
    with torch.no_grad():
        t = _gpu_time(lambda: acqf31(Xd), steps=10, warmup=2)
        v31 = acqf31(Xd)
    e = {"config": "C3 qNEI n=4096 d=6 q=16 S=512 b=512, lengthscale 0.15 noise 0.5, pruned baseline "
                   "(cache_root)", "r": int(acqf31.X_baseline.shape[0]), "init_ms": init31,
         "gpu_evals_per_s": q * S * b / t, "gpu_ms": 1e3 * t,
         "nonzero_values": int((v31 > 0).sum())}
    if cpu:
        orc31 = ExactGPOracle(X, Y, GPHyper(torch.full((6,), 0.15, dtype=f64), 0.5, 0.0))
        ref = oacq.QNEIOracle(orc31, acqf31.X_baseline.cpu(), S, seed=0)
        bs = 8
        vref = ref(Xc[:bs])
        e["check_max_abs_err"] = float((v31[:bs].cpu() - vref).abs().max())
        tc, runs = _cpu_time(lambda: ref(Xc[:bs]))
        e.update(cpu_evals_per_s=q * S * bs / tc,
                 cpu_sample=f"{bs} of {b} restarts (full (r+q) posterior as the reference), median of {runs}")
    out["C3_qNEI_r31"] = e

    # C3 with the section 8(f) rank-1 reductions: qLogEI (best_f = max Y) and
    # qLogNEI on the same pruned baseline, fat=True / default temperatures.
    from botorch_amd.acquisition import qLogExpectedImprovement, qLogNoisyExpectedImprovement
    best = float(Y.max())
    acqf = qLogExpectedImprovement(m, best, sampler=SobolQMCNormalSampler(torch.Size([S]), seed=0))
    with torch.no_grad():
        t = _gpu_time(lambda: acqf(Xd), steps=10, warmup=2)
    Xg = Xd.clone().requires_grad_(True)

    def fb():
        (gx,) = torch.autograd.grad(acqf(Xg).sum(), Xg)
        return gx

    tfb = _gpu_time(fb, steps=5, warmup=1)
    e = {"config": "C3 qLogEI n=4096 d=6 q=16 S=512 b=512 (fat, tau_relu=1e-6, tau_max=1e-2)",
         "gpu_evals_per_s": q * S * b / t, "gpu_ms": 1e3 * t,
         "fwd_bwd_evals_per_s": q * S * b / tfb, "fwd_bwd_ms": 1e3 * tfb}
    if cpu:
        orc = ExactGPOracle(X, Y, GPHyper(torch.full((6,), LENGTHSCALE, dtype=f64), NOISE, 0.0))
        Z = base_samples_single_output(S, q, 0)
        bs = 64
        tc, runs = _cpu_time(lambda: oacq.qlogei(orc, Xc[:bs], Z, best))
        e.update(cpu_evals_per_s=q * S * bs / tc, cpu_sample=f"{bs} of {b} restarts, median of {runs}")
    out["C3_qLogEI"] = e

    # Section 8(f) rank 2: raw-sample initialisation of optimize_acqf at C3 scale
    # (2048 raw q=16 designs, 512 restarts, init_batch_limit 512): on-device
    # Sobol designs + chunked forward + Boltzmann selection, against the
    # reference's protocol (host Sobol draw, per-chunk .cpu(), host selection).
    from botorch_amd.optim import (gen_batch_initial_conditions, initialize_q_batch_nonneg)
    from botorch_amd.utils_sampling import draw_sobol_samples as host_sobol
    acq_ei = qExpectedImprovement(m, best - 0.3, sampler=SobolQMCNormalSampler(torch.Size([S]), seed=0))
    bounds_d = unit(6).to(dev)
    raw = 2048
    opts = {"seed": 0, "init_batch_limit": 512}
    t_dev = _gpu_time(lambda: gen_batch_initial_conditions(acq_ei, bounds_d, q, b, raw, options=opts),
                      steps=5, warmup=1)

    def host_protocol():
        Xr = host_sobol(unit(6), raw, q, seed=0)
        with torch.no_grad():
            Yr = torch.cat([acq_ei(Xr[i:i + 512].to(dev)).cpu() for i in range(0, raw, 512)])
        return initialize_q_batch_nonneg(Xr, Yr, b).to(dev)

    t_host = _gpu_time(host_protocol, steps=5, warmup=1)
    # the reference default (no init_batch_limit): all 2048 raw designs in one
    # forward launch
    t_one = _gpu_time(lambda: gen_batch_initial_conditions(acq_ei, bounds_d, q, b, raw,
                                                           options={"seed": 0}), steps=5, warmup=1)
    out["C3_init"] = {"config": "C3 gen_batch_initial_conditions: qEI, 2048 raw x q=16, 512 restarts, "
                                "S=512, init_batch_limit=512 (and unlimited: one launch)",
                      "device_ms": 1e3 * t_dev, "host_roundtrip_ms": 1e3 * t_host,
                      "device_one_launch_ms": 1e3 * t_one,
                      "raw_evals_per_s": raw * q * S / min(t_dev, t_one)}
    acqf = qLogNoisyExpectedImprovement(m, X.to(dev), sampler=SobolQMCNormalSampler(torch.Size([S]), seed=0),
                                        prune_baseline=True)
    with torch.no_grad():
        t = _gpu_time(lambda: acqf(Xd), steps=10, warmup=2)
    e = {"config": "C3 qLogNEI n=4096 d=6 q=16 S=512 b=512, pruned baseline (cache_root)",
         "r": int(acqf.X_baseline.shape[0]), "gpu_evals_per_s": q * S * b / t, "gpu_ms": 1e3 * t}
    if cpu:
        ref = oacq.QNEIOracle(orc, acqf.X_baseline.cpu(), S, seed=0)
        bs = 8
        tc, runs = _cpu_time(lambda: oacq.qlognei(ref, Xc[:bs]))
        e.update(cpu_evals_per_s=q * S * bs / tc, cpu_sample=f"{bs} of {b} restarts, median of {runs}")
    out["C3_qLogNEI"] = e

    # Section 8(f) rank 3: optimize_acqf end to end (raw-sample init + candidate
    # generation) with the reference's host scipy L-BFGS-B loop vs the
    # device-resident multi-start L-BFGS (gen_candidates_device), C2 and C3 models.
    from botorch_amd.optim import gen_candidates_device, gen_candidates_scipy, optimize_acqf
    for tag, (mm, bfv, qq, SS, bb, raw_n) in {
            "C2": (m_c2, bf_c2, 8, 256, 64, 512),
            "C3": (m, best - 0.3, Q, MC, 128, 1024)}.items():
        acq_o = qExpectedImprovement(mm, bfv, sampler=SobolQMCNormalSampler(torch.Size([SS]), seed=0))
        bnd = unit(6).to(dev)
        res = {}
        for gname, gen, extra in (("scipy", gen_candidates_scipy, {}),
                                  ("device_joint", gen_candidates_device,
                                   {"algorithm": "lbfgsb", "joint": True}),
                                  ("device", gen_candidates_device, {"algorithm": "lbfgsb"}),
                                  ("device_no_compaction", gen_candidates_device,
                                   {"algorithm": "lbfgsb", "compact": False}),
                                  ("device_projected", gen_candidates_device,
                                   {"algorithm": "projected"})):
            opts = {"seed": 0, "maxiter": 100, **extra}
            optimize_acqf(acq_o, bnd, qq, bb, raw_n, options=opts, gen_candidates=gen)  # warm-up
            torch.cuda.synchronize()
            # the median of a few runs: one run after the warm-up swings by
            # 1.5x (C2 device_joint 12.2 ms median, 17.6 ms first; scipy 113
            # ms once in 7 -- tools/time_c2_joint.py)
            runs = []
            for _ in range(5 if tag == "C2" else 3):
                t0 = time.perf_counter()
                cand, val = optimize_acqf(acq_o, bnd, qq, bb, raw_n, options=opts, gen_candidates=gen)
                torch.cuda.synchronize()
                runs.append(1e3 * (time.perf_counter() - t0))
            res[gname] = {"ms": sorted(runs)[len(runs) // 2], "ms_runs": [round(r, 2) for r in runs],
                          "best_acq": float(val)}
            if gen is gen_candidates_device:
                res[gname]["evals"] = int(gen_candidates_device.last_evals)
                if extra["algorithm"] == "lbfgsb" and not extra.get("joint"):
                    res[gname]["shrinks"] = list(gen_candidates_device.last_shrinks)
                    stl = gen_candidates_device.last_state
                    res[gname]["max_nit"] = int(stl.nit.max())
                    u, cnt = torch.unique(stl.status.cpu(), return_counts=True)
                    res[gname]["status_counts"] = {str(int(k)): int(v) for k, v in zip(u, cnt)}
        # like with like: "device_joint" runs the reference's problem (one
        # L-BFGS-B over all restarts, gen.py:252-267), as scipy does here;
        # "device" (one L-BFGS-B per restart) is a different algorithm
        out[f"{tag}_optimize_acqf"] = {
            "config": f"{tag} optimize_acqf qEI q={qq} S={SS} restarts={bb} raw={raw_n} maxiter=100",
            **res, "speedup": res["scipy"]["ms"] / res["device_joint"]["ms"],
            "speedup_note": "scipy vs device_joint: the same joint L-BFGS-B problem",
            "speedup_per_restart_algorithm": res["scipy"]["ms"] / res["device"]["ms"]}

    # C4: qEHVI, ModelListGP of 3 on DTLZ2 (n=2048, d=6), q=8, S=128, b=128
    n, q, S, b, mo = 2048, 8, 128, 128, 3
    g = torch.Generator().manual_seed(0)
    X = torch.rand(n, 6, generator=g, dtype=f64)
    Y = DTLZ2(dim=6, num_objectives=mo, negate=True).evaluate_true(X)
    Y = -Y
    models = [stgp(X, Y[:, t:t + 1], 0.6, 1e-3) for t in range(mo)]
    ref_point = torch.full((mo,), -1.1, dtype=f64)
    part = FastNondominatedPartitioning(ref_point, Y)
    acqf = qExpectedHypervolumeImprovement(ModelListGP(*models), ref_point.tolist(), part,
                                           sampler=SobolQMCNormalSampler(torch.Size([S]), seed=0))
    Xc = draw_sobol_samples(unit(6), b, q, seed=1)
    Xd = Xc.to(dev)
    with torch.no_grad():
        t = _gpu_time(lambda: acqf(Xd), steps=20, warmup=3)
    lo, hi = part.get_hypercell_bounds()
    e = {"config": "C4 qEHVI ModelListGP(3) DTLZ2 n=2048 d=6 q=8 S=128 b=128",
         "cells": int(lo.shape[0]), "gpu_evals_per_s": q * S * b / t, "gpu_ms": 1e3 * t}
    if cpu:
        orcs = [ExactGPOracle(X, Y[:, t:t + 1], GPHyper(torch.full((6,), 0.6, dtype=f64), 1e-3, 0.0))
                for t in range(mo)]
        Zm = base_samples_multi_output(S, q, mo, 0)
        bs = 2
        tc, runs = _cpu_time(lambda: oacq.qehvi(orcs, Xc[:bs], Zm, lo, hi), budget_s=6.0, max_runs=3)
        e.update(cpu_evals_per_s=q * S * bs / tc, cpu_sample=f"{bs} of {b} restarts, median of {runs}")
    out["C4_qEHVI"] = e

    # Section 8(f) rank 4: qNEHVI on the C4 models, X_baseline = the 2048
    # training inputs pruned (prune_baseline=True), S=128 per-sample box
    # decompositions (host, as the reference for m > 2), cached baseline roots.
    from botorch_amd.acquisition import qNoisyExpectedHypervolumeImprovement
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    acqf = qNoisyExpectedHypervolumeImprovement(ModelListGP(*models), ref_point.tolist(), X.to(dev),
                                                sampler=SobolQMCNormalSampler(torch.Size([S]), seed=0),
                                                prune_baseline=True)
    torch.cuda.synchronize()
    init_ms = 1e3 * (time.perf_counter() - t0)
    with torch.no_grad():
        t = _gpu_time(lambda: acqf(Xd), steps=20, warmup=3)
    Xg = Xd.clone().requires_grad_(True)

    def fb_nehvi():
        (gx,) = torch.autograd.grad(acqf(Xg).sum(), Xg)
        return gx

    tfb = _gpu_time(fb_nehvi, steps=10, warmup=2)
    out["C4_qNEHVI"] = {"config": "C4 qNEHVI ModelListGP(3) DTLZ2 n=2048 d=6 q=8 S=128 b=128, pruned baseline",
                        "r": int(acqf.X_baseline.shape[0]),
                        "cells_per_sample_max": int(acqf.cell_lower_bounds.shape[1]),
                        "init_ms": init_ms, "gpu_evals_per_s": q * S * b / t, "gpu_ms": 1e3 * t,
                        "fwd_bwd_ms": 1e3 * tfb}
    if cpu:
        out["C4_qNEHVI"]["check"] = _check_qnehvi(acqf, Xd, X, Y, models, ref_point, S)

    # C5: SAAS (M=16 prior draws), d=50, n=256, qEI q=4, S=256, b=64
    d, n, M, q, S, b = 50, 256, 16, 4, 256, 64
    X = draw_sobol_samples(unit(d), n, 1, seed=0).squeeze(1)
    Y = Hartmann(negate=True)(X[:, :6]).unsqueeze(-1)
    Y = (Y - Y.mean()) / Y.std()
    smp = sample_saas_prior(d, M, seed=0)
    m = SaasFullyBayesianSingleTaskGP(X.to(dev), Y.to(dev))
    m.load_mcmc_samples({k: v.to(dev) for k, v in smp.items()})
    m.eval()
    acqf = qExpectedImprovement(m, float(Y.max()), sampler=SobolQMCNormalSampler(torch.Size([S]), seed=0))
    Xc = draw_sobol_samples(unit(d), b, q, seed=1)
    Xd = Xc.to(dev)
    with torch.no_grad():
        t = _gpu_time(lambda: acqf(Xd), steps=10, warmup=2)
    e = {"config": "C5 SAAS (16 prior draws) d=50 n=256 qEI q=4 S=256 b=64",
         "gpu_evals_per_s": q * S * b * M / t, "gpu_ms": 1e3 * t,
         "note": "evals counted per MCMC member (q x b x S x M)"}
    if cpu:
        members = oacq.saas_members(X, Y, smp)
        Z = base_samples_single_output(S, q, 0)
        bs = 16
        tc, runs = _cpu_time(lambda: oacq.saas_qei(members, Xc[:bs], Z, float(Y.max())))
        e.update(cpu_evals_per_s=q * S * bs * M / tc, cpu_sample=f"{bs} of {b} restarts, median of {runs}")
    out["C5_SAAS"] = e
    for v in out.values():
        if "cpu_evals_per_s" in v:
            v["speedup"] = v["gpu_evals_per_s"] / v["cpu_evals_per_s"]
    return out


def time_cholesky(Xtr, dev, reps=10, shapes=((3, 2048), (4, 4096), (8, 4096)), ainv=True):
    """Standalone n x n Cholesky + triangular inverse (bo_cholesky_inverse, the
    persistent task DAG) on the C3 kernel matrix ("standalone
    n x n Cholesky ms and MFMA %"): HIP events on the launch stream around the
    launch alone (the input copy excluded), median of ``reps``; flops n^3/3
    (factor) + n^3/3 (inverse); then the batched ``shapes`` (nb, n)."""
    import ctypes
    from botorch_amd import kernels
    from botorch_amd._lib import check, lib
    X = Xtr.to(dev) / LENGTHSCALE
    n = X.shape[0]
    # the RBF kernel matrix of the C3 training set (plain torch input preparation)
    A0 = torch.exp(-0.5 * torch.cdist(X, X) ** 2) + NOISE * torch.eye(n, dtype=torch.float64, device=dev)
    np_ = kernels.padded_order(n)
    base = torch.eye(np_, dtype=torch.float64, device=dev)
    base[:n, :n] = torch.tril(A0)
    W = torch.empty_like(base)
    Linv = torch.empty_like(base)
    work = torch.empty_like(base)
    info = torch.zeros(1, dtype=torch.int32, device=dev)
    st = torch.cuda.current_stream(dev)
    ts = []
    for r in range(reps + 2):
        W.copy_(base)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        check(lib().bo_cholesky_inverse(kernels._p(W), kernels._p(Linv), kernels._p(work), np_,
                                        kernels._p(info), ctypes.c_void_p(st.cuda_stream)), "chol")
        e1.record(st)
        torch.cuda.synchronize(dev)
        if r >= 2:
            ts.append(e0.elapsed_time(e1))
    if int(info.item()) != 0:
        raise RuntimeError(f"bench Cholesky: info {int(info.item())}")
    ts.sort()
    ms = ts[len(ts) // 2]
    fl = 2.0 * n ** 3 / 3.0
    out = {"n": n, "ms": ms, "flops": fl, "tflops": fl / (ms * 1e-3) / 1e12,
           "frac_of_spec": fl / (ms * 1e-3) / 1e12 / 78.6,
           "note": "factor + inverse, one persistent task-DAG launch, input in HBM"}
    if not ainv and not shapes:  # the single launch alone (tools/chol_only.py single)
        return out
    # the MLL closure's launch: factor + inverse + A^{-1} = L^{-T} L^{-1} (n^3/3
    # more) in one DAG (bo_cholesky_inverse_ainv), against the two launches
    # (DAG, then bo_ainv) it replaces
    T = np_ // 64
    work5 = torch.empty((16 + 5 * T * T + 1) // 2, dtype=torch.float64, device=dev)
    Ai = torch.empty_like(base)
    wk = ctypes.c_int64()
    check(lib().bo_ainv_work(n, ctypes.byref(wk)), "ainv_work")
    wa = torch.empty(max(1, wk.value), dtype=torch.float64, device=dev)
    t_fold, t_two = [], []
    for r in range(reps + 2):
        for fold, acc in ((True, t_fold), (False, t_two)):
            W.copy_(base)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            if fold:
                check(lib().bo_cholesky_inverse_ainv(kernels._p(W), kernels._p(Linv), kernels._p(Ai),
                                                     kernels._p(work5), np_, kernels._p(info),
                                                     ctypes.c_void_p(st.cuda_stream)), "chol_ainv")
            else:
                check(lib().bo_cholesky_inverse(kernels._p(W), kernels._p(Linv), kernels._p(work),
                                                np_, kernels._p(info), ctypes.c_void_p(st.cuda_stream)),
                      "chol")
                check(lib().bo_ainv(kernels._p(Linv), np_, n, kernels._p(Ai), kernels._p(wa),
                                    ctypes.c_void_p(st.cuda_stream)), "ainv")
            e1.record(st)
            torch.cuda.synchronize(dev)
            if r >= 2:
                acc.append(e0.elapsed_time(e1))
    t_fold.sort()
    t_two.sort()
    fl3 = fl + n ** 3 / 3.0
    out["with_ainv"] = {"ms_one_launch": t_fold[len(t_fold) // 2],
                        "ms_two_launches": t_two[len(t_two) // 2],
                        "flops": fl3,
                        "frac_of_spec_one_launch": fl3 / (t_fold[len(t_fold) // 2] * 1e-3) / 1e12 / 78.6,
                        "note": "factor + inverse + A^-1 (the MLL closure's), one DAG launch vs "
                                "the DAG then bo_ainv"}
    # batched: nb independent factor + inverse problems in one launch
    # (bo_cholesky_inverse_batched), the shapes of the path's multi-model fits
    # and caches: C4's ModelListGP(3) at n = 2048, multi-output models at C3's n
    batched = []
    for nb, nn in shapes:
        npb = kernels.padded_order(nn)
        Bb = torch.eye(npb, dtype=torch.float64, device=dev).repeat(nb, 1, 1)
        for m in range(nb):  # the C3 kernel matrix scaled per member (distinct SPD inputs)
            Bb[m, :nn, :nn] = torch.tril(A0[:nn, :nn]) * (1.0 + 0.1 * m)
        Wb, Lb = torch.empty_like(Bb), torch.empty_like(Bb)
        T = npb // 64
        wk = torch.empty((16 + 4 * nb * T * T + 3) // 4 * 2, dtype=torch.float64, device=dev)
        ib = torch.zeros(nb, dtype=torch.int32, device=dev)
        tb = []
        for r in range(reps + 2):
            Wb.copy_(Bb)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            check(lib().bo_cholesky_inverse_batched(kernels._p(Wb), kernels._p(Lb), kernels._p(wk),
                                                    nb, npb, kernels._p(ib),
                                                    ctypes.c_void_p(st.cuda_stream)), "chol_b")
            e1.record(st)
            torch.cuda.synchronize(dev)
            if r >= 2:
                tb.append(e0.elapsed_time(e1))
        if any(int(v) != 0 for v in ib.tolist()):
            raise RuntimeError(f"bench batched Cholesky: info {ib.tolist()}")
        tb.sort()
        msb = tb[len(tb) // 2]
        flb = nb * 2.0 * nn ** 3 / 3.0
        batched.append({"nb": nb, "n": nn, "ms": msb, "tflops": flb / (msb * 1e-3) / 1e12,
                        "frac_of_spec": flb / (msb * 1e-3) / 1e12 / 78.6})
        del Bb, Wb, Lb
    out["batched"] = batched
    return out


def time_gp_fit(Xtr, Ytr, dev, cpu=True):
    """GP-fit half of the metric: fit_gpytorch_mll (L-BFGS-B, exact MLL + gradient on
    the device) from BoTorch's default initialisation, n=4096, d=6.  CPU side: one
    closure (exact MLL + autograd gradient, torch fp64 restatement) on the host."""
    from botorch_amd import fit as fitmod
    from botorch_amd.models import SingleTaskGP
    model = SingleTaskGP(Xtr.to(dev), Ytr.to(dev))
    mll = fitmod.ExactMarginalLogLikelihood(model.likelihood, model)
    calls = [0]
    orig = fitmod.mll_value_and_grad

    def counted(*a, **k):
        calls[0] += 1
        return orig(*a, **k)

    # warm-up: one MLL closure on a throw-away copy of the model, untimed.  The
    # first closure in a process pays one-time costs (lazy code-object loads of
    # the closure's kernels, the n = 4096 task table): measured 507-517 ms for
    # the first fit of a process against 390-394 ms for every later one, or for
    # the first after one closure (tools/fit_breakdown.py)
    warm = SingleTaskGP(Xtr.to(dev), Ytr.to(dev))
    lay = fitmod._layout(warm)
    fitmod.mll_value_and_grad(warm, lay.get(), lay, sync_model=False)
    del warm, lay
    fitmod.mll_value_and_grad = counted
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    fitmod.fit_gpytorch_mll(mll)
    torch.cuda.synchronize(dev)
    ms = 1e3 * (time.perf_counter() - t0)
    fitmod.mll_value_and_grad = orig
    out = {"ms": ms, "closures": calls[0], "ms_per_closure": ms / max(1, calls[0]),
           "n": int(Xtr.shape[0]), "lengthscale": model.covar_module.lengthscale.detach().reshape(-1).tolist(),
           "noise": float(model.likelihood.noise.detach())}
    if cpu:
        from oracle.gp import neg_mll, standardize_fit
        torch.set_num_threads(cpu_cores())
        mu, sd = standardize_fit(Ytr)
        y = ((Ytr - mu) / sd).squeeze(-1)
        times = []
        for _ in range(3):
            ls = torch.full((D,), 0.5016, dtype=torch.float64, requires_grad=True)
            nz = torch.tensor(6.7e-3, dtype=torch.float64, requires_grad=True)
            c = torch.tensor(0.0, dtype=torch.float64, requires_grad=True)
            t0 = time.perf_counter()
            neg_mll(Xtr, y, ls, nz, c).backward()
            times.append(time.perf_counter() - t0)
        out["cpu_ms_per_closure"] = 1e3 * sorted(times)[1]
        out["cpu_cores"] = torch.get_num_threads()
        out["cpu_fit_ms_estimate"] = out["cpu_ms_per_closure"] * calls[0]
    return out


def _launch_ranks(n: int) -> int:
    """``--gpus N`` without torchrun's environment: start the N ranks (one
    process per GPU) under torch.distributed.run as a CHILD process -- this
    process has not touched the GPU -- and return its exit code."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.call(cmd)


def timed_steps(step, steps, warmup, dist, sync, dev=None):
    """W untimed steps, then exactly K timed steps bracketed by a barrier +
    device sync on both sides; the MAX over ranks of the elapsed time (one
    all-reduce on ``dev``, the device the process group reduces on)."""
    for _ in range(warmup):
        step()
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if dist is not None:
        dist.barrier()
    sync()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def rehearse_cpu(args, ws, rank):
    """BO_BENCH_REHEARSE=cpu: the multi-rank launch, the restart split, the
    collectives and rank 0's report over gloo on the CPU, with a stub in place
    of the acquisition forward (no GPU, no kernels: it measures nothing, the
    line says so).  Exercised by tests/test_bench_launch_cpu.py."""
    import torch.distributed as tdist
    from botorch_amd.distributed import allgather_rows, shard_range
    dist = None
    if ws > 1:
        tdist.init_process_group("gloo")
        dist = tdist
    strong = ws > 1 and not args.weak
    r0, r1 = shard_range(RESTARTS, ws, rank) if strong else (0, RESTARTS)
    best = torch.empty(1, dtype=torch.float64)

    def step():
        acq = torch.zeros(r1 - r0, dtype=torch.float64)   # stub of acqf(X[r0:r1])
        if strong:
            torch.amax(allgather_rows(acq, RESTARTS), dim=0, keepdim=True, out=best)
        else:
            torch.amax(acq, dim=0, keepdim=True, out=best)
            if dist is not None:
                dist.all_reduce(best, op=dist.ReduceOp.MAX)

    elapsed = timed_steps(step, args.steps, args.warmup, dist, lambda: None)
    if dist is not None:
        assert dist.get_world_size() == args.gpus
    if rank == 0:
        print(json.dumps({"metric": "acq-evals/sec (q x restarts x MC), qEI forward",
                          "value": None, "unit": "acq-evals/s", "n_gpus": ws,
                          "steps": args.steps, "warmup": args.warmup,
                          "ms_per_step": 1e3 * elapsed / args.steps,
                          "scaling": "single" if ws == 1 else ("strong" if strong else "weak"),
                          "rehearsal": "cpu stub: launch, split and collectives only",
                          "config": {"restarts_per_gpu": r1 - r0,
                                     "parallelism": f"restart-sharded x{ws}"}}), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def verify_step(acqf, Xd, r0, Xtr, Ytr, Xc_local, best_f, k=8):
    """Outside the timed region, on rank 0: the timed forward's values at k
    t-batches spread over this rank's slice against the CPU restatement
    (oracle/, the checker), at the MC bar of north_star (1e-2) and at 1e-7."""
    from oracle.acquisition import qei
    from oracle.gp import ExactGPOracle, GPHyper
    from oracle.sampling import draw_sobol_normal_samples
    b = Xd.shape[0]
    idx = torch.linspace(0, b - 1, k).round().long()
    with torch.no_grad():
        got = acqf(Xd).cpu()[idx]
    h = GPHyper(torch.full((D,), LENGTHSCALE, dtype=torch.float64), NOISE, CONSTANT)
    ref = qei(ExactGPOracle(Xtr, Ytr, h), Xc_local[idx], draw_sobol_normal_samples(Q, MC, 0), best_f)
    pos = ref > 0
    err = ((got - ref).abs()[pos] / ref[pos]).max().item() if pos.any() else 0.0
    ok = bool(torch.allclose(got, ref, rtol=1e-7, atol=1e-12))
    if not ok or int(pos.sum()) < k // 4:
        raise SystemExit(f"bench: the timed forward disagrees with the oracle (or is degenerate): "
                         f"{got} vs {ref}")
    return {"t_batches": [int(r0 + i) for i in idx], "nonzero": int(pos.sum()),
            "max_rel_err_nonzero": err, "rtol": 1e-7, "atol": 1e-12}


def verify_grad(acqf, Xd, r0, Xtr, Ytr, Xc_local, best_f, k=8):
    """Outside the timed region, on rank 0: dX of the timed forward + backward
    (the fused W = R L^-1 -> dX pass at this size, asserted) at k t-batches
    spread over those with a non-zero value, against torch.autograd through the
    CPU restatement (oracle/, the checker) on those t-batches, rtol 1e-5."""
    from oracle.acquisition import qei
    from oracle.gp import ExactGPOracle, GPHyper
    from oracle.sampling import draw_sobol_normal_samples
    Xg = Xd.detach().clone().requires_grad_(True)
    v = acqf(Xg)
    (g,) = torch.autograd.grad(v.sum(), Xg)
    route = int(torch.ops.bo.last_backward_route())
    v, g = v.detach().cpu(), g.cpu()
    nz = (v > 0).nonzero().flatten()
    if nz.numel() < k:
        raise SystemExit(f"bench: only {nz.numel()} non-zero values to check gradients on")
    idx = nz[torch.linspace(0, nz.numel() - 1, k).round().long()]
    h = GPHyper(torch.full((D,), LENGTHSCALE, dtype=torch.float64), NOISE, CONSTANT)
    Xo = Xc_local[idx].clone().requires_grad_(True)
    ref = qei(ExactGPOracle(Xtr, Ytr, h), Xo, draw_sobol_normal_samples(Q, MC, 0), best_f)
    (go,) = torch.autograd.grad(ref.sum(), Xo)
    err = ((g[idx] - go).abs() / go.abs().clamp_min(1e-8)).max().item()
    ok = bool(torch.allclose(g[idx], go, rtol=1e-5, atol=1e-8))
    if not ok or route != 1:
        raise SystemExit(f"bench: the timed gradient disagrees with the oracle (route {route}): "
                         f"max rel err {err}")
    return {"t_batches": [int(r0 + i) for i in idx], "route": "fused W -> dX (bo_post_w_dx)",
            "max_rel_err": err, "rtol": 1e-5, "atol": 1e-8}



class HookTimer:
    """HIP events around every post_partials launch issued through
    kernels.post_partials (the qNEI / qEHVI routes), recorded on the stream
    the launch is enqueued on (kernels.TIMING_HOOK)."""

    def __init__(self, dev):
        self.dev, self.pairs, self.on = dev, [], False

    def __call__(self, tag):
        if not self.on:
            return
        ev = torch.cuda.Event(enable_timing=True)
        ev.record(torch.cuda.current_stream(self.dev))
        if tag.endswith("_begin"):
            self.pairs.append([ev, None])
        else:
            self.pairs[-1][1] = ev

    def read(self):
        torch.cuda.synchronize(self.dev)
        out = [a.elapsed_time(b) for a, b in self.pairs]
        self.pairs = []
        return out


def c4_problem():
    """C4: DTLZ2(d=6, m=3) on torch.rand(2048, 6, seed 0),
    ref point -1.1, lengthscale 0.6, noise 1e-3 per member."""
    from botorch_amd.test_functions import DTLZ2
    g = torch.Generator().manual_seed(0)
    X = torch.rand(2048, D, generator=g, dtype=torch.float64)
    Y = -DTLZ2(dim=D, num_objectives=3, negate=True).evaluate_true(X)
    return X, Y, torch.full((3,), -1.1, dtype=torch.float64), 0.6, 1e-3


def make_workload(acq, dev):
    """The bench workload for ``--acq``: the acquisition on one GPU's
    replicated model, the GLOBAL candidate draw (sliced by the caller), and
    the algorithmic work of its dominant kernel.  qei / qnei: C3 (n = 4096,
    q = 16, S = 512, 512 restarts; qNEI prunes X_baseline = X_tr on every rank
    from the same seed, replicated); qehvi: C4 (ModelListGP(3) on DTLZ2,
    n = 2048, q = 8, S = 128, 128 restarts; the box decomposition built on
    every rank)."""
    from types import SimpleNamespace
    from botorch_amd.acquisition import (qExpectedHypervolumeImprovement, qExpectedImprovement,
                                         qNoisyExpectedImprovement)
    from botorch_amd.models import ModelListGP, SingleTaskGP
    from botorch_amd.sampling import SobolQMCNormalSampler
    from botorch_amd.utils_sampling import draw_sobol_samples
    unit = torch.stack([torch.zeros(D, dtype=torch.float64), torch.ones(D, dtype=torch.float64)])

    def stgp(X, Y, ls, noise):
        m = SingleTaskGP(X.to(dev), Y.to(dev))
        m.covar_module.lengthscale = torch.full((1, D), ls, dtype=torch.float64)
        m.likelihood.noise = torch.tensor([noise], dtype=torch.float64)
        m.mean_module.constant = torch.tensor(CONSTANT, dtype=torch.float64)
        return m.eval()

    if acq in ("qei", "qnei"):
        Xtr, Ytr, Xc = build_problem(dev, RESTARTS)
        model = stgp(Xtr, Ytr, LENGTHSCALE, NOISE)
        model.prediction_cache()  # the reference builds its caches on the first eval call
        sampler = SobolQMCNormalSampler(torch.Size([MC]), seed=0)
        w = SimpleNamespace(acq=acq, q=Q, S=MC, restarts=RESTARTS, n=N_TRAIN, Xtr=Xtr, Ytr=Ytr,
                            Xc=Xc, launches=1)
        if acq == "qei":
            # best_f 1.5 below the data maximum: with best_f =
            # max Y no Sobol candidate improves on 4096 observations and every value
            # would be exactly 0; the work per step does not depend on it
            w.best_f = Ytr.max().item() - 1.5
            w.acqf = qExpectedImprovement(model, w.best_f, sampler=sampler)
            w.name = "qEI"
            w.extra_flops = 0
            w.workload = "C3 qEI forward: SingleTaskGP n=4096 d=6, q=16"
            w.tail = "512 Sobol MC samples, best_f = max(Y) - 1.5"
        else:
            torch.manual_seed(0)  # the pruning's sampler seed: identical on every rank
            t0 = time.perf_counter()
            w.acqf = qNoisyExpectedImprovement(model, Xtr.to(dev), sampler=sampler,
                                               prune_baseline=True)
            torch.cuda.synchronize(dev)
            w.init_ms = 1e3 * (time.perf_counter() - t0)
            w.r = int(w.acqf.X_baseline.shape[0])
            w.name = "qNEI"
            # the cached-root cross term rides the posterior pass: + 2 B q r n
            w.extra_flops = 2 * Q * w.r * N_TRAIN
            w.workload = (f"C3 qNEI forward: SingleTaskGP n=4096 d=6, q=16, X_baseline = X_tr "
                          f"pruned on every rank (r = {w.r}, cache_root)")
            w.tail = "512 Sobol MC samples"
        w.flops_launch = lambda b: flops_post_partials(b, Q, N_TRAIN) + b * w.extra_flops
        w.bytes_launch = lambda b: post_partials_bytes(b, Q, N_TRAIN)
        w.kernel_prefix = "post_partials_kernel<0, 6, false, false, true, false>"
        return w
    X, Y, ref, ls, noise = c4_problem()
    from botorch_amd.multi_objective import FastNondominatedPartitioning
    models = [stgp(X, Y[:, t:t + 1], ls, noise) for t in range(3)]
    part = FastNondominatedPartitioning(ref, Y)
    q, S, b, n = 8, 128, 128, 2048
    w = SimpleNamespace(acq=acq, q=q, S=S, restarts=b, n=n, Xtr=X, Ytr=Y, ref=ref, ls=ls,
                        noise=noise, launches=3, name="qEHVI", extra_flops=0)
    w.acqf = qExpectedHypervolumeImprovement(ModelListGP(*models), ref.tolist(), part,
                                             sampler=SobolQMCNormalSampler(torch.Size([S]), seed=0))
    w.cells = part.get_hypercell_bounds()
    w.Xc = draw_sobol_samples(unit, b, q, seed=1)
    w.flops_launch = lambda bb: flops_post_partials(bb, q, n)
    w.bytes_launch = lambda bb: post_partials_bytes(bb, q, n)
    w.kernel_prefix = "post_partials_kernel<0, 6, false, false, true, false>"
    w.workload = (f"C4 qEHVI forward: ModelListGP(3) on DTLZ2 n=2048 d=6, q=8, "
                  f"{int(w.cells[0].shape[0])} hypercells")
    w.tail = "128 Sobol MC samples, ref point -1.1"
    return w


def verify_other(w, acqf, Xd, r0, Xc_local, k=4):
    """verify_step for qNEI / qEHVI: the timed forward's values at k spread
    t-batches against the CPU restatement (oracle/, the checker) at 1e-7."""
    from oracle import acquisition as oacq
    from oracle.gp import ExactGPOracle, GPHyper
    from oracle.sampling import base_samples_multi_output
    b = Xd.shape[0]
    idx = torch.linspace(0, b - 1, k).round().long()
    with torch.no_grad():
        got = acqf(Xd).cpu()[idx]
    if w.acq == "qnei":
        orc = ExactGPOracle(w.Xtr, w.Ytr, GPHyper(torch.full((D,), LENGTHSCALE, dtype=torch.float64),
                                                  NOISE, CONSTANT))
        ref = oacq.QNEIOracle(orc, acqf.X_baseline.cpu(), w.S, seed=0)(Xc_local[idx])
    else:
        orcs = [ExactGPOracle(w.Xtr, w.Ytr[:, t:t + 1],
                              GPHyper(torch.full((D,), w.ls, dtype=torch.float64), w.noise, 0.0))
                for t in range(3)]
        lo, hi = w.cells
        ref = oacq.qehvi(orcs, Xc_local[idx], base_samples_multi_output(w.S, w.q, 3, 0), lo, hi)
    ok = bool(torch.allclose(got, ref, rtol=1e-7, atol=1e-12))
    extra = None
    if ok and not bool((ref > 0).any()) and w.acq == "qnei":
        # the Sobol candidates of the timed batch improve on no baseline sample
        # at C3's hyperparameters (every value exactly 0 on both sides): check
        # the same acquisition also at 4 t-batches around the kept baseline
        # point, where it is positive
        g = torch.Generator().manual_seed(7)
        Xb = acqf.X_baseline.cpu()[:1]
        Xn = (Xb.unsqueeze(0) + 0.05 * torch.randn(4, w.q, D, generator=g, dtype=torch.float64)
              ).clamp(0, 1)
        with torch.no_grad():
            gn = acqf(Xn.to(Xd.device)).cpu()
        rn = oacq.QNEIOracle(orc, acqf.X_baseline.cpu(), w.S, seed=0)(Xn)
        ok = bool(torch.allclose(gn, rn, rtol=1e-7, atol=1e-12))
        got, ref = torch.cat([got, gn]), torch.cat([ref, rn])
        extra = "4 t-batches around the baseline point (the timed ones are all exactly 0)"
    if not ok or not bool((ref > 0).any()):
        raise SystemExit(f"bench: the timed {w.name} forward disagrees with the oracle (or is "
                         f"degenerate): {got} vs {ref}")
    pos = ref > 0
    return {"t_batches": [int(r0 + i) for i in idx], "nonzero": int(pos.sum()),
            "max_rel_err_nonzero": ((got - ref).abs()[pos] / ref[pos]).max().item(),
            "rtol": 1e-7, "atol": 1e-12, "extra_points": extra}


def cpu_baseline_other(w, acqf, budget_s=20.0):
    """cpu_baseline for qNEI / qEHVI: the oracle's forward on a bounded slice
    of the same workload (8 / 2 restarts), median per call."""
    from oracle import acquisition as oacq
    from oracle.gp import ExactGPOracle, GPHyper
    from oracle.sampling import base_samples_multi_output
    torch.set_num_threads(cpu_cores())
    if w.acq == "qnei":
        orc = ExactGPOracle(w.Xtr, w.Ytr, GPHyper(torch.full((D,), LENGTHSCALE, dtype=torch.float64),
                                                  NOISE, CONSTANT))
        ref = oacq.QNEIOracle(orc, acqf.X_baseline.cpu(), w.S, seed=0)
        bs = 8
        fn = lambda: ref(w.Xc[:bs])  # noqa: E731
        what = "full (r+q) posterior per t-batch, as the reference"
    else:
        orcs = [ExactGPOracle(w.Xtr, w.Ytr[:, t:t + 1],
                              GPHyper(torch.full((D,), w.ls, dtype=torch.float64), w.noise, 0.0))
                for t in range(3)]
        Zm = base_samples_multi_output(w.S, w.q, 3, 0)
        lo, hi = w.cells
        bs = 2
        fn = lambda: oacq.qehvi(orcs, w.Xc[:bs], Zm, lo, hi)  # noqa: E731
        what = "dense inclusion-exclusion over all 255 q-subsets x cells, as the reference"
    med, runs = _cpu_time(fn, budget_s=budget_s, max_runs=7)
    return {"value": bs * w.q * w.S / med, "unit": "acq-evals/s", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"{w.name} forward, {bs} of the {w.restarts} restarts ({what}), median of "
                      f"{runs} runs; torch fp64 CPU restatement (oracle/), {cpu_model()}"}


def sharded_other_acqs(dev, dist, ws, rank, steps, warmup):
    """N > 1: C3 qNEI (pruning replicated) and C4 qEHVI (partitioning
    replicated) with their restarts sharded over the ranks and the values
    gathered by one all-reduce, timed like the headline (barriers, max over
    ranks); SURVEY.md 8(e) for the configs BASELINE.json names on 8 / 4 GPUs."""
    from botorch_amd.distributed import allgather_rows, shard_range
    out = {}
    sync = lambda: torch.cuda.synchronize(dev)  # noqa: E731
    for acq in ("qnei", "qehvi"):
        w = make_workload(acq, dev)
        r0, r1 = shard_range(w.restarts, ws, rank)
        Xd = w.Xc[r0:r1].to(dev)
        best = torch.empty(1, dtype=torch.float64, device=dev)

        def step():
            with torch.no_grad():
                acq_v = w.acqf(Xd)
            torch.amax(allgather_rows(acq_v, w.restarts), dim=0, keepdim=True, out=best)

        el = timed_steps(step, steps, warmup, dist, sync, dev)
        out[w.name] = {"workload": w.workload, "value": w.q * w.restarts * w.S * steps / el,
                       "unit": "acq-evals/s", "ms_per_step": 1e3 * el / steps,
                       "restarts_per_gpu": r1 - r0, "scaling": "strong",
                       **({"r": w.r} if acq == "qnei" else {})}
        del w
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="number of GPUs (ranks); without torchrun's env, N > 1 launches them")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-fit", action="store_true", help="skip the GP-fit half of the metric")
    ap.add_argument("--no-bwd", action="store_true", help="skip the forward+backward timing")
    ap.add_argument("--weak", action="store_true",
                    help="N > 1: each rank its own 512 restarts (weak scaling) as the headline")
    ap.add_argument("--strong", action="store_true", help=argparse.SUPPRESS)  # the N > 1 default
    ap.add_argument("--acq", choices=("qei", "qnei", "qehvi"), default="qei",
                    help="the timed acquisition: C3 qEI (default, the BASELINE metric), C3 qNEI "
                         "(pruning replicated per rank) or C4 qEHVI (partitioning replicated)")
    ap.add_argument("--no-extra", action="store_true",
                    help="skip the other section-8 configurations (C2, C3 qNEI, C4, C5)")
    args = ap.parse_args()
    if args.gpus is None:
        args.gpus = int(os.environ.get("WORLD_SIZE", "1"))
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(_launch_ranks(args.gpus))
    ws, rank, local = _dist_env()
    if ws != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE={ws}")
    rehearse = os.environ.get("BO_BENCH_REHEARSE", "0")
    if rehearse == "cpu":
        return rehearse_cpu(args, ws, rank)
    # BO_BENCH_REHEARSE=1: every rank on cuda:0 over gloo -- a one-GPU rehearsal
    # of the multi-rank code path (barriers, max over ranks, rank-0 report);
    # never the measured configuration
    if rehearse == "1":
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if ws > 1:
        import torch.distributed as dist
        if rehearse == "1":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
        assert dist.get_world_size() == args.gpus
    # N > 1: the headline is north_star's C3 split -- ONE global draw of 512
    # restarts sharded over the ranks (strong scaling); --weak: 512 per rank
    strong = ws > 1 and not args.weak

    from botorch_amd import _lib, kernels
    from botorch_amd.distributed import allgather_rows, shard_range
    w = make_workload(args.acq, dev)
    acqf, R = w.acqf, w.restarts
    r0, r1 = 0, R
    Xc = w.Xc
    if strong:  # one global draw, each rank its contiguous slice
        r0, r1 = shard_range(R, ws, rank)
        Xc = w.Xc[r0:r1]
    elif ws > 1 and w.acq == "qei":
        Xc = build_problem(dev, RESTARTS, seed_offset=rank)[2]
    Xd = Xc.to(dev)
    Xtr, Ytr = w.Xtr, w.Ytr

    # HIP events around every post_partials launch of the timed steps, on the
    # stream it is launched on: recorded by the native operator (qEI,
    # bo::post_timing) or by kernels.post_partials's hook (qNEI / qEHVI)
    native = _lib.torch_ops()
    hook = HookTimer(dev)
    kernels.TIMING_HOOK = hook
    best = torch.empty(1, dtype=torch.float64, device=dev)

    def step():
        with torch.no_grad():
            acq = acqf(Xd)
        if strong:
            allv = allgather_rows(acq, R)   # every rank: all the step's values
            torch.amax(allv, dim=0, keepdim=True, out=best)
            return allv
        torch.amax(acq, dim=0, keepdim=True, out=best)
        if dist is not None:
            dist.all_reduce(best, op=dist.ReduceOp.MAX)
        return acq

    sync = lambda: torch.cuda.synchronize(dev)  # noqa: E731
    # warm-up outside the event window, then the timed K steps
    for _ in range(args.warmup):
        step()
    sync()
    native.post_timing_read()  # drop anything recorded before
    hook.read()
    native.post_timing(True)
    hook.on = True
    elapsed = timed_steps(step, args.steps, 0, dist, sync, dev)
    native.post_timing(False)
    hook.on = False
    kern_ms = native.post_timing_read().tolist() + hook.read()
    if not kern_ms or len(kern_ms) % args.steps:
        raise SystemExit(f"bench: {len(kern_ms)} timed posterior launches for {args.steps} steps")
    launches = len(kern_ms) // args.steps  # qEHVI: one batched launch for its three members
    ms_step = 1e3 * elapsed / args.steps
    evals_per_step = w.q * R * w.S * (1 if strong else ws)
    value = evals_per_step * args.steps / elapsed

    kern_avg_ms = sum(kern_ms) / len(kern_ms)
    fl = w.flops_launch(r1 - r0) * w.launches / launches  # the step's posterior flops per launch
    achieved = fl / (kern_avg_ms * 1e-3) / 1e12
    peak = 78.6  # MI355X dense FP64 matrix TFLOP/s (MI355X_MICROARCH.md / SURVEY.md 8(d))
    peak_box = mfma_f64_ceiling(dev)
    # the committed PMC passes are of the qEI bench command
    traffic, traffic_src, traffic_note = pmc_traffic(r1 - r0) if w.acq == "qei" else (None,) * 3
    alg_bytes = w.bytes_launch(r1 - r0)

    weak = None
    if strong and w.acq == "qei":
        # the weak line beside it: each rank its own 512 restarts (seed 1 + rank)
        Xw = build_problem(dev, RESTARTS, seed_offset=rank)[2].to(dev)

        def step_weak():
            with torch.no_grad():
                acq = acqf(Xw)
            torch.amax(acq, dim=0, keepdim=True, out=best)
            dist.all_reduce(best, op=dist.ReduceOp.MAX)

        ew = timed_steps(step_weak, args.steps, args.warmup, dist, sync, dev)
        weak = {"value": Q * RESTARTS * MC * ws * args.steps / ew,
                "ms_per_step": 1e3 * ew / args.steps, "restarts_per_gpu": RESTARTS,
                "note": "each rank its own 512 restarts, one all-reduce(MAX) per step"}
    sharded_other = None
    if ws > 1 and w.acq == "qei" and not args.no_extra:
        sharded_other = sharded_other_acqs(dev, dist, ws, rank, args.steps, args.warmup)

    # forward + backward (the optimize_acqf call pattern, gen.py:194-222)
    Xg = Xd.clone().requires_grad_(True)

    def fwd_bwd():
        v = acqf(Xg)
        torch.autograd.grad(v.sum(), Xg)

    if args.no_bwd:  # PMC passes: forward launches only (the gradient path also writes R^T)
        fwd_bwd = None
    else:
        fb_s = _gpu_time(fwd_bwd, steps=5, warmup=2)
        fwd_bwd = {"evals_per_s": w.q * (r1 - r0) * w.S / fb_s, "ms": 1e3 * fb_s}

    strong_proj = None
    if ws == 1 and not args.no_extra and w.acq == "qei":
        # the per-rank shard of the strong split, timed on this GPU (projection)
        strong_proj = {"note": "projection: the C3 qEI step at b = 512/W restarts on one GPU, "
                               "collectives excluded; value = 512*q*S / step time"}
        from botorch_amd.graphs import GraphedAcquisition
        for W in (1, 2, 4, 8):
            Xs = Xd[: RESTARTS // W]
            with torch.no_grad():
                tW = _gpu_time(lambda: acqf(Xs), steps=10, warmup=2)
            gW = GraphedAcquisition(acqf, Xs, share_input=True)  # the same forward as a HIP graph
            tG = _gpu_time(lambda: gW(Xs), steps=10, warmup=2)
            strong_proj[f"W{W}"] = {"restarts_per_gpu": RESTARTS // W, "ms": 1e3 * tW,
                                    "projected_value": Q * RESTARTS * MC / tW,
                                    "ms_graphed": 1e3 * tG,
                                    "projected_value_graphed": Q * RESTARTS * MC / tG}
            del gW
    gp_fit = None
    extra = None
    check = None
    chol = time_cholesky(build_problem(dev, 1)[0], dev) if rank == 0 else None
    if rank == 0 and ws == 1 and not args.no_extra and w.acq == "qei":
        extra = other_configs(dev, cpu=not args.no_cpu_baseline)
    if rank == 0 and not args.no_fit:
        Xf, Yf, _ = build_problem(dev, 1)
        gp_fit = time_gp_fit(Xf, Yf, dev, cpu=(not args.no_cpu_baseline and ws == 1))
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline:
            # the CPU leg: the oracle checks the timed forward, then (N = 1) is timed
            if w.acq == "qei":
                check = verify_step(acqf, Xd, r0, Xtr, Ytr, Xc, w.best_f)
                if fwd_bwd is not None:
                    fwd_bwd["check"] = verify_grad(acqf, Xd, r0, Xtr, Ytr, Xc, w.best_f)
                if ws == 1:
                    cpu = cpu_baseline(Xtr, Ytr, Xc, w.best_f)
            else:
                check = verify_other(w, acqf, Xd, r0, Xc)
                if ws == 1:
                    cpu = cpu_baseline_other(w, acqf)
        line = {
            "metric": f"acq-evals/sec (q x restarts x MC), {w.name} forward",
            "value": value,
            "unit": "acq-evals/s",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_step,
            "higher_is_better": True,
            "scaling": "single" if ws == 1 else ("strong" if strong else "weak"),
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("synthetic: Hartmann6 on Sobol(seed 0) training inputs, " if w.acq != "qehvi"
                     else "synthetic: DTLZ2 on torch.rand(seed 0) training inputs, ")
                    + ("Sobol(seed 1) candidates, rank slice" if strong
                       else ("Sobol(seed 1+rank) candidates" if w.acq == "qei"
                             else "Sobol(seed 1) candidates")),
            "config": {"workload": w.workload + ", "
                                   + (f"{R} restarts sharded over the GPUs" if strong
                                      else f"{R} restarts/GPU") + ", " + w.tail,
                       "n": w.n, "d": D, "q": w.q, "restarts_per_gpu": r1 - r0, "mc": w.S,
                       "parallelism": f"restart-sharded x{ws}"},
            "roofline": {"bound": "mfma", "kernel": "post_partials_kernel",
                         "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                         "frac": achieved / peak, "peak_measured": peak_box,
                         "frac_of_measured": achieved / peak_box if peak_box else None,
                         "traffic": traffic,
                         "traffic_unit": "bytes/launch", "traffic_source": traffic_src,
                         "algorithmic_bytes": alg_bytes,
                         "traffic_ratio": traffic / alg_bytes if traffic else None,
                         "traffic_note": traffic_note,
                         "kernel_ms": kern_avg_ms, "flops_per_launch": fl,
                         "launches_per_step": launches},
            "cpu_baseline": cpu,
            "check": check,
            "weak": weak,
            "sharded_other_acqs": sharded_other,
            "fwd_bwd": fwd_bwd,
            "strong_scaling_projection": strong_proj,
            "cholesky": chol,
            "gp_fit": gp_fit,
            "other_configs": extra,
        }
        if w.acq == "qnei":
            line["config"].update(r=w.r, init_ms=w.init_ms)
        if cpu:
            line["speedup_vs_cpu"] = value / cpu["value"]
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.barrier()  # rank 0's CPU baseline / report must finish before teardown
        dist.destroy_process_group()

if __name__ == "__main__":
    main()
