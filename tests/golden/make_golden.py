"""Generate the golden fixtures in ``tests/golden/`` from the reference BoTorch.

Runs ONLY in the development container, where ``/root/reference`` exists.  It
imports the gpytorch-free leaf modules of the reference (see ``_refload.py``)
and records their outputs as data (inputs + expected outputs) in
``golden.npz``.  The fixtures travel to the GPU box; the reference does not.

Usage:  python tests/golden/make_golden.py

Sources (reference file:line):
  * draw_sobol_normal_samples  botorch/utils/sampling.py:108-137
    (NormalQMCEngine.draw, botorch/sampling/qmc.py:60-98, inv_transform=True)
  * draw_sobol_samples         botorch/utils/sampling.py:66-105
  * Hartmann(dim=6)            botorch/test_functions/synthetic.py:359-455
  * DTLZ2                      botorch/test_functions/multi_objective.py:420-450
  * ndtr / phi                 botorch/utils/probability/utils.py:133-142
  * NondominatedPartitioning / FastNondominatedPartitioning
                               botorch/utils/multi_objective/box_decompositions/non_dominated.py
  * is_non_dominated           botorch/utils/multi_objective/pareto.py:16-64
  * DominatedPartitioning.compute_hypervolume
                               botorch/utils/multi_objective/box_decompositions/dominated.py
  * log_fatplus / log_softplus / fatmax / smooth_amax / logmeanexp
                               botorch/utils/safe_math.py:209-352, composed as
                               acquisition/logei.py:122, 219-234, 509-534
  * compute_feasibility_indicator / compute_smoothed_feasibility_indicator
                               botorch/utils/objective.py:101-180
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import _refload  # noqa: E402

from cases import HV_CASES, LOGEI_CASES, SOBOL_BOX_CASES, SOBOL_NORMAL_CASES  # noqa: E402


def main():
    sampling = _refload.load("botorch.utils.sampling")
    synth = _refload.load("botorch.test_functions.synthetic")
    mo = _refload.load("botorch.test_functions.multi_objective")
    prob = _refload.load("botorch.utils.probability.utils")
    nd = _refload.load("botorch.utils.multi_objective.box_decompositions.non_dominated")
    pareto = _refload.load("botorch.utils.multi_objective.pareto")

    out = {}
    for d, n, seed in SOBOL_NORMAL_CASES:
        z = sampling.draw_sobol_normal_samples(d=d, n=n, dtype=torch.double, seed=seed)
        out[f"sobol_normal_d{d}_n{n}_s{seed}"] = z.numpy()

    bounds = torch.stack([torch.zeros(6, dtype=torch.double), torch.ones(6, dtype=torch.double)])
    for n, q, d, seed in SOBOL_BOX_CASES:
        b = torch.stack([torch.zeros(d, dtype=torch.double), torch.ones(d, dtype=torch.double)])
        x = sampling.draw_sobol_samples(bounds=b, n=n, q=q, seed=seed)
        out[f"sobol_box_n{n}_q{q}_d{d}_s{seed}"] = x.numpy()

    # Hartmann6 (negate=True) on the C1/C2 training designs and a random set.
    h6 = synth.Hartmann(dim=6, negate=True)
    for key in ("sobol_box_n20_q1_d6_s0",):
        X = torch.from_numpy(out[key]).squeeze(1)
        out["hartmann6_X"] = X.numpy()
        out["hartmann6_Y"] = h6(X).numpy()
    g = torch.Generator().manual_seed(3)
    Xr = torch.rand(257, 6, generator=g, dtype=torch.double)
    out["hartmann6_rand_X"] = Xr.numpy()
    out["hartmann6_rand_Y"] = h6(Xr).numpy()

    # DTLZ2 (dim 6, 3 objectives, negate=True) on torch.rand(2048, 6) with seed 0.
    dtlz = mo.DTLZ2(dim=6, num_objectives=3, negate=True)
    g = torch.Generator().manual_seed(0)
    Xd = torch.rand(2048, 6, generator=g, dtype=torch.double)
    Yd = dtlz(Xd)
    out["dtlz2_X"] = Xd.numpy()
    out["dtlz2_Y"] = Yd.numpy()
    ref = torch.full((3,), -1.1, dtype=torch.double)
    part = nd.FastNondominatedPartitioning(ref_point=ref, Y=Yd)
    cb = part.get_hypercell_bounds()
    out["dtlz2_cells_lower"] = cb[0].numpy()
    out["dtlz2_cells_upper"] = cb[1].numpy()
    out["dtlz2_pareto_mask"] = pareto.is_non_dominated(Yd).numpy()
    out["dtlz2_hv"] = np.array(part.compute_hypervolume().item())

    # A small DTLZ2 subset (used by the fast CPU tests).
    Ys = Yd[:64]
    part_s = nd.FastNondominatedPartitioning(ref_point=ref, Y=Ys)
    cbs = part_s.get_hypercell_bounds()
    out["dtlz2_small_Y"] = Ys.numpy()
    out["dtlz2_small_cells_lower"] = cbs[0].numpy()
    out["dtlz2_small_cells_upper"] = cbs[1].numpy()
    out["dtlz2_small_hv"] = np.array(part_s.compute_hypervolume().item())

    # Box decompositions used by the reference's qEHVI known-answer tests
    # (test/acquisition/multi_objective/test_monte_carlo.py:160-510).
    ehvi_cases = {
        "m2": ([[4.0, 5.0], [5.0, 5.0], [8.5, 3.5], [8.5, 3.0], [9.0, 1.0]], [0.0, 0.0]),
        "m3a_refm1": ([[4.0, 2.0, 3.0], [3.0, 5.0, 1.0], [2.0, 4.0, 2.0], [1.0, 3.0, 4.0]], [-1.0] * 3),
        "m3a_ref0": ([[4.0, 2.0, 3.0], [3.0, 5.0, 1.0], [2.0, 4.0, 2.0], [1.0, 3.0, 4.0]], [0.0] * 3),
        "m3a_ref1": ([[4.0, 2.0, 3.0], [3.0, 5.0, 1.0], [2.0, 4.0, 2.0], [1.0, 3.0, 4.0]], [1.0] * 3),
        "m3b_refm1": ([[4.0, 2.0, 3.0], [3.0, 5.0, 1.0], [2.0, 4.0, 2.0]], [-1.0] * 3),
    }
    for name, (pY, rp) in ehvi_cases.items():
        pY = torch.tensor(pY, dtype=torch.double)
        rp = torch.tensor(rp, dtype=torch.double)
        for cls_name in ("NondominatedPartitioning", "FastNondominatedPartitioning"):
            p = getattr(nd, cls_name)(ref_point=rp, Y=pY)
            lo, hi = p.get_hypercell_bounds()
            tag = "nd" if cls_name.startswith("Non") else "fnd"
            out[f"ehvi_{name}_{tag}_lower"] = lo.numpy()
            out[f"ehvi_{name}_{tag}_upper"] = hi.numpy()
        out[f"ehvi_{name}_pareto_Y"] = pY.numpy()
        out[f"ehvi_{name}_ref_point"] = rp.numpy()

    # Normal CDF / PDF.
    x = torch.linspace(-8, 8, 161, dtype=torch.double)
    out["ndtr_x"] = x.numpy()
    out["ndtr_y"] = prob.ndtr(x).numpy()
    out["phi_y"] = prob.phi(x).numpy()

    # LogEI reductions (values and gradients w.r.t. the samples).
    sm = _refload.load("botorch.utils.safe_math")
    g = torch.Generator().manual_seed(11)
    obj = 0.3 * torch.randn(64, 5, 4, generator=g, dtype=torch.double)
    bf_s = 0.2 + 0.1 * torch.randn(64, generator=g, dtype=torch.double)
    out["logei_obj"] = obj.numpy()
    out["logei_best_f_s"] = bf_s.numpy()
    for tag, (fat, tau_relu, tau_max) in LOGEI_CASES.items():
        for bname, bf in (("scalar", torch.full((64,), 0.2, dtype=torch.double)), ("persample", bf_s)):
            x = obj.clone().requires_grad_(True)
            z = x - bf.view(-1, 1, 1)
            li = (sm.log_fatplus if fat else sm.log_softplus)(z, tau=tau_relu)
            u = (sm.fatmax if fat else sm.smooth_amax)(li, dim=-1, tau=tau_max)
            acq = sm.logmeanexp(u, dim=0)
            (gx,) = torch.autograd.grad(acq.sum(), x)
            out[f"logei_{tag}_{bname}_acq"] = acq.detach().numpy()
            out[f"logei_{tag}_{bname}_grad"] = gx.numpy()

    # Exact dominated hypervolumes (DominatedPartitioning.compute_hypervolume,
    # box_decompositions/dominated.py) of random point sets, with and without
    # one extra point: HV differences are the qNEHVI per-sample improvements.
    dom = _refload.load("botorch.utils.multi_objective.box_decompositions.dominated")
    g = torch.Generator().manual_seed(21)
    for m_, n_ in HV_CASES:
        Y = torch.rand(n_, m_, generator=g, dtype=torch.double)
        ref = torch.full((m_,), 0.1, dtype=torch.double)
        extra = torch.rand(4, m_, generator=g, dtype=torch.double) * 1.2
        hv = dom.DominatedPartitioning(ref_point=ref, Y=Y).compute_hypervolume()
        hv_plus = [dom.DominatedPartitioning(ref_point=ref, Y=torch.cat([Y, e.view(1, -1)]))
                   .compute_hypervolume().item() for e in extra]
        out[f"hv_m{m_}_n{n_}_Y"] = Y.numpy()
        out[f"hv_m{m_}_n{n_}_ref"] = ref.numpy()
        out[f"hv_m{m_}_n{n_}_hv"] = np.array(hv.item())
        out[f"hv_m{m_}_n{n_}_extra"] = extra.numpy()
        out[f"hv_m{m_}_n{n_}_hv_plus"] = np.array(hv_plus)

    # Outcome-constraint indicators (utils/objective.py:101-180) on fixed samples
    # with two constraints, all (log, fat) variants, scalar and per-constraint eta.
    objmod = _refload.load("botorch.utils.objective")
    g = torch.Generator().manual_seed(31)
    smp = torch.randn(16, 3, 4, 2, generator=g, dtype=torch.double)
    out["feas_samples"] = smp.numpy()
    cons = [lambda Z: Z[..., 0] - 0.2, lambda Z: 0.5 * Z[..., 1] + Z[..., 0] - 0.4]
    out["feas_hard"] = objmod.compute_feasibility_indicator(cons, smp).numpy()
    for log in (False, True):
        for fat in (False, True):
            for ename, eta in (("e1", 1e-1), ("e2", torch.tensor([0.05, 0.3], dtype=torch.double))):
                x = smp.clone().requires_grad_(True)
                ind = objmod.compute_smoothed_feasibility_indicator(cons, x, eta, log=log, fat=fat)
                (gx,) = torch.autograd.grad(ind.sum(), x)
                out[f"feas_l{int(log)}_f{int(fat)}_{ename}"] = ind.detach().numpy()
                out[f"feas_l{int(log)}_f{int(fat)}_{ename}_grad"] = gx.numpy()

    path = os.path.join(HERE, "golden.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path}: {len(out)} arrays, {os.path.getsize(path)} bytes")


if __name__ == "__main__":
    main()
