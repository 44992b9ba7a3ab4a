"""Golden fixtures of the linear-constraint path (``golden_polytope.npz``).

Runs ONLY in the development container, where ``/root/reference`` exists: it
imports two gpytorch-free leaf modules of the reference through ``_refload``
and records inputs and outputs as plain arrays.  The fixtures travel to the
GPU box; the reference does not.

Usage:  python tests/golden/make_golden_polytope.py

Sources (reference file:line):
  * sample_polytope               botorch/utils/sampling.py:219-309
  * find_interior_point           botorch/utils/sampling.py:376-454
  * HitAndRunPolytopeSampler      botorch/utils/sampling.py:457-704
  * get_polytope_samples          botorch/utils/sampling.py:882-954
  * sparse_to_dense_constraints   botorch/utils/sampling.py:957-985
  * normalize_{sparse,dense}_linear_constraints  botorch/utils/sampling.py:828-879
  * make_scipy_linear_constraints botorch/optim/parameter_constraints.py:68-312
  * make_scipy_bounds             botorch/optim/parameter_constraints.py:29-65
  * _generate_unfixed_lin_constraints  botorch/optim/parameter_constraints.py:412-471

The inter-point path of sample_q_batches_from_polytope (optim/initializers.py:
178-240) lives in a module that imports gpytorch; its fixture is the
reference's get_polytope_samples called on the q-stacked bounds and the
flattened constraints that initializers.py:72-175 builds (indices i*d + j),
written out here by hand from those lines.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import _refload  # noqa: E402

from cases import POLYTOPE_CASES  # noqa: E402

D = torch.double


def t(x, dtype=D):
    return torch.tensor(x, dtype=dtype)


def main():
    smp = _refload.load("botorch.utils.sampling")
    pc = _refload.load("botorch.optim.parameter_constraints")
    out = {}

    # -- sample_polytope: a triangle-cut box, interior start and a start on a face
    A = t([[1.0, 1.0], [-1.0, 0.0], [0.0, -1.0], [1.0, -2.0]])
    b = t([[1.5], [0.0], [0.0], [0.5]])
    out["sp_A"], out["sp_b"] = A.numpy(), b.numpy()
    for tag, x0 in (("interior", [[0.3], [0.4]]), ("face", [[0.0], [0.6]])):
        for n, n0, thin, seed in POLYTOPE_CASES["sample_polytope"]:
            s = smp.sample_polytope(A, b, t(x0), n=n, n0=n0, n_thinning=thin, seed=seed)
            out[f"sp_{tag}_x0"] = np.asarray(x0)
            out[f"sp_{tag}_n{n}_b{n0}_t{thin}_s{seed}"] = s.numpy()

    # -- find_interior_point: bounded, unbounded (slack capped at 1), with equality
    Ab = np.array([[1.0, 1.0], [-1.0, 0.0], [0.0, -1.0]])
    bb = np.array([[1.0], [0.0], [0.0]])
    out["fip_A"], out["fip_b"] = Ab, bb
    out["fip_bounded"] = smp.find_interior_point(Ab, bb)
    Au, bu = np.array([[-1.0, 0.0], [0.0, -1.0]]), np.array([[0.0], [0.0]])
    out["fip_unb_A"], out["fip_unb_b"] = Au, bu
    out["fip_unbounded"] = smp.find_interior_point(Au, bu)
    Aeq, beq = np.array([[1.0, -1.0, 0.0]]), np.array([0.2])
    out["fip_eq_A_eq"], out["fip_eq_b_eq"] = Aeq, beq
    out["fip_eq"] = smp.find_interior_point(Ab, bb, A_eq=Aeq, b_eq=beq)

    # -- HitAndRunPolytopeSampler: non-unit bounds, dense inequality + equality,
    #    two consecutive draws (burn-in on the first only, seed advanced by n)
    bounds = t([[-1.0, 0.0, 0.0, 2.0], [1.0, 2.0, 1.0, 5.0]])
    Ai = t([[1.0, 1.0, 0.0, 0.0], [0.0, -1.0, 1.0, 0.5]])
    bi = t([[1.5], [2.0]])
    C = t([[1.0, 0.0, 1.0, 0.0]])
    dc = t([[0.5]])
    out["hr_bounds"], out["hr_A"], out["hr_b"] = bounds.numpy(), Ai.numpy(), bi.numpy()
    out["hr_C"], out["hr_d"] = C.numpy(), dc.numpy()
    for burn, thin, seed, n1, n2 in POLYTOPE_CASES["hit_and_run"]:
        for eq in (False, True):
            sampler = smp.HitAndRunPolytopeSampler(
                inequality_constraints=(Ai, bi), equality_constraints=(C, dc) if eq else None,
                bounds=bounds, n_burnin=burn, n_thinning=thin, seed=seed)
            tag = f"hr_eq{int(eq)}_b{burn}_t{thin}_s{seed}"
            out[tag + "_x0"] = sampler.x0.numpy()
            out[tag + "_draw1"] = sampler.draw(n1).numpy()
            out[tag + "_draw2"] = sampler.draw(n2).numpy()

    # -- get_polytope_samples with sparse (indices, coefficients, rhs) constraints
    bnd5 = t([[0.0] * 5, [1.0, 1.0, 2.0, 1.0, 1.0]])
    ineq = [(torch.tensor([0, 2]), t([1.0, 1.0]), 0.5), (torch.tensor([1, 3, 4]), t([-1.0, -1.0, -1.0]), -2.0)]
    eqc = [(torch.tensor([0, 1]), t([1.0, 1.0]), 1.0)]
    out["gps_bounds"] = bnd5.numpy()
    for n, burn, thin, seed in POLYTOPE_CASES["get_polytope_samples"]:
        out[f"gps_ineq_n{n}_b{burn}_t{thin}_s{seed}"] = smp.get_polytope_samples(
            n=n, bounds=bnd5, inequality_constraints=ineq, seed=seed, n_burnin=burn,
            n_thinning=thin).numpy()
        out[f"gps_both_n{n}_b{burn}_t{thin}_s{seed}"] = smp.get_polytope_samples(
            n=n, bounds=bnd5, inequality_constraints=ineq, equality_constraints=eqc, seed=seed,
            n_burnin=burn, n_thinning=thin).numpy()
    Ad, bd = smp.sparse_to_dense_constraints(5, ineq)
    out["s2d_A"], out["s2d_b"] = Ad.numpy(), bd.numpy()
    An, bn = smp.normalize_dense_linear_constraints(bnd5, (Ad, bd))
    out["ndl_A"], out["ndl_b"] = An.numpy(), bn.numpy()
    nsl = smp.normalize_sparse_linear_constraints(bnd5, ineq)
    for i, (ix, cf, rhs) in enumerate(nsl):
        out[f"nsl_{i}_idx"], out[f"nsl_{i}_coef"] = ix.numpy(), cf.numpy()
        out[f"nsl_{i}_rhs"] = np.asarray(rhs)

    # -- the inter-point q-batch draw (initializers.py:216-229) on the stacked space
    q, dq = 3, 2
    bq = t([[0.0, 0.0], [1.0, 1.0]])
    inter = [(torch.tensor([[0, 0], [1, 0], [2, 1]]), t([1.0, 1.0, 1.0]), 0.8)]
    intra = [(torch.tensor([0, 1]), t([-1.0, -1.0]), -1.5)]
    # transform_constraints keeps the list order: an intra-point constraint is
    # repeated for every point of the q-batch where it stands, an inter-point
    # one is mapped in place to the flat index k * d + l
    ineq_q = []
    for c in inter + intra:
        if c[0].ndim == 1:
            ineq_q += [(torch.tensor([i * dq + j for j in c[0].tolist()]), c[1], c[2]) for i in range(q)]
        else:
            ineq_q.append((torch.tensor([r[0] * dq + r[1] for r in c[0].tolist()]), c[1], c[2]))
    n, burn, thin, seed = 6, 50, 2, 5
    s = smp.get_polytope_samples(n=n, bounds=torch.hstack([bq] * q), inequality_constraints=ineq_q,
                                 seed=seed, n_burnin=burn, n_thinning=thin * q)
    out["qb_inter"] = s.view(n, q, -1).numpy()
    s = smp.get_polytope_samples(n=n * q, bounds=bq, inequality_constraints=intra, seed=seed,
                                 n_burnin=burn, n_thinning=thin)
    out["qb_intra"] = s.view(n, q, -1).numpy()

    # -- make_scipy_linear_constraints: values and Jacobians at a fixed point
    shapeX = torch.Size([3, 2, 4])
    x = np.linspace(-1.0, 2.0, shapeX.numel())
    ineq1 = [(torch.tensor([1, 3]), t([1.0, 0.5]), -0.1)]
    eq2 = [(torch.tensor([[0, 1], [1, 3]]), t([1.0, -2.0]), 0.25)]
    cons = pc.make_scipy_linear_constraints(shapeX, inequality_constraints=ineq1,
                                            equality_constraints=eq2)
    out["msl_x"] = x
    out["msl_type"] = np.array([1 if c["type"] == "eq" else 0 for c in cons])
    out["msl_fun"] = np.array([c["fun"](x) for c in cons])
    out["msl_jac"] = np.stack([c["jac"](x) for c in cons])
    sb = pc.make_scipy_bounds(torch.zeros(shapeX, dtype=D), t([0.0, -1.0, 0.0, 0.5]), 2.0)
    out["msb_lb"], out["msb_ub"] = np.asarray(sb.lb), np.asarray(sb.ub)

    # -- fixed features removed from linear constraints
    cl = [(torch.tensor([0, 2, 3]), t([1.0, 2.0, -1.0]), 0.5),
          (torch.tensor([[0, 1], [1, 2]]), t([1.0, 1.0]), 0.3)]
    ff = {2: 0.25}
    new = pc._generate_unfixed_lin_constraints(cl, ff, dimension=4, eq=False)
    for i, (ix, cf, rhs) in enumerate(new):
        out[f"gul_{i}_idx"], out[f"gul_{i}_coef"] = ix.numpy(), cf.numpy()
        out[f"gul_{i}_rhs"] = np.asarray(rhs)
    out["gul_count"] = np.asarray(len(new))

    path = os.path.join(HERE, "golden_polytope.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {len(out)} arrays to {path}")


if __name__ == "__main__":
    main()
