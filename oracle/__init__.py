"""CPU oracle: a restatement of the reference's GP-posterior + MC-acquisition path.

TEST INFRASTRUCTURE ONLY.  Nothing in the product (``botorch_amd``) may import,
call, link or execute anything under ``oracle/``.  The only permitted users are
``tests/`` (as the parity checker), ``__graft_entry__.smoke()`` (as the checker
of the one smoke invocation) and ``bench.py``'s ``cpu_baseline`` leg (the
reference-equivalent CPU path timed on the host cores, ``kind: "port"``).

The reference (anand-12/botorch @ 2024-10-08) is pure Python on PyTorch,
GPyTorch 1.12 and linear_operator 0.5.2.  Neither of the latter two is vendored
or installed, so ``import botorch`` is impossible here and on the GPU box.  The
restatement is therefore torch fp64 on CPU -- the same device-agnostic tensor
program the reference runs on CPU -- with the [G] (gpytorch / linear_operator)
arithmetic written out explicitly.  Every function cites the reference
file:line (paths relative to the reference root) or the pinned [G] routine it
restates.

Parity pinning (see DESIGN.md "Oracle"):
  * pinned by golden fixtures produced by the reference's own gpytorch-free
    modules (``tests/golden/make_golden.py``): Sobol base samples, Sobol boxes,
    Hartmann6, DTLZ2, ndtr/phi, non-dominated box decompositions;
  * pinned by the reference's known-answer tests (transcribed in
    ``tests/test_oracle_known_answers.py``): qEI / qNEI reductions on mocked
    samples, qEHVI values 1.5 .. 22.0, analytic EI 0.19780 ..;
  * self-consistency (reference tests): cached vs. uncached qNEI,
    cached-Cholesky vs. full sampling, Standardize round trip;
  * the [G] numerics themselves (exact prediction, psd_safe_cholesky ladder,
    exact MLL) are **parity unpinned**: no reference test pins a numeric GP
    posterior, and gpytorch 1.12 cannot be run here.
"""
