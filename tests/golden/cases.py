"""Fixture case lists shared by make_golden.py and the tests (pure data)."""

# (d, n, seed) triples of the Sobol base samples the configs use:
#   C2 q=8 S=256, C3 q=16 S=512, C4 q*m=24 S=128, C5 q=4 S=256, small cases.
SOBOL_NORMAL_CASES = [
    (1, 4, 0),
    (3, 16, 1234),
    (8, 256, 0),
    (16, 512, 0),
    (24, 128, 0),
    (4, 256, 0),
    (40, 64, 7),
]

SOBOL_BOX_CASES = [  # (n, q, d, seed)
    (20, 1, 6, 0),
    (64, 8, 6, 1),
    (32, 16, 6, 1),
]

# LogEI reduction cases: tag -> (fat, tau_relu, tau_max); the first is the
# reference default (acquisition/logei.py:66-67, fat=True).
LOGEI_CASES = {
    "default": (True, 1e-6, 1e-2),
    "nofat": (False, 1e-6, 1e-2),
    "fat_wide": (True, 0.1, 0.5),
    "nofat_wide": (False, 0.1, 0.5),
}

# Dominated-hypervolume fixtures: (m objectives, n points).
HV_CASES = [(2, 30), (3, 25), (3, 8)]

# Linear-constraint / polytope fixtures (make_golden_polytope.py).
POLYTOPE_CASES = {
    # (n, n0 burn-in, n_thinning, seed)
    "sample_polytope": [(40, 50, 3, 7), (25, 0, 1, 123)],
    # (n_burnin, n_thinning, seed, first draw, second draw)
    "hit_and_run": [(30, 5, 11, 12, 7), (200, 20, 0, 16, 16)],
    # (n, n_burnin, n_thinning, seed)
    "get_polytope_samples": [(20, 100, 4, 3), (64, 1000, 32, 0)],
}

# Approximate box decompositions (make_golden_mo.py): (m, n, seed, alphas).
MO_ALPHA_CASES = [
    (2, 20, 0, (0.0, 0.1)),
    (3, 25, 1, (0.0, 0.001, 0.05)),
    (3, 40, 2, (0.0, 0.01)),
    (4, 12, 3, (0.0, 0.01)),
]
