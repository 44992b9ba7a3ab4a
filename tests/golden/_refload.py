"""Load gpytorch-free leaf modules of the reference BoTorch (fixture generation only).

`import botorch` fails in this container (gpytorch/linear_operator absent), so
parent packages are registered as empty namespace modules whose ``__path__``
points into the reference tree; only leaf modules that import nothing from
gpytorch are then imported normally.  Used ONLY by ``make_golden.py`` in the
development container -- never on the GPU box, never by the product.
"""
import importlib
import os
import sys
import types

REF = os.environ.get("BOTORCH_REF", "/root/reference")

_STUB_PACKAGES = [
    "botorch",
    "botorch.utils",
    "botorch.utils.probability",
    "botorch.utils.multi_objective",
    "botorch.utils.multi_objective.box_decompositions",
    "botorch.sampling",
    "botorch.test_functions",
    "botorch.optim",
]


def install():
    for name in _STUB_PACKAGES:
        if name in sys.modules:
            continue
        mod = types.ModuleType(name)
        mod.__path__ = [os.path.join(REF, *name.split("."))]
        sys.modules[name] = mod


def load(name):
    install()
    return importlib.import_module(name)
