"""Error / warning taxonomy mirrored from the reference.

botorch/exceptions/errors.py:34-50 and [G] linear_operator.utils.errors
(NotPSDError, NanError), botorch/exceptions/warnings.py:13-109.
"""


class BotorchError(Exception):
    pass


class UnsupportedError(BotorchError):
    pass


class InputDataError(BotorchError):
    pass


class NotPSDError(RuntimeError):
    """[G] linear_operator NotPSDError: Cholesky failed after the jitter ladder."""


class NanError(RuntimeError):
    """[G] linear_operator NanError (also raised by utils/low_rank.py:163-172)."""


class BotorchWarning(Warning):
    pass


class NumericalWarning(RuntimeWarning):
    """[G] linear_operator NumericalWarning (emitted when jitter is added)."""


class OptimizationWarning(BotorchWarning):
    pass


class InputDataWarning(BotorchWarning):
    pass


class ModelFittingError(Exception):
    """botorch/exceptions/errors.py ModelFittingError: every fit attempt of
    fit_gpytorch_mll failed (fit.py:255-259)."""


class OptimizationTimeoutError(BotorchError):
    """botorch/exceptions/errors.py OptimizationTimeoutError: raised inside the
    scipy callback when ``timeout_sec`` is exceeded (optim/utils/timeout.py:49-53)
    and turned into a "timed out" OptimizeResult by minimize_with_timeout."""

    def __init__(self, *args, current_x=None, runtime: float = 0.0):
        super().__init__(*args)
        self.current_x = current_x
        self.runtime = runtime


class BadInitialCandidatesWarning(RuntimeWarning):
    """botorch/exceptions/warnings.py BadInitialCandidatesWarning."""


class CandidateGenerationError(BotorchError):
    """botorch/exceptions/errors.py CandidateGenerationError: e.g. a linear
    constraint left without free variables by fixed features is violated
    (optim/parameter_constraints.py:448-454)."""


class UserInputWarning(BotorchWarning):
    """botorch/exceptions/warnings.py UserInputWarning."""
