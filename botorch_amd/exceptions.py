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
