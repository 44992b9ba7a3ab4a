"""Global flags of the reference (botorch/settings.py), mirrored for the path.

``propagate_grads`` (settings.py:44): in the reference it switches
[G] detach_test_caches off inside gpt_posterior_settings
(models/utils/assorted.py:286-298), so posterior gradients reach the training
data through the prediction caches (fantasy models, knowledge gradient).  The
prediction caches here are built by bo::gp_cache without a backward to the
training data; with the flag on and training data that require grad, the
posterior raises UnsupportedError instead of silently detaching them.  With
the flag on and no such training data it has, as in the reference, no effect.
``debug`` and ``validate_input_scaling`` keep the reference's switch semantics.
"""
from __future__ import annotations


class _Flag:
    """settings.py:16-42: a class-level boolean, set for the duration of a
    ``with`` block."""

    _state: bool = False

    @classmethod
    def on(cls) -> bool:
        return cls._state

    @classmethod
    def off(cls) -> bool:
        return not cls._state

    @classmethod
    def _set_state(cls, state: bool) -> None:
        cls._state = state

    def __init__(self, state: bool = True) -> None:
        self.prev = self.__class__.on()
        self.state = state

    def __enter__(self) -> None:
        self.__class__._set_state(self.state)

    def __exit__(self, *args) -> None:
        self.__class__._set_state(self.prev)


class propagate_grads(_Flag):
    """Propagate posterior gradients to the training inputs / targets."""

    _state: bool = False


class debug(_Flag):
    """Verbose warnings."""

    _state: bool = False


class validate_input_scaling(_Flag):
    """Validate train_X in the unit cube and standardized train_Y at model
    construction (settings.py:64-77)."""

    _state: bool = True
