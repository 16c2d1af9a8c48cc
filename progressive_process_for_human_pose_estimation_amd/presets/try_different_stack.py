"""Drop-in for the reference's `try_different_stack.py` model: the progressive 3-stack heads of
try_with_aspp (background CE -> skeleton CE -> keypoint MSE, concat re-injection,
try_different_stack.py:282-330) on the PRIMARY hourglass (with the innermost residual chain,
:245-262, and no ASPP registrations)."""
from .. import modules as _m
from ..modules import ResidualBlock, hourglass, lin  # noqa: F401  (reference names)
from . import try_with_aspp as _aspp


class creatModel(_aspp.creatModel):  # noqa: N801
    _hourglass_cls = _m.hourglass
