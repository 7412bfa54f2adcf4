"""LowerBound / UpperBound (reference modelling/layers/bound.py:28-59) on HIP.

forward: max(x, b) / min(x, b).  backward: the gradient passes where the input
is inside the bound or where it pushes the value back inside
(lower: x >= b or g < 0; upper: x <= b or g > 0)."""
import torch

from ...functional import BoundFn


def _bound_value(bound):
    if isinstance(bound, torch.Tensor):
        return float(bound.detach().cpu().reshape(-1)[0])
    return float(bound)


class LowerBound:
    """Use as the reference does: `LowerBound.apply(tensor, bound)`."""

    @staticmethod
    def apply(inputs, bound):
        return BoundFn.apply(inputs, _bound_value(bound), 0)


class UpperBound:
    @staticmethod
    def apply(inputs, bound):
        return BoundFn.apply(inputs, _bound_value(bound), 1)
