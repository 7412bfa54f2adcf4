"""ShapeSpec (reference modelling/layers/shape_spec.py:23-37): keyword-only
record of (channels, height, width, stride); exported, unused by the model."""
from typing import NamedTuple, Optional


class _Spec(NamedTuple):
    channels: Optional[int]
    height: Optional[int]
    width: Optional[int]
    stride: Optional[int]


class ShapeSpec(_Spec):
    def __new__(cls, *, channels=None, height=None, width=None, stride=None):
        return super().__new__(cls, channels, height, width, stride)
