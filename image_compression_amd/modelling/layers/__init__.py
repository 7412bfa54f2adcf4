from .shape_spec import ShapeSpec
from .gdn import GDN, NonNegativeParam
from .bound import UpperBound, LowerBound
from .conv import Conv2d, ConvTranspose2d, ReLU
