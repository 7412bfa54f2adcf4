"""Conv2d / ConvTranspose2d / ReLU modules whose forward runs the HIP kernels.

They subclass the torch modules only for parameter shapes, default
initialisation (same RNG consumption as the reference's nn.Conv2d /
nn.ConvTranspose2d, so `torch.manual_seed(s); build_model(cfg)` reproduces the
reference's weights) and state-dict keys (`weight`, `bias`)."""
import torch.nn as nn

from ...functional import ReLUFn, conv2d, conv_transpose2d


def _square(v, what):
    if isinstance(v, (tuple, list)):
        if len(set(v)) != 1:
            raise NotImplementedError(f"non-square {what} {v}")
        return int(v[0])
    return int(v)


class Conv2d(nn.Conv2d):
    math = 0   # IC_MATH_*: 0 fp32, 1 bf16 operands / fp32 accumulation (set_compute_dtype)

    def __init__(self, *args, **kw):
        super().__init__(*args, **kw)
        if self.groups != 1 or _square(self.dilation, "dilation") != 1 or self.padding_mode != "zeros":
            raise NotImplementedError("imgcomp Conv2d: groups=1, dilation=1, zero padding only")
        _square(self.kernel_size, "kernel")

    def forward(self, x):
        return conv2d(x, self.weight, self.bias, _square(self.stride, "stride"), _square(self.padding, "padding"),
                      math=self.math)


class ConvTranspose2d(nn.ConvTranspose2d):
    math = 0

    def __init__(self, *args, **kw):
        super().__init__(*args, **kw)
        if self.groups != 1 or _square(self.dilation, "dilation") != 1:
            raise NotImplementedError("imgcomp ConvTranspose2d: groups=1, dilation=1 only")
        _square(self.kernel_size, "kernel")

    def forward(self, x, output_size=None):
        if output_size is not None:
            raise NotImplementedError("output_size is not supported; use output_padding")
        return conv_transpose2d(x, self.weight, self.bias, _square(self.stride, "stride"),
                                _square(self.padding, "padding"), _square(self.output_padding, "output_padding"),
                                math=self.math)


class ReLU(nn.ReLU):
    def forward(self, x):
        return ReLUFn.apply(x)
