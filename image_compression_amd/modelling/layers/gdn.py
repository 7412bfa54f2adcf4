"""GDN / IGDN / RGDN (reference modelling/layers/gdn.py:42-88) on HIP.

y = x / sqrt(beta + conv1x1(x^2, gamma))   (inverse: x * sqrt(...); relu: ReLU first)
gamma, beta are re-parameterised by NonNegativeParam: max(p, bound)^2 - pedestal.
The 1x1 "conv" is a CxC GEMM with x^2 formed in the operand load and the x * norm^-1/2
epilogue fused (csrc/gdn_fused.hip): in the default fp32_split arithmetic the forward is
gdn_fwd_x3s_kernel (Gamma x^2 on the bf16 MFMA through the exact three-term split) and the
backward gdn_bwd_fused_kernel<C, true> (split dGamma GEMM, fp32-MFMA dx GEMM, dbeta and the
producing conv's bias column sums in the same pass); COMPUTE_DTYPE "fp32" runs the fp32-MFMA
forms, and shapes outside the fused kernels' layouts the generic csrc/gdn.hip kernels."""
import torch
import torch.nn as nn

from ...functional import GDNFn, NonNegFn, ReLUFn, nonneg_cached


class NonNegativeParam(nn.Module):
    """reference gdn.py:42-62.  `pedestal`/`bound` are plain attributes (not
    buffers), so the state dict holds only `param`, as in the reference."""

    def __init__(self, init_val, minimum=0, offset=2 ** (-18)):
        super().__init__()
        ped = torch.tensor(float(offset) ** 2)           # fp32, like the reference
        self.pedestal = ped
        self.bound = (float(minimum) + ped.clone().detach() ** 2) ** 0.5
        self.param = nn.Parameter(torch.sqrt(torch.max(init_val + ped, ped)))

    def forward(self):
        pre = self.__dict__.pop("_pre", None)  # this step's value, formed with its siblings' (see
        if pre is not None:                    # Compressor2018: one NonNegMultiFn per transform)
            return pre
        return nonneg_cached(self.param, float(self.bound), float(self.pedestal))


class GDN(nn.Module):
    math = 0       # IC_MATH_*: 2 forms the backward's dgamma in split arithmetic (C = 192; set_compute_dtype)
    math_fwd = 0   # IC_MATH_*: 2 runs the forward in split arithmetic (fused kernel at C = 192; set_compute_dtype)
    xb = 0         # bf16 operands (C3): 1 writes y's bf16 copy for the next conv, 2 dx's for the previous
                   # transposed conv's input gradient (functional._put_bf16; set_compute_dtype)

    def __init__(self, in_channels, inverse=False, relu=False,
                 gamma_init=0.1, beta_min=1e-6, offset=2 ** -18):
        super().__init__()
        self.inverse = inverse
        self.relu = relu
        # the reference builds both parameters with NonNegativeParam's default
        # offset (its `offset` argument is accepted but unused, gdn.py:69-74)
        eye = torch.eye(in_channels).view(in_channels, in_channels, 1, 1)
        self.gamma = NonNegativeParam(eye * gamma_init)
        self.beta = NonNegativeParam(torch.ones((in_channels,)), minimum=beta_min)

    def forward(self, x):
        if self.relu:
            x = ReLUFn.apply(x)
        return GDNFn.apply(x, self.gamma(), self.beta(), bool(self.inverse), int(self.math), int(self.math_fwd),
                           int(self.xb))
