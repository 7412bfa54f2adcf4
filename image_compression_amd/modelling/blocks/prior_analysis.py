"""h_a (reference modelling/blocks/prior_analysis.py:39-71): conv -> ReLU ->
conv -> ReLU -> conv (last conv without bias), kernels/strides from
MODEL.HYPER_PRIOR.  Applied to |y| by the meta-architecture."""
import math

import torch.nn as nn

from ..layers import Conv2d, ReLU


class HyperpriorAnalysisTransform(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        hp = cfg.MODEL.HYPER_PRIOR
        n = len(hp.STRIDES)
        mods = []
        for i, (s, k) in enumerate(zip(hp.STRIDES, hp.KERNELS)):
            last = i == n - 1
            cin = cfg.MODEL.LATENT_CHANNELS if i == 0 else cfg.MODEL.INTER_CHANNELS
            conv = Conv2d(cin, cfg.MODEL.INTER_CHANNELS, k, stride=s, padding=k // 2, bias=not last)
            nn.init.xavier_normal_(conv.weight.data, math.sqrt(2))
            if not last:
                nn.init.constant_(conv.bias.data, 0.01)
            mods.append(conv)
            if not last:
                mods.append(ReLU())
        self._layers = nn.Sequential(*mods)

    def forward(self, x):
        return self._layers(x)
