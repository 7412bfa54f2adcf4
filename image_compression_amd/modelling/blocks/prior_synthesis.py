"""h_s (reference modelling/blocks/prior_synthesis.py:40-72): transposed convs
with the hyper-prior kernels/strides reversed, ReLU between, then
sigma = clamp(exp(.), 1e-10, 1e10)."""
import math

import torch.nn as nn

from ...functional import ExpClampFn
from ..layers import ConvTranspose2d, ReLU


class HyperpriorSynthesisTransform(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        hp = cfg.MODEL.HYPER_PRIOR
        n = len(hp.STRIDES)
        mods = []
        for i, (s, k) in enumerate(zip(reversed(list(hp.STRIDES)), reversed(list(hp.KERNELS)))):
            cout = cfg.MODEL.INTER_CHANNELS if i < n - 1 else cfg.MODEL.LATENT_CHANNELS
            conv = ConvTranspose2d(cfg.MODEL.INTER_CHANNELS, cout, k, stride=s, padding=k // 2,
                                   bias=True, output_padding=s - 1)
            nn.init.xavier_normal_(conv.weight.data, math.sqrt(2))
            nn.init.constant_(conv.bias.data, 0.01)
            mods.append(conv)
            if i < n - 1:
                mods.append(ReLU())
        self._layers = nn.Sequential(*mods)

    def forward(self, x):
        return ExpClampFn.apply(self._layers(x), 1e-10, 1e10)
