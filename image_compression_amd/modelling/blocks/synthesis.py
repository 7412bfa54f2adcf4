"""g_s (reference modelling/blocks/synthesis.py:40-71): transposed convs
(k x k, stride s, pad k//2, output_padding s-1) with forward GDN (inverse=False,
as the reference builds it, synthesis.py:65) after every layer but the last."""
import math

import torch.nn as nn

from ..layers import GDN, ConvTranspose2d


class SynthesisTransform(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        strides = list(cfg.MODEL.STRIDES)
        k = cfg.MODEL.CONV_KERNEL
        n = len(strides)
        mods = []
        for i, s in enumerate(strides):
            cin = cfg.MODEL.LATENT_CHANNELS if i == 0 else cfg.MODEL.INTER_CHANNELS
            cout = cfg.DATA.IN_CHANNELS if i == n - 1 else cfg.MODEL.INTER_CHANNELS
            conv = ConvTranspose2d(cin, cout, k, stride=s, padding=k // 2, output_padding=s - 1)
            nn.init.xavier_normal_(conv.weight.data, math.sqrt(2))
            nn.init.constant_(conv.bias.data, 0.01)
            mods.append(conv)
            if i < n - 1:
                mods.append(GDN(cout))
        self.layers = nn.Sequential(*mods)

    def forward(self, x):
        return self.layers(x)
