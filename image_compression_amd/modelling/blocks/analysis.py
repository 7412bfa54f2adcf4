"""g_a (reference modelling/blocks/analysis.py:40-71): len(STRIDES) convs
(k x k, stride s, pad k//2), GDN after every conv but the last.
Init: xavier_normal_(gain sqrt 2), bias 0.01 — same RNG order as the reference."""
import math

import torch.nn as nn

from ..layers import GDN, Conv2d


class AnalysisTransform(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        strides = list(cfg.MODEL.STRIDES)
        k = cfg.MODEL.CONV_KERNEL
        n = len(strides)
        mods = []
        for i, s in enumerate(strides):
            cin = cfg.DATA.IN_CHANNELS if i == 0 else cfg.MODEL.INTER_CHANNELS
            cout = cfg.MODEL.LATENT_CHANNELS if i == n - 1 else cfg.MODEL.INTER_CHANNELS
            conv = Conv2d(cin, cout, k, stride=s, padding=k // 2)
            nn.init.xavier_normal_(conv.weight.data, math.sqrt(2))
            nn.init.constant_(conv.bias.data, 0.01)
            mods.append(conv)
            if i < n - 1:
                mods.append(GDN(cout))
        self.layers = nn.Sequential(*mods)

    def forward(self, x):
        return self.layers(x)
