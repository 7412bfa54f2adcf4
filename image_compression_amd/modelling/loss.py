"""Distortion losses (reference modelling/loss.py:22-188) on HIP kernels.

MSE (nn.MSELoss with the configured reduction) and SSIM / MS-SSIM (11x11
Gaussian window = outer product of two 1-D Gaussians, valid filtering, 5-level
pyramid with reflect-pad + 2x2 average pooling)."""
import torch
import torch.nn as nn

from ..functional import MSEFn, SqDiffFn, msssim


def get_loss_dict(cfg, names):
    lcfg = cfg.MODEL.LOSS
    s = lcfg.SSIM
    ssim_kw = dict(max_val=s.MAX_VAL, filter_size=s.FILTER_SIZE, filter_sigma=s.FILTER_SIGMA,
                   k1=s.K1, k2=s.K2, log_scale=s.LOG_SCALE, eps=s.EPS)
    makers = {
        "MSE": lambda: MSELoss(reduction=lcfg.REDUCTION),
        "SSIMLoss": lambda: SSIMLoss(**ssim_kw),
        "MS_SSIMLoss": lambda: MS_SSIMLoss(**ssim_kw),
    }
    return {name: makers[name]() for name in names}


class MSELoss(nn.Module):
    def __init__(self, reduction="mean"):
        super().__init__()
        if reduction not in ("mean", "sum", "none"):
            raise ValueError(f"{reduction} is not a valid value for reduction")
        self.reduction = reduction

    def forward(self, input, target):
        if self.reduction == "none":
            return SqDiffFn.apply(input, target)
        m = MSEFn.apply(input, target)
        return m * input.numel() if self.reduction == "sum" else m


class SSIMLoss(nn.Module):
    """Single-scale SSIM loss: 1 - mean(ssim), or -log(ssim) per image (log_scale)."""

    def __init__(self, max_val=255., filter_size=11, filter_sigma=1.5, k1=0.01, k2=0.03,
                 log_scale=False, eps=1e-5):
        super().__init__()
        self.max_val, self.filter_size, self.filter_sigma = max_val, filter_size, filter_sigma
        self.k1, self.k2, self.log_scale, self.eps = k1, k2, log_scale, eps
        self.c1 = (k1 * max_val) ** 2
        self.c2 = (k2 * max_val) ** 2

    def forward(self, img1, img2):
        out = msssim(img1, img2, self, weights=[1.0], single_scale=True)
        return out


class MS_SSIMLoss(SSIMLoss):
    def __init__(self, max_val=255., filter_size=11, filter_sigma=1.5, k1=0.01, k2=0.03,
                 log_scale=False, eps=1e-5, weights=(0.0448, 0.2856, 0.3001, 0.2363, 0.1333)):
        super().__init__(max_val, filter_size, filter_sigma, k1, k2, log_scale, eps)
        self.weights = list(weights)

    def forward(self, img1, img2):
        return msssim(img1, img2, self, weights=self.weights, single_scale=False)
