"""Entropy bottleneck (reference modelling/blocks/entropy_model.py).

EntropyModel (factorized prior on z, :188-269) and the symmetric conditional
models on y (:272-378).  Noise/round + likelihood run in fused HIP kernels
(csrc/entropy.hip): the factorized CDF MLP (1->3->3->3->1 per channel, softplus
weights, tanh gates) is evaluated twice per element in registers, and the
per-channel parameter gradients are deterministic block reductions.  Other
cfg.MODEL.ENTROPY_MODEL.DIMS and any BIN run the generic kernels
(ic_factorized_*_net, ic_conditional_*_bin): up to 5 hidden layers of width <= 8
with the activations in registers, larger nets (up to 31 hidden layers of width
<= 256) with them in a workspace.
"""
import math

import torch
import torch.nn as nn
import torch.nn.functional as F

from ... import noise as _noise
from ...functional import CELossFn, conditional, conditional_likelihood, factorized, quantize
from .build import ENTROPY_MODEL_REGISTRY

LOG2 = math.log(2.0)


class CDFLayer(nn.Module):
    """One per-channel affine(+gate) layer (entropy_model.py:47-78).
    Parameter shapes and init order match the reference (weight constant
    ln(expm1(1/scale/out)), bias U(-1/2, 1/2), factor 0)."""

    def __init__(self, channels, in_dim, out_dim, init_scale, act=True):
        super().__init__()
        self.act = act
        w0 = math.log(math.expm1(1.0 / init_scale / out_dim))
        self.weight = nn.Parameter(nn.init.constant_(torch.empty(1, channels, out_dim, in_dim), w0))
        self.bias = nn.Parameter(nn.init.uniform_(torch.empty(1, channels, out_dim, 1), -0.5, 0.5))
        if act:
            self.factor = nn.Parameter(nn.init.zeros_(torch.empty(1, channels, out_dim, 1)))

    def forward(self, x):
        # auxiliary API (the hot path evaluates the whole MLP in one kernel)
        x = torch.matmul(F.softplus(self.weight), x) + self.bias
        return x + torch.tanh(x) * torch.tanh(self.factor) if self.act else x


class CDFEstimator(nn.Module):
    """Per-channel monotone CDF logits (entropy_model.py:81-114)."""

    def __init__(self, channels, dims=(3, 3, 3), init_scale=10.):
        super().__init__()
        dims = [1] + list(dims) + [1]  # the reference inserts into the cfg list in place
        n = len(dims) - 1
        scale = init_scale ** (1 / n)
        self.layers = nn.Sequential(*[CDFLayer(channels, dims[i], dims[i + 1], scale, i < n - 1)
                                      for i in range(n)])
        self.dims = dims

    def forward(self, x):
        # auxiliary API; returns the reference's layout (see EntropyModel._ref_layout)
        N, C = x.shape[:2]
        order = [0] + list(range(2, x.dim())) + [1]
        h = x.permute(*order).reshape(-1, C, 1, 1)
        h = self.layers(h)
        return h.view(N, *x.shape[2:], C).permute(*order)

    def flat_params(self):
        out = []
        for i, layer in enumerate(self.layers):
            out += [layer.weight, layer.bias]
            if layer.act:
                out.append(layer.factor)
        return out


class BaseEntropyModel(nn.Module):
    """entropy_model.py:117-185."""

    def _prob_mass(self, x):
        raise NotImplementedError("to be inherited")

    def _quantize(self, x, mode):
        raise NotImplementedError()

    def _dequantize(self, x):
        raise NotImplementedError()

    def compress(self, x):
        raise NotImplementedError()

    def decompress(self, x):
        raise NotImplementedError()

    def _ce_loss(self, probs):
        """sum clamp(-log2(p + 1e-10), 0, 50) — deterministic HIP reduction."""
        return CELossFn.apply(probs)


def _ref_layout(p):
    """The reference re-permutes the CDF output with the forward permutation
    instead of its inverse (entropy_model.py:108-113): for (N, C, H, W) the
    probabilities come back as (N, W, C, H), p_ref[n, w, c, h] = p[n, c, h, w].
    Reproduced as a zero-copy view so parity holds on the returned tensor."""
    order = [0] + list(range(2, p.dim())) + [1]
    return p.movedim(1, -1).permute(*order)


@ENTROPY_MODEL_REGISTRY.register()
class EntropyModel(BaseEntropyModel):
    def __init__(self, in_channels, cfg):
        super().__init__()
        em = cfg.MODEL.ENTROPY_MODEL
        self._cdf_estimator = CDFEstimator(in_channels, em.DIMS, em.INIT_SCALE)
        self.bin = em.BIN

    def forward(self, x):
        u = _noise.pop_injected() if self.training else None
        q, p = factorized(x, self._cdf_estimator.flat_params(), self.training, u, self._cdf_estimator.dims, self.bin)
        probs = _ref_layout(p)
        return q, probs, self._ce_loss(probs)

    def _logit_cumulative(self, x):
        return self._cdf_estimator(x)


class SymmetricConditionalModel(BaseEntropyModel):
    """entropy_model.py:272-352; subclasses pick the standardized CDF."""
    KIND = None

    def __init__(self, cfg):
        super().__init__()
        self.bin = cfg.MODEL.ENTROPY_MODEL.BIN

    def quantize(self, x):
        """_quantize on its own (train: noise, eval: round): with likelihood() the two halves of
        forward(), which Compressor2018 runs apart so the hyperprior can run meanwhile."""
        u = _noise.pop_injected() if self.training else None
        return quantize(x, self.training, u, self.bin)

    def likelihood(self, q, scale):
        """_prob_mass of already-quantized q (mean 0)."""
        return conditional_likelihood(q, scale.expand_as(q), None, self.KIND, self.bin)

    def forward(self, x, scale, mean=0):
        if isinstance(mean, torch.Tensor):
            mean_t = mean.expand_as(x)
        elif mean == 0:
            mean_t = None
        else:
            mean_t = torch.full_like(x, float(mean))
        u = _noise.pop_injected() if self.training else None
        return conditional(x, scale.expand_as(x), mean_t, self.KIND, self.training, u, self.bin)


@ENTROPY_MODEL_REGISTRY.register()
class GaussianConditionalModel(SymmetricConditionalModel):
    """Normal(0,1) CDF (entropy_model.py:355-365)."""
    KIND = 1


@ENTROPY_MODEL_REGISTRY.register()
class LaplacianConditionalModel(SymmetricConditionalModel):
    """Laplace(0,1) CDF (entropy_model.py:368-378) — the default (config.py:70)."""
    KIND = 0
