"""Compressor2018 — Balle et al. 2018 scale hyperprior (reference
modelling/meta_arch/bmshl2018.py:49-110), every tensor op on HIP kernels.

forward(x) -> (x_tilde.detach(), losses) with losses =
{z_entropy, y_entropy, bpp, total_loss, <distortion names>}; only
total_loss carries grad."""
import os

import torch
import torch.nn as nn

from ... import noise as _noise
from ...functional import AbsFn, NonNegMultiFn, route_weight_gradients
from ..blocks import (ENTROPY_MODEL_REGISTRY, AnalysisTransform, HyperpriorAnalysisTransform,
                      HyperpriorSynthesisTransform, SynthesisTransform)
from ..layers import LowerBound, UpperBound
from ..loss import get_loss_dict
from .build import META_ARCH_REGISTRY


_SIDE = {}
_WGRAD = {}


class _StreamEdge(torch.autograd.Function):
    """Identity at a stream crossing.  Forward runs on the consumer stream of the value;
    backward (on that same stream) records the incoming gradient on `other`, the stream
    that consumes the gradient next, before handing it over."""

    @staticmethod
    def forward(ctx, t, other):
        ctx.other = other
        return t.view_as(t)

    @staticmethod
    def backward(ctx, g):
        if g is not None:
            g.record_stream(ctx.other)
        return g, None


def side_stream(device):
    """One side stream per device for the hyperprior branch, and beside it a stream for the
    hyperprior convs' weight gradients (functional: convs run on the side stream compute them there,
    off the chain of input gradients g_a's backward waits for).  Both at normal priority: a
    high-priority side stream dispatched its blocks ahead of the main stream's critical kernels
    whenever a CU freed up (C3 6.44 -> 6.35 ms per step at normal priority, C2 equal; r05s,
    profiles/r05s_side_priority_ab.txt)."""
    k = device.index if device.index is not None else torch.cuda.current_device()
    if k not in _SIDE:
        # IMGCOMP_SIDE_PRIORITY: stream priority of the two (0 normal, -1 high); diagnostic A/B knob
        prio = int(os.environ.get("IMGCOMP_SIDE_PRIORITY", "0"))
        _SIDE[k] = torch.cuda.Stream(device=device, priority=prio)
        _WGRAD[k] = torch.cuda.Stream(device=device, priority=prio)
        route_weight_gradients(_SIDE[k], _WGRAD[k])
    return _SIDE[k]


def wgrad_stream(device):
    """The stream the hyperprior convs' weight gradients run on (see side_stream)."""
    side_stream(device)
    return _WGRAD[device.index if device.index is not None else torch.cuda.current_device()]


@META_ARCH_REGISTRY.register()
class Compressor2018(nn.Module):
    def __init__(self, cfg):
        super().__init__()
        self.analysis_transform = AnalysisTransform(cfg)
        self.prior_analysis = HyperpriorAnalysisTransform(cfg)
        self.prior_synthesis = HyperpriorSynthesisTransform(cfg)
        self.synthesis_transform = SynthesisTransform(cfg)
        # The reference sizes the factorized model with LATENT_CHANNELS while z
        # carries INTER_CHANNELS (crash when they differ); z's
        # channel count is used here, identical whenever the reference runs.
        self.entropy_model = ENTROPY_MODEL_REGISTRY.get("EntropyModel")(cfg.MODEL.INTER_CHANNELS, cfg)
        self.conditional_model = ENTROPY_MODEL_REGISTRY.get(cfg.MODEL.ENTROPY_MODEL.CONDITIONAL_MODEL)(cfg)
        self.distortion_loss_fns = get_loss_dict(cfg, cfg.MODEL.LOSS.DISTORTION_LOSS_NAMES)
        self.distortion_loss_weight = cfg.MODEL.LOSS.DISTORTION_LOSS_WEIGHT
        self.loss_names = ["y_entropy", "z_entropy", "bpp"] + list(self.distortion_loss_fns.keys())
        # the hyperprior branch (h_a, factorized model, h_s, the y likelihood) on a second
        # stream, concurrent with the synthesis transform (see forward)
        self.concurrent_hyperprior = True

    def hyperprior_modules(self):
        """The modules whose forward, and so whose backward, run on the hyperprior side stream
        when concurrent_hyperprior is on (h_a, the factorized model, h_s, the conditional
        model): their parameters' gradients are produced on that stream (distributed.wrap)."""
        return [self.prior_analysis, self.entropy_model, self.prior_synthesis, self.conditional_model]

    def gradient_streams(self, device):
        """[(stream, parameters)]: the stream each hyperprior parameter's gradient is produced and
        accumulated on when concurrent_hyperprior is on -- the convs' weights and biases on the
        weight-gradient stream, the entropy models' parameters on the side stream (main-stream
        parameters are not listed).  distributed.wrap makes their AccumulateGrad nodes there."""
        convs = [p for blk in (self.prior_analysis, self.prior_synthesis) for m in blk.modules()
                 if isinstance(m, (nn.Conv2d, nn.ConvTranspose2d)) for p in m.parameters(recurse=False)]
        ids = {id(p) for p in convs}
        rest = [p for m in self.hyperprior_modules() for p in m.parameters() if id(p) not in ids]
        return [(wgrad_stream(device), convs), (side_stream(device), rest)]

    def _reparameterise_gdn(self, x):
        """Each main transform's GDN gamma / beta (NonNegativeParam) formed by one launch, their
        gradients by one more (functional.NonNegMultiFn), instead of two launches per parameter;
        every NonNegativeParam returns the value formed here at its next call.  Only with autograd
        on a device tensor (the eval weight cache keeps its own values)."""
        from ..layers.gdn import NonNegativeParam
        for blk in (self.analysis_transform, self.synthesis_transform):
            mods = [m for m in blk.modules() if isinstance(m, NonNegativeParam)]
            for m in mods:
                m.__dict__.pop("_pre", None)
            if mods and x.is_cuda and torch.is_grad_enabled():
                vals = NonNegMultiFn.apply([float(m.bound) for m in mods], [float(m.pedestal) for m in mods],
                                           *[m.param for m in mods])
                for m, v in zip(mods, vals):
                    m.__dict__["_pre"] = v

    def _clear_reparameterised(self):
        from ..layers.gdn import NonNegativeParam
        for blk in (self.analysis_transform, self.synthesis_transform):
            for m in blk.modules():
                if isinstance(m, NonNegativeParam):
                    m.__dict__.pop("_pre", None)

    def forward(self, x):
        # every GDN consumes its pre-formed value during the step; if the step raises first, none
        # may stay behind in the module (a stale value, and a graph kept alive by module state)
        try:
            return self._forward(x)
        finally:
            self._clear_reparameterised()

    def _forward(self, x):
        if self.training:
            _noise.begin_step(x.device)  # fresh Philox counters for this step
        self._reparameterise_gdn(x)
        N, _, H, W = x.shape
        num_pixels = N * H * W
        y = self.analysis_transform(x)
        cm = self.conditional_model
        # the split path calls cm.quantize / cm.likelihood instead of cm(y, sigma): with a
        # forward hook on cm (a caller observing its (q, p)) the call stays whole (serial)
        hooked = bool(cm._forward_hooks or cm._forward_pre_hooks or nn.modules.module._global_forward_hooks
                      or nn.modules.module._global_forward_pre_hooks)
        if self.concurrent_hyperprior and x.is_cuda and hasattr(cm, "quantize") and not hooked:
            # every tensor that crosses streams passes a _StreamEdge: its gradient, computed on
            # one stream and consumed on the other, is recorded on the consumer's stream, so the
            # caching allocator does not hand its memory to the producer stream's next
            # allocation while the consumer still reads it
            # y~ = y + noise (train) / round(y) (eval) does not depend on sigma, so the synthesis
            # transform need not wait for the hyperprior: the hyperprior branch and the y
            # likelihood run on a side stream while g_s runs here, and autograd runs their
            # backward on the same streams (the small hyperprior kernels hide under g_s's).
            # Same kernels, same draws in the same order (z, then y): bitwise the serial result.
            main = torch.cuda.current_stream(x.device)
            side = side_stream(x.device)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                y.record_stream(side)
                y_s = _StreamEdge.apply(y, main)
                z = self.prior_analysis(AbsFn.apply(y_s))
                z_tilde, _z_probs, z_ce = self.entropy_model(z)
                sigma = self.prior_synthesis(z_tilde)
            y_tilde = self.conditional_model.quantize(y)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                y_tilde.record_stream(side)
                y_probs = self.conditional_model.likelihood(_StreamEdge.apply(y_tilde, main), sigma)
                y_ce = self.conditional_model._ce_loss(y_probs)
            x_tilde = self.synthesis_transform(y_tilde)
            x_tilde = LowerBound.apply(UpperBound.apply(x_tilde, 1.), 0.)
            dist = self.distortion_loss(x, x_tilde)
            main.wait_stream(side)
            z_ce.record_stream(main)
            y_ce.record_stream(main)
            z_ce = _StreamEdge.apply(z_ce, side)
            y_ce = _StreamEdge.apply(y_ce, side)
        else:
            z = self.prior_analysis(AbsFn.apply(y))
            z_tilde, _z_probs, z_ce = self.entropy_model(z)
            sigma = self.prior_synthesis(z_tilde)
            y_tilde, y_probs = self.conditional_model(y, sigma)
            y_ce = self.conditional_model._ce_loss(y_probs)
            x_tilde = self.synthesis_transform(y_tilde)
            x_tilde = LowerBound.apply(UpperBound.apply(x_tilde, 1.), 0.)
            dist = self.distortion_loss(x, x_tilde)
        total_dist = sum(dist.values())
        entropy = (z_ce + y_ce) / num_pixels
        total = self.distortion_loss_weight * total_dist + entropy
        losses = {
            "z_entropy": z_ce.detach() / num_pixels,
            "y_entropy": y_ce.detach() / num_pixels,
            "bpp": entropy.detach(),
            "total_loss": total,
        }
        losses.update({k: v.detach() for k, v in dist.items()})
        return x_tilde.detach(), losses

    def distortion_loss(self, img1, img2):
        return {name: fn(img1, img2) for name, fn in self.distortion_loss_fns.items()}

    def compress(self, x):
        """Stub in the reference (bmshl2018.py:106-107): no entropy coder."""
        return None

    def decompress(self, x):
        return None
