"""Evaluation around the hot path: the reference's
Kodak evaluator and its metrics, on HIP kernels.

* `psnr(a, b)` — utils/metric.py:26-36, per image, dB (ic_psnr).
* `ms_ssim_db(a, b)` — utils/metric.py:100-138 MS_SSIM(in_dB=True): per image,
  non-negative SSIM/CS means, product of powers, -10 log10(1 - .) (the
  MS-SSIM kernels of the loss, ic_msssim_fwd mode single = 2).
  Both take images in [0,1] and score them at max_val = 255, as
  engine/monitor.py:113-121 does (x, x~ multiplied by 255 first).
* `Monitor` — engine/monitor.py: per-name AverageMeter for losses and
  BatchAverageMeter (per-image mean) for metrics.
* `Evaluator.run_eval(batches)` — engine/evaluator.py:67-105: eval mode,
  no_grad, forward, drop total_loss, update metrics and losses; returns the
  mean results dict {psnr, ms_ssim, bpp, y_entropy, z_entropy, <distortion>};
  `graph=True` replays a hipGraph-captured forward per input shape (`GraphForward`).
"""
import contextlib
import ctypes

import torch

from . import _lib
from . import functional as F

MS_SSIM_WEIGHTS = (0.0448, 0.2856, 0.3001, 0.2363, 0.1333)


def psnr(a, b, max_val=255.0):
    """Per-image PSNR in dB of images a, b in [0,1] scored at `max_val`."""
    _lib.require_device(a, b)
    a, b = a.contiguous(), b.contiguous()
    if a.shape != b.shape:
        raise RuntimeError(f"psnr: shape mismatch {tuple(a.shape)} vs {tuple(b.shape)}")
    N = a.shape[0]
    L = _lib.load()
    per = a.numel() // N
    out = torch.empty(N, device=a.device, dtype=torch.float32)
    nb = L.ic_psnr_ws(N, per)
    buf = _lib.workspace(nb, a.device)
    _lib.check(L.ic_psnr_ex(_lib.ptr(a), _lib.ptr(b), N, per, float(max_val), _lib.ptr(out), _lib.ptr(buf), nb,
                            _lib.stream_of(a)), "psnr")
    return out


def ms_ssim_db(a, b, max_val=255.0, filter_size=11, filter_sigma=1.5, k1=0.01, k2=0.03, weights=MS_SSIM_WEIGHTS):
    """Per-image MS-SSIM in dB (the reference's evaluation metric)."""
    _lib.require_device(a, b)
    L = _lib.load()
    a, b = a.contiguous(), b.contiguous()
    N, C, H, W = a.shape
    nlev = len(weights)
    sb = L.ic_msssim_state_bytes(N, C, H, W, nlev, filter_size)
    if sb == 0:
        raise RuntimeError(f"ms-ssim: image {H}x{W} too small for {nlev} levels")
    state = torch.empty(sb // 4, device=a.device, dtype=torch.float32)
    nb = L.ic_msssim_ws(N, C, H, W, nlev, filter_size)
    buf = _lib.workspace(nb, a.device)
    wts = (ctypes.c_float * nlev)(*weights)
    out = torch.empty(N, device=a.device, dtype=torch.float32)
    _lib.check(L.ic_msssim_fwd(_lib.ptr(a), _lib.ptr(b), N, C, H, W, nlev, filter_size, float(filter_sigma),
                               float(max_val), 0, 2, float(k1), float(k2), 0.0, ctypes.cast(wts, ctypes.c_void_p),
                               _lib.ptr(out), _lib.ptr(state), _lib.ptr(buf), nb, _lib.stream_of(a)), "msssim_metric")
    return out


class AverageMeter:
    """utils/logging.py AverageMeter (cache=False): running mean of per-call values."""

    def __init__(self):
        self.reset()

    def reset(self):
        self.val, self.sum, self.count = 0.0, 0.0, 0

    def update(self, val, n=1):
        self.val = float(val)
        self.sum += float(val) * n
        self.count += n

    @property
    def avg(self):
        return self.sum / max(self.count, 1)


class BatchAverageMeter(AverageMeter):
    """utils/logging.py BatchAverageMeter: a batch of per-item values counts each item."""

    def update(self, vals):
        v = vals.detach().double().cpu().reshape(-1)
        self.val = float(v.mean())
        self.sum += float(v.sum())
        self.count += v.numel()


class Monitor:
    """engine/monitor.py:25-184 (the parts evaluation uses)."""

    def __init__(self, loss_names, metric_dict=None):
        self.metric_fns = metric_dict or {"psnr": psnr, "ms_ssim": ms_ssim_db}
        self.loss_names = list(loss_names)
        self.meters = {n: AverageMeter() for n in self.loss_names}
        self.metrics = {n: BatchAverageMeter() for n in self.metric_fns}
        self.results = None

    def reset(self):
        for m in list(self.meters.values()) + list(self.metrics.values()):
            m.reset()
        self.results = None

    def update_loss(self, **losses):
        for k, v in losses.items():
            self.meters[k].update(v)

    def update_metric(self, preds, targets):
        """preds, targets in [0,1]; metrics are scored at max_val 255 (monitor.py:118-121)."""
        for name, fn in self.metric_fns.items():
            self.metrics[name].update(fn(preds, targets))

    def eval(self):
        self.results = {k: m.avg for k, m in self.metrics.items()}
        self.results.update({k: m.avg for k, m in self.meters.items()})
        return self.results


class GraphForward:
    """The eval-mode forward (model.eval(): rounding instead of noise) captured once into a
    hipGraph for one input shape and replayed per batch: the reference's Kodak evaluator runs
    batch-1 512x768 forwards (engine/evaluator.py:87-105), ~100 launches each, many of them on
    the 8x12..32x48 hyperprior maps where a launch costs more than its work.  `x_tilde` and
    `losses` are the graph's static outputs, overwritten by the next call.  The hyperprior side
    stream joins the capture (it forks from and rejoins the capture stream)."""

    def __init__(self, model, example_x, warmup=2):
        if not example_x.is_cuda:
            raise RuntimeError("GraphForward needs a ROCm device tensor")
        self.model = model
        self.x = example_x.detach().clone()
        dev = self.x.device
        was_training = model.training
        model.eval()
        try:
            with torch.no_grad():
                side = torch.cuda.Stream(dev)
                side.wait_stream(torch.cuda.current_stream(dev))
                with torch.cuda.stream(side):
                    for _ in range(warmup):  # allocator pools warm, kernels loaded
                        model(self.x)
                torch.cuda.current_stream(dev).wait_stream(side)
                self.graph = torch.cuda.CUDAGraph()
                with torch.cuda.graph(self.graph):
                    self.x_tilde, self.losses = model(self.x)
        finally:
            model.train(was_training)

    def __call__(self, x):
        self.x.copy_(x)
        self.graph.replay()
        return self.x_tilde, self.losses


class Evaluator:
    """engine/evaluator.py:44-123 without the data loader / file outputs:
    run_eval(batches) over an iterable of [N,3,H,W] images in [0,1].  graph=True replays one
    captured forward per input shape (GraphForward) instead of launching it eagerly;
    weight_cache=False re-packs the weights on every eager forward (functional.weight_cache)."""

    def __init__(self, model, device=None, graph=False, weight_cache=True):
        self.model = model
        self.device = device
        self.monitor = Monitor(model.loss_names)
        self.graph = graph
        self.weight_cache = weight_cache
        self._graphs = {}
        self._graph_ptrs = None

    def _forward(self, imgs):
        if not (self.graph and imgs.is_cuda):
            return self.model(imgs)
        # a captured graph holds raw device pointers to the parameters and buffers: if any of
        # them was reallocated since capture (load_state_dict(assign=True), .to(...), a rebuilt
        # module), replay would read freed memory, so the graphs are dropped and recaptured
        ptrs = tuple(t.data_ptr() for t in list(self.model.parameters()) + list(self.model.buffers()))
        if ptrs != self._graph_ptrs:
            self._graphs.clear()
            self._graph_ptrs = ptrs
        key = (tuple(imgs.shape), imgs.device)
        g = self._graphs.get(key)
        if g is None:
            g = self._graphs[key] = GraphForward(self.model, imgs)
        x_tilde, losses = g(imgs)
        return x_tilde, dict(losses)

    @torch.no_grad()
    def run_eval(self, batches):
        was_training = self.model.training
        self.model.eval()
        self.monitor.reset()
        # eager forwards reuse the weight packs and GDN re-parameterisations across images (the
        # weights are constant here); captured graphs hold their launches already
        scope = F.weight_cache() if (self.weight_cache and not self.graph) else contextlib.nullcontext()
        try:
            with scope:
                for imgs in batches:
                    if self.device is not None:
                        imgs = imgs.to(self.device, non_blocking=True)
                    x_tilde, losses = self._forward(imgs)
                    losses.pop("total_loss")
                    self.monitor.update_metric(x_tilde, imgs)
                    self.monitor.update_loss(**losses)
        finally:
            self.model.train(was_training)
        return self.monitor.eval()
