"""Optimizer, LR schedules and the training step around the hot path
(SURVEY.md 8f row 1).

* `AdamW` — torch.optim.Optimizer subclass (same param_groups / state_dict
  format as torch.optim.AdamW, so reference checkpoints' optimizer state
  loads) whose step() is ONE native multi-tensor kernel (csrc/optim.hip) with
  the reference's clip_grad_value_ fused in.
* `make_optimizer(cfg, model)` — reference solver/optim.py:20-45: one group per
  parameter, weight decay WEIGHT_DECAY except WEIGHT_DECAY_BIAS (and lr x
  BIAS_LR_FACTOR) for names containing "bias"; eps = SOLVER.EPS.  Only "adamw"
  (what every reference config uses) runs natively; sgd / rmsprop raise.
* `make_lr_scheduler(cfg, optimizer, iters_per_epoch)` — reference
  solver/lr_scheduler.py:22-64 (constant, constant_warmup, cosine_warmup,
  decay_warmup, multistep_warmup); the LR is a host scalar, so these are
  LambdaLR schedules exactly like the reference's.
* `train_step(...)` — reference engine/trainer.py:163-209: forward, NaN guard,
  backward, clipped AdamW step, scheduler step, zero_grad.
"""
import math
from bisect import bisect_right

import torch
from torch.optim.lr_scheduler import LambdaLR

from . import _lib


class AdamW(torch.optim.Optimizer):
    """torch.optim.AdamW semantics (amsgrad=False, maximize=False) on the
    native multi-tensor kernel.  `clip_value` > 0 clamps every gradient to
    [-clip, clip] first (clip_grad_value_), in the same pass."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2, clip_value=0.0):
        if lr < 0 or eps < 0 or not (0 <= betas[0] < 1 and 0 <= betas[1] < 1) or weight_decay < 0:
            raise ValueError("invalid AdamW hyper-parameter")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.clip_value = float(clip_value)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        # one launch per (betas, eps, step) family; the reference builds all
        # groups with the same betas / eps, and every parameter steps together
        fams, stepped = {}, []
        for group in self.param_groups:
            for p in group["params"]:
                if p.grad is None:
                    continue
                _lib.require_device(p, p.grad)
                if p.grad.is_sparse or not p.is_contiguous() or not p.grad.is_contiguous():
                    raise RuntimeError("AdamW: dense contiguous parameters / gradients expected")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                stepped.append(p)
                key = (p.device, tuple(group["betas"]), group["eps"], int(st["step"].item()))
                fams.setdefault(key, []).append(
                    _lib.ICAdamWTensor(p.data_ptr(), p.grad.data_ptr(), st["exp_avg"].data_ptr(),
                                       st["exp_avg_sq"].data_ptr(), p.numel(), float(group["lr"]),
                                       float(group["weight_decay"])))
        for (dev, betas, eps, step), lst in fams.items():
            arr = (_lib.ICAdamWTensor * len(lst))(*lst)
            _lib.check(_lib.load().ic_adamw_step(arr, len(lst), float(betas[0]), float(betas[1]), float(eps),
                                                 self.clip_value, step,
                                                 _lib.c_void(torch.cuda.current_stream(dev).cuda_stream)),
                       "adamw_step")
        # the kernel writes the parameters behind autograd's back: bump their version counters as
        # an in-place torch op would (saved-tensor checks, functional.weight_cache)
        if stepped:
            torch.autograd.graph.increment_version(stepped)
        return loss


def make_optimizer(cfg, model, clip_value=None):
    """reference solver/optim.py:20-45 (adamw only)."""
    s = cfg.SOLVER
    if s.OPT_NAME != "adamw":
        raise NotImplementedError(f"optimizer {s.OPT_NAME!r}: only 'adamw' (every reference config) is native")
    params = []
    for key, value in model.named_parameters():
        if not value.requires_grad:
            continue
        lr = s.BASE_LR
        wd = s.WEIGHT_DECAY
        if "bias" in key:
            wd = s.WEIGHT_DECAY_BIAS
            lr = s.BASE_LR * s.BIAS_LR_FACTOR
        params.append({"params": [value], "lr": lr, "weight_decay": wd})
    clip = float(s.GRAD_CLIP) if clip_value is None else float(clip_value)
    return AdamW(params, s.BASE_LR, eps=s.EPS, clip_value=clip)


# ---------------------------------------------------------------- schedules
def _constant(_):
    return 1.0


def make_lr_scheduler(cfg, optimizer, num_iters_per_epoch=None):
    """reference solver/lr_scheduler.py:22-64."""
    c = cfg.SOLVER
    schedule = c.SCHEDULER_NAME
    if c.USE_ITER and schedule not in ("cosine_warmup", "constant"):
        raise AssertionError(f"iteration-based training supports cosine_warmup / constant, not {schedule}")
    if c.USE_ITER:
        n_train, n_warm = c.NUM_ITERS, c.WARMUP_ITERS
    else:
        n_train = (c.NUM_EPOCHS * num_iters_per_epoch) // c.GD_STEPS
        n_warm = (c.WARMUP_EPOCHS * num_iters_per_epoch) // c.GD_STEPS
    if schedule == "constant":
        return LambdaLR(optimizer, _constant)
    if schedule == "constant_warmup":
        return LambdaLR(optimizer, lambda s_: float(s_) / float(max(1.0, n_warm)) if s_ < n_warm else 1.0)
    if schedule == "cosine_warmup":
        cycles = c.NUM_COSINE_CYCLE

        def cosine(s_):
            if s_ < n_warm:
                return float(s_) / float(max(1, n_warm))
            progress = float(s_ - n_warm) / float(max(1, n_train - n_warm))
            return max(0.0, math.cos(math.pi * 2.0 * float(cycles) * progress))
        return LambdaLR(optimizer, cosine)
    if schedule == "decay_warmup":
        n_decay = (c.DECAY_EPOCHS * num_iters_per_epoch) // c.GD_STEPS
        gamma = c.DECAY_RATE

        def decay(s_):
            if s_ < n_warm:
                return float(s_) / float(max(1, n_warm))
            return gamma ** math.floor(s_ / n_decay)
        return LambdaLR(optimizer, decay)
    if schedule == "multistep_warmup":
        steps, gamma, wf, wi, wm = list(c.STEPS), c.GAMMA, c.WARMUP_FACTOR, c.WARMUP_ITERS, c.WARMUP_METHOD

        def multistep(s_):
            warm = 1.0
            if s_ < wi:
                if wm == "constant":
                    warm = wf
                elif wm == "linear":
                    a = float(s_) / wi
                    warm = wf * (1 - a) + a
            return warm * gamma ** bisect_right(steps, s_)
        return LambdaLR(optimizer, multistep)
    raise ValueError(f"unknown scheduler: {schedule}")


def train_step(model, optimizer, scheduler, imgs, gd_steps=1, it=0, nan_guard=True):
    """reference engine/trainer.py:163-209 (one iteration; returns (x_tilde, losses)).
    The reference exits on a NaN loss; here a RuntimeError is raised."""
    x_tilde, losses = model(imgs)
    loss = losses.pop("total_loss").mean() / gd_steps
    if nan_guard and bool(torch.isnan(loss).any()):
        raise RuntimeError("get nan loss")
    loss.backward()
    if it % gd_steps == 0:
        optimizer.step()        # clip_grad_value_ fused into the kernel
        if scheduler is not None:
            scheduler.step()
        optimizer.zero_grad()
    losses["total_loss"] = loss.detach()
    return x_tilde, losses
