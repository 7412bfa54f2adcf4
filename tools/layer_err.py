"""Per-layer error of every conv / transposed conv of one Compressor2018
training step, on the real activations and gradients of that step: each
layer's forward, input gradient and weight gradient are recomputed alone in
each math mode and compared with fp64 torch (CPU).  The 'cancel' column is
||sum |a||b| || / ||sum a b|| of the weight gradient, the factor by which
cancellation magnifies a per-product error.

usage: python tools/layer_err.py --n 16 --size 256 [--prefix prior_]
"""
import argparse
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--prefix", default="")
    a = ap.parse_args()
    from image_compression_amd import get_cfg_defaults, injected_noise, modelling, _lib
    from image_compression_amd import functional as IF
    from image_compression_amd.modelling.layers import Conv2d, ConvTranspose2d
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    cfg = get_cfg_defaults()
    cfg.MODEL.LOSS.REDUCTION = "mean"
    cfg.MODEL.LOSS.DISTORTION_LOSS_WEIGHT = 256.0
    torch.manual_seed(0)
    model = modelling.build_model(cfg).cuda().train()
    caps = {}

    def fhook(name):
        def f(mod, inp, out):
            caps[name] = {"x": inp[0].detach().clone(), "mod": mod}
            out.register_hook(lambda g: caps[name].__setitem__("gy", g.detach().clone()))
        return f

    for name, m in model.named_modules():
        if isinstance(m, (Conv2d, ConvTranspose2d)) and name.startswith(a.prefix):
            m.register_forward_hook(fhook(name))
    g = torch.Generator().manual_seed(3)
    N, S = a.n, a.size
    x = torch.rand(N, 3, S, S, generator=g)
    uz = torch.rand(N, 192, S // 64, S // 64, generator=g)
    uy = torch.rand(N, 192, S // 16, S // 16, generator=g)
    with injected_noise([uz.cuda(), uy.cuda()]):
        _, losses = model(x.cuda())
    losses["total_loss"].backward()
    torch.cuda.synchronize()
    print(f"{'layer':34s} {'math':4s} {'kernel(fwd/dgrad/wgrad)':44s} {'y':>9s} {'dx':>9s} {'dW':>9s} {'cancel':>8s} {'sum dx':>9s} {'cancel':>8s}")
    for name, c in caps.items():
        mod = c["mod"]
        tr = isinstance(mod, ConvTranspose2d)
        xx = c["x"].float()
        gy = c["gy"].float()
        w = mod.weight.detach()
        s, p = mod.stride[0], mod.padding[0]
        k = w.shape[-1]
        xr = xx.double().cpu().requires_grad_(True)
        wr = w.double().cpu().requires_grad_(True)
        if tr:
            op = mod.output_padding[0]
            yr = F.conv_transpose2d(xr, wr, None, s, p, op)
        else:
            yr = F.conv2d(xr, wr, None, s, p)
        yr.backward(gy.double().cpu())
        # cancellation of the weight gradient: the same sum over |x| |gy|
        xa = xr.detach().abs()
        ga = gy.double().cpu().abs()
        wa = wr.detach().clone().requires_grad_(True)
        ya = (F.conv_transpose2d(xa, wa, None, s, p, op) if tr else F.conv2d(xa, wa, None, s, p))
        ya.backward(ga)
        cancel = float(np.linalg.norm(wa.grad.numpy()) / max(np.linalg.norm(wr.grad.numpy()), 1e-300))
        # per-channel sums of dx (what a following bias gradient adds up) and their cancellation
        sdx_r = xr.grad.sum(dim=(0, 2, 3)).numpy()
        cancel_dx = float(np.linalg.norm(xr.grad.abs().sum(dim=(0, 2, 3)).numpy()) / max(np.linalg.norm(sdx_r), 1e-300))
        for math in (0, 2):
            xd = xx.contiguous(memory_format=torch.channels_last) if xx.shape[1] >= 32 else xx.contiguous()
            xd = xd.clone().requires_grad_(True)
            wd = w.clone().requires_grad_(True)
            if tr:
                y = IF.conv_transpose2d(xd, wd, None, s, p, op, math=math)
                ops = ("conv_transpose2d_fwd", "conv_transpose2d_dgrad", "conv_transpose2d_wgrad")
            else:
                y = IF.conv2d(xd, wd, None, s, p, math=math)
                ops = ("conv2d_fwd", "conv2d_dgrad", "conv2d_wgrad")
            y.backward(gy)
            gyd = gy.contiguous(memory_format=torch.channels_last) if gy.shape[1] >= 32 else gy.contiguous()
            kern = []
            for o, (aa, bb) in zip(ops, ((xd, y), (gyd, xd), (xd, gyd))):
                try:
                    pl = _lib.plan(o, aa.detach(), bb.detach(), k, s, p, math)
                    kern.append(f"{pl['kernel']}/{pl['bm']}/k{pl['ksplit']}" + (f"/n{pl['nsplit']}" if pl['nsplit'] else ""))
                except RuntimeError:
                    kern.append("?")
            print(f"{name:34s} {math:<4d} {' '.join(kern):44s} {rel(y.detach().cpu(), yr.detach()):9.2e} "
                  f"{rel(xd.grad.cpu(), xr.grad):9.2e} {rel(wd.grad.cpu(), wr.grad):9.2e} {cancel:8.1f} "
                  f"{rel(xd.grad.double().cpu().sum(dim=(0, 2, 3)), sdx_r):9.2e} {cancel_dx:8.1f}")


if __name__ == "__main__":
    main()
