"""Where a whole-step gradient error enters: compare the gradients at the
hyperprior's boundary tensors (dL/dsigma, dL/dz, dL/dy) and the hyperprior
ReLU masks of one HIP training step with the fp64 oracle's, and print the
worst elements with their forward values.

usage: python tools/grad_probe.py --n 16 --size 256 --math fp32_split
"""
import argparse
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=16)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--math", default="fp32_split")
    a = ap.parse_args()
    from image_compression_amd import get_cfg_defaults, injected_noise, modelling
    from oracle import ref_cpu
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    cfg = get_cfg_defaults()
    cfg.MODEL.LOSS.REDUCTION = "mean"
    cfg.MODEL.LOSS.DISTORTION_LOSS_WEIGHT = 256.0
    cfg.MODEL.COMPUTE_DTYPE = a.math
    torch.manual_seed(0)
    model = modelling.build_model(cfg)
    params = {k: v.clone() for k, v in model.state_dict().items()}
    model = model.cuda().train()
    caps, grads = {}, {}

    def hook(key, idx=None):
        def f(mod, inp, out):
            t = out if idx is None else out[idx]
            caps[key] = t.detach().float().cpu()
            t.register_hook(lambda g: grads.__setitem__(key, g.detach().float().cpu()))
        return f

    model.analysis_transform.register_forward_hook(hook("y"))
    model.prior_analysis.register_forward_hook(hook("z"))
    model.prior_synthesis.register_forward_hook(hook("sigma"))
    model.conditional_model.register_forward_hook(hook("y_tilde", 0))
    model.conditional_model.register_forward_hook(hook("p_y", 1))
    relus = {}
    for name, m in list(model.prior_analysis.named_modules()) + list(model.prior_synthesis.named_modules()):
        if type(m).__name__ == "ReLU":
            m.register_forward_hook(lambda mod, i, o, name=name: relus.__setitem__(name + str(o.shape[-1]),
                                                                                (i[0] > 0).cpu()))
    g = torch.Generator().manual_seed(3)
    N, S = a.n, a.size
    x = torch.rand(N, 3, S, S, generator=g)
    uz = torch.rand(N, 192, S // 64, S // 64, generator=g)
    uy = torch.rand(N, 192, S // 16, S // 16, generator=g)
    with injected_noise([uz.cuda(), uy.cuda()]):
        _, losses = model(x.cuda())
    losses["total_loss"].backward()
    torch.cuda.synchronize()
    P = {k: torch.as_tensor(v).double().clone().requires_grad_(True) for k, v in params.items()}
    out, rl = ref_cpu.forward(P, x.double(), uz.double(), uy.double(), True, lam=256.0)
    for k in ("y", "z", "sigma", "y_tilde", "p_y"):
        out[k].retain_grad()
    rl["total_loss"].backward()
    for k in ("y", "z", "sigma", "y_tilde", "p_y"):
        r = out[k].grad.numpy()
        m = grads.get(k)
        if m is None:
            continue
        m = m.numpy()
        d = np.abs(m - r)
        print(f"d/d{k:8s} normwise {np.linalg.norm(m - r) / np.linalg.norm(r):.3e}  max|d| {d.max():.3e} "
              f"max|ref| {np.abs(r).max():.3e}")
        for i in np.argsort(d.ravel())[::-1][:4]:
            idx = np.unravel_index(i, d.shape)
            fw = {kk: float(caps[kk][idx]) for kk in ("y", "sigma", "y_tilde", "p_y") if caps[kk].shape == d.shape}
            fr = {kk: float(out[kk].detach()[idx]) for kk in ("y", "sigma", "y_tilde", "p_y")
                  if out[kk].shape == d.shape}
            print(f"   {idx} mine {m[idx]:.6e} ref {r[idx]:.6e}  fwd mine {fw}  ref {fr}")


if __name__ == "__main__":
    main()
