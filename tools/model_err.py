"""Per-tensor error report of one Compressor2018 training step on the HIP path
against the fp64 CPU oracle (oracle/ref_cpu.py), at a chosen size / math.

usage: python tools/model_err.py --n 16 --size 256 --math fp32_split [--loss msssim] [--latent 320]
Prints normwise relative errors of x_tilde, losses and every parameter
gradient, sorted worst first, plus the implicit-GEMM plans the step ran.
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

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
    ap.add_argument("--math", default="fp32_split")
    ap.add_argument("--loss", default="mse")
    ap.add_argument("--latent", type=int, default=192)
    ap.add_argument("--lam", type=float, default=256.0)
    ap.add_argument("--gdn-math", type=int, default=-1, help="override GDN math / math_fwd (-1: keep)")
    ap.add_argument("--conv-math", type=int, default=-1, help="override every conv's math (-1: keep)")
    ap.add_argument("--bwd-math", type=int, default=-1, help="override the convs' backward math only (-1: keep)")
    ap.add_argument("--hyper-math", type=int, default=-1, help="override the hyperprior convs' math (-1: keep)")
    a = ap.parse_args()
    from image_compression_amd import get_cfg_defaults, injected_noise, modelling
    from oracle import ref_cpu
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    cfg = get_cfg_defaults()
    cfg.MODEL.LOSS.REDUCTION = "mean"
    cfg.MODEL.LOSS.DISTORTION_LOSS_WEIGHT = a.lam
    cfg.MODEL.LATENT_CHANNELS = a.latent
    cfg.MODEL.COMPUTE_DTYPE = a.math
    kw = dict(lam=a.lam)
    if a.loss == "msssim":
        cfg.MODEL.LOSS.DISTORTION_LOSS_NAMES = ["MS_SSIMLoss"]
        cfg.MODEL.LOSS.SSIM.LOG_SCALE = True
        kw.update(loss_names=("MS_SSIMLoss",), ssim_log=True)
    torch.manual_seed(0)
    model = modelling.build_model(cfg)
    params = {k: v.clone() for k, v in model.state_dict().items()}
    model = model.cuda().train()
    from image_compression_amd.modelling.layers import GDN, Conv2d, ConvTranspose2d
    for m in model.modules():
        if a.gdn_math >= 0 and isinstance(m, GDN):
            m.math = m.math_fwd = a.gdn_math
        if a.conv_math >= 0 and isinstance(m, (Conv2d, ConvTranspose2d)):
            m.math = a.conv_math
    if a.hyper_math >= 0:
        for m in list(model.prior_analysis.modules()) + list(model.prior_synthesis.modules()):
            if isinstance(m, (Conv2d, ConvTranspose2d)):
                m.math = a.hyper_math
    if a.bwd_math >= 0:
        from image_compression_amd import functional as IF
        for cls in (IF.Conv2dFn, IF.ConvTranspose2dFn):
            orig = cls.backward

            def bwd(ctx, gy, _orig=orig):
                ctx.conf = ctx.conf[:-1] + (a.bwd_math,)
                return _orig(ctx, gy)
            cls.backward = staticmethod(bwd)
    caps = {}

    def hook(key):
        def f(mod, inp, out):
            caps[key] = out
        return f

    model.analysis_transform.register_forward_hook(hook("y"))
    model.prior_analysis.register_forward_hook(hook("z"))
    model.entropy_model.register_forward_hook(hook("em"))
    model.prior_synthesis.register_forward_hook(hook("sigma"))
    model.conditional_model.register_forward_hook(hook("cm"))
    g = torch.Generator().manual_seed(3)
    N, S = a.n, a.size
    x = torch.rand(N, 3, S, S, generator=g)
    uz = torch.rand(N, 192, S // 64, S // 64, generator=g)
    uy = torch.rand(N, a.latent, S // 16, S // 16, generator=g)
    with injected_noise([uz.cuda(), uy.cuda()]):
        xt, losses = model(x.cuda())
    losses["total_loss"].backward()
    torch.cuda.synchronize()
    t = time.time()
    out, rl, rg = ref_cpu.run(params, x, uz, uy, train=True, dtype=torch.float64, **kw)
    print(f"oracle {time.time() - t:.1f} s  ({N}x{S}^2, {a.math}, {a.loss}, latent {a.latent})")
    print(f"x_tilde  {rel(xt.cpu(), out['x_tilde'].detach()):.3e}")
    mine = {"y": caps["y"], "z": caps["z"], "z_tilde": caps["em"][0], "p_z": caps["em"][1], "sigma": caps["sigma"],
            "y_tilde": caps["cm"][0], "p_y": caps["cm"][1]}
    for k, v in mine.items():
        print(f"{k:8s} {rel(v.detach().float().cpu(), out[k].detach()):.3e}")
    for k in losses:
        if k in rl:
            va, vb = float(losses[k]), float(rl[k])
            print(f"loss {k:12s} {abs(va - vb) / max(abs(vb), 1e-300):.3e}")
    errs = sorted(((rel(p.grad.cpu(), rg[n]), n) for n, p in model.named_parameters()), reverse=True)
    for e, n in errs:
        print(f"grad {e:.3e}  {n}")


if __name__ == "__main__":
    main()
