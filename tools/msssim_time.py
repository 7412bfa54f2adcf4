#!/usr/bin/env python3
"""Time the MS-SSIM loss (C4: ssim_64 log-scale MS-SSIM, 16 x 3 x 256^2) forward and backward with HIP
events, and report it against its HBM floor: the forward reads a and b at every level, the backward
reads a, b and writes the gradient (plus the pyramid's pooling passes).  Run once per library
(IMGCOMP_LIB selects an ablation build).  GPU only.

    python tools/msssim_time.py [--batch 16] [--size 256] [--reps 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from image_compression_amd.modelling.loss import MS_SSIMLoss
    print("lib", os.environ.get("IMGCOMP_LIB", "in-tree"))
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.rand(a.batch, 3, a.size, a.size, device="cuda", generator=g)
    xt = (x + 0.05 * torch.randn(x.shape, device="cuda", generator=g)).clamp(0, 1).requires_grad_(True)
    loss = MS_SSIMLoss(log_scale=True)
    for _ in range(3):
        loss(x, xt).sum().backward()
    torch.cuda.synchronize()
    tf, tb = [], []
    for _ in range(5):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
        fwd = bwd = 0.0
        for _ in range(a.reps):
            e[0].record()
            l = loss(x, xt).sum()
            e[1].record()
            l.backward()
            e[2].record()
            torch.cuda.synchronize()
            fwd += e[0].elapsed_time(e[1])
            bwd += e[1].elapsed_time(e[2])
        tf.append(fwd / a.reps)
        tb.append(bwd / a.reps)
    tf, tb = sorted(tf)[2], sorted(tb)[2]
    n = a.batch * 3 * a.size * a.size * 4
    pyr = sum(4 ** -l for l in range(5))  # bytes of a level pyramid / level-0 bytes
    fb = 2 * n * pyr + 2 * n * (pyr - 1)          # read a, b per level; write the pooled levels
    bb = 2 * n * pyr + 2 * n * pyr + 2 * n        # read a, b; read+write the per-level gradients; final scale
    print(f"{a.batch}x3x{a.size}^2: fwd {tf:.4f} ms ({fb / 1e9:.3f} GB floor -> {fb / tf / 1e9:.2f} TB/s), "
          f"bwd {tb:.4f} ms ({bb / 1e9:.3f} GB floor -> {bb / tb / 1e9:.2f} TB/s); loss {float(l):.6f} "
          f"grad sum {float(xt.grad.double().sum()):.6e}", flush=True)


if __name__ == "__main__":
    main()
