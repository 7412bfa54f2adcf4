#!/usr/bin/env python3
"""MS-SSIM log-scale loss forward + backward at C4's shape (16 x 3 x 256^2), timed with HIP events:
    IMGCOMP_LIB=... python tools/ssim_time.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from image_compression_amd.modelling.loss import MS_SSIMLoss
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    a = torch.rand(16, 3, 256, 256, device=dev, generator=g)
    b = (a + 0.05 * torch.randn(16, 3, 256, 256, device=dev, generator=g)).clamp(0, 1).requires_grad_(True)
    loss = MS_SSIMLoss(max_val=1.0, log_scale=True)
    for _ in range(5):
        loss(a, b).sum().backward()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    res = []
    for _ in range(5):
        e0.record()
        for _ in range(20):
            loss(a, b).sum().backward()
        e1.record()
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) / 20)
    print("ms-ssim fwd+bwd ms per call:", " ".join(f"{r:.4f}" for r in res), "min", f"{min(res):.4f}")


if __name__ == "__main__":
    main()
