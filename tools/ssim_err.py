"""SSIM / MS-SSIM loss gradient errors of the HIP kernels and of the fp32 CPU
oracle, both against the fp64 oracle (elementwise max |d| / max |ref| and normwise)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from image_compression_amd.modelling.loss import MS_SSIMLoss, SSIMLoss
    from oracle import ref_cpu
    for H, W in [(192, 192), (181, 207), (256, 256)]:
        for log_scale in (True, False):
            a = torch.rand(2, 3, H, W, generator=torch.Generator().manual_seed(21))
            b = (a + 0.1 * torch.randn(2, 3, H, W, generator=torch.Generator().manual_seed(22))).clamp(0, 1)
            for name, ref_fn, mod in (("msssim", ref_cpu.ms_ssim_loss, MS_SSIMLoss), ("ssim", ref_cpu.ssim_loss, SSIMLoss)):
                res = {}
                for dt in (torch.float64, torch.float32):
                    br = b.to(dt).clone().requires_grad_(True)
                    l = ref_fn(a.to(dt), br, log_scale=log_scale)
                    l.sum().backward()
                    res[dt] = br.grad.double().numpy()
                bd = b.cuda().requires_grad_(True)
                l = mod(log_scale=log_scale)(a.cuda(), bd)
                l.sum().backward()
                hip = bd.grad.double().cpu().numpy()
                r = res[torch.float64]
                for tag, v in (("hip", hip), ("cpu32", res[torch.float32])):
                    print(f"{name:6s} {H}x{W} log={int(log_scale)} {tag:5s} max|d|/max|ref| "
                          f"{np.abs(v - r).max() / np.abs(r).max():.2e}  normwise "
                          f"{np.linalg.norm(v - r) / np.linalg.norm(r):.2e}")


if __name__ == "__main__":
    main()
