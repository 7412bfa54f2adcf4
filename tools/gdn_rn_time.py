#!/usr/bin/env python3
"""C3 GDN forward / backward with and without the stored norm (torch.ops.imgcomp.gdn_*_xb vs gdn_*_rn),
HIP events around `reps` launches each, at the C3 layer sizes (32 x 192 x {128, 64, 32}^2).  GPU only."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from image_compression_amd import _lib  # noqa: E402


def t_ms(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    ops = _lib.ops()
    g = torch.Generator(device="cuda").manual_seed(0)
    for hw in (128, 64, 32):
        x = torch.randn(32, 192, hw, hw, device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
        dy = torch.randn_like(x)
        gamma = (torch.eye(192, device="cuda") * 0.1 + 0.001).reshape(192, 192, 1, 1).contiguous()
        beta = torch.ones(192, device="cuda")
        _, norm, _ = ops.gdn_fwd_xb(x, gamma, beta, False, 3)
        f0 = t_ms(lambda: ops.gdn_fwd_xb(x, gamma, beta, False, 3))
        f1 = t_ms(lambda: ops.gdn_fwd_rn(x, gamma, beta, False, 3, True))
        b0 = t_ms(lambda: ops.gdn_bwd_sum_xb(x, norm, dy, gamma, False, 3))
        b1 = t_ms(lambda: ops.gdn_bwd_sum_rn(x, beta, dy, gamma, False, 3, True))
        print(f"{hw:4d}^2  fwd stored {f0:.4f}  recompute {f1:.4f} ms | bwd stored {b0:.4f}  recompute {b1:.4f} ms")


if __name__ == "__main__":
    main()
