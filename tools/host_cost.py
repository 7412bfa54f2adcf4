#!/usr/bin/env python3
"""Host (CPU) cost per call of the ops on the hyperprior's backward chain: N calls issued
back to back without synchronising, timed on the host (launch-bound when the GPU keeps up),
against the GPU time of the same calls (HIP events).  GPU only.

    python tools/host_cost.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from image_compression_amd import _lib, functional as F  # noqa: E402

CL = torch.channels_last


def cost(name, fn, n=200):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    e1.record()
    torch.cuda.synchronize()
    print(f"{name:40s} host {1e6 * (t1 - t0) / n:7.1f} us/call   gpu {1e3 * e0.elapsed_time(e1) / n:7.1f} us/call")


def main():
    ops = _lib.ops()
    d = "cuda"
    x = torch.randn(32, 192, 16, 16, device=d).contiguous(memory_format=CL)
    w = torch.randn(192, 192, 3, 3, device=d) * 0.05
    w5 = torch.randn(192, 192, 5, 5, device=d) * 0.05
    gy = torch.randn(32, 192, 16, 16, device=d).contiguous(memory_format=CL)
    y8 = torch.randn(32, 192, 8, 8, device=d).contiguous(memory_format=CL)
    cost("relu_fwd 32x192x16x16", lambda: ops.relu_fwd(x))
    cost("empty_like (allocator)", lambda: torch.empty_like(x))
    cost("conv2d_fwd 3x3 s1 16^2 split", lambda: ops.conv2d_fwd(x, w, None, 1, 1, 0, 2))
    cost("conv2d_dgrad 3x3 s1 16^2 split", lambda: ops.conv2d_dgrad(gy, w, x, 1, 1, 2))
    cost("conv2d_wgrad 3x3 s1 16^2 split", lambda: ops.conv2d_wgrad(x, gy, w, 1, 1, True, 2))
    cost("conv_transpose2d_dgrad 5x5 s2 8->16", lambda: ops.conv_transpose2d_dgrad(gy, w5, y8, 2, 2, 2))
    xr = x.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)

    def fb():
        y = F.conv2d(xr, wr, None, 1, 1, 0, 2)
        y.backward(gy)
    cost("Conv2dFn fwd+bwd (autograd, 3x3 16^2)", fb, n=100)


if __name__ == "__main__":
    main()
