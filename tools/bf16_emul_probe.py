#!/usr/bin/env python3
"""Each bf16-operand conv op of config C3 against fp64 (exact) and against fp64 with bf16-rounded
operands (oracle.ref_cpu._ConvRounded): the kernels' error should be fp32-class against the
second.  GPU only.   python tools/bf16_emul_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from conftest import rel_err  # noqa: E402
from oracle import ref_cpu  # noqa: E402
from image_compression_amd import functional as IF  # noqa: E402


def r(*s, seed, scale=1.0):
    return torch.randn(*s, generator=torch.Generator().manual_seed(seed)) * scale


for tr, n, cin, cout, h in [(False, 2, 192, 192, 64), (False, 2, 192, 320, 16), (False, 2, 192, 192, 16),
                            (True, 2, 320, 192, 8), (True, 2, 192, 192, 32)]:
    x = r(n, cin, h, h, seed=1)
    w = r(*((cin, cout) if tr else (cout, cin)), 5, 5, seed=2, scale=0.05)
    b = r(cout, seed=3, scale=0.1)
    res = {}
    for mode in ("exact", "emul"):
        f = (True, True, True) if mode == "emul" else (False, False, False)
        xr, wr, br = x.double().requires_grad_(True), w.double().requires_grad_(True), b.double().requires_grad_(True)
        y = ref_cpu._ConvRounded.apply(xr, wr, br, 2, 2, 1 if tr else 0, tr, *f)
        gy = r(*y.shape, seed=4)
        y.backward(gy.double())
        res[mode] = (y.detach(), xr.grad, wr.grad)
    xd = x.cuda().contiguous(memory_format=torch.channels_last).requires_grad_(True)
    wd = w.cuda().requires_grad_(True)
    with IF.record_plans() as log:
        y = (IF.conv_transpose2d(xd, wd, b.cuda(), 2, 2, 1, math=3) if tr
             else IF.conv2d(xd, wd, b.cuda(), 2, 2, math=3))
        y.backward(gy.cuda().contiguous(memory_format=torch.channels_last))
    got = (y.detach().cpu(), xd.grad.cpu(), wd.grad.cpu())
    kern = [p["kernel"] for p in log]
    print(f"tr={tr} {n}x{cin}->{cout} @{h}: kernels {kern}")
    for i, nm in enumerate(("y", "dx", "dw")):
        print(f"   {nm}: vs exact {rel_err(got[i], res['exact'][i]):.2e}  vs emulated {rel_err(got[i], res['emul'][i]):.2e}"
              f"  floor {rel_err(res['emul'][i], res['exact'][i]):.2e}")
