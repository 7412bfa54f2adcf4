#!/usr/bin/env python3
"""Weight gradients of the 5x5 stride-2 192x192 layers (conv and transposed conv; 128/64, 32/16 and a
3-image 64/32 map; fp32_split and bf16) on fixed inputs: save them (--out F) or compare bitwise with a
saved run (--ref F) -- run once per library build (IMGCOMP_LIB) to check that two kernels agree bitwise
(r05m: wg_x3g_kernel vs wg_x3d_kernel).  GPU only."""
import argparse, os, sys, torch
sys.path.insert(0, os.getcwd())
from image_compression_amd import _lib
from image_compression_amd import functional as IF
ap = argparse.ArgumentParser(); ap.add_argument("--out"); ap.add_argument("--ref"); a = ap.parse_args()
ops = _lib.ops(); dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(11)
res = {}
for name, big, n in (("128", 128, 32), ("32", 32, 32), ("odd", 64, 3)):
    x = torch.randn(n, 192, big, big, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
    gy = torch.randn(n, 192, big // 2, big // 2, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
    w = torch.randn(192, 192, 5, 5, device=dev, generator=g)
    for mname in ("fp32_split", "bf16"):
        m = IF.MATH[mname]
        dw, db = ops.conv2d_wgrad(x, gy, w, 2, 2, True, m)
        res[f"conv_{name}_{mname}"] = dw.clone()
        # transposed conv 192 -> 192 (64^2 -> 128^2): G = its input (gy here), X = its output gradient (x)
        dwt, dbt = ops.conv_transpose2d_wgrad(gy, x, w, 2, 2, True, m)
        res[f"tconv_{name}_{mname}"] = dwt.clone()
torch.cuda.synchronize()
if a.out:
    torch.save({k: v.cpu() for k, v in res.items()}, a.out); print("saved", len(res))
if a.ref:
    ref = torch.load(a.ref, weights_only=True)
    bad = [k for k in ref if not torch.equal(ref[k], res[k].cpu())]
    for k in bad:
        d = (ref[k] - res[k].cpu()).abs().max().item(); print("DIFF", k, d, ref[k].abs().max().item())
    print("bitwise equal" if not bad else f"{len(bad)} of {len(ref)} differ")
    sys.exit(1 if bad else 0)
