#!/usr/bin/env python3
"""The round-3 factorized-backward fault outside the model: fact_bwd_k (entropy.hip) launched
again and again on a side stream while the main stream runs a hog, every result compared
bitwise with the result of the same launch on an idle GPU.  Hogs: `conv` (ig_kernel_x3d: MFMA +
LDS-DMA, 137 KB of LDS), `gdnb` (gdn_bwd_fused_kernel: MFMA + LDS-DMA), `wgrad` (wg_x3d_kernel:
MFMA, register-staged LDS), `gemm` (a torch bf16 matmul: MFMA, no kernel of ours), `none`.
Run under IMGCOMP_LIB=<variant>/libimgcomp.so to pick the build (tools/abl_build.sh; e.g.
entropy.hip with packed-fp32 VALU, as in round 3, or without).  One JSON line per hog.  GPU only.

    python tools/race_fact.py --hogs none,gemm,conv,gdnb,wgrad --iters 40
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from image_compression_amd import _lib, get_cfg_defaults, modelling  # noqa: E402
from image_compression_amd import functional as IF  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hogs", default="none,gemm,conv,gdnb,wgrad")
    ap.add_argument("--iters", type=int, default=40, help="hog launches per hog kind")
    ap.add_argument("--per", type=int, default=8, help="fact_bwd launches queued per hog launch")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    ops = _lib.ops()
    cfg = get_cfg_defaults()
    torch.manual_seed(0)
    em = modelling.build_model(cfg).entropy_model.to(dev)
    prm = [t.detach().contiguous() for t in em._cdf_estimator.flat_params()]
    g = torch.Generator(device=dev).manual_seed(1)
    C = 192
    q = (torch.randn(32 * 4 * 4, C, device=dev, generator=g) * 3).round().contiguous()  # C2's z~, (N H W, C)
    gq = torch.randn(32 * 4 * 4, C, device=dev, generator=g) * 1e-3
    gp = -1.0 / (torch.rand(32 * 4 * 4, C, device=dev, generator=g) + 0.05) * 1e-4
    ref = ops.factorized_bwd(q, C, prm, gq, gp)
    torch.cuda.synchronize()
    ref = [ref[0].clone()] + [t.clone() for t in ref[1]]

    # hog operands
    xc = torch.rand(32, 192, 128, 128, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
    wc = torch.randn(192, 192, 5, 5, device=dev, generator=g) * 0.02
    bc = torch.zeros(192, device=dev)
    yc = torch.randn(32, 192, 64, 64, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
    ga = torch.randn(8192, 8192, device=dev, generator=g, dtype=torch.bfloat16)
    xg = torch.rand(32, 192, 128, 128, device=dev, generator=g).contiguous(memory_format=torch.channels_last) + 0.1
    gam = torch.rand(192, 192, 1, 1, device=dev, generator=g) * 0.1
    bet = torch.ones(192, device=dev)
    ng = torch.rand(32, 192, 128, 128, device=dev, generator=g).contiguous(memory_format=torch.channels_last) + 1
    dyg = torch.randn_like(xg).contiguous(memory_format=torch.channels_last)

    def hog(kind):
        with torch.no_grad():
            if kind == "conv":
                IF.conv2d(xc, wc, bc, 2, 2, math=IF.MATH["fp32_split"])
            elif kind == "wgrad":
                ops.conv2d_wgrad(xc, yc, wc, 2, 2, False, IF.MATH["fp32_split"])
            elif kind == "gdnb":
                ops.gdn_bwd(xg, ng, dyg, gam.view(192, 192), False, IF.MATH["fp32_split"])
            elif kind == "gemm":
                ga @ ga

    main_s = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(dev, priority=-1)
    for kind in a.hogs.split(","):
        bad, total, elems = 0, 0, 0
        outs = []
        for it in range(a.iters):
            side.wait_stream(main_s)
            hog(kind)
            with torch.cuda.stream(side):
                for _ in range(a.per):
                    r = ops.factorized_bwd(q, C, prm, gq, gp)
                    outs.append([r[0]] + list(r[1]))
            main_s.wait_stream(side)
            if len(outs) >= 64 or it == a.iters - 1:
                torch.cuda.synchronize()
                for o in outs:
                    total += 1
                    d = [int((u != v).sum()) for u, v in zip(o, ref)]
                    if any(d):
                        bad += 1
                        elems += sum(d)
                outs.clear()
        print(json.dumps({"hog": kind, "lib": os.environ.get("IMGCOMP_LIB", "in-tree"), "launches": total,
                          "mismatching_launches": bad, "mismatching_elements": elems}), flush=True)


if __name__ == "__main__":
    main()
