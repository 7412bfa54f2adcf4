#!/usr/bin/env python3
"""Time the fused GDN backward (math 2 = fp32_split, C = 192) at the C2 shapes, 32 x {128, 64, 32}^2,
with HIP events on the launch stream: the kernel plus its slab reduce, as the step launches them.
Run once per library (IMGCOMP_LIB selects an ablation build).  GPU only.

    python tools/gdn_bwd_time.py [--reps 20]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from image_compression_amd import _lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--math", type=int, default=2)
    ap.add_argument("--sizes", default="128,64,32", help="map sizes (comma-separated)")
    a = ap.parse_args()
    L = _lib.load()
    st = _lib.c_void(torch.cuda.current_stream().cuda_stream)
    print("lib", os.environ.get("IMGCOMP_LIB", "in-tree"))
    for h in [int(v) for v in a.sizes.split(",")]:
        C, N = 192, 32
        g = torch.Generator(device="cuda").manual_seed(0)
        x = torch.randn(N, C, h, h, device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
        nrm = (1 + torch.rand(N, C, h, h, device="cuda", generator=g)).contiguous(memory_format=torch.channels_last)
        gy = torch.randn(N, C, h, h, device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
        gam = (torch.rand(C, C, device="cuda", generator=g) * 0.01 + torch.eye(C, device="cuda") * 0.1).contiguous()
        dx = torch.empty_like(x)
        dg = torch.empty_like(gam)
        db = torch.empty(C, device="cuda")
        ax, adx = _lib.act(x), _lib.act(dx)
        nb = L.ic_gdn_bwd_ws(ax)
        ws = _lib.workspace(nb, "cuda")

        def run():
            rc = L.ic_gdn_bwd_ex(ax, _lib.ptr(nrm), _lib.ptr(gy), _lib.ptr(gam), 0, adx, _lib.ptr(dg), _lib.ptr(db),
                                 a.math, _lib.ptr(ws), nb, st)
            assert rc == 0, rc
        for _ in range(3):
            run()
        times = []
        for _ in range(5):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(a.reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) / a.reps)
        P = N * h * h
        gb = 4 * C * 4 * P / 1e9
        t = sorted(times)[2]
        print(f"{h}x{h}: {t:.4f} ms (min {min(times):.4f}); compulsory {gb:.3f} GB -> {gb / t:.2f} TB/s; "
              f"dx sum {float(dx.double().sum()):.6e} dgamma sum {float(dg.double().sum()):.6e}", flush=True)


if __name__ == "__main__":
    main()
