#!/usr/bin/env python3
"""Launch only the dominant kernel of the bench step — the g_a.2 forward conv
(conv 5x5 s2, 192->192, 32x192x128x128 -> 32x192x64x64, fp32) — a fixed
number of times, for rocprofv3 PMC passes (FETCH_SIZE / WRITE_SIZE in
separate runs).  The counters it yields are per launch of
ig_kernel<128,192,64,96,false>, the kernel bench.py's `roofline` times.

    rocprofv3 --pmc FETCH_SIZE --kernel-trace -d OUT -o fetch --output-format csv -- \
        python3 tools/dominant_kernel.py [reps] [fp32|fp32_split]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from image_compression_amd import functional as IF  # noqa: E402


def main(reps=10, math="fp32"):
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.rand(32, 192, 128, 128, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
    w = torch.randn(192, 192, 5, 5, device=dev, generator=g) * 0.02
    b = torch.zeros(192, device=dev)
    with torch.no_grad():
        for _ in range(reps):
            IF.conv2d(x, w, b, 2, 2, math=IF.MATH[math])
    torch.cuda.synchronize()
    print("dominant kernel launched", reps, "times")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 10, sys.argv[2] if len(sys.argv) > 2 else "fp32")
