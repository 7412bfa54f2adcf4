#!/usr/bin/env python3
"""Per-K-step phase times of the weight-gradient kernel from a WG_PROF build
(s_memtime stamps of wave 0 of the first 1024 blocks, first 64 K steps):
    IMGCOMP_LIB=$PWD/tools/_abl/lib_wgprof.so python tools/wg_prof.py
"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from image_compression_amd import _lib  # noqa: E402
from image_compression_amd import functional as IF  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.rand(32, 192, 128, 128, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(192, 192, 5, 5, device=dev, generator=g) * 0.02).requires_grad_(True)
    b = torch.zeros(192, device=dev, requires_grad=True)
    gy = torch.randn(32, 192, 64, 64, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
    for _ in range(3):
        y = IF.conv2d(x, w, b, 2, 2)
        y.backward(gy)
    torch.cuda.synchronize()
    lib = _lib.load()
    buf = np.zeros(1024 * 64 * 3, dtype=np.uint64)
    fn = lib.ic_debug_wg_prof
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    assert fn(buf.ctypes.data, buf.nbytes) == 0
    t = buf.reshape(1024, 64, 3).astype(np.int64)
    ok = (t[:, 1:, 0] > 0) & (t[:, :-1, 0] > 0)
    per = (t[:, 1:, 0] - t[:, :-1, 0])[ok]
    bar = (t[:, :-1, 1] - t[:, :-1, 0])[ok]
    stg = (t[:, :-1, 2] - t[:, :-1, 1])[ok]
    mf = (t[:, 1:, 0] - t[:, :-1, 2])[ok]
    for n, v in (("period", per), ("barrier", bar), ("stage issue", stg), ("mfma+rest", mf)):
        print(f"  {n:12s} median {np.median(v):7.0f}  mean {v.mean():7.0f}  p90 {np.percentile(v, 90):7.0f}")


if __name__ == "__main__":
    main()
