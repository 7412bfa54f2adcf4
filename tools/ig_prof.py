#!/usr/bin/env python3
"""Per-chunk phase times of the implicit-GEMM conv kernel from an IG_PROF
build (s_memtime stamps of wave 0 of the first 1024 blocks, first 32 K chunks):

    hipcc ... -DIG_PROF -c igemm.hip  (linked into tools/_abl/lib_igprof.so)
    IMGCOMP_LIB=$PWD/tools/_abl/lib_igprof.so python tools/ig_prof.py
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
    w = torch.randn(192, 192, 5, 5, device=dev, generator=g) * 0.02
    b = torch.zeros(192, device=dev)
    with torch.no_grad():
        for _ in range(3):
            IF.conv2d(x, w, b, 2, 2)
    torch.cuda.synchronize()
    lib = _lib.load()
    buf = np.zeros(1024 * 32 * 6, dtype=np.uint64)
    fn = lib.ic_debug_ig_prof
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    assert fn(buf.ctypes.data, buf.nbytes) == 0
    t = buf.reshape(1024, 32, 6).astype(np.int64)
    ok = t[:, :, 0] > 0
    names = ["gload", "mfma(issue)", "bar1", "sstore", "bar2"]
    d = np.diff(t, axis=2)
    per = t[:, 1:, 0] - t[:, :-1, 0]
    sel = ok[:, 1:] & ok[:, :-1]
    print(f"chunk period (clk): median {np.median(per[sel]):.0f}  mean {per[sel].mean():.0f}")
    for e, n in enumerate(names):
        v = d[:, 1:-1, e][ok[:, 1:-1]]
        print(f"  {n:12s} median {np.median(v):7.0f}  mean {v.mean():7.0f}")


if __name__ == "__main__":
    main()
