#!/usr/bin/env python3
"""Phase cycles of edge_conv_x3_kernel from a stamp build (EC_STAMP=1, tools/abl_build.sh):
g_a.0's forward (32 x 3 x 256^2 -> 192 x 128^2, 5x5 stride 2) in split or bf16 arithmetic; per wave and
unit the s_memtime stamps EC_ST(0..6): loop top, after the barrier, after the patch DMA issue, after the
plane build, after the MFMAs (their results consumed), after the output stores, after the end-of-unit
wait.  Prints the mean cycles of each phase over all waves and units 1..38 (unit 0 and the tail excluded).

    IMGCOMP_LIB=tools/_abl/ecst/libimgcomp.so python tools/edge_stamps.py [--math 2|1]
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--math", type=int, default=2)
    a = ap.parse_args()
    from image_compression_amd import _lib
    ops = _lib.ops()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.rand(32, 3, 256, 256, device=dev, generator=g)
    w = torch.randn(192, 3, 5, 5, device=dev, generator=g) * 0.1
    b = torch.randn(192, device=dev, generator=g) * 0.1
    for _ in range(3):
        ops.conv2d_fwd(x, w, b, 2, 2, 0, a.math)
    torch.cuda.synchronize()
    lib = ctypes.CDLL(_lib.LIB_PATH)
    IT, N = 40, 8
    buf = np.zeros(256 * 8 * IT * N, dtype=np.uint64)
    rc = lib.ic_debug_edge_stamps(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_size_t(buf.nbytes))
    assert rc == 0
    st = buf.reshape(256, 8, IT, N).astype(np.int64)
    names = ["barrier", "DMA issue", "build", "MFMA+epilogue math", "stores issue", "end wait", "loop back"]
    it = slice(1, 31)
    d = np.diff(st[:, :, it, :7], axis=-1)             # phases 0->1 .. 5->6
    nxt = st[:, :, 2:32, 0] - st[:, :, it, 6]          # 6 -> next iteration's 0
    print(f"math {a.math}: mean cycles per unit and wave (units 1..30, all 256 blocks x 8 waves)")
    for k in range(6):
        v = d[..., k]
        print(f"  {names[k]:22s} {v.mean():8.0f}   (p10 {np.percentile(v, 10):7.0f}, p90 {np.percentile(v, 90):7.0f})")
    print(f"  {names[6]:22s} {nxt.mean():8.0f}")
    tot = st[:, :, 31, 0] - st[:, :, 1, 0]
    print(f"  unit total             {tot.mean() / 30:8.0f}")
    for wv in range(8):
        print(f"  wave {wv}: " + " ".join(f"{d[:, wv, :, k].mean():6.0f}" for k in range(6)))


if __name__ == "__main__":
    main()
