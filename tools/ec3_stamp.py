#!/usr/bin/env python3
"""Per-phase cycles of edge_conv_x3 (diagnostic EC3_STAMP=1 build, selected with IMGCOMP_LIB):
runs g_a.0's forward at the bench shape (32 x 3 x 256^2 -> 192 x 128^2, split arithmetic), then
prints, per phase, the s_memtime cycles per unit averaged over waves 0-3 and 4-7 of all blocks."""
import ctypes
import sys

import numpy as np
import torch

from image_compression_amd import _lib, functional as IF

PH = ["loop", "barrier", "patch-ld issue", "build", "mfma issue", "patch-st(wait)", "ob(wait mfma)", "stores"]


def main():
    L = _lib.load()
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    x = torch.randn(n, 3, 256, 256, device="cuda")
    w = torch.randn(192, 3, 5, 5, device="cuda") * 0.1
    b = torch.randn(192, device="cuda")
    with torch.no_grad():
        for _ in range(20):
            IF.conv2d(x, w, b, 2, 2, math=2)
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        IF.conv2d(x, w, b, 2, 2, math=2)
        ev1.record()
        torch.cuda.synchronize()
    buf = np.zeros(256 * 8 * 8, dtype=np.uint64)
    rc = L.ic_edge_stamps(ctypes.c_void_p(buf.ctypes.data))
    assert rc == 0, rc
    st = buf.reshape(256, 8, 8).astype(np.float64)
    units = n * 128 * 2 / 256
    print(f"launch {ev0.elapsed_time(ev1):.3f} ms, {units:.0f} units per block")
    tot = st.sum(axis=2)
    print(f"total cycles per wave: mean {tot.mean():.0f} (min {tot.min():.0f} max {tot.max():.0f}) "
          f"-> {tot.mean() / units:.0f} per unit")
    for k, name in enumerate(PH):
        a, c = st[:, :4, k].mean() / units, st[:, 4:, k].mean() / units
        print(f"  {name:16s} waves0-3 {a:8.0f}  waves4-7 {c:8.0f}  cycles/unit")


if __name__ == "__main__":
    main()
