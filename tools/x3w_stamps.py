#!/usr/bin/env python3
"""Per-phase cycles of gdn_bwd_x3w_kernel from a diagnostic build (-DX3W_STAMP=1, via IMGCOMP_LIB): one
launch at 32 x 192 x 128^2, then the s_memtime stamps each wave wrote at four points of every iteration
(loop top, after the dx GEMM + phase A, after the dgamma GEMM + epilogue, after the barrier).  GPU only."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from image_compression_amd import _lib  # noqa: E402


def main():
    L = _lib.load()
    st = _lib.c_void(torch.cuda.current_stream().cuda_stream)
    C, N, h = 192, 32, 128
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(N, C, h, h, device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
    nrm = (1 + torch.rand(N, C, h, h, device="cuda", generator=g)).contiguous(memory_format=torch.channels_last)
    gy = torch.randn(N, C, h, h, device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
    gam = (torch.rand(C, C, device="cuda", generator=g) * 0.01 + torch.eye(C, device="cuda") * 0.1).contiguous()
    dx, dg, db = torch.empty_like(x), torch.empty_like(gam), torch.empty(C, device="cuda")
    ax, adx = _lib.act(x), _lib.act(dx)
    nb = L.ic_gdn_bwd_ws(ax)
    ws = torch.zeros(nb // 4, device="cuda", dtype=torch.float32)
    for _ in range(3):
        L.ic_gdn_bwd_ex(ax, _lib.ptr(nrm), _lib.ptr(gy), _lib.ptr(gam), 0, adx, _lib.ptr(dg), _lib.ptr(db), 2,
                        _lib.ptr(ws), nb, st)
    torch.cuda.synchronize()
    grid = 256
    base = grid * (C * C + 2 * C + 1024)
    stamps = ws[base:base + grid * 4 * 160 * 8].view(torch.int64).view(grid, 4, 160, 4).cpu().double()
    ntiles = N * h * h // 16
    iters = ntiles // grid
    s = stamps[:, :, 1:iters - 1, :]   # drop the first and the last iteration
    d01 = (s[..., 1] - s[..., 0]).mean().item()
    d12 = (s[..., 2] - s[..., 1]).mean().item()
    d23 = (s[..., 3] - s[..., 2]).mean().item()
    per = (stamps[:, :, 2:iters - 1, 0] - stamps[:, :, 1:iters - 2, 0]).mean().item()
    print(f"iterations {iters}; cycles per iteration {per:.0f}: dx GEMM + phase A {d01:.0f}, "
          f"dgamma GEMM + epilogue {d12:.0f}, barrier wait {d23:.0f}")
    for w in range(4):
        sw = s[:, w]
        print(f"  wave {w}: {(sw[..., 1] - sw[..., 0]).mean().item():.0f} / {(sw[..., 2] - sw[..., 1]).mean().item():.0f}"
              f" / {(sw[..., 3] - sw[..., 2]).mean().item():.0f}")


if __name__ == "__main__":
    main()
