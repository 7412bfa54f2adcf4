#!/usr/bin/env python3
"""A/B of the fused GDN kernels in one process, alternating, on the 128x128
and 64x64 C2 shapes: backward with fp32 dgamma (math 0) vs split dgamma
(math 2); forward fp32 (math 0) vs split (math 2).  GPU only."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from image_compression_amd import _lib  # noqa: E402


def main():
    L = _lib.load()
    st = _lib.c_void(torch.cuda.current_stream().cuda_stream)
    for h in (128, 64):
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
        res = {0: [], 2: []}
        for rep in range(6):
            for m in (0, 2):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                for _ in range(2):
                    L.ic_gdn_bwd_ex(ax, _lib.ptr(nrm), _lib.ptr(gy), _lib.ptr(gam), 0, adx, _lib.ptr(dg), _lib.ptr(db),
                                    m, _lib.ptr(ws), nb, st)
                e0.record()
                for _ in range(10):
                    L.ic_gdn_bwd_ex(ax, _lib.ptr(nrm), _lib.ptr(gy), _lib.ptr(gam), 0, adx, _lib.ptr(dg), _lib.ptr(db),
                                    m, _lib.ptr(ws), nb, st)
                e1.record()
                torch.cuda.synchronize()
                res[m].append(e0.elapsed_time(e1) / 10)
        print(f"{h}x{h}: bwd fp32 dgamma {min(res[0]):.3f} ms (median {sorted(res[0])[3]:.3f}), "
              f"split dgamma {min(res[2]):.3f} ms (median {sorted(res[2])[3]:.3f})")
        y = torch.empty_like(x)
        ay = _lib.act(y)
        be = torch.ones(C, device="cuda")
        res = {0: [], 2: []}
        for rep in range(6):
            for m in (0, 2):
                nb = L.ic_gdn_fwd_ws_ex(ax, m)
                wsf = _lib.workspace(max(nb, 256), "cuda")
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                for _ in range(2):
                    L.ic_gdn_fwd_ex(ax, _lib.ptr(gam), _lib.ptr(be), 0, ay, _lib.ptr(nrm), m, _lib.ptr(wsf), nb, st)
                e0.record()
                for _ in range(10):
                    L.ic_gdn_fwd_ex(ax, _lib.ptr(gam), _lib.ptr(be), 0, ay, _lib.ptr(nrm), m, _lib.ptr(wsf), nb, st)
                e1.record()
                torch.cuda.synchronize()
                res[m].append(e0.elapsed_time(e1) / 10)
        print(f"{h}x{h}: fwd fp32 {min(res[0]):.3f} ms (median {sorted(res[0])[3]:.3f}), "
              f"split {min(res[2]):.3f} ms (median {sorted(res[2])[3]:.3f})")


if __name__ == "__main__":
    main()
