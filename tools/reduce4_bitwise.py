#!/usr/bin/env python3
"""Outputs of the convolutions whose implicit GEMM splits K (small maps: the split-K reduction runs) and of
GDN on channel counts the fused kernels do not take (its 1x1 GEMM with the GDN epilogue), on fixed inputs:
save them (--out F) or compare bitwise with a saved run (--ref F) -- run once per library build
(IMGCOMP_LIB) to check that two reductions agree bitwise (r09zo: ig_reduce4_kernel vs ig_reduce_kernel).
Covers bias / ReLU epilogues, NHWC and NCHW outputs, ragged batches and a Cout that is not a multiple of 4.
GPU only."""
import argparse, os, sys, torch
sys.path.insert(0, os.getcwd())
from image_compression_amd import _lib
from image_compression_amd import functional as IF
ap = argparse.ArgumentParser(); ap.add_argument("--out"); ap.add_argument("--ref"); a = ap.parse_args()
ops = _lib.ops(); dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(13)
CL = torch.channels_last
res = {}


def put(key, fn):
    try:
        r = fn()
    except RuntimeError as e:  # a combination the op refuses: refused the same way by both builds
        print("skip", key, str(e).splitlines()[0][:100]); return None
    res[key] = (r[0] if isinstance(r, tuple) else r).clone()
    return r


def rnd(*s, cl=True):
    t = torch.randn(*s, device=dev, generator=g)
    return t.contiguous(memory_format=CL) if cl else t.contiguous()


for mname in ("fp32_split", "bf16", "fp32"):
    m = IF.MATH[mname]
    for (n, cin, cout, hw, k, s, p, cl) in ((32, 192, 192, 32, 5, 2, 2, True), (3, 192, 192, 32, 5, 2, 2, True),
                                           (32, 192, 192, 16, 3, 1, 1, True), (8, 192, 320, 16, 5, 2, 2, True),
                                           (8, 192, 192, 16, 5, 2, 2, False), (4, 192, 3, 32, 5, 2, 2, True),
                                           (8, 128, 128, 16, 3, 1, 1, True)):
        x = rnd(n, cin, hw, hw, cl=cl)
        w = rnd(cout, cin, k, k, cl=False)
        b = rnd(cout, cl=False)
        tag = f"{mname}_{n}x{cin}to{cout}_{hw}_k{k}s{s}_{'nhwc' if cl else 'nchw'}"
        for act in (0, 1):
            put(f"fwd_{tag}_act{act}", lambda: ops.conv2d_fwd(x, w, b, s, p, act, m))
        y = put(f"fwd_{tag}_nobias", lambda: ops.conv2d_fwd(x, w, None, s, p, 0, m))
        if y is not None:
            gy = rnd(*y.shape, cl=cl)
            put(f"dgrad_{tag}", lambda: ops.conv2d_dgrad(gy, w, x, s, p, m))
        if s == 2:
            wt = rnd(cin, cout, k, k, cl=False)
            bt = rnd(cout, cl=False)
            xt = rnd(n, cin, hw // 2, hw // 2, cl=cl)
            yt = put(f"tfwd_{tag}", lambda: ops.conv_transpose2d_fwd(xt, wt, bt, s, p, 1, 0, m))
            if yt is not None:
                gyt = rnd(*yt.shape, cl=cl)
                put(f"tdgrad_{tag}", lambda: ops.conv_transpose2d_dgrad(gyt, wt, xt, s, p, m))
    for c in (128, 64):
        x = rnd(16, c, 16, 16)
        gam = (torch.rand(c, c, device=dev, generator=g) * 0.1).contiguous()
        bet = (torch.rand(c, device=dev, generator=g) + 0.5).contiguous()
        for inv in (False, True):
            r = put(f"gdn_{mname}_{c}_{inv}_y", lambda: ops.gdn_fwd(x, gam, bet, inv, m))
            if r is not None:
                res[f"gdn_{mname}_{c}_{inv}_norm"] = r[1].clone()
                dyg = rnd(*x.shape)
                put(f"gdn_{mname}_{c}_{inv}_dx", lambda: ops.gdn_bwd(x, r[1], dyg, gam, inv, m))
torch.cuda.synchronize()
if a.out:
    torch.save({k: v.cpu() for k, v in res.items()}, a.out); print("saved", len(res))
if a.ref:
    ref = torch.load(a.ref, weights_only=True)
    bad = [k for k in ref if not torch.equal(ref[k], res[k].cpu())]
    for k in bad:
        d = (ref[k] - res[k].cpu()).abs().max().item(); print("DIFF", k, d, ref[k].abs().max().item())
    print("bitwise equal" if not bad else f"{len(bad)} of {len(ref)} differ", len(ref), "tensors")
    sys.exit(1 if bad else 0)
