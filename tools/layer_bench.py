#!/usr/bin/env python3
"""Per-layer timing of every conv / GDN op of one C2 training step (batch 32,
256x256, 192/192 channels) through the C ABI, with HIP events on torch's
current stream.  Prints one row per op: ms, algorithmic GFLOP, TFLOP/s and the
fraction of the fp32 MFMA peak.  GPU only.

    python tools/layer_bench.py [--batch 32] [--size 256] [--reps 5] [--json out.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from image_compression_amd import _lib  # noqa: E402

PEAK = 157.3
CL = torch.channels_last


ONLY = None


def t_ms(fn, reps, tag=None):
    if ONLY is not None and tag is not None and not any(o in tag for o in ONLY.split(",")):
        return float("nan")
    fn()
    torch.cuda.synchronize()
    st = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        fn()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def act_t(N, C, H, W, nchw=False):
    if nchw or C < 32:
        return torch.randn(N, C, H, W, device="cuda")
    return torch.randn(N, C, H, W, device="cuda").contiguous(memory_format=CL)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--size", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--json", default=None)
    ap.add_argument("--only", default=None, help="run only ops whose 'layer op' contains this text (comma-separated alternatives)")
    ap.add_argument("--math", type=int, default=0, help="IC_MATH_* of the conv fwd / dgrad / wgrad (0 fp32, 2 fp32 split)")
    ap.add_argument("--gdn-math", type=int, default=0, help="IC_MATH_* of the GDN forward")
    a = ap.parse_args()
    global ONLY
    ONLY = a.only
    L = _lib.load()
    st = _lib.c_void(torch.cuda.current_stream().cuda_stream)
    N, S = a.batch, a.size
    rows = []

    def ws(n):
        return _lib.workspace(n, "cuda")

    def conv_layer(name, cin, cout, hin, k, s, p, transposed, op=0):
        if transposed:
            hout = (hin - 1) * s - 2 * p + k + op
            w = torch.randn(cin, cout, k, k, device="cuda") * 0.02
        else:
            hout = (hin + 2 * p - k) // s + 1
            w = torch.randn(cout, cin, k, k, device="cuda") * 0.02
        x = act_t(N, cin, hin, hin)
        y = act_t(N, cout, hout, hout)
        b = torch.zeros(cout, device="cuda")
        ax, ay = _lib.act(x), _lib.act(y)
        # algorithmic MACs of the forward (identical for dgrad and wgrad)
        if transposed:
            macs = N * hin * hin * cin * cout * k * k
        else:
            macs = N * hout * hout * cin * cout * k * k
        gf = 2.0 * macs / 1e9
        pref = "ic_conv_transpose2d" if transposed else "ic_conv2d"
        fwd, fws = getattr(L, pref + "_fwd"), getattr(L, pref + "_fwd_ws")
        dg, dgws = getattr(L, pref + "_dgrad"), getattr(L, pref + "_dgrad_ws")
        wg, wgws = getattr(L, pref + "_wgrad"), getattr(L, pref + "_wgrad_ws")
        if a.math:
            fwd_ex, fws_ex = getattr(L, pref + "_fwd_ex"), getattr(L, pref + "_fwd_ws_ex")
            dg_ex, dgws_ex = getattr(L, pref + "_dgrad_ex"), getattr(L, pref + "_dgrad_ws_ex")
            fws = lambda *q: fws_ex(*q, a.math)  # noqa: E731
            fwd = lambda *q: fwd_ex(*q[:8], a.math, *q[8:])  # noqa: E731
            dgws = lambda *q: dgws_ex(*q, a.math)  # noqa: E731
            dg = lambda *q: dg_ex(*q[:6], a.math, *q[6:])  # noqa: E731
            wg_ex, wgws_ex = getattr(L, pref + "_wgrad_ex"), getattr(L, pref + "_wgrad_ws_ex")
            wgws = lambda *q: wgws_ex(*q, a.math)  # noqa: E731
            wg = lambda *q: wg_ex(*q[:7], a.math, *q[7:])  # noqa: E731
        n1 = fws(ax, k, s, p, ay)
        b1 = ws(n1)
        ms = t_ms(lambda: _lib.check(fwd(ax, _lib.ptr(w), _lib.ptr(b), k, s, p, ay, 0, _lib.ptr(b1), n1, st), "fwd"), a.reps, name + " fwd")
        rows.append((name, "fwd", ms, gf))
        if not (name.startswith("g_a.0")):
            n2 = dgws(ay, k, s, p, ax)
            b2 = ws(n2)
            ms = t_ms(lambda: _lib.check(dg(ay, _lib.ptr(w), k, s, p, ax, _lib.ptr(b2), n2, st), "dgrad"), a.reps, name + " dgrad")
            rows.append((name, "dgrad", ms, gf))
        dw = torch.empty_like(w)
        db = torch.empty(cout, device="cuda")
        n3 = wgws(ax, ay, k, s, p)
        b3 = ws(n3)
        ms = t_ms(lambda: _lib.check(wg(ax, ay, k, s, p, _lib.ptr(dw), _lib.ptr(db), _lib.ptr(b3), n3, st), "wgrad"), a.reps, name + " wgrad")
        rows.append((name, "wgrad", ms, gf))

    def gdn_layer(name, c, h):
        x = act_t(N, c, h, h)
        y = torch.empty_like(x)
        nrm = torch.empty_like(x)
        gy = torch.randn_like(x)
        g = (torch.eye(c, device="cuda") * 0.1 + 0.001).reshape(c, c, 1, 1).contiguous()
        be = torch.ones(c, device="cuda")
        ax, ay = _lib.act(x), _lib.act(y)
        gf = 2.0 * N * h * h * c * c / 1e9
        n1 = L.ic_gdn_fwd_ws_ex(ax, a.gdn_math)
        b1 = ws(n1)
        ms = t_ms(lambda: _lib.check(L.ic_gdn_fwd_ex(ax, _lib.ptr(g), _lib.ptr(be), 0, ay, _lib.ptr(nrm), a.gdn_math,
                                                     _lib.ptr(b1), n1, st), "gdn"), a.reps, name + " gdn_fwd")
        rows.append((name, "gdn_fwd", ms, gf))
        dx = torch.empty_like(x)
        dg = torch.empty_like(g)
        dbe = torch.empty_like(be)
        n2 = L.ic_gdn_bwd_ws(ax)
        b2 = ws(n2)
        ms = t_ms(lambda: _lib.check(L.ic_gdn_bwd_ex(ax, _lib.ptr(nrm), _lib.ptr(gy), _lib.ptr(g), 0, _lib.act(dx),
                                                     _lib.ptr(dg), _lib.ptr(dbe), a.math, _lib.ptr(b2), n2, st), "gdnb"),
                  a.reps, name + " gdn_bwd")
        rows.append((name, "gdn_bwd", ms, 2 * gf))

    h = S
    conv_layer("g_a.0 conv3->192", 3, 192, h, 5, 2, 2, False)
    gdn_layer("g_a.1 gdn", 192, h // 2)
    conv_layer("g_a.2 conv", 192, 192, h // 2, 5, 2, 2, False)
    gdn_layer("g_a.3 gdn", 192, h // 4)
    conv_layer("g_a.4 conv", 192, 192, h // 4, 5, 2, 2, False)
    gdn_layer("g_a.5 gdn", 192, h // 8)
    conv_layer("g_a.6 conv", 192, 192, h // 8, 5, 2, 2, False)
    conv_layer("h_a.0 conv3x3", 192, 192, h // 16, 3, 1, 1, False)
    conv_layer("h_a.2 conv", 192, 192, h // 16, 5, 2, 2, False)
    conv_layer("h_a.4 conv", 192, 192, h // 32, 5, 2, 2, False)
    conv_layer("h_s.0 tconv", 192, 192, h // 64, 5, 2, 2, True, 1)
    conv_layer("h_s.2 tconv", 192, 192, h // 32, 5, 2, 2, True, 1)
    conv_layer("h_s.4 tconv3x3", 192, 192, h // 16, 3, 1, 1, True, 0)
    conv_layer("g_s.0 tconv", 192, 192, h // 16, 5, 2, 2, True, 1)
    gdn_layer("g_s.1 gdn", 192, h // 8)
    conv_layer("g_s.2 tconv", 192, 192, h // 8, 5, 2, 2, True, 1)
    gdn_layer("g_s.3 gdn", 192, h // 4)
    conv_layer("g_s.4 tconv", 192, 192, h // 4, 5, 2, 2, True, 1)
    gdn_layer("g_s.5 gdn", 192, h // 2)
    conv_layer("g_s.6 tconv192->3", 192, 3, h // 2, 5, 2, 2, True, 1)

    tot_ms = sum(r[2] for r in rows)
    tot_gf = sum(r[3] for r in rows)
    print(f"{'layer':22s} {'op':8s} {'ms':>8s} {'GFLOP':>8s} {'TF/s':>7s} {'frac':>6s}")
    rows = [r for r in rows if r[2] == r[2]]  # drop skipped (nan) ops
    tot_ms = sum(r[2] for r in rows)
    tot_gf = sum(r[3] for r in rows)
    for name, op, ms, gf in rows:
        tf = gf / ms
        print(f"{name:22s} {op:8s} {ms:8.3f} {gf:8.1f} {tf:7.1f} {tf / PEAK:6.3f}")
    print(f"{'TOTAL':22s} {'':8s} {tot_ms:8.3f} {tot_gf:8.1f} {tot_gf / tot_ms:7.1f} {tot_gf / tot_ms / PEAK:6.3f}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump({"batch": N, "size": S, "rows": [dict(layer=r[0], op=r[1], ms=r[2], gflop=r[3]) for r in rows]}, f, indent=1)


if __name__ == "__main__":
    main()
