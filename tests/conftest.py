import glob
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")
    # an AccumulateGrad node fed from another stream than its own is a cross-stream use of a
    # gradient's memory that the caching allocator is not told about: an error everywhere
    config.addinivalue_line("filterwarnings", "error:(?s).*AccumulateGrad node's stream does not match")


def load_golden(name):
    d = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    meta = json.loads(str(d["meta"]))
    return meta, d


def golden_names(prefix=""):
    return sorted(os.path.basename(p)[:-4]
                  for p in glob.glob(os.path.join(GOLDEN, prefix + "*.npz")))


def params_of(d):
    return {k[len("param/"):]: d[k] for k in d.files if k.startswith("param/")}


def oracle_kwargs(meta):
    over = meta["over"]
    cond = over.get("MODEL.ENTROPY_MODEL.CONDITIONAL_MODEL", "LaplacianConditionalModel")
    return dict(
        cond="laplace" if cond.startswith("Laplacian") else "gauss",
        loss_names=tuple(over.get("MODEL.LOSS.DISTORTION_LOSS_NAMES", ["MSE"])),
        lam=float(over.get("MODEL.LOSS.DISTORTION_LOSS_WEIGHT", 1.0)),
        ssim_log=bool(over.get("MODEL.LOSS.SSIM.LOG_SCALE", False)),
        bin_=float(over.get("MODEL.ENTROPY_MODEL.BIN", 1.0)),
    )


def rel_err(a, b):
    """normwise relative error ||a-b|| / ||b||"""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    nb = np.linalg.norm(b)
    return float(np.linalg.norm(a - b) / (nb if nb > 0 else 1.0))


def assert_close(a, b, rtol=1e-4, name=""):
    """The parity criterion of SURVEY.md 8(c): allclose(rtol, atol=rtol*max|ref|)."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    assert a.shape == b.shape, (name, a.shape, b.shape)
    atol = rtol * max(float(np.abs(b).max()) if b.size else 0.0, 1e-30)
    bad = np.abs(a - b) > (atol + rtol * np.abs(b))
    if bad.any():
        i = np.argmax(np.abs(a - b))
        raise AssertionError(
            f"{name}: {int(bad.sum())}/{a.size} elements off; max|d|={np.abs(a-b).max():.3e} "
            f"at {np.unravel_index(i, a.shape)} a={a.flat[i]:.6g} b={b.flat[i]:.6g} atol={atol:.3e}")


def check_round_ties(sym, pre, tau=1e-4, name=""):
    """Eval-mode rounding (entropy_model.py:234,337: torch.round, half to even): every symbol
    of `sym` (the HIP path's) must equal round(`pre`) (the reference's / oracle's pre-round
    value), except where `pre` sits on a tie: within tau * max|pre| of a .5 boundary, where two
    correct fp32 evaluations may round either way; there the two symbols must be
    the two neighbours of the boundary.  Returns the number of such flips."""
    sym = np.asarray(sym, dtype=np.float64)
    pre = np.asarray(pre, dtype=np.float64)
    assert sym.shape == pre.shape, (name, sym.shape, pre.shape)
    assert np.array_equal(sym, np.round(sym)), f"{name}: symbols are not integers"
    diff = sym != np.round(pre)
    if diff.any():
        lim = tau * max(float(np.abs(pre).max()), 1e-30)
        d = np.abs(np.abs(pre - np.floor(pre)) - 0.5)[diff]
        assert float(d.max()) <= lim, (f"{name}: {int(diff.sum())} symbol(s) differ, one {float(d.max()):.3e} "
                                       f"from a .5 boundary > {lim:.3e}")
        assert np.all(np.abs(sym[diff] - np.round(pre[diff])) == 1), name
        assert np.all(np.abs(sym[diff] - pre[diff]) <= 0.5 + lim), name
    return int(diff.sum())


class HipReluMasks:
    """Records, in call order, the gradient masks (input > 0) of the HIP model's
    hyperprior ReLUs (the only ReLUs of Compressor2018), for the oracle's
    relu_ctl (oracle/ref_cpu.py _relu)."""

    def __init__(self, model):
        self.masks = []
        self.handles = []
        for blk in (model.prior_analysis, model.prior_synthesis):
            for m in blk.modules():
                if type(m).__name__ == "ReLU":
                    self.handles.append(m.register_forward_hook(
                        lambda mod, inp, out: self.masks.append((inp[0] > 0).detach().cpu())))

    def remove(self):
        for h in self.handles:
            h.remove()


def check_relu_ties(masks, ctl, tau=1e-4):
    """Every ReLU mask the HIP path and the oracle disagree on must sit on a tie:
    |oracle pre-activation| <= tau * max |pre-activation| of that layer.
    Returns the number of disagreements."""
    assert len(masks) == len(ctl["pre"]), (len(masks), len(ctl["pre"]))
    flips = 0
    for i, (m, pre) in enumerate(zip(masks, ctl["pre"])):
        pre = pre.double()
        diff = m != (pre > 0)
        if diff.any():
            lim = tau * float(pre.abs().max())
            worst = float(pre[diff].abs().max())
            assert worst <= lim, f"ReLU {i}: mask differs at |pre| = {worst:.3e} > {lim:.3e}"
            flips += int(diff.sum())
    return flips


BF16_KERNELS = ("ig_bf16", "ig_split_bf16", "wg_bf16", "gdn_fused_bf16", "edge_conv_bf16", "tconv_few_rows_bf16",
                "edge_wgrad_bf16", "ig_bf16_dma")


def edges_bf16():
    """Whether this build runs C3's 3-channel image edges on bf16 operands (csrc/conv_api.hip
    EDGE_BF16), from the library's own plan query (no launch)."""
    from image_compression_amd import _lib
    img = _lib.ICAct(256, 2, 3, 64, 64, 3 * 64 * 64, 64 * 64, 64, 1)
    x = _lib.ICAct(256, 2, 192, 32, 32, 192 * 32 * 32, 1, 32 * 192, 192)
    return _lib.plan("conv2d_fwd", img, x, 5, 2, 2, 3)["kernel"] == "edge_conv_bf16"


def c3_bf16_flags(n, size, latent, edges=None):
    """Which GEMMs of the convolutions take bf16 operands in the "bf16" compute dtype
    (BASELINE config C3), per weight name: (forward, input gradient, weight gradient) — the
    rule of csrc/conv_api.hip and csrc/wgrad.hip wg_plan, restated: conv / transposed-conv
    forward and input gradient on the implicit GEMM when the reduction channels are a multiple
    of 64; weight gradients when both channel counts
    are >= 128 and the output-gradient grid (transposed: the input grid) is >= 16 wide with
    row-aligned 32-pixel steps; the 3-channel image edges (csrc/edge.hip, NP = 1) in every GEMM they
    run when the build has them on (edges_bf16); the GDN forward's Gamma x^2 and the backward's two contractions (csrc/gdn_fused.hip).  Returns (flags for oracle.ref_cpu's bf16 emulation, the number
    of bf16 launches one training step makes)."""
    flags, launches = {}, 0
    e = edges_bf16() if edges is None else edges

    def wg_ok(cg, cx, w_, p_):
        return cg >= 128 and cx >= 128 and w_ % 16 == 0 and (w_ % 32 == 0 or p_ % 32 == 0)

    ch = [3, 192, 192, 192, latent]
    for i in range(4):  # analysis: conv ch[i] -> ch[i+1], output size / 2^(i+1)
        cin, cout, wo = ch[i], ch[i + 1], size >> (i + 1)
        # the 3-channel image edge (i = 0) on the edge kernels: forward and weight gradient (the
        # image needs no gradient)
        f = (cin % 64 == 0 or (e and cin <= 4), i > 0 and cout % 64 == 0,
             (e and cin <= 4) or (cin > 4 and wg_ok(cout, cin, wo, n * wo * wo)))
        flags[f"analysis_transform.layers.{2 * i}.weight"] = f
        launches += sum(f)
    ch = [latent, 192, 192, 192, 3]
    for i in range(4):  # synthesis: tconv ch[i] -> ch[i+1], input size / 2^(4-i)
        cin, cout, wi = ch[i], ch[i + 1], size >> (4 - i)
        # the image edge (cout 3): forward, input and weight gradient on the edge kernels
        f = (cin % 64 == 0 and (e or cout > 4), cout % 64 == 0 or (e and cout <= 4),
             (e and cout <= 4) or (cout > 4 and wg_ok(cin, cout, wi, n * wi * wi)))
        flags[f"synthesis_transform.layers.{2 * i}.weight"] = f
        launches += sum(f)
    # the hyperprior (round 6): every forward and input gradient (reduction channels 192 or the
    # latent, multiples of 64); the weight gradients of the two 16-wide 3x3 layers by the same rule
    s16 = size // 16
    hyp = (("prior_analysis._layers.0.weight", s16, latent, 192), ("prior_analysis._layers.2.weight", s16 // 2, 192, 192),
           ("prior_analysis._layers.4.weight", s16 // 4, 192, 192))
    for nm, wo, cin, cout in hyp:  # conv: G = dy (cout channels) on the output grid wo
        f = (cin % 64 == 0, cout % 64 == 0, wg_ok(cout, cin, wo, n * wo * wo))
        flags[nm] = f
        launches += sum(f)
    hyp = (("prior_synthesis._layers.0.weight", s16 // 4, 192, 192), ("prior_synthesis._layers.2.weight", s16 // 2, 192, 192),
           ("prior_synthesis._layers.4.weight", s16, 192, latent))
    for nm, wi, cin, cout in hyp:  # transposed conv: the roles of conv wgrad with x on the input grid wi
        f = (cin % 64 == 0, cout % 64 == 0, wg_ok(cin, cout, wi, n * wi * wi))
        flags[nm] = f
        launches += sum(f)
    # every GDN (C = 192, NHWC-dense: the fused kernels) has a bf16 forward and backward
    for t in ("analysis_transform", "synthesis_transform"):
        for i in range(3):
            flags[f"{t}.layers.{2 * i + 1}.gamma.param"] = (True, True)
            launches += 2
    return flags, launches


class MainLayerIO:
    """Records, during a HIP step, every main-transform layer's (input, output) (forward hooks
    on analysis_transform / synthesis_transform layers), for c3_check's per-layer comparison."""

    def __init__(self, model):
        self.io, self.handles = [], []
        for tname in ("analysis_transform", "synthesis_transform"):
            for i, m in enumerate(getattr(model, tname).layers):
                self.handles.append(m.register_forward_hook(
                    lambda mod, inp, out, nm=f"{tname}.layers.{i}": self.io.append(
                        (nm, type(mod).__name__, inp[0].detach().cpu(), out.detach().cpu()))))

    def remove(self):
        for h in self.handles:
            h.remove()


def c3_check(model, params, x, uz, uy, xt, losses, masks, log, lam, latent, layer_io, name="C3"):
    """One C3 (bf16) training step of the HIP model against the fp64 oracle.

    bf16 operands make the step a chaotic function of rounding boundaries: the HIP step and an
    fp64 step with the same bf16-rounded operands (oracle.ref_cpu._conv emulation) agree per
    layer to fp32 accuracy, yet a 1e-7 difference in a layer's input flips the bf16 rounding
    of a few operands, and the flips multiply layer by layer (measured: per layer 1e-7, end to
    end ~3e-3).  So the check is split:
      * the step's plan log shows exactly the bf16 launches of the rule (c3_bf16_flags);
      * every main-transform layer's HIP output equals the emulated layer on the HIP layer's own
        input within 1e-5 (layer_io: MainLayerIO) — the kernels compute what the config says;
      * the config's floor = the distance between the emulating and the exact fp64 oracle (an
        independent sample of the same rounding noise); x_tilde, the losses and every gradient
        must lie within 2x that floor (+1e-4) of the exact oracle.
    Prints the per-tensor floors."""
    import torch
    from oracle import ref_cpu
    n, size = x.shape[0], x.shape[2]
    flags, nb = c3_bf16_flags(n, size, latent)
    got = sum(p["kernel"] in BF16_KERNELS for p in log)
    assert got == nb, (f"{got} bf16 launches, the rule says {nb}",
                       sorted({(p["op"], p["kernel"]) for p in log}))
    P = {k: v.double() for k, v in params.items()}
    for nm, kind, a, b in layer_io.io:
        a = a.double()
        if kind in ("Conv2d", "ConvTranspose2d"):
            tr = kind == "ConvTranspose2d"
            ref = ref_cpu._conv(a, P[nm + ".weight"], P[nm + ".bias"], 2, 2, nm + ".weight", flags, transposed=tr,
                                opad=1 if tr else 0)
        else:
            ref = ref_cpu.gdn(a, P[nm + ".gamma.param"], P[nm + ".beta.param"],
                              bf16_fwd=bool(flags[nm + ".gamma.param"][0]))
        e = rel_err(b, ref)
        assert e < 1e-5, (nm, kind, e)
    ctl_x, ctl_e = {"masks": masks}, {"masks": masks}
    out_x, loss_x, g_x = ref_cpu.run(params, x, uz, uy, train=True, dtype=torch.float64, lam=lam, relu_ctl=ctl_x)
    out_e, loss_e, g_e = ref_cpu.run(params, x, uz, uy, train=True, dtype=torch.float64, lam=lam, relu_ctl=ctl_e,
                                     bf16=flags)
    # y (and so h_a's pre-activations) moves by the bf16 floor: a mask flip is a tie at that scale
    flips = check_relu_ties(masks, ctl_x, tau=2e-2)
    xt = xt.detach().cpu()
    e_x = rel_err(xt, out_x["x_tilde"].detach())
    floor_x = rel_err(out_e["x_tilde"].detach(), out_x["x_tilde"].detach())
    print(f"{name}: x_tilde vs exact {e_x:.2e}, floor {floor_x:.2e}; ReLU ties {flips}")
    assert e_x <= 2 * floor_x + 1e-4, (e_x, floor_x)
    for k in ("total_loss", "bpp", "MSE"):
        a, c, f = float(losses[k].detach()), float(loss_x[k].detach()), abs(float(loss_e[k].detach() - loss_x[k].detach()))
        assert abs(a - c) <= 2 * f + 1e-4 * abs(c), (k, a, c, f)
    rows = []
    for k, p in model.named_parameters():
        g = p.grad.cpu()
        rows.append((rel_err(g_e[k], g_x[k]), rel_err(g, g_x[k]), k))
    for floor, e_ex, k in sorted(rows, reverse=True)[:8]:
        print(f"   {k:55s} floor {floor:.2e}  HIP vs exact {e_ex:.2e}")
    for floor, e_ex, k in rows:
        assert e_ex <= 2 * floor + 1e-4, (k, e_ex, floor)
