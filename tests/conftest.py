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
