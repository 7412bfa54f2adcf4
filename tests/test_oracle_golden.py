"""Pin the CPU oracle (oracle/ref_cpu.py) against golden vectors produced by the
real reference (tools/gen_golden.py).  CPU only."""
import numpy as np
import pytest
import torch

import os

from conftest import (GOLDEN, assert_close, check_round_ties, golden_names, load_golden, oracle_kwargs,
                      params_of, rel_err)
from oracle import ref_cpu

SMALL = golden_names("small_")


@pytest.mark.parametrize("name", SMALL)
@pytest.mark.parametrize("dtype", [torch.float32, torch.float64])
def test_oracle_matches_reference(name, dtype):
    meta, d = load_golden(name)
    train = meta["train"]
    out, losses, grads = ref_cpu.run(
        params_of(d), d["x"], d["u_z"] if train else None,
        d["u_y"] if train else None, train=train, dtype=dtype, **oracle_kwargs(meta))
    tol = 2e-5 if dtype == torch.float32 else 1e-4
    if not train:
        # eval rounds (entropy_model.py:234,337): every symbol equals the reference's except on
        # a .5 tie; with a flip the reference's own symbols are fed and the rest held to tol
        for k in ("y", "z"):
            assert_close(out[k].detach().numpy(), d["out/" + k], tol, name=f"{name}:{k}")
        flips = (check_round_ties(out["z_tilde"].detach().numpy(), d["out/z"], name="z_tilde")
                 + check_round_ties(out["y_tilde"].detach().numpy(), d["out/y"], name="y_tilde"))
        if flips:
            out, losses, grads = ref_cpu.run(params_of(d), d["x"], train=False, dtype=dtype, sym_z=d["out/z_tilde"],
                                             sym_y=d["out/y_tilde"], **oracle_kwargs(meta))
    for k in ["y", "z", "z_tilde", "p_z", "sigma", "y_tilde", "p_y", "x_tilde_raw", "x_tilde"]:
        assert_close(out[k].detach().numpy(), d["out/" + k], tol, name=f"{name}:{k}")
    for k in meta["loss_names"] + ["total_loss"]:
        assert_close(losses[k].detach().numpy(), d["loss/" + k], tol, name=f"{name}:loss:{k}")
    for k, g in grads.items():
        ref = d["grad/" + k]
        assert rel_err(g.numpy(), ref) < (5e-5 if dtype == torch.float32 else 5e-4), (name, k, rel_err(g.numpy(), ref))


def test_gdn_known_answers():
    """The reference's own known-answer tests (test/test_gdn.py:20-48):
    at init GDN(x) = x / sqrt(1 + 0.1 x^2), IGDN = x * sqrt(...), RGDN = GDN(relu(x))."""
    torch.manual_seed(0)
    gp, bp = ref_cpu.gdn_init(3)
    x = torch.rand(2, 3, 4, 5)
    exp = x / torch.sqrt(1 + 0.1 * x ** 2)
    assert (ref_cpu.gdn(x, gp, bp) - exp).abs().max() <= 1e-6
    exp = x * torch.sqrt(1 + 0.1 * x ** 2)
    assert (ref_cpu.gdn(x, gp, bp, inverse=True) - exp).abs().max() <= 1e-6
    x = torch.rand(2, 3, 4, 5) - 0.5
    xr = torch.clamp(x, min=0)
    exp = xr / torch.sqrt(1 + 0.1 * xr ** 2)
    assert (ref_cpu.gdn(x, gp, bp, relu=True) - exp).abs().max() <= 1e-6


def test_oracle_eval_metrics_match_reference():
    """oracle/ref_cpu.py psnr_metric / ms_ssim_metric_db vs the reference's
    utils/metric.py (tests/golden/eval_metrics.npz)."""
    import torch
    from test_eval import _metric_inputs
    gold = np.load(os.path.join(GOLDEN, "eval_metrics.npz"))
    for name, (x, xt) in _metric_inputs().items():
        p = ref_cpu.psnr_metric(xt * 255.0, x * 255.0).numpy()
        m = ref_cpu.ms_ssim_metric_db(xt * 255.0, x * 255.0).numpy()
        assert np.abs(p - gold[f"{name}_psnr"]).max() < 1e-4
        assert np.abs(m - gold[f"{name}_msssim_db"]).max() < 1e-4
