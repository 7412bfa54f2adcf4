"""Parity at the kernel instances the benchmark runs.

The implicit GEMM and weight-gradient kernels pick their tile and K / pixel
split from the problem size (ic_conv_plan; csrc/igemm.hip ig_plan, csrc/wgrad.hip
wg_plan): the 128-row, no-split-K tiles only appear once a layer has >= 65,536
output pixels, i.e. at the BASELINE configurations' batch sizes.  These tests
  * check single layers at C2 shapes (16 x 192 x 128^2 convs, 16 x 192 x 64^2
    transposed convs) against fp64 torch, asserting the plan they ran;
  * run one whole training step per BASELINE config against the fp64 oracle --
    at the benchmark's own batch for C2 / C3 / C4 / C5 (32, 32, 16 x 256^2 and 16 x 512^2)
    -- and assert that every kernel instance the benchmark's batch
    launches (recorded through functional.record_plans on a bench-size step)
    was launched by the test step.  The oracle takes the HIP path's
    hyperprior ReLU masks; a mask may differ only where the pre-activation is
    a tie (|pre| <= 1e-4 max|pre|, 2e-2 with bf16 operands; conftest.check_relu_ties).
Reference: modelling/meta_arch/bmshl2018.py:68-98 (the step), analysis.py:55 /
synthesis.py:55 (the layers)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import HipReluMasks, MainLayerIO, assert_close, c3_check, check_relu_ties, rel_err

pytestmark = pytest.mark.gpu
DEV = "cuda"
CL = torch.channels_last


def _r(*shape, seed, scale=1.0):
    return torch.randn(*shape, generator=torch.Generator().manual_seed(seed)) * scale


def _key(p):
    """kernel instance: op, kernel, tile, split-K or not, template variant, column buffer"""
    return (p["op"], p["kernel"], p["bm"], p["bn"], p["ksplit"] > 1, p["variant"], p["im2col"])


# ------------------------------------------------------------------ single layers at C2 shapes
@pytest.mark.parametrize("math", [2, 1])
def test_c2_conv_layer(math):
    """g_a.2: conv 192 -> 192, 5x5 stride 2, 16 x 192 x 128^2 -> 64^2 (the roofline kernel)."""
    from image_compression_amd import _lib, functional as IF
    torch.set_num_threads(16)
    x = _r(16, 192, 128, 128, seed=1)
    w = _r(192, 192, 5, 5, seed=2, scale=0.02)
    b = _r(192, seed=3, scale=0.1)
    xd = x.to(DEV).contiguous(memory_format=CL).requires_grad_(True)
    wd = w.to(DEV).requires_grad_(True)
    y = IF.conv2d(xd, wd, b.to(DEV), 2, 2, math=math)
    gy = _r(*y.shape, seed=4).to(DEV).contiguous(memory_format=CL)
    y.backward(gy)
    kern, bm = {2: ("ig_split_dma", 256), 1: ("ig_bf16", 128)}[math]
    pf = _lib.plan("conv2d_fwd", xd.detach(), y.detach(), 5, 2, 2, math)
    pd = _lib.plan("conv2d_dgrad", gy, xd.detach(), 5, 2, 2, math)
    pw = _lib.plan("conv2d_wgrad", xd.detach(), gy, 5, 2, 2, math)
    # bf16 operands: the forward and the four-phase dgrad on the DMA tiles (ig_kernel_b16d)
    if math == 1:
        kern, bm = "ig_bf16_dma", 256
    assert (pf["kernel"], pf["bm"], pf["ksplit"]) == (kern, bm, 1), pf
    assert (pd["kernel"], pd["bm"], pd["ksplit"]) == (kern, bm, 1), pd
    # weight gradients: split arithmetic, or bf16 operands on the same two-wave kernel
    assert (pw["kernel"], pw["variant"]) == ("wg_split" if math == 2 else "wg_bf16", 1), pw
    xr = x.double().requires_grad_(True)
    wr = w.double().requires_grad_(True)
    yr = F.conv2d(xr, wr, b.double(), stride=2, padding=2)
    yr.backward(gy.double().cpu())
    tol = 1e-4 if math == 2 else 1e-2
    if math == 2:
        assert_close(y.detach().cpu(), yr.detach(), tol, "y")
        assert_close(xd.grad.cpu(), xr.grad, tol, "dx")
    else:  # bf16 operands: normwise bar
        assert rel_err(y.detach().cpu(), yr.detach()) < tol
        assert rel_err(xd.grad.cpu(), xr.grad) < tol
    if math == 2:
        assert_close(wd.grad.cpu(), wr.grad, 1e-4, "dw")
    else:
        assert rel_err(wd.grad.cpu(), wr.grad) < tol


@pytest.mark.parametrize("math", [2, 1])
def test_c2_tconv_layer(math):
    """g_s.4: transposed conv 192 -> 192, 5x5 stride 2, 16 x 192 x 64^2 -> 128^2."""
    from image_compression_amd import _lib, functional as IF
    torch.set_num_threads(16)
    x = _r(16, 192, 64, 64, seed=5)
    w = _r(192, 192, 5, 5, seed=6, scale=0.02)
    xd = x.to(DEV).contiguous(memory_format=CL).requires_grad_(True)
    wd = w.to(DEV).requires_grad_(True)
    y = IF.conv_transpose2d(xd, wd, None, 2, 2, 1, math=math)
    gy = _r(*y.shape, seed=7).to(DEV).contiguous(memory_format=CL)
    y.backward(gy)
    kern, bm = {2: ("ig_split_dma", 256), 1: ("ig_bf16", 128)}[math]
    pf = _lib.plan("conv_transpose2d_fwd", xd.detach(), y.detach(), 5, 2, 2, math)
    pd = _lib.plan("conv_transpose2d_dgrad", gy, xd.detach(), 5, 2, 2, math)
    pw = _lib.plan("conv_transpose2d_wgrad", xd.detach(), gy, 5, 2, 2, math)
    # bf16 operands: the four-phase forward and the one-phase dgrad on the DMA tiles (ig_kernel_b16d)
    if math == 1:
        kern, bm = "ig_bf16_dma", 256
    assert (pf["kernel"], pf["bm"], pf["ksplit"]) == (kern, bm, 1), pf
    assert (pd["kernel"], pd["bm"], pd["ksplit"]) == (kern, bm, 1), pd
    assert pw["kernel"] == ("wg_split" if math == 2 else "wg_bf16"), pw
    xr = x.double().requires_grad_(True)
    wr = w.double().requires_grad_(True)
    yr = F.conv_transpose2d(xr, wr, None, stride=2, padding=2, output_padding=1)
    yr.backward(gy.double().cpu())
    tol = 1e-4 if math == 2 else 1e-2
    if math == 2:
        assert_close(y.detach().cpu(), yr.detach(), tol, "y")
        assert_close(xd.grad.cpu(), xr.grad, tol, "dx")
    else:
        assert rel_err(y.detach().cpu(), yr.detach()) < tol
        assert rel_err(xd.grad.cpu(), xr.grad) < tol
    if math == 2:
        assert_close(wd.grad.cpu(), wr.grad, 1e-4, "dw")
    else:
        assert rel_err(wd.grad.cpu(), wr.grad) < tol


# ------------------------------------------------------------------ whole steps per BASELINE config
CONFIGS = {
    # name: (bench batch, test batch, size, compute dtype, latent, loss, lambda)
    "C2": (32, 32, 256, "fp32_split", 192, "mse", 256.0),
    "C3": (32, 32, 256, "bf16", 320, "mse", 4096.0),
    "C4": (16, 16, 256, "fp32_split", 192, "msssim", 64.0),
    "C5": (16, 16, 512, "fp32_split", 192, "mse", 8192.0),  # the bench batch: tile choices depend on it
}


def _model(dtype, latent, loss, lam):
    from image_compression_amd import get_cfg_defaults, modelling
    cfg = get_cfg_defaults()
    cfg.MODEL.LOSS.REDUCTION = "mean"
    cfg.MODEL.LOSS.DISTORTION_LOSS_WEIGHT = lam
    cfg.MODEL.LATENT_CHANNELS = latent
    cfg.MODEL.COMPUTE_DTYPE = dtype
    if loss == "msssim":
        cfg.MODEL.LOSS.DISTORTION_LOSS_NAMES = ["MS_SSIMLoss"]
        cfg.MODEL.LOSS.SSIM.LOG_SCALE = True
    torch.manual_seed(0)
    return modelling.build_model(cfg)


def _step_plans(model, n, size, latent):
    from image_compression_amd import functional as IF, injected_noise
    g = torch.Generator().manual_seed(11)
    x = torch.rand(n, 3, size, size, generator=g).to(DEV)
    uz = torch.rand(n, 192, size // 64, size // 64, generator=g).to(DEV)
    uy = torch.rand(n, latent, size // 16, size // 16, generator=g).to(DEV)
    with IF.record_plans() as log, injected_noise([uz, uy]):
        _, losses = model(x)
        losses["total_loss"].backward()
    torch.cuda.synchronize()
    model.zero_grad(set_to_none=True)
    return {_key(p) for p in log}


@pytest.mark.parametrize("name", list(CONFIGS))
def test_config_step_vs_oracle_and_bench_plans(name):
    from image_compression_amd import functional as IF, injected_noise
    from oracle import ref_cpu
    bench_n, n, size, dtype, latent, loss, lam = CONFIGS[name]
    torch.set_num_threads(16)
    model = _model(dtype, latent, loss, lam)
    params = {k: v.clone() for k, v in model.state_dict().items()}
    model = model.to(DEV).train()
    bench_plans = _step_plans(model, bench_n, size, latent)
    g = torch.Generator().manual_seed(3)
    x = torch.rand(n, 3, size, size, generator=g)
    uz = torch.rand(n, 192, size // 64, size // 64, generator=g)
    uy = torch.rand(n, latent, size // 16, size // 16, generator=g)
    hm = HipReluMasks(model)
    lio = MainLayerIO(model) if dtype == "bf16" else None
    with IF.record_plans() as log, injected_noise([uz.to(DEV), uy.to(DEV)]):
        xt, losses = model(x.to(DEV))
        losses["total_loss"].backward()
    hm.remove()
    if lio:
        lio.remove()
    test_plans = {_key(p) for p in log}
    missing = bench_plans - test_plans
    assert not missing, f"bench kernel instances this test does not reach: {sorted(missing)}"
    # the oracle takes the HIP path's hyperprior ReLU masks; a mask may differ only on a tie
    ctl = {"masks": hm.masks}
    kw = dict(lam=lam, relu_ctl=ctl)
    if loss == "msssim":
        kw.update(loss_names=("MS_SSIMLoss",), ssim_log=True)
    if dtype == "bf16":
        c3_check(model, params, x, uz, uy, xt, losses, hm.masks, log, lam, latent, lio, name)
        return
    out, ref_losses, ref_grads = ref_cpu.run(params, x, uz, uy, train=True, dtype=torch.float64, **kw)
    flips = check_relu_ties(hm.masks, ctl, tau=1e-4)
    errs = {k: rel_err(p.grad.cpu(), ref_grads[k]) for k, p in model.named_parameters()}
    worst = sorted(((e, k) for k, e in errs.items()), reverse=True)[:5]
    print(f"{name}: x_tilde {rel_err(xt.cpu(), out['x_tilde'].detach()):.2e}; ReLU ties {flips}; worst grads {worst}")
    assert_close(xt.cpu(), out["x_tilde"].detach(), 1e-4, "x_tilde")
    for k in ["total_loss", "bpp"] + (["MS_SSIMLoss"] if loss == "msssim" else ["MSE"]):
        a, b = float(losses[k].detach()), float(ref_losses[k].detach())
        assert abs(a - b) <= 1e-4 * abs(b), (k, a, b)
    for k, e in errs.items():
        assert e < 1e-4, (k, e, worst)
