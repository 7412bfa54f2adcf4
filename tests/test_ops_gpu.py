"""Per-op parity: HIP kernels (through the C ABI) vs CPU fp64 references of
the same op (torch CPU ops / the oracle restatement).  GPU only."""
import math

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import assert_close, rel_err

pytestmark = pytest.mark.gpu

if torch.cuda.is_available():
    from image_compression_amd import functional as IF
    from oracle import ref_cpu

DEV = "cuda"


def _rand(*shape, seed=0, scale=1.0, cl=False):
    g = torch.Generator().manual_seed(seed)
    t = torch.randn(*shape, generator=g) * scale
    return t


def _to_dev(t, cl=False, grad=True):
    d = t.to(DEV)
    if cl and d.dim() == 4:
        d = d.contiguous(memory_format=torch.channels_last)
    return d.detach().requires_grad_(grad)


def _check_grads(pairs, rtol=1e-4):
    for name, a, b in pairs:
        assert a is not None, name
        assert_close(a.detach().cpu().double().numpy(), b.detach().double().numpy(), rtol, name)


CONV_CASES = [
    # N, Cin, H, W, Cout, k, stride, pad
    (2, 192, 16, 16, 192, 5, 2, 2),
    (2, 192, 8, 12, 192, 3, 1, 1),
    (2, 3, 32, 32, 192, 5, 2, 2),     # first analysis layer (generic gather)
    (1, 64, 9, 7, 96, 5, 2, 2),       # ragged sizes, Cout not a multiple of 192
    (2, 320, 8, 8, 192, 3, 1, 1),     # latent-320 hyper-analysis input
    (2, 192, 8, 8, 320, 5, 2, 2),
]


@pytest.mark.parametrize("case", CONV_CASES)
def test_conv2d_fwd_bwd(case):
    N, Cin, H, W, Cout, k, s, p = case
    x = _rand(N, Cin, H, W, seed=1)
    w = _rand(Cout, Cin, k, k, seed=2, scale=1.0 / math.sqrt(Cin * k * k))
    b = _rand(Cout, seed=3, scale=0.1)
    xr, wr, br = (t.double().requires_grad_(True) for t in (x, w, b))
    yr = F.conv2d(xr, wr, br, stride=s, padding=p)
    gy = _rand(*yr.shape, seed=4)
    yr.backward(gy.double())
    xd, wd, bd = _to_dev(x, cl=True), _to_dev(w), _to_dev(b)
    y = IF.conv2d(xd, wd, bd, s, p)
    y.backward(gy.to(DEV))
    assert_close(y.detach().cpu().numpy(), yr.detach().numpy(), 1e-4, "y")
    _check_grads([("dx", xd.grad, xr.grad), ("dw", wd.grad, wr.grad), ("db", bd.grad, br.grad)])


TCONV_CASES = [
    # N, Cin, H, W, Cout, k, stride, pad, outpad
    (2, 192, 8, 8, 192, 5, 2, 2, 1),
    (2, 192, 4, 6, 192, 3, 1, 1, 0),   # h_s last layer form
    (2, 192, 16, 16, 3, 5, 2, 2, 1),   # last synthesis layer (Cout = 3, NCHW out)
    (1, 64, 9, 7, 3, 5, 2, 2, 1),      # row-stationary few-channel kernel: ragged width
    (1, 32, 3, 70, 3, 5, 2, 2, 1),     # 2 m-tiles per wave
    (1, 16, 2, 130, 3, 3, 2, 1, 1),    # 4 m-tiles per wave, k = 3
    (1, 48, 6, 5, 4, 3, 2, 1, 1),      # Cout = 4
    (1, 32, 5, 5, 3, 5, 2, 2, 0),      # odd output height (no output padding)
    (3, 192, 20, 24, 3, 5, 2, 2, 1),   # input-row-stationary kernel: several runs per image, halo rows
    (1, 96, 5, 7, 64, 5, 2, 2, 1),
    (2, 320, 4, 4, 192, 5, 2, 2, 1),
]


@pytest.mark.parametrize("case", TCONV_CASES)
def test_conv_transpose2d_fwd_bwd(case):
    N, Cin, H, W, Cout, k, s, p, op = case
    x = _rand(N, Cin, H, W, seed=5)
    w = _rand(Cin, Cout, k, k, seed=6, scale=1.0 / math.sqrt(Cin * k * k / (s * s)))
    b = _rand(Cout, seed=7, scale=0.1)
    xr, wr, br = (t.double().requires_grad_(True) for t in (x, w, b))
    yr = F.conv_transpose2d(xr, wr, br, stride=s, padding=p, output_padding=op)
    gy = _rand(*yr.shape, seed=8)
    yr.backward(gy.double())
    xd, wd, bd = _to_dev(x, cl=True), _to_dev(w), _to_dev(b)
    y = IF.conv_transpose2d(xd, wd, bd, s, p, op)
    y.backward(gy.to(DEV))
    assert_close(y.detach().cpu().numpy(), yr.detach().numpy(), 1e-4, "y")
    _check_grads([("dx", xd.grad, xr.grad), ("dw", wd.grad, wr.grad), ("db", bd.grad, br.grad)])


@pytest.mark.parametrize("C,H,W,inverse", [(192, 16, 16, False), (192, 8, 5, True), (3, 4, 5, False), (64, 7, 7, False)])
def test_gdn_fwd_bwd(C, H, W, inverse):
    from image_compression_amd.modelling.layers import GDN
    torch.manual_seed(0)
    m = GDN(C, inverse=inverse)
    with torch.no_grad():  # perturb away from the identity-like init
        m.gamma.param.add_(torch.rand_like(m.gamma.param) * 0.05)
        m.beta.param.add_(torch.rand_like(m.beta.param) * 0.1)
    x = _rand(2, C, H, W, seed=9)
    gp = m.gamma.param.detach().double().requires_grad_(True)
    bp = m.beta.param.detach().double().requires_grad_(True)
    xr = x.double().requires_grad_(True)
    yr = ref_cpu.gdn(xr, gp, bp, inverse=inverse)
    gy = _rand(*yr.shape, seed=10)
    yr.backward(gy.double())
    md = m.to(DEV)
    xd = _to_dev(x, cl=C >= 32)
    y = md(xd)
    y.backward(gy.to(DEV))
    assert_close(y.detach().cpu().numpy(), yr.detach().numpy(), 1e-4, "y")
    _check_grads([("dx", xd.grad, xr.grad), ("dgamma", md.gamma.param.grad, gp.grad),
                  ("dbeta", md.beta.param.grad, bp.grad)])


def test_gdn_known_answers_gpu():
    """reference test/test_gdn.py:20-48 on the HIP path."""
    from image_compression_amd.modelling.layers import GDN
    x = torch.rand(2, 3, 4, 5)
    out = GDN(3).to(DEV)(x.to(DEV)).cpu()
    assert (out - x / torch.sqrt(1 + 0.1 * x ** 2)).abs().max() <= 1e-6
    out = GDN(3, inverse=True).to(DEV)(x.to(DEV)).cpu()
    assert (out - x * torch.sqrt(1 + 0.1 * x ** 2)).abs().max() <= 1e-6
    x = torch.rand(2, 3, 4, 5) - 0.5
    out = GDN(3, relu=True).to(DEV)(x.to(DEV)).cpu()
    xr = torch.clamp(x, min=0)
    assert (out - xr / torch.sqrt(1 + 0.1 * xr ** 2)).abs().max() <= 1e-6
    layer = GDN(3).to(DEV)
    layer(torch.rand(2, 3, 4, 5, device=DEV)).mean().backward()
    for _, p in layer.named_parameters():
        assert p.grad is not None


# (DIMS, BIN): the default runs the fused fixed-width kernels, the others the generic
# ones (ic_factorized_*_net; entropy_model.py:88-99, :198, :229-232, :259-269)
# (8 x 5 is the register kernels' largest net; the last three run the wide kernels: a hidden width
# past 8, more than five hidden layers, both)
ENTROPY_GEOMS = [([3, 3, 3], 1.0), ([3, 3, 3], 2.0), ([2, 4, 2], 1.0), ([5], 0.5), ([8, 8, 8, 8, 8], 1.0),
                 ([16, 16], 1.0), ([3] * 7, 0.5), ([40, 12, 3, 9, 5, 4], 1.0)]


@pytest.mark.parametrize("dims,bin_", ENTROPY_GEOMS)
@pytest.mark.parametrize("train", [True, False])
def test_factorized_entropy_model(train, dims, bin_):
    from image_compression_amd import get_cfg_defaults, injected_noise
    from image_compression_amd.modelling.blocks import EntropyModel
    cfg = get_cfg_defaults()
    cfg.MODEL.ENTROPY_MODEL.DIMS = list(dims)
    cfg.MODEL.ENTROPY_MODEL.BIN = bin_
    torch.manual_seed(0)
    C = 24
    em = EntropyModel(C, cfg)
    with torch.no_grad():
        for p in em.parameters():
            p.add_(torch.randn_like(p) * 0.3)
    z = _rand(3, C, 4, 5, seed=11, scale=3.0)
    u = torch.rand(3, C, 4, 5, generator=torch.Generator().manual_seed(12))
    P = {"entropy_model." + k: v.detach().double().requires_grad_(True) for k, v in em.state_dict().items()}
    zr = z.double().requires_grad_(True)
    qr, pr, cer = ref_cpu.factorized(P, zr, u.double(), train, bin_)
    gq = _rand(*qr.shape, seed=13)
    gp = _rand(*pr.shape, seed=14, scale=0.1)
    (cer * 0.37 + (qr * gq.double()).sum() + (pr * gp.double()).sum()).backward()
    emd = em.to(DEV).train(train)
    zd = _to_dev(z, cl=True)
    with injected_noise([u.to(DEV)] if train else []):
        q, p, ce = emd(zd)
    assert p.shape == pr.shape  # the reference's (N, W, C, H) probability layout
    (ce * 0.37 + (q * gq.to(DEV)).sum() + (p * gp.to(DEV)).sum()).backward()
    assert_close(q.detach().cpu().numpy(), qr.detach().numpy(), 1e-5, "q")
    assert_close(p.detach().cpu().numpy(), pr.detach().numpy(), 1e-4, "p")
    assert_close(ce.detach().cpu().numpy(), cer.detach().numpy(), 1e-4, "ce")
    if train:
        assert_close(zd.grad.cpu().numpy(), zr.grad.numpy(), 1e-4, "dz")
    for k, v in emd.named_parameters():
        assert_close(v.grad.cpu().numpy(), P["entropy_model." + k].grad.numpy(), 2e-4, k)


@pytest.mark.parametrize("bin_", [1.0, 0.5, 2.0])
@pytest.mark.parametrize("kind", ["laplace", "gauss"])
@pytest.mark.parametrize("train", [True, False])
def test_conditional_model(kind, train, bin_):
    from image_compression_amd import get_cfg_defaults, injected_noise
    from image_compression_amd.modelling.blocks import GaussianConditionalModel, LaplacianConditionalModel
    cfg = get_cfg_defaults()
    cfg.MODEL.ENTROPY_MODEL.BIN = bin_
    cm = (LaplacianConditionalModel if kind == "laplace" else GaussianConditionalModel)(cfg).train(train)
    # realistic latent statistics (|y| up to ~8, scales 0.3..5): in fp32 the
    # likelihood of a far-tail symbol is F(u)-F(l) with both near 1, so its
    # -log2 is cancellation-limited in the reference's own arithmetic; the CE
    # is therefore compared with the fp32 oracle and p with the fp64 one.
    # (Gaussian: 0.5*(1+erf(v)) of the reference loses all digits for v << 0 in
    # fp32, so its test data stays within ~4 sigma of the bin.)
    y = _rand(2, 64, 6, 7, seed=15, scale=2.0 if kind == "laplace" else 1.0)
    s = torch.exp(_rand(2, 64, 6, 7, seed=16, scale=0.5)) + (0.2 if kind == "laplace" else 0.5)
    u = torch.rand(2, 64, 6, 7, generator=torch.Generator().manual_seed(17))
    yr, sr = y.double().requires_grad_(True), s.double().requires_grad_(True)
    qr, pr = ref_cpu.conditional(yr, sr, u.double(), train, kind, bin_=bin_)
    cer = ref_cpu.ce_loss(pr)
    gq = _rand(*qr.shape, seed=18)
    (cer + (qr * gq.double()).sum()).backward()
    yd, sd = _to_dev(y, cl=True), _to_dev(s, cl=True)
    with injected_noise([u.to(DEV)] if train else []):
        q, p = cm(yd, sd)
    ce = cm._ce_loss(p)
    (ce + (q * gq.to(DEV)).sum()).backward()
    assert_close(q.detach().cpu().numpy(), qr.detach().numpy(), 1e-6, "q")
    assert_close(p.detach().cpu().numpy(), pr.detach().numpy(), 1e-4, "p")
    _, pr32 = ref_cpu.conditional(y, s, u, train, kind, bin_=bin_)
    assert_close(ce.detach().cpu().numpy(), ref_cpu.ce_loss(pr32).numpy(), 1e-4, "ce")
    # vs fp64: the Gaussian tail likelihood is cancellation-limited in fp32
    assert_close(ce.detach().cpu().numpy(), cer.detach().numpy(), 1e-3 if kind == "laplace" else 1e-2, "ce_vs_fp64")
    if train:
        assert_close(yd.grad.cpu().numpy(), yr.grad.numpy(), 1e-4, "dy")
    assert_close(sd.grad.cpu().numpy(), sr.grad.numpy(), 1e-4, "dscale")


def test_bounds_relu_abs_expclamp_mse():
    from image_compression_amd.modelling.layers import LowerBound, UpperBound
    x = _rand(2, 3, 8, 8, seed=19, scale=1.5)
    g = _rand(2, 3, 8, 8, seed=20)
    xr = x.double().requires_grad_(True)
    yr = ref_cpu.lower_bound(ref_cpu.upper_bound(xr, 1.0), 0.0)
    yr.backward(g.double())
    xd = _to_dev(x)
    y = LowerBound.apply(UpperBound.apply(xd, 1.0), 0.0)
    y.backward(g.to(DEV))
    assert torch.equal(y.detach().cpu(), yr.detach().float())
    assert torch.equal(xd.grad.cpu(), xr.grad.float())
    # relu / abs / exp-clamp
    for fn, ref in [(IF.ReLUFn.apply, torch.relu), (IF.AbsFn.apply, torch.abs),
                    (lambda t: IF.ExpClampFn.apply(t, 1e-10, 1e10), lambda t: torch.clamp(t.exp(), 1e-10, 1e10))]:
        xr = (x * 8).double().requires_grad_(True)
        ref(xr).backward(g.double())
        xd = _to_dev(x * 8)
        fn(xd).backward(g.to(DEV))
        assert_close(xd.grad.cpu().numpy(), xr.grad.numpy(), 1e-5, "grad")
    # MSE
    a, b = torch.rand(4, 3, 16, 16), torch.rand(4, 3, 16, 16)
    ar, br = a.double().requires_grad_(True), b.double().requires_grad_(True)
    lr = ref_cpu.mse(ar, br)
    lr.backward()
    ad, bd = _to_dev(a), _to_dev(b)
    l = IF.MSEFn.apply(ad, bd)
    l.backward()
    assert_close(l.detach().cpu().numpy(), lr.detach().numpy(), 1e-5, "mse")
    assert_close(bd.grad.cpu().numpy(), br.grad.numpy(), 1e-5, "dmse")


@pytest.mark.parametrize("log_scale", [True, False])
@pytest.mark.parametrize("hw", [(192, 192), (181, 207)])
def test_ms_ssim(log_scale, hw):
    from image_compression_amd.modelling.loss import MS_SSIMLoss, SSIMLoss
    H, W = hw
    a = torch.rand(2, 3, H, W, generator=torch.Generator().manual_seed(21))
    b = (a + 0.1 * torch.randn(2, 3, H, W, generator=torch.Generator().manual_seed(22))).clamp(0, 1)
    ar, br = a.double(), b.double().requires_grad_(True)
    lr = ref_cpu.ms_ssim_loss(ar, br, log_scale=log_scale)
    lr.backward()
    bd = _to_dev(b)
    l = MS_SSIMLoss(log_scale=log_scale)(a.to(DEV), bd)
    l.backward()
    assert_close(l.detach().cpu().numpy(), lr.detach().numpy(), 1e-4, "msssim")
    assert_close(bd.grad.cpu().numpy(), br.grad.numpy(), 1e-4, "dmsssim")
    # single-scale SSIMLoss
    br2 = b.double().requires_grad_(True)
    lr = ref_cpu.ssim_loss(ar, br2, log_scale=log_scale)
    lr.sum().backward()
    bd = _to_dev(b)
    l = SSIMLoss(log_scale=log_scale)(a.to(DEV), bd)
    l.sum().backward()
    assert_close(l.detach().cpu().numpy(), lr.detach().numpy(), 1e-4, "ssim")
    assert_close(bd.grad.cpu().numpy(), br2.grad.numpy(), 1e-4, "dssim")


@pytest.mark.parametrize("C,H,W,math", [(192, 16, 16, 2), (192, 9, 7, 0), (128, 8, 8, 0), (64, 5, 6, 0), (48, 4, 4, 0),
                                          (192, 67, 61, 2)])
def test_gdn_bwd_dx_column_sums(C, H, W, math):
    """gdn_bwd_sum: dx as gdn_bwd, plus dxsum[c] = sum over pixels of dx (the producing conv's
    bias gradient, formed by the fused backward from its dx tiles; C = 48 takes the GEMM path,
    which sums dx in a separate pass)."""
    from image_compression_amd import _lib
    g = torch.Generator().manual_seed(11)
    x = torch.randn(3, C, H, W, generator=g).to(DEV).contiguous(memory_format=torch.channels_last)
    gamma = (0.1 * torch.eye(C) + 0.01 * torch.rand(C, C, generator=g)).reshape(C, C, 1, 1).to(DEV)
    beta = (1.0 + torch.rand(C, generator=g)).to(DEV)
    y, norm = _lib.ops().gdn_fwd(x, gamma, beta, False, 0)
    dy = torch.randn(x.shape, generator=g).to(DEV).contiguous(memory_format=torch.channels_last)
    dx, dg, db = _lib.ops().gdn_bwd(x, norm, dy, gamma, False, math)
    dx2, dg2, db2, dxs = _lib.ops().gdn_bwd_sum(x, norm, dy, gamma, False, math)
    assert torch.equal(dx, dx2) and torch.equal(dg, dg2) and torch.equal(db, db2)
    ref = dx.double().sum(dim=(0, 2, 3))
    assert ((dxs.double() - ref).abs().max() / ref.abs().max()).item() < 1e-5


def test_conv_bias_from_gdn_column_sums():
    """conv -> GDN: the conv's bias gradient taken from the GDN backward's dx column sums equals
    the conv's own pass over its output gradient (and conv -> ReLU -> GDN keeps its own pass)."""
    from image_compression_amd import functional as IF
    g = torch.Generator().manual_seed(12)
    x = torch.randn(2, 192, 16, 16, generator=g).to(DEV)
    w = (0.05 * torch.randn(192, 192, 5, 5, generator=g)).to(DEV)
    b = (0.1 * torch.randn(192, generator=g)).to(DEV)
    gamma = (0.1 * torch.eye(192) + 0.001).reshape(192, 192, 1, 1).to(DEV)
    beta = torch.ones(192, device=DEV)
    gout = torch.randn(2, 192, 8, 8, generator=g).to(DEV)
    grads = []
    for fused in (True, False):
        bb = b.clone().requires_grad_(True)
        h = IF.conv2d(x, w, bb, 2, 2)
        if not fused:
            h = h * 1.0  # another op between: the conv's own bias pass
        IF.gdn(h, gamma, beta).backward(gout)
        grads.append(bb.grad.double())
    assert ((grads[0] - grads[1]).abs().max() / grads[1].abs().max()).item() < 1e-5
