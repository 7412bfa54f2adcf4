"""BASELINE config C3 — psnr_4096 (lambda = 4096), 320-channel latent, bf16
compute — against the fp64 CPU oracle.  bf16 operands with fp32 accumulation
on the wide convolutions' forward / input-gradient / weight-gradient GEMMs; tolerance 1e-2
normwise ("bf16 (C3): 1e-2 normwise"), and a floor that proves
the bf16 kernels (not the fp32 ones) ran."""
import pytest
import torch
import torch.nn.functional as F

from conftest import HipReluMasks, MainLayerIO, c3_check, rel_err

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _r(*shape, seed, scale=1.0):
    return torch.randn(*shape, generator=torch.Generator().manual_seed(seed)) * scale


@pytest.mark.parametrize("cin,cout,hw,k,s", [(192, 192, 16, 5, 2), (320, 192, 8, 3, 1), (192, 320, 16, 5, 2)])
def test_conv_bf16_fwd_dgrad(cin, cout, hw, k, s):
    from image_compression_amd import functional as IF
    x = _r(2, cin, hw, hw, seed=1)
    w = _r(cout, cin, k, k, seed=2, scale=0.05)
    b = _r(cout, seed=3, scale=0.1)
    xr, wr = x.double().requires_grad_(True), w.double().requires_grad_(True)
    yr = F.conv2d(xr, wr, b.double(), stride=s, padding=k // 2)
    gy = _r(*yr.shape, seed=4)
    yr.backward(gy.double())
    xd = x.to(DEV).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    wd = w.to(DEV).requires_grad_(True)
    y = IF.conv2d(xd, wd, b.to(DEV), s, k // 2, math=1)
    y.backward(gy.to(DEV))
    ey, edx = rel_err(y.detach().cpu(), yr.detach()), rel_err(xd.grad.cpu(), xr.grad)
    assert 1e-5 < ey < 1e-2, ey            # bf16 error, not fp32 exactness
    assert 1e-5 < edx < 1e-2, edx
    # and fp32-class against fp64 of the same bf16-rounded operands (the oracle's C3 emulation)
    from oracle import ref_cpu
    xe = x.double().requires_grad_(True)
    ye = ref_cpu._ConvRounded.apply(xe, w.double(), b.double(), s, k // 2, 0, False, True, True, False)
    ye.backward(gy.double())
    assert rel_err(y.detach().cpu(), ye.detach()) < 1e-5
    assert rel_err(xd.grad.cpu(), xe.grad) < 1e-5
    assert rel_err(wd.grad.cpu(), wr.grad) < 1e-5   # weight gradient stays fp32 on maps < 16 wide


@pytest.mark.parametrize("case", ["conv_ragged_ksplit", "conv_four_phase_dgrad", "tconv_four_phase_fwd",
                                  "tconv_ksplit_dgrad"])
def test_b16d_vs_bf16_emulation(case):
    """ig_kernel_b16d (the C3 bf16 DMA tiles) in isolation at 1e-5 against fp64 of the same bf16-rounded
    operands (oracle.ref_cpu._ConvRounded): a one-phase conv forward with a ragged last tile and K split
    (41 tiles of 256 rows), a stride-2 conv's four-phase input gradient (272 tiles), the four-phase
    transposed-conv forward, and the transposed conv's one-phase input gradient with K split; each
    asserts the plan it ran (advisor round 5: these had been held only at the 1e-2 bar)."""
    from image_compression_amd import _lib, functional as IF
    from oracle import ref_cpu
    torch.set_num_threads(16)
    tr = case.startswith("tconv")
    n, hw = {"conv_ragged_ksplit": (5, (90, 94)), "conv_four_phase_dgrad": (4, (128, 136)),
             "tconv_four_phase_fwd": (4, (64, 68)), "tconv_ksplit_dgrad": (4, (64, 68))}[case]
    x = _r(n, 192, *hw, seed=41)
    w = _r(192, 192, 5, 5, seed=42, scale=0.03)
    b = _r(192, seed=43, scale=0.1)
    xe = x.double().requires_grad_(True)
    ye = ref_cpu._ConvRounded.apply(xe, w.double(), b.double(), 2, 2, 1 if tr else 0, tr, True, True, False)
    gy = _r(*ye.shape, seed=44)
    ye.backward(gy.double())
    xd = x.to(DEV).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    wd = w.to(DEV)
    if tr:
        y = IF.conv_transpose2d(xd, wd, b.to(DEV), 2, 2, 1, math=1)
    else:
        y = IF.conv2d(xd, wd, b.to(DEV), 2, 2, math=1)
    gyd = gy.to(DEV).contiguous(memory_format=torch.channels_last)
    y.backward(gyd)
    op = {"conv_ragged_ksplit": ("conv2d_fwd", xd, y), "conv_four_phase_dgrad": ("conv2d_dgrad", gyd, xd),
          "tconv_four_phase_fwd": ("conv_transpose2d_fwd", xd, y), "tconv_ksplit_dgrad": ("conv_transpose2d_dgrad", gyd, xd)}[case]
    plan = _lib.plan(op[0], op[1].detach(), op[2].detach(), 5, 2, 2, 1)
    assert plan["kernel"] == "ig_bf16_dma", plan
    if case in ("conv_ragged_ksplit", "tconv_ksplit_dgrad"):
        assert plan["ksplit"] > 1, plan
    ey, edx = rel_err(y.detach().cpu(), ye.detach()), rel_err(xd.grad.cpu(), xe.grad)
    print(f"{case}: y {ey:.2e}, dx {edx:.2e} vs fp64 of the bf16 operands; plan {plan}")
    assert ey < 1e-5 and edx < 1e-5, (ey, edx)


@pytest.mark.parametrize("transposed", [False, True])
def test_wgrad_bf16(transposed):
    """Weight gradients with bf16 operands (the two-wave kernel with one product per tile and
    step, maps >= 16 wide): bf16 error, not fp32 exactness, against fp64; narrower maps keep
    fp32 (test_conv_bf16_fwd_dgrad)."""
    from image_compression_amd import _lib, functional as IF
    n, h = (2, 64) if not transposed else (2, 16)
    x = _r(n, 192, h, h, seed=11)
    w = _r(192, 192, 5, 5, seed=12, scale=0.05)
    xr, wr = x.double(), w.double().requires_grad_(True)
    if transposed:
        yr = F.conv_transpose2d(xr, wr, None, stride=2, padding=2, output_padding=1)
    else:
        yr = F.conv2d(xr, wr, None, stride=2, padding=2)
    gy = _r(*yr.shape, seed=13)
    yr.backward(gy.double())
    xd = x.to(DEV).contiguous(memory_format=torch.channels_last)
    wd = w.to(DEV).requires_grad_(True)
    gyd = gy.to(DEV).contiguous(memory_format=torch.channels_last)
    if transposed:
        y = IF.conv_transpose2d(xd, wd, None, 2, 2, 1, math=1)
        plan = _lib.plan("conv_transpose2d_wgrad", xd, gyd, 5, 2, 2, 1)
    else:
        y = IF.conv2d(xd, wd, None, 2, 2, math=1)
        plan = _lib.plan("conv2d_wgrad", xd, gyd, 5, 2, 2, 1)
    assert plan["kernel"] == "wg_bf16", plan
    y.backward(gyd)
    e = rel_err(wd.grad.cpu(), wr.grad)
    # fp64 with the same bf16-rounded operands (the oracle's C3 emulation): fp32-class agreement
    from oracle import ref_cpu
    we = w.double().requires_grad_(True)
    ye = ref_cpu._ConvRounded.apply(x.double(), we, None, 2, 2, 1 if transposed else 0, transposed,
                                    False, False, True)
    ye.backward(gy.double())
    e_em = rel_err(wd.grad.cpu(), we.grad)
    print(f"bf16 wgrad transposed={transposed}: vs fp64 {e:.2e}, vs fp64 of the bf16 operands {e_em:.2e}")
    assert 1e-5 < e < 1e-2, e
    assert e_em < 1e-5, e_em


def test_tconv_bf16_fwd_dgrad():
    from image_compression_amd import functional as IF
    x = _r(2, 192, 8, 8, seed=5)
    w = _r(192, 192, 5, 5, seed=6, scale=0.05)
    xr, wr = x.double().requires_grad_(True), w.double()
    yr = F.conv_transpose2d(xr, wr, None, stride=2, padding=2, output_padding=1)
    gy = _r(*yr.shape, seed=7)
    yr.backward(gy.double())
    xd = x.to(DEV).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    y = IF.conv_transpose2d(xd, w.to(DEV), None, 2, 2, 1, math=1)
    y.backward(gy.to(DEV))
    assert 1e-5 < rel_err(y.detach().cpu(), yr.detach()) < 1e-2
    assert 1e-5 < rel_err(xd.grad.cpu(), xr.grad) < 1e-2


@pytest.mark.parametrize("transposed", [False, True])
def test_image_edges_bf16(transposed):
    """C3's 3-channel image edges on bf16 operands (edge_conv_x3_kernel / tconv_few2_kernel /
    edge_wgrad_kernel with one product): g_a.0 (conv 3 -> 192) forward and weight gradient, g_s.6
    (transposed conv 192 -> 3) forward, input gradient and weight gradient, against the fp64 oracle
    of the same bf16-rounded operands (oracle.ref_cpu._ConvRounded, the C3 emulation: within
    1e-5) and against exact fp64 (within the 1e-2 bf16 bar, above 1e-5: the operands were rounded);
    the plans name the bf16 edge kernels."""
    from conftest import edges_bf16
    from image_compression_amd import _lib
    from image_compression_amd import functional as IF
    from oracle import ref_cpu
    if not edges_bf16():
        pytest.skip("this build runs the image edges in split arithmetic in C3 (EDGE_BF16 = 0)")
    m = IF.MATH["bf16"] | IF.MATH["fp32_split"]   # what set_compute_dtype gives the main transforms in C3
    if transposed:
        x = _r(2, 192, 16, 24, seed=21)
        w = _r(192, 3, 5, 5, seed=22, scale=0.05)
        xd = x.to(DEV).contiguous(memory_format=torch.channels_last).requires_grad_(True)
        wd = w.to(DEV).requires_grad_(True)
        y = IF.conv_transpose2d(xd, wd, None, 2, 2, 1, math=m)
        kinds = [_lib.plan("conv_transpose2d_fwd", xd, y, 5, 2, 2, m)["kernel"],
                 _lib.plan("conv_transpose2d_wgrad", xd, y, 5, 2, 2, m)["kernel"]]
        assert kinds == ["tconv_few_rows_bf16", "edge_wgrad_bf16"], kinds
    else:
        x = _r(2, 3, 40, 72, seed=21)
        w = _r(192, 3, 5, 5, seed=22, scale=0.2)
        xd = x.to(DEV).requires_grad_(False)
        wd = w.to(DEV).requires_grad_(True)
        y = IF.conv2d(xd, wd, None, 2, 2, math=m)
        kinds = [_lib.plan("conv2d_fwd", xd, y, 5, 2, 2, m)["kernel"], _lib.plan("conv2d_wgrad", xd, y, 5, 2, 2, m)["kernel"]]
        assert kinds == ["edge_conv_bf16", "edge_wgrad_bf16"], kinds
    gy = _r(*y.shape, seed=23)
    y.backward(gy.to(DEV))
    outs = {"y": y.detach().cpu(), "dw": wd.grad.cpu()}
    if transposed:
        outs["dx"] = xd.grad.cpu()
    for flags in ((True, True, True), None):
        xr = x.double().requires_grad_(transposed)
        wr = w.double().requires_grad_(True)
        yr = ref_cpu._conv(xr, wr, None, 2, 2, "w", {"w": flags} if flags else None, transposed=transposed,
                           opad=1 if transposed else 0)
        yr.backward(gy.double())
        refs = {"y": yr.detach(), "dw": wr.grad}
        if transposed:
            refs["dx"] = xr.grad
        for k, ref in refs.items():
            e = rel_err(outs[k], ref)
            print(f"edge bf16 transposed={transposed} {k}: vs {'emulation' if flags else 'exact fp64'} {e:.2e}")
            if flags:
                assert e < 1e-5, (k, e)
            else:
                assert 1e-5 < e < 1e-2, (k, e)


def test_model_c3_bf16_vs_oracle():
    from image_compression_amd import functional as IF, get_cfg_defaults, injected_noise, modelling
    cfg = get_cfg_defaults()
    cfg.MODEL.LOSS.REDUCTION = "mean"
    cfg.MODEL.LOSS.DISTORTION_LOSS_WEIGHT = 4096.0
    cfg.MODEL.LATENT_CHANNELS = 320
    cfg.MODEL.COMPUTE_DTYPE = "bf16"
    torch.manual_seed(0)
    model = modelling.build_model(cfg)
    params = {k: v.clone() for k, v in model.state_dict().items()}
    model = model.to(DEV).train()
    g = torch.Generator().manual_seed(9)
    x = torch.rand(2, 3, 128, 128, generator=g)
    uz = torch.rand(2, 192, 2, 2, generator=g)
    uy = torch.rand(2, 320, 8, 8, generator=g)
    hm, lio = HipReluMasks(model), MainLayerIO(model)
    with IF.record_plans() as log, injected_noise([uz.to(DEV), uy.to(DEV)]):
        xt, losses = model(x.to(DEV))
        losses["total_loss"].backward()
    hm.remove()
    lio.remove()
    # per-layer against the fp64 emulation of the bf16 operands, end to end against the exact
    # fp64 oracle within the config's floor (conftest.c3_check)
    c3_check(model, params, x, uz, uy, xt, losses, hm.masks, log, 4096.0, 320, lio)


@pytest.mark.parametrize("n,h,w,inverse", [(2, 16, 16, False), (3, 7, 5, False), (4, 33, 31, True)])
def test_gdn_bwd_bf16(n, h, w, inverse):
    """GDN backward with IC_MATH_BF16 (fused kernel, C = 192): dx's q.gamma and dgamma's
    q^T x^2 on bf16 operands.  Against fp64: bf16-level error; against the oracle's emulation of
    those bf16 operands (forward GDN): fp32-class.  dbeta is a plain sum: fp32-class."""
    from image_compression_amd import _lib
    from image_compression_amd.modelling.layers import GDN
    from oracle import ref_cpu
    torch.manual_seed(0)
    m = GDN(192, inverse=inverse)
    with torch.no_grad():
        m.gamma.param.add_(torch.rand_like(m.gamma.param) * 0.05)
        m.beta.param.add_(torch.rand_like(m.beta.param) * 0.1)
    x = _r(n, 192, h, w, seed=12)
    gy = _r(n, 192, h, w, seed=13)
    ref = {}
    for emul in (False, True):
        if emul and inverse:
            continue
        gp = m.gamma.param.detach().double().requires_grad_(True)
        bp = m.beta.param.detach().double().requires_grad_(True)
        xr = x.double().requires_grad_(True)
        yr = ref_cpu.gdn(xr, gp, bp, inverse=inverse, bf16_bwd=emul)
        yr.backward(gy.double())
        ref[emul] = (xr.grad, gp.grad, bp.grad)
    md = m.to(DEV)
    md.math = 3   # split | bf16: the bf16 fused backward
    xd = x.to(DEV).contiguous(memory_format=torch.channels_last).requires_grad_(True)
    assert _lib.plan("gdn_bwd", xd.detach(), None, math=3)["kernel"] == "gdn_fused_bf16"
    md(xd).backward(gy.to(DEV).contiguous(memory_format=torch.channels_last))
    got = (xd.grad.cpu(), md.gamma.param.grad.cpu(), md.beta.param.grad.cpu())
    for i, nm in enumerate(("dx", "dgamma")):
        e = rel_err(got[i], ref[False][i])
        msg = f"{nm}: vs fp64 {e:.2e}"
        assert e < 1e-2, (nm, e)
        if not inverse:
            e2 = rel_err(got[i], ref[True][i])
            msg += f", vs fp64 of the bf16 operands {e2:.2e}"
            assert e2 < 1e-4, (nm, e2)  # q rounds from fp32 here, from fp64 there: rare neighbour flips
        print(msg)
    assert rel_err(got[2], ref[False][2]) < 1e-5


@pytest.mark.parametrize("n,h,w", [(2, 16, 16), (3, 7, 5), (4, 33, 31)])
def test_gdn_fwd_bf16(n, h, w):
    """GDN forward with IC_MATH_BF16 (gdn_fwd_x3s_kernel<192, 1>): Gamma x^2 on bf16 operands (one
    plane, one product, fp32 accumulation).  Against fp64: bf16-level error; against the oracle's
    emulation of those operands: fp32-class (x^2 rounds from fp32 here, from fp64 there)."""
    from image_compression_amd import _lib
    from image_compression_amd.modelling.layers import GDN
    from oracle import ref_cpu
    torch.manual_seed(0)
    m = GDN(192)
    with torch.no_grad():
        m.gamma.param.add_(torch.rand_like(m.gamma.param) * 0.05)
        m.beta.param.add_(torch.rand_like(m.beta.param) * 0.1)
    x = _r(n, 192, h, w, seed=14)
    gp, bp = m.gamma.param.detach().double(), m.beta.param.detach().double()
    exact = ref_cpu.gdn(x.double(), gp, bp)
    emul = ref_cpu.gdn(x.double(), gp, bp, bf16_fwd=True)
    md = m.to(DEV)
    md.math_fwd = 3   # split | bf16
    xd = x.to(DEV).contiguous(memory_format=torch.channels_last)
    assert _lib.plan("gdn_fwd", xd, None, math=3)["kernel"] == "gdn_fused_bf16"
    with torch.no_grad():
        y = md(xd).cpu()
    e, e2 = rel_err(y, exact), rel_err(y, emul)
    print(f"gdn fwd bf16: vs fp64 {e:.2e}, vs fp64 of the bf16 operands {e2:.2e}")
    assert e < 1e-2 and e2 < 1e-4, (e, e2)
    assert e2 < e / 4  # the kernel computes what the config says, not plain fp32


@pytest.mark.parametrize("n,h,w,inverse", [(2, 16, 16, False), (3, 7, 5, False), (4, 33, 31, True), (32, 16, 16, False)])
def test_gdn_norm_recompute_bitwise(n, h, w, inverse):
    """C3's GDN pair without a stored norm (round 6, include/imgcomp.h ic_gdn_fwd_rn / ic_gdn_bwd_sum_rn):
    the forward leaves norm out and the backward forms it again per tile from x, Gamma and beta with the
    forward's bf16 operands and MFMA order -- so y, its bf16 copy, dx, dx's copy, dGamma, dbeta and the dx
    column sums are bitwise those of the pair that stores norm (ragged pixel counts, IGDN, the 4-tile
    split across the two wave groups, and a C3-sized 16^2 layer).  The model path takes it whenever
    both directions run on bf16 operands at C = 192 (functional._norm_recompute)."""
    from image_compression_amd import _lib
    ops = _lib.ops()
    g = torch.Generator().manual_seed(31)
    x = (torch.randn(n, 192, h, w, generator=g)).to(DEV).contiguous(memory_format=torch.channels_last)
    dy = (torch.randn(n, 192, h, w, generator=g)).to(DEV).contiguous(memory_format=torch.channels_last)
    gamma = (torch.eye(192) * 0.1 + torch.rand(192, 192, generator=g) * 0.01).reshape(192, 192, 1, 1).to(DEV)
    beta = (1.0 + torch.rand(192, generator=g) * 0.1).to(DEV)
    for xb in (True, False):
        y0, norm, yb0 = ops.gdn_fwd_xb(x, gamma, beta, inverse, 3)
        y1, yb1 = ops.gdn_fwd_rn(x, gamma, beta, inverse, 3, xb)
        assert torch.equal(y0, y1)
        if xb:
            assert torch.equal(yb0, yb1)
        r0 = ops.gdn_bwd_sum_xb(x, norm, dy, gamma, inverse, 3)
        r1 = ops.gdn_bwd_sum_rn(x, beta, dy, gamma, inverse, 3, xb)
        for i, nm in enumerate(("dx", "dgamma", "dbeta", "dxsum", "dxb")):
            if nm == "dxb" and not xb:
                continue
            assert torch.equal(r0[i], r1[i]), (nm, xb, (r0[i].float() - r1[i].float()).abs().max().item())
    # any other arithmetic refuses the norm-free form
    with pytest.raises(RuntimeError):
        ops.gdn_fwd_rn(x, gamma, beta, inverse, 2, False)


def test_c3_bf16_copies_bitwise():
    """Config C3's bf16 activation copies (round 5): every GDN / IGDN of g_a and g_s whose output feeds
    a 192-output conv or transposed conv writes that output's bf16 copy for the conv's forward, and
    every one behind a 192-input conv its input gradient's for that conv's input gradient; those
    convs run on the bf16 DMA tiles (ig_kernel_b16d, the stride-2 phases included) reading the copies.
    The copies are the same round-to-nearest-even values the convs would form from the fp32 tensors,
    so one training step is bitwise the step with the copies switched off (each conv converting its
    own input), and all eight copies are taken."""
    from image_compression_amd import functional as IF, get_cfg_defaults, injected_noise, modelling
    from image_compression_amd.modelling.layers.gdn import GDN
    cfg = get_cfg_defaults()
    cfg.MODEL.LOSS.REDUCTION = "mean"
    cfg.MODEL.LOSS.DISTORTION_LOSS_WEIGHT = 4096.0
    cfg.MODEL.LATENT_CHANNELS = 320
    cfg.MODEL.COMPUTE_DTYPE = "bf16"
    torch.manual_seed(0)
    model = modelling.build_model(cfg).to(DEV).train()
    assert [g.xb for g in model.modules() if isinstance(g, GDN)] == [1, 3, 2, 1, 3, 2]
    g = torch.Generator().manual_seed(3)
    x = torch.rand(4, 3, 256, 256, generator=g).to(DEV)
    uz = torch.rand(4, 192, 4, 4, generator=g).to(DEV)
    uy = torch.rand(4, 320, 16, 16, generator=g).to(DEV)

    def step():
        model.zero_grad(set_to_none=True)
        with IF.record_plans() as log, injected_noise([uz, uy]):
            _, losses = model(x)
            losses["total_loss"].backward()
        torch.cuda.synchronize()
        return ({k: v.detach().clone() for k, v in losses.items()},
                {n: p.grad.detach().clone() for n, p in model.named_parameters()}, log)

    before = dict(IF.BF16_COPY_STATS)
    la, ga, log = step()
    assert IF.BF16_COPY_STATS["put"] - before["put"] == 8 and IF.BF16_COPY_STATS["hit"] - before["hit"] == 8
    kinds = [e["kernel"] for e in log]
    # g_a.2 fwd / dgrad, g_s.4 fwd / dgrad (the 32^2 layers take smaller tiles at batch 4)
    assert kinds.count("ig_bf16_dma") >= 4, kinds
    flags = {n: m.xb for n, m in model.named_modules() if isinstance(m, GDN)}
    for m in model.modules():
        if isinstance(m, GDN):
            m.xb = 0
    lb, gb, _ = step()
    for n, m in model.named_modules():
        if isinstance(m, GDN):
            m.xb = flags[n]
    for k in la:
        assert torch.equal(la[k], lb[k]), k
    for n in ga:
        assert torch.equal(ga[n], gb[n]), n
