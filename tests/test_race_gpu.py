"""The concurrent C2 step (hyperprior + entropy models on a side stream, the hyperprior convs'
weight gradients on a stream of their own, beside the synthesis transform's MFMA kernels) against a
serial reference step, bitwise, with every factorized-backward and hyperprior weight-gradient
launch recomputed on its own inputs on an idle GPU.  Guards the fault found in round 3: with
packed-fp32 VALU instructions (v_pk_*_f32) the factorized backward (csrc/entropy.hip fact_bwd_k)
returned wrong w1 / w2 gradient elements in concurrent steps only (1 of 120; 53 of 80 with an
LDS-only reduction), never without those instructions; every source is now built without them
(csrc/Makefile NOPK, tests/test_isa_scan.py) -- DESIGN.md 10a.  GPU only."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_concurrent_steps_exact_and_factorized_backward_recomputes():
    """30 concurrent C2 steps bitwise equal to the serial step; in each, every factorized-backward
    launch (side stream) and every hyperprior conv weight / bias gradient (its weight-gradient
    stream: the wgrad kernels, split-K reduce and bias column sums) is recomputed on its saved
    inputs on an idle GPU and must match bitwise."""
    from image_compression_amd import _lib, get_cfg_defaults, injected_noise, modelling
    from image_compression_amd import functional as IF
    ops = _lib.ops()
    snaps, wsnaps = [], []
    orig = IF.FactorizedFn.backward
    orig_wg = IF._ConvWGradFn.backward

    def wrapped(ctx, gq, gp):
        q, *prm = ctx.saved_tensors
        res = orig(ctx, gq, gp)
        snaps.append((q.clone(), [t.clone() for t in prm], None if gq is None else IF._to_last(gq).clone(),
                      None if gp is None else IF._to_last(gp).clone(), ctx.C,
                      [t.detach().clone() for t in res[5:]]))
        return res

    def wrapped_wg(ctx, gz):
        x, w = ctx.saved_tensors
        res = orig_wg(ctx, gz)
        # stream-ordered clones on the weight-gradient stream (the backward's own stream)
        wsnaps.append((x.clone(), IF._cl(gz).clone(), w.detach(), ctx.conf, ctx.has_b, res[1].clone(),
                       None if res[2] is None else res[2].clone()))
        return res

    cfg = get_cfg_defaults()
    cfg.MODEL.LOSS.REDUCTION = "mean"
    cfg.MODEL.LOSS.DISTORTION_LOSS_WEIGHT = 256.0
    torch.manual_seed(0)
    m = modelling.build_model(cfg).cuda().train()
    g = torch.Generator().manual_seed(3)
    x = torch.rand(32, 3, 256, 256, generator=g).cuda()
    uz = torch.rand(32, 192, 4, 4, generator=g).cuda()
    uy = torch.rand(32, 192, 16, 16, generator=g).cuda()

    def step(conc):
        m.concurrent_hyperprior = conc
        m.zero_grad(set_to_none=True)
        with injected_noise([uz, uy]):
            _, losses = m(x)
            losses["total_loss"].backward()
        del losses
        torch.cuda.synchronize()
        return {k: p.grad.clone() for k, p in m.named_parameters()}

    ref = step(False)
    IF.FactorizedFn.backward = staticmethod(wrapped)
    IF._ConvWGradFn.backward = staticmethod(wrapped_wg)
    try:
        for i in range(30):
            try:
                r = step(True)
            except UserWarning as e:   # conftest makes the AccumulateGrad stream warning an error
                raise AssertionError(f"concurrent step {i}: {str(e)[:120]}") from e
            # recomputes without autograd: a call on the parameter itself in grad mode would hang a
            # graph node (and the parameter's AccumulateGrad, made on this stream) on its output
            with torch.no_grad():
                for q, prm, gq, gp, C, out in snaps:
                    dz, grads = ops.factorized_bwd(q, C, prm, gq, gp)
                    torch.cuda.synchronize()
                    for j, (a, b) in enumerate(zip(out, grads)):
                        assert torch.equal(a, b), ("factorized backward differs from its recompute", i, j)
                assert len(wsnaps) == 6, len(wsnaps)   # h_a's three convs and h_s's three
                for xs, gy, w, conf, has_b, dw, db in wsnaps:
                    transposed, stride, padding, act, math = conf
                    assert not act
                    fn = ops.conv_transpose2d_wgrad if transposed else ops.conv2d_wgrad
                    dw2, db2 = fn(xs, gy, w, stride, padding, has_b, math)
                    torch.cuda.synchronize()
                    assert torch.equal(dw, dw2), ("hyperprior weight gradient differs from its recompute", i, conf)
                    assert db is None or torch.equal(db, db2), ("hyperprior bias gradient differs", i, conf)
            snaps.clear()
            wsnaps.clear()
            for k in ref:
                assert torch.equal(r[k], ref[k]), (i, k)
    finally:
        IF.FactorizedFn.backward = orig
        IF._ConvWGradFn.backward = orig_wg
