"""Training-step harness around the path: LR schedules
against the reference's own scheduler code (golden vectors from
tools/gen_golden_solver.py), the reference's parameter grouping, and the
native AdamW + clip kernel against torch.optim.AdamW + clip_grad_value_ (the
reference's optimizer, solver/optim.py:38 and engine/trainer.py:189-190)."""
import copy
import json
import os

import pytest
import torch

from conftest import GOLDEN, assert_close


class _Cfg(dict):
    def __getattr__(self, k):
        return self[k]


def test_lr_schedules_match_reference_golden():
    from image_compression_amd.solver import make_lr_scheduler
    cases = json.load(open(os.path.join(GOLDEN, "lr_schedules.json")))
    assert len(cases) >= 7
    for case in cases:
        solver = _Cfg(case["solver"])
        cfg = _Cfg(SOLVER=solver)
        opt = torch.optim.SGD([torch.nn.Parameter(torch.zeros(1))], lr=1.0)
        sch = make_lr_scheduler(cfg, opt, case["iters_per_epoch"])
        got = []
        for _ in case["lrs"]:
            opt.step()
            sch.step()
            got.append(sch.get_last_lr()[0])
        assert got == pytest.approx(case["lrs"], rel=1e-12, abs=1e-15), case["name"]


def test_optimizer_groups_follow_reference_rules():
    from image_compression_amd import get_cfg_defaults, modelling
    from image_compression_amd.solver import make_optimizer
    cfg = get_cfg_defaults()
    cfg.MODEL.INTER_CHANNELS = 16
    cfg.MODEL.LATENT_CHANNELS = 16
    cfg.SOLVER.OPT_NAME = "adamw"
    cfg.SOLVER.BASE_LR = 1e-4
    cfg.SOLVER.GRAD_CLIP = 5.0
    model = modelling.build_model(cfg)
    opt = make_optimizer(cfg, model)
    names = [n for n, p in model.named_parameters() if p.requires_grad]
    assert len(opt.param_groups) == len(names)
    for n, g in zip(names, opt.param_groups):
        assert g["weight_decay"] == (0.0 if "bias" in n else 5e-4), n
        assert g["lr"] == 1e-4 and g["eps"] == 1e-4
    assert opt.clip_value == 5.0
    # GDN beta / CDF factor are decayed (no "bias" in the name), CDF biases are not
    wd = {n: g["weight_decay"] for n, g in zip(names, opt.param_groups)}
    assert wd["analysis_transform.layers.1.beta.param"] == 5e-4
    assert wd["entropy_model._cdf_estimator.layers.0.bias"] == 0.0
    cfg.SOLVER.OPT_NAME = "sgd"
    with pytest.raises(NotImplementedError):
        make_optimizer(cfg, model)


@pytest.mark.gpu
def test_adamw_kernel_matches_torch_adamw_with_clip():
    from image_compression_amd.solver import AdamW
    g = torch.Generator().manual_seed(0)
    shapes = [(192, 192, 5, 5), (192,), (3, 192, 5, 5), (1,), (192, 1, 3, 3), (4097,)]
    ref_p = [torch.nn.Parameter(torch.randn(s, generator=g) * 0.1) for s in shapes]
    dev_p = [torch.nn.Parameter(p.detach().clone().cuda()) for p in ref_p]
    groups = lambda ps: [{"params": [p], "lr": 1e-3 * (1 + i), "weight_decay": (5e-4 if i % 2 == 0 else 0.0)}
                         for i, p in enumerate(ps)]
    ref = torch.optim.AdamW(groups(ref_p), lr=1e-3, eps=1e-4)
    opt = AdamW(groups(dev_p), lr=1e-3, eps=1e-4, clip_value=5.0)
    for step in range(4):
        for rp, dp in zip(ref_p, dev_p):
            gr = torch.randn(rp.shape, generator=g) * (8.0 if step == 1 else 1.0)  # step 1 exercises clipping
            rp.grad = gr.clone()
            dp.grad = gr.cuda()
        torch.nn.utils.clip_grad_value_(ref_p, 5.0)
        ref.step()
        opt.step()
    torch.cuda.synchronize()
    for rp, dp in zip(ref_p, dev_p):
        d = (dp.detach().cpu() - rp.detach()).abs().max().item()
        assert d <= 1e-6 * max(rp.detach().abs().max().item(), 1e-3), d
        assert torch.allclose(dp.grad.cpu(), rp.grad)                # clipped grads written back
        st, rst = opt.state[dp], ref.state[rp]
        assert int(st["step"]) == int(rst["step"]) == 4
        assert_close(st["exp_avg"].cpu().numpy(), rst["exp_avg"].numpy(), 1e-6, "exp_avg")
        assert_close(st["exp_avg_sq"].cpu().numpy(), rst["exp_avg_sq"].numpy(), 1e-6, "exp_avg_sq")
    # optimizer state_dict round-trips in torch's format
    sd = copy.deepcopy(opt.state_dict())
    assert set(sd["state"][0]) == {"step", "exp_avg", "exp_avg_sq"}


@pytest.mark.gpu
def test_train_step_runs_reference_loop():
    from image_compression_amd import get_cfg_defaults, modelling
    from image_compression_amd.solver import make_lr_scheduler, make_optimizer, train_step
    cfg = get_cfg_defaults()
    cfg.MODEL.LOSS.DISTORTION_LOSS_WEIGHT = 256.0
    cfg.MODEL.LOSS.REDUCTION = "mean"
    cfg.SOLVER.OPT_NAME = "adamw"
    cfg.SOLVER.BASE_LR = 1e-4
    cfg.SOLVER.GRAD_CLIP = 5.0
    cfg.SOLVER.SCHEDULER_NAME = "constant"
    torch.manual_seed(0)
    model = modelling.build_model(cfg).cuda().train()
    opt = make_optimizer(cfg, model)
    sch = make_lr_scheduler(cfg, opt)
    x = torch.rand(2, 3, 64, 64, generator=torch.Generator().manual_seed(1)).cuda()
    before = model.analysis_transform.layers[0].weight.detach().clone()
    for it in range(3):
        _, losses = train_step(model, opt, sch, x, it=it)
        assert torch.isfinite(losses["total_loss"])
    assert not torch.equal(before, model.analysis_transform.layers[0].weight.detach())
    assert all(p.grad is None for p in model.parameters())
