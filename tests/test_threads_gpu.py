"""Re-entrancy of the HIP path (Threading): the reference trainer wraps the
model in nn.DataParallel unconditionally (engine/trainer.py:256-259), which runs module
replicas from one Python thread per GPU (parallel_apply).  The ops must hold no unlocked
global state and launch on the current stream of the calling thread.  GPU only."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model():
    from image_compression_amd import get_cfg_defaults, modelling
    cfg = get_cfg_defaults()
    cfg.MODEL.LOSS.REDUCTION = "mean"
    cfg.MODEL.LOSS.DISTORTION_LOSS_WEIGHT = 256.0
    torch.manual_seed(0)
    return modelling.build_model(cfg).to(DEV).train()


class _WithNoise(torch.nn.Module):
    """Feeds fixed training-noise draws to the wrapped model in whatever thread runs it
    (the injected-noise queue is thread-local, like the Philox state)."""

    def __init__(self, model, uz, uy):
        super().__init__()
        self.model, self.uz, self.uy = model, uz, uy

    def forward(self, x):
        from image_compression_amd import injected_noise
        with injected_noise([self.uz, self.uy]):
            return self.model(x)


def _inputs(seed, n=2, s=128):
    g = torch.Generator().manual_seed(seed)
    return (torch.rand(n, 3, s, s, generator=g).to(DEV), torch.rand(n, 192, s // 64, s // 64, generator=g).to(DEV),
            torch.rand(n, 192, s // 16, s // 16, generator=g).to(DEV))


def _grads(m):
    return {k: p.grad.detach().clone() for k, p in m.named_parameters()}


def test_data_parallel_single_device_matches_unwrapped():
    base = _model()
    x, uz, uy = _inputs(1)
    ref = copy.deepcopy(base)
    xt_r, l_r = _WithNoise(ref, uz, uy)(x)
    l_r["total_loss"].backward()
    dp = torch.nn.DataParallel(_WithNoise(copy.deepcopy(base), uz, uy), device_ids=[0])
    xt, l = dp(x)
    l["total_loss"].backward()
    torch.cuda.synchronize()
    assert torch.equal(xt, xt_r)
    for k in l_r:
        assert torch.equal(l[k], l_r[k]), k
    g, g_r = _grads(dp.module.model), _grads(ref)
    for k in g_r:
        assert torch.equal(g[k], g_r[k]), k


def test_replicas_on_two_threads_match_serial():
    """Two replicas driven concurrently from two threads (torch's parallel_apply, both on
    cuda:0), one backward over both losses: every output and gradient bitwise equal to the
    replicas run one after the other.  Exercises the colsum hand-off table, the workspace and
    noise state under threads."""
    base = _model()
    ins = [_inputs(2), _inputs(3)]
    serial = [copy.deepcopy(base) for _ in ins]
    outs_s = [_WithNoise(m, uz, uy)(x) for m, (x, uz, uy) in zip(serial, ins)]
    (outs_s[0][1]["total_loss"] + outs_s[1][1]["total_loss"]).backward()
    reps = [copy.deepcopy(base) for _ in ins]
    mods = [_WithNoise(m, uz, uy) for m, (_, uz, uy) in zip(reps, ins)]
    for _ in range(3):  # a few rounds: thread interleavings differ from run to run
        for m in reps:
            m.zero_grad(set_to_none=True)
        outs = torch.nn.parallel.parallel_apply(mods, [(x,) for x, _, _ in ins], devices=[0, 0])
        (outs[0][1]["total_loss"] + outs[1][1]["total_loss"]).backward()
        torch.cuda.synchronize()
        for i in range(2):
            assert torch.equal(outs[i][0], outs_s[i][0]), i
            for k in outs_s[i][1]:
                assert torch.equal(outs[i][1][k], outs_s[i][1][k]), (i, k)
            g, g_s = _grads(reps[i]), _grads(serial[i])
            for k in g_s:
                assert torch.equal(g[k], g_s[k]), (i, k)
