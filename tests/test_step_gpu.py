"""The hipGraph-replayed training step (image_compression_amd.step.TrainStep)
against the same step run eagerly, and the graph-safe noise stream."""
import pytest
import torch

DEV = "cuda"

pytestmark = pytest.mark.gpu


def _model(train):
    from image_compression_amd import get_cfg_defaults, modelling
    cfg = get_cfg_defaults()
    cfg.MODEL.LOSS.REDUCTION = "mean"
    cfg.MODEL.LOSS.DISTORTION_LOSS_WEIGHT = 256.0
    torch.manual_seed(0)
    return modelling.build_model(cfg).to(DEV).train(train)


def _x():
    return torch.rand(4, 3, 128, 128, generator=torch.Generator().manual_seed(5)).to(DEV)


def test_graph_replay_equals_eager_in_eval_mode():
    """Eval mode (rounding, no noise): replay and eager step are bitwise equal
    (deterministic kernels, fixed-order reductions)."""
    from image_compression_amd.step import TrainStep
    x = _x()
    eager = TrainStep(_model(False), x, graph=False)
    le = {k: v.clone() for k, v in eager(x).items()}
    ge_grad = eager.grads().clone()
    graph = TrainStep(_model(False), x, graph=True)
    for _ in range(2):
        lg = graph(x)
    torch.cuda.synchronize()
    for k in le:
        assert torch.equal(le[k], lg[k]), k
    assert torch.equal(ge_grad, graph.grads())
    assert torch.isfinite(graph.grads()).all()
    flat = TrainStep(_model(False), x, graph=True, flat=True)
    flat(x)
    assert torch.equal(ge_grad, flat.grads())


def test_graph_replay_draws_fresh_noise_and_is_reproducible():
    from image_compression_amd import noise
    from image_compression_amd.step import TrainStep
    x = _x()
    st = TrainStep(_model(True), x, graph=True)
    state = noise.device_state(x.device)
    saved = state.clone()
    b1 = float(st(x)["bpp"])
    g1 = st.grads().clone()
    b2 = float(st(x)["bpp"])
    assert b1 != b2                      # the base advanced inside the graph
    assert int(state[1]) - int(saved[1]) == 2 * (4 * 192 * 2 * 2 + 4 * 192 * 8 * 8)
    state.copy_(saved)                   # same counters -> same step
    b3 = float(st(x)["bpp"])
    assert b3 == b1
    assert torch.equal(g1, st.grads())
    # an eager step of the same model after the graph, with the same counters, is bitwise the
    # replay: losses and every gradient.  The captured step must not have left AccumulateGrad
    # nodes of the capture stream behind (the suite turns torch's stream-mismatch warning into
    # an error, conftest.py), or this step would accumulate its gradients on that stream.
    from image_compression_amd.step import TrainStep as TS
    state.copy_(saved)
    eager = TS(st.model, x, graph=False)
    noise._st().offset[noise._key(x.device)] = 4 * 192 * 2 * 2 + 4 * 192 * 8 * 8
    le = eager(x)
    torch.cuda.synchronize()
    assert float(le["bpp"]) == b1
    assert torch.equal(g1, eager.grads())


@pytest.mark.parametrize("train", [True, False])
def test_concurrent_hyperprior_is_bitwise_serial(train):
    """Compressor2018 runs the hyperprior branch and the y likelihood on a side stream while
    the synthesis transform runs (the backward follows the same streams).  Same kernels, same
    noise counters in the same order: losses, x~ and every gradient bitwise equal to the serial
    step -- with the in-kernel Philox noise (train) and with rounding (eval)."""
    from image_compression_amd import noise
    x = _x()
    out = {}
    for conc in (False, True):
        m = _model(train)
        m.concurrent_hyperprior = conc
        state = noise.device_state(x.device)
        saved = state.clone()
        for _ in range(2):  # the second step exercises begin_step's advance after a concurrent step
            state.copy_(saved) if _ == 0 else None
            m.zero_grad(set_to_none=True)
            xt, losses = m(x)
            losses["total_loss"].backward()
        torch.cuda.synchronize()
        out[conc] = (xt.clone(), {k: v.clone() for k, v in losses.items()},
                     {k: p.grad.clone() for k, p in m.named_parameters()})
        state.copy_(saved)
    assert torch.equal(out[False][0], out[True][0])
    for k in out[False][1]:
        assert torch.equal(out[False][1][k], out[True][1][k]), k
    for k in out[False][2]:
        assert torch.equal(out[False][2][k], out[True][2][k]), k


def test_concurrent_step_repeatable_at_c2():
    """The C2 step (32 x 256^2, fp32_split, injected noise) with the hyperprior side stream,
    repeated: every gradient bitwise equal run to run and to the serial step.  Guards the
    stream crossings (bmshl2018._StreamEdge): without the gradients recorded on their
    consumer stream the caching allocator handed a gradient's memory to the other stream's
    next allocation while it was still read, and about one step in five came out with a
    changed CDF-estimator weight gradient element (tools/determinism_probe.py).  Each run drops
    its graph before the next one (see below): a serial run's AccumulateGrad nodes kept alive into
    a concurrent run make torch accumulate side-stream gradients on the main stream."""
    from image_compression_amd import get_cfg_defaults, injected_noise, modelling
    cfg = get_cfg_defaults()
    cfg.MODEL.LOSS.REDUCTION = "mean"
    cfg.MODEL.LOSS.DISTORTION_LOSS_WEIGHT = 256.0
    cfg.MODEL.COMPUTE_DTYPE = "fp32_split"
    torch.manual_seed(0)
    m = modelling.build_model(cfg).to(DEV).train()
    g = torch.Generator().manual_seed(3)
    x = torch.rand(32, 3, 256, 256, generator=g).to(DEV)
    uz = torch.rand(32, 192, 4, 4, generator=g).to(DEV)
    uy = torch.rand(32, 192, 16, 16, generator=g).to(DEV)
    runs = []
    import warnings
    with warnings.catch_warnings():
        # a stream mismatch would mean an AccumulateGrad node outlived its run (see below)
        warnings.filterwarnings("error", message="The AccumulateGrad node's stream does not match")
        for conc in [False] + [True] * 8:
            m.concurrent_hyperprior = conc
            m.zero_grad(set_to_none=True)
            with injected_noise([uz, uy]):
                xt, losses = m(x)
                losses["total_loss"].backward()
            # drop the graph: a live graph keeps the parameters' AccumulateGrad nodes, and a node
            # made by the serial run (main stream) would then accumulate the side stream's
            # gradients of the next, concurrent run on the main stream
            del xt, losses
            torch.cuda.synchronize()
            runs.append({k: p.grad.clone() for k, p in m.named_parameters()})
    for i, r in enumerate(runs[1:], 1):
        for k, v in r.items():
            assert torch.equal(v, runs[0][k]), (i, k)
