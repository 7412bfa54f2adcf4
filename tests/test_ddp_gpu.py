"""The data-parallel path with the HIP kernels: two ranks (gloo over GPU
tensors, sharing the box's one GPU — the RCCL path needs one GPU per rank),
each on half the batch, average to the single-process gradient of the whole
batch (injected noise, fixed weights) -- under DistributedDataParallel with the
hyperprior side stream (D.wrap's comm hook issues each bucket's all-reduce on a comm
stream that waits for every gradient-producing stream; bitwise equal to the single-stream DDP step) and through TrainStep's flat
gradient buffer and one all-reduce.  The ranks'
training-noise keys differ (noise.rank_key).  Unmeasured on RCCL hardware:
the box has one GPU."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
N, S = 4, 64


def _cfg():
    from image_compression_amd import get_cfg_defaults
    cfg = get_cfg_defaults()
    cfg.MODEL.LOSS.REDUCTION = "mean"
    cfg.MODEL.LOSS.DISTORTION_LOSS_WEIGHT = 256.0
    return cfg


def _inputs():
    g = torch.Generator().manual_seed(21)
    x = torch.rand(N, 3, S, S, generator=g)
    uz = torch.rand(N, 192, S // 64, S // 64, generator=g)
    uy = torch.rand(N, 192, S // 16, S // 16, generator=g)
    return x, uz, uy


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), IMGCOMP_DIST_BACKEND="gloo")
    import warnings
    # as tests/conftest.py: a gradient accumulated on another stream than its producer's is an error
    warnings.filterwarnings("error", message="(?s).*AccumulateGrad node's stream does not match")
    from image_compression_amd import distributed as D
    from image_compression_amd import injected_noise, modelling
    from image_compression_amd import noise
    from image_compression_amd.step import TrainStep
    _, _, dev = D.setup()
    x, uz, uy = (D.shard(t, rank, world).to(dev) for t in _inputs())
    ddp_grads = {}
    for conc in (True, False):
        torch.manual_seed(0)
        model = D.wrap(modelling.build_model(_cfg()).to(dev).train(), dev, bucket_cap_mb=4.0, concurrent=conc)
        assert model.module.concurrent_hyperprior is conc     # the side stream stays on under DDP
        for _ in range(3):       # DDP raises on the 2nd iteration if a parameter went unused; buckets rebuilt
            model.zero_grad(set_to_none=True)
            with injected_noise([uz, uy]):
                _, losses = model(x)
            losses["total_loss"].backward()
        torch.cuda.synchronize()
        ddp_grads[conc] = {n: p.grad.detach().cpu() for n, p in model.module.named_parameters()}
        del model, losses
    # the concurrent DDP step run under another stream than the one current at wrap(): the hook also
    # follows the stream current at hook time (torch syncs the mismatched accumulations itself; its
    # warning about them is expected here)
    torch.manual_seed(0)
    model = D.wrap(modelling.build_model(_cfg()).to(dev).train(), dev, bucket_cap_mb=4.0, concurrent=True)
    other = torch.cuda.Stream(device=dev)
    other.wait_stream(torch.cuda.current_stream(dev))
    with warnings.catch_warnings():
        warnings.filterwarnings("ignore", message="(?s).*AccumulateGrad node's stream does not match")
        with torch.cuda.stream(other):
            for _ in range(3):
                model.zero_grad(set_to_none=True)
                with injected_noise([uz, uy]):
                    _, losses = model(x)
                losses["total_loss"].backward()
    torch.cuda.synchronize()
    ddp_grads["other"] = {n: p.grad.detach().cpu() for n, p in model.module.named_parameters()}
    del model, losses
    # the hipGraph-capable step without DDP: gradients as views of one flat buffer, one
    # all-reduce after the backward, hyperprior side stream on
    torch.manual_seed(0)
    m2 = modelling.build_model(_cfg()).to(dev).train()
    assert m2.concurrent_hyperprior
    st = TrainStep(m2, x, graph=False)
    assert st.flat_grad is not None
    with injected_noise([uz, uy]):
        st(x)
    torch.cuda.synchronize()
    flat_grads = {n: p.grad.detach().cpu() for n, p in m2.named_parameters()}
    # the training-noise keys of the two ranks (device state, rank folded in)
    key = noise.device_state(dev)[0:1].clone()
    keys = [torch.zeros_like(key) for _ in range(world)]
    torch.distributed.all_gather(keys, key)
    if rank == 0:
        torch.save({"ddp": ddp_grads[True], "ddp_serial": ddp_grads[False], "ddp_other": ddp_grads["other"],
                    "flat": flat_grads,
                    "keys": [int(k) for k in keys], "seed": noise._st().seed}, os.path.join(outdir, "g.pt"))
    D.teardown()


def test_ddp_two_ranks_match_full_batch(tmp_path):
    from conftest import rel_err
    from image_compression_amd import injected_noise, modelling
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.start_processes(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    res = torch.load(os.path.join(tmp_path, "g.pt"), weights_only=True)
    from image_compression_amd import noise
    assert res["keys"] == [noise.rank_key(res["seed"], r) for r in range(2)] and res["keys"][0] != res["keys"][1]
    torch.manual_seed(0)
    model = modelling.build_model(_cfg()).cuda().train()
    x, uz, uy = (t.cuda() for t in _inputs())
    with injected_noise([uz, uy]):
        _, losses = model(x)
    losses["total_loss"].backward()
    # the concurrent-hyperprior DDP step (the measured step) is bitwise the single-stream one
    for n in res["ddp"]:
        assert torch.equal(res["ddp"][n], res["ddp_serial"][n]), n
        assert torch.equal(res["ddp_other"][n], res["ddp_serial"][n]), n
    for kind in ("ddp", "flat"):
        g = res[kind]
        worst = max((rel_err(g[n], p.grad.cpu()), n) for n, p in model.named_parameters())
        assert worst[0] < 1e-4, (kind, worst)
