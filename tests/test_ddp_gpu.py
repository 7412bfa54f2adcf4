"""The data-parallel path with the HIP kernels: two ranks (gloo over GPU
tensors, sharing the box's one GPU — the RCCL path needs one GPU per rank),
each on half the batch under DistributedDataParallel, average to the
single-process gradient of the whole batch (injected noise, fixed weights)."""
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
    from image_compression_amd import distributed as D
    from image_compression_amd import injected_noise, modelling
    _, _, dev = D.setup()
    torch.manual_seed(0)
    model = D.wrap(modelling.build_model(_cfg()).to(dev).train(), dev, bucket_cap_mb=4.0)
    x, uz, uy = (D.shard(t, rank, world).to(dev) for t in _inputs())
    for _ in range(2):       # DDP raises on the 2nd iteration if a parameter went unused
        model.zero_grad(set_to_none=True)
        with injected_noise([uz, uy]):
            _, losses = model(x)
        losses["total_loss"].backward()
    torch.cuda.synchronize()
    if rank == 0:
        torch.save({n: p.grad.detach().cpu() for n, p in model.module.named_parameters()},
                   os.path.join(outdir, "g.pt"))
    D.teardown()


def test_ddp_two_ranks_match_full_batch(tmp_path):
    from conftest import rel_err
    from image_compression_amd import injected_noise, modelling
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.start_processes(_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    g = torch.load(os.path.join(tmp_path, "g.pt"), weights_only=True)
    torch.manual_seed(0)
    model = modelling.build_model(_cfg()).cuda().train()
    x, uz, uy = (t.cuda() for t in _inputs())
    with injected_noise([uz, uy]):
        _, losses = model(x)
    losses["total_loss"].backward()
    worst = max((rel_err(g[n], p.grad.cpu()), n) for n, p in model.named_parameters())
    assert worst[0] < 1e-4, worst
