"""Data-parallel path on CPU (gloo, world_size 2): the per-rank shards with
DDP gradient averaging reproduce the single-process gradient of the whole
batch, through image_compression_amd.distributed — the same
setup / wrap / shard / max-over-ranks helpers bench.py runs over RCCL.

The model computed here is the CPU oracle (oracle/ref_cpu.py) wrapped as an
nn.Module: the HIP path cannot run without a GPU, and the property under test
(loss normalisation + bucketed all-reduce = full-batch gradient) is a
property of the data-parallel decomposition, not of the kernels.  The GPU
kernels' parity is covered by the -m gpu tests."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from oracle import ref_cpu

N, S = 4, 64   # global batch, image size (reduced width keeps it fast)


def _small_cfg():
    from image_compression_amd import get_cfg_defaults
    cfg = get_cfg_defaults()
    cfg.MODEL.INTER_CHANNELS = 16
    cfg.MODEL.LATENT_CHANNELS = 16
    cfg.MODEL.LOSS.REDUCTION = "mean"
    cfg.MODEL.LOSS.DISTORTION_LOSS_WEIGHT = 256.0
    return cfg


class OracleModel(torch.nn.Module):
    """ref_cpu.forward over parameters registered under the reference's
    state-dict names (dots mapped to '__' for registration)."""

    def __init__(self, params):
        super().__init__()
        self.keys = sorted(params)
        for k in self.keys:
            self.register_parameter(k.replace(".", "__"), torch.nn.Parameter(params[k].clone().double()))

    def forward(self, x, uz, uy):
        P = {k: getattr(self, k.replace(".", "__")) for k in self.keys}
        _, losses = ref_cpu.forward(P, x, uz, uy, train=True, lam=256.0)
        return losses


def _inputs():
    g = torch.Generator().manual_seed(7)
    x = torch.rand(N, 3, S, S, generator=g, dtype=torch.float64)
    uz = torch.rand(N, 16, S // 64, S // 64, generator=g, dtype=torch.float64)
    uy = torch.rand(N, 16, S // 16, S // 16, generator=g, dtype=torch.float64)
    return x, uz, uy


def _params():
    from image_compression_amd import modelling
    torch.manual_seed(3)
    return {k: v.clone() for k, v in modelling.build_model(_small_cfg()).state_dict().items()}


def _worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from image_compression_amd import distributed as D
    r, w, dev = D.setup("gloo", device_type="cpu")
    assert (r, w, dev.type) == (rank, world, "cpu")
    torch.set_num_threads(2)
    model = D.wrap(OracleModel(_params()), dev, bucket_cap_mb=1.0)
    assert isinstance(model, torch.nn.parallel.DistributedDataParallel)
    x, uz, uy = (D.shard(t, rank, world) for t in _inputs())
    # two iterations: DDP raises on the second if any parameter went unused
    for _ in range(2):
        model.zero_grad(set_to_none=True)
        losses = model(x, uz, uy)
        losses["total_loss"].backward()
    grads = {k: p.grad.detach().clone() for k, p in model.module.named_parameters()}
    mean = D.mean_over_ranks({"total_loss": losses["total_loss"], "bpp": losses["bpp"]}, dev)
    t = D.max_over_ranks(float(rank + 1), dev)
    D.barrier(dev)
    if rank == 0:
        torch.save({"grads": grads, "mean": mean, "tmax": t}, os.path.join(outdir, "rank0.pt"))
    D.teardown()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_ddp_gloo_matches_full_batch(tmp_path):
    world = 2
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    res = torch.load(os.path.join(tmp_path, "rank0.pt"), weights_only=True)
    # single process, whole batch
    full = OracleModel(_params())
    losses = full(*_inputs())
    losses["total_loss"].backward()
    assert res["tmax"] == 2.0
    assert abs(res["mean"]["total_loss"] - float(losses["total_loss"].detach())) <= 1e-9 * abs(float(losses["total_loss"].detach()))
    assert abs(res["mean"]["bpp"] - float(losses["bpp"])) <= 1e-9 * max(abs(float(losses["bpp"])), 1e-12)
    for k, p in full.named_parameters():
        g = res["grads"][k]
        rel = ((g - p.grad).norm() / p.grad.norm().clamp_min(1e-30)).item()
        assert rel < 1e-9, (k, rel)


def test_shard_and_single_rank_helpers():
    from image_compression_amd import distributed as D
    t = torch.arange(12).view(6, 2)
    assert torch.equal(D.shard(t, 1, 3), t[2:4])
    with pytest.raises(ValueError):
        D.shard(t, 0, 4)
    m = torch.nn.Linear(2, 2)
    assert D.wrap(m, torch.device("cpu")) is m          # no process group: no wrapper
    assert D.max_over_ranks(3.5, torch.device("cpu")) == 3.5


def _key_worker(rank, world, port, outdir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    from image_compression_amd import distributed as D
    from image_compression_amd import noise
    # a device state made before the process group exists carries rank 0's key ...
    noise.reseed(99)
    dev = torch.device("cpu", 0)
    early = int(noise.device_state(dev)[0])
    assert early == noise.rank_key(99, 0)
    D.setup("gloo", device_type="cpu")
    # ... and is re-keyed for this rank at its next use (counters kept)
    noise.device_state(dev)[1] += 12
    st, off = noise.philox_stream(8, dev)
    assert int(st[0]) == noise.rank_key(99, rank) and int(st[1]) == 12 and off == 0
    noise.reseed()
    torch.manual_seed(0)                       # every rank seeds alike, as bench.py does
    seed = int(torch.randint(0, 2 ** 62, (1,)).item())
    keys = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    torch.distributed.all_gather(keys, torch.tensor([noise.process_key(seed)]))
    if rank == 0:
        torch.save({"seed": seed, "keys": [int(k) for k in keys]}, os.path.join(outdir, "keys.pt"))
    D.teardown()


def test_ranks_draw_independent_noise(tmp_path):
    """Under data parallelism every rank seeds alike; the rank folded into the Philox key
    gives each rank its own z / y draws (the reference's one process draws torch.rand_like
    over its whole batch: no image shares noise with another, entropy_model.py:230,333)."""
    import numpy as np

    from image_compression_amd import noise
    from oracle import philox
    world = 4
    mp.start_processes(_key_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    res = torch.load(os.path.join(tmp_path, "keys.pt"), weights_only=True)
    seed, keys = res["seed"], res["keys"]
    assert keys[0] == seed                                   # rank 0 keeps the single-process stream
    assert keys == [noise.rank_key(seed, r) for r in range(world)]
    assert len(set(keys)) == world and all(0 <= k < 2 ** 62 for k in keys)
    # one C2-sized step per rank: z (32 x 192 x 4 x 4) then y (32 x 192 x 16 x 16), 4-aligned offsets
    nz, ny = 32 * 192 * 16, 32 * 192 * 256
    draws = [np.concatenate([philox.uniform(nz, k, 0), philox.uniform(ny, k, nz)]) for k in keys]
    for a in range(world):
        for b in range(a + 1, world):
            same = int((draws[a] == draws[b]).sum())
            # independent 24-bit uniforms coincide with probability 2^-24 per element
            assert same <= 8, (a, b, same)
            assert abs(float(np.corrcoef(draws[a], draws[b])[0, 1])) < 0.01


def test_rank_key_is_a_fixed_function():
    from image_compression_amd import noise
    assert noise.rank_key(12345, 0) == 12345
    assert noise.rank_key(12345, 1) == noise.rank_key(12345, 1) != noise.rank_key(12345, 2)
    assert noise.rank_key(12345, 1) != noise.rank_key(12346, 1)
    assert noise.process_key(777) == 777                     # no process group: rank 0
