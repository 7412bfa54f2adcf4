"""Data-parallel plumbing: one process per GPU, gradients averaged by RCCL.

The reference wraps the model in `nn.DataParallel` (engine/trainer.py:256-259):
one process, one Python thread per GPU, replicas re-broadcast every step.
Here each GPU is its own process (launched by `torch.distributed.run`), the
model is replicated once, and `DistributedDataParallel` all-reduces the
gradients in buckets while the backward pass is still running (backend
"nccl" = RCCL over xGMI on ROCm; "gloo" for CPU tests).

Why averaged per-rank gradients equal the reference's single-device gradients
(SURVEY.md 8e): with equal shards of the batch, every loss term is a mean over
the batch (MSE mean, bpp = sum(ce) / (N*H*W), MS-SSIM-log = -mean over N), so
the mean of per-rank losses is the full-batch loss and the mean of per-rank
gradients is its gradient.  tests/test_distributed.py checks this with gloo.
"""
import os

import torch
import torch.distributed as dist

# RCCL over the dmabuf IPC path (the only one the host driver supports)
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")


def env_ranks():
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def setup(backend=None, device_type=None):
    """Initialise the process group when WORLD_SIZE > 1 and pick this rank's
    device.  Returns (rank, world, device).

    backend: None -> "nccl" (RCCL) on GPUs, "gloo" on CPU; IMGCOMP_DIST_BACKEND
    overrides it (e.g. gloo over GPU tensors to rehearse several ranks on one
    GPU).  device_type: "cuda" / "cpu" (default: cuda when available).  When
    there are fewer GPUs than local ranks (rehearsal only), ranks share GPUs
    round-robin."""
    rank, world, local = env_ranks()
    backend = os.environ.get("IMGCOMP_DIST_BACKEND", backend)
    use_gpu = (device_type or ("cuda" if torch.cuda.is_available() else "cpu")) == "cuda"
    if use_gpu:
        ndev = torch.cuda.device_count()
        dev_idx = local % ndev if ndev else local
        torch.cuda.set_device(dev_idx)
        device = torch.device("cuda", dev_idx)
    else:
        device = torch.device("cpu")
    if world > 1 and not dist.is_initialized():
        dist.init_process_group(backend or ("nccl" if use_gpu else "gloo"))
    return rank, world, device


def teardown():
    if dist.is_initialized():
        dist.destroy_process_group()


def wrap(model, device, bucket_cap_mb=12.0):
    """DDP over the model.  12 MB buckets ~ one bucket per transform
    (g_s 11.6 MB, h_s+EM 8.7 MB, h_a 8.7 MB, g_a 11.6 MB): the
    first all-reduce starts as soon as g_s's gradients are ready and overlaps
    the rest of the backward.  Gradients are views into the buckets (no copy).

    The one place that decides the hyperprior side stream under data parallelism:
    off.  DDP keeps the AccumulateGrad nodes it made at wrap time (on the current
    stream) for the model's life, and its bucket all-reduce waits only for the
    stream that readied the bucket; with the hyperprior's backward on a second
    stream a bucket would mix gradients finished on two streams with no per-bucket
    stream join.  The side stream is worth ~1 % of a C2 step at one rank
    (14.39 -> 14.24-14.29 ms); under DDP every rank runs the
    single-stream step, bitwise the same arithmetic."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return model
    if hasattr(model, "concurrent_hyperprior"):
        model.concurrent_hyperprior = False
    from torch.nn.parallel import DistributedDataParallel as DDP
    ids = [device.index] if device.type == "cuda" else None
    return DDP(model, device_ids=ids, bucket_cap_mb=bucket_cap_mb, gradient_as_bucket_view=True,
               broadcast_buffers=False)


def shard(t, rank, world):
    """This rank's contiguous slice of a batch-major tensor (equal shards)."""
    n = t.shape[0]
    if n % world:
        raise ValueError(f"batch {n} does not split evenly over {world} ranks")
    per = n // world
    return t[rank * per:(rank + 1) * per]


def max_over_ranks(value, device):
    """Max of a host float over all ranks (the timed region's wall clock)."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return float(value)
    t = torch.tensor([float(value)], device=device, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def mean_over_ranks(values, device):
    """Average a dict of 0-dim loss tensors over ranks (logging only)."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return {k: float(v) for k, v in values.items()}
    keys = sorted(values)
    t = torch.stack([values[k].detach().to(device=device, dtype=torch.float64) for k in keys])
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    t /= dist.get_world_size()
    return {k: float(v) for k, v in zip(keys, t.tolist())}


def all_reduce_mean_(t):
    """In-place average of `t` over all ranks: one RCCL all-reduce with ReduceOp.AVG
    ("nccl"), SUM and a division where the backend has no AVG (gloo)."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return t
    if dist.get_backend() == "nccl":
        dist.all_reduce(t, op=dist.ReduceOp.AVG)
    else:
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        t.div_(dist.get_world_size())
    return t


def barrier(device):
    if dist.is_initialized() and dist.get_world_size() > 1:
        if device.type == "cuda" and dist.get_backend() == "nccl":
            dist.barrier(device_ids=[device.index])
        else:
            dist.barrier()
