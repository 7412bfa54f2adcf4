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


class _CommState:
    """State of the comm hook: the streams that produce gradients and a dedicated comm stream."""

    def __init__(self, streams, device):
        self.streams = list(streams)
        self.comm = torch.cuda.Stream(device=device)
        self.world = dist.get_world_size()


def _comm_stream_allreduce_hook(state, bucket):
    """DDP comm hook: each bucket's all-reduce on a dedicated comm stream that waits for every
    gradient-producing stream; no compute stream ever waits on another here.

    The reducer calls a hook when the last gradient of a bucket has been accumulated, on that
    gradient's stream.  With the hyperprior on its side stream (and its convs' weight gradients on
    a third stream) a bucket can mix gradients finished on several streams, so the collective must
    follow all of them.  The comm stream waits on an event recorded at each producing stream's tail
    (recording costs the producer nothing: the main, side and weight-gradient streams go on with
    the backward), then divides the bucket by the world size and all-reduces it (SUM) in place --
    the default hook's arithmetic, issued under the comm stream, which RCCL's own stream then
    follows.  DDP's finalize waits for every bucket's future on the stream that ends the backward,
    and the next step's side-stream work follows that stream, so the gradient views are never
    rewritten while a collective reads them.  Unmeasured on RCCL hardware (one GPU per box here);
    tests/test_ddp_gpu.py checks the gradients bitwise with gloo over GPU tensors."""
    comm = state.comm
    for s in state.streams:
        comm.wait_stream(s)
    # and the stream current at hook time (a step run under another stream than the one current at
    # wrap() still has its bucket's gradients followed)
    comm.wait_stream(torch.cuda.current_stream(comm.device))
    buf = bucket.buffer()
    with torch.cuda.stream(comm):
        buf.div_(state.world)
        fut = dist.all_reduce(buf, async_op=True).get_future()
    return fut.then(lambda f: f.value()[0])


def wrap(model, device, bucket_cap_mb=12.0, concurrent=True):
    """DDP over the model.  12 MB buckets ~ one bucket per transform
    (g_s 11.6 MB, h_s+EM 8.7 MB, h_a 8.7 MB, g_a 11.6 MB): the
    first all-reduce starts as soon as g_s's gradients are ready and overlaps
    the rest of the backward.  Gradients are views into the buckets (no copy).

    The hyperprior side stream stays on under DDP (concurrent=True, on GPUs), so every rank
    runs the step bench.py measures at one rank.  Two things make that safe:
    * the hyperprior parameters' AccumulateGrad nodes are made on the streams their gradients
      are produced on (model.gradient_streams: the side stream, and the hyperprior convs'
      weight-gradient stream) before DDP takes them (DDP keeps the nodes it finds at
      construction for the model's life; made on the main stream, they would accumulate the
      other streams' gradients there, a cross-stream use of the gradient's memory the caching
      allocator is not told about);
    * a comm hook (_comm_stream_allreduce_hook) issues each bucket's all-reduce on a comm stream
      that waits for every such stream (the compute streams never wait for each other there).
    concurrent=False runs the single-stream step (bitwise the same arithmetic)."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return model
    from torch.nn.parallel import DistributedDataParallel as DDP
    conc = (concurrent and device.type == "cuda" and getattr(model, "concurrent_hyperprior", False)
            and hasattr(model, "hyperprior_modules"))
    if hasattr(model, "concurrent_hyperprior"):
        model.concurrent_hyperprior = conc
    keep, streams = [], [torch.cuda.current_stream(device)] if conc else []
    if conc:
        # (under enable_grad: a view made under no_grad has no grad_fn).  The nodes must not exist
        # yet: a node made earlier (by a forward in grad mode whose graph is still alive) would be
        # returned as it is, on whatever stream it was made -- wrap the model before its first step.
        with torch.enable_grad():
            for stream, params in model.gradient_streams(device):
                streams.append(stream)
                with torch.cuda.stream(stream):
                    for p in params:
                        if p.requires_grad:
                            gf = p.view_as(p).grad_fn
                            if gf is None:
                                raise RuntimeError("distributed.wrap: no AccumulateGrad node for a hyperprior "
                                                   "parameter")
                            keep.append(gf.next_functions[0][0])  # AccumulateGrad on `stream`
    ids = [device.index] if device.type == "cuda" else None
    ddp = DDP(model, device_ids=ids, bucket_cap_mb=bucket_cap_mb, gradient_as_bucket_view=True,
              broadcast_buffers=False)
    if conc:
        ddp.register_comm_hook(_CommState(streams, device), _comm_stream_allreduce_hook)
    del keep  # DDP holds the nodes now
    return ddp


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
