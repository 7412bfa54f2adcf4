#!/usr/bin/env python3
"""Rehearsal of the DDP step's stream behaviour on ONE GPU (verdict item 5): two ranks, gloo over GPU
tensors on the box's one GPU (RCCL needs a GPU per rank), each running the C2 model (batch 8, 256^2)
under distributed.wrap -- 12 MB buckets, the hyperprior side stream, the comm-stream all-reduce hook.
Run it under `rocprofv3 --kernel-trace` and read each process's trace with tools/trace_timeline.py:
the main queue's gaps during the backward, and what the comm queue (the hook's divide and gloo's
device copies) was doing meanwhile.  GPU only.

    rocprofv3 --kernel-trace -d OUT -o run --output-format csv -- python3 tools/ddp_trace.py
"""
import os
import socket
import sys

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _worker(rank, world, port, steps):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), IMGCOMP_DIST_BACKEND="gloo")
    import bench
    from image_compression_amd import distributed as D
    from image_compression_amd import modelling
    _, _, dev = D.setup()
    torch.manual_seed(0)
    model = D.wrap(modelling.build_model(bench._cfg(conf=dict(bench.CONFIGS["C2"]))).to(dev).train(), dev)
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    x = torch.rand(8, 3, 256, 256, device=dev, generator=g)
    for _ in range(steps):
        model.zero_grad(set_to_none=True)
        _, losses = model(x)
        losses["total_loss"].backward()
    torch.cuda.synchronize()
    D.barrier(dev)
    if rank == 0:
        print("ddp rehearsal done:", steps, "steps, 2 ranks (gloo, one GPU)", flush=True)
    D.teardown()


def main():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    mp.spawn(_worker, args=(2, port, 6), nprocs=2, join=True)


if __name__ == "__main__":
    main()
