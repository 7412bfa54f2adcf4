#!/usr/bin/env python3
"""Host-side timing of the C2 training step: how long the CPU spends issuing the forward and the
backward (no synchronisation inside) against the step's wall time, and a torch.profiler CPU
summary of one backward.  GPU only.

    python tools/host_step.py
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from image_compression_amd import modelling  # noqa: E402


def main():
    conf = dict(bench.CONFIGS["C2"])
    torch.manual_seed(0)
    model = modelling.build_model(bench._cfg(conf=conf)).cuda().train()
    x = torch.rand(conf["batch"], 3, conf["size"], conf["size"], device="cuda")
    for _ in range(5):
        model.zero_grad(set_to_none=True)
        _, losses = model(x)
        losses["total_loss"].backward()
    torch.cuda.synchronize()
    fw, bw, wall = [], [], []
    for _ in range(10):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        model.zero_grad(set_to_none=True)
        _, losses = model(x)
        t1 = time.perf_counter()
        losses["total_loss"].backward()
        t2 = time.perf_counter()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        fw.append(t1 - t0); bw.append(t2 - t1); wall.append(t3 - t0)
    med = lambda v: 1e3 * sorted(v)[len(v) // 2]
    print(f"host forward {med(fw):.3f} ms, host backward {med(bw):.3f} ms, step wall {med(wall):.3f} ms")
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU]) as prof:
        model.zero_grad(set_to_none=True)
        _, losses = model(x)
        losses["total_loss"].backward()
        torch.cuda.synchronize()
    print(prof.key_averages().table(sort_by="self_cpu_time_total", row_limit=25))


if __name__ == "__main__":
    main()
