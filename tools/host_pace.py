#!/usr/bin/env python3
"""Does the host or the GPU pace the eager training step?  Runs the bench step of a config and reports,
per step, the host's enqueue time (the Python loop without a synchronize) beside the GPU's time per
step (the loop bracketed by synchronizes).  If the enqueue time is close to the step time the host
paces and main-queue gaps are launch gaps.  GPU only.

    python tools/host_pace.py [--config C4] [--steps 20]
"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="C4")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--serial-hyperprior", action="store_true")
    a = ap.parse_args()
    import bench
    from image_compression_amd import modelling
    conf = dict(bench.CONFIGS[a.config])
    torch.manual_seed(0)
    dev = torch.device("cuda:0")
    model = modelling.build_model(bench._cfg(conf=conf)).to(dev).train()
    if a.serial_hyperprior:
        model.concurrent_hyperprior = False
    x = torch.rand(conf["batch"], 3, conf["size"], conf["size"], device=dev)

    def step():
        model.zero_grad(set_to_none=True)
        _, losses = model(x)
        losses["total_loss"].backward()
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    for rep in range(3):
        t0 = time.perf_counter()
        marks = []
        for _ in range(a.steps):
            step()
            marks.append(time.perf_counter())
        t_enq = marks[-1] - t0
        torch.cuda.synchronize()
        t_all = time.perf_counter() - t0
        per = [1e3 * (b - a_) for a_, b in zip([t0] + marks[:-1], marks)]
        print(f"{a.config}: host enqueue {1e3 * t_enq / a.steps:.3f} ms/step (first {per[0]:.2f}, min {min(per):.2f}, median "
              f"{sorted(per)[len(per) // 2]:.2f}), GPU {1e3 * t_all / a.steps:.3f} ms/step", flush=True)


if __name__ == "__main__":
    main()
