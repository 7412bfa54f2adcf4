#!/usr/bin/env python3
"""A/B of a BASELINE config's training step (C2 default) with and without the hyperprior side
stream (Compressor2018.concurrent_hyperprior), alternating in one process.  GPU only.
    python tools/step_ab.py [--config C3] [--reps 4] [--steps 10]"""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from image_compression_amd import modelling  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--config", default="C2")
    a = ap.parse_args()
    conf = bench.CONFIGS[a.config]
    torch.manual_seed(0)
    m = modelling.build_model(bench._cfg(conf=conf)).cuda().train()
    x = torch.rand(conf["batch"], 3, conf["size"], conf["size"], device="cuda")

    def step():
        m.zero_grad(set_to_none=True)
        _, losses = m(x)
        losses["total_loss"].backward()
    arms = {"serial": False, "hyper": True}
    res = {k: [] for k in arms}
    for _ in range(a.reps):
        for name, hp in arms.items():
            m.concurrent_hyperprior = hp
            for _ in range(3):
                step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(a.steps):
                step()
            torch.cuda.synchronize()
            res[name].append(1e3 * (time.perf_counter() - t0) / a.steps)
    for name, v in res.items():
        print(f"{name:10s} ms/step min {min(v):.3f} median {sorted(v)[len(v) // 2]:.3f}")


if __name__ == "__main__":
    main()
