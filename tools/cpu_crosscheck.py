#!/usr/bin/env python3
"""CPU-baseline cross-check: the oracle restatement (oracle/ref_cpu.py, the
`cpu_baseline` leg of bench.py) must time within +-10 % of the reference itself on the same
host, threads and workload: psnr_256 semantics, batch 8, 256x256, fp32, fwd + RD loss + bwd.

Runs ONLY in the build container (imports /root/reference through tools/_refimport.py; the
reference never ships).  Writes one JSON record:

    python tools/cpu_crosscheck.py [--iters 5] [--threads 8] [--out profiles/r02_cpu_crosscheck.json]
"""
import argparse
import json
import os
import platform
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(1, os.path.dirname(HERE))
from _refimport import available, import_reference  # noqa: E402


def _time(fn, iters):
    fn()  # warm-up
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    return (time.perf_counter() - t0) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--out", default=os.path.join(os.path.dirname(HERE), "profiles", "r02_cpu_crosscheck.json"))
    a = ap.parse_args()
    if not available():
        sys.exit("reference tree not present: this cross-check runs only in the build container")
    torch.set_num_threads(a.threads)
    modelling, get_cfg_defaults = import_reference()
    from oracle import ref_cpu
    cfg = get_cfg_defaults()
    cfg.MODEL.LOSS.REDUCTION = "mean"
    cfg.MODEL.LOSS.DISTORTION_LOSS_WEIGHT = 256.0
    torch.manual_seed(0)
    model = modelling.build_model(cfg).train()
    g = torch.Generator().manual_seed(0)
    N = 8
    x = torch.rand(N, 3, 256, 256, generator=g)
    uz = torch.rand(N, 192, 4, 4, generator=g)
    uy = torch.rand(N, 192, 16, 16, generator=g)
    params = {k: v.detach().clone() for k, v in model.state_dict().items()}

    def ref_step():
        model.zero_grad(set_to_none=True)
        _, losses = model(x)
        losses["total_loss"].backward()

    def oracle_step():
        ref_cpu.run(params, x, uz, uy, train=True, dtype=torch.float32, lam=256.0)

    # interleave the two so drift of the host's clock affects both alike
    t_ref, t_orc = [], []
    for _ in range(2):
        t_ref.append(_time(ref_step, a.iters))
        t_orc.append(_time(oracle_step, a.iters))
    ref_ips = N / min(t_ref)
    orc_ips = N / min(t_orc)
    rec = {"workload": "psnr_256: batch 8, 256x256, fp32, fwd + RD loss + bwd (train mode)",
           "threads": a.threads, "iters_per_sample": a.iters, "host": platform.processor() or platform.machine(),
           "torch": torch.__version__,
           "reference_images_per_s": round(ref_ips, 3), "oracle_images_per_s": round(orc_ips, 3),
           "oracle_over_reference": round(orc_ips / ref_ips, 4),
           "within_10pct": abs(orc_ips / ref_ips - 1) <= 0.10}
    with open(a.out, "w") as f:
        json.dump(rec, f, indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
