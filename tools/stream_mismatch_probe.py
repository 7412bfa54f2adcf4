#!/usr/bin/env python3
"""Which autograd state survives a C2 step and makes the next step's AccumulateGrad streams mismatch
(tests/conftest.py turns torch's warning into an error).  Three cases on fresh models: concurrent
steps only; a serial step then concurrent steps; the same with gc.collect() in between.  After each
step it lists the live tensors that still carry a grad_fn.  GPU only.

    python tools/stream_mismatch_probe.py
"""
import gc
import os
import sys
import warnings

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from image_compression_amd import get_cfg_defaults, injected_noise, modelling  # noqa: E402


def live_graph_tensors():
    out = []
    for o in gc.get_objects():
        try:
            if torch.is_tensor(o) and o.grad_fn is not None:
                out.append((tuple(o.shape), type(o.grad_fn).__name__))
        except Exception:
            pass
    return out


def main():
    warnings.filterwarnings("error", message="(?s).*AccumulateGrad node's stream does not match")
    cfg = get_cfg_defaults()
    cfg.MODEL.LOSS.REDUCTION = "mean"
    cfg.MODEL.LOSS.DISTORTION_LOSS_WEIGHT = 256.0
    g = torch.Generator().manual_seed(3)
    x = torch.rand(32, 3, 256, 256, generator=g).cuda()
    uz = torch.rand(32, 192, 4, 4, generator=g).cuda()
    uy = torch.rand(32, 192, 16, 16, generator=g).cuda()
    for case, pattern, collect in (("conc-only", [True, True, True], False),
                                   ("serial-then-conc", [False, True, True], False),
                                   ("serial-gc-conc", [False, True, True], True)):
        torch.manual_seed(0)
        m = modelling.build_model(cfg).cuda().train()
        res = []
        for i, conc in enumerate(pattern):
            m.concurrent_hyperprior = conc
            m.zero_grad(set_to_none=True)
            try:
                with injected_noise([uz, uy]):
                    _, losses = m(x)
                    losses["total_loss"].backward()
                del losses
                torch.cuda.synchronize()
                res.append("ok")
            except UserWarning as e:
                res.append("MISMATCH")
                print(f"  {case} step {i}: {str(e)[:90]}", flush=True)
                break
            if collect:
                print(f"  {case} step {i}: gc.collect() freed {gc.collect()} objects", flush=True)
            live = live_graph_tensors()
            print(f"  {case} step {i} ({'conc' if conc else 'serial'}): {len(live)} live tensors with grad_fn: "
                  f"{live[:12]}", flush=True)
        print(f"{case}: {res}", flush=True)
        del m
        gc.collect()


if __name__ == "__main__":
    main()
