#!/usr/bin/env python3
"""Golden LR-schedule vectors from the reference's own scheduler code
(solver/lr_scheduler.py — plain torch, importable here) for
tests/test_solver.py.  Runs only in the build container; writes
tests/golden/lr_schedules.json (data only).

Each case: a one-parameter optimizer with lr = 1 driven through the
reference's make_lr_scheduler(cfg, optimizer, iters_per_epoch) for N steps;
the recorded values are the multipliers get_last_lr()[0] after each step.
"""
import importlib.util
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from _refimport import REF_ROOT, _CfgNode  # noqa: E402

OUT = os.path.join(os.path.dirname(HERE), "tests", "golden", "lr_schedules.json")

BASE = dict(USE_ITER=False, NUM_EPOCHS=6, DECAY_EPOCHS=2, NUM_COSINE_CYCLE=0.21875, DECAY_RATE=0.97,
            WARMUP_EPOCHS=1, GD_STEPS=1, NUM_ITERS=40, WARMUP_ITERS=5, STEPS=(12, 25), GAMMA=0.1,
            WARMUP_FACTOR=1.0 / 3, WARMUP_METHOD="linear")
CASES = [
    ("constant", dict(USE_ITER=True)),
    ("cosine_warmup", dict(USE_ITER=True)),
    ("cosine_warmup", dict()),
    ("constant_warmup", dict()),
    ("decay_warmup", dict()),
    ("multistep_warmup", dict()),
    ("multistep_warmup", dict(WARMUP_METHOD="constant")),
]
ITERS_PER_EPOCH, NSTEPS = 7, 45


def main():
    spec = importlib.util.spec_from_file_location("ref_lr", os.path.join(REF_ROOT, "solver", "lr_scheduler.py"))
    ref = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ref)
    out = []
    for name, over in CASES:
        solver = _CfgNode(BASE)
        solver.update(over)
        solver["SCHEDULER_NAME"] = name
        cfg = _CfgNode(SOLVER=solver)
        opt = torch.optim.SGD([torch.nn.Parameter(torch.zeros(1))], lr=1.0)
        sch = ref.make_lr_scheduler(cfg, opt, ITERS_PER_EPOCH)
        vals = []
        for _ in range(NSTEPS):
            opt.step()
            sch.step()
            vals.append(float(sch.get_last_lr()[0]))
        out.append({"name": name, "solver": {k: (list(v) if isinstance(v, tuple) else v) for k, v in solver.items()},
                    "iters_per_epoch": ITERS_PER_EPOCH, "lrs": vals})
    with open(OUT, "w") as f:
        json.dump(out, f, indent=0)
    print("wrote", OUT, len(out), "cases")


if __name__ == "__main__":
    main()
