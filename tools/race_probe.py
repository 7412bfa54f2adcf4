#!/usr/bin/env python3
"""Hunt the rare gradient mismatch of the concurrent hyperprior step (C2: batch 32, 256^2,
fp32_split, injected noise): many steps, each compared bitwise with a serial reference step.
Patterns: 'conc' (concurrent steps back to back), 'alt' (serial, concurrent, serial, ...).
Reports every mismatching run, the tensors and elements that differ.  GPU only.

    python tools/race_probe.py --reps 60 --pattern alt
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from image_compression_amd import get_cfg_defaults, injected_noise, modelling  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=60)
    ap.add_argument("--pattern", default="conc", choices=["conc", "alt"])
    ap.add_argument("--keep-graph", action="store_true", help="keep each run's graph alive into the next")
    ap.add_argument("--check-fact", action="store_true",
                    help="snapshot every factorized-backward launch's inputs and outputs (stream-ordered clones) "
                         "and recompute it on an idle GPU after the step: tells an in-kernel fault from bad inputs")
    a = ap.parse_args()
    from image_compression_amd import _lib
    from image_compression_amd import functional as IF
    snaps = []
    if a.check_fact:
        ops = _lib.ops()
        orig = IF.FactorizedFn.backward

        def wrapped(ctx, gq, gp):
            q, *prm = ctx.saved_tensors
            res = orig(ctx, gq, gp)
            gql = None if (gq is None or ctx.mode == 1) else IF._to_last(gq)
            gpl = None if gp is None else IF._to_last(gp)
            snaps.append(dict(q=q.clone(), prm=[t.clone() for t in prm], gq=None if gql is None else gql.clone(),
                              gp=None if gpl is None else gpl.clone(), C=ctx.C,
                              out=[t.detach().clone() for t in res if torch.is_tensor(t)]))
            return res
        IF.FactorizedFn.backward = staticmethod(wrapped)
    cfg = get_cfg_defaults()
    cfg.MODEL.LOSS.REDUCTION = "mean"
    cfg.MODEL.LOSS.DISTORTION_LOSS_WEIGHT = 256.0
    cfg.MODEL.COMPUTE_DTYPE = "fp32_split"
    torch.manual_seed(0)
    m = modelling.build_model(cfg).cuda().train()
    g = torch.Generator().manual_seed(3)
    x = torch.rand(32, 3, 256, 256, generator=g).cuda()
    uz = torch.rand(32, 192, 4, 4, generator=g).cuda()
    uy = torch.rand(32, 192, 16, 16, generator=g).cuda()

    def step(conc):
        m.concurrent_hyperprior = conc
        m.zero_grad(set_to_none=True)
        with injected_noise([uz, uy]):
            xt, losses = m(x)
            losses["total_loss"].backward()
        torch.cuda.synchronize()
        out = {k: p.grad.clone() for k, p in m.named_parameters()}
        out["x_tilde"] = xt.clone()
        return out, (xt, losses)

    ref, keep = step(False)
    snaps.clear()
    if not a.keep_graph:
        del keep
    seq = [True] * a.reps if a.pattern == "conc" else [c for _ in range(a.reps) for c in (False, True)]
    bad = {True: 0, False: 0}
    for i, conc in enumerate(seq):
        r, keep2 = step(conc)
        if a.keep_graph:
            keep = keep2
        del keep2
        if a.check_fact:
            torch.cuda.synchronize()
            for sn in snaps:
                dz, grads = ops.factorized_bwd(sn["q"], sn["C"], sn["prm"], sn["gq"], sn["gp"])
                torch.cuda.synchronize()
                again = [dz] + list(grads)
                # out[0] is dz in (N, C, *) order; compare the parameter gradients and dz's storage
                bad_k = [j for j, (u, v) in enumerate(zip(sn["out"][1:], again[1:])) if not torch.equal(u, v)]
                if bad_k:
                    print(f"run {i}: factorized_bwd output differs from its recompute on the same inputs: "
                          f"grads {bad_k}", flush=True)
                    for j in bad_k[:3]:
                        u, v = sn["out"][1 + j].flatten(), again[1 + j].flatten()
                        idx = (u != v).nonzero().flatten()
                        print(f"   grad {j}: {idx.numel()} elements, first {idx[:6].tolist()} "
                              f"got {[float(u[t]) for t in idx[:3]]} recomputed {[float(v[t]) for t in idx[:3]]}",
                              flush=True)
            snaps.clear()
        diffs = [k for k in r if not torch.equal(r[k], ref[k])]
        if diffs:
            bad[conc] += 1
            print(f"run {i} concurrent={conc}: {len(diffs)} tensors differ", flush=True)
            for k in diffs[:6]:
                va, vb = r[k].flatten(), ref[k].flatten()
                idx = (va != vb).nonzero().flatten()
                print(f"   {k}: {idx.numel()}/{va.numel()} elements, first {idx[:8].tolist()}, "
                      f"got {[float(va[j]) for j in idx[:3]]} want {[float(vb[j]) for j in idx[:3]]}", flush=True)
    n_c = sum(1 for c in seq if c)
    print(f"pattern={a.pattern} keep_graph={a.keep_graph}: mismatching concurrent runs {bad[True]}/{n_c}, "
          f"serial runs {bad[False]}/{len(seq) - n_c}", flush=True)


if __name__ == "__main__":
    main()
