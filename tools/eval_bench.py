#!/usr/bin/env python3
"""Eval-path (inference) throughput: the reference's Kodak evaluator workload
(engine/evaluator.py:87-105 — model.eval(), batch-1 512x768 forwards, then bpp / PSNR /
MS-SSIM), on synthetic images resident in HBM with random-init weights (Kodak and trained
checkpoints are not in the container).  Times, per image: the eager forward (without and with
functional.weight_cache), the hipGraph
replay (evaluation.GraphForward), and the whole Evaluator.run_eval with and without the graph
(metrics included, host sync per image as the reference's monitor does).  One JSON line.

    python tools/eval_bench.py [--images 24] [--reps 3] [--config C2] [--batch 1]
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--images", type=int, default=24)  # the Kodak set
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1)
    ap.add_argument("--height", type=int, default=512)
    ap.add_argument("--width", type=int, default=768)
    args = ap.parse_args()
    from image_compression_amd import get_cfg_defaults, modelling
    from image_compression_amd import functional as F
    from image_compression_amd.evaluation import Evaluator, GraphForward
    cfg = get_cfg_defaults()
    cfg.MODEL.LOSS.REDUCTION = "mean"
    cfg.MODEL.LOSS.DISTORTION_LOSS_WEIGHT = 256.0
    torch.manual_seed(0)
    model = modelling.build_model(cfg).cuda().eval()
    g = torch.Generator(device="cuda").manual_seed(5)
    imgs = [torch.rand(args.batch, 3, args.height, args.width, device="cuda", generator=g)
            for _ in range(args.images)]

    def timed(fn):
        best = None
        for _ in range(args.reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        return best

    with torch.no_grad():
        for im in imgs[:2]:
            model(im)
        t_eager = timed(lambda: [model(im) for im in imgs])
        with F.weight_cache():  # weight packs / GDN re-parameterisations kept across images
            t_cached = timed(lambda: [model(im) for im in imgs])
            xc, lc = model(imgs[0])
        xe0, le0 = model(imgs[0])
        same_cached = bool(torch.equal(xe0, xc)) and all(torch.equal(le0[k], lc[k]) for k in le0)
        gf = GraphForward(model, imgs[0])
        t_graph = timed(lambda: [gf(im) for im in imgs])
        xe, le = model(imgs[0])
        xg, lg = gf(imgs[0])
        same = bool(torch.equal(xe, xg)) and all(torch.equal(le[k], lg[k]) for k in le)
    ev, evg = Evaluator(model), Evaluator(model, graph=True)
    evg.run_eval(imgs[:1])
    t_ev = timed(lambda: ev.run_eval(imgs))
    t_evg = timed(lambda: evg.run_eval(imgs))
    n = args.images * args.batch
    out = {
        "metric": f"eval forward images/s ({args.height}x{args.width}, batch {args.batch})",
        "unit": "images/s",
        "eager_forward": round(n / t_eager, 2),
        "eager_forward_weight_cache": round(n / t_cached, 2),
        "graph_forward": round(n / t_graph, 2),
        "evaluator_eager": round(n / t_ev, 2),
        "evaluator_graph": round(n / t_evg, 2),
        "ms_per_image": {"eager": round(1e3 * t_eager / n, 3), "eager_weight_cache": round(1e3 * t_cached / n, 3),
                         "graph": round(1e3 * t_graph / n, 3),
                         "evaluator_eager": round(1e3 * t_ev / n, 3), "evaluator_graph": round(1e3 * t_evg / n, 3)},
        "graph_bitwise_equal_eager": same,
        "weight_cache_bitwise_equal_eager": same_cached,
        "images": n,
        "compute_dtype": cfg.MODEL.COMPUTE_DTYPE,
        "data": "synthetic uniform [0,1) images resident in HBM; random-init weights (reference init, seed 0)",
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
