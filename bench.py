#!/usr/bin/env python3
"""Throughput benchmark of the hot path: Compressor2018 forward + RD loss +
backward (+ RCCL gradient all-reduce when N > 1) on synthetic 256x256 batches.

Workload (BASELINE.json configs[1], "C2"): psnr_256 semantics — lambda=256,
MSE distortion, Laplacian conditional, 192/192 channels, fp32, batch 32 per
GPU (weak scaling: the per-GPU batch stays 32 as N grows).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N ...

Rank 0 prints ONE JSON line.  `roofline` times the dominant kernel (the
implicit-GEMM conv, measured on the analysis transform's 128->64 5x5 192->192
layer) with events on the launch stream; `cpu_baseline` times the CPU oracle
(oracle/ref_cpu.py, a restatement of the reference path) on a bounded sample
on this host.
"""
import argparse
import json
import math
import os
import sys
import time

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

FP32_PEAK_TFLOPS = 157.3          # MI355X dense fp32 (matrix = vector), MI355X_MICROARCH.md
FWD_GMAC_PER_IMG = 12.2837        # SURVEY.md 6.2 (latent 192, 256x256)
STEP_GFLOP_PER_IMG = 3 * 2 * FWD_GMAC_PER_IMG   # fwd + dgrad + wgrad = 73.70
METRIC = "256x256 images/s fwd+bwd at 1/2/4/8 GPUs; bpp & PSNR vs ref on Kodak"


# BASELINE.json configs.  C2 is the metric's workload and the
# default; the others select the same path at their own lambda / loss / width /
# precision / size (per-GPU batch for weak scaling; C4 = 64 over 4 GPUs, C5 =
# 128 over 8 GPUs).
# `math` is cfg.MODEL.COMPUTE_DTYPE: "fp32_split" = fp32 arithmetic on the bf16 MFMA (each
# fp32 operand split exactly into three bf16 terms, six cross products accumulated in fp32:
# the error of an fp32 fma chain, tests/test_split_gpu.py), "fp32" = the fp32 MFMA,
# "bf16" = bf16 operands (C3's reduced precision).
CONFIGS = {
    "C2": dict(desc="psnr_256 (lambda=256, MSE, Laplacian conditional, 192/192 ch), fp32",
               lam=256.0, loss=["MSE"], latent=192, dtype="fp32", math="fp32_split", batch=32, size=256,
               gflop=73.70),
    "C3": dict(desc="psnr_4096 (lambda=4096, MSE, latent 320), bf16 operands / fp32 accumulation",
               lam=4096.0, loss=["MSE"], latent=320, dtype="bf16", math="bf16", batch=32, size=256, gflop=76.27),
    "C4": dict(desc="ssim_64 (lambda=64, MS-SSIM log-scale loss), fp32",
               lam=64.0, loss=["MS_SSIMLoss"], latent=192, dtype="fp32", math="fp32_split", batch=16, size=256,
               gflop=74.55),
    "C5": dict(desc="psnr_8192 (lambda=8192, MSE), 512x512 crops, fp32",
               lam=8192.0, loss=["MSE"], latent=192, dtype="fp32", math="fp32_split", batch=16, size=512,
               gflop=73.70),
}
MATH_NOTE = {
    "fp32_split": "fp32 via exact 3-term bf16 operand split, 6 products on the bf16 MFMA, fp32 "
                  "accumulation (fp32 fma-chain error): wide conv fwd/dgrad/wgrad, GDN (C=192) forward and both "
                  "backward contractions, the 3-channel edges; entropy models on the fp32 MFMA / VALU",
    "fp32": "fp32 MFMA (v_mfma_f32_32x32x2_f32, exact fp32 fma chain)",
    "bf16": "bf16 operands, fp32 accumulation (g_a/g_s conv fwd/dgrad/wgrad, GDN forward and backward "
            "contractions{edges}); hyperprior{edges_split} and wgrad of maps < 16 wide in fp32_split; "
            "entropy models fp32",
}


def _math_note(math):
    """MATH_NOTE of `math`; for bf16, where the 3-channel image edges run is read from the built
    library's plan (csrc/conv_api.hip EDGE_BF16; the query launches nothing)."""
    note = MATH_NOTE[math]
    if math == "bf16":
        from image_compression_amd import _lib
        img = _lib.ICAct(256, 2, 3, 64, 64, 3 * 64 * 64, 64 * 64, 64, 1)
        x = _lib.ICAct(256, 2, 192, 32, 32, 192 * 32 * 32, 1, 32 * 192, 192)
        on = _lib.plan("conv2d_fwd", img, x, 5, 2, 2, 3)["kernel"] == "edge_conv_bf16"
        note = note.format(edges=", the 3-channel image edges" if on else "",
                           edges_split="" if on else ", the 3-channel image edges")
    return note
BF16_PEAK_TFLOPS = 2500.0         # MI355X dense bf16 MFMA spec
# configs whose dominant kernel (g_a layer 2 fwd at 32 x 128^2) bench times live: C2 (fp32_split) and
# C3 (bf16 operands; same layer shape, the latent width does not touch it)
ROOFLINE_CONFIGS = ("C2", "C3")


def _bound_spec(math):
    """Spec bound (TFLOP/s of the config's algorithmic work) of the arithmetic `math` runs on."""
    return {"fp32": FP32_PEAK_TFLOPS, "fp32_split": BF16_PEAK_TFLOPS / 6, "bf16": BF16_PEAK_TFLOPS}[math]


def _frac_measured(tflops, math):
    pm = _mfma_peak_measured()
    if not pm or math not in pm["bound_tflops"]:
        return None
    return round(tflops / pm["bound_tflops"][math], 4)


def _cfg(lam=256.0, conf=None):
    from image_compression_amd import get_cfg_defaults
    cfg = get_cfg_defaults()
    cfg.MODEL.LOSS.REDUCTION = "mean"
    cfg.MODEL.LOSS.DISTORTION_LOSS_WEIGHT = lam
    if conf is not None:
        cfg.MODEL.LOSS.DISTORTION_LOSS_WEIGHT = conf["lam"]
        cfg.MODEL.LOSS.DISTORTION_LOSS_NAMES = list(conf["loss"])
        cfg.MODEL.LOSS.SSIM.LOG_SCALE = True      # the ssim_* configs
        cfg.MODEL.LATENT_CHANNELS = conf["latent"]
        cfg.MODEL.COMPUTE_DTYPE = conf["math"]
    return cfg


def dominant_kernel_roofline(dev, reps=20, live_ms=None, live_launches=0, math="fp32"):
    """The implicit-GEMM conv kernel on g_a layer 2 (conv 5x5 s2, 192->192,
    128x128 -> 64x64, batch 32): one launch = 2 * (32*64*64) * 192 * (25*192)
    = 241.6 GFLOP of algorithmic work.  `live_ms` is its average duration
    measured by LiveLaunchTimer inside the timed steps (used when given); the
    same launch is also timed in an isolated loop and reported beside it."""
    from image_compression_amd import functional as IF
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.rand(32, 192, 128, 128, device=dev, generator=g).contiguous(memory_format=torch.channels_last)
    w = torch.randn(192, 192, 5, 5, device=dev, generator=g) * 0.02
    b = torch.zeros(192, device=dev)
    flop = 2.0 * (32 * 64 * 64) * 192 * (25 * 192)
    with torch.no_grad():
        for _ in range(3):
            IF.conv2d(x, w, b, 2, 2, math=IF.MATH[math])
        torch.cuda.synchronize()
        st = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            IF.conv2d(x, w, b, 2, 2, math=IF.MATH[math])
        e1.record(st)
        torch.cuda.synchronize()
    iso_ms = e0.elapsed_time(e1) / reps
    ms = live_ms if live_ms else iso_ms
    achieved = flop / (ms * 1e-3) / 1e12
    pm = _mfma_peak_measured()
    if math == "fp32_split":
        # every fp32 MAC costs six bf16 MACs: the bound is the bf16 MFMA peak / 6
        peak, kern = BF16_PEAK_TFLOPS / 6, ("ig_kernel_x3d (256x192 tiles, operands by LDS-DMA; fp32 by 3-term bf16 "
                                           "split, 16x16x32 bf16 MFMA)")
    elif math == "bf16":
        peak, kern = BF16_PEAK_TFLOPS, ("ig_kernel_b16d (256x192 tiles, bf16 operands by LDS-DMA from an NHWC bf16 "
                                        "copy of the input, fp32 accumulation, 16x16x32 bf16 MFMA)")
    else:
        peak, kern = FP32_PEAK_TFLOPS, "ig_kernel<128,192,64,96> (fp32 MFMA)"
    return {"bound": "mfma", "achieved": round(achieved, 2), "peak": round(peak, 2), "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4), "traffic": _pmc_traffic(kern.split(" ")[0]),
            "peak_note": {"fp32_split": "algorithmic fp32 FLOP/s; peak = bf16 dense MFMA 2500 TF / 6 products per fp32 MAC",
                          "bf16": "algorithmic FLOP/s; peak = bf16 dense MFMA spec (2500 TF)"}.get(math, "fp32 dense MFMA spec"),
            "frac_of_fp32_mfma_peak": round(achieved / FP32_PEAK_TFLOPS, 4),
            "kernel": kern + (" + weight pack (live: the input's bf16 copy comes from the GDN before it; the isolated "
                              "loop converts x itself)" if math == "bf16" else " + weight pack") +
                      ": conv2d 5x5 s2 192->192 @ 32x128x128 (g_a layer 2 fwd)",
            "flop_per_launch": flop, "ms_per_launch": round(ms, 4),
            "timing": (f"live: HIP events on the launch stream around the layer's {live_launches} launches "
                       "inside the timed steps" if live_ms else "isolated loop of the same launch"),
            "isolated_ms_per_launch": round(iso_ms, 4),
            "peak_measured": pm,
            "frac_of_measured_peak": (round(achieved / pm["bound_tflops"][math], 4)
                                      if pm and math in pm["bound_tflops"] else None)}


class LiveLaunchTimer:
    """HIP events around one module's forward on the stream it launches on,
    recorded inside bench's timed steps (the roofline's kernel measured live,
    not in a separate loop).  The module's forward is the dominant kernel plus
    its weight pack."""

    def __init__(self, module):
        self.on = False
        self.pairs = []
        self._e0 = None
        module.register_forward_pre_hook(self._pre)
        module.register_forward_hook(self._post)

    def _event(self):
        e = torch.cuda.Event(enable_timing=True)
        e.record(torch.cuda.current_stream())
        return e

    def _pre(self, mod, inp):
        if self.on:
            self._e0 = self._event()

    def _post(self, mod, inp, out):
        if self.on and self._e0 is not None:
            self.pairs.append((self._e0, self._event()))
            self._e0 = None

    def ms(self):
        """Average launch duration (call after synchronize), or None."""
        if not self.pairs:
            return None
        return sum(a.elapsed_time(b) for a, b in self.pairs) / len(self.pairs)


def optimizer_step_ms(model, dev, reps=20):
    """The training step's optimizer (reference: AdamW + clip_grad_value_,
    solver/optim.py, engine/trainer.py:189-191), timed on its own and reported
    beside the fwd+bwd metric: one native multi-tensor kernel
    over the model's 10.1 M parameters."""
    from image_compression_amd.solver import make_optimizer
    cfg = _cfg()
    cfg.SOLVER.OPT_NAME = "adamw"
    cfg.SOLVER.BASE_LR = 1e-4
    cfg.SOLVER.GRAD_CLIP = 5.0
    m = getattr(model, "module", model)
    for p in m.parameters():
        if p.grad is None:
            p.grad = torch.zeros_like(p)
    opt = make_optimizer(cfg, m)
    opt.step()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        opt.step()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) / reps, 4)


def _pmc_traffic(kernel):
    """HBM bytes per launch of the dominant kernel from the committed rocprofv3
    PMC passes (tools/gpu_pmc.sh -> tools/pmc_summary.py -> profiles/*_pmc_dominant.json):
    FETCH_SIZE x2 (gfx950 correction) + WRITE_SIZE.  The algorithmic bytes of
    the launch are 0.51 GB (input 403 MB, weights 3.7 MB, output 101 MB)."""
    import glob
    for f in sorted(glob.glob(os.path.join(HERE, "profiles", "*_pmc_dominant.json")), reverse=True):
        with open(f) as fh:
            rec = json.load(fh)
        if rec["kernel"].split("<")[0] == kernel.split("<")[0]:
            return round(rec["traffic_bytes_per_launch"])
    return None


def _mfma_peak_measured():
    """Sustained MFMA rates measured on an MI355X by tools/mfma_peak.hip (committed as
    profiles/*_mfma_peak.json; SURVEY.md 8d: report the spec peak and the measured one):
    v_mfma_f32_32x32x2_f32 and, on RANDOM operands (the chip holds a lower clock on random
    bf16 data than the spec assumes), v_mfma_f32_16x16x32_bf16 -- the instruction the
    fp32_split kernels run six of per fp32 MAC, so the measured split bound is its rate / 6."""
    import glob
    files = sorted(glob.glob(os.path.join(HERE, "profiles", "*_mfma_peak.json")))
    if not files:
        return None
    with open(files[-1]) as fh:
        rows = [json.loads(line) for line in fh if line.strip()]
    fp32 = max((r["tflops"] for r in rows if "f32_32x32x2" in r.get("instr", "v_mfma_f32_32x32x2_f32")), default=None)
    bf16 = max((r["tflops"] for r in rows if "16x16x32_bf16" in r.get("instr", "")), default=None)
    out = {"file": os.path.relpath(files[-1], HERE), "fp32_mfma_tflops": fp32,
           "bf16_16x16x32_random_tflops": bf16, "bound_tflops": {}}
    if fp32:
        out["bound_tflops"]["fp32"] = fp32
    if bf16:
        out["bound_tflops"]["fp32_split"] = round(bf16 / 6, 2)
        out["bound_tflops"]["bf16"] = bf16
    return out


def cpu_baseline(seconds_target=12.0):
    """The CPU oracle (torch CPU restatement of the reference path) on a
    bounded sample: batch 8, 256x256, fwd + RD loss + bwd."""
    from image_compression_amd import modelling
    from oracle import ref_cpu
    threads = torch.get_num_threads()
    torch.manual_seed(0)
    params = {k: v.clone() for k, v in modelling.build_model(_cfg()).state_dict().items()}
    g = torch.Generator().manual_seed(0)
    N = 8
    x = torch.rand(N, 3, 256, 256, generator=g)
    uz = torch.rand(N, 192, 4, 4, generator=g)
    uy = torch.rand(N, 192, 16, 16, generator=g)
    ref_cpu.run(params, x, uz, uy, train=True, dtype=torch.float32, lam=256.0)  # warm-up
    t0 = time.perf_counter()
    iters = 0
    while True:
        ref_cpu.run(params, x, uz, uy, train=True, dtype=torch.float32, lam=256.0)
        iters += 1
        if time.perf_counter() - t0 >= seconds_target or iters >= 10:
            break
    dt = time.perf_counter() - t0
    return {"value": round(N * iters / dt, 3), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"{iters} iteration(s) of batch {N} at 256x256 fp32 fwd+loss+bwd "
                      f"(oracle/ref_cpu.py, torch CPU, {threads} threads)"}


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_plan(gpus, env, visible, argv, port=None):
    """What `bench.py --gpus N` does before anything touches the GPU.

    Returns ("run", None) when this process is the (only) rank to run: N == 1 outside a
    torch.distributed.run launch, or a launched rank whose WORLD_SIZE equals N.  Returns
    ("launch", cmd) when N > 1 and WORLD_SIZE is unset: the parent starts cmd -- N ranks
    under torch.distributed.run on 127.0.0.1 -- as a child process (never an exec), relays
    rank 0's JSON line and exits with the children's return code.  The reference reaches
    every visible GPU from one command (engine/trainer.py:256-258, nn.DataParallel); this
    is that entry point with one process per GPU.  Raises SystemExit (non-zero) when the
    world cannot be the one asked for: WORLD_SIZE != N, N < 1, or N above the visible
    devices under RCCL (gloo over GPU tensors, IMGCOMP_DIST_BACKEND=gloo, may share one GPU
    between ranks -- a rehearsal, never a measurement of N GPUs).  `visible` is
    torch.cuda.device_count(), which does not initialise the GPU on this image."""
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus {gpus} < 1")
    backend = env.get("IMGCOMP_DIST_BACKEND", "nccl")
    if gpus > 1 and backend == "nccl" and gpus > visible:
        raise SystemExit(f"bench.py: --gpus {gpus} but {visible} visible GPU(s): RCCL needs one GPU per rank "
                         "(no silent smaller run)")
    world = env.get("WORLD_SIZE")
    if world is not None:
        if int(world) != gpus:
            raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world}")
        return "run", None
    if gpus == 1:
        return "run", None
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr=127.0.0.1", f"--master-port={port or _free_port()}", os.path.abspath(__file__)]
    return "launch", cmd + list(argv)


def _launch_children(cmd):
    """Run the N-rank launch as a child process; rank 0's JSON line passes through on stdout."""
    import subprocess
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "8")
    proc = subprocess.run(cmd, env=env)
    return proc.returncode


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="C2", choices=sorted(CONFIGS),
                    help="BASELINE.json workload (C2 = the metric's; default)")
    ap.add_argument("--batch", type=int, default=None, help="images per GPU (default: the config's)")
    ap.add_argument("--size", type=int, default=None)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--profile-step-only", action="store_true",
                    help="only warmup+timed steps (for rocprofv3 runs)")
    ap.add_argument("--graph", action="store_true",
                    help="one GPU only: replay the step from a hipGraph (TrainStep) instead of eager "
                         "launches.  Slower than eager (about 20 us of runtime cost per graph node, "
                         "DESIGN.md 10b); the multi-GPU path is eager DDP with 12 MB buckets overlapped "
                         "with the backward, never a graph replay followed by an unbucketed all-reduce.")
    ap.add_argument("--math", default=None, choices=["fp32", "fp32_split", "bf16"],
                    help="override the config's cfg.MODEL.COMPUTE_DTYPE")
    ap.add_argument("--serial-hyperprior", action="store_true",
                    help="run the hyperprior branch on the main stream (Compressor2018.concurrent_hyperprior "
                         "= False; bitwise the same arithmetic)")
    args = ap.parse_args()
    what, cmd = launch_plan(args.gpus, os.environ, torch.cuda.device_count(), sys.argv[1:])
    if what == "launch":
        sys.exit(_launch_children(cmd))
    conf = dict(CONFIGS[args.config])
    if args.math:
        conf["math"] = args.math
    args.batch = args.batch or conf["batch"]
    args.size = args.size or conf["size"]

    from image_compression_amd import distributed as D
    from image_compression_amd import modelling
    rank, world, dev = D.setup()
    dist = world > 1
    if args.graph and dist:
        raise SystemExit("bench.py --graph is single-GPU only (see --help)")
    from image_compression_amd.step import TrainStep
    torch.manual_seed(0)
    model = modelling.build_model(_cfg(conf=conf)).to(dev).train()
    if args.serial_hyperprior:
        model.concurrent_hyperprior = False
    # each rank draws its own shard of the synthetic global batch (weak scaling)
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    x = torch.rand(args.batch, 3, args.size, args.size, device=dev, generator=g)
    if not args.graph:
        model = D.wrap(model, dev)

        def step():
            model.zero_grad(set_to_none=True)
            _, losses = model(x)
            losses["total_loss"].backward()
            return losses
        mode = ("eager, DDP 12 MB buckets" if dist else "eager") + (
            ", hyperprior on the main stream" if args.serial_hyperprior else ", hyperprior on a side stream")
    else:
        # fwd + loss + bwd captured once into a hipGraph and replayed (one GPU)
        step = TrainStep(model, x, graph=True)
        mode = "hipGraph"

    live = None
    if not args.graph and args.config in ROOFLINE_CONFIGS and not args.no_roofline:
        core = getattr(model, "module", model)
        live = LiveLaunchTimer(core.analysis_transform.layers[2])
    for _ in range(args.warmup):
        losses = step()
    torch.cuda.synchronize()
    D.barrier(dev)
    torch.cuda.synchronize()
    if live is not None:
        live.on = True
    t0 = time.perf_counter()
    for _ in range(args.steps):
        losses = step()
    torch.cuda.synchronize()
    if live is not None:
        live.on = False
    D.barrier(dev)
    elapsed = D.max_over_ranks(time.perf_counter() - t0, dev)
    dname = conf["loss"][0]
    avg = D.mean_over_ranks({"bpp": losses["bpp"], dname: losses[dname]}, dev)
    bpp, dist_val = avg["bpp"], avg[dname]
    if args.profile_step_only:
        if rank == 0:
            print(json.dumps({"ms_per_step": 1e3 * elapsed / args.steps}))
        D.teardown()
        return

    opt_ms = optimizer_step_ms(step.model if hasattr(step, "model") else model, dev)
    images = args.batch * world * args.steps
    value = images / elapsed
    ms = 1e3 * elapsed / args.steps
    roof = None
    if not args.no_roofline and args.config in ROOFLINE_CONFIGS:
        roof = dominant_kernel_roofline(dev, live_ms=live.ms() if live else None,
                                        live_launches=len(live.pairs) if live else 0, math=conf["math"])
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config == "C2":
        cpu = cpu_baseline()
    if rank == 0:
        # model FLOPs per image (3 x forward MACs x 2), x4 per 512^2 image
        step_tflops = value / world * conf["gflop"] * (args.size / 256) ** 2 / 1e3
        rec = {
            "metric": METRIC, "value": round(value, 2), "unit": "images/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": conf["dtype"],
            "data": "synthetic: torch.rand uniform [0,1) images resident in HBM; random-init weights "
                    "(reference init, seed 0); training noise from in-kernel Philox",
            "config": {"workload": f"{args.config}: {conf['desc']}, "
                                   f"{args.size}x{args.size}, {args.batch} images/GPU, fwd+loss+bwd"
                                   + (" + grad all-reduce" if dist else "") + f" [{mode}]",
                       "math": f"{conf['math']}: {_math_note(conf['math'])}",
                       "global_batch": args.batch * world, "image_size": args.size,
                       "parallelism": f"dp{world}"},
            "model_tflops_per_gpu": round(step_tflops, 2),
            # the whole step's algorithmic fp32 FLOP/s over the bound of the arithmetic it runs on:
            # fp32_split -> bf16 MFMA spec / 6 (and the measured random-operand rate / 6); fp32 -> fp32 MFMA
            "model_frac_of_bound": round(step_tflops / _bound_spec(conf["math"]), 4),
            "model_frac_of_measured_bound": _frac_measured(step_tflops, conf["math"]),
            "bpp": round(bpp, 4), dname.lower(): dist_val,
            "optimizer_step_ms": opt_ms,
            "images_256_equiv_per_s": round(value * (args.size / 256) ** 2, 2),
            "roofline": roof, "cpu_baseline": cpu,
        }
        print(json.dumps(rec))
    D.teardown()


if __name__ == "__main__":
    main()
