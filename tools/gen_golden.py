#!/usr/bin/env python3
"""Generate golden parity fixtures from the upstream reference.

Runs ONLY in the build container (needs /root/reference); the fixtures it
writes under tests/golden/ are plain data (inputs, injected noise, parameters,
intermediates, losses, gradients) and are what the GPU box sees.

How the reference is driven (no reference file is modified or copied):
  * `torch.manual_seed(seed)` then `modelling.build_model(cfg)` — the
    reference's own initialisation (analysis.py:58-59, synthesis.py:58-59,
    prior_*.py, entropy_model.py:56-65, gdn.py:69-74).
  * `torch.rand_like` is patched for the duration of the forward so the two
    training-noise draws (entropy_model.py:230 for z, then :333 for y,
    call order bmshl2018.py:73,76) come from tensors this script generates
    and stores as `u_z`, `u_y` (the raw U[0,1) values).
  * forward hooks capture y, z, (z~, p_z, ce_z), sigma, (y~, p_y), and the raw
    synthesis output; `losses["total_loss"].backward()` gives every `.grad`.

Usage:  python tools/gen_golden.py [case ...]   (writes tests/golden/*.npz; all cases by default)
"""
import copy
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from _refimport import available, import_reference  # noqa: E402

OUT = os.path.join(os.path.dirname(HERE), "tests", "golden")


def _cfg(get_cfg_defaults, over):
    cfg = get_cfg_defaults()
    cfg.MODEL.LOSS.REDUCTION = "mean"
    for key, val in over.items():
        node = cfg
        parts = key.split(".")
        for p in parts[:-1]:
            node = node[p]
        # a copy: CDFEstimator inserts the 1-wide ends into cfg DIMS in place
        # (entropy_model.py:92-93), which must not leak into the recorded `over`
        node[parts[-1]] = copy.deepcopy(val)
    return cfg


def run_case(modelling, get_cfg_defaults, name, over, N, H, W, train, seed,
             full_params=True):
    cfg = _cfg(get_cfg_defaults, over)
    torch.manual_seed(seed)
    model = modelling.build_model(cfg)
    model.train(train)
    g = torch.Generator().manual_seed(seed + 1000)
    x = torch.rand(N, 3, H, W, generator=g)

    caps = {}

    def hook(key):
        def f(mod, inp, out):
            caps[key] = out
        return f

    model.analysis_transform.register_forward_hook(hook("y"))
    model.prior_analysis.register_forward_hook(hook("z"))
    model.entropy_model.register_forward_hook(hook("em"))
    model.prior_synthesis.register_forward_hook(hook("sigma"))
    model.conditional_model.register_forward_hook(hook("cm"))
    model.synthesis_transform.register_forward_hook(hook("x_tilde_raw"))

    draws = []
    orig_rand_like = torch.rand_like

    def fake_rand_like(t, *a, **k):
        u = torch.rand(t.shape, generator=g, dtype=t.dtype)
        draws.append(u.clone())
        return u

    torch.rand_like = fake_rand_like
    try:
        x_tilde, losses = model(x)
    finally:
        torch.rand_like = orig_rand_like
    losses["total_loss"].backward()

    d = {}
    meta = dict(name=name, over=over, N=N, H=H, W=W, train=train, seed=seed,
                torch=torch.__version__, full_params=full_params,
                loss_names=list(model.loss_names))
    d["meta"] = np.array(json.dumps(meta))
    d["x"] = x.numpy()
    if train:
        assert len(draws) == 2, len(draws)
        d["u_z"] = draws[0].numpy()
        d["u_y"] = draws[1].numpy()
    em = caps["em"]
    cm = caps["cm"]
    inter = {
        "y": caps["y"], "z": caps["z"], "z_tilde": em[0], "p_z": em[1],
        "ce_z": em[2], "sigma": caps["sigma"], "y_tilde": cm[0], "p_y": cm[1],
        "x_tilde_raw": caps["x_tilde_raw"], "x_tilde": x_tilde,
    }
    for k, v in inter.items():
        d["out/" + k] = v.detach().numpy()
    for k, v in losses.items():
        d["loss/" + k] = v.detach().numpy()
    for k, p in model.named_parameters():
        pv = p.detach().numpy()
        gv = p.grad.detach().numpy()
        if full_params:
            d["param/" + k] = pv
            d["grad/" + k] = gv
        else:
            # full-width case: parameters are re-created on the box from the
            # same seed and checked by checksum; gradients by norm + samples.
            d["psum/" + k] = np.array([pv.astype(np.float64).sum(),
                                       (pv.astype(np.float64) ** 2).sum()])
            flat = gv.reshape(-1)
            rs = np.random.RandomState(7)
            idx = np.unique(np.concatenate([
                np.arange(min(64, flat.size)),
                rs.randint(0, flat.size, size=min(256, flat.size))]))
            d["gidx/" + k] = idx.astype(np.int64)
            d["gval/" + k] = flat[idx]
            d["gnorm/" + k] = np.array(np.linalg.norm(flat.astype(np.float64)))
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **d)
    print("wrote", path, os.path.getsize(path), "bytes")


SMALL = {"MODEL.INTER_CHANNELS": 16, "MODEL.LATENT_CHANNELS": 16,
         "MODEL.LOSS.DISTORTION_LOSS_WEIGHT": 256.0}


def main():
    if not available():
        print("reference not present; nothing to do")
        return 0
    modelling, get_cfg_defaults = import_reference()
    os.makedirs(OUT, exist_ok=True)
    cases = [
        ("small_laplace_mse_train", dict(SMALL), 2, 64, 64, True, 0),
        ("small_laplace_mse_eval", dict(SMALL), 2, 64, 64, False, 1),
        ("small_gauss_mse_train",
         dict(SMALL, **{"MODEL.ENTROPY_MODEL.CONDITIONAL_MODEL":
                        "GaussianConditionalModel"}), 2, 64, 64, True, 2),
        ("small_gauss_mse_eval",
         dict(SMALL, **{"MODEL.ENTROPY_MODEL.CONDITIONAL_MODEL":
                        "GaussianConditionalModel"}), 2, 64, 64, False, 3),
        # MS-SSIM (5 levels of an 11x11 valid filter) needs >= 176 px.
        ("small_laplace_msssim_train",
         dict(SMALL, **{"MODEL.LOSS.DISTORTION_LOSS_NAMES": ["MS_SSIMLoss"],
                        "MODEL.LOSS.SSIM.LOG_SCALE": True,
                        "MODEL.LOSS.DISTORTION_LOSS_WEIGHT": 64.0}),
         1, 192, 192, True, 4),
        # non-square, non-power-of-two spatial size (H,W % 64 == 0)
        ("small_laplace_mse_rect_train", dict(SMALL), 1, 64, 128, True, 5),
        # entropy-model generality: other CDF MLP widths (DIMS) and quantization bins (BIN)
        ("small_dims242_bin2_laplace_train",
         dict(SMALL, **{"MODEL.ENTROPY_MODEL.DIMS": [2, 4, 2], "MODEL.ENTROPY_MODEL.BIN": 2.0}),
         2, 64, 64, True, 6),
        ("small_dims5_bin05_gauss_train",
         dict(SMALL, **{"MODEL.ENTROPY_MODEL.DIMS": [5], "MODEL.ENTROPY_MODEL.BIN": 0.5,
                        "MODEL.ENTROPY_MODEL.CONDITIONAL_MODEL": "GaussianConditionalModel"}),
         2, 64, 64, True, 7),
        ("small_dims8x5_bin1_laplace_eval",
         dict(SMALL, **{"MODEL.ENTROPY_MODEL.DIMS": [8, 8, 8, 8, 8]}), 2, 64, 64, False, 8),
    ]
    only = set(sys.argv[1:])
    for name, over, N, H, W, train, seed in cases:
        if only and name not in only:
            continue
        run_case(modelling, get_cfg_defaults, name, over, N, H, W, train, seed)
    if only and "full_laplace_mse_train" not in only:
        return 0
    # full-width default config (192/192, Laplacian, MSE, lambda=256)
    run_case(modelling, get_cfg_defaults, "full_laplace_mse_train",
             {"MODEL.LOSS.DISTORTION_LOSS_WEIGHT": 256.0}, 1, 64, 64, True, 0,
             full_params=False)
    return 0


if __name__ == "__main__":
    sys.exit(main())
