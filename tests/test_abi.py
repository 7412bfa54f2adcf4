"""CPU-side checks of the drop-in boundary: the C-ABI library loads, exports
every symbol include/imgcomp.h declares, and the Python mirror of the
reference API builds with the reference's parameter names/shapes/init."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

from conftest import ROOT


def _header_symbols():
    txt = open(os.path.join(ROOT, "include", "imgcomp.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return set(re.findall(r"\b(ic_[a-z0-9_]+)\s*\(", txt))


def test_library_exports_every_header_symbol():
    from image_compression_amd import _lib
    declared = _header_symbols()
    assert len(declared) >= 40
    lib = _lib.load()
    missing = [s for s in sorted(declared) if not hasattr(lib, s)]
    assert not missing, missing
    # every declared symbol has a ctypes signature and vice versa
    assert declared == set(_lib.SIGNATURES), declared ^ set(_lib.SIGNATURES)
    assert lib.ic_version() >= 3  # the ctypes structs in _lib.py mirror the version-3 layout


def test_workspace_queries_without_gpu():
    from image_compression_amd import _lib
    L = _lib.load()
    x = torch.empty(0)
    a = _lib.ICAct(None, 32, 192, 128, 128, 192 * 128 * 128, 1, 128 * 192, 192)
    y = _lib.ICAct(None, 32, 192, 64, 64, 192 * 64 * 64, 1, 64 * 192, 192)
    assert L.ic_conv2d_fwd_ws(a, 5, 2, 2, y) > 0
    assert L.ic_conv2d_wgrad_ws(a, y, 5, 2, 2) > 0
    assert L.ic_conv2d_dgrad_ws(y, 5, 2, 2, a) > 0
    assert L.ic_gdn_bwd_ws(a) > 0
    # inconsistent geometry is rejected (0 bytes)
    bad = _lib.ICAct(None, 32, 192, 63, 64, 192 * 63 * 64, 1, 64 * 192, 192)
    assert L.ic_conv2d_fwd_ws(a, 5, 2, 2, bad) == 0
    assert L.ic_msssim_state_bytes(2, 3, 64, 64, 5, 11) == 0  # too small for 5 levels
    assert L.ic_msssim_state_bytes(2, 3, 192, 192, 5, 11) > 0
    # the fused MS-SSIM forward writes one (cs, ssim) partial per 64 x 16 tile of valid outputs and plane:
    # a Kodak-sized image (758 x 502 valid outputs at level 0 = 12 x 32 tiles) needs more than the
    # round-4 fixed 64 partials per plane
    assert L.ic_msssim_ws(1, 3, 512, 768, 5, 11) >= 3 * 12 * 32 * 2 * 4
    # the fused backward needs no moment / derivative planes: C4's workspace is the per-level gradients
    n0 = 16 * 3 * 256 * 256
    grads = sum(2 * n0 // 4 ** l for l in range(5)) * 4
    assert grads <= L.ic_msssim_ws(16, 3, 256, 256, 5, 11) < grads + 4 * 1024 * 1024


def test_cpu_tensors_fail_loudly():
    from image_compression_amd import functional as IF
    with pytest.raises(RuntimeError, match="ROCm"):
        IF.conv2d(torch.rand(1, 3, 8, 8), torch.rand(4, 3, 3, 3), None, 1, 1)


def test_state_dict_and_init_match_reference_names():
    from image_compression_amd import get_cfg_defaults, modelling
    from conftest import load_golden
    cfg = get_cfg_defaults()
    cfg.MODEL.LOSS.REDUCTION = "mean"
    meta, d = load_golden("full_laplace_mse_train")
    torch.manual_seed(meta["seed"])
    model = modelling.build_model(cfg)
    keys = {k[len("psum/"):] for k in d.files if k.startswith("psum/")}
    assert set(model.state_dict().keys()) == keys
    for k, v in model.state_dict().items():
        s, s2 = d["psum/" + k]
        pv = v.double()
        assert abs(float(pv.sum()) - s) <= 1e-6 * max(1.0, abs(s)), k
        assert abs(float((pv ** 2).sum()) - s2) <= 1e-6 * max(1.0, s2), k
    assert model.loss_names == ["y_entropy", "z_entropy", "bpp", "MSE"]


@pytest.mark.parametrize("name", [n for n in __import__("conftest").golden_names("small_")])
def test_small_configs_build_the_reference_state_dict(name):
    """Every golden config -- including other CDF MLP widths (DIMS) and bins (BIN) -- builds
    the reference's parameter names and shapes, and the same initial values from the same
    seed (tools/gen_golden.py: torch.manual_seed(seed) then build_model)."""
    import copy
    from image_compression_amd import get_cfg_defaults, modelling
    from conftest import load_golden, params_of
    meta, d = load_golden(name)
    cfg = get_cfg_defaults()
    cfg.MODEL.LOSS.REDUCTION = "mean"
    for key, val in meta["over"].items():
        node = cfg
        parts = key.split(".")
        for q in parts[:-1]:
            node = node[q]
        node[parts[-1]] = copy.deepcopy(val)
    torch.manual_seed(meta["seed"])
    model = modelling.build_model(cfg)
    ref = params_of(d)
    sd = model.state_dict()
    assert set(sd) == set(ref), sorted(set(sd) ^ set(ref))
    # the golden params are the reference's values after its backward (unchanged: no step),
    # so they are its initial values
    for k, v in sd.items():
        assert tuple(v.shape) == ref[k].shape, k
        assert np.array_equal(v.numpy(), ref[k]), k


def test_registries_and_errors():
    from image_compression_amd.modelling.blocks import ENTROPY_MODEL_REGISTRY
    from image_compression_amd.modelling.meta_arch import META_ARCH_REGISTRY
    assert "Compressor2018" in META_ARCH_REGISTRY
    for n in ["EntropyModel", "GaussianConditionalModel", "LaplacianConditionalModel"]:
        assert n in ENTROPY_MODEL_REGISTRY
    with pytest.raises(KeyError):
        META_ARCH_REGISTRY.get("Nope")
    with pytest.raises(AssertionError):
        META_ARCH_REGISTRY.register(META_ARCH_REGISTRY.get("Compressor2018"))


def test_yaml_configs_merge(tmp_path):
    from image_compression_amd import get_cfg_defaults
    p = tmp_path / "c.yaml"
    p.write_text("MODEL:\n  LOSS:\n    DISTORTION_LOSS_NAMES: [\"MS_SSIMLoss\"]\n    SSIM:\n      LOG_SCALE: True\n"
                 "    DISTORTION_LOSS_WEIGHT: 64.\n    REDUCTION: \"mean\"\n")
    cfg = get_cfg_defaults()
    cfg.merge_from_file(str(p))
    assert cfg.MODEL.LOSS.DISTORTION_LOSS_NAMES == ["MS_SSIMLoss"]
    assert cfg.MODEL.LOSS.SSIM.LOG_SCALE is True
    assert cfg.MODEL.LOSS.DISTORTION_LOSS_WEIGHT == 64.0


def test_modelling_alias_imports_reference_style():
    """`import modelling` (the reference's package name, engine/trainer.py:248-261) yields
    the same module objects as image_compression_amd.modelling."""
    import modelling
    from modelling import build_model
    from modelling.layers import GDN
    from modelling.meta_arch import META_ARCH_REGISTRY
    import image_compression_amd.modelling as real
    assert modelling is real
    assert build_model is real.build_model and GDN is real.layers.GDN
    assert META_ARCH_REGISTRY is real.meta_arch.META_ARCH_REGISTRY


def _act(n, c, h, w, cl=True, data=256):
    from image_compression_amd import _lib
    if cl:
        return _lib.ICAct(data, n, c, h, w, c * h * w, 1, w * c, c)
    return _lib.ICAct(data, n, c, h, w, c * h * w, h * w, w, 1)


def test_plan_query_c2_instances():
    """ic_conv_plan (no launch): the kernel instances the C2 benchmark batch takes."""
    from image_compression_amd import _lib
    x, y = _act(32, 192, 128, 128), _act(32, 192, 64, 64)
    p = _lib.plan("conv2d_fwd", x, y, 5, 2, 2, 2)
    assert (p["kernel"], p["bm"], p["bn"], p["ksplit"]) == ("ig_split_dma", 256, 192, 1)
    assert p["blocks"] == 32 * 64 * 64 // 256
    p = _lib.plan("conv2d_dgrad", y, x, 5, 2, 2, 2)
    assert (p["kernel"], p["bm"], p["ksplit"]) == ("ig_split_dma", 256, 1)
    # 32 k output pixels: 128 tiles of 256 rows, K split in 2 to fill the chip
    p = _lib.plan("conv2d_fwd", _act(8, 192, 128, 128), _act(8, 192, 64, 64), 5, 2, 2, 2)
    assert (p["kernel"], p["bm"], p["ksplit"]) == ("ig_split_dma", 256, 2)
    # ... but a transposed conv's four unequal phases stay on 64-row tiles
    p = _lib.plan("conv_transpose2d_fwd", _act(32, 192, 16, 16), _act(32, 192, 32, 32), 5, 2, 2, 2)
    assert (p["kernel"], p["bm"]) == ("ig_split", 64)
    p = _lib.plan("conv2d_wgrad", x, y, 5, 2, 2, 2)
    assert (p["kernel"], p["variant"]) == ("wg_split", 1) and p["nsplit"] >= 1
    p = _lib.plan("conv2d_fwd", x, y, 5, 2, 2, 0)
    assert p["kernel"] == "ig_fp32"
    p = _lib.plan("conv2d_fwd", x, y, 5, 2, 2, 1)
    assert (p["kernel"], p["bm"], p["ksplit"]) == ("ig_bf16_dma", 256, 1)
    # bf16 operands: a transposed conv's four phases on the DMA tiles too (each >= 256 tiles) ...
    p = _lib.plan("conv2d_dgrad", y, x, 5, 2, 2, 1)
    assert (p["kernel"], p["bm"], p["ksplit"]) == ("ig_bf16_dma", 256, 1)
    # ... but not below 256 tiles (no K split across unequal phases)
    p = _lib.plan("conv_transpose2d_fwd", _act(8, 192, 32, 32), _act(8, 192, 64, 64), 5, 2, 2, 1)
    assert (p["kernel"], p["bm"]) == ("ig_split_bf16", 64)
    p = _lib.plan("conv_transpose2d_dgrad", x, y, 5, 2, 2, 1)
    assert (p["kernel"], p["bm"]) == ("ig_bf16_dma", 256)
    # small maps: 64-row tiles with split-K
    p = _lib.plan("conv2d_fwd", _act(32, 192, 16, 16), _act(32, 192, 8, 8), 5, 2, 2, 2)
    assert (p["kernel"], p["bm"]) == ("ig_split", 64) and p["ksplit"] > 1
    p = _lib.plan("conv2d_fwd", _act(32, 192, 32, 32), _act(32, 192, 16, 16), 5, 2, 2, 2)
    assert (p["kernel"], p["bm"]) == ("ig_split_dma", 256) and p["ksplit"] == 8
    # image edges and GDN
    img = _act(32, 3, 256, 256, cl=False)
    assert _lib.plan("conv2d_fwd", img, x, 5, 2, 2, 2)["kernel"] == "edge_conv"
    assert _lib.plan("conv_transpose2d_fwd", x, img, 5, 2, 2, 2)["kernel"] == "tconv_few_rows"
    # C3 (split | bf16): the image edges on bf16 operands when the build has them on (EDGE_BF16)
    bf = _lib.plan("conv2d_fwd", img, x, 5, 2, 2, 3)["kernel"] == "edge_conv_bf16"
    sfx = "_bf16" if bf else ""
    assert _lib.plan("conv2d_fwd", img, x, 5, 2, 2, 3)["kernel"] == "edge_conv" + sfx
    assert _lib.plan("conv_transpose2d_fwd", x, img, 5, 2, 2, 3)["kernel"] == "tconv_few_rows" + sfx
    assert _lib.plan("conv2d_wgrad", img, x, 5, 2, 2, 3)["kernel"] == "edge_wgrad" + sfx
    assert _lib.plan("conv2d_wgrad", img, x, 5, 2, 2, 2)["kernel"] == "edge_wgrad"
    assert _lib.plan("gdn_fwd", x, math=2)["kernel"] == "gdn_fused_split"
    assert _lib.plan("gdn_fwd", x, math=3)["kernel"] == "gdn_fused_bf16"   # C3: split | bf16
    assert _lib.plan("gdn_bwd", x, math=3)["kernel"] == "gdn_fused_bf16"
    assert _lib.plan("gdn_bwd", x, math=0)["kernel"] == "gdn_fused"


def test_extent_guard_rejects_32bit_overflow():
    """Tensors whose element offsets reach 2^31 are rejected (IC_ERR_ARG), not wrapped."""
    from image_compression_amd import _lib
    L = _lib.load()
    big = _act(1024, 192, 512, 512)       # 5.2e10 elements
    out = _act(1024, 192, 256, 256)
    with pytest.raises(RuntimeError, match="1001"):
        _lib.plan("conv2d_fwd", big, out, 5, 2, 2, 2)
    with pytest.raises(RuntimeError, match="1001"):
        _lib.plan("conv2d_wgrad", big, out, 5, 2, 2, 2)
    with pytest.raises(RuntimeError, match="1001"):
        _lib.plan("conv_transpose2d_fwd", out, big, 5, 2, 2, 2)
    with pytest.raises(RuntimeError, match="1001"):
        _lib.plan("gdn_fwd", big, math=2)
    assert L.ic_conv2d_fwd_ws_ex(big, 5, 2, 2, out, 2) == 0   # the workspace query reports failure as 0
    # just below the limit is accepted: 2^31 - 1 addressable elements
    ok = _act(43, 192, 512, 512)          # 2.16e9 > 2^31 -> rejected
    ok2 = _act(42, 192, 512, 512)         # 2.11e9 < 2^31
    with pytest.raises(RuntimeError):
        _lib.plan("gdn_fwd", ok, math=2)
    assert _lib.plan("gdn_fwd", ok2, math=2)["kernel"] == "gdn_fused_split"


def test_torch_ops_registered_with_shape_kernels():
    """torch.ops.imgcomp.* (TORCH_LIBRARY, csrc/torch_ops.cpp) load and infer shapes on the meta device."""
    from image_compression_amd import _lib
    ops = _lib.ops()
    x = torch.empty(2, 192, 32, 32, device="meta").contiguous(memory_format=torch.channels_last)
    w = torch.empty(192, 192, 5, 5, device="meta")
    y = ops.conv2d_fwd(x, w, None, 2, 2, 0, 2)
    assert y.shape == (2, 192, 16, 16) and y.is_contiguous(memory_format=torch.channels_last)
    assert ops.conv2d_dgrad(y, w, x, 2, 2, 2).shape == x.shape
    dw, db = ops.conv2d_wgrad(x, y, w, 2, 2, True, 2)
    assert dw.shape == w.shape and db.shape == (192,)
    assert ops.conv_transpose2d_fwd(y, w, None, 2, 2, 1, 0, 2).shape == x.shape
    yy, nn = ops.gdn_fwd(x, torch.empty(192, 192, device="meta"), torch.empty(192, device="meta"), False, 2)
    assert yy.shape == nn.shape == x.shape
    for name in ("conv2d_fwd", "conv2d_dgrad", "conv2d_wgrad", "conv_transpose2d_fwd", "conv_transpose2d_dgrad",
                 "conv_transpose2d_wgrad", "gdn_fwd", "gdn_bwd"):
        assert hasattr(ops, name), name


def _meta(*shape, cl=False, dtype=torch.float32):
    t = torch.empty(*shape, device="meta", dtype=dtype)
    return t.contiguous(memory_format=torch.channels_last) if cl else t


# every torch.ops.imgcomp op -> a call on meta tensors and the output shapes it must infer
def _meta_cases():
    x = _meta(2, 192, 16, 16, cl=True)
    img = _meta(2, 3, 64, 64)
    zl = _meta(2, 4, 4, 192)
    fact = [_meta(192 * n) for n in (3, 3, 3, 9, 3, 3, 9, 3, 3, 3, 1)]
    net = [_meta(192 * n) for n in (2, 2, 2, 8, 4, 4, 4, 1)]   # DIMS [2, 4]: 1 -> 2 -> 4 -> 1
    st = _meta(2, dtype=torch.int64)
    w = [.0448, .2856, .3001, .2363, .1333]
    s = x.shape
    return {
        "nonneg_fwd": (lambda o: o.nonneg_fwd(_meta(192, 192), 0.0, 2 ** -36), [(192, 192)]),
        "nonneg_bwd": (lambda o: o.nonneg_bwd(_meta(192), _meta(192), 0.0), [(192,)]),
        "nonneg_multi_fwd": (lambda o: tuple(o.nonneg_multi_fwd([_meta(192, 192), _meta(192)], [0.0, 1e-3],
                                                                 [2 ** -36, 2 ** -36])), [(192, 192), (192,)]),
        "nonneg_multi_bwd": (lambda o: tuple(o.nonneg_multi_bwd([_meta(192, 192), _meta(192)],
                                                                 [_meta(192, 192), _meta(192)], [0.0, 1e-3])),
                             [(192, 192), (192,)]),
        "bound_fwd": (lambda o: o.bound_fwd(img, 1.0, True), [img.shape]),
        "bound_bwd": (lambda o: o.bound_bwd(img, img, 0.0, False), [img.shape]),
        "relu_fwd": (lambda o: o.relu_fwd(x), [s]),
        "relu_bwd": (lambda o: o.relu_bwd(x, x), [s]),
        "abs_fwd": (lambda o: o.abs_fwd(x), [s]),
        "abs_bwd": (lambda o: o.abs_bwd(x, x), [s]),
        "exp_clamp_fwd": (lambda o: o.exp_clamp_fwd(x, 1e-10, 1e10), [s, s]),
        "exp_clamp_bwd": (lambda o: o.exp_clamp_bwd(x, x, 1e-10, 1e10), [s]),
        "ce_loss_fwd": (lambda o: o.ce_loss_fwd(x), [()]),
        "ce_loss_bwd": (lambda o: o.ce_loss_bwd(x, _meta(())), [s]),
        "mse_fwd": (lambda o: o.mse_fwd(img, img), [()]),
        "mse_bwd": (lambda o: o.mse_bwd(img, img, _meta(()), True, False), [img.shape, (0,)]),
        "sqdiff_fwd": (lambda o: o.sqdiff_fwd(img, img), [img.shape]),
        "sqdiff_bwd": (lambda o: o.sqdiff_bwd(img, img, img, True, True), [img.shape, img.shape]),
        "factorized_fwd": (lambda o: o.factorized_fwd(zl, 192, fact, 3, st, 0, 0), [zl.shape, zl.shape]),
        "factorized_bwd": (lambda o: (lambda r: (r[0], *r[1]))(o.factorized_bwd(zl, 192, fact, zl, zl)),
                           [zl.shape] + [t.shape for t in fact]),
        "factorized_net_fwd": (lambda o: o.factorized_net_fwd(zl, 192, [1, 2, 4, 1], 2.0, net, 1, None, 0, 0),
                               [zl.shape, zl.shape]),
        "factorized_net_bwd": (lambda o: (lambda r: (r[0], *r[1]))(o.factorized_net_bwd(zl, 192, [1, 2, 4, 1], 2.0,
                                                                                          net, None, zl)),
                               [zl.shape] + [t.shape for t in net]),
        "quantize": (lambda o: o.quantize(x, 3, st, 0, 0, 1.0), [s]),
        "conditional_fwd": (lambda o: o.conditional_fwd(x, x, None, 0, 4, None, 0, 0, 1.0), [s, s]),
        "conditional_bwd": (lambda o: o.conditional_bwd(x, x, None, 1, 1.0, x, x, True, True, True), [s, s, (0,)]),
        "philox_advance": (lambda o: (o.philox_advance(st, 100), ())[1], []),
        "msssim_fwd": (lambda o: o.msssim_fwd(_meta(2, 3, 256, 256), _meta(2, 3, 256, 256), 5, 11, 1.5, 255.0,
                                              True, 0, 0.01, 0.03, 1e-5, w), [(), None]),
        "msssim_bwd": (lambda o: o.msssim_bwd(_meta(()), _meta(1000), [2, 3, 256, 256], 5, 11, 1.5, 255.0, True, 0,
                                              0.01, 0.03, 1e-5, w, True, False), [(2, 3, 256, 256), (0,)]),
        "conv2d_fwd": (lambda o: o.conv2d_fwd(x, _meta(192, 192, 5, 5), None, 2, 2, 0, 2), [(2, 192, 8, 8)]),
        "conv2d_fwd_ws": (lambda o: o.conv2d_fwd_ws(x, _meta(192, 192, 5, 5), None, 2, 2, 0, 2,
                                                    _meta(16, dtype=torch.uint8)), [(2, 192, 8, 8)]),
        "conv_transpose2d_fwd_ws": (lambda o: o.conv_transpose2d_fwd_ws(_meta(2, 192, 8, 8, cl=True),
                                                                        _meta(192, 192, 5, 5), None, 2, 2, 1, 0, 2,
                                                                        _meta(16, dtype=torch.uint8)), [s]),
        "conv2d_dgrad": (lambda o: o.conv2d_dgrad(_meta(2, 192, 8, 8, cl=True), _meta(192, 192, 5, 5), x, 2, 2, 2),
                         [s]),
        "conv2d_wgrad": (lambda o: o.conv2d_wgrad(x, _meta(2, 192, 8, 8, cl=True), _meta(192, 192, 5, 5), 2, 2, True,
                                                  2), [(192, 192, 5, 5), (192,)]),
        "conv_transpose2d_fwd": (lambda o: o.conv_transpose2d_fwd(_meta(2, 192, 8, 8, cl=True), _meta(192, 192, 5, 5),
                                                                  None, 2, 2, 1, 0, 2), [s]),
        "conv_transpose2d_dgrad": (lambda o: o.conv_transpose2d_dgrad(x, _meta(192, 192, 5, 5),
                                                                      _meta(2, 192, 8, 8, cl=True), 2, 2, 2),
                                   [(2, 192, 8, 8)]),
        "conv_transpose2d_wgrad": (lambda o: o.conv_transpose2d_wgrad(_meta(2, 192, 8, 8, cl=True), x,
                                                                      _meta(192, 192, 5, 5), 2, 2, True, 2),
                                   [(192, 192, 5, 5), (192,)]),
        "gdn_fwd": (lambda o: o.gdn_fwd(x, _meta(192, 192), _meta(192), False, 2), [s, s]),
        "gdn_bwd": (lambda o: o.gdn_bwd(x, x, x, _meta(192, 192), False, 2), [s, (192, 192), (192,)]),
        "gdn_bwd_sum": (lambda o: o.gdn_bwd_sum(x, x, x, _meta(192, 192), False, 2),
                        [s, (192, 192), (192,), (192,)]),
        "gdn_fwd_xb": (lambda o: o.gdn_fwd_xb(x, _meta(192, 192), _meta(192), False, 3), [s, s, s]),
        "gdn_bwd_sum_xb": (lambda o: o.gdn_bwd_sum_xb(x, x, x, _meta(192, 192), False, 3),
                           [s, (192, 192), (192,), (192,), s]),
        "gdn_fwd_rn": (lambda o: o.gdn_fwd_rn(x, _meta(192, 192), _meta(192), False, 3, True), [s, s]),
        "gdn_bwd_sum_rn": (lambda o: o.gdn_bwd_sum_rn(x, _meta(192), x, _meta(192, 192), False, 3, True),
                           [s, (192, 192), (192,), (192,), s]),
        "conv2d_fwd_xb": (lambda o: o.conv2d_fwd_xb(x, _meta(*s, cl=True, dtype=torch.bfloat16), _meta(192, 192, 5, 5),
                                                    None, 2, 2, 0, 3), [(2, 192, 8, 8)]),
        "conv2d_wgrad_xb": (lambda o: o.conv2d_wgrad_xb(x, _meta(*s, cl=True, dtype=torch.bfloat16),
                                                        _meta(2, 192, 8, 8, cl=True),
                                                        _meta(2, 192, 8, 8, cl=True, dtype=torch.bfloat16),
                                                        _meta(192, 192, 5, 5), 2, 2, True, 3),
                            [(192, 192, 5, 5), (192,)]),
        "conv_transpose2d_wgrad_xb": (lambda o: o.conv_transpose2d_wgrad_xb(
            _meta(2, 192, 8, 8, cl=True), _meta(2, 192, 8, 8, cl=True, dtype=torch.bfloat16), x,
            _meta(*s, cl=True, dtype=torch.bfloat16), _meta(192, 192, 5, 5), 2, 2, True, 3),
                                      [(192, 192, 5, 5), (192,)]),
        "conv2d_dgrad_xb": (lambda o: o.conv2d_dgrad_xb(_meta(2, 192, 8, 8, cl=True),
                                                        _meta(2, 192, 8, 8, cl=True, dtype=torch.bfloat16),
                                                        _meta(192, 192, 5, 5), x, 2, 2, 3), [s]),
        "conv_transpose2d_fwd_xb": (lambda o: o.conv_transpose2d_fwd_xb(
            _meta(2, 192, 8, 8, cl=True), _meta(2, 192, 8, 8, cl=True, dtype=torch.bfloat16), _meta(192, 192, 5, 5),
            None, 2, 2, 1, 0, 3), [s]),
        "conv_transpose2d_dgrad_xb": (lambda o: o.conv_transpose2d_dgrad_xb(
            x, _meta(*s, cl=True, dtype=torch.bfloat16), _meta(192, 192, 5, 5), _meta(2, 192, 8, 8, cl=True), 2, 2, 3),
                                      [(2, 192, 8, 8)]),
    }


def test_every_registered_op_has_a_meta_kernel():
    """every launcher the training step calls is a torch.ops.imgcomp operator with a
    shape (Meta) kernel -- convolutions, GDN, elementwise bounds / ReLU / abs / exp-clamp, the
    factorized and conditional entropy models, the quantizer, the losses (CE, MSE, MS-SSIM) and
    the noise-state advance.  Each is called on meta tensors here (no GPU)."""
    from image_compression_amd import _lib
    ops = _lib.ops()
    cases = _meta_cases()
    registered = {name.split("::")[1] for name in torch._C._dispatch_get_all_op_names() if name.startswith("imgcomp::")}
    assert registered == set(cases), sorted(registered ^ set(cases))
    for name, (call, shapes) in cases.items():
        out = call(ops)
        out = out if isinstance(out, tuple) else (out,)
        assert len(out) == len(shapes), name
        for t, shp in zip(out, shapes):
            assert t.device.type == "meta", name
            if shp is not None:
                assert tuple(t.shape) == tuple(shp), (name, tuple(t.shape), shp)


def test_training_step_path_has_no_ctypes_call():
    """functional.py (the autograd Functions of the training step) dispatches every launch
    through torch.ops.imgcomp; the ctypes binding stays for the non-torch C ABI users."""
    import inspect

    from image_compression_amd import functional, noise
    for mod in (functional, noise):
        src = inspect.getsource(mod)
        assert "ctypes" not in src and "_lib.load()" not in src and "_L()" not in src, mod.__name__


def test_factorized_net_workspace_selects_the_kernels():
    """ic_factorized_net_ws (host code): 0 -- the register kernels -- up to 5 hidden layers of width <= 8,
    the wide kernels' workspace beyond, 0 past their limits (the call then returns IC_ERR_ARG)."""
    from image_compression_amd import _lib
    lib = _lib.load()

    def ws(dims, bwd):
        net = _lib.ICFactNet()
        net.nlayers = len(dims) - 1
        for i, d in enumerate(dims):
            net.dims[i] = d
        for l in range(net.nlayers):
            net.w[l] = net.b[l] = net.f[l] = 256   # never dereferenced by the query
        return lib.ic_factorized_net_ws(192 * 16, 192, ctypes.byref(net), bwd)

    for bwd in (0, 1):
        assert ws([1, 3, 3, 3, 1], bwd) == 0
        assert ws([1, 8, 8, 8, 8, 8, 1], bwd) == 0
        assert ws([1, 16, 16, 1], bwd) > 0
        assert ws([1] + [3] * 7 + [1], bwd) > 0
        assert ws([1] + [256] * 31 + [1], bwd) > 0
        assert ws([1, 257, 1], bwd) == 0                 # past IC_FACT_WIDE_MAXW
        net = _lib.ICFactNet()
        net.nlayers = _lib.FACT_NET_MAXL + 1                # past IC_FACT_NET_MAXL layers
        assert lib.ic_factorized_net_ws(192 * 16, 192, ctypes.byref(net), bwd) == 0
