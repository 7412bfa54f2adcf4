from ...registry import Registry

META_ARCH_REGISTRY = Registry("META_ARCH")


def build_model(cfg):
    """cfg.MODEL.META_ARCHITECTURE -> nn.Module (reference meta_arch/build.py:30-36).
    cfg.MODEL.COMPUTE_DTYPE ("fp32" default, or "bf16": BASELINE config C3) is
    this build's addition; see set_compute_dtype."""
    model = META_ARCH_REGISTRY.get(cfg.MODEL.META_ARCHITECTURE)(cfg)
    set_compute_dtype(model, cfg.MODEL.get("COMPUTE_DTYPE", "fp32"))
    return model


def set_compute_dtype(model, dtype):
    """Operand precision of the main transforms' (g_a, g_s) wide convolution
    forward / input-gradient GEMMs: "fp32" (exact fp32 MFMA) or "bf16" (bf16
    operands, fp32 accumulation) — 97 % of the model's FLOPs.  The
    hyperprior transforms (h_a, h_s: 1.3 % of the FLOPs, but they shape the
    rate term's gradients), weight gradients, GDN, the entropy models and the
    3-channel image edges always compute in fp32."""
    from ...functional import MATH
    from ..layers.conv import Conv2d, ConvTranspose2d
    if dtype not in MATH:
        raise ValueError(f"compute dtype {dtype!r}: expected one of {sorted(MATH)}")
    for name in ("analysis_transform", "synthesis_transform"):
        sub = getattr(model, name, None)
        if sub is None:
            continue
        for m in sub.modules():
            if isinstance(m, (Conv2d, ConvTranspose2d)):
                m.math = MATH[dtype]
    return model
