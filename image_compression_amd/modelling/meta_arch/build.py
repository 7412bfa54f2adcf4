from ...registry import Registry

META_ARCH_REGISTRY = Registry("META_ARCH")


def build_model(cfg):
    """cfg.MODEL.META_ARCHITECTURE -> nn.Module (reference meta_arch/build.py:30-36).
    cfg.MODEL.COMPUTE_DTYPE ("fp32_split" default, "fp32", or "bf16": BASELINE
    config C3) is this build's addition; see set_compute_dtype.  The default is the
    arithmetic bench.py measures: fp32 accuracy (held to the fp32 bar by
    tests/test_split_gpu.py) on the bf16 MFMA."""
    model = META_ARCH_REGISTRY.get(cfg.MODEL.META_ARCHITECTURE)(cfg)
    set_compute_dtype(model, cfg.MODEL.get("COMPUTE_DTYPE", "fp32_split"))
    return model


def set_compute_dtype(model, dtype):
    """Arithmetic of the wide convolutions' GEMMs.
    "fp32": the fp32 MFMA (an exact fp32 fma chain).  "fp32_split": fp32
    arithmetic on the bf16 MFMA — both operands split exactly into three bf16
    terms, six cross products accumulated in fp32, error of an fp32 fma chain
    (functional.MATH) — for the forward, input gradient and weight gradient of
    every wide conv (g_a, g_s, h_a, h_s).  "bf16": bf16 operands with fp32
    accumulation (reduced precision, BASELINE config C3) for the forward, input
    gradient and weight gradient of every wide conv (g_a, g_s, h_a, h_s; the 3-channel
    image edges too when the library is built with EDGE_BF16); where a bf16 kernel does
    not apply (weight gradients of maps narrower than 16) they fall back to
    "fp32_split".  Round 6 moved C3's hyperprior convs from "fp32_split" to bf16
    operands: their split GEMMs ran on the side stream beside g_s / g_a and took
    CU time from them (C3 5,430 -> 5,675 images/s alternating on one box,
    profiles/r09b_c3_hyper_bf16_ab.txt).  GDN and
    the entropy models compute in fp32 in every mode, except that "fp32_split"
    runs GDN (C = 192) in split arithmetic too:
    the fused forward (GDN.math_fwd = 2: 0.37 -> 0.30 ms at 128^2) and the fused
    backward's dgamma GEMM (GDN.math = 2: 4 % faster; A/B in one process,
    tools/gdn_ab.py), and "bf16" runs both of the backward's contractions and the
    forward's Gamma x^2 on bf16 operands (C = 192)."""
    from ...functional import MATH
    from ..layers.conv import Conv2d, ConvTranspose2d
    from ..layers.gdn import GDN
    if dtype not in MATH:
        raise ValueError(f"compute dtype {dtype!r}: expected one of {sorted(MATH)}")
    main = ("analysis_transform", "synthesis_transform")
    hyper = ("prior_analysis", "prior_synthesis")
    # IC_MATH_* per transform: bf16 (C3) falls back to split arithmetic (fp32-accurate,
    # faster than the fp32 MFMA) where no bf16 kernel applies, and runs the hyperprior split
    split = MATH["fp32_split"]
    flags = {"fp32": (0, 0), "fp32_split": (split, split), "bf16": (MATH["bf16"] | split, MATH["bf16"] | split)}[dtype]
    for m in model.modules():
        if isinstance(m, (Conv2d, ConvTranspose2d, GDN)):
            m.math = 0
        if isinstance(m, GDN) and dtype != "fp32":
            # the fused backward's dgamma GEMM in split arithmetic; bf16: both of its GEMMs on
            # bf16 operands (C = 192)
            m.math = split | (MATH["bf16"] if dtype == "bf16" else 0)
            # the fused forward (C = 192) in split arithmetic; bf16: its Gamma x^2 GEMM on bf16 operands
            m.math_fwd = split | (MATH["bf16"] if dtype == "bf16" else 0)
    for names, flag in ((main, flags[0]), (hyper, flags[1])):
        for name in names:
            sub = getattr(model, name, None)
            if sub is None:
                continue
            for m in sub.modules():
                if isinstance(m, (Conv2d, ConvTranspose2d)):
                    m.math = flag
    # bf16 (C3): a GDN feeding a 192-output conv / transposed conv writes its output's bf16 copy for
    # that conv's forward, and one behind a 192-input conv / transposed conv its input gradient's for
    # that conv's input gradient, both on the bf16 DMA tiles (csrc/igemm.hip ig_kernel_b16d: Cout 192,
    # Cin % 64 == 0; a copy the plan does not use is ignored)
    for m in model.modules():
        if isinstance(m, GDN):
            m.xb = 0
    if dtype == "bf16":
        for name in main:
            seq = getattr(getattr(model, name, None), "layers", None)
            if seq is None:
                continue
            mods = list(seq)
            for i, m in enumerate(mods):
                if not isinstance(m, GDN):
                    continue
                nxt = mods[i + 1] if i + 1 < len(mods) else None
                prv = mods[i - 1] if i > 0 else None
                # the next conv's forward / the previous conv's input gradient: out 192, in % 64 == 0
                if isinstance(nxt, Conv2d) and nxt.out_channels == 192 and nxt.in_channels % 64 == 0:
                    m.xb |= 1
                if isinstance(nxt, ConvTranspose2d) and nxt.out_channels == 192 and nxt.in_channels % 64 == 0:
                    m.xb |= 1
                if isinstance(prv, ConvTranspose2d) and prv.in_channels == 192 and prv.out_channels % 64 == 0:
                    m.xb |= 2
                if isinstance(prv, Conv2d) and prv.in_channels == 192 and prv.out_channels % 64 == 0:
                    m.xb |= 2
    return model
