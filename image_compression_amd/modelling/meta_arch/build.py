from ...registry import Registry

META_ARCH_REGISTRY = Registry("META_ARCH")


def build_model(cfg):
    """cfg.MODEL.META_ARCHITECTURE -> nn.Module (reference meta_arch/build.py:30-36)."""
    return META_ARCH_REGISTRY.get(cfg.MODEL.META_ARCHITECTURE)(cfg)
