"""image_compression_amd — MI355X-native (gfx950) hot path of
hieu1999210/image_compression: the Balle-2018 scale-hyperprior forward and
backward on hand-written HIP kernels, behind the reference's
`modelling.meta_arch` / `modelling.layers` API.

    from image_compression_amd import modelling, get_cfg_defaults
    model = modelling.build_model(cfg).cuda()
"""
from . import modelling
from .config import get_cfg_defaults, CfgNode
from .noise import injected_noise

__all__ = ["modelling", "get_cfg_defaults", "CfgNode", "injected_noise"]
