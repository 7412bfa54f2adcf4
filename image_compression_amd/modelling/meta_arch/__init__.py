from .build import META_ARCH_REGISTRY, build_model
from .bmshl2018 import Compressor2018
